// Motion-compensation inputs of the subpel search on gfx950:
//  * half-pel planes (reference x264_frame_filter common/mc.c:704-726, hpel_filter
//    mc.c:173-196, x264_frame_expand_border_filtered common/frame.c:599-625);
//  * SAD / SATD of blocks fetched at quarter-pel positions (get_ref, mc.c:221-249,
//    with x264_hpel_ref0/1 of common/tables.c:183-184 and pixel_avg mc.c:49-61),
//    i.e. the candidate costs of refine_subpel (encoder/me.c:865-992).
#include "hipcommon.h"

#include <stdlib.h>
#include <type_traits>

namespace x264hip {

// ------------------------------------------------------------ hpel filter
// The reference filters x in [-8, W+8) and y in [-8, H+8) of each plane, then
// re-expands the border from the last trusted column/row (x = -4 / W+3, y = -8 / H+7)
// over the 32-pixel padding: a border pixel is the filter at the clamped coordinate.
__device__ __forceinline__ int tap6( int a, int b, int c, int d, int e, int f )
{
    return a + f - 5 * (b + e) + 20 * (c + d);   // TAPFILTER, mc.c:172
}

// Fused kernel (10 bit, and 8-bit planes whose rows are not 16-byte aligned): one pass over
// the whole padded plane.  A pixel of
// the border takes the value the reference copies into it, i.e. the filter at
// the clamped coordinate (x in [-4, W+3], y in [-8, H+7]); since the clamp is
// monotonic, a 64x16 output tile needs at most a 76x21 source tile around its
// clamped coordinates (plus alignment).  The source tile is fetched as aligned dwords, each
// thread produces 4 horizontally adjacent pixels of each plane (dword stores
// at 8 bit), and the expand pass with its read-back disappears.
constexpr int HF_W = 64, HF_H = 16, HF_SW = 76, HF_SH = HF_H + 5;   // SW: 4..7 px of alignment + 64 + 2 + 3 halo

// clip( v >> S ) to a pixel, written as a clamp before the shift.  The form
// clip( v >> S ) packed into bytes is lowered by this ROCm's compiler to
// v_ashr_pk_u8_i32, whose packed result came back with the high half not
// cleared on the box (bytes 2-3 of every stored dword corrupted); the
// clamp-first form computes the same value and avoids that lowering.
template <int BD, int S>
__device__ __forceinline__ int shr_clip( int v )
{
    constexpr int HI = (PT<BD>::PIXEL_MAX << S) | ((1 << S) - 1);
    return (v < 0 ? 0 : v > HI ? HI : v) >> S;
}

template <int BD>
__global__ __launch_bounds__( 256 ) void hpel_fused_kernel( const typename PT<BD>::pixel *__restrict__ src,
                                                            typename PT<BD>::pixel *__restrict__ dh,
                                                            typename PT<BD>::pixel *__restrict__ dv,
                                                            typename PT<BD>::pixel *__restrict__ dc,
                                                            intptr_t stride, intptr_t fstride, int width, int height )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int PPD = PT<BD>::PPD;
    constexpr int pad = BD > 9 ? -10 * PT<BD>::PIXEL_MAX : 0;    // mc.c:176
    __shared__ __align__( 16 ) int s_src[HF_SH][HF_SW];
    __shared__ __align__( 16 ) int s_v[HF_H][HF_SW];
    const int x0 = -32 + HF_W * blockIdx.x, y0 = -32 + HF_H * blockIdx.y;
    const int cx0 = min( max( x0, -4 ), width + 3 ), cy0 = min( max( y0, -8 ), height + 7 );
    const int sx0 = ((cx0 - 4) & ~3);                       // dword-aligned source origin (4 px)
    const int sy0 = cy0 - 2;
    const intptr_t fo = (intptr_t)blockIdx.z * fstride;
    const pixel *s = src + fo;
    // source tile: HF_SH rows x HF_SW pixels from aligned dwords, unpacked to
    // ints with 16-byte LDS stores; columns past the right padding are never
    // read by a written pixel and are not fetched
    constexpr int QPR = HF_SW / 4;                           // 4-pixel groups per tile row
    for( int i = threadIdx.x; i < HF_SH * QPR; i += 256 )
    {
        const int r = i / QPR, k = i % QPR;
        const int col = sx0 + 4 * k;
        uint32_t w[4 / PPD] = {};
        if( col + 4 <= width + 32 )
#pragma unroll
            for( int q = 0; q < 4 / PPD; q++ )
                w[q] = *(const uint32_t *)(s + (intptr_t)(sy0 + r) * stride + col + q * PPD);
        int4 v;
        v.x = upix<BD>( w[0], 0 );
        v.y = upix<BD>( w[1 / PPD], 1 % PPD );
        v.z = upix<BD>( w[2 / PPD], 2 % PPD );
        v.w = upix<BD>( w[3 / PPD], 3 % PPD );
        *(int4 *)&s_src[r][4 * k] = v;
    }
    __syncthreads();
    // vertical 6-tap intermediates, four columns per thread
    for( int i = threadIdx.x; i < HF_H * QPR; i += 256 )
    {
        const int r = i / QPR, c = 4 * (i % QPR);
        int4 a[6];
#pragma unroll
        for( int k = 0; k < 6; k++ )
            a[k] = *(const int4 *)&s_src[r + k][c];
        int4 v;
        v.x = tap6( a[0].x, a[1].x, a[2].x, a[3].x, a[4].x, a[5].x );
        v.y = tap6( a[0].y, a[1].y, a[2].y, a[3].y, a[4].y, a[5].y );
        v.z = tap6( a[0].z, a[1].z, a[2].z, a[3].z, a[4].z, a[5].z );
        v.w = tap6( a[0].w, a[1].w, a[2].w, a[3].w, a[4].w, a[5].w );
        *(int4 *)&s_v[r][c] = v;
    }
    __syncthreads();
    const int ty = threadIdx.x >> 4, xq = (threadIdx.x & 15) * 4;
    const int y = y0 + ty;
    const int xs = x0 + xq;
    if( y >= height + 32 || xs >= width + 32 )
        return;
    const int ry = min( max( y, -8 ), height + 7 ) - sy0 - 2;      // row of s_v / centre row of s_src is ry+2
    int vh[4], vv[4], vc[4];
    if( xs >= -4 && xs + 3 <= width + 3 )
    {
        // unclamped columns: the 12-value windows [c-4, c+8) of the two rows are aligned
        const int c = xs - sx0;                                    // multiple of 4
        int hs_[12], vs_[12];
#pragma unroll
        for( int k = 0; k < 3; k++ )
        {
            const int4 a = *(const int4 *)&s_src[ry + 2][c - 4 + 4 * k];
            const int4 b = *(const int4 *)&s_v[ry][c - 4 + 4 * k];
            hs_[4 * k] = a.x; hs_[4 * k + 1] = a.y; hs_[4 * k + 2] = a.z; hs_[4 * k + 3] = a.w;
            vs_[4 * k] = b.x; vs_[4 * k + 1] = b.y; vs_[4 * k + 2] = b.z; vs_[4 * k + 3] = b.w;
        }
#pragma unroll
        for( int j = 0; j < 4; j++ )
        {
            vv[j] = shr_clip<BD, 5>( vs_[4 + j] + 16 );
            vh[j] = shr_clip<BD, 5>( tap6( hs_[j + 2], hs_[j + 3], hs_[j + 4], hs_[j + 5], hs_[j + 6], hs_[j + 7] ) + 16 );
            int b[6];
#pragma unroll
            for( int q = 0; q < 6; q++ )
                b[q] = (int16_t)(vs_[j + 2 + q] + pad);
            vc[j] = shr_clip<BD, 10>( tap6( b[0], b[1], b[2], b[3], b[4], b[5] ) - 32 * pad + 512 );
        }
    }
    else
    {
#pragma unroll
        for( int j = 0; j < 4; j++ )
        {
            const int cxl = min( max( xs + j, -4 ), width + 3 ) - sx0;   // column of the pixel in the tile
            vv[j] = shr_clip<BD, 5>( s_v[ry][cxl] + 16 );
            const int hs = tap6( s_src[ry + 2][cxl - 2], s_src[ry + 2][cxl - 1], s_src[ry + 2][cxl],
                                 s_src[ry + 2][cxl + 1], s_src[ry + 2][cxl + 2], s_src[ry + 2][cxl + 3] );
            vh[j] = shr_clip<BD, 5>( hs + 16 );
            int b[6];
#pragma unroll
            for( int q = 0; q < 6; q++ )
                b[q] = (int16_t)(s_v[ry][cxl - 2 + q] + pad);
            vc[j] = shr_clip<BD, 10>( tap6( b[0], b[1], b[2], b[3], b[4], b[5] ) - 32 * pad + 512 );
        }
    }
    const intptr_t o = fo + (intptr_t)y * stride + xs;
#pragma unroll
    for( int k = 0; k < 4 / PPD; k++ )
    {
        uint32_t wh = 0, wv = 0, wc = 0;
#pragma unroll
        for( int j = 0; j < PPD; j++ )
        {
            const int sh = j * (32 / PPD);
            wh |= (uint32_t)vh[k * PPD + j] << sh;
            wv |= (uint32_t)vv[k * PPD + j] << sh;
            wc |= (uint32_t)vc[k * PPD + j] << sh;
        }
        *(uint32_t *)(dh + o + k * PPD) = wh;
        *(uint32_t *)(dv + o + k * PPD) = wv;
        *(uint32_t *)(dc + o + k * PPD) = wc;
    }
}

// Streaming variant (default at 8 bit): a lane owns 16 adjacent output columns
// (16 bytes of each plane) of a strip of HS_ROWS rows and walks it top to bottom
// with the 6-row source window in registers as 16-bit pixel pairs; the columns
// beside its 16 come from the adjacent lanes through DPP wave shifts (a wave
// covers 62 column quads plus a halo lane on each side), so a lane loads one
// aligned 16-byte row piece per source row, stores 16-byte pieces, and no LDS is
// used.  The vertical 6-tap runs on packed pairs (v_pk_mad: the 8-bit
// intermediates -2550..10710 fit int16), the horizontal ones (H from pixels,
// centre from the int16 intermediates, both mc.c:173-196) as v_dot2_i32_i16
// chains over even-aligned pairs.  Border pixels are the filter at the clamped
// coordinate (x in [-4, W+3], y in [-8, H+7]) as in the fused kernel: lanes are
// laid on x = -16 + 16q, so the first / last quad replicate pixel -4 / W+3 into
// their outer 12 columns and store one more piece for x in [-32, -16) /
// [W+16, W+32); the first / last strip repeat rows -8 / H+7.
typedef short hs2 __attribute__( ( ext_vector_type( 2 ) ) );

__device__ __forceinline__ hs2 as_s2( uint32_t v ) { return __builtin_bit_cast( hs2, v ); }
__device__ __forceinline__ uint32_t as_u( hs2 v ) { return __builtin_bit_cast( uint32_t, v ); }

// the four outputs x..x+3 of a horizontal 6-tap over the even pairs P[J..J+4] =
// (x-2, x-1), (x, x+1), (x+2, x+3), (x+4, x+5), (x+6, x+7), unscaled, the first tap of each chain taking its
// coefficient pair from a VGPR (k15 = (1, -5), k01 = (0, 1)): that dot2 is then the
// three-operand form with the SGPR bias as its accumulator, where a literal
// coefficient forces the two-operand form and a v_mov of the bias into each
// chain's destination (32 per output row).
// (the compiler turns even the three-operand builtin into v_mov + v_dot2c, so the
// first tap is written out)
template <int BIAS> __device__ __forceinline__ int dot2_first( hs2 p, hs2 k )
{
    int d;
    if constexpr( BIAS <= 64 )
        asm( "v_dot2_i32_i16 %0, %1, %2, %3" : "=v"( d ) : "v"( as_u( p ) ), "v"( as_u( k ) ), "i"( BIAS ) );
    else
        asm( "v_dot2_i32_i16 %0, %1, %2, %3" : "=v"( d ) : "v"( as_u( p ) ), "v"( as_u( k ) ), "s"( BIAS ) );
    return d;
}

template <int J, int BIAS, int N>
__device__ __forceinline__ void tap6_h4v( const hs2 (&P)[N], hs2 k15, hs2 k01, int (&o)[4] )
{
    o[0] = dot2_first<BIAS>( P[J], k15 );
    o[0] = __builtin_amdgcn_sdot2( P[J + 1], (hs2){ 20, 20 }, o[0], false );
    o[0] = __builtin_amdgcn_sdot2( P[J + 2], (hs2){ -5, 1 }, o[0], false );
    o[1] = dot2_first<BIAS>( P[J], k01 );
    o[1] = __builtin_amdgcn_sdot2( P[J + 1], (hs2){ -5, 20 }, o[1], false );
    o[1] = __builtin_amdgcn_sdot2( P[J + 2], (hs2){ 20, -5 }, o[1], false );
    o[1] = __builtin_amdgcn_sdot2( P[J + 3], (hs2){ 1, 0 }, o[1], false );
    o[2] = dot2_first<BIAS>( P[J + 1], k15 );
    o[2] = __builtin_amdgcn_sdot2( P[J + 2], (hs2){ 20, 20 }, o[2], false );
    o[2] = __builtin_amdgcn_sdot2( P[J + 3], (hs2){ -5, 1 }, o[2], false );
    o[3] = dot2_first<BIAS>( P[J + 1], k01 );
    o[3] = __builtin_amdgcn_sdot2( P[J + 2], (hs2){ -5, 20 }, o[3], false );
    o[3] = __builtin_amdgcn_sdot2( P[J + 3], (hs2){ 20, -5 }, o[3], false );
    o[3] = __builtin_amdgcn_sdot2( P[J + 4], (hs2){ 1, 0 }, o[3], false );
}

// bytes 0-1 = clip( lo >> S ), clip( hi >> S ) by gfx950's v_ashr_pk_u8_i32 (signed
// shift, unsigned byte saturation).  Bytes 2-3 of its result are not cleared
// (see shr_clip), so callers take only the low half.
template <int S> __device__ __forceinline__ uint32_t ashr_pk_u8( int lo, int hi )
{
    uint32_t d;
    asm( "v_ashr_pk_u8_i32 %0, %1, %2, %3" : "=v"( d ) : "v"( lo ), "v"( hi ), "i"( S ) );
    return d;
}

// four filter sums (bias included) as four pixels: two packed shifts, one perm
template <int S> __device__ __forceinline__ uint32_t pack_shr4( const int (&o)[4] )
{
    return __builtin_amdgcn_perm( ashr_pk_u8<S>( o[2], o[3] ), ashr_pk_u8<S>( o[0], o[1] ), 0x05040100u );
}

// two int16 pairs as four pixels clip( v >> 5 ): packed shifts, gfx950's
// v_sat_pk_u8_i16 (low half only, as above), one perm
__device__ __forceinline__ uint32_t sat_pk_u8( hs2 v )
{
    uint32_t d;
    asm( "v_sat_pk_u8_i16 %0, %1" : "=v"( d ) : "v"( as_u( v ) ) );
    return d;
}

template <int HS_ROWS, bool NT = false>
__device__ __forceinline__ void hpel_stream_body( const uint8_t *__restrict__ src, uint8_t *__restrict__ dh,
                                                  uint8_t *__restrict__ dv, uint8_t *__restrict__ dc,
                                                  intptr_t stride, intptr_t fstride, int width, int height,
                                                  Blk3 B, int nstrips )
{
    const int lane = threadIdx.x & 63;
    const int nq = (width + 32) >> 4;                       // column quads over x in [-16, W+16)
    const int chunk = (int)B.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if( chunk * 62 >= nq )
        return;                                              // wave-uniform
    const int q = chunk * 62 - 1 + lane;
    const bool st = lane >= 1 && lane <= 62 && q < nq;
    const int x0 = -16 + 16 * min( max( q, -1 ), nq );       // halo lanes load clamped columns
    // strips 0 .. nstrips-1 cover rows [-8, H+8); the last four replicate row -8 into
    // rows -32..-9 / row H+7 into H+8..H+31, 12 rows each, so no wave stores more
    // rows than a strip does (a wave storing all 25 border rows was the launch's tail)
    const int sy = (int)B.y - nstrips;                      // >= 0: border strip
    const int r0 = sy < 0 ? -8 + (int)B.y * HS_ROWS : sy < 2 ? -8 : height + 7;
    const int r1 = sy < 0 ? min( r0 + HS_ROWS, height + 8 ) : r0 + 1;
    const int b0 = sy < 0 ? 0 : sy < 2 ? -32 + 12 * sy : height + 8 + 12 * (sy - 2);
    const intptr_t fo = (intptr_t)B.z * fstride + x0;
    const uint8_t *sp = src + fo;
    auto ld = [&]( int row ) { return *(const uint4 *)(sp + (intptr_t)row * stride); };
    auto unpack = [&]( uint4 d, hs2 (&P)[11] ) {
        const uint32_t dl = (uint32_t)__builtin_amdgcn_mov_dpp( (int)d.w, 0x138, 0xF, 0xF, true );   // lane - 1
        const uint32_t dr = (uint32_t)__builtin_amdgcn_mov_dpp( (int)d.x, 0x130, 0xF, 0xF, true );   // lane + 1
        P[0] = as_s2( __builtin_amdgcn_perm( 0u, dl, 0x0c030c02u ) );
        const uint32_t w[4] = { d.x, d.y, d.z, d.w };
#pragma unroll
        for( int j = 0; j < 4; j++ )
        {
            P[1 + 2 * j] = as_s2( __builtin_amdgcn_perm( 0u, w[j], 0x0c010c00u ) );
            P[2 + 2 * j] = as_s2( __builtin_amdgcn_perm( 0u, w[j], 0x0c030c02u ) );
        }
        P[9] = as_s2( __builtin_amdgcn_perm( 0u, dr, 0x0c010c00u ) );
        P[10] = as_s2( __builtin_amdgcn_perm( 0u, dr, 0x0c030c02u ) );
    };
    // opaque VGPR coefficient pairs (1, -5) / (0, 1) for tap6_h4v's first taps
    uint32_t k15u, k01u;
    asm( "v_mov_b32 %0, 0xfffb0001" : "=v"( k15u ) );
    asm( "v_mov_b32 %0, 0x10000" : "=v"( k01u ) );
    const hs2 k15 = as_s2( k15u ), k01 = as_s2( k01u );
    hs2 win[6][11];                                          // source rows as even pairs, ring of 6
    uint4 raw[6];                                            // next block's source rows, in flight
#pragma unroll
    for( int k = 0; k < 5; k++ )
        raw[k] = ld( r0 - 2 + k );
#pragma unroll
    for( int k = 0; k < 5; k++ )
        unpack( raw[k], win[k] );
#pragma unroll
    for( int k = 0; k < 6; k++ )
        raw[k] = ld( r0 + 3 + k );
    for( int cy = r0; cy < r1; cy += 6 )
    {
#pragma unroll
        for( int k = 0; k < 6; k++ )
        {
            const int y = cy + k;
            if( y >= r1 )
                break;                                       // wave-uniform
            // source row y + 3 arrived; its slot now fetches row y + 9 (six rows of lead)
            uint4 cur[6];
            cur[k] = raw[k];
            raw[k] = ld( y + 9 );
            // vertical 6-tap intermediates at columns x-2 .. x+19 (int16, exact at 8 bit)
            hs2 vi[11], hrow[11];
            unpack( cur[k], win[(k + 5) % 6] );              // source row y + 3
#pragma unroll
            for( int p = 0; p < 11; p++ )
            {
                const hs2 a = win[k % 6][p], b = win[(k + 1) % 6][p], c = win[(k + 2) % 6][p];
                const hs2 d = win[(k + 3) % 6][p], e = win[(k + 4) % 6][p], f = win[(k + 5) % 6][p];
                vi[p] = (a + f) + (c + d) * (hs2)20 - (b + e) * (hs2)5;
                hrow[p] = c;
            }
            uint32_t oh[4], ov[4], oc[4];
            int o[4];
            // V: clip( (v + 16) >> 5 ) by packed arithmetic shift + byte saturation;
            // H: clip( (t + 16) >> 5 ), centre: clip( (t + 512) >> 10 ) with the
            // bias in the accumulator and v_ashr_pk_u8_i32 doing shift and clip
#pragma unroll
            for( int j = 0; j < 4; j++ )
                ov[j] = __builtin_amdgcn_perm( sat_pk_u8( (vi[2 + 2 * j] + (hs2)16) >> (hs2)5 ),
                                               sat_pk_u8( (vi[1 + 2 * j] + (hs2)16) >> (hs2)5 ), 0x05040100u );
            tap6_h4v<0, 16>( hrow, k15, k01, o ); oh[0] = pack_shr4<5>( o );
            tap6_h4v<2, 16>( hrow, k15, k01, o ); oh[1] = pack_shr4<5>( o );
            tap6_h4v<4, 16>( hrow, k15, k01, o ); oh[2] = pack_shr4<5>( o );
            tap6_h4v<6, 16>( hrow, k15, k01, o ); oh[3] = pack_shr4<5>( o );
            tap6_h4v<0, 512>( vi, k15, k01, o ); oc[0] = pack_shr4<10>( o );
            tap6_h4v<2, 512>( vi, k15, k01, o ); oc[1] = pack_shr4<10>( o );
            tap6_h4v<4, 512>( vi, k15, k01, o ); oc[2] = pack_shr4<10>( o );
            tap6_h4v<6, 512>( vi, k15, k01, o ); oc[3] = pack_shr4<10>( o );
            if( st )
            {
                intptr_t ox = 0;                             // extra piece: x in [-32, -16) / [W+16, W+32)
                if( q == 0 )
                {
                    // x -16..-5 take pixel -4 (byte 0 of the last dword)
                    oh[0] = oh[1] = oh[2] = __builtin_amdgcn_perm( 0u, oh[3], 0 );
                    ov[0] = ov[1] = ov[2] = __builtin_amdgcn_perm( 0u, ov[3], 0 );
                    oc[0] = oc[1] = oc[2] = __builtin_amdgcn_perm( 0u, oc[3], 0 );
                    ox = -16;
                }
                else if( q == nq - 1 )
                {
                    // x W+4..W+15 take pixel W+3 (byte 3 of the first dword)
                    oh[1] = oh[2] = oh[3] = __builtin_amdgcn_perm( 0u, oh[0], 0x03030303u );
                    ov[1] = ov[2] = ov[3] = __builtin_amdgcn_perm( 0u, ov[0], 0x03030303u );
                    oc[1] = oc[2] = oc[3] = __builtin_amdgcn_perm( 0u, oc[0], 0x03030303u );
                    ox = 16;
                }
                const uint4 vh = make_uint4( oh[0], oh[1], oh[2], oh[3] );
                const uint4 vv = make_uint4( ov[0], ov[1], ov[2], ov[3] );
                const uint4 vc = make_uint4( oc[0], oc[1], oc[2], oc[3] );
                const uint4 eh = ox < 0 ? make_uint4( oh[0], oh[0], oh[0], oh[0] ) : make_uint4( oh[3], oh[3], oh[3], oh[3] );
                const uint4 ev = ox < 0 ? make_uint4( ov[0], ov[0], ov[0], ov[0] ) : make_uint4( ov[3], ov[3], ov[3], ov[3] );
                const uint4 ec = ox < 0 ? make_uint4( oc[0], oc[0], oc[0], oc[0] ) : make_uint4( oc[3], oc[3], oc[3], oc[3] );
                // rows: y, or the replicated border rows -32..-8 / H+7..H+31
                const int ya = sy < 0 ? y : b0, yb = sy < 0 ? y : b0 + 11;
                for( int yy = ya; yy <= yb; yy++ )
                {
                    const intptr_t o0 = fo + (intptr_t)yy * stride;
                    st16<NT>( dh + o0, vh );
                    st16<NT>( dv + o0, vv );
                    st16<NT>( dc + o0, vc );
                    if( ox )
                    {
                        st16<NT>( dh + o0 + ox, eh );
                        st16<NT>( dv + o0 + ox, ev );
                        st16<NT>( dc + o0 + ox, ec );
                    }
                }
            }
        }
    }
}

// the fallback for widths the line-aligned chunks cannot take (below): 62 working lanes and
// two halo lanes per wave
template <int HS_ROWS, bool NT = false>
__global__ __launch_bounds__( 64 ) void hpel_stream_kernel( const uint8_t *__restrict__ src, uint8_t *__restrict__ dh,
                                                             uint8_t *__restrict__ dv, uint8_t *__restrict__ dc,
                                                             intptr_t stride, intptr_t fstride, int width,
                                                             int height, int xcd )
{
    hpel_stream_body<HS_ROWS, NT>( src, dh, dv, dc, stride, fstride, width, height, blk3( xcd ), (int)gridDim.y - 4 );
}

// Variant 7 (8-bit default): variant 3's streaming strips with every wave's stores on whole
// 128-B lines.  Variant 3's waves own 62 column quads (992 bytes of each output row), so
// every wave boundary splits a line between two waves -- often on two XCDs -- and the
// partial lines streamed no faster than 0.57 of HBM even with nontemporal stores (the
// pattern alone: profiles/r03v_pattern64.txt, `s3nt62u` 0.569 vs 0.823 line-aligned).  Here a
// wave owns 64 16-pixel pieces of x in [-32, W+32) (1 KB, line-aligned), its edge lanes
// fetch their outer neighbour's dword from memory instead of by DPP, and the replicated
// border pieces are ordinary lanes: 64 frames 0.1383 -> 0.0927 ms (0.53 -> 0.79 of HBM),
// 16 frames 0.0312 -> 0.0267 ms with nontemporal stores (profiles/r03w_stream_var.json).
// Also: a slot is unpacked before it is reloaded (one register tuple, no loop-carried copy:
// 118 VGPRs, 4 waves per SIMD against variant 3's 140 and 3); every row issues the same
// three buffer stores (lanes past the row address beyond the buffer's range, so the store
// is dropped); the source pointer is not __restrict__ and each reload is followed by a
// compiler memory barrier (as invariant loads the compiler sank the reloads to the end of
// the six-row group, leaving one row of lead).  The compiler's waitcnt pass, with loads
// and stores both in flight, waits vmcnt(0) once per six rows.  (Counted waits on asm
// loads were tried: the compiler copied and reused the registers of loads it could not
// see in flight.)  The four border strips (rows -32..-9 / H+8..H+31, replicas of rows -8 /
// H+7) take their own path.
template <bool NT>
__device__ __forceinline__ void st16b( uint4 v, __amdgpu_buffer_rsrc_t r, uint32_t off )
{
    typedef unsigned int v4u __attribute__( ( ext_vector_type( 4 ) ) );
    __builtin_amdgcn_raw_buffer_store_b128( (v4u){ v.x, v.y, v.z, v.w }, r, (int)off, 0, NT ? 2 : 0 );
}

typedef unsigned int hv4u __attribute__( ( ext_vector_type( 4 ) ) );

template <int HS_ROWS, bool NT, bool BORDER>
__device__ __forceinline__ void hpel_strip7( const uint8_t *src, uint8_t *__restrict__ dh,
                                             uint8_t *__restrict__ dv, uint8_t *__restrict__ dc, intptr_t stride,
                                             intptr_t fstride, int width, int height, Blk3 B, int nstrips )
{
    // 16-pixel pieces p over x in [-32, W+32): a wave owns 64 of them (1 KB of each output row,
    // on the 128-B line grid), lane L piece 64 * chunk + L.  q = p - 1 is variant 3's column
    // quad (x0 = -16 + 16 q); q = -1 / q = nq are the replicated 16-pixel border pieces.
    const int lane = threadIdx.x & 63;
    const int nq = (width + 32) >> 4, np = nq + 2;
    const int chunk = (int)B.x;
    if( chunk * 64 >= np )
        return;
    const int p = chunk * 64 + lane, q = p - 1;
    const bool st = p < np;
    const int x0 = -16 + 16 * min( q, nq );                 // lanes past the row load the last piece
    // lanes 0 / 63 take their outer neighbour's dword from memory, the others by DPP
    const int xn = lane == 0 ? max( x0 - 4, -32 ) : lane == 63 ? x0 + 16 : x0;
    const int sy = (int)B.y - nstrips;
    const int r0 = !BORDER ? -8 + (int)B.y * HS_ROWS : sy < 2 ? -8 : height + 7;
    const int r1 = !BORDER ? min( r0 + HS_ROWS, height + 8 ) : r0 + 1;
    const int b0 = !BORDER ? 0 : sy < 2 ? -32 + 12 * sy : height + 8 + 12 * (sy - 2);
    const uint8_t *sp = src + (intptr_t)B.z * fstride + x0;
    const uint8_t *spn = src + (intptr_t)B.z * fstride + xn;
    auto ld = [&]( int row ) { return *(const hv4u *)(sp + (intptr_t)row * stride); };
    auto ldn = [&]( int row ) { return *(const uint32_t *)(spn + (intptr_t)row * stride); };
    // the frame's three output planes from row -32, column -32: byte offsets below 2^31
    const intptr_t fb = (intptr_t)B.z * fstride - 32 * stride - 32;
    const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc( dh + fb, (short)0, 0x7fffffff, 0x00020000 );
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc( dv + fb, (short)0, 0x7fffffff, 0x00020000 );
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc( dc + fb, (short)0, 0x7fffffff, 0x00020000 );
    constexpr uint32_t OOB = 0x80000000u;                   // >= the range: the store is dropped
    const uint32_t xo = st ? (uint32_t)(16 * p) : OOB;
    auto unpack = [&]( hv4u d, uint32_t n, hs2 (&P)[11] ) {
        uint32_t dl = (uint32_t)__builtin_amdgcn_mov_dpp( (int)d.w, 0x138, 0xF, 0xF, true );   // lane - 1
        uint32_t dr = (uint32_t)__builtin_amdgcn_mov_dpp( (int)d.x, 0x130, 0xF, 0xF, true );   // lane + 1
        dl = lane == 0 ? n : dl;
        dr = lane == 63 ? n : dr;
        P[0] = as_s2( __builtin_amdgcn_perm( 0u, dl, 0x0c030c02u ) );
        const uint32_t w[4] = { d.x, d.y, d.z, d.w };
#pragma unroll
        for( int j = 0; j < 4; j++ )
        {
            P[1 + 2 * j] = as_s2( __builtin_amdgcn_perm( 0u, w[j], 0x0c010c00u ) );
            P[2 + 2 * j] = as_s2( __builtin_amdgcn_perm( 0u, w[j], 0x0c030c02u ) );
        }
        P[9] = as_s2( __builtin_amdgcn_perm( 0u, dr, 0x0c010c00u ) );
        P[10] = as_s2( __builtin_amdgcn_perm( 0u, dr, 0x0c030c02u ) );
    };
    uint32_t k15u, k01u;
    asm( "v_mov_b32 %0, 0xfffb0001" : "=v"( k15u ) );
    asm( "v_mov_b32 %0, 0x10000" : "=v"( k01u ) );
    const hs2 k15 = as_s2( k15u ), k01 = as_s2( k01u );
    hs2 win[6][11];
    hv4u raw[6];
    uint32_t rawn[6];
#pragma unroll
    for( int k = 0; k < 5; k++ )
    {
        raw[k] = ld( r0 - 2 + k );
        rawn[k] = ldn( r0 - 2 + k );
    }
#pragma unroll
    for( int k = 0; k < 5; k++ )
        unpack( raw[k], rawn[k], win[k] );
#pragma unroll
    for( int k = 0; k < 6; k++ )
    {
        raw[k] = ld( r0 + 3 + k );
        rawn[k] = ldn( r0 + 3 + k );
    }
    auto do_row = [&]( auto K, const int y ) {
        constexpr int k = decltype( K )::value;
        unpack( raw[k], rawn[k], win[(k + 5) % 6] );
        const int yl = min( y + 9, r1 + 2 );                // past the strip's last source row: a repeat
        raw[k] = ld( yl );
        rawn[k] = ldn( yl );
        asm volatile( "" ::: "memory" );                    // keep the loads six rows ahead of their use
        hs2 vi[11], hrow[11];
#pragma unroll
        for( int j = 0; j < 11; j++ )
        {
            const hs2 a = win[k % 6][j], b = win[(k + 1) % 6][j], c = win[(k + 2) % 6][j];
            const hs2 d = win[(k + 3) % 6][j], e = win[(k + 4) % 6][j], f = win[(k + 5) % 6][j];
            vi[j] = (a + f) + (c + d) * (hs2)20 - (b + e) * (hs2)5;
            hrow[j] = c;
        }
        uint32_t oh[4], ov[4], oc[4];
        int o[4];
#pragma unroll
        for( int j = 0; j < 4; j++ )
            ov[j] = __builtin_amdgcn_perm( sat_pk_u8( (vi[2 + 2 * j] + (hs2)16) >> (hs2)5 ),
                                           sat_pk_u8( (vi[1 + 2 * j] + (hs2)16) >> (hs2)5 ), 0x05040100u );
        tap6_h4v<0, 16>( hrow, k15, k01, o ); oh[0] = pack_shr4<5>( o );
        tap6_h4v<2, 16>( hrow, k15, k01, o ); oh[1] = pack_shr4<5>( o );
        tap6_h4v<4, 16>( hrow, k15, k01, o ); oh[2] = pack_shr4<5>( o );
        tap6_h4v<6, 16>( hrow, k15, k01, o ); oh[3] = pack_shr4<5>( o );
        tap6_h4v<0, 512>( vi, k15, k01, o ); oc[0] = pack_shr4<10>( o );
        tap6_h4v<2, 512>( vi, k15, k01, o ); oc[1] = pack_shr4<10>( o );
        tap6_h4v<4, 512>( vi, k15, k01, o ); oc[2] = pack_shr4<10>( o );
        tap6_h4v<6, 512>( vi, k15, k01, o ); oc[3] = pack_shr4<10>( o );
        // the edge quads: x -16..-5 take pixel -4 / x W+4..W+15 take pixel W+3; the border pieces
        // (q = -1 / nq) are those pixels repeated, taken from the neighbouring lane
        const bool lo = q == 0, hi = q == nq - 1, mid = lo || hi;
        uint32_t selh = lo ? __builtin_amdgcn_perm( 0u, oh[3], 0 ) : __builtin_amdgcn_perm( 0u, oh[0], 0x03030303u );
        uint32_t selv = lo ? __builtin_amdgcn_perm( 0u, ov[3], 0 ) : __builtin_amdgcn_perm( 0u, ov[0], 0x03030303u );
        uint32_t selc = lo ? __builtin_amdgcn_perm( 0u, oc[3], 0 ) : __builtin_amdgcn_perm( 0u, oc[0], 0x03030303u );
        const uint32_t rh_ = (uint32_t)__builtin_amdgcn_mov_dpp( (int)selh, 0x130, 0xF, 0xF, true );
        const uint32_t rv_ = (uint32_t)__builtin_amdgcn_mov_dpp( (int)selv, 0x130, 0xF, 0xF, true );
        const uint32_t rc_ = (uint32_t)__builtin_amdgcn_mov_dpp( (int)selc, 0x130, 0xF, 0xF, true );
        const uint32_t lh_ = (uint32_t)__builtin_amdgcn_mov_dpp( (int)selh, 0x138, 0xF, 0xF, true );
        const uint32_t lv_ = (uint32_t)__builtin_amdgcn_mov_dpp( (int)selv, 0x138, 0xF, 0xF, true );
        const uint32_t lc_ = (uint32_t)__builtin_amdgcn_mov_dpp( (int)selc, 0x138, 0xF, 0xF, true );
        const bool bl = q == -1, br = q == nq, bd = bl || br;
        selh = bl ? rh_ : br ? lh_ : selh;
        selv = bl ? rv_ : br ? lv_ : selv;
        selc = bl ? rc_ : br ? lc_ : selc;
        const uint4 vh = make_uint4( lo || bd ? selh : oh[0], mid || bd ? selh : oh[1], mid || bd ? selh : oh[2],
                                     hi || bd ? selh : oh[3] );
        const uint4 vv = make_uint4( lo || bd ? selv : ov[0], mid || bd ? selv : ov[1], mid || bd ? selv : ov[2],
                                     hi || bd ? selv : ov[3] );
        const uint4 vc = make_uint4( lo || bd ? selc : oc[0], mid || bd ? selc : oc[1], mid || bd ? selc : oc[2],
                                     hi || bd ? selc : oc[3] );
        if constexpr( !BORDER )
        {
            const uint32_t ro = (uint32_t)((y + 32) * stride);
            st16b<NT>( vh, rh, xo + ro );
            st16b<NT>( vv, rv, xo + ro );
            st16b<NT>( vc, rc, xo + ro );
        }
        else
        {
            for( int yy = b0; yy < b0 + 12; yy++ )
            {
                const uint32_t ro = (uint32_t)((yy + 32) * stride);
                st16b<NT>( vh, rh, xo + ro );
                st16b<NT>( vv, rv, xo + ro );
                st16b<NT>( vc, rc, xo + ro );
            }
        }
    };
    for( int cy = r0; cy < r1; cy += 6 )
    {
        do_row( std::integral_constant<int, 0>{}, cy );
        if( cy + 1 >= r1 ) break;
        do_row( std::integral_constant<int, 1>{}, cy + 1 );
        if( cy + 2 >= r1 ) break;
        do_row( std::integral_constant<int, 2>{}, cy + 2 );
        if( cy + 3 >= r1 ) break;
        do_row( std::integral_constant<int, 3>{}, cy + 3 );
        if( cy + 4 >= r1 ) break;
        do_row( std::integral_constant<int, 4>{}, cy + 4 );
        if( cy + 5 >= r1 ) break;
        do_row( std::integral_constant<int, 5>{}, cy + 5 );
    }
}

template <int HS_ROWS, bool NT>
__global__ __launch_bounds__( 64 ) void hpel_strip7_kernel( const uint8_t *src, uint8_t *__restrict__ dh,
                                                            uint8_t *__restrict__ dv, uint8_t *__restrict__ dc,
                                                            intptr_t stride, intptr_t fstride, int width, int height,
                                                            int xcd )
{
    const Blk3 B = blk3( xcd );
    const int nstrips = (int)gridDim.y - 4;
    if( (int)B.y >= nstrips )
        hpel_strip7<HS_ROWS, NT, true>( src, dh, dv, dc, stride, fstride, width, height, B, nstrips );
    else
        hpel_strip7<HS_ROWS, NT, false>( src, dh, dv, dc, stride, fstride, width, height, B, nstrips );
}

template <int BD>
hipError_t launch_hpel_filter( const typename PT<BD>::pixel *src, typename PT<BD>::pixel *dh,
                               typename PT<BD>::pixel *dv, typename PT<BD>::pixel *dc, intptr_t stride,
                               intptr_t fstride, int width, int height, int nframes, hipStream_t stream )
{
    if( nframes <= 0 || width <= 0 || height <= 0 )
        return hipSuccess;
    if constexpr( BD == 8 )
    {
        // streaming strips: need 16-byte aligned rows (pixel (0,0) and the strides)
        if( !(((uintptr_t)src | (uintptr_t)dh | (uintptr_t)dv | (uintptr_t)dc | (uintptr_t)stride |
               (uintptr_t)fstride) & 15) )
        {
            // one wave per workgroup and 12-row strips: twice the waves of 24-row ones for 5
            // halo rows per strip (16 frames: 0.0455 -> 0.0398 ms; 64 frames: 0.166 -> 0.158 ms;
            // 6 / 8 / 16 / 24 rows all slower, profiles/r02k_hpel_rows*.json)
            constexpr int ROWS = 12;
            const int nq = (width + 32) / 16;
            dim3 g( (nq + 61) / 62, (height + 16 + ROWS - 1) / ROWS + 4, nframes );
            // XCD-contiguous strips (adjacent strips' halo rows in one L2; X264HIP_STREAM_XCD=0
            // turns it off): 0.0329 -> 0.0324 ms at 16 frames, 0.1514 -> 0.1499 at 64
            // (profiles/r03i_stream_var.json)
            const int sxcd = variant( V_STREAM_XCD ) != 0;
            const bool snt = stream_nt();
            // line-aligned 64-piece chunks (hpel_strip7_kernel) unless the right border piece
            // would lack its left neighbour in its wave, or the width is not a multiple of 16
            const int np = nq + 2;
            if( !(width & 15) && (np - 1) % 64 != 0 )
            {
                g.x = (np + 63) / 64;
                if( snt )
                    hipLaunchKernelGGL( ( hpel_strip7_kernel<ROWS, true> ), g, dim3( 64 ), 0, stream, src, dh, dv, dc,
                                        stride, fstride, width, height, sxcd );
                else
                    hipLaunchKernelGGL( ( hpel_strip7_kernel<ROWS, false> ), g, dim3( 64 ), 0, stream, src, dh, dv,
                                        dc, stride, fstride, width, height, sxcd );
            }
            else if( snt )
                hipLaunchKernelGGL( ( hpel_stream_kernel<ROWS, true> ), g, dim3( 64 ), 0, stream, src, dh, dv, dc,
                                    stride, fstride, width, height, sxcd );
            else
                hipLaunchKernelGGL( ( hpel_stream_kernel<ROWS, false> ), g, dim3( 64 ), 0, stream, src, dh, dv, dc,
                                    stride, fstride, width, height, sxcd );
            return hipGetLastError();
        }
    }
    // fused single pass; needs 4-pixel aligned rows (width + 64 covered by whole tiles of 4)
    dim3 g( (width + 64 + HF_W - 1) / HF_W, (height + 64 + HF_H - 1) / HF_H, nframes );
    hipLaunchKernelGGL( ( hpel_fused_kernel<BD> ), g, dim3( 256 ), 0, stream, src, dh, dv, dc, stride, fstride, width,
                        height );
    return hipGetLastError();
}

// ------------------------------------------------------------ qpel candidates
constexpr uint8_t c_hpel_ref0[16] = { 0, 1, 1, 1, 0, 1, 1, 1, 2, 3, 3, 3, 0, 1, 1, 1 };
constexpr uint8_t c_hpel_ref1[16] = { 0, 0, 1, 0, 2, 2, 3, 2, 2, 2, 3, 2, 2, 2, 3, 2 };

// rounding-up average of packed pixels, (a + b + 1) >> 1 per pixel (pixel_avg, mc.c:57)
template <int BD> __device__ __forceinline__ uint32_t avg_packed( uint32_t a, uint32_t b )
{
    constexpr uint32_t keep = BD == 8 ? 0x7F7F7F7Fu : 0x7FFF7FFFu;
    return (a | b) - (((a ^ b) >> 1) & keep);
}

// Row of NDW packed dwords at an arbitrary pixel address from dword-aligned loads:
// the NDW words of an aligned row, else the NDW + 1 words holding it realigned with
// v_alignbyte (no byte outside the row's dwords is touched).  On gfx950 the address
// path takes ~14.6 cycles per CU for a wave's dword-aligned dwordx2 / x3 / x4 load of
// 8-16 bytes per lane against 28.5 (x2) and 56.8 (x4) when the lanes' addresses are
// byte-misaligned (tools/ta_probe.hip, profiles/r01d_ta_probe.txt).
template <int NDW>
__device__ __forceinline__ void load_row_al( const void *p, uint32_t (&out)[NDW] )
{
    typedef const __attribute__( ( address_space( 1 ) ) ) uint32_t gword;
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3);
    gword *base = (gword *)((uintptr_t)p & ~(uintptr_t)3);
    uint32_t w[NDW + 1];
#pragma unroll
    for( int i = 0; i < NDW; i++ )
        w[i] = base[i];
    w[NDW] = base[sh ? NDW : NDW - 1];      // branch-free: re-reads word NDW-1 when aligned
#pragma unroll
    for( int i = 0; i < NDW; i++ )
        out[i] = __builtin_amdgcn_alignbyte( w[i + 1], w[i], sh );
}

// One lane per candidate (LD = 0 at 8 bit, 1 at 10 bit).  The second plane pointer equals the first when the
// qpel phase needs one plane (avg(a, a) = a), so every band's rows are issued
// as one burst of loads; rows are fetched with unaligned 4/8/16-byte global
// loads (amdhsa runs with unaligned access enabled: no alignbyte) or, LD = 1,
// dword-aligned loads + alignbyte (load_row_al); the 8-bit
// rounding average is one v_lerp_u8 per dword (pixel_avg, mc.c:57).
template <int BD, int OP, int IPIX, int LD>
__device__ __forceinline__ int subpel_score( const typename PT<BD>::pixel *a, intptr_t fs,
                                             const typename PT<BD>::pixel *p0, const typename PT<BD>::pixel *p1,
                                             const typename PT<BD>::pixel *p2, const typename PT<BD>::pixel *p3,
                                             intptr_t rs, int qx, int qy )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int PPD = PT<BD>::PPD;
    constexpr int W = pix_w( IPIX ), H = pix_h( IPIX );
    constexpr int NDW = W / PPD;
    constexpr int BAND = (16 / NDW) < 4 ? 4 : (16 / NDW) > H ? H : (16 / NDW);   // rows per load burst
    const int idx = ((qy & 3) << 2) + (qx & 3);
    const intptr_t off = (intptr_t)(qy >> 2) * rs + (qx >> 2);
    constexpr uint32_t k0 = pack_fields( c_hpel_ref0, 2 ), k1 = pack_fields( c_hpel_ref1, 2 );
    const int i0 = field( k0, 2, idx ), i1 = field( k1, 2, idx );
    const pixel *s1 = (i0 == 0 ? p0 : i0 == 1 ? p1 : i0 == 2 ? p2 : p3) + off + ((qy & 3) == 3) * rs;
    const pixel *s2 = (i1 == 0 ? p0 : i1 == 1 ? p1 : i1 == 2 ? p2 : p3) + off + ((qx & 3) == 3);
    if( !(idx & 5) )
        s2 = s1;
    uint32_t acc = 0;
    int sum = 0;
#pragma unroll
    for( int ty = 0; ty < H; ty += BAND )
    {
        uint32_t fr[BAND][NDW], rr[BAND][NDW], r2[BAND][NDW];
#pragma unroll
        for( int y = 0; y < BAND; y++ )
        {
            if constexpr( LD == 0 )
            {
                load_row_u<NDW>( a + (ty + y) * fs, fr[y] );
                load_row_u<NDW>( s1 + (ty + y) * rs, rr[y] );
                load_row_u<NDW>( s2 + (ty + y) * rs, r2[y] );
            }
            else
            {
                load_row_al<NDW>( a + (ty + y) * fs, fr[y] );
                load_row_al<NDW>( s1 + (ty + y) * rs, rr[y] );
                load_row_al<NDW>( s2 + (ty + y) * rs, r2[y] );
            }
        }
#pragma unroll
        for( int y = 0; y < BAND; y++ )
#pragma unroll
            for( int k = 0; k < NDW; k++ )
                rr[y][k] = avg_round<BD>( rr[y][k], r2[y][k] );
        if constexpr( OP == 0 )
        {
#pragma unroll
            for( int y = 0; y < BAND; y++ )
#pragma unroll
                for( int k = 0; k < NDW; k++ )
                    acc = sadp<BD>( fr[y][k], rr[y][k], acc );
        }
        else if constexpr( W >= 8 )
        {
#pragma unroll
            for( int by = 0; by < BAND; by += 4 )
#pragma unroll
                for( int tx = 0; tx < W; tx += 8 )
                {
                    uint32_t fa[4][8 / PPD], ra[4][8 / PPD];
#pragma unroll
                    for( int y = 0; y < 4; y++ )
#pragma unroll
                        for( int k = 0; k < 8 / PPD; k++ )
                        {
                            fa[y][k] = fr[by + y][tx / PPD + k];
                            ra[y][k] = rr[by + y][tx / PPD + k];
                        }
                    acc += satd8x4_packed<BD>( fa, ra );
                }
        }
        else
        {
#pragma unroll
            for( int by = 0; by < BAND; by += 4 )
            {
                int d[4][4];
#pragma unroll
                for( int y = 0; y < 4; y++ )
                {
#pragma unroll
                    for( int x = 0; x < 4; x++ )
                        d[y][x] = upix<BD>( fr[by + y][x / PPD], x % PPD ) - upix<BD>( rr[by + y][x / PPD], x % PPD );
                    int t0 = d[y][0] + d[y][1], t1 = d[y][0] - d[y][1], t2 = d[y][2] + d[y][3], t3 = d[y][2] - d[y][3];
                    d[y][0] = t0 + t2; d[y][2] = t0 - t2; d[y][1] = t1 + t3; d[y][3] = t1 - t3;
                }
                int s4 = 0;
#pragma unroll
                for( int x = 0; x < 4; x++ )
                {
                    int t0 = d[0][x] + d[1][x], t1 = d[0][x] - d[1][x], t2 = d[2][x] + d[3][x], t3 = d[2][x] - d[3][x];
                    s4 += abs( t0 + t2 ) + abs( t0 - t2 ) + abs( t1 + t3 ) + abs( t1 - t3 );
                }
                sum += s4 >> 1;
            }
        }
    }
    if constexpr( OP == 0 )
        sum = (int)acc;
    else if constexpr( W >= 8 )
        sum = (int)(acc >> 1);
    return sum;
}

template <int BD, int OP, int IPIX, int LD>
__global__ __launch_bounds__( 256 ) void subpel_cmp3_kernel( const typename PT<BD>::pixel *__restrict__ fenc,
                                                             intptr_t fs, const typename PT<BD>::pixel *p0,
                                                             const typename PT<BD>::pixel *p1,
                                                             const typename PT<BD>::pixel *p2,
                                                             const typename PT<BD>::pixel *p3, intptr_t rs,
                                                             const int64_t *__restrict__ fenc_off,
                                                             const int32_t *__restrict__ qxy, int n,
                                                             int32_t *__restrict__ scores )
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if( i >= n )
        return;
    const int2 q = *(const int2 *)(qxy + 2 * i);
    scores[i] = subpel_score<BD, OP, IPIX, LD>( fenc + fenc_off[i], fs, p0, p1, p2, p3, rs, q.x, q.y );
}

// ------------------------------------------------------------ qpel neighbourhood of an hpel centre
// x264hip_*_subpel_qpel9_batch: for block i the 3x3 quarter-pel neighbourhood (dx, dy in
// -1..1) of a centre (cx, cy) -- refine_subpel's first quarter-pel diamond and its corners
// (encoder/me.c:950-963), each candidate get_ref (common/mc.c:221-249) + SAD / SATD.
//
// In half-pel grid units the four planes are one grid G(u, v) = plane[(v & 1) * 2 + (u & 1)]
// at pixel (u >> 1, v >> 1) (F, H, V, C; mc.c:173-196).  For a half-pel centre (cx, cy even,
// hx = cx / 2, hy = cy / 2) every candidate pixel (column k, row j of the block) is G at
// (hx + 2k + {-1, 0, 1}, hy + 2j + {-1, 0, 1}) or the rounded average of two such samples,
// x264_hpel_ref0/1 (common/tables.c:183-184) read as: the axial candidates average the centre
// sample with its half-pel neighbour, and a diagonal candidate averages {centre, diagonal
// neighbour} when the centre's quarter-pel phases differ ((cx ^ cy) & 2) and {horizontal,
// vertical neighbour} otherwise -- for all nine candidates of the lane.  So one lane loads four
// register windows once (the centre samples, the horizontal / vertical / diagonal neighbour
// samples: 8 x 8, 9 x 8, 8 x 9, 9 x 9 pixels per 8 x 8 tile of the block, streamed in 4-row
// bands) from its own planes -- the plane choice is a per-lane pointer, not a branch -- and
// forms all nine predictions in registers: ~5 aligned loads per candidate against 24
// unaligned ones when each candidate is fetched on its own (subpel_cmp_batch).  A quarter-pel
// centre (odd cx or cy) takes the per-candidate path for its lane.
template <int BD>
__device__ __forceinline__ const typename PT<BD>::pixel *hpel_grid( const typename PT<BD>::pixel *p0,
                                                                    const typename PT<BD>::pixel *p1,
                                                                    const typename PT<BD>::pixel *p2,
                                                                    const typename PT<BD>::pixel *p3, intptr_t rs,
                                                                    int u, int v )
{
    const int pl = ((v & 1) << 1) | (u & 1);
    const typename PT<BD>::pixel *b = pl == 0 ? p0 : pl == 1 ? p1 : pl == 2 ? p2 : p3;
    return b + (intptr_t)(v >> 1) * rs + (u >> 1);
}

template <int BD, int OP, int IPIX>
__global__ __launch_bounds__( 256 ) void subpel_qpel9_kernel( const typename PT<BD>::pixel *__restrict__ fenc,
                                                              intptr_t fs, const typename PT<BD>::pixel *p0,
                                                              const typename PT<BD>::pixel *p1,
                                                              const typename PT<BD>::pixel *p2,
                                                              const typename PT<BD>::pixel *p3, intptr_t rs,
                                                              const int64_t *__restrict__ fenc_off,
                                                              const int32_t *__restrict__ cxy, int n,
                                                              int32_t *__restrict__ scores )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int PPD = PT<BD>::PPD;
    constexpr int W = pix_w( IPIX ), H = pix_h( IPIX );
    constexpr int N8 = 8 / PPD;                       // dwords of 8 pixels
    constexpr int SH = BD == 8 ? 1 : 2;               // bytes of one pixel
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if( i >= n )
        return;
    const int2 c = *(const int2 *)(cxy + 2 * i);
    const pixel *a = fenc + fenc_off[i];
    int32_t *out = scores + (int64_t)9 * i;
    if( (c.x | c.y) & 1 )
    {
        for( int k = 0; k < 9; k++ )
            out[k] = subpel_score<BD, OP, IPIX, 1>( a, fs, p0, p1, p2, p3, rs, c.x + k % 3 - 1, c.y + k / 3 - 1 );
        return;
    }
    const int hx = c.x >> 1, hy = c.y >> 1;
    const bool ccxy = (c.x ^ c.y) & 2;
    const pixel *gcc = hpel_grid<BD>( p0, p1, p2, p3, rs, hx, hy );
    const pixel *gxc = hpel_grid<BD>( p0, p1, p2, p3, rs, hx - 1, hy );
    const pixel *gcy = hpel_grid<BD>( p0, p1, p2, p3, rs, hx, hy - 1 );
    const pixel *gxy = hpel_grid<BD>( p0, p1, p2, p3, rs, hx - 1, hy - 1 );
    uint32_t acc[9];
#pragma unroll
    for( int k = 0; k < 9; k++ )
        acc[k] = 0;
#pragma unroll
    for( int ty = 0; ty < H; ty += 4 )
#pragma unroll
        for( int tx = 0; tx < W; tx += 8 )
        {
            uint32_t f[4][N8], cc[4][N8], xc[4][N8 + 1], cy[5][N8], xy[5][N8 + 1];
#pragma unroll
            for( int y = 0; y < 4; y++ )
            {
                load_row_al<N8>( a + (ty + y) * fs + tx, f[y] );
                load_row_al<N8>( gcc + (ty + y) * rs + tx, cc[y] );
                load_row_al<N8 + 1>( gxc + (ty + y) * rs + tx, xc[y] );
            }
#pragma unroll
            for( int y = 0; y < 5; y++ )
            {
                load_row_al<N8>( gcy + (ty + y) * rs + tx, cy[y] );
                load_row_al<N8 + 1>( gxy + (ty + y) * rs + tx, xy[y] );
            }
            // SATD: the fenc tile's biased Hadamards once for the nine candidates (had8x4_biased)
            uint32_t hf[16];
            if constexpr( OP != 0 )
                had8x4_biased<BD>( f, hf );
#pragma unroll
            for( int k = 0; k < 9; k++ )
            {
                const int dx = k % 3 - 1, dy = k / 3 - 1;
                uint32_t pr[4][N8];
#pragma unroll
                for( int r = 0; r < 4; r++ )
#pragma unroll
                    for( int d = 0; d < N8; d++ )
                    {
                        const int ry = r + (dy > 0);
                        const uint32_t cv = cc[r][d];
                        const uint32_t xs = dx < 0 ? xc[r][d] : __builtin_amdgcn_alignbyte( xc[r][d + 1], xc[r][d], SH );
                        const uint32_t ys = cy[ry][d];
                        const uint32_t ds = dx < 0 ? xy[ry][d] : __builtin_amdgcn_alignbyte( xy[ry][d + 1], xy[ry][d], SH );
                        uint32_t v;
                        if( dx == 0 && dy == 0 )
                            v = cv;
                        else if( dy == 0 )
                            v = avg_round<BD>( cv, xs );
                        else if( dx == 0 )
                            v = avg_round<BD>( cv, ys );
                        else    // the operands chosen per lane, one average (not two and a select)
                            v = avg_round<BD>( ccxy ? cv : xs, ccxy ? ds : ys );
                        pr[r][d] = v;
                    }
                if constexpr( OP == 0 )
                {
#pragma unroll
                    for( int r = 0; r < 4; r++ )
#pragma unroll
                        for( int d = 0; d < N8; d++ )
                            acc[k] = sadp<BD>( f[r][d], pr[r][d], acc[k] );
                }
                else
                {
                    uint32_t o[16];
                    had8x4_biased<BD>( pr, o );
#pragma unroll
                    for( int q = 0; q < 16; q++ )
                        acc[k] = __builtin_amdgcn_sad_u16( o[q], hf[q], acc[k] );
                }
            }
        }
#pragma unroll
    for( int k = 0; k < 9; k++ )
        out[k] = OP == 0 ? (int)acc[k] : (int)(acc[k] >> 1);
}

template <int BD>
hipError_t launch_subpel_qpel9( int op, int i_pixel, const typename PT<BD>::pixel *fenc, intptr_t fs,
                                const typename PT<BD>::pixel *const planes[4], intptr_t rs, const int64_t *fenc_off,
                                const int32_t *cxy, int n, int32_t *scores, hipStream_t stream )
{
    if( n <= 0 )
        return hipSuccess;
    dim3 blk( 256 ), g( (n + 255) / 256 );
#define Q9_CASE( OP, I )                                                                                       \
    case I:                                                                                                    \
        hipLaunchKernelGGL( ( subpel_qpel9_kernel<BD, OP, I> ), g, blk, 0, stream, fenc, fs, planes[0], planes[1], \
                            planes[2], planes[3], rs, fenc_off, cxy, n, scores );                              \
        break;
    if( op == 0 )
    {
        switch( i_pixel ) { Q9_CASE( 0, 0 ) Q9_CASE( 0, 1 ) Q9_CASE( 0, 2 ) Q9_CASE( 0, 3 ) default: return hipErrorInvalidValue; }
    }
    else if( op == 2 )
    {
        switch( i_pixel ) { Q9_CASE( 2, 0 ) Q9_CASE( 2, 1 ) Q9_CASE( 2, 2 ) Q9_CASE( 2, 3 ) default: return hipErrorInvalidValue; }
    }
    else
        return hipErrorInvalidValue;
#undef Q9_CASE
    return hipGetLastError();
}

template <int BD>
hipError_t launch_subpel_cmp( int op, int i_pixel, const typename PT<BD>::pixel *fenc, intptr_t fs,
                              const typename PT<BD>::pixel *const planes[4], intptr_t rs, const int64_t *fenc_off,
                              const int32_t *qxy, int n, int32_t *scores, hipStream_t stream )
{
    if( n <= 0 )
        return hipSuccess;
    dim3 blk( 256 ), g( (n + 255) / 256 );
    // the row loads (a round-2 A/B over 4.7 M 8x8 SATD candidates of bench.py's list; the A/B driver was removed
    // with the losing variants):
    // unaligned multi-dword loads at 8 bit (0.101 ms against 0.115 for dword-aligned loads +
    // alignbyte, and 0.129 for the first dwordx2 + dword kernel), dword-aligned loads +
    // alignbyte at 10 bit (0.186 against 0.193; 0.178 against 0.276 on block-major lists)
    constexpr int LD = BD == 8 ? 0 : 1;
#define SP_CASE( OP, I )                                                                                      \
    case I:                                                                                                   \
        hipLaunchKernelGGL( ( subpel_cmp3_kernel<BD, OP, I, LD> ), g, blk, 0, stream, fenc, fs, planes[0],    \
                            planes[1], planes[2], planes[3], rs, fenc_off, qxy, n, scores );                  \
        break;
    if( op == 0 )
    {
        switch( i_pixel ) { SP_CASE( 0, 0 ) SP_CASE( 0, 1 ) SP_CASE( 0, 2 ) SP_CASE( 0, 3 ) SP_CASE( 0, 4 )
                            SP_CASE( 0, 5 ) SP_CASE( 0, 6 ) SP_CASE( 0, 7 ) default: return hipErrorInvalidValue; }
    }
    else if( op == 2 )
    {
        switch( i_pixel ) { SP_CASE( 2, 0 ) SP_CASE( 2, 1 ) SP_CASE( 2, 2 ) SP_CASE( 2, 3 ) SP_CASE( 2, 4 )
                            SP_CASE( 2, 5 ) SP_CASE( 2, 6 ) SP_CASE( 2, 7 ) default: return hipErrorInvalidValue; }
    }
    else
        return hipErrorInvalidValue;
#undef SP_CASE
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// x264_frame_init_lowres (mc.c:458-482): frame_init_lowres_core's four
// half-resolution planes (mc.c:484-507, FILTER = nested rounding averages)
// over the core [0, W/2) x [0, H/2) plus the 32-pixel border replication of
// x264_frame_expand_border_lowres (frame.c:627-631), in one pass: a border
// pixel takes the value of the clamped core pixel.  The source column W and
// row H, which the reference duplicates from W-1 / H-1 before filtering, are
// read through the same clamp.  One lane per PPD output pixels (one dword of
// each plane).
template <int BD>
__global__ __launch_bounds__( 256 ) void lowres_kernel( const typename PT<BD>::pixel *src, intptr_t stride,
                                                        intptr_t fstride, int width, int height,
                                                        typename PT<BD>::pixel *d0, typename PT<BD>::pixel *dh,
                                                        typename PT<BD>::pixel *dv, typename PT<BD>::pixel *dc,
                                                        intptr_t ds, intptr_t dfs )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int PPD = PT<BD>::PPD, PAD = 32;
    const int wl = width / 2, hl = height / 2;
    const int gw = (wl + 2 * PAD) / PPD;                   // dword groups per output row
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = (int)blockIdx.y - PAD;
    if( g >= gw )
        return;
    const int f = blockIdx.z;
    const pixel *s = src + f * fstride;
    const int yc = min( max( y, 0 ), hl - 1 );
    const pixel *r0 = s + (intptr_t)(2 * yc) * stride;
    const pixel *r1 = s + (intptr_t)min( 2 * yc + 1, height - 1 ) * stride;
    const pixel *r2 = s + (intptr_t)min( 2 * yc + 2, height - 1 ) * stride;
    uint32_t w0 = 0, wh = 0, wv = 0, wc = 0;
#define FILTER( a, b, c, d ) ((((a + b + 1) >> 1) + ((c + d + 1) >> 1) + 1) >> 1)
    const int xg = g * PPD - PAD;                            // first output column of the lane
    if( xg >= 0 && xg + PPD <= wl - 1 && 2 * yc + 2 <= height - 1 )
    {
        // unclamped: source columns 2*xg .. 2*xg + 2*PPD as aligned dwords of three rows
        constexpr int ND = 2 * PPD / PPD + 1;                // dwords covering 2*PPD + 1 pixels
        uint32_t q0[ND], q1[ND], q2[ND];
#pragma unroll
        for( int k = 0; k < ND; k++ )
        {
            q0[k] = ((const uint32_t *)(r0 + 2 * xg))[k];
            q1[k] = ((const uint32_t *)(r1 + 2 * xg))[k];
            q2[k] = ((const uint32_t *)(r2 + 2 * xg))[k];
        }
#pragma unroll
        for( int j = 0; j < PPD; j++ )
        {
            const int i0 = 2 * j, i1 = 2 * j + 1, i2 = 2 * j + 2;
            const int a0 = upix<BD>( q0[i0 / PPD], i0 % PPD ), a1 = upix<BD>( q0[i1 / PPD], i1 % PPD ),
                      a2 = upix<BD>( q0[i2 / PPD], i2 % PPD );
            const int b0 = upix<BD>( q1[i0 / PPD], i0 % PPD ), b1 = upix<BD>( q1[i1 / PPD], i1 % PPD ),
                      b2 = upix<BD>( q1[i2 / PPD], i2 % PPD );
            const int e0 = upix<BD>( q2[i0 / PPD], i0 % PPD ), e1 = upix<BD>( q2[i1 / PPD], i1 % PPD ),
                      e2 = upix<BD>( q2[i2 / PPD], i2 % PPD );
            const int sh = j * (32 / PPD);
            w0 |= (uint32_t)FILTER( a0, b0, a1, b1 ) << sh;
            wh |= (uint32_t)FILTER( a1, b1, a2, b2 ) << sh;
            wv |= (uint32_t)FILTER( b0, e0, b1, e1 ) << sh;
            wc |= (uint32_t)FILTER( b1, e1, b2, e2 ) << sh;
        }
    }
    else
    {
#pragma unroll
        for( int j = 0; j < PPD; j++ )
        {
            const int x = xg + j;
            const int xc = min( max( x, 0 ), wl - 1 );
            const int c0 = 2 * xc, c1 = min( 2 * xc + 1, width - 1 ), c2 = min( 2 * xc + 2, width - 1 );
            const int a0 = r0[c0], a1 = r0[c1], a2 = r0[c2];
            const int b0 = r1[c0], b1 = r1[c1], b2 = r1[c2];
            const int e0 = r2[c0], e1 = r2[c1], e2 = r2[c2];
            const int sh = j * (32 / PPD);
            w0 |= (uint32_t)FILTER( a0, b0, a1, b1 ) << sh;
            wh |= (uint32_t)FILTER( a1, b1, a2, b2 ) << sh;
            wv |= (uint32_t)FILTER( b0, e0, b1, e1 ) << sh;
            wc |= (uint32_t)FILTER( b1, e1, b2, e2 ) << sh;
        }
    }
#undef FILTER
    const intptr_t o = f * dfs + (intptr_t)y * ds + g * PPD - PAD;
    *(uint32_t *)(d0 + o) = w0;
    *(uint32_t *)(dh + o) = wh;
    *(uint32_t *)(dv + o) = wv;
    *(uint32_t *)(dc + o) = wc;
}

// 8 bit, default: one single-wave workgroup per R output rows of all four planes.
// Lane k < wl/16 makes output columns 16k .. 16k+15: its three source rows arrive as
// 33-pixel runs (two aligned 16-byte loads and a dword), v_perm gathers the even / odd /
// next-even columns, and FILTER(a, b, c, d) = avg( avg( a, b ), avg( c, d ) ) with
// avg = (x + y + 1) >> 1 per byte is v_lerp_u8 -- ten per output dword-quad, bit-exact --
// so each plane row leaves as one 16-byte store per lane.  In the last
// group the source column 2*16k+32 the run ends on would be column W, which the
// reference duplicates from W-1 (mc.c:465-468), so that one byte is taken from W-1.
// The wl % 16 columns left over (widths that are not a multiple of 32) go to the next
// lanes through the clamped per-pixel form, four columns each.  The 32-pixel borders
// are replicas of columns 0 and wl-1 (plane_expand_border, frame.c:627-631), stored by
// the lanes that hold those columns: no border wave, every lane's loads for its R rows
// independent of the other rows.
template <int R, bool NT = false>
__device__ __forceinline__ void lowres_rows_body( const uint8_t *__restrict__ src, intptr_t stride, intptr_t fstride,
                                                  int width, int height, uint8_t *__restrict__ d0,
                                                  uint8_t *__restrict__ dh, uint8_t *__restrict__ dv,
                                                  uint8_t *__restrict__ dc, intptr_t ds, intptr_t dfs, int by, int f )
{
    constexpr int PAD = 32;
    const int wl = width / 2, hl = height / 2;
    const uint8_t *s = src + f * fstride;
    const int nfull = wl / 16;
    const int nrem = (wl - 16 * nfull + 3) / 4;               // clamped groups of 4 columns
    uint8_t *const dst[4] = { d0, dh, dv, dc };
    auto splat = []( uint32_t w, int byte ) { return __builtin_amdgcn_perm( 0u, w, 0x01010101u * (uint32_t)byte ); };
    for( int k = threadIdx.x; k < nfull + nrem; k += 64 )
    {
#pragma unroll
        for( int rr = 0; rr < R; rr++ )
        {
            const int y = by * R + rr - PAD;
            const bool live = y < hl + PAD;
            const int yc = min( max( y, 0 ), hl - 1 );
            const uint8_t *r0 = s + (intptr_t)(2 * yc) * stride;
            const uint8_t *r1 = s + (intptr_t)min( 2 * yc + 1, height - 1 ) * stride;
            const uint8_t *r2 = s + (intptr_t)min( 2 * yc + 2, height - 1 ) * stride;
            const intptr_t orow = f * dfs + (intptr_t)y * ds;
            if( k < nfull )
            {
                const int xg = 16 * k;
                const bool edge = 2 * xg + 32 >= width;      // the run's last column is W: take W-1
                uint32_t E[3][5], O[3][4];
                const uint8_t *rp[3] = { r0, r1, r2 };
#pragma unroll
                for( int r = 0; r < 3; r++ )
                {
                    const uint4 a = *(const uint4 *)(rp[r] + 2 * xg), b = *(const uint4 *)(rp[r] + 2 * xg + 16);
                    const uint32_t v[8] = { a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w };
#pragma unroll
                    for( int j = 0; j < 4; j++ )
                    {
                        E[r][j] = __builtin_amdgcn_perm( v[2 * j + 1], v[2 * j], 0x06040200u );
                        O[r][j] = __builtin_amdgcn_perm( v[2 * j + 1], v[2 * j], 0x07050301u );
                    }
                    E[r][4] = edge ? b.w >> 24 : *(const uint32_t *)(rp[r] + 2 * xg + 32);
                }
                uint32_t w[4][4];
#pragma unroll
                for( int j = 0; j < 4; j++ )
                {
                    auto avg = []( uint32_t p, uint32_t q ) { return __builtin_amdgcn_lerp( p, q, 0x01010101u ); };
                    const uint32_t x0 = __builtin_amdgcn_alignbyte( E[0][j + 1], E[0][j], 1 );
                    const uint32_t x1 = __builtin_amdgcn_alignbyte( E[1][j + 1], E[1][j], 1 );
                    const uint32_t x2 = __builtin_amdgcn_alignbyte( E[2][j + 1], E[2][j], 1 );
                    const uint32_t e01 = avg( E[0][j], E[1][j] ), o01 = avg( O[0][j], O[1][j] ), x01 = avg( x0, x1 );
                    const uint32_t e12 = avg( E[1][j], E[2][j] ), o12 = avg( O[1][j], O[2][j] ), x12 = avg( x1, x2 );
                    w[0][j] = avg( e01, o01 );
                    w[1][j] = avg( o01, x01 );
                    w[2][j] = avg( e12, o12 );
                    w[3][j] = avg( o12, x12 );
                }
                if( live )
                {
                    const intptr_t o = orow + xg;
#pragma unroll
                    for( int pl = 0; pl < 4; pl++ )
                    {
                        st16<NT>( dst[pl] + o, make_uint4( w[pl][0], w[pl][1], w[pl][2], w[pl][3] ) );
                        if( k == 0 )
                        {
                            // left border: column 0 repeated over x in [-32, 0)
                            const uint32_t bb = splat( w[pl][0], 0 );
                            st16<NT>( dst[pl] + orow - 32, make_uint4( bb, bb, bb, bb ) );
                            st16<NT>( dst[pl] + orow - 16, make_uint4( bb, bb, bb, bb ) );
                        }
                        if( k == nfull - 1 && !nrem )
                        {
                            // right border: column wl-1 repeated over x in [wl, wl+32)
                            const uint32_t bb = splat( w[pl][3], 3 );
                            st16<NT>( dst[pl] + o + 16, make_uint4( bb, bb, bb, bb ) );
                            st16<NT>( dst[pl] + o + 32, make_uint4( bb, bb, bb, bb ) );
                        }
                    }
                }
            }
            else
            {
                const int xg = 16 * nfull + 4 * (k - nfull);
                uint32_t w[4] = { 0, 0, 0, 0 };
#define FILTER( a, b, c, d ) ((((a + b + 1) >> 1) + ((c + d + 1) >> 1) + 1) >> 1)
#pragma unroll
                for( int j = 0; j < 4; j++ )
                {
                    const int xc = min( xg + j, wl - 1 );
                    const int c0 = 2 * xc, c1 = min( 2 * xc + 1, width - 1 ), c2 = min( 2 * xc + 2, width - 1 );
                    const int a0 = r0[c0], a1 = r0[c1], a2 = r0[c2];
                    const int b0 = r1[c0], b1 = r1[c1], b2 = r1[c2];
                    const int e0 = r2[c0], e1 = r2[c1], e2 = r2[c2];
                    w[0] |= (uint32_t)FILTER( a0, b0, a1, b1 ) << (8 * j);
                    w[1] |= (uint32_t)FILTER( a1, b1, a2, b2 ) << (8 * j);
                    w[2] |= (uint32_t)FILTER( b0, e0, b1, e1 ) << (8 * j);
                    w[3] |= (uint32_t)FILTER( b1, e1, b2, e2 ) << (8 * j);
                }
#undef FILTER
                if( live )
                {
                    const bool last = k == nfull + nrem - 1;
                    const int nv = wl - xg;                  // valid columns of this group (1..4)
#pragma unroll
                    for( int pl = 0; pl < 4; pl++ )
                    {
                        uint32_t v = w[pl];
                        if( last )
                        {
                            // columns past wl - 1 repeat it: fill the group, then x in [xg+4, wl+32)
                            const uint32_t bb = splat( v, nv - 1 );
                            v = nv >= 4 ? v : (v & (0xFFFFFFFFu >> (8 * (4 - nv)))) | (bb & (0xFFFFFFFFu << (8 * nv)));
                            for( int x = xg + 4; x < wl + PAD; x += 4 )
                                *(uint32_t *)(dst[pl] + orow + x) = bb;
                        }
                        *(uint32_t *)(dst[pl] + orow + xg) = v;
                    }
                }
            }
        }
    }
}

template <int R, bool NT = false>
__global__ __launch_bounds__( 64 ) void lowres_rows_kernel( const uint8_t *__restrict__ src, intptr_t stride,
                                                            intptr_t fstride, int width, int height,
                                                            uint8_t *__restrict__ d0, uint8_t *__restrict__ dh,
                                                            uint8_t *__restrict__ dv, uint8_t *__restrict__ dc,
                                                            intptr_t ds, intptr_t dfs, int xcd )
{
    const Blk3 B = blk3( xcd );
    lowres_rows_body<R, NT>( src, stride, fstride, width, height, d0, dh, dv, dc, ds, dfs, (int)B.y, (int)B.z );
}

template <int BD>
hipError_t launch_frame_init_lowres( const typename PT<BD>::pixel *src, intptr_t stride, intptr_t fstride, int width,
                                     int height, int nframes, typename PT<BD>::pixel *const dst[4], intptr_t ds,
                                     intptr_t dfs, hipStream_t st )
{
    if( nframes <= 0 )
        return hipSuccess;
    const int wl = width / 2, hl = height / 2;
    if constexpr( BD == 8 )
    {
        // 16-pixel lanes with 16-byte loads and stores, two output rows per wave (one / four
        // rows, the one-row-per-workgroup kernel and a persistent grid were all slower,
        // profiles/r02h_lowres_variants*.json, r03i_stream_var.json): needs 16-byte aligned
        // rows and a width of whole macroblocks; else the dword kernel below
        const uintptr_t al = (uintptr_t)src | (uintptr_t)stride | (uintptr_t)fstride | (uintptr_t)dst[0] |
                             (uintptr_t)dst[1] | (uintptr_t)dst[2] | (uintptr_t)dst[3] | (uintptr_t)ds | (uintptr_t)dfs;
        if( !(al & 15) && !(width & 15) )
        {
            dim3 gr( 1, (unsigned)((hl + 64 + 1) / 2), (unsigned)nframes );
            if( stream_nt() )
                // nontemporal stores + XCD-contiguous row blocks (which lost with plain stores):
                // 64 frames 0.0789 -> 0.0510 ms, 16 frames 0.0165 -> 0.0145 ms
                // (profiles/r03r_stream_nt.json)
                hipLaunchKernelGGL( ( lowres_rows_kernel<2, true> ), gr, dim3( 64 ), 0, st, src, stride, fstride, width,
                                    height, dst[0], dst[1], dst[2], dst[3], ds, dfs, variant( V_STREAM_XCD ) != 0 );
            else
                hipLaunchKernelGGL( lowres_rows_kernel<2>, gr, dim3( 64 ), 0, st, src, stride, fstride, width, height,
                                    dst[0], dst[1], dst[2], dst[3], ds, dfs, variant( V_STREAM_XCD ) == 1 );
            return hipGetLastError();
        }
    }
    const int gw = (wl + 64) / PT<BD>::PPD;
    dim3 blk( 256 ), g( (unsigned)((gw + 255) / 256), (unsigned)(hl + 64), (unsigned)nframes );
    hipLaunchKernelGGL( lowres_kernel<BD>, g, blk, 0, st, src, stride, fstride, width, height, dst[0], dst[1], dst[2],
                        dst[3], ds, dfs );
    return hipGetLastError();
}

#define INST( BD )                                                                                              \
    template hipError_t launch_hpel_filter<BD>( const PT<BD>::pixel *, PT<BD>::pixel *, PT<BD>::pixel *,       \
                                                PT<BD>::pixel *, intptr_t, intptr_t, int, int, int, hipStream_t ); \
    template hipError_t launch_subpel_cmp<BD>( int, int, const PT<BD>::pixel *, intptr_t,                      \
                                               const PT<BD>::pixel *const[4], intptr_t, const int64_t *,       \
                                               const int32_t *, int, int32_t *, hipStream_t );      \
    template hipError_t launch_subpel_qpel9<BD>( int, int, const PT<BD>::pixel *, intptr_t,                    \
                                                 const PT<BD>::pixel *const[4], intptr_t, const int64_t *,     \
                                                 const int32_t *, int, int32_t *, hipStream_t );               \
    template hipError_t launch_frame_init_lowres<BD>( const PT<BD>::pixel *, intptr_t, intptr_t, int, int, int,  \
                                                      PT<BD>::pixel *const[4], intptr_t, intptr_t, hipStream_t );
INST( 8 )
INST( 10 )

} // namespace x264hip

namespace x264hip {

// ---------------------------------------------------------------------------
// Frame upload from page-locked host memory (configs[3]'s streaming form): the
// GPU reads the pinned pages itself over PCIe, 16-byte pieces with four loads in
// flight per lane, instead of one SDMA engine copy.  Ragged head / tail bytes go
// one per lane.
__global__ __launch_bounds__( 256 ) void upload_kernel( uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
                                                        size_t n16, size_t bytes )
{
    const size_t nthr = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint4 *s = (const uint4 *)src;
    uint4 *d = (uint4 *)dst;
    for( ; i + 3 * nthr < n16; i += 4 * nthr )
    {
        const uint4 a = s[i], b = s[i + nthr], c = s[i + 2 * nthr], e = s[i + 3 * nthr];
        d[i] = a;
        d[i + nthr] = b;
        d[i + 2 * nthr] = c;
        d[i + 3 * nthr] = e;
    }
    for( ; i < n16; i += nthr )
        d[i] = s[i];
    const size_t t = 16 * n16 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if( t < bytes )
        dst[t] = src[t];
}

// x264_weight_scale_plane (frame.c:825-842) / mc_weight (mc.c:117-137): the weighted copy
// of a plane region for the lookahead's weighted-reference search (slicetype.c:490-499).
// Columns [0, cov) of every row, cov = the reference's strip coverage (16-wide blocks while
// x < width-8, then one 8-wide block: up to 7 columns past width); one lane per 4 pixels.
template <int BD>
__global__ __launch_bounds__( 256 ) void weight_plane_kernel( typename PT<BD>::pixel *__restrict__ dst, intptr_t ds,
                                                              intptr_t dfs, const typename PT<BD>::pixel *__restrict__ src,
                                                              intptr_t ss, intptr_t sfs, int cov, int height, int scale,
                                                              int rnd, int sh, int off )
{
    const int x = 4 * (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int y = (int)blockIdx.y;
    if( x >= cov )
        return;
    const typename PT<BD>::pixel *s = src + (intptr_t)blockIdx.z * sfs + (intptr_t)y * ss + x;
    typename PT<BD>::pixel *d = dst + (intptr_t)blockIdx.z * dfs + (intptr_t)y * ds + x;
    constexpr int PMAX = (1 << BD) - 1;
#pragma unroll
    for( int k = 0; k < 4; k++ )
        if( x + k < cov )
            d[k] = (typename PT<BD>::pixel)min( max( (((int)s[k] * scale + rnd) >> sh) + off, 0 ), PMAX );
}

template <int BD>
hipError_t launch_weight_plane( typename PT<BD>::pixel *dst, intptr_t ds, intptr_t dfs,
                                const typename PT<BD>::pixel *src, intptr_t ss, intptr_t sfs, int width, int height,
                                int nframes, int scale, int denom, int offset, hipStream_t stream )
{
    if( width <= 0 || height <= 0 || nframes <= 0 )
        return hipSuccess;
    int cov = 0;
    while( cov < width - 8 )
        cov += 16;
    if( cov < width )
        cov += 8;
    if( height > 65535 || nframes > 65535 )
        return hipErrorInvalidValue;
    const int rnd = denom >= 1 ? 1 << (denom - 1) : 0, sh = denom >= 1 ? denom : 0;
    hipLaunchKernelGGL( weight_plane_kernel<BD>, dim3( (unsigned)((cov + 1023) / 1024), (unsigned)height,
                                                       (unsigned)nframes ),
                        dim3( 256 ), 0, stream, dst, ds, dfs, src, ss, sfs, cov, height, scale, rnd, sh,
                        offset * (1 << (BD - 8)) );
    return hipGetLastError();
}
template hipError_t launch_weight_plane<8>( uint8_t *, intptr_t, intptr_t, const uint8_t *, intptr_t, intptr_t, int,
                                            int, int, int, int, int, hipStream_t );
template hipError_t launch_weight_plane<10>( uint16_t *, intptr_t, intptr_t, const uint16_t *, intptr_t, intptr_t,
                                             int, int, int, int, int, int, hipStream_t );

// ---------------------------------------------------------------------------
// A picture plane from page-locked host memory into a padded frame plane: x264_frame_copy_
// picture's plane copy (common/frame.c:393-521) fused with plane_expand_border (frame.c:535-554,
// as x264_frame_expand_border / _chroma run it over a whole frame), so the link carries the
// picture's own bytes and the pads are written from the registers that hold the edge.  Lane i
// of the grid-stride loop moves 16-byte chunk i of the w16 x h chunk grid (four in flight per
// lane, as upload_kernel); the chunk at a row's left / right end also writes its row's pad
// band (the edge element of `unit` bytes repeated: 1 or 2 for luma, 2 or 4 for an NV12 /
// NV16 plane), and rows 0 / h-1 are written again into the pad_y rows above / below (the
// padded rows, corners included).
__device__ __forceinline__ uint4 unit_fill( uint4 v, int unit, bool last )
{
    // the first (last = false) or last element of v, repeated over 16 bytes
    uint32_t w = last ? v.w : v.x;
    if( unit == 1 )
        w = last ? (w >> 24) * 0x01010101u : (w & 0xff) * 0x01010101u;
    else if( unit == 2 )
        w = last ? (w >> 16) * 0x00010001u : (w & 0xffff) * 0x00010001u;
    return make_uint4( w, w, w, w );
}

// up to three planes of one picture per launch (luma + NV12, or Y, U, V): one chunk grid over
// all of them, so the link never drains between planes
struct UpPlanes
{
    uint8_t *dst[3];
    const uint8_t *src[3];
    intptr_t ds[3], ss[3];
    uint32_t w16[3], h[3], end[3];      // chunks per row, rows, cumulative chunk count
    uint32_t unit[3], padx16[3], pad_y[3];
    int n;
};

// (the plane's fields by select, never by a dynamic index: indexing the kernel-argument arrays
// copies them to scratch memory)
template <typename T> __device__ __forceinline__ T psel( const T (&a)[3], int k ) { return k == 0 ? a[0] : k == 1 ? a[1] : a[2]; }

__global__ __launch_bounds__( 256 ) void upload_plane_kernel( const UpPlanes P )
{
    const uint32_t total = P.end[2], nthr = gridDim.x * blockDim.x;
    // plane, row and column of chunk i (32-bit index math: a 2160p picture is 0.78 M chunks)
    auto locate = [&]( uint32_t i, int &k, uint32_t &y, uint32_t &c ) __attribute__( ( always_inline ) ) {
        k = i >= P.end[0] ? (i >= P.end[1] ? 2 : 1) : 0;
        const uint32_t j = i - (k == 0 ? 0u : k == 1 ? P.end[0] : P.end[1]), w = psel( P.w16, k );
        y = j / w;
        c = j - y * w;
    };
    auto get = [&]( uint32_t i ) __attribute__( ( always_inline ) ) {
        int k;
        uint32_t y, c;
        locate( i, k, y, c );
        return *((const uint4 *)(psel( P.src, k ) + (intptr_t)y * psel( P.ss, k )) + c);
    };
    auto put = [&]( uint32_t i, uint4 v ) __attribute__( ( always_inline ) ) {
        int k;
        uint32_t y, c;
        locate( i, k, y, c );
        const int h = (int)psel( P.h, k ), py = (int)psel( P.pad_y, k ), px = (int)psel( P.padx16, k );
        const int y0 = y == 0 ? -py : (int)y, y1 = (int)y == h - 1 ? h - 1 + py : (int)y;
        const bool l = c == 0, r = c == psel( P.w16, k ) - 1;
        const int unit = (int)psel( P.unit, k );
        const uint4 fl = l ? unit_fill( v, unit, false ) : v;
        const uint4 fr = r ? unit_fill( v, unit, true ) : v;
        uint8_t *const dk = psel( P.dst, k );
        const intptr_t dsk = psel( P.ds, k );
        for( int yy = y0; yy <= y1; yy++ )
        {
            uint4 *d = (uint4 *)(dk + (intptr_t)yy * dsk) + c;
            *d = v;
            if( l )
                for( int q = 1; q <= px; q++ )
                    d[-q] = fl;
            if( r )
                for( int q = 1; q <= px; q++ )
                    d[q] = fr;
        }
    };
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    for( ; i + 3 * nthr < total; i += 4 * nthr )
    {
        const uint4 a = get( i ), b = get( i + nthr ), c = get( i + 2 * nthr ), e = get( i + 3 * nthr );
        put( i, a );
        put( i + nthr, b );
        put( i + 2 * nthr, c );
        put( i + 3 * nthr, e );
    }
    for( ; i < total; i += nthr )
        put( i, get( i ) );
}

hipError_t launch_upload_planes( int n, const UploadPlane *pl, hipStream_t stream )
{
    if( n < 1 || n > 3 )
        return hipErrorInvalidValue;
    UpPlanes P = {};
    uint64_t total = 0;
    for( int k = 0; k < n; k++ )
    {
        const UploadPlane &q = pl[k];
        if( q.width_bytes <= 0 || q.height <= 0 || ((q.width_bytes | q.pad_x | (int)(q.ds & 15) | (int)(q.ss & 15)) & 15) ||
            (((uintptr_t)q.dst | (uintptr_t)q.src) & 15) || (q.unit != 1 && q.unit != 2 && q.unit != 4) ||
            q.pad_x < 0 || q.pad_y < 0 )
            return hipErrorInvalidValue;
        P.dst[k] = (uint8_t *)q.dst;
        P.src[k] = (const uint8_t *)q.src;
        P.ds[k] = q.ds;
        P.ss[k] = q.ss;
        P.w16[k] = (uint32_t)(q.width_bytes / 16);
        P.h[k] = (uint32_t)q.height;
        total += (uint64_t)P.w16[k] * P.h[k];
        if( total >= (1ull << 31) )
            return hipErrorInvalidValue;
        P.end[k] = (uint32_t)total;
        P.unit[k] = (uint32_t)q.unit;
        P.padx16[k] = (uint32_t)(q.pad_x / 16);
        P.pad_y[k] = (uint32_t)q.pad_y;
    }
    for( int k = n; k < 3; k++ )
        P.end[k] = (uint32_t)total;
    P.n = n;
    const int wv = variant( V_UPLOAD_WGS );
    // 32 workgroups (two per CU of the copy stream's 16): a 2160p 4:2:0 picture in 0.232 ms
    // against 0.247 with upload_kernel's 16 (profiles/r06f_upload_wgs.txt)
    const size_t cap = wv > 0 ? (size_t)wv : 32;
    const unsigned g = (unsigned)std::min<size_t>( cap, std::max<size_t>( 1, (total + 1023) / 1024 ) );
    hipLaunchKernelGGL( upload_plane_kernel, dim3( g ), dim3( 256 ), 0, stream, P );
    return hipGetLastError();
}

hipError_t launch_upload( void *dst, const void *src, size_t bytes, hipStream_t stream )
{
    if( !bytes )
        return hipSuccess;
    // 16-byte pieces need both ends 16-byte aligned; otherwise the byte path only
    const bool al = !(((uintptr_t)dst | (uintptr_t)src) & 15);
    const size_t n16 = al ? bytes / 16 : 0;
    // 16 grid-stride workgroups (64 waves, 16 B x 4 loads in flight per lane: 256 KB in
    // flight) cover the PCIe round trip: 8.68 MB in 0.156 ms = 55.5 GB/s, against 0.198 ms
    // for one workgroup per 4 KB (profiles/r03b_stream_probe.json), and they leave the rest
    // of the chip to the kernels the upload overlaps.  X264HIP_UPLOAD_WGS overrides the cap.
    const int wv = variant( V_UPLOAD_WGS );
    const size_t cap = wv > 0 ? (size_t)wv : 16;
    const unsigned g = (unsigned)std::min<size_t>( cap, std::max<size_t>( 1, (n16 + 1023) / 1024 ) );
    if( !al && bytes > (size_t)g * 256 )
    {
        hipLaunchKernelGGL( upload_kernel, dim3( (unsigned)((bytes + 255) / 256) ), dim3( 256 ), 0, stream,
                            (uint8_t *)dst, (const uint8_t *)src, (size_t)0, bytes );
        return hipGetLastError();
    }
    hipLaunchKernelGGL( upload_kernel, dim3( g ), dim3( 256 ), 0, stream, (uint8_t *)dst, (const uint8_t *)src, n16,
                        bytes );
    return hipGetLastError();
}

} // namespace x264hip
