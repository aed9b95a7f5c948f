// Weighted-prediction analysis: x264_weights_analyse (reference encoder/slicetype.c:284-501)
// and the frame statistics it reads (encoder/ratecontrol.c:225-257, 406-414).
//
// The reference walks a small (scale, offset) grid one candidate at a time, each candidate
// a full pass over the lowres (luma) or full-resolution (chroma) planes.  Every candidate
// of a plane is fixed before the first cost is known -- the grid comes from the frame
// statistics alone -- so here ONE launch scores the unweighted reference and every
// candidate of the grid (the data is read once per 8-row block group and re-weighted in
// registers per candidate), one D2H copy brings the costs back, and the host replays the
// reference's loop over them, early break and all.  Luma is one launch; chroma (outside
// the lookahead, after a luma weight) one more.
#include "hipcommon.h"
#include "x264hip.h"

#include <math.h>
#include <string.h>

#include <algorithm>

namespace x264hip {

// candidate list of one launch: c = scale | denom << 8 | weighted << 11 | (offset + 256) << 12;
// hdr = weight_slice_header_cost of the candidate (0 when unweighted), added once
struct WpCands
{
    uint32_t c[64];
    uint32_t hdr[64];
    int n;
};

constexpr uint8_t c_hpel_ref0[16] = { 0, 1, 1, 1, 0, 1, 1, 1, 2, 3, 3, 3, 0, 1, 1, 1 };   // common/tables.c:183
constexpr uint8_t c_hpel_ref1[16] = { 0, 0, 1, 0, 2, 2, 3, 2, 2, 2, 3, 2, 2, 2, 3, 2 };   // common/tables.c:184

template <int BD>
__device__ __forceinline__ void wp_row8( const typename PT<BD>::pixel *p, int (&o)[8] )
{
    constexpr int PPD = PT<BD>::PPD, NDW = 8 / PPD;
    uint32_t w[NDW];
    load_al_pad<NDW>( p, w );
#pragma unroll
    for( int k = 0; k < 8; k++ )
        o[k] = upix<BD>( w[k / PPD], k % PPD );
}

// mc_weight's per-pixel op (common/mc.c:117-137): rnd = 1 << (denom-1) or 0 for denom 0
template <int BD>
__device__ __forceinline__ int wp_px( int v, int scale, int denom, int rnd, int off )
{
    return clip_pix<BD>( ((v * scale + rnd) >> denom) + off );
}

__device__ __forceinline__ int dpp_i( int v, int ctrl )
{
    switch( ctrl )   // (the control must be a constant expression)
    {
    case 0xB1: return __builtin_amdgcn_update_dpp( 0, v, 0xB1, 0xF, 0xF, false );   // quad xor 1
    case 0x4E: return __builtin_amdgcn_update_dpp( 0, v, 0x4E, 0xF, 0xF, false );   // quad xor 2
    case 0x141: return __builtin_amdgcn_update_dpp( 0, v, 0x141, 0xF, 0xF, false ); // half mirror: r <-> 7-r
    default: return __builtin_amdgcn_update_dpp( 0, v, 0x140, 0xF, 0xF, false );   // row mirror: r <-> 15-r
    }
}

// The 8x8 block costs of one candidate list.  One wave = 8 blocks (lane = block * 8 + row);
// each lane holds its row of the fenc block and of the (motion-compensated) reference in
// registers and, per candidate, weights the row, takes the differences and either
//  * SATD: a horizontal 4-point Hadamard in the lane, the vertical one across the lane quad
//    (rows 0-3 / 4-7) by DPP, sum |coef| per quad = one 8x4 band, halved, the two bands
//    added (pixel_satd_8x4, common/pixel.c:290-309; satd 8x8 = two bands and satd 16x16 the
//    sum of its four 8x8 blocks' bands), or
//  * SAD over the block,
// caps it at the block's intra cost (luma), sums the wave's blocks and adds the sum to the
// workgroup's LDS accumulator of the candidate; one global atomic per (workgroup,
// candidate) at the end.
//   MV 0: reference at the block (no motion search done, 0x7FFF marker)
//   MV 1: lowres get_ref of lowres_mvs[block] + the block position (weight_cost_init_luma,
//         slicetype.c:77-103; mc_luma common/mc.c:198-219)
//   MV 2: 4:4:4 chroma: full-pel copy at lowres_mvs[MB] / 2 (weight_cost_init_chroma444,
//         slicetype.c:142-168); blocks are the 8x8 quarters of each 16x16 MB
template <int BD, int MV, bool SATD>
__global__ __launch_bounds__( 256 ) void wp_cost8_kernel( const typename PT<BD>::pixel *__restrict__ fenc,
                                                          intptr_t fs, const typename PT<BD>::pixel *r0,
                                                          const typename PT<BD>::pixel *r1,
                                                          const typename PT<BD>::pixel *r2,
                                                          const typename PT<BD>::pixel *r3, intptr_t rs, int bw,
                                                          int bh, const int16_t *__restrict__ mvs, int mvw,
                                                          const uint16_t *__restrict__ intra, WpCands cd,
                                                          uint32_t *__restrict__ out )
{
    __shared__ uint32_t acc[64];
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 7;
    if( tid < 64 )
        acc[tid] = 0;
    __syncthreads();
    const int b0 = (blockIdx.x * 4 + (tid >> 6)) * 8 + (lane >> 3);
    const bool valid = b0 < bw * bh;
    const int b = valid ? b0 : 0;          // invalid lanes read block 0 and contribute nothing
    const int by = b / bw, bx = b - by * bw;
    int f[8], g[8];
    wp_row8<BD>( fenc + (intptr_t)(8 * by + r) * fs + 8 * bx, f );
    if constexpr( MV == 0 )
        wp_row8<BD>( r0 + (intptr_t)(8 * by + r) * rs + 8 * bx, g );
    else if constexpr( MV == 1 )
    {
        const int mvx = mvs[2 * b] + 32 * bx, mvy = mvs[2 * b + 1] + 32 * by;
        const int q = ((mvy & 3) << 2) + (mvx & 3);
        const intptr_t off = (intptr_t)(mvy >> 2) * rs + (mvx >> 2) + (intptr_t)r * rs;
        const typename PT<BD>::pixel *P[4] = { r0, r1, r2, r3 };
        const typename PT<BD>::pixel *s1 = P[field( pack_fields( c_hpel_ref0, 2 ), 2, q )] + off + ((mvy & 3) == 3) * rs;
        constexpr int PPD = PT<BD>::PPD, NDW = 8 / PPD;
        uint32_t w1[NDW];
        load_al_pad<NDW>( s1, w1 );
        if( q & 5 )
        {
            uint32_t w2[NDW];
            load_al_pad<NDW>( P[field( pack_fields( c_hpel_ref1, 2 ), 2, q )] + off + ((mvx & 3) == 3), w2 );
#pragma unroll
            for( int i = 0; i < NDW; i++ )
                w1[i] = avg_round<BD>( w1[i], w2[i] );
        }
#pragma unroll
        for( int k = 0; k < 8; k++ )
            g[k] = upix<BD>( w1[k / PPD], k % PPD );
    }
    else
    {
        const int mb = (by >> 1) * mvw + (bx >> 1);
        const int mvx = mvs[2 * mb] / 2, mvy = mvs[2 * mb + 1] / 2;
        wp_row8<BD>( r0 + (intptr_t)(8 * by + r + mvy) * rs + 8 * bx + mvx, g );
    }
    const uint32_t icap = intra ? (uint32_t)intra[b] : 0xFFFFFFFFu;

    for( int k = 0; k < cd.n; k++ )
    {
        const uint32_t c = cd.c[k];
        const int scale = c & 255, denom = (c >> 8) & 7, wtd = (c >> 11) & 1;
        const int off = (((int)(c >> 12) & 511) - 256) * (1 << (BD - 8));
        const int rnd = denom ? 1 << (denom - 1) : 0;
        int d[8];
#pragma unroll
        for( int i = 0; i < 8; i++ )
            d[i] = (wtd ? wp_px<BD>( g[i], scale, denom, rnd, off ) : g[i]) - f[i];
        uint32_t t = 0;
        if constexpr( SATD )
        {
            int h[8];
#pragma unroll
            for( int j = 0; j < 8; j += 4 )
            {
                const int a0 = d[j] + d[j + 1], a1 = d[j] - d[j + 1], a2 = d[j + 2] + d[j + 3],
                          a3 = d[j + 2] - d[j + 3];
                h[j] = a0 + a2; h[j + 1] = a1 + a3; h[j + 2] = a0 - a2; h[j + 3] = a1 - a3;
            }
#pragma unroll
            for( int i = 0; i < 8; i++ )
            {
                int p = dpp_i( h[i], 0xB1 );
                h[i] = (r & 1) ? p - h[i] : h[i] + p;
                p = dpp_i( h[i], 0x4E );
                h[i] = (r & 2) ? p - h[i] : h[i] + p;
                t += (uint32_t)abs( h[i] );
            }
            t += (uint32_t)dpp_i( (int)t, 0xB1 );
            t += (uint32_t)dpp_i( (int)t, 0x4E );
            t >>= 1;
        }
        else
        {
#pragma unroll
            for( int i = 0; i < 8; i++ )
                t += (uint32_t)abs( d[i] );
            t += (uint32_t)dpp_i( (int)t, 0xB1 );
            t += (uint32_t)dpp_i( (int)t, 0x4E );
        }
        t += (uint32_t)dpp_i( (int)t, 0x141 );
        t = min( t, icap );
        t = (r == 0 && valid) ? t : 0;
        t += __shfl_xor( t, 8 );
        t += __shfl_xor( t, 16 );
        t += __shfl_xor( t, 32 );
        if( lane == 0 )
            atomicAdd( &acc[k], t );
    }
    __syncthreads();
    if( tid < cd.n )
        atomicAdd( out + tid, acc[tid] + (blockIdx.x == 0 ? cd.hdr[tid] : 0u) );
}

// 4:2:0 / 4:2:2 chroma (weight_cost_chroma, slicetype.c:224-255): per 8 x H block (H = 8 /
// 16) of plane `pl` (0 = U, 1 = V), |sum(weighted reference) - sum(fenc)| (pixel_asd8,
// common/pixel.c:747-754).  One lane per block row: the lane deinterleaves its fenc row and
// its reference row -- mc_chroma of lowres_mvs[MB] (common/mc.c:252-283; weight_cost_init_
// chroma, slicetype.c:111-140) or the plane itself -- and the block's rows are summed by DPP.
template <int BD, int H, bool MV>
__global__ __launch_bounds__( 256 ) void wp_chroma_kernel( const typename PT<BD>::pixel *__restrict__ fenc,
                                                           intptr_t fs, const typename PT<BD>::pixel *__restrict__ ref,
                                                           intptr_t rs, int mbw, int mbh,
                                                           const int16_t *__restrict__ mvs, int pl, WpCands cd,
                                                           uint32_t *__restrict__ out )
{
    constexpr int PPD = PT<BD>::PPD;
    __shared__ uint32_t acc[64];
    const int tid = threadIdx.x, lane = tid & 63, r = lane % H;
    if( tid < 64 )
        acc[tid] = 0;
    __syncthreads();
    const int b0 = (blockIdx.x * 4 + (tid >> 6)) * (64 / H) + lane / H;
    const bool valid = b0 < mbw * mbh;
    const int b = valid ? b0 : 0;
    const int by = b / mbw, bx = b - by * mbw;
    int sf = 0;
    {
        constexpr int NDW = 16 / PPD;
        uint32_t w[NDW];
        load_al_pad<NDW>( fenc + (intptr_t)(H * by + r) * fs + 16 * bx, w );
#pragma unroll
        for( int x = 0; x < 8; x++ )
        {
            const int k = 2 * x;   // pixel pl of pair x
            sf += pl ? upix<BD>( w[(k + 1) / PPD], (k + 1) % PPD ) : upix<BD>( w[k / PPD], k % PPD );
        }
    }
    int g[8];
    if constexpr( MV )
    {
        const int mvx = mvs[2 * b], mvy = (2 * mvs[2 * b + 1]) >> (H == 8 ? 1 : 0);
        const int dx = mvx & 7, dy = mvy & 7;
        const int cA = (8 - dx) * (8 - dy), cB = dx * (8 - dy), cC = (8 - dx) * dy, cD = dx * dy;
        const typename PT<BD>::pixel *s =
            ref + (intptr_t)(H * by + r + (mvy >> 3)) * rs + 16 * bx + (mvx >> 3) * 2 + pl;
        constexpr int NDW = (18 + PPD - 1) / PPD;
        uint32_t a[NDW], c[NDW];
        load_al_pad<NDW>( s, a );
        load_al_pad<NDW>( s + rs, c );
#pragma unroll
        for( int x = 0; x < 8; x++ )
        {
            const int k0 = 2 * x, k1 = 2 * x + 2;
            g[x] = (cA * upix<BD>( a[k0 / PPD], k0 % PPD ) + cB * upix<BD>( a[k1 / PPD], k1 % PPD ) +
                    cC * upix<BD>( c[k0 / PPD], k0 % PPD ) + cD * upix<BD>( c[k1 / PPD], k1 % PPD ) + 32) >> 6;
        }
    }
    else
    {
        constexpr int NDW = 16 / PPD;
        uint32_t w[NDW];
        load_al_pad<NDW>( ref + (intptr_t)(H * by + r) * rs + 16 * bx, w );
#pragma unroll
        for( int x = 0; x < 8; x++ )
        {
            const int k = 2 * x;
            g[x] = pl ? upix<BD>( w[(k + 1) / PPD], (k + 1) % PPD ) : upix<BD>( w[k / PPD], k % PPD );
        }
    }

    for( int k = 0; k < cd.n; k++ )
    {
        const uint32_t c = cd.c[k];
        const int scale = c & 255, denom = (c >> 8) & 7, wtd = (c >> 11) & 1;
        const int off = (((int)(c >> 12) & 511) - 256) * (1 << (BD - 8));
        const int rnd = denom ? 1 << (denom - 1) : 0;
        int s = -sf;
#pragma unroll
        for( int i = 0; i < 8; i++ )
            s += wtd ? wp_px<BD>( g[i], scale, denom, rnd, off ) : g[i];
        s += dpp_i( s, 0xB1 );
        s += dpp_i( s, 0x4E );
        s += dpp_i( s, 0x141 );
        if constexpr( H == 16 )
            s += dpp_i( s, 0x140 );
        uint32_t t = (r == 0 && valid) ? (uint32_t)abs( s ) : 0u;
#pragma unroll
        for( int m = H; m < 64; m <<= 1 )
            t += __shfl_xor( t, m );
        if( lane == 0 )
            atomicAdd( &acc[k], t );
    }
    __syncthreads();
    if( tid < cd.n )
        atomicAdd( out + tid, acc[tid] + (blockIdx.x == 0 ? cd.hdr[tid] : 0u) );
}

// ---- weight_slice_header_cost (slicetype.c:170-189) ----
static int ue_tab( unsigned v )   // x264_ue_size_tab[v] (common/bitstream.h:201-219)
{
    int n = 0;
    while( v >> (n + 1) )
        n++;
    return v ? 2 * n + 1 : 1;
}
static int size_ue( unsigned v ) { return ue_tab( v + 1 ); }
static int size_se( int v )
{
    int tmp = 1 - v * 2;
    if( tmp < 0 )
        tmp = v * 2;
    return tmp < 256 ? ue_tab( tmp ) : ue_tab( tmp >> 8 ) + 16;
}
static uint32_t header_cost( const x264hip_weight_t &w, int b_chroma, int lambda, int numslices )
{
    if( b_chroma )
        lambda *= 4;
    const int denom_cost = size_ue( w.denom ) * (2 - b_chroma);
    return (uint32_t)(lambda * numslices * (10 + denom_cost + 2 * (size_se( w.scale ) + size_se( w.offset ))));
}

// One launch scoring n (<= 64) candidates of one kind into out[0..n) (zeroed here).
//   kind 0: luma lowres 8x8 mbcmp capped by intra cost; 1 / 2: 4:2:0 / 4:2:2 chroma asd8 of
//   plane pl; 3: 4:4:4 chroma 16x16 mbcmp.
template <int BD>
static hipError_t launch_wp_cost( int kind, const typename PT<BD>::pixel *fenc, intptr_t fs,
                                  const typename PT<BD>::pixel *const ref[4], intptr_t rs, int mbw, int mbh,
                                  const uint16_t *intra, const int16_t *mvs, int satd, int pl, const WpCands &cd,
                                  uint32_t *out, hipStream_t stream )
{
    hipError_t e = hipMemsetAsync( out, 0, sizeof( uint32_t ) * (size_t)cd.n, stream );
    if( e != hipSuccess || cd.n == 0 || mbw <= 0 || mbh <= 0 )
        return e;
    if( kind == 0 || kind == 3 )
    {
        const int bw = kind ? 2 * mbw : mbw, bh = kind ? 2 * mbh : mbh;
        const unsigned grid = (unsigned)((bw * bh + 31) / 32);
        const int mv = mvs ? (kind ? 2 : 1) : 0;
#define WP8( M, S )                                                                                                  \
    hipLaunchKernelGGL( ( wp_cost8_kernel<BD, M, S> ), dim3( grid ), dim3( 256 ), 0, stream, fenc, fs, ref[0],       \
                        ref[1], ref[2], ref[3], rs, bw, bh, mvs, mbw, kind ? nullptr : intra, cd, out )
        if( mv == 0 ) { if( satd ) WP8( 0, true ); else WP8( 0, false ); }
        else if( mv == 1 ) { if( satd ) WP8( 1, true ); else WP8( 1, false ); }
        else { if( satd ) WP8( 2, true ); else WP8( 2, false ); }
#undef WP8
    }
    else
    {
        const int H = kind == 1 ? 8 : 16;
        const unsigned grid = (unsigned)((mbw * mbh + 4 * (64 / H) - 1) / (4 * (64 / H)));
#define WPC( HH, M )                                                                                                 \
    hipLaunchKernelGGL( ( wp_chroma_kernel<BD, HH, M> ), dim3( grid ), dim3( 256 ), 0, stream, fenc, fs, ref[0], rs, \
                        mbw, mbh, mvs, pl, cd, out )
        if( H == 8 ) { if( mvs ) WPC( 8, true ); else WPC( 8, false ); }
        else { if( mvs ) WPC( 16, true ); else WPC( 16, false ); }
#undef WPC
    }
    return hipGetLastError();
}

static uint32_t pack_cand( const x264hip_weight_t &w )
{
    return (uint32_t)(w.scale & 255) | (uint32_t)(w.denom & 7) << 8 | (uint32_t)(w.weighted ? 1 : 0) << 11 |
           (uint32_t)((w.offset + 256) & 511) << 12;
}

// the batched entry: weight_cost_luma / _chroma / _chroma444 (slicetype.c:191-282) of n
// candidates, header cost included for the weighted ones; chunks of 64 per launch
template <int BD>
hipError_t launch_weight_cost( int kind, const typename PT<BD>::pixel *fenc, intptr_t fs,
                               const typename PT<BD>::pixel *const ref[4], intptr_t rs, int mbw, int mbh,
                               const uint16_t *intra, const int16_t *mvs, int satd, int plane, int lambda,
                               int numslices, const x264hip_weight_t *cands, int n, uint32_t *out, hipStream_t stream )
{
    for( int i = 0; i < n; i += 64 )
    {
        WpCands cd;
        memset( &cd, 0, sizeof( cd ) );
        cd.n = n - i < 64 ? n - i : 64;
        for( int k = 0; k < cd.n; k++ )
        {
            cd.c[k] = pack_cand( cands[i + k] );
            cd.hdr[k] = cands[i + k].weighted ? header_cost( cands[i + k], kind != 0, lambda, numslices ) : 0;
        }
        const hipError_t e = launch_wp_cost<BD>( kind, fenc, fs, ref, rs, mbw, mbh, intra, mvs, satd, plane, cd,
                                                 out + i, stream );
        if( e != hipSuccess )
            return e;
    }
    return hipSuccess;
}
template hipError_t launch_weight_cost<8>( int, const uint8_t *, intptr_t, const uint8_t *const[4], intptr_t, int, int,
                                           const uint16_t *, const int16_t *, int, int, int, int,
                                           const x264hip_weight_t *, int, uint32_t *, hipStream_t );
template hipError_t launch_weight_cost<10>( int, const uint16_t *, intptr_t, const uint16_t *const[4], intptr_t, int,
                                            int, const uint16_t *, const int16_t *, int, int, int, int,
                                            const x264hip_weight_t *, int, uint32_t *, hipStream_t );

// ---- frame statistics: ac_energy_mb's stores (ratecontrol.c:225-257, 289-299) ----
__device__ __forceinline__ unsigned long long wave_sum64( unsigned long long v )
{
#pragma unroll
    for( int m = 1; m < 64; m <<= 1 )
        v += __shfl_xor( v, m );
    return v;
}

// PIXEL_VAR_C's (sum, sum of squares) of every MB's 16x16 luma block and chroma blocks (8 x
// 16>>vshift deinterleaved from the NV12 / NV16 plane, or the 16x16 blocks of the 4:4:4
// planes), summed into acc[plane] (sums) / acc[3 + plane] (squares).  A wave walks MBs
// grid-stride (luma: lane = row * 4 + 4-pixel column group) with 64-bit lane accumulators;
// one wave reduction and one atomic per quantity per workgroup at the end.  The sums' low 32
// bits are the uint32 field's wrapped total (addition mod 2^32 commutes).
template <int BD>
__global__ __launch_bounds__( 256 ) void frame_stats_kernel( const typename PT<BD>::pixel *__restrict__ y,
                                                             intptr_t ys, const typename PT<BD>::pixel *__restrict__ u,
                                                             const typename PT<BD>::pixel *__restrict__ v,
                                                             intptr_t cs, int mbw, int mbh, int cf,
                                                             unsigned long long *__restrict__ acc )
{
    constexpr int PPD = PT<BD>::PPD, NDW = 4 / PPD;
    __shared__ unsigned long long part[4][6];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned long long a[6] = { 0, 0, 0, 0, 0, 0 };
    const int nmb = mbw * mbh;
    auto sq4 = [&]( const typename PT<BD>::pixel *p, intptr_t s, int mbx, int mby, int plane ) {
        uint32_t w[NDW];
        load_al_pad<NDW>( p + (intptr_t)(16 * mby + (lane >> 2)) * s + 16 * mbx + 4 * (lane & 3), w );
        uint32_t sum = 0, sqr = 0;
#pragma unroll
        for( int k = 0; k < 4; k++ )
        {
            const uint32_t x = (uint32_t)upix<BD>( w[k / PPD], k % PPD );
            sum += x;
            sqr += x * x;
        }
        a[plane] += sum;
        a[3 + plane] += sqr;
    };
    for( int mb = blockIdx.x * 4 + wave; mb < nmb; mb += gridDim.x * 4 )
    {
        const int mby = mb / mbw, mbx = mb - mby * mbw;
        sq4( y, ys, mbx, mby, 0 );
        if( cf == 3 )
        {
            sq4( u, cs, mbx, mby, 1 );
            sq4( v, cs, mbx, mby, 2 );
        }
        else if( cf )
        {
            const int H = cf == 1 ? 8 : 16;
            for( int row = lane >> 3; row < H; row += 8 )
            {
                const typename PT<BD>::pixel *q = u + (intptr_t)(H * mby + row) * cs + 16 * mbx + 2 * (lane & 7);
                const uint32_t p0 = q[0], p1 = q[1];
                a[1] += p0; a[4] += p0 * p0; a[2] += p1; a[5] += p1 * p1;
            }
        }
    }
#pragma unroll
    for( int i = 0; i < 6; i++ )
    {
        const unsigned long long t = wave_sum64( a[i] );
        if( lane == 0 )
            part[wave][i] = t;
    }
    __syncthreads();
    if( threadIdx.x < 6 )
    {
        const int i = threadIdx.x;
        atomicAdd( acc + i, part[0][i] + part[1][i] + part[2][i] + part[3][i] );
    }
}

// i_pixel_sum as the uint32 field holds it, i_pixel_ssd with the mean removed
// (ratecontrol.c:406-414)
__global__ void frame_stats_finish_kernel( unsigned long long *acc, int mbw, int mbh, int cf )
{
    const int i = threadIdx.x;
    if( i >= 3 )
        return;
    const int hs = (cf == 1 || cf == 2) && i, vs = cf == 1 && i;
    const unsigned long long s = (uint32_t)acc[i];
    const unsigned long long w = (unsigned long long)(16 * mbw >> hs), h = (unsigned long long)(16 * mbh >> vs);
    acc[i] = s;
    acc[3 + i] = acc[3 + i] - (s * s + w * h / 2) / (w * h);
}

template <int BD>
hipError_t launch_frame_stats( const typename PT<BD>::pixel *y, intptr_t ys, const typename PT<BD>::pixel *u,
                               const typename PT<BD>::pixel *v, intptr_t cs, int mbw, int mbh, int cf,
                               uint64_t *stats, hipStream_t stream )
{
    hipError_t e = hipMemsetAsync( stats, 0, 6 * sizeof( uint64_t ), stream );
    if( e != hipSuccess )
        return e;
    if( mbw > 0 && mbh > 0 )
        hipLaunchKernelGGL( frame_stats_kernel<BD>, dim3( (unsigned)std::min( (mbw * mbh + 3) / 4, 1024 ) ), dim3( 256 ), 0, stream,
                            y, ys, u, v, cs, mbw, mbh, cf, (unsigned long long *)stats );
    hipLaunchKernelGGL( frame_stats_finish_kernel, dim3( 1 ), dim3( 64 ), 0, stream, (unsigned long long *)stats,
                        mbw > 0 ? mbw : 1, mbh > 0 ? mbh : 1, cf );
    return hipGetLastError();
}
template hipError_t launch_frame_stats<8>( const uint8_t *, intptr_t, const uint8_t *, const uint8_t *, intptr_t, int,
                                           int, int, uint64_t *, hipStream_t );
template hipError_t launch_frame_stats<10>( const uint16_t *, intptr_t, const uint16_t *, const uint16_t *, intptr_t,
                                            int, int, int, uint64_t *, hipStream_t );

// ---- x264_weights_analyse (slicetype.c:284-501): the host walk ----
#pragma clang fp contract( off )

static int clip3( int v, int lo, int hi ) { return v < lo ? lo : v > hi ? hi : v; }
static double clip3f( double v, double lo, double hi ) { return v < lo ? lo : v > hi ? hi : v; }

// weight_get_h264 (slicetype.c:63-75)
static void get_h264( int weight_nonh264, int offset, x264hip_weight_t *w )
{
    w->offset = offset;
    w->denom = 7;
    w->scale = weight_nonh264;
    while( w->denom > 0 && w->scale > 127 )
    {
        w->denom--;
        w->scale >>= 1;
    }
    w->scale = w->scale < 127 ? w->scale : 127;
}

static void set_w( x264hip_weight_t &w, int b, int s, int d, int o )
{
    w.scale = s;
    w.denom = d;
    w.offset = o;
    w.weighted = b;
}

// One plane's (scale, offset) walk of slicetype.c:401-439.  The grid depends only on the
// plane's statistics, so the walk runs twice: once collecting every (scale, offset) the
// loops could visit (no early break), once replaying the reference's loop -- early break
// included -- over the costs the GPU returned for that list.  f( cur_scale, i_off,
// start_offset, idx ) gets idx = the position of the pair in the unbroken walk and returns
// false to break the offset loop.
struct PlaneWalk
{
    int mindenom, minscale, start_scale, end_scale, offset_dist, b_lookahead;
    float fenc_mean, ref_mean;

    template <class F> void visit( F &&f ) const
    {
        int base = 0;
        for( int i_scale = start_scale; i_scale <= end_scale; i_scale++ )
        {
            int cur_scale = i_scale;
            int cur_offset = fenc_mean - ref_mean * cur_scale / (1 << mindenom) + 0.5f * b_lookahead;
            if( cur_offset < -128 || cur_offset > 127 )
            {
                cur_offset = clip3( cur_offset, -128, 127 );
                cur_scale = clip3f( (1 << mindenom) * (fenc_mean - cur_offset) / ref_mean + 0.5f, 0, 127 );
            }
            const int start_offset = clip3( cur_offset - offset_dist, -128, 127 );
            const int end_offset = clip3( cur_offset + offset_dist, -128, 127 );
            for( int i_off = start_offset; i_off <= end_offset; i_off++ )
                if( !f( cur_scale, i_off, start_offset, base + i_off - start_offset ) )
                    break;
            base += end_offset - start_offset + 1;
        }
    }
};

template <int BD>
hipError_t weights_analyse( const WpInput<BD> &in, x264hip_weight_t weights[3], float *cost_delta,
                            typename PT<BD>::pixel *wlr, hipStream_t stream )
{
    using pixel = typename PT<BD>::pixel;
    const int cf = in.cf, mbw = in.mbw, mbh = in.mbh, b_lookahead = in.b_lookahead;
    const int hs = cf == 1 || cf == 2, vs = cf == 1;
    const float epsilon = 1.f / 128.f;
    set_w( weights[0], 0, 1, 0, 0 );
    set_w( weights[1], 0, 1, 0, 0 );
    set_w( weights[2], 0, 1, 0, 0 );
    float guess_scale[3], fenc_mean[3], ref_mean[3];
    for( int plane = 0; plane <= 2 * !b_lookahead; plane++ )
    {
        if( !plane || cf )
        {
            const int zero_bias = !in.ref_ssd[plane];
            const float fenc_var = in.fenc_ssd[plane] + zero_bias;
            const float ref_var = in.ref_ssd[plane] + zero_bias;
            const int npx = (16 * mbh >> (plane ? vs : 0)) * (16 * mbw >> (plane ? hs : 0));
            guess_scale[plane] = sqrtf( fenc_var / ref_var );
            fenc_mean[plane] = (float)(in.fenc_sum[plane] + zero_bias) / npx / (1 << (BD - 8));
            ref_mean[plane] = (float)(in.ref_sum[plane] + zero_bias) / npx / (1 << (BD - 8));
        }
        else
        {
            guess_scale[plane] = 1;
            fenc_mean[plane] = 0;
            ref_mean[plane] = 0;
        }
    }
    int chroma_denom = 7;
    if( !b_lookahead )
        while( chroma_denom > 0 )
        {
            const float thresh = 127.f / (1 << chroma_denom);
            if( guess_scale[1] < thresh && guess_scale[2] < thresh )
                break;
            chroma_denom--;
        }

    static const uint8_t check_distance[][2] = { { 0, 0 }, { 0, 0 }, { 0, 1 }, { 0, 1 }, { 0, 1 }, { 0, 1 },
                                                 { 0, 1 }, { 1, 1 }, { 1, 1 }, { 2, 1 }, { 2, 1 }, { 4, 2 } };
    const int scale_dist = b_lookahead ? 0 : check_distance[in.subme][0];
    const int offset_dist = b_lookahead ? 0 : check_distance[in.subme][1];

    // Per plane: candidate 0 = the unweighted reference (origscore), then the unbroken walk
    // (<= 9 scales x 5 offsets at subme 11).
    x264hip_weight_t cand[3][64];
    int ncand[3] = { 0, 0, 0 };
    PlaneWalk walk[3];

    // the pre-search state of a plane (slicetype.c:336-359) applied to w[]; returns whether
    // the plane is searched, *stop when the chroma loop breaks (scale > 127)
    auto prepare = [&]( int plane, x264hip_weight_t *w, bool *stop ) -> bool {
        *stop = false;
        if( fabsf( ref_mean[plane] - fenc_mean[plane] ) < 0.5f && fabsf( 1.f - guess_scale[plane] ) < epsilon )
        {
            set_w( w[plane], 0, 1, 0, 0 );
            return false;
        }
        if( plane )
        {
            w[plane].denom = chroma_denom;
            w[plane].scale = clip3( (int)round( guess_scale[plane] * (1 << chroma_denom) ), 0, 255 );
            if( w[plane].scale > 127 )
            {
                w[1].weighted = w[2].weighted = 0;
                *stop = true;
                return false;
            }
        }
        else
            get_h264( (int)round( guess_scale[plane] * 128 ), 0, &w[plane] );
        PlaneWalk &pw = walk[plane];
        pw.mindenom = w[plane].denom;
        pw.minscale = w[plane].scale;
        pw.start_scale = clip3( pw.minscale - scale_dist, 0, 127 );
        pw.end_scale = clip3( pw.minscale + scale_dist, 0, 127 );
        pw.offset_dist = offset_dist;
        pw.fenc_mean = fenc_mean[plane];
        pw.ref_mean = ref_mean[plane];
        pw.b_lookahead = b_lookahead;
        int n = 1;
        cand[plane][0] = { 0, 1, 0, 0 };
        pw.visit( [&]( int s, int o, int, int ) {
            cand[plane][n++] = { 1, s, pw.mindenom, o };
            return true;
        } );
        ncand[plane] = n;
        return true;
    };

    // the reference's search and decision (slicetype.c:391-463) over costs[] of cand[plane]
    auto finish = [&]( int plane, const uint32_t *costs ) {
        const PlaneWalk &pw = walk[plane];
        const unsigned origscore = costs[0];
        unsigned minscore = origscore;
        if( !minscore )
            return;
        int minscale = pw.minscale, minoff = 0, mindenom = pw.mindenom, found = 0;
        pw.visit( [&]( int cur_scale, int i_off, int start_offset, int idx ) {
            const unsigned s = costs[1 + idx];
            set_w( weights[plane], 1, cur_scale, mindenom, i_off );
            if( s < minscore )
            {
                minscore = s;
                minscale = cur_scale;
                minoff = i_off;
                found = 1;
            }
            return !(minoff == start_offset && i_off != start_offset);
        } );
        if( !plane )
            while( mindenom > 0 && !(minscale & 1) )
            {
                mindenom--;
                minscale >>= 1;
            }
        if( !found || (minscale == 1 << mindenom && minoff == 0) || (float)minscore / origscore > 0.998f )
        {
            set_w( weights[plane], 0, 1, 0, 0 );
            return;
        }
        set_w( weights[plane], 1, minscale, mindenom, minoff );
        if( in.weightp_fake && weights[0].weighted && !plane && cost_delta )
            *cost_delta = (float)minscore / origscore;
    };

    uint32_t *dcost = nullptr;
    hipError_t e = scratch_alloc( (void **)&dcost, 3 * 64 * sizeof( uint32_t ), stream );
    if( e != hipSuccess )
        return e;
    uint32_t hcost[3][64];
    bool stop = false;

    // ---- luma (slicetype.c:362-372) ----
    if( prepare( 0, weights, &stop ) )
    {
        const pixel *const ref[4] = { in.ref_lr[0], in.ref_lr[1], in.ref_lr[2], in.ref_lr[3] };
        e = launch_weight_cost<BD>( 0, in.fenc_lr, in.lrs, ref, in.lrs, mbw, mbh, in.intra, in.mvs, in.satd, 0,
                                    in.lambda, in.numslices, cand[0], ncand[0], dcost, stream );
        if( e == hipSuccess )
            e = hipMemcpyAsync( hcost[0], dcost, sizeof( uint32_t ) * ncand[0], hipMemcpyDeviceToHost, stream );
        if( e == hipSuccess )
            e = hipStreamSynchronize( stream );
        if( e == hipSuccess )
            finish( 0, hcost[0] );
    }

    // ---- chroma, outside the lookahead and after a luma weight (slicetype.c:330, 373-389):
    // a dry run of the planes' pre-search state finds which are searched, their candidates
    // go in one batch, then the plane loop runs in order over the costs ----
    if( e == hipSuccess && cf && !b_lookahead && weights[0].weighted )
    {
        x264hip_weight_t dry[3] = { weights[0], weights[1], weights[2] };
        bool searched[3] = { false, false, false }, any = false;
        for( int plane = 1; plane <= 2; plane++ )
        {
            searched[plane] = prepare( plane, dry, &stop );
            any |= searched[plane];
            if( stop )
                break;
        }
        for( int plane = 1; plane <= 2 && e == hipSuccess; plane++ )
            if( searched[plane] )
            {
                const int kind = cf == 3 ? 3 : cf;
                const pixel *fp = cf == 3 ? in.fenc_c[plane - 1] : in.fenc_c[0];
                const pixel *const ref[4] = { cf == 3 ? in.ref_c[plane - 1] : in.ref_c[0], nullptr, nullptr,
                                              nullptr };
                e = launch_weight_cost<BD>( kind, fp, in.cs, ref, in.cs, mbw, mbh, nullptr, in.mvs, in.satd,
                                            cf == 3 ? 0 : plane - 1, in.lambda, in.numslices, cand[plane],
                                            ncand[plane], dcost + 64 * plane, stream );
                if( e == hipSuccess )
                    e = hipMemcpyAsync( hcost[plane], dcost + 64 * plane, sizeof( uint32_t ) * ncand[plane],
                                        hipMemcpyDeviceToHost, stream );
            }
        if( e == hipSuccess && any )
            e = hipStreamSynchronize( stream );
        for( int plane = 1; plane <= 2 && e == hipSuccess; plane++ )
        {
            if( !prepare( plane, weights, &stop ) )
            {
                if( stop )
                    break;
                continue;
            }
            finish( plane, hcost[plane] );
        }
    }
    const hipError_t ef = hipFreeAsync( dcost, stream );
    if( e == hipSuccess )
        e = ef;
    if( e != hipSuccess )
        return e;

    // optimize and unify the chroma denominator (slicetype.c:466-485)
    if( weights[1].weighted || weights[2].weighted )
    {
        int denom = weights[1].weighted ? weights[1].denom : weights[2].denom;
        const int both = weights[1].weighted && weights[2].weighted;
        while( (!both && denom == 7) || (denom > 0 && !(weights[1].weighted && (weights[1].scale & 1)) &&
                                         !(weights[2].weighted && (weights[2].scale & 1))) )
        {
            denom--;
            for( int i = 1; i <= 2; i++ )
                if( weights[i].weighted )
                {
                    weights[i].scale >>= 1;
                    weights[i].denom = denom;
                }
        }
    }

    // the lookahead's weighted lowres reference (slicetype.c:490-500)
    if( weights[0].weighted && b_lookahead && wlr )
        return launch_weight_plane<BD>( wlr - 32 - 32 * in.lrs, in.lrs, 0, in.ref_lr[0] - 32 - 32 * in.lrs, in.lrs, 0,
                                        8 * mbw + 64, 8 * mbh + 64, 1, weights[0].scale, weights[0].denom,
                                        weights[0].offset, stream );
    return hipSuccess;
}
template hipError_t weights_analyse<8>( const WpInput<8> &, x264hip_weight_t *, float *, uint8_t *, hipStream_t );
template hipError_t weights_analyse<10>( const WpInput<10> &, x264hip_weight_t *, float *, uint16_t *, hipStream_t );

} // namespace x264hip
