// Block metrics over block lists in device memory: SAD / SSD / SATD / SA8D
// (int scores), var / hadamard_ac / sa8d_satd / vsad / asd8 (u64 statistics),
// var2, successive-elimination ads and the ESA integral image.
//
// Semantics: reference common/pixel.c — PIXEL_SAD_C :55-70, PIXEL_SSD_C :85-101,
// satd 4x4 / 8x4 and the PIXEL_SATD_C tiling :265-332, sa8d :334-381,
// hadamard_ac :383-435, var / var2 :181-227, vsad :716-723, asd8 :747-754,
// ads :759-803; integral_init* common/mc.c:424-456 as used by
// x264_frame_filter mc.c:748-782.  SATD is computed in
// plain (unpacked) Hadamard form: every coefficient of a 4x4 Hadamard has the
// parity of the block's difference sum, so the per-4x4 |coef| sum is even and
// the reference's ">>1 per 8x4 pair" equals ">>1 per 4x4" (checked against the
// packed-form oracle in tests).
//
// One lane per (fenc block, ref block) pair; rows are fetched as aligned dwords
// and realigned with v_alignbyte_b32, SAD uses v_sad_u8 / v_sad_u16.
#include "hipcommon.h"

#include <algorithm>
#include <atomic>
#include <mutex>

namespace x264hip {

template <int BD, int W>
__device__ __forceinline__ void load_row( const typename PT<BD>::pixel *p, uint32_t (&o)[W / PT<BD>::PPD] )
{
    load_packed<W / PT<BD>::PPD>( p, o );
}

// 4-point Hadamard with the reference's output order (pixel.c:242-251)
__device__ __forceinline__ void had4( int &a0, int &a1, int &a2, int &a3 )
{
    int t0 = a0 + a1, t1 = a0 - a1, t2 = a2 + a3, t3 = a2 - a3;
    a0 = t0 + t2;
    a2 = t0 - t2;
    a1 = t1 + t3;
    a3 = t1 - t3;
}

// SATD of one 4x4 tile: (sum |H(d)|) >> 1
template <int BD>
__device__ __forceinline__ int satd4x4( const typename PT<BD>::pixel *a, intptr_t sa,
                                        const typename PT<BD>::pixel *b, intptr_t sb )
{
    constexpr int NDW = 4 / PT<BD>::PPD;
    int d[4][4];
#pragma unroll
    for( int y = 0; y < 4; y++ )
    {
        uint32_t ra[NDW], rb[NDW];
        load_packed<NDW>( a + y * sa, ra );
        load_packed<NDW>( b + y * sb, rb );
#pragma unroll
        for( int x = 0; x < 4; x++ )
            d[y][x] = upix<BD>( ra[x / PT<BD>::PPD], x % PT<BD>::PPD ) - upix<BD>( rb[x / PT<BD>::PPD], x % PT<BD>::PPD );
        had4( d[y][0], d[y][1], d[y][2], d[y][3] );
    }
    int s = 0;
#pragma unroll
    for( int x = 0; x < 4; x++ )
    {
        had4( d[0][x], d[1][x], d[2][x], d[3][x] );
        s += abs( d[0][x] ) + abs( d[1][x] ) + abs( d[2][x] ) + abs( d[3][x] );
    }
    return s >> 1;
}

// 8-point Hadamard (Sylvester order; only sums of |coef| are taken, so the
// order is irrelevant)
__device__ __forceinline__ void had8( int (&v)[8] )
{
#pragma unroll
    for( int h = 1; h < 8; h <<= 1 )
#pragma unroll
        for( int i = 0; i < 8; i++ )
            if( !(i & h) )
            {
                int a = v[i], b = v[i + h];
                v[i] = a + b;
                v[i + h] = a - b;
            }
}

// load 8 pixels of a row as ints
template <int BD>
__device__ __forceinline__ void row8( const typename PT<BD>::pixel *p, int (&v)[8] )
{
    constexpr int PPD = PT<BD>::PPD;
    uint32_t r[8 / PPD];
    load_packed<8 / PPD>( p, r );
#pragma unroll
    for( int x = 0; x < 8; x++ )
        v[x] = upix<BD>( r[x / PPD], x % PPD );
}

// unnormalised sa8d of one 8x8 tile: sum |H8 . D . H8^T| (equals the packed
// sa8d_8x8 of pixel.c:334-366; cross-checked in tests/test_cpu_pixel_ext.py)
template <int BD>
__device__ __forceinline__ int sa8d8x8( const typename PT<BD>::pixel *a, intptr_t sa,
                                        const typename PT<BD>::pixel *b, intptr_t sb )
{
    int d[8][8];
#pragma unroll
    for( int y = 0; y < 8; y++ )
    {
        int va[8], vb[8];
        row8<BD>( a + y * sa, va );
        row8<BD>( b + y * sb, vb );
#pragma unroll
        for( int x = 0; x < 8; x++ )
            d[y][x] = va[x] - vb[x];
        had8( d[y] );
    }
    int s = 0;
#pragma unroll
    for( int x = 0; x < 8; x++ )
    {
        int c[8];
#pragma unroll
        for( int y = 0; y < 8; y++ )
            c[y] = d[y][x];
        had8( c );
#pragma unroll
        for( int y = 0; y < 8; y++ )
            s += abs( c[y] );
    }
    return s;
}

template <int BD, int OP, int IPIX>
__global__ __launch_bounds__( 256 ) void cmp_batch_kernel( const typename PT<BD>::pixel *fenc, intptr_t fs,
                                                           const typename PT<BD>::pixel *ref, intptr_t rs,
                                                           const int64_t *fenc_off, const int64_t *ref_off,
                                                           int n, int32_t *scores )
{
    constexpr int W = pix_w( IPIX ), H = pix_h( IPIX );
    constexpr int NDW = W / PT<BD>::PPD;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if( i >= n )
        return;
    const typename PT<BD>::pixel *a = fenc + fenc_off[i];
    const typename PT<BD>::pixel *b = ref + ref_off[i];
    int sum = 0;
    if constexpr( OP == 0 )          // SAD
    {
        uint32_t acc = 0;
#pragma unroll
        for( int y = 0; y < H; y++ )
        {
            uint32_t ra[NDW], rb[NDW];
            load_packed<NDW>( a + y * fs, ra );
            load_packed<NDW>( b + y * rs, rb );
#pragma unroll
            for( int k = 0; k < NDW; k++ )
                acc = sadp<BD>( ra[k], rb[k], acc );
        }
        sum = (int)acc;
    }
    else if constexpr( OP == 1 )     // SSD
    {
#pragma unroll
        for( int y = 0; y < H; y++ )
        {
            uint32_t ra[NDW], rb[NDW];
            load_packed<NDW>( a + y * fs, ra );
            load_packed<NDW>( b + y * rs, rb );
#pragma unroll
            for( int k = 0; k < NDW; k++ )
#pragma unroll
                for( int j = 0; j < PT<BD>::PPD; j++ )
                {
                    int d = upix<BD>( ra[k], j ) - upix<BD>( rb[k], j );
                    sum += d * d;
                }
        }
    }
    else if constexpr( OP == 3 )     // SA8D (16x16, 8x8): (sum + 2) >> 2
    {
#pragma unroll
        for( int y = 0; y < H; y += 8 )
#pragma unroll
            for( int x = 0; x < W; x += 8 )
                sum += sa8d8x8<BD>( a + y * fs + x, fs, b + y * rs + x, rs );
        sum = (sum + 2) >> 2;
    }
    else if constexpr( W >= 8 )      // SATD, 8x4 bands in packed 16-bit pairs (one >> 1 at the end)
    {
        uint32_t acc = 0;
#pragma unroll
        for( int y = 0; y < H; y += 4 )
#pragma unroll
            for( int x = 0; x < W; x += 8 )
            {
                uint32_t ra[4][8 / PT<BD>::PPD], rb[4][8 / PT<BD>::PPD];
#pragma unroll
                for( int k = 0; k < 4; k++ )
                {
                    load_packed<8 / PT<BD>::PPD>( a + (y + k) * fs + x, ra[k] );
                    load_packed<8 / PT<BD>::PPD>( b + (y + k) * rs + x, rb[k] );
                }
                acc += satd8x4_packed<BD>( ra, rb );
            }
        sum = (int)(acc >> 1);
    }
    else                             // SATD, 4-wide blocks
    {
#pragma unroll
        for( int y = 0; y < H; y += 4 )
#pragma unroll
            for( int x = 0; x < W; x += 4 )
                sum += satd4x4<BD>( a + y * fs + x, fs, b + y * rs + x, rs );
    }
    scores[i] = sum;
}

template <int BD, int OP>
static hipError_t cmp_dispatch( int i_pixel, dim3 g, dim3 blk, hipStream_t st,
                                const typename PT<BD>::pixel *fenc, intptr_t fs, const typename PT<BD>::pixel *ref,
                                intptr_t rs, const int64_t *fo, const int64_t *ro, int n, int32_t *sc )
{
#define CMP_CASE( I ) \
    case I: hipLaunchKernelGGL( ( cmp_batch_kernel<BD, OP, I> ), g, blk, 0, st, fenc, fs, ref, rs, fo, ro, n, sc ); break;
    switch( i_pixel )
    {
        CMP_CASE( 0 ) CMP_CASE( 1 ) CMP_CASE( 2 ) CMP_CASE( 3 )
        CMP_CASE( 4 ) CMP_CASE( 5 ) CMP_CASE( 6 ) CMP_CASE( 7 )
        default: return hipErrorInvalidValue;
    }
#undef CMP_CASE
    return hipGetLastError();
}

template <int BD>
hipError_t launch_cmp_batch( int op, int i_pixel, const typename PT<BD>::pixel *fenc, intptr_t fs,
                             const typename PT<BD>::pixel *ref, intptr_t rs, const int64_t *fenc_off,
                             const int64_t *ref_off, int n, int32_t *scores, hipStream_t stream )
{
    if( n <= 0 )
        return hipSuccess;
    dim3 blk( 256 ), g( (n + 255) / 256 );
    switch( op )
    {
        case 0: return cmp_dispatch<BD, 0>( i_pixel, g, blk, stream, fenc, fs, ref, rs, fenc_off, ref_off, n, scores );
        case 1: return cmp_dispatch<BD, 1>( i_pixel, g, blk, stream, fenc, fs, ref, rs, fenc_off, ref_off, n, scores );
        case 2: return cmp_dispatch<BD, 2>( i_pixel, g, blk, stream, fenc, fs, ref, rs, fenc_off, ref_off, n, scores );
        case 3:
            if( i_pixel == 0 )
                hipLaunchKernelGGL( ( cmp_batch_kernel<BD, 3, 0> ), g, blk, 0, stream, fenc, fs, ref, rs, fenc_off,
                                    ref_off, n, scores );
            else if( i_pixel == 3 )
                hipLaunchKernelGGL( ( cmp_batch_kernel<BD, 3, 3> ), g, blk, 0, stream, fenc, fs, ref, rs, fenc_off,
                                    ref_off, n, scores );
            else
                return hipErrorInvalidValue;
            return hipGetLastError();
    }
    return hipErrorInvalidValue;
}

template hipError_t launch_cmp_batch<8>( int, int, const uint8_t *, intptr_t, const uint8_t *, intptr_t,
                                         const int64_t *, const int64_t *, int, int32_t *, hipStream_t );
template hipError_t launch_cmp_batch<10>( int, int, const uint16_t *, intptr_t, const uint16_t *, intptr_t,
                                          const int64_t *, const int64_t *, int, int32_t *, hipStream_t );


// ---------------------------------------------------------------------------
// u64 statistics, one lane per item:
//   OP 0 var (pixel.c:181-198)          OP 1 hadamard_ac (pixel.c:383-435)
//   OP 2 sa8d_satd (16x16; low = sa8d, high = satd: checkasm.c:424-460)
//   OP 3 vsad (16 wide, `height` rows)  OP 4 asd8 (8 wide, `height` rows)
template <int BD>
__device__ __forceinline__ void hadac8x8( const typename PT<BD>::pixel *p, intptr_t s, uint32_t &s4, uint32_t &s8 )
{
    // 4x4 Hadamards of the four quadrants, then the 2x2 Hadamard across the
    // quadrants gives the 8x8 Hadamard coefficients (H8 = [[H4,H4],[H4,-H4]]
    // up to row order)
    int q[4][4][4];
#pragma unroll
    for( int y = 0; y < 8; y++ )
    {
        int v[8];
        row8<BD>( p + y * s, v );
#pragma unroll
        for( int h = 0; h < 2; h++ )
        {
            int a0 = v[4 * h], a1 = v[4 * h + 1], a2 = v[4 * h + 2], a3 = v[4 * h + 3];
            had4( a0, a1, a2, a3 );
            int *r = q[(y >> 2) * 2 + h][y & 3];
            r[0] = a0; r[1] = a1; r[2] = a2; r[3] = a3;
        }
    }
    int sum4 = 0, sum8 = 0;
#pragma unroll
    for( int x = 0; x < 4; x++ )
    {
#pragma unroll
        for( int k = 0; k < 4; k++ )
        {
            had4( q[k][0][x], q[k][1][x], q[k][2][x], q[k][3][x] );
#pragma unroll
            for( int y = 0; y < 4; y++ )
                sum4 += abs( q[k][y][x] );
        }
#pragma unroll
        for( int y = 0; y < 4; y++ )
        {
            int a = q[0][y][x], b = q[1][y][x], c = q[2][y][x], d = q[3][y][x];
            int e = a + b, f = a - b, g = c + d, h = c - d;
            sum8 += abs( e + g ) + abs( e - g ) + abs( f + h ) + abs( f - h );
        }
    }
    const int dc = q[0][0][0] + q[1][0][0] + q[2][0][0] + q[3][0][0];   // sum of the 64 pixels
    s4 += (uint32_t)(sum4 - dc);
    s8 += (uint32_t)(sum8 - dc);
}

template <int BD, int OP, int IPIX>
__global__ __launch_bounds__( 256 ) void stat_batch_kernel( const typename PT<BD>::pixel *p1, intptr_t s1,
                                                            const typename PT<BD>::pixel *p2, intptr_t s2,
                                                            const int64_t *off1, const int64_t *off2, int height,
                                                            int n, uint64_t *out )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int W = pix_w( IPIX ), H = pix_h( IPIX );
    constexpr int PPD = PT<BD>::PPD;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if( i >= n )
        return;
    const pixel *a = p1 + off1[i];
    uint64_t r = 0;
    if constexpr( OP == 0 )
    {
        uint32_t sum = 0, sqr = 0;
#pragma unroll
        for( int y = 0; y < H; y++ )
        {
            uint32_t w[W / PPD];
            load_packed<W / PPD>( a + y * s1, w );
#pragma unroll
            for( int k = 0; k < W; k++ )
            {
                uint32_t v = (uint32_t)upix<BD>( w[k / PPD], k % PPD );
                sum += v;
                sqr += v * v;
            }
        }
        r = sum + ((uint64_t)sqr << 32);
    }
    else if constexpr( OP == 1 )
    {
        uint32_t s4 = 0, s8 = 0;
#pragma unroll
        for( int y = 0; y < H; y += 8 )
#pragma unroll
            for( int x = 0; x < W; x += 8 )
                hadac8x8<BD>( a + y * s1 + x, s1, s4, s8 );
        r = ((uint64_t)(s8 >> 2) << 32) + (s4 >> 1);
    }
    else if constexpr( OP == 2 )
    {
        const pixel *b = p2 + off2[i];
        int sa = 0, st = 0;
#pragma unroll 1
        for( int t = 0; t < 4; t++ )
            sa += sa8d8x8<BD>( a + (t >> 1) * 8 * s1 + (t & 1) * 8, s1, b + (t >> 1) * 8 * s2 + (t & 1) * 8, s2 );
#pragma unroll 1
        for( int y = 0; y < 16; y += 4 )
#pragma unroll
            for( int x = 0; x < 16; x += 4 )
                st += satd4x4<BD>( a + y * s1 + x, s1, b + y * s2 + x, s2 );
        r = (uint32_t)((sa + 2) >> 2) | ((uint64_t)(uint32_t)st << 32);
    }
    else if constexpr( OP == 3 )
    {
        uint32_t acc = 0, prev[16 / PPD];
        load_packed<16 / PPD>( a, prev );
        for( int y = 1; y < height; y++ )
        {
            uint32_t cur[16 / PPD];
            load_packed<16 / PPD>( a + y * s1, cur );
#pragma unroll
            for( int k = 0; k < 16 / PPD; k++ )
            {
                acc = sadp<BD>( prev[k], cur[k], acc );
                prev[k] = cur[k];
            }
        }
        r = acc;
    }
    else
    {
        const pixel *b = p2 + off2[i];
        int sum = 0;
        for( int y = 0; y < height; y++ )
        {
            int va[8], vb[8];
            row8<BD>( a + y * s1, va );
            row8<BD>( b + y * s2, vb );
#pragma unroll
            for( int x = 0; x < 8; x++ )
                sum += va[x] - vb[x];
        }
        r = (uint32_t)abs( sum );
    }
    out[i] = r;
}

template <int BD>
hipError_t launch_stat_batch( int op, int i_pixel, const typename PT<BD>::pixel *p1, intptr_t s1,
                              const typename PT<BD>::pixel *p2, intptr_t s2, const int64_t *off1,
                              const int64_t *off2, int height, int n, uint64_t *out, hipStream_t st )
{
    if( n <= 0 )
        return hipSuccess;
    dim3 blk( 256 ), g( (n + 255) / 256 );
#define STAT( OP, I ) \
    hipLaunchKernelGGL( ( stat_batch_kernel<BD, OP, I> ), g, blk, 0, st, p1, s1, p2, s2, off1, off2, height, n, out )
    switch( op )
    {
        case 0:
            if( i_pixel == 0 ) STAT( 0, 0 ); else if( i_pixel == 2 ) STAT( 0, 2 ); else if( i_pixel == 3 ) STAT( 0, 3 );
            else return hipErrorInvalidValue;
            break;
        case 1:
            if( i_pixel == 0 ) STAT( 1, 0 ); else if( i_pixel == 1 ) STAT( 1, 1 ); else if( i_pixel == 2 ) STAT( 1, 2 );
            else if( i_pixel == 3 ) STAT( 1, 3 ); else return hipErrorInvalidValue;
            break;
        case 2:
            if( i_pixel != 0 ) return hipErrorInvalidValue;
            STAT( 2, 0 );
            break;
        case 3: STAT( 3, 0 ); break;
        case 4: STAT( 4, 3 ); break;
        default: return hipErrorInvalidValue;
    }
#undef STAT
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// var2 (pixel.c:203-227), one lane per (U,V) block pair: out[3i] = result,
// out[3i+1] = ssd_u, out[3i+2] = ssd_v.  V blocks sit at +vd from the U blocks.
template <int BD, int H>
__global__ __launch_bounds__( 256 ) void var2_batch_kernel( const typename PT<BD>::pixel *fenc, intptr_t fs,
                                                            intptr_t fvd, const typename PT<BD>::pixel *fdec,
                                                            intptr_t ds, intptr_t dvd, const int64_t *fo,
                                                            const int64_t *dof, int n, int32_t *out )
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if( i >= n )
        return;
    const typename PT<BD>::pixel *a = fenc + fo[i], *b = fdec + dof[i];
    int su = 0, sv = 0, qu = 0, qv = 0;
#pragma unroll
    for( int y = 0; y < H; y++ )
    {
        int au[8], bu[8], av[8], bv[8];
        row8<BD>( a + y * fs, au );
        row8<BD>( b + y * ds, bu );
        row8<BD>( a + y * fs + fvd, av );
        row8<BD>( b + y * ds + dvd, bv );
#pragma unroll
        for( int x = 0; x < 8; x++ )
        {
            int du = au[x] - bu[x], dv = av[x] - bv[x];
            su += du; sv += dv;
            qu += du * du; qv += dv * dv;
        }
    }
    constexpr int SHIFT = H == 16 ? 7 : 6;
    out[3 * i] = (int)(qu - ((int64_t)su * su >> SHIFT) + qv - ((int64_t)sv * sv >> SHIFT));
    out[3 * i + 1] = qu;
    out[3 * i + 2] = qv;
}

template <int BD>
hipError_t launch_var2_batch( int i_pixel, const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t fvd,
                              const typename PT<BD>::pixel *fdec, intptr_t ds, intptr_t dvd, const int64_t *fo,
                              const int64_t *dof, int n, int32_t *out, hipStream_t st )
{
    if( n <= 0 )
        return hipSuccess;
    dim3 blk( 256 ), g( (n + 255) / 256 );
    if( i_pixel == 2 )
        hipLaunchKernelGGL( ( var2_batch_kernel<BD, 16> ), g, blk, 0, st, fenc, fs, fvd, fdec, ds, dvd, fo, dof, n, out );
    else if( i_pixel == 3 )
        hipLaunchKernelGGL( ( var2_batch_kernel<BD, 8> ), g, blk, 0, st, fenc, fs, fvd, fdec, ds, dvd, fo, dof, n, out );
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// successive elimination (x264_pixel_ads4/2/1, pixel.c:759-803), one wave per
// call: each lane scores one candidate, the passing indices are compacted in
// candidate order with a ballot + mbcnt prefix, as the reference's mvs[nmv++].
template <int NS>
__global__ __launch_bounds__( 256 ) void ads_batch_kernel( const int32_t *enc_dc, const uint16_t *sums, int delta,
                                                           const int64_t *sums_off, const uint16_t *cost,
                                                           const int64_t *cost_off, const int32_t *width,
                                                           const int32_t *thresh, int n, int16_t *mvs,
                                                           int mvs_pitch, int32_t *nmv )
{
    const int job = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if( job >= n )
        return;
    const uint16_t *sm = sums + sums_off[job];
    const uint16_t *cm = cost + cost_off[job];
    const int w = width[job], th = thresh[job];
    const int d0 = enc_dc[4 * job], d1 = enc_dc[4 * job + 1], d2 = enc_dc[4 * job + 2], d3 = enc_dc[4 * job + 3];
    int16_t *o = mvs + (int64_t)job * mvs_pitch;
    int cnt = 0;
    for( int base = 0; base < w; base += 64 )
    {
        const int i = base + lane;
        bool pass = false;
        if( i < w )
        {
            int a = abs( d0 - (int)sm[i] );
            if constexpr( NS == 4 )
                a += abs( d1 - (int)sm[i + 8] ) + abs( d2 - (int)sm[i + delta] ) + abs( d3 - (int)sm[i + delta + 8] );
            else if constexpr( NS == 2 )
                a += abs( d1 - (int)sm[i + delta] );
            a += cm[i];
            pass = a < th;
        }
        const uint64_t m = __ballot( pass );
        const int pos = cnt + (int)__builtin_amdgcn_mbcnt_hi( (uint32_t)(m >> 32),
                                                              __builtin_amdgcn_mbcnt_lo( (uint32_t)m, 0u ) );
        if( pass )
            o[pos] = (int16_t)i;
        cnt += __popcll( m );
    }
    if( lane == 0 )
        nmv[job] = cnt;
}

hipError_t launch_ads_batch( int i_pixel, const int32_t *enc_dc, const uint16_t *sums, int delta,
                             const int64_t *sums_off, const uint16_t *cost, const int64_t *cost_off,
                             const int32_t *width, const int32_t *thresh, int n, int16_t *mvs, int mvs_pitch,
                             int32_t *nmv, hipStream_t st )
{
    if( n <= 0 )
        return hipSuccess;
    dim3 blk( 256 ), g( (n + 3) / 4 );
    switch( ads_nsums( i_pixel ) )
    {
        case 4: hipLaunchKernelGGL( ads_batch_kernel<4>, g, blk, 0, st, enc_dc, sums, delta, sums_off, cost, cost_off,
                                    width, thresh, n, mvs, mvs_pitch, nmv ); break;
        case 2: hipLaunchKernelGGL( ads_batch_kernel<2>, g, blk, 0, st, enc_dc, sums, delta, sums_off, cost, cost_off,
                                    width, thresh, n, mvs, mvs_pitch, nmv ); break;
        default: hipLaunchKernelGGL( ads_batch_kernel<1>, g, blk, 0, st, enc_dc, sums, delta, sums_off, cost,
                                     cost_off, width, thresh, n, mvs, mvs_pitch, nmv ); break;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// ESA integral image (x264_frame_filter, mc.c:748-782): the reference builds a
// running 2-D prefix in uint16 and differences it (integral_init8h/8v or
// 4h/4v, mc.c:424-456); every value it leaves in rows [1-PADV, lines+PADV-8)
// and columns [-padh, stride-padh-8) is an exact 8x8 (and, with sub8x8, 4x4)
// box sum with that top-left, which is what this kernel writes directly: one
// lane per column walks a strip of rows with a sliding window of horizontal
// sums (coalesced row loads and stores).
constexpr int INTEGRAL_STRIP = 64;

template <int BD, bool SUB8>
__global__ __launch_bounds__( 256 ) void integral_kernel( const typename PT<BD>::pixel *__restrict__ plane,
                                                          intptr_t stride, intptr_t fstride, int lines, int padh,
                                                          uint16_t *__restrict__ integral, intptr_t ifstride )
{
    constexpr int PADV = 32;
    constexpr int PPD = PT<BD>::PPD;
    const int c = blockIdx.x * blockDim.x + threadIdx.x;     // column, 0 = x -padh
    if( c >= stride - 8 )
        return;
    const int rows_end = lines + 2 * PADV - 8;               // buffer rows [1, rows_end) are box rows
    const int t0 = 1 + blockIdx.y * INTEGRAL_STRIP;
    if( t0 >= rows_end )
        return;
    const int t1 = min( t0 + INTEGRAL_STRIP, rows_end );
    const typename PT<BD>::pixel *src = plane + blockIdx.z * fstride - PADV * stride - padh + c;
    uint16_t *o8 = integral + blockIdx.z * ifstride - PADV * stride - padh + c;
    uint16_t *o4 = o8 + stride * (lines + 2 * PADV);
    uint32_t ring8[8] = {}, ring4[4] = {};
    uint32_t acc8 = 0, acc4 = 0;
    // input rows t0 .. t1+6; after adding row r, acc8 holds rows r-7..r, acc4 rows r-3..r.
    // A batch's eight row loads are issued together at clamped (valid) rows before any
    // of them is summed (a per-row guard around each load serialised them: one memory
    // round trip per row); rows past the strip only feed stores that are masked off.
    for( int r0 = t0; r0 < t1 + 7; r0 += 8 )
    {
        uint32_t wb[8][8 / PPD];
#pragma unroll
        for( int k = 0; k < 8; k++ )
            load_packed<8 / PPD>( src + (intptr_t)min( r0 + k, t1 + 6 ) * stride, wb[k] );
#pragma unroll
        for( int k = 0; k < 8; k++ )
        {
            const int r = r0 + k;
            if( r < t1 + 7 )
            {
                const uint32_t( &w )[8 / PPD] = wb[k];
                uint32_t h4 = 0, h8 = 0;
#pragma unroll
                for( int x = 0; x < 4; x++ )
                    h4 += (uint32_t)upix<BD>( w[x / PPD], x % PPD );
                h8 = h4;
#pragma unroll
                for( int x = 4; x < 8; x++ )
                    h8 += (uint32_t)upix<BD>( w[x / PPD], x % PPD );
                acc8 += h8 - ring8[k];
                ring8[k] = h8;
                acc4 += h4 - ring4[k & 3];
                ring4[k & 3] = h4;
                if( r - 7 >= t0 )
                    o8[(intptr_t)(r - 7) * stride] = (uint16_t)acc8;
                if( SUB8 && r - 3 >= t0 && r - 3 < t1 )
                    o4[(intptr_t)(r - 3) * stride] = (uint16_t)acc4;
            }
        }
    }
}

// Default form: one lane per source dword (4 columns at 8 bit, 2 at 10 bit).  A lane
// loads the dwords covering its columns' 8-pixel windows once per row (three at 8 bit, five
// at 10 bit; neighbouring lanes share cache lines), forms each column's 4- and 8-pixel sums
// from byte-shifted dwords with v_sad against zero, and stores its columns' sums as one
// 8- (4-) byte store: 3 loads and 1-2 stores per 4 columns against 8 and 4-8 before.
template <int BD, bool SUB8>
__global__ __launch_bounds__( 256 ) void integral_dw_kernel( const typename PT<BD>::pixel *__restrict__ plane,
                                                             intptr_t stride, intptr_t fstride, int lines, int padh,
                                                             uint16_t *__restrict__ integral, intptr_t ifstride )
{
    constexpr int PADV = 32;
    constexpr int PPD = PT<BD>::PPD;                        // columns per lane
    constexpr int ND = 8 / PPD + 1;                          // dwords per row window
    const int j = blockIdx.x * blockDim.x + threadIdx.x;     // dword index, column PPD * j
    const int c0 = PPD * j, ncol = (int)stride - 8;
    if( c0 >= ncol )
        return;
    const int rows_end = lines + 2 * PADV - 8;
    const int t0 = 1 + blockIdx.y * INTEGRAL_STRIP;
    if( t0 >= rows_end )
        return;
    const int t1 = min( t0 + INTEGRAL_STRIP, rows_end );
    const uint32_t *src = (const uint32_t *)(plane + blockIdx.z * fstride - PADV * stride - padh) + j;
    const intptr_t sdw = stride / PPD;
    uint16_t *o8 = integral + blockIdx.z * ifstride - PADV * stride - padh + c0;
    uint16_t *o4 = o8 + stride * (lines + 2 * PADV);
    const bool whole = c0 + PPD <= ncol;
    uint32_t ring8[8][PPD] = {}, ring4[4][PPD] = {};
    uint32_t acc8[PPD] = {}, acc4[PPD] = {};
    for( int r0 = t0; r0 < t1 + 7; r0 += 8 )
    {
        uint32_t wb[8][ND];
#pragma unroll
        for( int k = 0; k < 8; k++ )
        {
            const uint32_t *rp = src + (intptr_t)min( r0 + k, t1 + 6 ) * sdw;
#pragma unroll
            for( int d = 0; d < ND; d++ )
                wb[k][d] = rp[d];
        }
#pragma unroll
        for( int k = 0; k < 8; k++ )
        {
            const int r = r0 + k;
            if( r >= t1 + 7 )
                break;
            uint32_t h4[PPD], h8[PPD];
#pragma unroll
            for( int s = 0; s < PPD; s++ )
            {
                // column c0 + s: pixels s .. s+3 and s+4 .. s+7 of the window
                constexpr int SB = BD == 8 ? 1 : 2;          // bytes per pixel
                uint32_t lo[4 / PPD], hi[4 / PPD];
#pragma unroll
                for( int d = 0; d < 4 / PPD; d++ )
                {
                    const int b = s * SB;                    // byte shift within dword d
                    lo[d] = b ? __builtin_amdgcn_alignbyte( wb[k][d + 1], wb[k][d], b ) : wb[k][d];
                    hi[d] = b ? __builtin_amdgcn_alignbyte( wb[k][d + 1 + 4 / PPD], wb[k][d + 4 / PPD], b )
                              : wb[k][d + 4 / PPD];
                }
                uint32_t a = 0;
#pragma unroll
                for( int d = 0; d < 4 / PPD; d++ )
                    a = sadp<BD>( lo[d], 0u, a );
                h4[s] = a;
#pragma unroll
                for( int d = 0; d < 4 / PPD; d++ )
                    a = sadp<BD>( hi[d], 0u, a );
                h8[s] = a;
            }
            uint32_t v8[PPD], v4[PPD];
#pragma unroll
            for( int s = 0; s < PPD; s++ )
            {
                acc8[s] += h8[s] - ring8[k][s];
                ring8[k][s] = h8[s];
                acc4[s] += h4[s] - ring4[k & 3][s];
                ring4[k & 3][s] = h4[s];
                v8[s] = acc8[s];
                v4[s] = acc4[s];
            }
            auto put = [&]( uint16_t *o, const uint32_t (&v)[PPD] ) {
                if( whole )
                {
                    if constexpr( PPD == 4 )
                        *(uint2 *)o = make_uint2( (v[0] & 0xffff) | (v[1] << 16), (v[2] & 0xffff) | (v[3] << 16) );
                    else
                        *(uint32_t *)o = (v[0] & 0xffff) | (v[1] << 16);
                }
                else
                {
#pragma unroll
                    for( int s = 0; s < PPD; s++ )
                        if( c0 + s < ncol )
                            o[s] = (uint16_t)v[s];
                }
            };
            if( r - 7 >= t0 )
                put( o8 + (intptr_t)(r - 7) * stride, v8 );
            if( SUB8 && r - 3 >= t0 && r - 3 < t1 )
                put( o4 + (intptr_t)(r - 3) * stride, v4 );
        }
    }
}

template <int BD>
hipError_t launch_frame_integral( const typename PT<BD>::pixel *plane, intptr_t stride, intptr_t fstride, int lines,
                                  int padh, int sub8x8, int nframes, uint16_t *integral, intptr_t ifstride,
                                  hipStream_t st )
{
    if( nframes <= 0 )
        return hipSuccess;
    const int rows = lines + 64 - 9;
    constexpr int PPD = PT<BD>::PPD;
    // the dword form needs dword-aligned source rows and output columns at multiples of
    // the lane width (X264HIP_INTEGRAL_VARIANT=1: the column-per-lane kernel)
    using pixel = typename PT<BD>::pixel;
    const uintptr_t sb = (uintptr_t)(plane - 32 * stride - padh);
    const uintptr_t ob = (uintptr_t)(integral - 32 * stride - padh);
    if( variant( V_INTEGRAL ) != 1 && !((sb | (uintptr_t)(stride * sizeof( pixel )) | (uintptr_t)(fstride * sizeof( pixel ))) & 3) &&
        !((ob | (uintptr_t)(stride * 2) | (uintptr_t)(ifstride * 2)) & (PPD * 2 - 1)) )
    {
        const int ndw = (int)((stride - 8 + PPD - 1) / PPD);
        dim3 blk( 256 ), g( (unsigned)((ndw + 255) / 256), (unsigned)((rows + INTEGRAL_STRIP - 1) / INTEGRAL_STRIP),
                            (unsigned)nframes );
        if( sub8x8 )
            hipLaunchKernelGGL( ( integral_dw_kernel<BD, true> ), g, blk, 0, st, plane, stride, fstride, lines, padh,
                                integral, ifstride );
        else
            hipLaunchKernelGGL( ( integral_dw_kernel<BD, false> ), g, blk, 0, st, plane, stride, fstride, lines, padh,
                                integral, ifstride );
        return hipGetLastError();
    }
    dim3 blk( 256 ), g( (unsigned)((stride - 8 + 255) / 256), (unsigned)((rows + INTEGRAL_STRIP - 1) / INTEGRAL_STRIP),
                        (unsigned)nframes );
    if( sub8x8 )
        hipLaunchKernelGGL( ( integral_kernel<BD, true> ), g, blk, 0, st, plane, stride, fstride, lines, padh,
                            integral, ifstride );
    else
        hipLaunchKernelGGL( ( integral_kernel<BD, false> ), g, blk, 0, st, plane, stride, fstride, lines, padh,
                            integral, ifstride );
    return hipGetLastError();
}

#define INST( BD )                                                                                                     \
    template hipError_t launch_stat_batch<BD>( int, int, const PT<BD>::pixel *, intptr_t, const PT<BD>::pixel *,       \
                                               intptr_t, const int64_t *, const int64_t *, int, int, uint64_t *,       \
                                               hipStream_t );                                                          \
    template hipError_t launch_var2_batch<BD>( int, const PT<BD>::pixel *, intptr_t, intptr_t, const PT<BD>::pixel *,  \
                                               intptr_t, intptr_t, const int64_t *, const int64_t *, int, int32_t *,   \
                                               hipStream_t );                                                          \
    template hipError_t launch_frame_integral<BD>( const PT<BD>::pixel *, intptr_t, intptr_t, int, int, int, int,      \
                                                   uint16_t *, intptr_t, hipStream_t );
INST( 8 )
INST( 10 )
#undef INST

} // namespace x264hip

namespace x264hip {

// ---------------------------------------------------------------------------
// Plane SSD: x264_pixel_ssd_wxh (reference common/pixel.c:112-151) and
// x264_pixel_ssd_nv12 (:153-178).  ssd_wxh tiles the plane into 16x16 / 8x16 / 8x8
// ssd calls plus per-pixel tails; every tile sum is an exact int (<= 256 * 1023^2)
// and the tiles and tails cover each pixel of the w x h rectangle once, so the
// uint64 result is the plain sum of d^2 over the rectangle -- what this reduction
// computes, in any order.  ssd_nv12 runs the core over the first w&~7 (u, v) pairs
// of each interleaved row and then the tail over w&7 pairs starting at PIXEL
// offset w&~7 (not pair offset: the tail re-reads pixels of the core, as the
// reference does); both are segments [c0, c1) of pixel columns with even columns
// counted as u and odd as v.  One lane per 16-byte chunk of a row (coalesced
// rows), d^2 pairs by v_dot2_i32_i16 on packed differences, a wave reduction and
// one 64-bit atomic add per wave.
template <int BD, bool NV12>
__device__ __forceinline__ void ssd_chunk( uint4 a4, uint4 b4, uint32_t &iu, uint32_t &iv )
{
    const uint32_t wa[4] = { a4.x, a4.y, a4.z, a4.w }, wb[4] = { b4.x, b4.y, b4.z, b4.w };
#pragma unroll
    for( int k = 0; k < 4; k++ )
    {
        if constexpr( BD == 8 )
        {
            // even pixels (bytes 0, 2) and odd pixels (bytes 1, 3) as 16-bit pairs
            const x264hip_short2 ea = __builtin_bit_cast( x264hip_short2, __builtin_amdgcn_perm( 0u, wa[k], 0x0c020c00u ) );
            const x264hip_short2 eb = __builtin_bit_cast( x264hip_short2, __builtin_amdgcn_perm( 0u, wb[k], 0x0c020c00u ) );
            const x264hip_short2 oa = __builtin_bit_cast( x264hip_short2, __builtin_amdgcn_perm( 0u, wa[k], 0x0c030c01u ) );
            const x264hip_short2 ob = __builtin_bit_cast( x264hip_short2, __builtin_amdgcn_perm( 0u, wb[k], 0x0c030c01u ) );
            const x264hip_short2 de = ea - eb, dd = oa - ob;
            iu = (uint32_t)__builtin_amdgcn_sdot2( de, de, (int)iu, false );
            if( NV12 )
                iv = (uint32_t)__builtin_amdgcn_sdot2( dd, dd, (int)iv, false );
            else
                iu = (uint32_t)__builtin_amdgcn_sdot2( dd, dd, (int)iu, false );
        }
        else
        {
            const x264hip_short2 d = __builtin_bit_cast( x264hip_short2, wa[k] ) -
                                     __builtin_bit_cast( x264hip_short2, wb[k] );
            if( NV12 )
            {
                iu += (uint32_t)((int)d.x * d.x);
                iv += (uint32_t)((int)d.y * d.y);
            }
            else
                iu = (uint32_t)__builtin_amdgcn_sdot2( d, d, (int)iu, false );
        }
    }
}

// grid: x = 64-chunk column groups (the nv12 tail columns as extra groups after nbx0), y =
// bands of 4 x SSD_ROWS rows (one wave per SSD_ROWS rows), z = frame.  A lane loads its chunk
// of all SSD_ROWS rows of both planes before any arithmetic (2 x SSD_ROWS independent 16-byte
// loads in flight); the four waves' sums meet in LDS.  The frame total needs no zeroed output: each
// workgroup adds into its frame's slot of a library-owned accumulator ring and takes a
// ticket; the last arriver moves the total to out[] and leaves the slot zero for the next
// launch (one kernel, no memset and no dependent dispatch).
struct SsdSlot
{
    unsigned long long su, sv;
    unsigned int cnt, pad[3];
};
constexpr int SSD_RING = 1 << 16;

template <int BD, bool NV12, int SSD_ROWS = 16>
__global__ __launch_bounds__( 256 ) void plane_ssd_kernel( const typename PT<BD>::pixel *__restrict__ p1, intptr_t s1,
                                                           intptr_t f1, const typename PT<BD>::pixel *__restrict__ p2,
                                                           intptr_t s2, intptr_t f2, int c0a, int c1a, int nbx0,
                                                           int c0b, int c1b, int height,
                                                           unsigned long long *__restrict__ out, SsdSlot *ring,
                                                           int slot0 )
{
    constexpr int CH = 16 / (int)sizeof( typename PT<BD>::pixel );   // pixels per chunk
    __shared__ uint64_t part[2][4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int f = blockIdx.z;
    const bool tail = (int)blockIdx.x >= nbx0;
    const int c0 = tail ? c0b : c0a, c1 = tail ? c1b : c1a;
    const int x = c0 + ((int)blockIdx.x - (tail ? nbx0 : 0)) * 64 * CH + lane * CH;
    const int y0 = ((int)blockIdx.y * 4 + wv) * SSD_ROWS;
    const typename PT<BD>::pixel *a = p1 + f * f1 + (intptr_t)y0 * s1 + x, *b = p2 + f * f2 + (intptr_t)y0 * s2 + x;
    uint32_t iu = 0, iv = 0;
    if( x + CH <= c1 && y0 + SSD_ROWS <= height )
    {
        uint4 va[SSD_ROWS], vb[SSD_ROWS];
#pragma unroll
        for( int r = 0; r < SSD_ROWS; r++ )
        {
            __builtin_memcpy( &va[r], a + r * s1, 16 );
            __builtin_memcpy( &vb[r], b + r * s2, 16 );
        }
#pragma unroll
        for( int r = 0; r < SSD_ROWS; r++ )
            ssd_chunk<BD, NV12>( va[r], vb[r], iu, iv );   // <= 16 rows x 16 x 65025 (8 bit) / 8 x 1046529: u32
    }
    else if( x < c1 )
    {
        for( int r = 0; r < SSD_ROWS && y0 + r < height; r++ )
            for( int k = 0; k < CH && x + k < c1; k++ )
            {
                const int d = (int)a[r * s1 + k] - (int)b[r * s2 + k];
                if( NV12 && ((x + k) & 1) )
                    iv += (uint32_t)(d * d);
                else
                    iu += (uint32_t)(d * d);
            }
    }
    uint64_t su = iu, sv = iv;
#pragma unroll
    for( int off = 32; off >= 1; off >>= 1 )
    {
        su += (uint64_t)__shfl_xor( (unsigned long long)su, off );
        if( NV12 )
            sv += (uint64_t)__shfl_xor( (unsigned long long)sv, off );
    }
    if( lane == 0 )
    {
        part[0][wv] = su;
        part[1][wv] = sv;
    }
    __syncthreads();
    if( threadIdx.x == 0 && !NV12 )
    {
        // one atomic per workgroup: the count in bits 48-63 and the sum below it (a frame's SSD
        // is < 2^48: 10-bit 8K is 2^45), so the returned word tells the last arriver and the
        // total at once -- no wait for the add before a separate ticket (one memory round
        // trip less in every workgroup's tail)
        SsdSlot *sl = ring + ((slot0 + f) & (SSD_RING - 1));
        su = part[0][0] + part[0][1] + part[0][2] + part[0][3];
        const unsigned long long nwg = gridDim.x * gridDim.y, mine = (1ull << 48) + su;
        const unsigned long long old =
            __hip_atomic_fetch_add( &sl->su, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
        if( (old >> 48) == nwg - 1 )
        {
            out[f] = (old + mine) & ((1ull << 48) - 1);
            __hip_atomic_store( &sl->su, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
        }
    }
    else if( threadIdx.x == 0 )
    {
        SsdSlot *sl = ring + ((slot0 + f) & (SSD_RING - 1));
        su = part[0][0] + part[0][1] + part[0][2] + part[0][3];
        if( su )
            __hip_atomic_fetch_add( &sl->su, (unsigned long long)su, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
        if( NV12 )
        {
            sv = part[1][0] + part[1][1] + part[1][2] + part[1][3];
            if( sv )
                __hip_atomic_fetch_add( &sl->sv, (unsigned long long)sv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
        }
        // the ticket: device-scope atomics are performed at one point for all XCDs; waiting
        // for this workgroup's adds to return (vmcnt(0)) before taking the ticket orders them
        // before it, so the last arriver's exchange sees every add.  (A release / acquire
        // ticket instead writes back the XCD's L2 per workgroup: 0.022 -> 0.035 ms per 16
        // 1080p frames.)
        __builtin_amdgcn_s_waitcnt( 0 );
        const unsigned int nwg = gridDim.x * gridDim.y;
        if( __hip_atomic_fetch_add( &sl->cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT ) == nwg - 1 )
        {
            const unsigned long long tu =
                __hip_atomic_exchange( &sl->su, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
            if( NV12 )
            {
                const unsigned long long tv =
                    __hip_atomic_exchange( &sl->sv, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
                out[2 * f] = tu;
                out[2 * f + 1] = tv;
            }
            else
                out[f] = tu;
            __hip_atomic_store( &sl->cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
        }
    }
}

// the accumulator ring of the launch stream's device (zeroed once; every launch leaves its
// slots zero), and disjoint slot ranges for launches that may be in flight together.  The
// slot range is fixed when a launch is enqueued, so a captured graph holds its range: replays
// of one graph must not run concurrently with each other (sequential replays are fine).
static hipError_t ssd_ring( hipStream_t stream, SsdSlot **ring, int nslots, int *slot0 )
{
    static std::mutex mu;
    static SsdSlot *rings[64] = {};
    static std::atomic<uint64_t> next{ 0 };
    int dev = 0;
    hipError_t e = stream_device( stream, &dev );
    if( e != hipSuccess )
        return e;
    if( dev < 0 || dev >= 64 || nslots > SSD_RING )
        return hipErrorInvalidValue;
    {
        std::lock_guard<std::mutex> lk( mu );
        if( !rings[dev] )
        {
            int cur = 0;
            if( (e = hipGetDevice( &cur )) != hipSuccess || (cur != dev && (e = hipSetDevice( dev )) != hipSuccess) )
                return e;
            SsdSlot *r = nullptr;
            e = hipMalloc( (void **)&r, sizeof( SsdSlot ) * SSD_RING );
            if( e == hipSuccess && ((e = hipMemset( r, 0, sizeof( SsdSlot ) * SSD_RING )) != hipSuccess ||
                                    (e = hipDeviceSynchronize()) != hipSuccess) )
                (void)hipFree( r );
            if( cur != dev )
                (void)hipSetDevice( cur );
            if( e != hipSuccess )
                return e;
            rings[dev] = r;
        }
    }
    *ring = rings[dev];
    const uint64_t b = next.fetch_add( (uint64_t)nslots );
    *slot0 = (int)(b % SSD_RING);
    return hipSuccess;
}

template <int BD>
hipError_t launch_plane_ssd( int nv12, const typename PT<BD>::pixel *p1, intptr_t s1, intptr_t f1,
                             const typename PT<BD>::pixel *p2, intptr_t s2, intptr_t f2, int width, int height,
                             int nframes, uint64_t *out, hipStream_t stream )
{
    if( nframes <= 0 )
        return hipSuccess;
    if( width <= 0 || height <= 0 )
        return hipMemsetAsync( out, 0, (size_t)nframes * (nv12 ? 2 : 1) * sizeof( uint64_t ), stream );
    if( nframes > 65535 )
        return hipErrorInvalidValue;
    // the plane path's packed accumulator: a frame's SSD below 2^48, fewer than 2^16 workgroups
    const double pmax = (double)((1 << BD) - 1);
    if( !nv12 && ((double)width * height * pmax * pmax >= 281474976710656.0 ||
                  (double)((width + 1023) / 1024 + 1) * ((height + 3) / 4 + 1) >= 65536.0) )
        return hipErrorInvalidValue;
    SsdSlot *ring = nullptr;
    int slot0 = 0;
    hipError_t e = ssd_ring( stream, &ring, nframes, &slot0 );
    if( e != hipSuccess )
        return e;
    constexpr int CH = 16 / (int)sizeof( typename PT<BD>::pixel );
    // column ranges in pixels of the row: the plane, or for nv12 the 8-pair core and the
    // tail over the last w&7 pairs, which starts at PIXEL offset w&~7 (pixel.c:153-178)
    int c0a = 0, c1a = width, c0b = 0, c1b = 0;
    if( nv12 )
    {
        const int w8 = width & ~7, w7 = width & 7;
        c1a = 2 * w8;
        c0b = w8;
        c1b = w7 ? w8 + 2 * w7 : w8;
    }
    const int nbx0 = (c1a - c0a + 64 * CH - 1) / (64 * CH), nbx1 = (c1b - c0b + 64 * CH - 1) / (64 * CH);
    // 8 rows per wave: 16 1080p pairs 0.0195 / 0.0137 / 0.0141 ms for 16 / 8 / 4 rows with the
    // packed accumulator (profiles/r03aa_ssd_ab.json); the 16-frame leg is one burst of loads,
    // and twice the waves of half the rows issue it faster
    constexpr int rows = 8;
    dim3 g( (unsigned)std::max( 1, nbx0 + nbx1 ), (unsigned)((height + 4 * rows - 1) / (4 * rows)), (unsigned)nframes ),
        blk( 256 );
    unsigned long long *o = (unsigned long long *)out;
#define SSD_GO( R )                                                                                                \
    if( nv12 )                                                                                                     \
        hipLaunchKernelGGL( ( plane_ssd_kernel<BD, true, R> ), g, blk, 0, stream, p1, s1, f1, p2, s2, f2, c0a, c1a, \
                            nbx0, c0b, c1b, height, o, ring, slot0 );                                              \
    else                                                                                                           \
        hipLaunchKernelGGL( ( plane_ssd_kernel<BD, false, R> ), g, blk, 0, stream, p1, s1, f1, p2, s2, f2, c0a,    \
                            c1a, nbx0, c0b, c1b, height, o, ring, slot0 )
    SSD_GO( rows );
#undef SSD_GO
    return hipGetLastError();
}

template hipError_t launch_plane_ssd<8>( int, const uint8_t *, intptr_t, intptr_t, const uint8_t *, intptr_t, intptr_t,
                                         int, int, int, uint64_t *, hipStream_t );
template hipError_t launch_plane_ssd<10>( int, const uint16_t *, intptr_t, intptr_t, const uint16_t *, intptr_t,
                                          intptr_t, int, int, int, uint64_t *, hipStream_t );

} // namespace x264hip
