// Forward transforms and quantisation on gfx950.
//
// Semantics (all integer, bit-exact):
//   sub4x4_dct     reference common/dct.c:157-189  (int16 temps at 8 bit)
//   sub8x8/16x16   reference common/dct.c:191-205  (quadrant-major block order)
//   *_dct_dc       reference common/dct.c:207-270
//   sub8x8_dct8    reference common/dct.c:332-377  (column pass, int16 temps, row pass)
//   dct4x4dc/2x4dc reference common/dct.c:47-76, 109-143
//   QUANT_ONE      reference common/quant.c:50-57 (uint32 arithmetic), entries :59-104
// Every block lives in one lane's registers; pixels arrive as aligned dwords
// realigned with v_alignbyte_b32, coefficients leave as contiguous stores.
#include "hipcommon.h"
#include <stdlib.h>

namespace x264hip {

// ---------------------------------------------------------------- helpers
template <int BD, int N>
__device__ __forceinline__ void load_diff( int (&d)[N][N], const typename PT<BD>::pixel *a, intptr_t sa,
                                           const typename PT<BD>::pixel *b, intptr_t sb )
{
    constexpr int NDW = N / PT<BD>::PPD;
#pragma unroll
    for( int y = 0; y < N; y++ )
    {
        uint32_t ra[NDW], rb[NDW];
        load_packed<NDW>( a + y * sa, ra );
        load_packed<NDW>( b + y * sb, rb );
#pragma unroll
        for( int x = 0; x < N; x++ )
            d[y][x] = upix<BD>( ra[x / PT<BD>::PPD], x % PT<BD>::PPD ) - upix<BD>( rb[x / PT<BD>::PPD], x % PT<BD>::PPD );
    }
}


// sub4x4_dct on a difference block: out[i*4+k] (reference order)
template <int BD>
__device__ __forceinline__ void dct4x4_core( int (&d)[4][4], int (&out)[16] )
{
    int tmp[4][4];   // tmp[k][i]: second index = source row
#pragma unroll
    for( int i = 0; i < 4; i++ )
    {
        int s03 = d[i][0] + d[i][3], s12 = d[i][1] + d[i][2];
        int d03 = d[i][0] - d[i][3], d12 = d[i][1] - d[i][2];
        tmp[0][i] = sto<BD>( s03 + s12 );
        tmp[1][i] = sto<BD>( 2 * d03 + d12 );
        tmp[2][i] = sto<BD>( s03 - s12 );
        tmp[3][i] = sto<BD>( d03 - 2 * d12 );
    }
#pragma unroll
    for( int i = 0; i < 4; i++ )
    {
        int s03 = tmp[i][0] + tmp[i][3], s12 = tmp[i][1] + tmp[i][2];
        int d03 = tmp[i][0] - tmp[i][3], d12 = tmp[i][1] - tmp[i][2];
        out[i * 4 + 0] = sto<BD>( s03 + s12 );
        out[i * 4 + 1] = sto<BD>( 2 * d03 + d12 );
        out[i * 4 + 2] = sto<BD>( s03 - s12 );
        out[i * 4 + 3] = sto<BD>( d03 - 2 * d12 );
    }
}

// DCT8_1D, reference common/dct.c:332-356 (src/dst via lambdas on indices)
#define DCT8_1D_ARR( S, D )                                                             \
    {                                                                                   \
        int s07 = S( 0 ) + S( 7 ), s16 = S( 1 ) + S( 6 ), s25 = S( 2 ) + S( 5 ),        \
            s34 = S( 3 ) + S( 4 );                                                      \
        int a0 = s07 + s34, a1 = s16 + s25, a2 = s07 - s34, a3 = s16 - s25;             \
        int d07 = S( 0 ) - S( 7 ), d16 = S( 1 ) - S( 6 ), d25 = S( 2 ) - S( 5 ),        \
            d34 = S( 3 ) - S( 4 );                                                      \
        int a4 = d16 + d25 + ( d07 + ( d07 >> 1 ) );                                    \
        int a5 = d07 - d34 - ( d25 + ( d25 >> 1 ) );                                    \
        int a6 = d07 + d34 - ( d16 + ( d16 >> 1 ) );                                    \
        int a7 = d16 - d25 + ( d34 + ( d34 >> 1 ) );                                    \
        D( 0, a0 + a1 );                                                                \
        D( 1, a4 + ( a7 >> 2 ) );                                                       \
        D( 2, a2 + ( a3 >> 1 ) );                                                       \
        D( 3, a5 + ( a6 >> 2 ) );                                                       \
        D( 4, a0 - a1 );                                                                \
        D( 5, a6 - ( a5 >> 2 ) );                                                       \
        D( 6, ( a2 >> 1 ) - a3 );                                                       \
        D( 7, ( a4 >> 2 ) - a7 );                                                       \
    }

// sub8x8_dct8 on a difference block (d[y][x]); out[x*8+i] reference order
template <int BD>
__device__ __forceinline__ void dct8x8_core( int (&d)[8][8], int (&out)[64] )
{
    // column pass in place: column i, SRC(x) = d[x][i]
#pragma unroll
    for( int i = 0; i < 8; i++ )
    {
#define S( x ) d[x][i]
#define D( x, v ) t[x] = sto<BD>( v )
        int t[8];
        DCT8_1D_ARR( S, D )
#pragma unroll
        for( int x = 0; x < 8; x++ )
            d[x][i] = t[x];
#undef S
#undef D
    }
    // row pass: row i, SRC(x) = d[i][x], DST(x) = dct[x*8+i]
#pragma unroll
    for( int i = 0; i < 8; i++ )
    {
#define S( x ) d[i][x]
#define D( x, v ) out[(x) * 8 + i] = sto<BD>( v )
        DCT8_1D_ARR( S, D )
#undef S
#undef D
    }
}

// QUANT_ONE, reference common/quant.c:50-57, branch-free: s = 0 for coef > 0,
// -1 otherwise (coef == 0 takes the reference's negative branch too), so
// |coef| = (coef ^ s) - s and the result is (q ^ s) - s.
__device__ __forceinline__ int quant_one( int coef, uint32_t mf, uint32_t f )
{
    const int s = (coef > 0) - 1;
    const uint32_t mag = (uint32_t)((coef ^ s) - s);
    const int q = (int)(((f + mag) * mf) >> 16);
    return (q ^ s) - s;
}

// k-th entry of a uniform mf / bias row, read as dwords so the loads are
// scalar (s_load) even for the 16-bit tables of 8-bit depth
template <typename U>
__device__ __forceinline__ uint32_t urow( const U *__restrict__ p, int k )
{
    if constexpr( sizeof( U ) == 2 )
    {
        const uint32_t w = ((const uint32_t *)p)[k >> 1];
        return (k & 1) ? w >> 16 : w & 0xffff;
    }
    else
        return p[k];
}

template <typename T, int N>
__device__ __forceinline__ void store_coefs( T *dst, const int (&v)[N] )
{
#pragma unroll
    for( int k = 0; k < N; k++ )
        dst[k] = (T)v[k];
}

// ------------------------------------------------------- sub_dct_batch
template <int BD, int KIND>
__global__ __launch_bounds__( 256 ) void sub_dct_kernel( const typename PT<BD>::pixel *fenc, intptr_t fs,
                                                         const typename PT<BD>::pixel *fdec, intptr_t ds,
                                                         const int64_t *fo, const int64_t *dofs, int n,
                                                         typename PT<BD>::dctcoef *out )
{
    using dctcoef = typename PT<BD>::dctcoef;
    constexpr int NSUB = KIND == 0 ? 1 : KIND == 1 ? 4 : KIND == 2 ? 16 : KIND == 5 ? 1 : KIND == 6 ? 4 : 1;
    constexpr int OSZ = KIND == 0 ? 16 : KIND == 1 ? 64 : KIND == 2 ? 256 : KIND == 3 ? 4 : KIND == 4 ? 8 : KIND == 5 ? 64 : 256;
    // one lane per (block, sub-block) for the multi-block kinds
    const int64_t gi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t i = gi / NSUB;
    const int sub = (int)(gi % NSUB);
    if( i >= n )
        return;
    const typename PT<BD>::pixel *a = fenc + fo[i];
    const typename PT<BD>::pixel *b = fdec + dofs[i];
    dctcoef *o = out + i * OSZ;
    if constexpr( KIND <= 2 )
    {
        // quadrant-major 4x4 order (dct.c:191-205)
        int i8 = sub >> 2, i4 = sub & 3;
        int x = (i8 & 1) * 8 + (i4 & 1) * 4, y = (i8 >> 1) * 8 + (i4 >> 1) * 4;
        int d[4][4], c[16];
        load_diff<BD, 4>( d, a + y * fs + x, fs, b + y * ds + x, ds );
        dct4x4_core<BD>( d, c );
        store_coefs( o + sub * 16, c );
    }
    else if constexpr( KIND == 3 || KIND == 4 )
    {
        // DC sums of 4x4 sub-blocks then the 2x2 / 2x4 butterflies
        constexpr int NB = KIND == 3 ? 4 : 8;
        int s[8];
#pragma unroll
        for( int k = 0; k < NB; k++ )
        {
            int d[4][4];
            int x = (k & 1) * 4, y = (k >> 1) * 4;
            load_diff<BD, 4>( d, a + y * fs + x, fs, b + y * ds + x, ds );
            int t = 0;
#pragma unroll
            for( int yy = 0; yy < 4; yy++ )
#pragma unroll
                for( int xx = 0; xx < 4; xx++ )
                    t += d[yy][xx];
            s[k] = t;
        }
        if constexpr( KIND == 3 )
        {
            // sums are stored to dctcoef before the 2x2 transform (dct.c:218-231)
            int e0 = sto<BD>( s[0] ), e1 = sto<BD>( s[1] ), e2 = sto<BD>( s[2] ), e3 = sto<BD>( s[3] );
            int d0 = e0 + e1, d1 = e2 + e3, d2 = e0 - e1, d3 = e2 - e3;
            o[0] = (dctcoef)(d0 + d1);
            o[1] = (dctcoef)(d0 - d1);
            o[2] = (dctcoef)(d2 + d3);
            o[3] = (dctcoef)(d2 - d3);
        }
        else
        {
            int b0 = s[0] + s[1], b1 = s[2] + s[3], b2 = s[4] + s[5], b3 = s[6] + s[7];
            int b4 = s[0] - s[1], b5 = s[2] - s[3], b6 = s[4] - s[5], b7 = s[6] - s[7];
            int c0 = b0 + b1, c1 = b2 + b3, c2 = b4 + b5, c3 = b6 + b7;
            int c4 = b0 - b1, c5 = b2 - b3, c6 = b4 - b5, c7 = b6 - b7;
            o[0] = (dctcoef)(c0 + c1);
            o[1] = (dctcoef)(c2 + c3);
            o[2] = (dctcoef)(c0 - c1);
            o[3] = (dctcoef)(c2 - c3);
            o[4] = (dctcoef)(c4 - c5);
            o[5] = (dctcoef)(c6 - c7);
            o[6] = (dctcoef)(c4 + c5);
            o[7] = (dctcoef)(c6 + c7);
        }
    }
    else
    {
        int x = (sub & 1) * 8, y = (sub >> 1) * 8;
        int d[8][8], c[64];
        load_diff<BD, 8>( d, a + y * fs + x, fs, b + y * ds + x, ds );
        dct8x8_core<BD>( d, c );
        store_coefs( o + sub * 64, c );
    }
}

template <int BD>
hipError_t launch_sub_dct( int kind, const typename PT<BD>::pixel *fenc, intptr_t fs,
                           const typename PT<BD>::pixel *fdec, intptr_t ds, const int64_t *fo,
                           const int64_t *dofs, int n, typename PT<BD>::dctcoef *dct, hipStream_t stream )
{
    static const int nsub[7] = { 1, 4, 16, 1, 1, 1, 4 };
    if( kind < 0 || kind > 6 )
        return hipErrorInvalidValue;
    if( n <= 0 )
        return hipSuccess;
    int64_t lanes = (int64_t)n * nsub[kind];
    dim3 blk( 256 ), g( (unsigned)((lanes + 255) / 256) );
    switch( kind )
    {
#define SD_CASE( K ) \
        case K: hipLaunchKernelGGL( ( sub_dct_kernel<BD, K> ), g, blk, 0, stream, fenc, fs, fdec, ds, fo, dofs, n, dct ); break;
        SD_CASE( 0 ) SD_CASE( 1 ) SD_CASE( 2 ) SD_CASE( 3 ) SD_CASE( 4 ) SD_CASE( 5 ) SD_CASE( 6 )
#undef SD_CASE
    }
    return hipGetLastError();
}

// ------------------------------------------------------------ dc_batch
template <int BD>
__global__ __launch_bounds__( 256 ) void dc4x4_kernel( typename PT<BD>::dctcoef *dct, int n )
{
    using dctcoef = typename PT<BD>::dctcoef;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if( i >= n )
        return;
    dctcoef *d = dct + i * 16;
    int v[16], tmp[16];
#pragma unroll
    for( int k = 0; k < 16; k++ )
        v[k] = d[k];
#pragma unroll
    for( int r = 0; r < 4; r++ )
    {
        int s01 = v[r * 4 + 0] + v[r * 4 + 1], d01 = v[r * 4 + 0] - v[r * 4 + 1];
        int s23 = v[r * 4 + 2] + v[r * 4 + 3], d23 = v[r * 4 + 2] - v[r * 4 + 3];
        tmp[0 * 4 + r] = sto<BD>( s01 + s23 );
        tmp[1 * 4 + r] = sto<BD>( s01 - s23 );
        tmp[2 * 4 + r] = sto<BD>( d01 - d23 );
        tmp[3 * 4 + r] = sto<BD>( d01 + d23 );
    }
#pragma unroll
    for( int r = 0; r < 4; r++ )
    {
        int s01 = tmp[r * 4 + 0] + tmp[r * 4 + 1], d01 = tmp[r * 4 + 0] - tmp[r * 4 + 1];
        int s23 = tmp[r * 4 + 2] + tmp[r * 4 + 3], d23 = tmp[r * 4 + 2] - tmp[r * 4 + 3];
        d[r * 4 + 0] = (dctcoef)((s01 + s23 + 1) >> 1);
        d[r * 4 + 1] = (dctcoef)((s01 - s23 + 1) >> 1);
        d[r * 4 + 2] = (dctcoef)((d01 - d23 + 1) >> 1);
        d[r * 4 + 3] = (dctcoef)((d01 + d23 + 1) >> 1);
    }
}

template <int BD>
__global__ __launch_bounds__( 256 ) void dc2x4_kernel( typename PT<BD>::dctcoef *dct,
                                                       typename PT<BD>::dctcoef *dct4x4, int n )
{
    using dctcoef = typename PT<BD>::dctcoef;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if( i >= n )
        return;
    dctcoef *o = dct + i * 8;
    dctcoef *s = dct4x4 + i * 128;
    int a[8];
#pragma unroll
    for( int k = 0; k < 8; k++ )
        a[k] = s[k * 16];
    int a0 = a[0] + a[1], a1 = a[2] + a[3], a2 = a[4] + a[5], a3 = a[6] + a[7];
    int a4 = a[0] - a[1], a5 = a[2] - a[3], a6 = a[4] - a[5], a7 = a[6] - a[7];
    int b0 = a0 + a1, b1 = a2 + a3, b2 = a4 + a5, b3 = a6 + a7;
    int b4 = a0 - a1, b5 = a2 - a3, b6 = a4 - a5, b7 = a6 - a7;
    o[0] = (dctcoef)(b0 + b1);
    o[1] = (dctcoef)(b2 + b3);
    o[2] = (dctcoef)(b0 - b1);
    o[3] = (dctcoef)(b2 - b3);
    o[4] = (dctcoef)(b4 - b5);
    o[5] = (dctcoef)(b6 - b7);
    o[6] = (dctcoef)(b4 + b5);
    o[7] = (dctcoef)(b6 + b7);
#pragma unroll
    for( int k = 0; k < 8; k++ )
        s[k * 16] = 0;
}

template <int BD>
hipError_t launch_dc( int kind, typename PT<BD>::dctcoef *dct, typename PT<BD>::dctcoef *dct4x4, int n,
                      hipStream_t stream )
{
    if( n <= 0 )
        return hipSuccess;
    dim3 blk( 256 ), g( (n + 255) / 256 );
    if( kind == 0 )
        hipLaunchKernelGGL( ( dc4x4_kernel<BD> ), g, blk, 0, stream, dct, n );
    else if( kind == 1 )
        hipLaunchKernelGGL( ( dc2x4_kernel<BD> ), g, blk, 0, stream, dct, dct4x4, n );
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// --------------------------------------------------------- quant_batch
// KIND as X264HIP_QUANT_*: 0 8x8, 1 4x4, 2 4x4x4, 3 4x4_dc, 4 2x2_dc
template <int BD, int KIND>
__global__ __launch_bounds__( 256 ) void quant_kernel( typename PT<BD>::dctcoef *dct,
                                                       const typename PT<BD>::udctcoef *__restrict__ mf,
                                                       const typename PT<BD>::udctcoef *__restrict__ bias,
                                                       int mf_dc, int bias_dc, int n, int32_t *nz )
{
    using dctcoef = typename PT<BD>::dctcoef;
    constexpr int N = KIND == 0 ? 64 : KIND == 2 ? 64 : KIND == 4 ? 4 : 16;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if( i >= n )
        return;
    dctcoef *d = dct + i * N;
    int acc = 0, mask = 0;
#pragma unroll
    for( int k = 0; k < N; k++ )
    {
        uint32_t m, f;
        if constexpr( KIND >= 3 )
            m = (uint32_t)mf_dc, f = (uint32_t)bias_dc;
        else
            m = mf[k & (KIND == 0 ? 63 : 15)], f = bias[k & (KIND == 0 ? 63 : 15)];
        int q = sto<BD>( quant_one( d[k], m, f ) );   // nz sees the stored value (quant.c:56)
        d[k] = (dctcoef)q;
        acc |= q;
        if constexpr( KIND == 2 )
            if( (k & 15) == 15 )
            {
                mask |= (acc != 0) << (k >> 4);
                acc = 0;
            }
    }
    if( nz )
        nz[i] = KIND == 2 ? mask : (acc != 0);
}

template <int BD>
hipError_t launch_quant( int kind, typename PT<BD>::dctcoef *dct, const typename PT<BD>::udctcoef *mf,
                         const typename PT<BD>::udctcoef *bias, int mf_dc, int bias_dc, int n, int32_t *nz,
                         hipStream_t stream )
{
    if( n <= 0 )
        return hipSuccess;
    dim3 blk( 256 ), g( (n + 255) / 256 );
    switch( kind )
    {
#define Q_CASE( K ) \
        case K: hipLaunchKernelGGL( ( quant_kernel<BD, K> ), g, blk, 0, stream, dct, mf, bias, mf_dc, bias_dc, n, nz ); break;
        Q_CASE( 0 ) Q_CASE( 1 ) Q_CASE( 2 ) Q_CASE( 3 ) Q_CASE( 4 )
#undef Q_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ------------------------------------------------- fused mb_dct_quant
// Strip mapping (10-bit transform 8): one wave = one 256-pixel-wide strip of one MB row
// (16 macroblocks).  For T=4 lane l owns the 4-pixel column l of the strip and
// walks its 4 block rows, so every row load is 64 contiguous dwords (fully
// coalesced); for T=8 lane l owns 8x8 column l%32 of block row l/32 (two
// 256-byte row segments per load).  The per-MB nz mask is OR-combined across
// the MB's lanes with DPP / lane swaps.
// NT: nontemporal coefficient stores; WPB waves per workgroup (4, or 1: a quarter of the
// LDS stage per workgroup -- 16 KB instead of 64 at 10 bit, where the stage held the kernel
// to 2 resident waves per SIMD)
template <int BD, int T, bool STAGE, bool NT = false, int WPB = 4>
__global__ __launch_bounds__( 64 * WPB ) void mb_dct_quant_strip_kernel(
    const typename PT<BD>::pixel *__restrict__ fenc, intptr_t fs, intptr_t ffs,
    const typename PT<BD>::pixel *__restrict__ pred, intptr_t ps, intptr_t pfs, int mbw, int mbh, int nframes,
    const typename PT<BD>::udctcoef *__restrict__ mf, const typename PT<BD>::udctcoef *__restrict__ bias,
    typename PT<BD>::dctcoef *__restrict__ dct, int32_t *__restrict__ nz )
{
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int spr = (mbw + 15) >> 4;
    if( wave >= (int64_t)nframes * mbh * spr )
        return;                                               // wave-uniform
    const int strip = (int)(wave % spr);
    const int64_t t = wave / spr;
    const int mby = (int)(t % mbh);
    const int64_t f = t / mbh;
    const typename PT<BD>::pixel *a0 = fenc + f * ffs + (intptr_t)16 * mby * fs + 256 * strip;
    const typename PT<BD>::pixel *b0 = pred + f * pfs + (intptr_t)16 * mby * ps + 256 * strip;
    const int64_t mbrow = (f * mbh + mby) * (int64_t)mbw;
    // STAGE: the wave's 16 MBs of coefficients are assembled in LDS and leave as
    // one contiguous run of 16 B per lane stores
    using dctcoef = typename PT<BD>::dctcoef;
    __shared__ dctcoef lds[STAGE ? WPB * 16 * 256 : 1];
    dctcoef *stage = lds + (threadIdx.x >> 6) * (16 * 256);
    if constexpr( T == 4 )
    {
        const int mbx = strip * 16 + (lane >> 2);
        const bool live = mbx < mbw;
        const int cx = lane & 3;                              // 4-px column inside the MB
        int mask = 0;
#pragma unroll
        for( int by = 0; by < 4; by++ )
        {
            if( live )
            {
                int d[4][4], c[16];
                load_diff<BD, 4>( d, a0 + 4 * by * fs + 4 * lane, fs, b0 + 4 * by * ps + 4 * lane, ps );
                dct4x4_core<BD>( d, c );
                int acc = 0;
#pragma unroll
                for( int k = 0; k < 16; k++ )
                {
                    c[k] = sto<BD>( quant_one( c[k], urow( mf, k ), urow( bias, k ) ) );
                    acc |= c[k];
                }
                const int i8 = (by >> 1) * 2 + (cx >> 1), i4 = (by & 1) * 2 + (cx & 1);
                if constexpr( STAGE )
                    store_coefs( stage + (lane >> 2) * 256 + (i8 * 4 + i4) * 16, c );
                else
                    store_coefs( dct + (mbrow + mbx) * 256 + (i8 * 4 + i4) * 16, c );
                mask |= (acc != 0) << (4 * i8 + i4);
            }
        }
        // OR over the four lanes of the MB: quad_perm [1,0,3,2] then [2,3,0,1]
        mask |= __builtin_amdgcn_update_dpp( 0, mask, 0xB1, 0xF, 0xF, false );
        mask |= __builtin_amdgcn_update_dpp( 0, mask, 0x4E, 0xF, 0xF, false );
        if( live && cx == 0 )
            nz[mbrow + mbx] = mask;
    }
    else
    {
        const int bx = lane & 31, by = lane >> 5;             // 8x8 block column / row in the strip
        const int mbx = strip * 16 + (bx >> 1);
        const bool live = mbx < mbw;
        int mask = 0;
        if( live )
        {
            int d[8][8], c[64];
            load_diff<BD, 8>( d, a0 + 8 * by * fs + 8 * bx, fs, b0 + 8 * by * ps + 8 * bx, ps );
            dct8x8_core<BD>( d, c );
            int acc = 0;
#pragma unroll
            for( int k = 0; k < 64; k++ )
            {
                c[k] = sto<BD>( quant_one( c[k], urow( mf, k ), urow( bias, k ) ) );
                acc |= c[k];
            }
            const int i8 = by * 2 + (bx & 1);
            if constexpr( STAGE )
                store_coefs( stage + (bx >> 1) * 256 + i8 * 64, c );
            else
                store_coefs( dct + (mbrow + mbx) * 256 + i8 * 64, c );
            mask = (acc != 0) << i8;
        }
        mask |= __builtin_amdgcn_update_dpp( 0, mask, 0xB1, 0xF, 0xF, false );   // lane ^ 1
        mask |= __shfl_xor( mask, 32 );                                           // other block row
        if( live && by == 0 && !(bx & 1) )
            nz[mbrow + mbx] = mask;
    }
    if constexpr( STAGE )
    {
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence( __ATOMIC_RELEASE, "wavefront" );
        // the wave's MBs are consecutive in the table: copy n*256 coefficients
        const int nmb = min( 16, mbw - strip * 16 );
        const int nvec = nmb * 256 * (int)sizeof( dctcoef ) / 16;
        const uint4 *src = (const uint4 *)stage;
        uint4 *dst = (uint4 *)(dct + (mbrow + strip * 16) * 256);
        for( int i = lane; i < nvec; i += 64 )
            st16<NT>( dst + i, src[i] );
    }
}

// 16 pixels of a row as one vector load when aligned
template <int BD>
__device__ __forceinline__ void load16( const typename PT<BD>::pixel *p, uint32_t (&w)[16 / PT<BD>::PPD] )
{
    constexpr int N = 16 / PT<BD>::PPD;
    if( ((uintptr_t)p & 15) == 0 )
    {
#pragma unroll
        for( int k = 0; k < N / 4; k++ )
        {
            const uint4 v = ((const uint4 *)p)[k];
            w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
        }
    }
    else
        load_packed<N>( p, w );
}

// Transform 4 (both depths): one lane per (4-row band, MB, half) of an 8-MB strip: a lane
// reads 8 pixels per row and transforms two 4x4 blocks, stages them in LDS so the strip's
// coefficients leave as contiguous 16-byte stores (0.62-0.71 of HBM against 0.50-0.52 for
// the 16-MB strip with a lane per 4-pixel column, and a lane per (MB, band) of a 16-MB
// strip in between: a round-3 A/B whose driver was removed with the losing kernels).
template <int BD, bool NT = false>
__global__ __launch_bounds__( 256 ) void mb_dct_quant_halfband_kernel(
    const typename PT<BD>::pixel *__restrict__ fenc, intptr_t fs, intptr_t ffs,
    const typename PT<BD>::pixel *__restrict__ pred, intptr_t ps, intptr_t pfs, int mbw, int mbh, int nframes,
    const typename PT<BD>::udctcoef *__restrict__ mf, const typename PT<BD>::udctcoef *__restrict__ bias,
    typename PT<BD>::dctcoef *__restrict__ dct, int32_t *__restrict__ nz, int xcd, int sh )
{
    using dctcoef = typename PT<BD>::dctcoef;
    constexpr int PPD = PT<BD>::PPD;
    const int lane = threadIdx.x & 63;
    const uint32_t blk = xcd ? xcd_block( blockIdx.x, gridDim.x ) : blockIdx.x;
    const int64_t wave = ((int64_t)blk * blockDim.x + threadIdx.x) >> 6;
    const int spr = (mbw + sh + 7) >> 3;
    if( wave >= (int64_t)nframes * mbh * spr )
        return;                                               // wave-uniform
    const int strip = (int)(wave % spr);
    const int64_t t = wave / spr;
    const int mby = (int)(t % mbh);
    const int64_t f = t / mbh;
    const int m = (lane & 15) >> 1, half = lane & 1, by = lane >> 4;
    const int first = strip * 8 - sh;                         // the strip's first MB (< 0: left of the row)
    const int mbx = first + m;
    const bool live = mbx >= 0 && mbx < mbw;
    const int64_t mbrow = (f * mbh + mby) * (int64_t)mbw;
    __shared__ dctcoef lds[4 * 8 * 256];
    dctcoef *stage = lds + (threadIdx.x >> 6) * (8 * 256);
    int mask = 0;
    if( live )
    {
        const typename PT<BD>::pixel *a = fenc + f * ffs + (intptr_t)(16 * mby + 4 * by) * fs + 16 * mbx + 8 * half;
        const typename PT<BD>::pixel *b = pred + f * pfs + (intptr_t)(16 * mby + 4 * by) * ps + 16 * mbx + 8 * half;
        int d[2][4][4];
#pragma unroll
        for( int y = 0; y < 4; y++ )
        {
            uint32_t wa[8 / PPD], wb[8 / PPD];
            load_packed<8 / PPD>( a + y * fs, wa );
            load_packed<8 / PPD>( b + y * ps, wb );
#pragma unroll
            for( int x = 0; x < 8; x++ )
                d[x >> 2][y][x & 3] = upix<BD>( wa[x / PPD], x % PPD ) - upix<BD>( wb[x / PPD], x % PPD );
        }
#pragma unroll
        for( int k2 = 0; k2 < 2; k2++ )
        {
            int c[16];
            dct4x4_core<BD>( d[k2], c );
            int acc = 0;
#pragma unroll
            for( int k = 0; k < 16; k++ )
            {
                c[k] = sto<BD>( quant_one( c[k], urow( mf, k ), urow( bias, k ) ) );
                acc |= c[k];
            }
            const int i8 = (by >> 1) * 2 + half, i4 = (by & 1) * 2 + k2;
            store_coefs( stage + m * 256 + (i8 * 4 + i4) * 16, c );
            mask |= (acc != 0) << (4 * i8 + i4);
        }
    }
    mask |= __builtin_amdgcn_update_dpp( 0, mask, 0xB1, 0xF, 0xF, false );   // lane ^ 1
    mask |= __shfl_xor( mask, 16 );
    mask |= __shfl_xor( mask, 32 );
    if( live && by == 0 && half == 0 )
        nz[mbrow + mbx] = mask;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence( __ATOMIC_RELEASE, "wavefront" );
    const int lo = max( first, 0 ), hi = min( first + 8, mbw );
    const int nvec = (hi - lo) * 256 * (int)sizeof( dctcoef ) / 16;
    const uint4 *src = (const uint4 *)(stage + (lo - first) * 256);
    uint4 *dst = (uint4 *)(dct + (mbrow + lo) * 256);
    for( int i = lane; i < nvec; i += 64 )
        st16<NT>( dst + i, src[i] );
}

// Variant 6 (8 bit, transform 8, the default there): sub8x8_dct8 + quant_8x8 on
// packed 16-bit pairs.  For 8-bit residuals the reference's int16 intermediates
// (dct.c:332-377) never leave int16 range -- column-pass outputs are at most
// 8*255 = 2040 in magnitude and every row-pass partial sum at most ~17.9k -- so
// v_pk_* arithmetic on pairs gives the reference's values bit for bit: the
// column pass runs on pairs of adjacent columns as the pixels arrive, one
// v_perm per register regroups them into pairs of rows, and the row pass then
// yields the reference's out[x*8+i], out[x*8+i+1] already paired in memory
// order.  QUANT_ONE runs on pairs too: |c| and the sign with v_pk ops, the
// uint32 (f + |c|) * mf as |c| * mf + f*mf (f*mf from the scalar unit, wrap
// preserved) in 24-bit multiply-adds, and one v_perm takes both >> 16 results.
// Same strip mapping as mb_dct_quant_strip_kernel; the LDS stage is
// XOR-swizzled per 16-B chunk so the eight lanes of a ds_write_b128 group hit
// distinct banks.
typedef short dq_s2 __attribute__( ( ext_vector_type( 2 ) ) );

__device__ __forceinline__ dq_s2 dq_as2( uint32_t v ) { return __builtin_bit_cast( dq_s2, v ); }
__device__ __forceinline__ uint32_t dq_asu( dq_s2 v ) { return __builtin_bit_cast( uint32_t, v ); }

#define DCT8_1D_PK( S, D )                                                              \
    {                                                                                   \
        const dq_s2 s07 = S( 0 ) + S( 7 ), s16 = S( 1 ) + S( 6 ), s25 = S( 2 ) + S( 5 ), \
                    s34 = S( 3 ) + S( 4 );                                              \
        const dq_s2 a0 = s07 + s34, a1 = s16 + s25, a2 = s07 - s34, a3 = s16 - s25;     \
        const dq_s2 d07 = S( 0 ) - S( 7 ), d16 = S( 1 ) - S( 6 ), d25 = S( 2 ) - S( 5 ), \
                    d34 = S( 3 ) - S( 4 );                                              \
        const dq_s2 a4 = d16 + d25 + ( d07 + ( d07 >> 1 ) );                            \
        const dq_s2 a5 = d07 - d34 - ( d25 + ( d25 >> 1 ) );                            \
        const dq_s2 a6 = d07 + d34 - ( d16 + ( d16 >> 1 ) );                            \
        const dq_s2 a7 = d16 - d25 + ( d34 + ( d34 >> 1 ) );                            \
        D( 0, a0 + a1 );                                                                \
        D( 1, a4 + ( a7 >> 2 ) );                                                       \
        D( 2, a2 + ( a3 >> 1 ) );                                                       \
        D( 3, a5 + ( a6 >> 2 ) );                                                       \
        D( 4, a0 - a1 );                                                                \
        D( 5, a6 - ( a5 >> 2 ) );                                                       \
        D( 6, ( a2 >> 1 ) - a3 );                                                       \
        D( 7, ( a4 >> 2 ) - a7 );                                                       \
    }

template <bool STAGE, bool NT = false>
__global__ __launch_bounds__( 256 ) void mb_dct8_quant_pk_kernel( const uint8_t *__restrict__ fenc, intptr_t fs,
                                                                  intptr_t ffs, const uint8_t *__restrict__ pred,
                                                                  intptr_t ps, intptr_t pfs, int mbw, int mbh,
                                                                  int nframes, const uint16_t *__restrict__ mf,
                                                                  const uint16_t *__restrict__ bias,
                                                                  int16_t *__restrict__ dct, int32_t *__restrict__ nz,
                                                                  int xcd, int sh )
{
    const int lane = threadIdx.x & 63;
    const uint32_t blk = xcd ? xcd_block( blockIdx.x, gridDim.x ) : blockIdx.x;
    const int64_t wave = ((int64_t)blk * blockDim.x + threadIdx.x) >> 6;
    const int spr = (mbw + sh + 15) >> 4;
    if( wave >= (int64_t)nframes * mbh * spr )
        return;                                               // wave-uniform
    const int strip = (int)(wave % spr);
    const int64_t t = wave / spr;
    const int mby = (int)(t % mbh);
    const int64_t f = t / mbh;
    const int64_t mbrow = (f * mbh + mby) * (int64_t)mbw;
    __shared__ uint4 lds[STAGE ? 4 * 64 * 8 : 1];             // per wave: 64 blocks x 8 chunks of 16 B
    uint4 *stage = lds + (threadIdx.x >> 6) * 512;
    const int first = strip * 16 - sh;                        // the strip's first MB (< 0: left of the row)
    const int lo = max( first, 0 ), hi = min( first + 16, mbw );
    // chunk i (16 B) of the strip's MB (first + i / 32) lives at dst[i - c0]
    const int c0 = (lo - first) * 32;
    uint4 *dst = (uint4 *)(dct + (mbrow + lo) * 256);
    const int bx = lane & 31, by = lane >> 5;                 // 8x8 block column / row in the strip
    const int mbx = first + (bx >> 1);
    const bool live = mbx >= 0 && mbx < mbw;
    const int slot = (bx >> 1) * 4 + by * 2 + (bx & 1);      // block of the wave's 16 MBs, table order
    const int key = bx & 7;
    int mask = 0;
    if( live )
    {
        const uint8_t *a = fenc + f * ffs + (intptr_t)(16 * mby + 8 * by) * fs + 16 * first + 8 * bx;
        const uint8_t *b = pred + f * pfs + (intptr_t)(16 * mby + 8 * by) * ps + 16 * first + 8 * bx;
        dq_s2 P[8][4];                                        // P[row][k] = (d[row][2k], d[row][2k+1])
#pragma unroll
        for( int y = 0; y < 8; y++ )
        {
            uint32_t wa[2], wb[2];
            load_packed<2>( a + y * fs, wa );
            load_packed<2>( b + y * ps, wb );
#pragma unroll
            for( int k = 0; k < 2; k++ )
            {
                P[y][2 * k] = dq_as2( __builtin_amdgcn_perm( 0u, wa[k], 0x0c010c00u ) ) -
                              dq_as2( __builtin_amdgcn_perm( 0u, wb[k], 0x0c010c00u ) );
                P[y][2 * k + 1] = dq_as2( __builtin_amdgcn_perm( 0u, wa[k], 0x0c030c02u ) ) -
                                  dq_as2( __builtin_amdgcn_perm( 0u, wb[k], 0x0c030c02u ) );
            }
        }
        // column pass on column pairs: SRC(x) = d[x][i]
#pragma unroll
        for( int k = 0; k < 4; k++ )
        {
            dq_s2 o[8];
#define S( x ) P[x][k]
#define D( x, v ) o[x] = ( v )
            DCT8_1D_PK( S, D )
#undef S
#undef D
#pragma unroll
            for( int x = 0; x < 8; x++ )
                P[x][k] = o[x];
        }
        // row pass on row pairs (2j, 2j+1): out[x*8+2j], out[x*8+2j+1] = dword x*4+j
        uint32_t out[8][4];
        uint32_t acc = 0;
#pragma unroll
        for( int j = 0; j < 4; j++ )
        {
            dq_s2 q[8];
#pragma unroll
            for( int k = 0; k < 4; k++ )
            {
                q[2 * k] = dq_as2( __builtin_amdgcn_perm( dq_asu( P[2 * j + 1][k] ), dq_asu( P[2 * j][k] ), 0x05040100u ) );
                q[2 * k + 1] =
                    dq_as2( __builtin_amdgcn_perm( dq_asu( P[2 * j + 1][k] ), dq_asu( P[2 * j][k] ), 0x07060302u ) );
            }
            dq_s2 r[8];
#define S( x ) q[x]
#define D( x, v ) r[x] = ( v )
            DCT8_1D_PK( S, D )
#undef S
#undef D
#pragma unroll
            for( int x = 0; x < 8; x++ )
            {
                const uint32_t mfw = ((const uint32_t *)mf)[x * 4 + j];
                const uint32_t bw = ((const uint32_t *)bias)[x * 4 + j];
                const uint32_t fml = (mfw & 0xffff) * (bw & 0xffff), fmh = (mfw >> 16) * (bw >> 16);
                const dq_s2 c = r[x];
                const dq_s2 ng = (dq_s2)0 - c;
                const uint32_t mg = dq_asu( __builtin_elementwise_max( c, ng ) );
                const uint32_t ql = (mg & 0xffff) * (mfw & 0xffff) + fml;
                const uint32_t qh = (mg >> 16) * (mfw >> 16) + fmh;
                const dq_s2 qv = dq_as2( __builtin_amdgcn_perm( qh, ql, 0x07060302u ) );
                const dq_s2 sg = ng >> 15;                    // -1 where c > 0, else 0 (QUANT_ONE's branches)
                const uint32_t v = dq_asu( sg - (qv ^ sg) );
                out[x][j] = v;
                acc |= v;
            }
        }
        mask = (acc != 0) << (by * 2 + (bx & 1));
#pragma unroll
        for( int x = 0; x < 8; x++ )
        {
            const uint4 v = make_uint4( out[x][0], out[x][1], out[x][2], out[x][3] );
            if constexpr( STAGE )
                stage[slot * 8 + (x ^ key)] = v;
            else
                dst[slot * 8 + x - c0] = v;
        }
    }
    mask |= __builtin_amdgcn_update_dpp( 0, mask, 0xB1, 0xF, 0xF, false );   // lane ^ 1
    mask |= __shfl_xor( mask, 32 );                                           // other block row
    if( live && by == 0 && !(bx & 1) )
        nz[mbrow + mbx] = mask;
    if constexpr( !STAGE )
        return;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence( __ATOMIC_RELEASE, "wavefront" );
    for( int i = c0 + lane; i < (hi - first) * 32; i += 64 )
    {
        const int s = i >> 3;
        const int k = (((s >> 2) * 2 + (s & 1)) & 7);        // the writer's key
        st16<NT>( dst + i - c0, stage[s * 8 + ((i & 7) ^ k)] );
    }
}
#undef DCT8_1D_PK

template <int BD>
hipError_t launch_mb_dct_quant( int transform, const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                                const typename PT<BD>::pixel *pred, intptr_t ps, intptr_t pfs, int mbw, int mbh,
                                int nframes, const typename PT<BD>::udctcoef *mf,
                                const typename PT<BD>::udctcoef *bias, typename PT<BD>::dctcoef *dct, int32_t *nz,
                                hipStream_t stream )
{
    if( transform != 4 && transform != 8 )
        return hipErrorInvalidValue;
    const int64_t waves = (int64_t)nframes * mbh * ((mbw + 15) / 16);
    if( waves <= 0 )
        return hipSuccess;
    dim3 blk( 256 );
    // nontemporal coefficient stores (stream_nt): 64 frames 4x4 0.0985 -> 0.0876 ms, 8x8
    // 0.1029 -> 0.0776 ms; 16 frames 0.0279 -> 0.0267, 0.0263 -> 0.0247 (profiles/r03s_nt_ab.json)
    const bool nt = stream_nt();
    // XCD-contiguous strips (X264HIP_STREAM_XCD=1 turns them on): a row's neighbouring
    // strips share the 128-B lines their MB columns straddle, so in one XCD's L2 those
    // lines are fetched once instead of once per XCD.  With the sector shift below no
    // line is shared and the order only cost time (64 frames: 0.1056 vs 0.1023 ms for 4x4,
    // profiles/r03af_dq_ab.log), so it is off by default
    const int xcd = variant( V_STREAM_XCD ) == 1;
    // Sector-aligned strips (as launch_mb_recon does for its stores): with row and frame
    // strides multiples of 64 bytes, x = 0 sits at the same offset in a 64-byte sector on
    // every row, so shifting the strips left by that offset (in MBs) puts every wave's
    // row pieces of the source on whole sectors, none shared by two waves (fetch 1.27x ->
    // 1.00x of the algorithmic reads for 4x4, 1.11x -> 1.01x for 8x8, profiles/r03ae-af)
    const size_t psz = sizeof( typename PT<BD>::pixel );
    const bool al = !(((size_t)fs * psz) & 63) && !(((size_t)ffs * psz) & 63);
    const int off = al ? (int)((uintptr_t)fenc & 63) : 0;
    const int sh = off % (16 * (int)psz) ? 0 : off / (16 * (int)psz);
    if( transform == 4 )
    {
        const int64_t hw = (int64_t)nframes * mbh * ((mbw + sh + 7) / 8);
        if( nt )
            hipLaunchKernelGGL( ( mb_dct_quant_halfband_kernel<BD, true> ), dim3( (unsigned)((hw + 3) / 4) ), blk, 0,
                                stream, fenc, fs, ffs, pred, ps, pfs, mbw, mbh, nframes, mf, bias, dct, nz, xcd, sh );
        else
            hipLaunchKernelGGL( mb_dct_quant_halfband_kernel<BD>, dim3( (unsigned)((hw + 3) / 4) ), blk, 0, stream,
                                fenc, fs, ffs, pred, ps, pfs, mbw, mbh, nframes, mf, bias, dct, nz, xcd, sh );
        return hipGetLastError();
    }
    if constexpr( BD == 8 )
    {
        // 8 bit: packed 16-bit pair arithmetic, swizzled LDS staging (0.56 -> 0.66 of HBM)
        const dim3 g( (unsigned)(((int64_t)nframes * mbh * ((mbw + sh + 15) / 16) + 3) / 4) );
        if( nt )
            hipLaunchKernelGGL( ( mb_dct8_quant_pk_kernel<true, true> ), g, blk, 0, stream, fenc, fs, ffs, pred, ps,
                                pfs, mbw, mbh, nframes, mf, bias, dct, nz, xcd, sh );
        else
            hipLaunchKernelGGL( mb_dct8_quant_pk_kernel<true>, g, blk, 0, stream, fenc, fs, ffs, pred, ps, pfs, mbw,
                                mbh, nframes, mf, bias, dct, nz, xcd, sh );
    }
    else
    {
        // 10 bit: staged 16-MB strips in one-wave workgroups (0.2011 vs 0.2165 ms for four-wave
        // workgroups at 64 1080p pairs, 0.665 vs 0.618 of HBM: the 64 KB stage of a four-wave
        // workgroup held it to 2 waves per SIMD; profiles/r03aj_dq_ab10.log)
        if( nt )
            hipLaunchKernelGGL( ( mb_dct_quant_strip_kernel<BD, 8, true, true, 1> ), dim3( (unsigned)waves ),
                                dim3( 64 ), 0, stream, fenc, fs, ffs, pred, ps, pfs, mbw, mbh, nframes, mf, bias, dct,
                                nz );
        else
            hipLaunchKernelGGL( ( mb_dct_quant_strip_kernel<BD, 8, true, false, 1> ), dim3( (unsigned)waves ),
                                dim3( 64 ), 0, stream, fenc, fs, ffs, pred, ps, pfs, mbw, mbh, nframes, mf, bias, dct,
                                nz );
    }
    return hipGetLastError();
}

#define INST( BD )                                                                                                 \
    template hipError_t launch_sub_dct<BD>( int, const PT<BD>::pixel *, intptr_t, const PT<BD>::pixel *, intptr_t, \
                                            const int64_t *, const int64_t *, int, PT<BD>::dctcoef *, hipStream_t ); \
    template hipError_t launch_dc<BD>( int, PT<BD>::dctcoef *, PT<BD>::dctcoef *, int, hipStream_t );             \
    template hipError_t launch_quant<BD>( int, PT<BD>::dctcoef *, const PT<BD>::udctcoef *,                        \
                                          const PT<BD>::udctcoef *, int, int, int, int32_t *, hipStream_t );        \
    template hipError_t launch_mb_dct_quant<BD>( int, const PT<BD>::pixel *, intptr_t, intptr_t,                   \
                                                 const PT<BD>::pixel *, intptr_t, intptr_t, int, int, int,        \
                                                 const PT<BD>::udctcoef *, const PT<BD>::udctcoef *,              \
                                                 PT<BD>::dctcoef *, int32_t *, hipStream_t );
INST( 8 )
INST( 10 )

} // namespace x264hip
