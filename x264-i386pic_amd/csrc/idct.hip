// Inverse path: dequantisation, inverse transforms with reconstruction,
// coefficient statistics and zigzag scans over block lists in device memory,
// plus the fused frame-level dequant + idct + add reconstruction.
//
// Semantics (reference):
//   add4x4_idct / add8x8_idct / add16x16_idct   common/dct.c:272-326
//   add8x8_idct8 / add16x16_idct8               common/dct.c:388-446
//   add*_idct_dc                                 common/dct.c:448-476
//   idct4x4dc                                    common/dct.c:78-107
//   dequant_4x4 / 8x8 / 4x4_dc                   common/quant.c:106-162
//   idct_dequant_2x4_dc / _dconly                common/quant.c:164-208
//   optimize_chroma_2x2_dc / 2x4_dc              common/quant.c:210-293
//   denoise_dct                                  common/quant.c:295-306
//   decimate_score15/16/64, coeff_last*, coeff_level_run*   common/quant.c:318-398
//   zigzag scans / sub / interleave              common/dct.c:768-940
// Every dctcoef store of the reference (int16 at 8 bit) is reproduced with sto<BD>.
#include "hipcommon.h"

#include <stdlib.h>

namespace x264hip {

// ------------------------------------------------------------------ helpers
// read N pixels of a row at any alignment
template <int BD, int N>
__device__ __forceinline__ void read_row( const typename PT<BD>::pixel *p, int (&v)[N] )
{
    constexpr int PPD = PT<BD>::PPD;
    uint32_t r[N / PPD];
    load_packed<N / PPD>( p, r );
#pragma unroll
    for( int x = 0; x < N; x++ )
        v[x] = upix<BD>( r[x / PPD], x % PPD );
}

// write N pixels of a row: packed dword stores when aligned, pixel stores otherwise
template <int BD, int N>
__device__ __forceinline__ void write_row( typename PT<BD>::pixel *p, const int (&v)[N] )
{
    constexpr int PPD = PT<BD>::PPD;
    if( ((uintptr_t)p & 3) == 0 )
    {
#pragma unroll
        for( int k = 0; k < N / PPD; k++ )
        {
            uint32_t w = 0;
#pragma unroll
            for( int j = 0; j < PPD; j++ )
                w |= (uint32_t)v[k * PPD + j] << (j * (32 / PPD));
            ((uint32_t *)p)[k] = w;
        }
    }
    else
    {
#pragma unroll
        for( int x = 0; x < N; x++ )
            p[x] = (typename PT<BD>::pixel)v[x];
    }
}

// residual of add4x4_idct: r[y][x] (dct.c:272-301, tmp and d stored as dctcoef)
template <int BD>
__device__ __forceinline__ void idct4_residual( const int (&c)[16], int (&r)[4][4] )
{
    int t[16];
#pragma unroll
    for( int i = 0; i < 4; i++ )
    {
        int s02 = c[0 * 4 + i] + c[2 * 4 + i], d02 = c[0 * 4 + i] - c[2 * 4 + i];
        int s13 = c[1 * 4 + i] + (c[3 * 4 + i] >> 1), d13 = (c[1 * 4 + i] >> 1) - c[3 * 4 + i];
        t[i * 4 + 0] = sto<BD>( s02 + s13 );
        t[i * 4 + 1] = sto<BD>( d02 + d13 );
        t[i * 4 + 2] = sto<BD>( d02 - d13 );
        t[i * 4 + 3] = sto<BD>( s02 - s13 );
    }
#pragma unroll
    for( int i = 0; i < 4; i++ )
    {
        int s02 = t[0 * 4 + i] + t[2 * 4 + i], d02 = t[0 * 4 + i] - t[2 * 4 + i];
        int s13 = t[1 * 4 + i] + (t[3 * 4 + i] >> 1), d13 = (t[1 * 4 + i] >> 1) - t[3 * 4 + i];
        r[0][i] = sto<BD>( (s02 + s13 + 32) >> 6 );
        r[1][i] = sto<BD>( (d02 + d13 + 32) >> 6 );
        r[2][i] = sto<BD>( (d02 - d13 + 32) >> 6 );
        r[3][i] = sto<BD>( (s02 - s13 + 32) >> 6 );
    }
}

// add a residual block to pred and store to dst (may alias pred)
template <int BD, int N>
__device__ __forceinline__ void add_block( const typename PT<BD>::pixel *pred, intptr_t ps, typename PT<BD>::pixel *dst,
                                           intptr_t ds, const int (&r)[N][N] )
{
#pragma unroll
    for( int y = 0; y < N; y++ )
    {
        int v[N];
        read_row<BD, N>( pred + y * ps, v );
#pragma unroll
        for( int x = 0; x < N; x++ )
            v[x] = clip_pix<BD>( v[x] + r[y][x] );
        write_row<BD, N>( dst + y * ds, v );
    }
}

// IDCT8_1D, dct.c:388-418
#define IDCT8_1D( SRC, DST )                                                                   \
    {                                                                                          \
        int a0 = SRC( 0 ) + SRC( 4 ), a2 = SRC( 0 ) - SRC( 4 );                                \
        int a4 = (SRC( 2 ) >> 1) - SRC( 6 ), a6 = (SRC( 6 ) >> 1) + SRC( 2 );                  \
        int b0 = a0 + a6, b2 = a2 + a4, b4 = a2 - a4, b6 = a0 - a6;                            \
        int a1 = -SRC( 3 ) + SRC( 5 ) - SRC( 7 ) - (SRC( 7 ) >> 1);                            \
        int a3 = SRC( 1 ) + SRC( 7 ) - SRC( 3 ) - (SRC( 3 ) >> 1);                             \
        int a5 = -SRC( 1 ) + SRC( 7 ) + SRC( 5 ) + (SRC( 5 ) >> 1);                            \
        int a7 = SRC( 3 ) + SRC( 5 ) + SRC( 1 ) + (SRC( 1 ) >> 1);                             \
        int b1 = (a7 >> 2) + a1, b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5, b7 = a7 - (a1 >> 2); \
        DST( 0, b0 + b7 ); DST( 1, b2 + b5 ); DST( 2, b4 + b3 ); DST( 3, b6 + b1 );            \
        DST( 4, b6 - b1 ); DST( 5, b4 - b3 ); DST( 6, b2 - b5 ); DST( 7, b0 - b7 );            \
    }

// residual of add8x8_idct8 (dct.c:420-440): c is modified as the reference does
// in place (dc rounding and the column pass stored as dctcoef); r[row][col]
template <int BD>
__device__ __forceinline__ void idct8_residual( int (&c)[64], int (&r)[8][8] )
{
    c[0] = sto<BD>( c[0] + 32 );
#pragma unroll
    for( int i = 0; i < 8; i++ )
    {
#define SRC( x ) c[(x) * 8 + i]
#define DST( x, v ) o[x] = sto<BD>( v )
        int o[8];
        IDCT8_1D( SRC, DST )
#pragma unroll
        for( int x = 0; x < 8; x++ )
            c[x * 8 + i] = o[x];
#undef SRC
#undef DST
    }
#pragma unroll
    for( int i = 0; i < 8; i++ )
    {
#define SRC( x ) c[i * 8 + (x)]
#define DST( x, v ) r[x][i] = (v) >> 6
        IDCT8_1D( SRC, DST )
#undef SRC
#undef DST
    }
}

template <int BD, int N>
__device__ __forceinline__ void load_coefs( const typename PT<BD>::dctcoef *p, int (&c)[N] )
{
    // 16-byte vector loads when aligned
    if constexpr( sizeof( typename PT<BD>::dctcoef ) == 2 && N % 8 == 0 )
    {
        if( ((uintptr_t)p & 15) == 0 )
        {
#pragma unroll
            for( int k = 0; k < N / 8; k++ )
            {
                uint4 w = ((const uint4 *)p)[k];
                uint32_t ww[4] = { w.x, w.y, w.z, w.w };
#pragma unroll
                for( int j = 0; j < 4; j++ )
                {
                    c[k * 8 + 2 * j] = (int)(int16_t)(ww[j] & 0xffff);
                    c[k * 8 + 2 * j + 1] = (int)(int16_t)(ww[j] >> 16);
                }
            }
            return;
        }
    }
    else if constexpr( sizeof( typename PT<BD>::dctcoef ) == 4 && N % 4 == 0 )
    {
        if( ((uintptr_t)p & 15) == 0 )
        {
#pragma unroll
            for( int k = 0; k < N / 4; k++ )
            {
                int4 w = ((const int4 *)p)[k];
                c[4 * k] = w.x; c[4 * k + 1] = w.y; c[4 * k + 2] = w.z; c[4 * k + 3] = w.w;
            }
            return;
        }
    }
#pragma unroll
    for( int k = 0; k < N; k++ )
        c[k] = p[k];
}

// ------------------------------------------------------------------ add_idct batch
// One lane per independent unit of a call: 4x4 sub-block (kinds 0-2), DC 4x4
// (3, 4) or 8x8 block (5, 6); units of one call never overlap.
template <int KIND> struct IdctKind;
template <> struct IdctKind<0> { static constexpr int U = 1, SIZE = 16; };
template <> struct IdctKind<1> { static constexpr int U = 4, SIZE = 64; };
template <> struct IdctKind<2> { static constexpr int U = 16, SIZE = 256; };
template <> struct IdctKind<3> { static constexpr int U = 4, SIZE = 4; };
template <> struct IdctKind<4> { static constexpr int U = 16, SIZE = 16; };
template <> struct IdctKind<5> { static constexpr int U = 1, SIZE = 64; };
template <> struct IdctKind<6> { static constexpr int U = 4, SIZE = 256; };

template <int BD, int KIND>
__global__ __launch_bounds__( 256 ) void add_idct_batch_kernel( typename PT<BD>::pixel *dst, intptr_t ds,
                                                                const int64_t *dst_off,
                                                                const typename PT<BD>::dctcoef *dct, int n )
{
    using K = IdctKind<KIND>;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if( t >= (int64_t)n * K::U )
        return;
    const int64_t call = t / K::U;
    const int u = (int)(t % K::U);
    const typename PT<BD>::dctcoef *c = dct + call * K::SIZE;
    typename PT<BD>::pixel *p = dst + dst_off[call];
    if constexpr( KIND <= 2 )
    {
        int x, y;
        if constexpr( KIND == 2 )
        {
            const int q = u >> 2, k = u & 3;
            x = (q & 1) * 8 + (k & 1) * 4;
            y = (q >> 1) * 8 + (k >> 1) * 4;
        }
        else
        {
            x = (u & 1) * 4;
            y = (u >> 1) * 4;
        }
        int cc[16], r[4][4];
        load_coefs<BD, 16>( c + u * 16, cc );
        idct4_residual<BD>( cc, r );
        add_block<BD, 4>( p + y * ds + x, ds, p + y * ds + x, ds, r );
    }
    else if constexpr( KIND <= 4 )
    {
        const int x = KIND == 3 ? (u & 1) * 4 : (u & 3) * 4;
        const int y = KIND == 3 ? (u >> 1) * 4 : (u >> 2) * 4;
        const int dc = sto<BD>( ((int)c[u] + 32) >> 6 );
        int r[4][4];
#pragma unroll
        for( int i = 0; i < 4; i++ )
#pragma unroll
            for( int j = 0; j < 4; j++ )
                r[i][j] = dc;
        add_block<BD, 4>( p + y * ds + x, ds, p + y * ds + x, ds, r );
    }
    else
    {
        const int x = KIND == 6 ? (u & 1) * 8 : 0, y = KIND == 6 ? (u >> 1) * 8 : 0;
        int cc[64], r[8][8];
        load_coefs<BD, 64>( c + u * 64, cc );
        idct8_residual<BD>( cc, r );
        add_block<BD, 8>( p + y * ds + x, ds, p + y * ds + x, ds, r );
    }
}

template <int BD>
hipError_t launch_add_idct( int kind, typename PT<BD>::pixel *dst, intptr_t ds, const int64_t *dst_off,
                            const typename PT<BD>::dctcoef *dct, int n, hipStream_t st )
{
    if( n <= 0 )
        return hipSuccess;
    static const int units[7] = { 1, 4, 16, 4, 16, 1, 4 };
    if( kind < 0 || kind > 6 )
        return hipErrorInvalidValue;
    const int64_t total = (int64_t)n * units[kind];
    dim3 blk( 256 ), g( (unsigned)((total + 255) / 256) );
#define K( I ) case I: hipLaunchKernelGGL( ( add_idct_batch_kernel<BD, I> ), g, blk, 0, st, dst, ds, dst_off, dct, n ); break;
    switch( kind ) { K( 0 ) K( 1 ) K( 2 ) K( 3 ) K( 4 ) K( 5 ) K( 6 ) }
#undef K
    return hipGetLastError();
}

// ------------------------------------------------------------------ dequant batch
// one lane per coefficient; per-block qp (quant.c:106-162)
template <int BD, int KIND>
__global__ __launch_bounds__( 256 ) void dequant_batch_kernel( typename PT<BD>::dctcoef *dct, const int32_t *dmf,
                                                               const int32_t *qp, int n )
{
    constexpr int SIZE = KIND == 1 ? 64 : 16;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if( t >= (int64_t)n * SIZE )
        return;
    const int64_t b = t / SIZE;
    const int j = (int)(t % SIZE);
    const int q = qp[b];
    const int v = dct[t];
    int r;
    if constexpr( KIND == 2 )     // dequant_4x4_dc
    {
        const int qb = q / 6 - 6;
        if( qb >= 0 )
            r = v * (dmf[(q % 6) * 16] << qb);
        else
            r = (v * dmf[(q % 6) * 16] + (1 << (-qb - 1))) >> (-qb);
    }
    else
    {
        const int qb = q / 6 - (KIND == 1 ? 6 : 4);
        const int m = dmf[(q % 6) * SIZE + j];
        if( qb >= 0 )
            r = (v * m) * (1 << qb);
        else
            r = (v * m + (1 << (-qb - 1))) >> (-qb);
    }
    dct[t] = (typename PT<BD>::dctcoef)r;
}

template <int BD>
hipError_t launch_dequant( int kind, typename PT<BD>::dctcoef *dct, const int32_t *dmf, const int32_t *qp, int n,
                           hipStream_t st )
{
    if( n <= 0 )
        return hipSuccess;
    const int64_t total = (int64_t)n * (kind == 1 ? 64 : 16);
    dim3 blk( 256 ), g( (unsigned)((total + 255) / 256) );
    switch( kind )
    {
        case 0: hipLaunchKernelGGL( ( dequant_batch_kernel<BD, 0> ), g, blk, 0, st, dct, dmf, qp, n ); break;
        case 1: hipLaunchKernelGGL( ( dequant_batch_kernel<BD, 1> ), g, blk, 0, st, dct, dmf, qp, n ); break;
        case 2: hipLaunchKernelGGL( ( dequant_batch_kernel<BD, 2> ), g, blk, 0, st, dct, dmf, qp, n ); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------ DC transforms
// idct4x4dc (dct.c:78-107), in place, one lane per block
template <int BD>
__global__ __launch_bounds__( 256 ) void idct4x4dc_kernel( typename PT<BD>::dctcoef *dct, int n )
{
    const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
    if( i0 >= n )
        return;
    typename PT<BD>::dctcoef *d = dct + (int64_t)i0 * 16;
    int c[16], t[16];
    load_coefs<BD, 16>( d, c );
#pragma unroll
    for( int i = 0; i < 4; i++ )
    {
        int s01 = c[i * 4 + 0] + c[i * 4 + 1], d01 = c[i * 4 + 0] - c[i * 4 + 1];
        int s23 = c[i * 4 + 2] + c[i * 4 + 3], d23 = c[i * 4 + 2] - c[i * 4 + 3];
        t[0 * 4 + i] = sto<BD>( s01 + s23 );
        t[1 * 4 + i] = sto<BD>( s01 - s23 );
        t[2 * 4 + i] = sto<BD>( d01 - d23 );
        t[3 * 4 + i] = sto<BD>( d01 + d23 );
    }
#pragma unroll
    for( int i = 0; i < 4; i++ )
    {
        int s01 = t[i * 4 + 0] + t[i * 4 + 1], d01 = t[i * 4 + 0] - t[i * 4 + 1];
        int s23 = t[i * 4 + 2] + t[i * 4 + 3], d23 = t[i * 4 + 2] - t[i * 4 + 3];
        d[i * 4 + 0] = (typename PT<BD>::dctcoef)(s01 + s23);
        d[i * 4 + 1] = (typename PT<BD>::dctcoef)(s01 - s23);
        d[i * 4 + 2] = (typename PT<BD>::dctcoef)(d01 - d23);
        d[i * 4 + 3] = (typename PT<BD>::dctcoef)(d01 + d23);
    }
}

template <int BD>
hipError_t launch_idct4x4dc( typename PT<BD>::dctcoef *dct, int n, hipStream_t st )
{
    if( n <= 0 )
        return hipSuccess;
    hipLaunchKernelGGL( idct4x4dc_kernel<BD>, dim3( (n + 255) / 256 ), dim3( 256 ), 0, st, dct, n );
    return hipGetLastError();
}

// idct_dequant_2x4_dc / _dconly (quant.c:164-208), one lane per call, per-call qp
template <int BD, bool DCONLY>
__global__ __launch_bounds__( 256 ) void idct_dequant_2x4_kernel( typename PT<BD>::dctcoef *dct,
                                                                  typename PT<BD>::dctcoef *dct4x4,
                                                                  const int32_t *dmf, const int32_t *qp, int n )
{
    const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
    if( i0 >= n )
        return;
    typename PT<BD>::dctcoef *d = dct + (int64_t)i0 * 8;
    int c[8];
#pragma unroll
    for( int k = 0; k < 8; k++ )
        c[k] = d[k];
    int a0 = c[0] + c[1], a1 = c[2] + c[3], a2 = c[4] + c[5], a3 = c[6] + c[7];
    int a4 = c[0] - c[1], a5 = c[2] - c[3], a6 = c[4] - c[5], a7 = c[6] - c[7];
    int b0 = a0 + a1, b1 = a2 + a3, b2 = a4 + a5, b3 = a6 + a7;
    int b4 = a0 - a1, b5 = a2 - a3, b6 = a4 - a5, b7 = a6 - a7;
    const int q = qp[i0];
    const int m = dmf[(q % 6) * 16] << (q / 6);
    int o[8] = { b0 + b1, b2 + b3, b0 - b1, b2 - b3, b4 - b5, b6 - b7, b4 + b5, b6 + b7 };
#pragma unroll
    for( int k = 0; k < 8; k++ )
    {
        const typename PT<BD>::dctcoef v = (typename PT<BD>::dctcoef)((o[k] * m + 32) >> 6);
        if( DCONLY )
            d[k] = v;
        else
            dct4x4[(int64_t)i0 * 128 + k * 16] = v;
    }
}

template <int BD>
hipError_t launch_idct_dequant_2x4( int dconly, typename PT<BD>::dctcoef *dct, typename PT<BD>::dctcoef *dct4x4,
                                    const int32_t *dmf, const int32_t *qp, int n, hipStream_t st )
{
    if( n <= 0 )
        return hipSuccess;
    dim3 blk( 256 ), g( (n + 255) / 256 );
    if( dconly )
        hipLaunchKernelGGL( ( idct_dequant_2x4_kernel<BD, true> ), g, blk, 0, st, dct, dct4x4, dmf, qp, n );
    else
        hipLaunchKernelGGL( ( idct_dequant_2x4_kernel<BD, false> ), g, blk, 0, st, dct, dct4x4, dmf, qp, n );
    return hipGetLastError();
}

// optimize_chroma_2x2_dc / 2x4_dc (quant.c:210-293): the reference's greedy
// search, one lane per call; per-call dequant factor
template <int NC>
__device__ __forceinline__ void oc_idq( const int (&d)[NC], int dmf, int (&out)[NC] )
{
    if constexpr( NC == 8 )
    {
        int a0 = d[0] + d[1], a1 = d[2] + d[3], a2 = d[4] + d[5], a3 = d[6] + d[7];
        int a4 = d[0] - d[1], a5 = d[2] - d[3], a6 = d[4] - d[5], a7 = d[6] - d[7];
        int b0 = a0 + a1, b1 = a2 + a3, b2 = a4 + a5, b3 = a6 + a7;
        int b4 = a0 - a1, b5 = a2 - a3, b6 = a4 - a5, b7 = a6 - a7;
        const int v[8] = { b0 + b1, b2 + b3, b0 - b1, b2 - b3, b4 - b5, b6 - b7, b4 + b5, b6 + b7 };
#pragma unroll
        for( int k = 0; k < 8; k++ )
            out[k] = (v[k] * dmf + 2080) >> 6;
    }
    else
    {
        int d0 = d[0] + d[1], d1 = d[2] + d[3], d2 = d[0] - d[1], d3 = d[2] - d[3];
        out[0] = ((d0 + d1) * dmf >> 5) + 32;
        out[1] = ((d0 - d1) * dmf >> 5) + 32;
        out[2] = ((d2 + d3) * dmf >> 5) + 32;
        out[3] = ((d2 - d3) * dmf >> 5) + 32;
    }
}

template <int BD, int NC>
__global__ __launch_bounds__( 256 ) void optimize_chroma_kernel( typename PT<BD>::dctcoef *dct, const int32_t *dmfs,
                                                                 int n, int32_t *nzo )
{
    const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
    if( i0 >= n )
        return;
    typename PT<BD>::dctcoef *p = dct + (int64_t)i0 * NC;
    const int dmf = dmfs[i0];
    int d[NC], orig[NC], out[NC];
#pragma unroll
    for( int k = 0; k < NC; k++ )
        d[k] = p[k];
    oc_idq<NC>( d, dmf, orig );
    int sum = 0;
#pragma unroll
    for( int k = 0; k < NC; k++ )
        sum |= sto<BD>( orig[k] );
    int nz = 0;
    if( sum >> 6 )
    {
#pragma unroll
        for( int k = 0; k < NC; k++ )
            orig[k] = sto<BD>( orig[k] );
#pragma unroll
        for( int coeff = NC - 1; coeff >= 0; coeff-- )
        {
            int level = d[coeff];
            const int sign = (level >> 31) | 1;
            while( level )
            {
                d[coeff] = sto<BD>( level - sign );
                oc_idq<NC>( d, dmf, out );
                int diff = 0;
#pragma unroll
                for( int k = 0; k < NC; k++ )
                    diff |= orig[k] ^ sto<BD>( out[k] );
                if( diff >> 6 )
                {
                    nz = 1;
                    d[coeff] = level;
                    break;
                }
                level -= sign;
            }
        }
#pragma unroll
        for( int k = 0; k < NC; k++ )
            p[k] = (typename PT<BD>::dctcoef)d[k];
    }
    nzo[i0] = nz;
}

template <int BD>
hipError_t launch_optimize_chroma( int c422, typename PT<BD>::dctcoef *dct, const int32_t *dmf, int n, int32_t *nz,
                                   hipStream_t st )
{
    if( n <= 0 )
        return hipSuccess;
    dim3 blk( 256 ), g( (n + 255) / 256 );
    if( c422 )
        hipLaunchKernelGGL( ( optimize_chroma_kernel<BD, 8> ), g, blk, 0, st, dct, dmf, n, nz );
    else
        hipLaunchKernelGGL( ( optimize_chroma_kernel<BD, 4> ), g, blk, 0, st, dct, dmf, n, nz );
    return hipGetLastError();
}

// denoise_dct (quant.c:295-306): one lane per coefficient; the running sums are
// integer atomics, so their result is independent of lane order
template <int BD>
__global__ __launch_bounds__( 256 ) void denoise_kernel( typename PT<BD>::dctcoef *dct, int size, int64_t total,
                                                         uint32_t *sum, const typename PT<BD>::udctcoef *offset )
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if( t >= total )
        return;
    const int j = (int)(t % size);
    int level = dct[t];
    const int sign = level >> 31;
    level = (level + sign) ^ sign;
    atomicAdd( &sum[j], (uint32_t)level );
    level -= (int)offset[j];
    dct[t] = (typename PT<BD>::dctcoef)(level < 0 ? 0 : (level ^ sign) - sign);
}

template <int BD>
hipError_t launch_denoise( typename PT<BD>::dctcoef *dct, int size, int n, uint32_t *sum,
                           const typename PT<BD>::udctcoef *offset, hipStream_t st )
{
    if( n <= 0 || size <= 0 )
        return hipSuccess;
    const int64_t total = (int64_t)n * size;
    hipLaunchKernelGGL( denoise_kernel<BD>, dim3( (unsigned)((total + 255) / 256) ), dim3( 256 ), 0, st, dct, size,
                        total, sum, offset );
    return hipGetLastError();
}

// ------------------------------------------------------------------ coefficient statistics
__constant__ uint8_t c_decimate4[16] = { 3, 2, 2, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0 };
__constant__ uint8_t c_decimate8[64] = { 3, 3, 3, 3, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                         1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                         0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0 };

// kind: 0 decimate15 (reads dct+1), 1 decimate16, 2 decimate64,
//       3 last4, 4 last8, 5 last15, 6 last16, 7 last64
template <int BD, int KIND>
__global__ __launch_bounds__( 256 ) void coef_stat_kernel( const typename PT<BD>::dctcoef *dct, int64_t pitch, int n,
                                                           int32_t *out )
{
    const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
    if( i0 >= n )
        return;
    const typename PT<BD>::dctcoef *d = dct + i0 * pitch;
    constexpr int NUM = KIND == 0 ? 15 : KIND == 1 ? 16 : KIND == 2 ? 64 : KIND == 3 ? 4 : KIND == 4 ? 8
                      : KIND == 5 ? 15 : KIND == 6 ? 16 : 64;
    if constexpr( KIND == 0 )
        d += 1;
    int idx = NUM - 1;
    while( idx >= 0 && d[idx] == 0 )
        idx--;
    if constexpr( KIND >= 3 )
    {
        out[i0] = idx;
    }
    else
    {
        const uint8_t *tab = NUM == 64 ? c_decimate8 : c_decimate4;
        int score = 0;
        while( idx >= 0 )
        {
            if( (unsigned)((int)d[idx--] + 1) > 2 )
            {
                score = 9;
                break;
            }
            int run = 0;
            while( idx >= 0 && d[idx] == 0 )
            {
                idx--;
                run++;
            }
            score += tab[run];
        }
        out[i0] = score;
    }
}

template <int BD>
hipError_t launch_coef_stat( int kind, const typename PT<BD>::dctcoef *dct, int64_t pitch, int n, int32_t *out,
                             hipStream_t st )
{
    if( n <= 0 )
        return hipSuccess;
    dim3 blk( 256 ), g( (n + 255) / 256 );
#define K( I ) case I: hipLaunchKernelGGL( ( coef_stat_kernel<BD, I> ), g, blk, 0, st, dct, pitch, n, out ); break;
    switch( kind )
    {
        K( 0 ) K( 1 ) K( 2 ) K( 3 ) K( 4 ) K( 5 ) K( 6 ) K( 7 )
        default: return hipErrorInvalidValue;
    }
#undef K
    return hipGetLastError();
}

// coeff_level_run4/8/15/16 (quant.c:380-398): out per call = last, mask, count,
// levels[18]
template <int BD>
__global__ __launch_bounds__( 256 ) void level_run_kernel( int num, const typename PT<BD>::dctcoef *dct, int64_t pitch,
                                                           int n, int32_t *last, int32_t *mask, int32_t *count,
                                                           typename PT<BD>::dctcoef *level )
{
    const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
    if( i0 >= n )
        return;
    const typename PT<BD>::dctcoef *d = dct + i0 * pitch;
    typename PT<BD>::dctcoef *lv = level + (int64_t)i0 * 18;
    int i_last = num - 1;
    while( i_last >= 0 && d[i_last] == 0 )
        i_last--;
    last[i0] = i_last;
    int total = 0, m = 0;
    do
    {
        lv[total++] = d[i_last];
        m |= 1 << i_last;
        while( --i_last >= 0 && d[i_last] == 0 )
            ;
    } while( i_last >= 0 );
    mask[i0] = m;
    count[i0] = total;
}

template <int BD>
hipError_t launch_level_run( int num, const typename PT<BD>::dctcoef *dct, int64_t pitch, int n, int32_t *last,
                             int32_t *mask, int32_t *count, typename PT<BD>::dctcoef *level, hipStream_t st )
{
    if( n <= 0 )
        return hipSuccess;
    if( num != 4 && num != 8 && num != 15 && num != 16 )
        return hipErrorInvalidValue;
    hipLaunchKernelGGL( level_run_kernel<BD>, dim3( (n + 255) / 256 ), dim3( 256 ), 0, st, num, dct, pitch, n, last,
                        mask, count, level );
    return hipGetLastError();
}

// ------------------------------------------------------------------ zigzag
// (y, x) per scan index, dct.c:768-816; level[i] = dct[x*W + y] for scans,
// src/dst pixel (x, y) for zigzag_sub
__constant__ uint8_t c_zz8[2][64][2] = {
    { {0,0},{0,1},{1,0},{2,0},{1,1},{0,2},{0,3},{1,2},{2,1},{3,0},{4,0},{3,1},{2,2},{1,3},{0,4},{0,5},
      {1,4},{2,3},{3,2},{4,1},{5,0},{6,0},{5,1},{4,2},{3,3},{2,4},{1,5},{0,6},{0,7},{1,6},{2,5},{3,4},
      {4,3},{5,2},{6,1},{7,0},{7,1},{6,2},{5,3},{4,4},{3,5},{2,6},{1,7},{2,7},{3,6},{4,5},{5,4},{6,3},
      {7,2},{7,3},{6,4},{5,5},{4,6},{3,7},{4,7},{5,6},{6,5},{7,4},{7,5},{6,6},{5,7},{6,7},{7,6},{7,7} },
    { {0,0},{1,0},{2,0},{0,1},{1,1},{3,0},{4,0},{2,1},{0,2},{3,1},{5,0},{6,0},{7,0},{4,1},{1,2},{0,3},
      {2,2},{5,1},{6,1},{7,1},{3,2},{1,3},{0,4},{2,3},{4,2},{5,2},{6,2},{7,2},{3,3},{1,4},{0,5},{2,4},
      {4,3},{5,3},{6,3},{7,3},{3,4},{1,5},{0,6},{2,5},{4,4},{5,4},{6,4},{7,4},{3,5},{1,6},{2,6},{4,5},
      {5,5},{6,5},{7,5},{3,6},{0,7},{1,7},{4,6},{5,6},{6,6},{7,6},{2,7},{3,7},{4,7},{5,7},{6,7},{7,7} } };
__constant__ uint8_t c_zz4[2][16][2] = {
    { {0,0},{0,1},{1,0},{2,0},{1,1},{0,2},{0,3},{1,2},{2,1},{3,0},{3,1},{2,2},{1,3},{2,3},{3,2},{3,3} },
    { {0,0},{1,0},{0,1},{2,0},{3,0},{1,1},{2,1},{3,1},{0,2},{1,2},{2,2},{3,2},{0,3},{1,3},{2,3},{3,3} } };

template <int BD, int W>
__global__ __launch_bounds__( 256 ) void zigzag_scan_kernel( int field, typename PT<BD>::dctcoef *level,
                                                             const typename PT<BD>::dctcoef *dct, int n )
{
    // one lane per coefficient
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if( t >= (int64_t)n * W * W )
        return;
    const int64_t b = t / (W * W);
    const int i = (int)(t % (W * W));
    const uint8_t *yx = W == 8 ? c_zz8[field][i] : c_zz4[field][i];
    level[t] = dct[b * W * W + yx[1] * W + yx[0]];
}

template <int BD>
hipError_t launch_zigzag_scan( int size, int field, typename PT<BD>::dctcoef *level,
                               const typename PT<BD>::dctcoef *dct, int n, hipStream_t st )
{
    if( n <= 0 )
        return hipSuccess;
    const int64_t total = (int64_t)n * size * size;
    dim3 blk( 256 ), g( (unsigned)((total + 255) / 256) );
    if( size == 8 )
        hipLaunchKernelGGL( ( zigzag_scan_kernel<BD, 8> ), g, blk, 0, st, field, level, dct, n );
    else if( size == 4 )
        hipLaunchKernelGGL( ( zigzag_scan_kernel<BD, 4> ), g, blk, 0, st, field, level, dct, n );
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// compile-time copies of the scan tables so fully unrolled loops index registers
template <int W, int FIELD> struct ZZ;
template <int FIELD> struct ZZ<8, FIELD>
{
    static constexpr uint8_t yx[2][64][2] = {
        { {0,0},{0,1},{1,0},{2,0},{1,1},{0,2},{0,3},{1,2},{2,1},{3,0},{4,0},{3,1},{2,2},{1,3},{0,4},{0,5},
          {1,4},{2,3},{3,2},{4,1},{5,0},{6,0},{5,1},{4,2},{3,3},{2,4},{1,5},{0,6},{0,7},{1,6},{2,5},{3,4},
          {4,3},{5,2},{6,1},{7,0},{7,1},{6,2},{5,3},{4,4},{3,5},{2,6},{1,7},{2,7},{3,6},{4,5},{5,4},{6,3},
          {7,2},{7,3},{6,4},{5,5},{4,6},{3,7},{4,7},{5,6},{6,5},{7,4},{7,5},{6,6},{5,7},{6,7},{7,6},{7,7} },
        { {0,0},{1,0},{2,0},{0,1},{1,1},{3,0},{4,0},{2,1},{0,2},{3,1},{5,0},{6,0},{7,0},{4,1},{1,2},{0,3},
          {2,2},{5,1},{6,1},{7,1},{3,2},{1,3},{0,4},{2,3},{4,2},{5,2},{6,2},{7,2},{3,3},{1,4},{0,5},{2,4},
          {4,3},{5,3},{6,3},{7,3},{3,4},{1,5},{0,6},{2,5},{4,4},{5,4},{6,4},{7,4},{3,5},{1,6},{2,6},{4,5},
          {5,5},{6,5},{7,5},{3,6},{0,7},{1,7},{4,6},{5,6},{6,6},{7,6},{2,7},{3,7},{4,7},{5,7},{6,7},{7,7} } };
    static constexpr int y( int i ) { return yx[FIELD][i][0]; }
    static constexpr int x( int i ) { return yx[FIELD][i][1]; }
};
template <int FIELD> struct ZZ<4, FIELD>
{
    static constexpr uint8_t yx[2][16][2] = {
        { {0,0},{0,1},{1,0},{2,0},{1,1},{0,2},{0,3},{1,2},{2,1},{3,0},{3,1},{2,2},{1,3},{2,3},{3,2},{3,3} },
        { {0,0},{1,0},{0,1},{2,0},{3,0},{1,1},{2,1},{3,1},{0,2},{1,2},{2,2},{3,2},{0,3},{1,3},{2,3},{3,3} } };
    static constexpr int y( int i ) { return yx[FIELD][i][0]; }
    static constexpr int x( int i ) { return yx[FIELD][i][1]; }
};

// zigzag_sub_4x4 / 4x4ac / 8x8 (dct.c:856-925), one lane per call
template <int BD, int KIND, int FIELD>
__global__ __launch_bounds__( 256 ) void zigzag_sub_kernel( typename PT<BD>::dctcoef *level,
                                                            typename PT<BD>::dctcoef *dc,
                                                            const typename PT<BD>::pixel *src, intptr_t ss,
                                                            typename PT<BD>::pixel *dst, intptr_t ds,
                                                            const int64_t *so, const int64_t *dso, int n, int32_t *nzo )
{
    constexpr int W = KIND == 2 ? 8 : 4;
    using Z = ZZ<W, FIELD>;
    const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
    if( i0 >= n )
        return;
    const typename PT<BD>::pixel *s = src + so[i0];
    typename PT<BD>::pixel *d = dst + dso[i0];
    int a[W][W], b[W][W];
#pragma unroll
    for( int y = 0; y < W; y++ )
    {
        read_row<BD, W>( s + y * ss, a[y] );
        read_row<BD, W>( d + y * ds, b[y] );
    }
    typename PT<BD>::dctcoef *lv = level + (int64_t)i0 * W * W;
    int nz = 0;
#pragma unroll
    for( int i = 0; i < W * W; i++ )
    {
        const int v = a[Z::y( i )][Z::x( i )] - b[Z::y( i )][Z::x( i )];
        if( KIND == 1 && i == 0 )
        {
            dc[i0] = (typename PT<BD>::dctcoef)v;
            lv[0] = 0;
            continue;
        }
        lv[i] = (typename PT<BD>::dctcoef)v;
        nz |= sto<BD>( v );
    }
#pragma unroll
    for( int y = 0; y < W; y++ )
        write_row<BD, W>( d + y * ds, a[y] );
    nzo[i0] = nz != 0;
}

template <int BD>
hipError_t launch_zigzag_sub( int kind, int field, typename PT<BD>::dctcoef *level, typename PT<BD>::dctcoef *dc,
                              const typename PT<BD>::pixel *src, intptr_t ss, typename PT<BD>::pixel *dst,
                              intptr_t ds, const int64_t *so, const int64_t *dso, int n, int32_t *nz, hipStream_t st )
{
    if( n <= 0 )
        return hipSuccess;
    dim3 blk( 256 ), g( (n + 255) / 256 );
#define K( I, F ) \
    case I * 2 + F: hipLaunchKernelGGL( ( zigzag_sub_kernel<BD, I, F> ), g, blk, 0, st, level, dc, src, ss, dst, ds, so, dso, n, nz ); break;
    switch( kind * 2 + (field ? 1 : 0) )
    {
        K( 0, 0 ) K( 0, 1 ) K( 1, 0 ) K( 1, 1 ) K( 2, 0 ) K( 2, 1 )
        default: return hipErrorInvalidValue;
    }
#undef K
    return hipGetLastError();
}

// zigzag_interleave_8x8_cavlc (dct.c:927-940), one lane per call
template <int BD>
__global__ __launch_bounds__( 256 ) void interleave_kernel( typename PT<BD>::dctcoef *dst,
                                                            const typename PT<BD>::dctcoef *src, uint8_t *nnz, int n )
{
    const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
    if( i0 >= n )
        return;
    const typename PT<BD>::dctcoef *s = src + (int64_t)i0 * 64;
    typename PT<BD>::dctcoef *d = dst + (int64_t)i0 * 64;
    uint8_t *nn = nnz + (int64_t)i0 * 16;
#pragma unroll
    for( int i = 0; i < 4; i++ )
    {
        int nz = 0;
#pragma unroll
        for( int j = 0; j < 16; j++ )
        {
            nz |= s[i + j * 4];
            d[i * 16 + j] = s[i + j * 4];
        }
        nn[(i & 1) + (i >> 1) * 8] = nz != 0;
    }
}

template <int BD>
hipError_t launch_interleave( typename PT<BD>::dctcoef *dst, const typename PT<BD>::dctcoef *src, uint8_t *nnz, int n,
                              hipStream_t st )
{
    if( n <= 0 )
        return hipSuccess;
    hipLaunchKernelGGL( interleave_kernel<BD>, dim3( (n + 255) / 256 ), dim3( 256 ), 0, st, dst, src, nnz, n );
    return hipGetLastError();
}

// ------------------------------------------------------------------ fused reconstruction
// recon = clip( pred + idct( dequant( dct ) ) ) per macroblock for the inter
// luma residual (x264_mb_encode_* order: dequant_4x4 / dequant_8x8 then
// add16x16_idct / add16x16_idct8, encoder/macroblock.c), dct[mb][256] as
// written by mb_dct_quant (not modified), per-MB qp.  One lane per 4x4 (T=4)
// or 8x8 (T=8) block; lanes of a wave cover consecutive blocks of a block row
// so pixel rows are written contiguously.
template <int BD, int T>
__global__ __launch_bounds__( 256 ) void mb_recon_kernel( const typename PT<BD>::dctcoef *dct, int mbw, int mbh,
                                                          int nframes, const int32_t *dmf, const int32_t *qp,
                                                          const typename PT<BD>::pixel *pred, intptr_t ps,
                                                          intptr_t pfs, typename PT<BD>::pixel *recon, intptr_t rs,
                                                          intptr_t rfs )
{
    constexpr int BPR = 16 / T;                          // blocks per MB row
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int bw = mbw * BPR, bh = mbh * BPR;            // blocks per frame row / column
    if( t >= (int64_t)nframes * bw * bh )
        return;
    const int bx = (int)(t % bw);
    const int64_t r = t / bw;
    const int by = (int)(r % bh);
    const int f = (int)(r / bh);
    const int mbx = bx / BPR, mby = by / BPR;
    const int64_t mb = ((int64_t)f * mbh + mby) * mbw + mbx;
    const int lx = bx % BPR, ly = by % BPR;
    const int q = qp[mb];
    const typename PT<BD>::pixel *pp = pred + f * pfs + (intptr_t)(by * T) * ps + bx * T;
    typename PT<BD>::pixel *rp = recon + f * rfs + (intptr_t)(by * T) * rs + bx * T;
    if constexpr( T == 4 )
    {
        // block index inside the MB in the reference's dct4x4[16] quadrant order
        const int blk = ((ly >> 1) * 2 + (lx >> 1)) * 4 + (ly & 1) * 2 + (lx & 1);
        int c[16], res[4][4];
        load_coefs<BD, 16>( dct + mb * 256 + blk * 16, c );
        const int qb = q / 6 - 4;
        const int32_t *m = dmf + (q % 6) * 16;
#pragma unroll
        for( int j = 0; j < 16; j++ )
            c[j] = sto<BD>( qb >= 0 ? (c[j] * m[j]) * (1 << qb) : (c[j] * m[j] + (1 << (-qb - 1))) >> (-qb) );
        idct4_residual<BD>( c, res );
        add_block<BD, 4>( pp, ps, rp, rs, res );
    }
    else
    {
        const int blk = ly * 2 + lx;
        int c[64], res[8][8];
        load_coefs<BD, 64>( dct + mb * 256 + blk * 64, c );
        const int qb = q / 6 - 6;
        const int32_t *m = dmf + (q % 6) * 64;
#pragma unroll
        for( int j = 0; j < 64; j++ )
            c[j] = sto<BD>( qb >= 0 ? (c[j] * m[j]) * (1 << qb) : (c[j] * m[j] + (1 << (-qb - 1))) >> (-qb) );
        idct8_residual<BD>( c, res );
        add_block<BD, 8>( pp, ps, rp, rs, res );
    }
}

// transform 4, 8-pixel variant: one lane per pair of horizontally adjacent
// 4x4 blocks (their 32 coefficients are contiguous in the dct4x4 order), so
// pixel rows move as 8-pixel pieces and a wave covers 8 MBs of one MB row
// `sh` (0..3) shifts the 8-MB strips left by sh MBs so each strip's 128-byte rows start on a
// 64-byte sector of the output plane (the plane origin sits 32 bytes into a sector when the
// padding is 32 pixels): every store then writes whole sectors, and no sector is shared by
// two waves (see launch_mb_recon)
template <int BD>
__global__ __launch_bounds__( 256 ) void mb_recon_pair_kernel( const typename PT<BD>::dctcoef *dct, int mbw, int mbh,
                                                               int nframes, const int32_t *dmf, const int32_t *qp,
                                                               const typename PT<BD>::pixel *pred, intptr_t ps,
                                                               intptr_t pfs, typename PT<BD>::pixel *recon,
                                                               intptr_t rs, intptr_t rfs, int sh )
{
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int spr = (mbw + sh + 7) >> 3;
    if( wave >= (int64_t)nframes * mbh * spr )
        return;
    const int strip = (int)(wave % spr);
    const int64_t t = wave / spr;
    const int mby = (int)(t % mbh);
    const int f = (int)(t / mbh);
    const int m = (lane & 15) >> 1, half = lane & 1, by = lane >> 4;
    const int mbx = strip * 8 + m - sh;
    if( mbx < 0 || mbx >= mbw )
        return;
    const int64_t mb = ((int64_t)f * mbh + mby) * mbw + mbx;
    const int q = qp[mb];
    const int qb = q / 6 - 4;
    const int32_t *mq = dmf + (q % 6) * 16;
    const int i8 = (by >> 1) * 2 + half, i4 = (by & 1) * 2;
    int c[32];
    load_coefs<BD, 32>( dct + mb * 256 + (i8 * 4 + i4) * 16, c );
    int res[4][8];
#pragma unroll
    for( int k = 0; k < 2; k++ )
    {
        int cc[16], r[4][4];
#pragma unroll
        for( int j = 0; j < 16; j++ )
        {
            const int v = c[k * 16 + j], mm = mq[j];
            cc[j] = sto<BD>( qb >= 0 ? (v * mm) * (1 << qb) : (v * mm + (1 << (-qb - 1))) >> (-qb) );
        }
        idct4_residual<BD>( cc, r );
#pragma unroll
        for( int y = 0; y < 4; y++ )
#pragma unroll
            for( int x = 0; x < 4; x++ )
                res[y][4 * k + x] = r[y][x];
    }
    const intptr_t px = 16 * mbx + 8 * half;
    const typename PT<BD>::pixel *pp = pred + (intptr_t)f * pfs + (intptr_t)(16 * mby + 4 * by) * ps + px;
    typename PT<BD>::pixel *rp = recon + (intptr_t)f * rfs + (intptr_t)(16 * mby + 4 * by) * rs + px;
#pragma unroll
    for( int y = 0; y < 4; y++ )
    {
        int v[8];
        read_row<BD, 8>( pp + y * ps, v );
#pragma unroll
        for( int x = 0; x < 8; x++ )
            v[x] = clip_pix<BD>( v[x] + res[y][x] );
        write_row<BD, 8>( rp + y * rs, v );
    }
}

// 8 bit, transform 8 (the default there): the coefficients stay packed as the
// int16 pairs they are stored as -- (c[x*8+2k], c[x*8+2k+1]) in one dword --
// and only the eight values one IDCT8_1D consumes are widened to int32, so a
// lane holds a block in 32 registers instead of 64 and the int16 stores of
// add8x8_idct8 (dct.c:420-440) become the v_perm that packs each result pair.
// The column pass works on column pairs straight from that layout; the row
// pass reads row i's pairs and yields residual columns i, which are packed
// per pixel row and added to the prediction in 16-bit pairs (clip by
// v_pk_max / v_pk_min).  dequant_8x8 (quant.c:106-146) multiplies in 24 bits
// when every dequant_mf entry fits (checked per workgroup while the table is
// staged in LDS; the 24-bit product keeps the low 32 bits the int32 product
// wraps to), else with the full 32-bit multiply.
typedef short rc_s2 __attribute__( ( ext_vector_type( 2 ) ) );

__device__ __forceinline__ rc_s2 rc_as2( uint32_t v ) { return __builtin_bit_cast( rc_s2, v ); }
__device__ __forceinline__ uint32_t rc_asu( rc_s2 v ) { return __builtin_bit_cast( uint32_t, v ); }
__device__ __forceinline__ uint32_t rc_pack( int lo, int hi )
{
    return __builtin_amdgcn_perm( (uint32_t)hi, (uint32_t)lo, 0x05040100u );
}

#define IDCT8_1D_PK( SRC, DST )                                                                \
    {                                                                                          \
        const rc_s2 a0 = SRC( 0 ) + SRC( 4 ), a2 = SRC( 0 ) - SRC( 4 );                        \
        const rc_s2 a4 = (SRC( 2 ) >> 1) - SRC( 6 ), a6 = (SRC( 6 ) >> 1) + SRC( 2 );          \
        const rc_s2 b0 = a0 + a6, b2 = a2 + a4, b4 = a2 - a4, b6 = a0 - a6;                    \
        const rc_s2 a1 = -SRC( 3 ) + SRC( 5 ) - SRC( 7 ) - (SRC( 7 ) >> 1);                    \
        const rc_s2 a3 = SRC( 1 ) + SRC( 7 ) - SRC( 3 ) - (SRC( 3 ) >> 1);                     \
        const rc_s2 a5 = -SRC( 1 ) + SRC( 7 ) + SRC( 5 ) + (SRC( 5 ) >> 1);                    \
        const rc_s2 a7 = SRC( 3 ) + SRC( 5 ) + SRC( 1 ) + (SRC( 1 ) >> 1);                     \
        const rc_s2 b1 = (a7 >> 2) + a1, b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5, b7 = a7 - (a1 >> 2); \
        DST( 0, b0 + b7 ); DST( 1, b2 + b5 ); DST( 2, b4 + b3 ); DST( 3, b6 + b1 );            \
        DST( 4, b6 - b1 ); DST( 5, b4 - b3 ); DST( 6, b2 - b5 ); DST( 7, b0 - b7 );            \
    }

// max over the pairs of C of |v| + 4096 as unsigned 16-bit (<= 8192 iff every |v| <= 4096)
__device__ __forceinline__ bool recon8_small( const uint32_t (&C)[8][4] )
{
    typedef unsigned short u2 __attribute__( ( ext_vector_type( 2 ) ) );
    u2 mx = (u2)0;
#pragma unroll
    for( int x = 0; x < 8; x++ )
#pragma unroll
        for( int k = 0; k < 4; k++ )
            mx = __builtin_elementwise_max( mx, __builtin_bit_cast( u2, C[x][k] ) + (u2)4096 );
    return mx.x <= 8192 && mx.y <= 8192;
}

template <bool M24>
__device__ __forceinline__ void recon8_pk_block( const int16_t *__restrict__ dct, const int32_t *m, int q,
                                                 const uint8_t *pp, intptr_t ps, uint8_t *rp, intptr_t rs )
{
    uint32_t C[8][4];                                     // C[x][k] = (c[x*8+2k], c[x*8+2k+1])
#pragma unroll
    for( int x = 0; x < 8; x++ )
    {
        const uint4 w = ((const uint4 *)dct)[x];
        C[x][0] = w.x; C[x][1] = w.y; C[x][2] = w.z; C[x][3] = w.w;
    }
    const int qb = q / 6 - 6;
#pragma unroll
    for( int x = 0; x < 8; x++ )
    {
        const int4 m0 = ((const int4 *)(m + x * 8))[0], m1 = ((const int4 *)(m + x * 8))[1];
        const int mm[8] = { m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w };
#pragma unroll
        for( int k = 0; k < 4; k++ )
        {
            int v[2];
#pragma unroll
            for( int h = 0; h < 2; h++ )
            {
                const int c = h ? (int)(int16_t)(C[x][k] >> 16) : (int)(int16_t)C[x][k];
                const int mv = mm[2 * k + h];
                const int p = M24 ? __mul24( c, mv ) : c * mv;
                v[h] = qb >= 0 ? (int)((uint32_t)p << qb) : (p + (1 << (-qb - 1))) >> (-qb);
            }
            C[x][k] = rc_pack( v[0], v[1] );
        }
    }
    C[0][0] = rc_asu( rc_as2( C[0][0] ) + (rc_s2){ 32, 0 } );   // dct[0] += 32, stored as dctcoef
    // column pass (SRC(x) = c[x*8+i], stored back as dctcoef) on column pairs.  Every partial
    // sum of IDCT8_1D is at most 7.875 max|input| (+ the floor shifts' units), so with all
    // inputs within +-4096 the int16 pair arithmetic is exact; otherwise int32 per column.
    if( recon8_small( C ) )
    {
#pragma unroll
        for( int k = 0; k < 4; k++ )
        {
            rc_s2 o[8];
#define SRC( x ) rc_as2( C[x][k] )
#define DST( x, v ) o[x] = ( v )
            IDCT8_1D_PK( SRC, DST )
#undef SRC
#undef DST
#pragma unroll
            for( int x = 0; x < 8; x++ )
                C[x][k] = rc_asu( o[x] );
        }
    }
    else
    {
#pragma unroll
        for( int k = 0; k < 4; k++ )
        {
            int o[2][8];
#pragma unroll
            for( int h = 0; h < 2; h++ )
            {
#define SRC( x ) (h ? (int)(int16_t)(C[x][k] >> 16) : (int)(int16_t)C[x][k])
#define DST( x, v ) o[h][x] = ( v )
                IDCT8_1D( SRC, DST )
#undef SRC
#undef DST
            }
#pragma unroll
            for( int x = 0; x < 8; x++ )
                C[x][k] = rc_pack( o[0][x], o[1][x] );
        }
    }
    // row pass on row pairs (i, i+1): SRC(x) = c[i*8+x]; residual r[y][i] = v >> 6 goes onto
    // the prediction pixel pair (y; i, i+1) in place (16-bit pairs, clip by v_pk_max/min)
    uint32_t P[8][2];
#pragma unroll
    for( int y = 0; y < 8; y++ )
        load_packed<2>( pp + y * ps, P[y] );
    const bool small = recon8_small( C );
#pragma unroll
    for( int k = 0; k < 4; k++ )
    {
        rc_s2 r[8];
        if( small )
        {
            rc_s2 sv[8];
#pragma unroll
            for( int x = 0; x < 8; x++ )
                sv[x] = rc_as2( __builtin_amdgcn_perm( C[2 * k + 1][x >> 1], C[2 * k][x >> 1],
                                                       (x & 1) ? 0x07060302u : 0x05040100u ) );
#define SRC( x ) sv[x]
#define DST( x, v ) r[x] = ( v ) >> 6
            IDCT8_1D_PK( SRC, DST )
#undef SRC
#undef DST
        }
        else
        {
            int o[2][8];
#pragma unroll
            for( int h = 0; h < 2; h++ )
            {
                const int i = 2 * k + h;
#define SRC( x ) (((x) & 1) ? (int)(int16_t)(C[i][(x) >> 1] >> 16) : (int)(int16_t)C[i][(x) >> 1])
#define DST( x, v ) o[h][x] = ( v ) >> 6
                IDCT8_1D( SRC, DST )
#undef SRC
#undef DST
            }
#pragma unroll
            for( int y = 0; y < 8; y++ )
                r[y] = rc_as2( rc_pack( o[0][y], o[1][y] ) );
        }
        const uint32_t SEL = (k & 1) ? 0x0c030c02u : 0x0c010c00u;   // pixels 2k, 2k+1 of the dword
#pragma unroll
        for( int y = 0; y < 8; y++ )
        {
            rc_s2 v = rc_as2( __builtin_amdgcn_perm( 0u, P[y][k >> 1], SEL ) ) + r[y];
            v = __builtin_elementwise_min( __builtin_elementwise_max( v, (rc_s2)0 ), (rc_s2)255 );
            // the two result bytes replace the two prediction bytes
            P[y][k >> 1] = (k & 1) ? __builtin_amdgcn_perm( rc_asu( v ), P[y][k >> 1], 0x06040100u )
                                   : __builtin_amdgcn_perm( P[y][k >> 1], rc_asu( v ), 0x07060200u );
        }
    }
#pragma unroll
    for( int y = 0; y < 8; y++ )
    {
        if( ((uintptr_t)(rp + y * rs) & 3) == 0 )
        {
            ((uint32_t *)(rp + y * rs))[0] = P[y][0];
            ((uint32_t *)(rp + y * rs))[1] = P[y][1];
        }
        else
        {
#pragma unroll
            for( int x = 0; x < 8; x++ )
                rp[y * rs + x] = (uint8_t)(P[y][x >> 2] >> (8 * (x & 3)));
        }
    }
}
#undef IDCT8_1D_PK

// lanes per 8x8-block row: the row's bw blocks shifted right by sh (0..7) lanes and padded to
// whole waves, so every wave's 512-byte row pieces start on a 64-byte sector (launch_mb_recon)
__global__ __launch_bounds__( 256 ) void mb_recon8_pk_kernel( const int16_t *__restrict__ dct, int mbw, int mbh,
                                                              int nframes, const int32_t *__restrict__ dmf,
                                                              const int32_t *__restrict__ qp,
                                                              const uint8_t *pred, intptr_t ps, intptr_t pfs,
                                                              uint8_t *recon, intptr_t rs, intptr_t rfs, int sh )
{
    // the 6 x 64 dequant_mf table in LDS, rows 68 dwords apart (lanes on different qp%6
    // rows read different 16-B slots of a bank row)
    __shared__ int32_t tab[6 * 68];
    int ok = 1;
    for( int i = threadIdx.x; i < 6 * 64; i += blockDim.x )
    {
        const int v = dmf[i];
        tab[(i >> 6) * 68 + (i & 63)] = v;
        ok &= v >= -(1 << 23) && v < (1 << 23);
    }
    const bool m24 = __syncthreads_and( ok );
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int bw = mbw * 2, bh = mbh * 2, lpr = (bw + sh + 63) & ~63;
    if( t >= (int64_t)nframes * lpr * bh )
        return;
    const int bx = (int)(t % lpr) - sh;
    if( bx < 0 || bx >= bw )
        return;
    const int64_t r = t / lpr;
    const int by = (int)(r % bh);
    const int f = (int)(r / bh);
    const int64_t mb = ((int64_t)f * mbh + (by >> 1)) * mbw + (bx >> 1);
    const int q = qp[mb];
    const int16_t *c = dct + mb * 256 + ((by & 1) * 2 + (bx & 1)) * 64;
    const uint8_t *pp = pred + f * pfs + (intptr_t)(by * 8) * ps + bx * 8;
    uint8_t *rp = recon + f * rfs + (intptr_t)(by * 8) * rs + bx * 8;
    const int32_t *m = tab + (q % 6) * 68;
    if( m24 )
        recon8_pk_block<true>( c, m, q, pp, ps, rp, rs );
    else
        recon8_pk_block<false>( c, m, q, pp, ps, rp, rs );
}

template <int BD>
hipError_t launch_mb_recon( int transform, const typename PT<BD>::dctcoef *dct, int mbw, int mbh, int nframes,
                            const int32_t *dmf, const int32_t *qp, const typename PT<BD>::pixel *pred, intptr_t ps,
                            intptr_t pfs, typename PT<BD>::pixel *recon, intptr_t rs, intptr_t rfs, hipStream_t st )
{
    if( mbw <= 0 || mbh <= 0 || nframes <= 0 )
        return hipSuccess;
    if( transform != 4 && transform != 8 )
        return hipErrorInvalidValue;
    // 8 bit: block pairs for transform 4 (0.55 vs 0.43 of HBM in a round-3 A/B, driver since removed) and
    // the packed int16-pair kernel for transform 8; 10 bit: one lane per block (0.68 vs 0.58
    // for the pairs).
    // Sector alignment of the stores: with row and frame strides multiples of 64 bytes, every
    // row of the output plane has x = 0 at the same offset within a 64-byte sector; shifting
    // the waves' pixel ranges by that offset puts every wave's row pieces on whole sectors
    // (partial sectors shared by two waves were the half-pel planes' bottleneck).
    const size_t psz = sizeof( typename PT<BD>::pixel );
    const bool al = !(((size_t)rs * psz) & 63) && !(((size_t)rfs * psz) & 63);
    const int off = al ? (int)((uintptr_t)recon & 63) : 0;       // byte offset of x = 0 in its sector
    if constexpr( BD == 8 )
    {
        if( transform == 8 )
        {
            const int sh8 = off % 8 ? 0 : off / 8;                 // 8-pixel blocks
            const int64_t total = (int64_t)nframes * mbh * 2 * ((mbw * 2 + sh8 + 63) & ~63);
            hipLaunchKernelGGL( mb_recon8_pk_kernel, dim3( (unsigned)((total + 255) / 256) ), dim3( 256 ), 0, st, dct,
                                mbw, mbh, nframes, dmf, qp, pred, ps, pfs, recon, rs, rfs, sh8 );
            return hipGetLastError();
        }
        const int sh = off % 16 ? 0 : off / 16;                    // 16-pixel MBs
        const int64_t waves = (int64_t)nframes * mbh * ((mbw + sh + 7) / 8);
        hipLaunchKernelGGL( mb_recon_pair_kernel<BD>, dim3( (unsigned)((waves + 3) / 4) ), dim3( 256 ), 0, st, dct,
                            mbw, mbh, nframes, dmf, qp, pred, ps, pfs, recon, rs, rfs, sh );
        return hipGetLastError();
    }
    const int bpm = transform == 8 ? 4 : 16;
    const int64_t total = (int64_t)nframes * mbw * mbh * bpm;
    dim3 blk( 256 ), g( (unsigned)((total + 255) / 256) );
    if( transform == 8 )
        hipLaunchKernelGGL( ( mb_recon_kernel<BD, 8> ), g, blk, 0, st, dct, mbw, mbh, nframes, dmf, qp, pred, ps, pfs,
                            recon, rs, rfs );
    else
        hipLaunchKernelGGL( ( mb_recon_kernel<BD, 4> ), g, blk, 0, st, dct, mbw, mbh, nframes, dmf, qp, pred, ps, pfs,
                            recon, rs, rfs );
    return hipGetLastError();
}

#define INST( BD )                                                                                                     \
    template hipError_t launch_add_idct<BD>( int, PT<BD>::pixel *, intptr_t, const int64_t *, const PT<BD>::dctcoef *, \
                                             int, hipStream_t );                                                       \
    template hipError_t launch_dequant<BD>( int, PT<BD>::dctcoef *, const int32_t *, const int32_t *, int,             \
                                            hipStream_t );                                                             \
    template hipError_t launch_idct4x4dc<BD>( PT<BD>::dctcoef *, int, hipStream_t );                                   \
    template hipError_t launch_idct_dequant_2x4<BD>( int, PT<BD>::dctcoef *, PT<BD>::dctcoef *, const int32_t *,       \
                                                     const int32_t *, int, hipStream_t );                              \
    template hipError_t launch_optimize_chroma<BD>( int, PT<BD>::dctcoef *, const int32_t *, int, int32_t *,           \
                                                    hipStream_t );                                                     \
    template hipError_t launch_denoise<BD>( PT<BD>::dctcoef *, int, int, uint32_t *, const PT<BD>::udctcoef *,         \
                                            hipStream_t );                                                             \
    template hipError_t launch_coef_stat<BD>( int, const PT<BD>::dctcoef *, int64_t, int, int32_t *, hipStream_t );    \
    template hipError_t launch_level_run<BD>( int, const PT<BD>::dctcoef *, int64_t, int, int32_t *, int32_t *,        \
                                              int32_t *, PT<BD>::dctcoef *, hipStream_t );                             \
    template hipError_t launch_zigzag_scan<BD>( int, int, PT<BD>::dctcoef *, const PT<BD>::dctcoef *, int,             \
                                                hipStream_t );                                                         \
    template hipError_t launch_zigzag_sub<BD>( int, int, PT<BD>::dctcoef *, PT<BD>::dctcoef *, const PT<BD>::pixel *,  \
                                               intptr_t, PT<BD>::pixel *, intptr_t, const int64_t *, const int64_t *,  \
                                               int, int32_t *, hipStream_t );                                          \
    template hipError_t launch_interleave<BD>( PT<BD>::dctcoef *, const PT<BD>::dctcoef *, uint8_t *, int,             \
                                               hipStream_t );                                                          \
    template hipError_t launch_mb_recon<BD>( int, const PT<BD>::dctcoef *, int, int, int, const int32_t *,             \
                                             const int32_t *, const PT<BD>::pixel *, intptr_t, intptr_t,               \
                                             PT<BD>::pixel *, intptr_t, intptr_t, hipStream_t );
INST( 8 )
INST( 10 )
#undef INST

} // namespace x264hip
