// Block metrics (SAD / SSD / SATD) over block lists in device memory.
//
// Semantics: reference common/pixel.c — PIXEL_SAD_C :55-70, PIXEL_SSD_C :85-101,
// satd 4x4 / 8x4 and the PIXEL_SATD_C tiling :265-332.  SATD is computed in
// plain (unpacked) Hadamard form: every coefficient of a 4x4 Hadamard has the
// parity of the block's difference sum, so the per-4x4 |coef| sum is even and
// the reference's ">>1 per 8x4 pair" equals ">>1 per 4x4" (checked against the
// packed-form oracle in tests).
//
// One lane per (fenc block, ref block) pair; rows are fetched as aligned dwords
// and realigned with v_alignbyte_b32, SAD uses v_sad_u8 / v_sad_u16.
#include "hipcommon.h"

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
    else                             // SATD
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
    }
    return hipErrorInvalidValue;
}

template hipError_t launch_cmp_batch<8>( int, int, const uint8_t *, intptr_t, const uint8_t *, intptr_t,
                                         const int64_t *, const int64_t *, int, int32_t *, hipStream_t );
template hipError_t launch_cmp_batch<10>( int, int, const uint16_t *, intptr_t, const uint16_t *, intptr_t,
                                          const int64_t *, const int64_t *, int, int32_t *, hipStream_t );

} // namespace x264hip
