// HBM probe for the streaming frame kernels' access patterns at 64 padded 1080p frames
// (no arithmetic): what the half-pel filter's 1-in-3-out and frame_init_lowres's
// 1-in-4-quarter-out patterns reach with each store / load flavour and grid shape.
//   s3   : the hpel grid (a wave per 62..64-piece column chunk x ROWS-row strip), plain
//   s3nt : the same with nontemporal stores
//   s3ntl: nontemporal loads and stores
//   s3w4 : four strips per 256-thread workgroup
//   f3 / f3nt : a grid-stride copy of the same bytes (1 plane in, 3 out)
//   wo3  : write-only (three planes from registers), rd1: read-only (one plane, reduced)
//   l4 / l4nt : the lowres pattern (three source rows per output row, 4 half planes out)
//   c1 / c1nt : plain 1-in-1-out copy (reference)
// Usage: stream_pattern [frames]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int v4u __attribute__( ( ext_vector_type( 4 ) ) );

template <bool NT> __device__ __forceinline__ void st( uint8_t *p, v4u v )
{
    if constexpr( NT )
        __builtin_nontemporal_store( v, (v4u *)p );
    else
        *(v4u *)p = v;
}
template <bool NT> __device__ __forceinline__ v4u ld( const uint8_t *p )
{
    if constexpr( NT )
        return __builtin_nontemporal_load( (const v4u *)p );
    else
        return *(const v4u *)p;
}

template <int ROWS, bool NTS, bool NTL>
__global__ __launch_bounds__( 256 ) void strip3( const uint8_t *src, uint8_t *a, uint8_t *b, uint8_t *c, long stride,
                                                 long fstride, int pieces, int rows_total )
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int q = blockIdx.x * 64 + lane;
    if( q >= pieces )
        return;
    const int r0 = (blockIdx.y * (blockDim.x >> 6) + w) * ROWS;
    const long fo = (long)blockIdx.z * fstride + 16 * q;
    for( int r = r0; r < r0 + ROWS && r < rows_total; r++ )
    {
        const v4u v = ld<NTL>( src + fo + r * stride );
        st<NTS>( a + fo + r * stride, v );
        st<NTS>( b + fo + r * stride, v );
        st<NTS>( c + fo + r * stride, v );
    }
}

// the hpel kernel's chunking: 62 storing lanes per wave (lanes 1..62), pieces at byte
// offset 16 + 16 q -- chunk boundaries and the row start off the 128-B line grid (OFF = 16)
// or on it (OFF = 0, CH = 56: 7 lines per wave)
template <int ROWS, int CH, int OFF>
__global__ __launch_bounds__( 64 ) void strip3c( const uint8_t *src, uint8_t *a, uint8_t *b, uint8_t *c, long stride,
                                                 long fstride, int pieces, int rows_total )
{
    const int lane = threadIdx.x & 63;
    const int q = (int)blockIdx.x * CH + lane - 1;
    if( lane < 1 || lane > CH || q >= pieces )
        return;
    const int r0 = blockIdx.y * ROWS;
    const long fo = (long)blockIdx.z * fstride + OFF + 16 * q;
    for( int r = r0; r < r0 + ROWS && r < rows_total; r++ )
    {
        const v4u v = ld<false>( src + fo + r * stride );
        st<true>( a + fo + r * stride, v );
        st<true>( b + fo + r * stride, v );
        st<true>( c + fo + r * stride, v );
    }
}

template <bool NT> __global__ void flat3( const uint8_t *src, uint8_t *a, uint8_t *b, uint8_t *c, long n )
{
    for( long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x )
    {
        const v4u v = ld<false>( src + 16 * i );
        st<NT>( a + 16 * i, v );
        st<NT>( b + 16 * i, v );
        st<NT>( c + 16 * i, v );
    }
}

template <bool NT> __global__ void wo3( uint8_t *a, uint8_t *b, uint8_t *c, long n )
{
    const v4u v = { (unsigned)threadIdx.x, 1u, 2u, 3u };
    for( long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x )
    {
        st<NT>( a + 16 * i, v );
        st<NT>( b + 16 * i, v );
        st<NT>( c + 16 * i, v );
    }
}

__global__ void rd1( const uint8_t *src, uint8_t *out, long n )
{
    v4u acc = { 0, 0, 0, 0 };
    for( long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x )
        acc ^= ld<false>( src + 16 * i );
    if( (acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u )
        out[threadIdx.x] = 1;
}

template <bool NT> __global__ void c1( const uint8_t *src, uint8_t *a, long n )
{
    for( long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x )
        st<NT>( a + 16 * i, ld<false>( src + 16 * i ) );
}

template <bool NT>
__global__ __launch_bounds__( 64 ) void lowres4( const uint8_t *src, uint8_t *a, uint8_t *b, uint8_t *c, uint8_t *d,
                                                 long stride, long fstride, long ds, long dfs, int lanes, int hl )
{
    const int k = threadIdx.x;
    if( k >= lanes )
        return;
    for( int rr = 0; rr < 2; rr++ )
    {
        const int y = blockIdx.y * 2 + rr;
        if( y >= hl )
            return;
        const uint8_t *s = src + blockIdx.z * fstride + (long)(2 * y) * stride + 32 * k;
        const v4u x0 = ld<false>( s ), x1 = ld<false>( s + 16 );
        const v4u y0 = ld<false>( s + stride ), y1 = ld<false>( s + stride + 16 );
        const v4u z0 = ld<false>( s + 2 * stride ), z1 = ld<false>( s + 2 * stride + 16 );
        const v4u v = x0 ^ x1 ^ y0 ^ y1 ^ z0 ^ z1;
        const long o = blockIdx.z * dfs + (long)y * ds + 16 * k;
        st<NT>( a + o, v );
        st<NT>( b + o, v );
        st<NT>( c + o, v );
        st<NT>( d + o, v );
    }
}

int main( int argc, char **argv )
{
    const int F = argc > 1 ? atoi( argv[1] ) : 64;
    const long stride = 1984, rows = 1152, fstride = stride * rows;
    const long bytes = F * fstride;
    uint8_t *s, *a, *b, *c;
    if( hipMalloc( &s, bytes ) || hipMalloc( &a, bytes ) || hipMalloc( &b, bytes ) || hipMalloc( &c, bytes ) )
        return 1;
    (void)hipMemset( s, 1, bytes );
    hipEvent_t e0, e1;
    (void)hipEventCreate( &e0 );
    (void)hipEventCreate( &e1 );
    const int pieces = (int)(stride / 16);
    uint8_t *l[4];
    const long ds = 1024, dfs = ds * (544 + 64), lbytes = F * dfs;
    for( int i = 0; i < 4; i++ )
        if( hipMalloc( &l[i], lbytes ) )
            return 1;
    const char *names[] = { "", "s3", "s3nt", "s3ntl", "s3w4", "f3", "f3nt", "wo3", "wo3nt", "rd1", "l4", "l4nt",
                            "c1", "c1nt", "s3_24", "s3nt_24", "s3nt62u", "s3nt56a" };
    const int NV = 17;
    const dim3 gs( (pieces + 63) / 64, (rows + 11) / 12, F );
    double ms_sum[NV + 1] = {};
    int cnt[NV + 1] = {};
    for( int round = 0; round < 4; round++ )
        for( int v = 1; v <= NV; v++ )
        {
            auto run = [&]() {
                switch( v )
                {
                case 1: hipLaunchKernelGGL( ( strip3<12, false, false> ), gs, dim3( 64 ), 0, 0, s, a, b, c, stride, fstride, pieces, (int)rows ); break;
                case 2: hipLaunchKernelGGL( ( strip3<12, true, false> ), gs, dim3( 64 ), 0, 0, s, a, b, c, stride, fstride, pieces, (int)rows ); break;
                case 3: hipLaunchKernelGGL( ( strip3<12, true, true> ), gs, dim3( 64 ), 0, 0, s, a, b, c, stride, fstride, pieces, (int)rows ); break;
                case 4: hipLaunchKernelGGL( ( strip3<12, false, false> ), dim3( gs.x, (gs.y + 3) / 4, F ), dim3( 256 ), 0, 0, s, a, b, c, stride, fstride, pieces, (int)rows ); break;
                case 5: hipLaunchKernelGGL( flat3<false>, dim3( 4096 ), dim3( 256 ), 0, 0, s, a, b, c, bytes / 16 ); break;
                case 6: hipLaunchKernelGGL( flat3<true>, dim3( 4096 ), dim3( 256 ), 0, 0, s, a, b, c, bytes / 16 ); break;
                case 7: hipLaunchKernelGGL( wo3<false>, dim3( 4096 ), dim3( 256 ), 0, 0, a, b, c, bytes / 16 ); break;
                case 8: hipLaunchKernelGGL( wo3<true>, dim3( 4096 ), dim3( 256 ), 0, 0, a, b, c, bytes / 16 ); break;
                case 9: hipLaunchKernelGGL( rd1, dim3( 4096 ), dim3( 256 ), 0, 0, s, a, bytes / 16 ); break;
                case 10: hipLaunchKernelGGL( lowres4<false>, dim3( 1, 272, F ), dim3( 64 ), 0, 0, s, l[0], l[1], l[2], l[3], stride, fstride, ds, dfs, 60, 544 ); break;
                case 11: hipLaunchKernelGGL( lowres4<true>, dim3( 1, 272, F ), dim3( 64 ), 0, 0, s, l[0], l[1], l[2], l[3], stride, fstride, ds, dfs, 60, 544 ); break;
                case 12: hipLaunchKernelGGL( c1<false>, dim3( 4096 ), dim3( 256 ), 0, 0, s, a, bytes / 16 ); break;
                case 13: hipLaunchKernelGGL( c1<true>, dim3( 4096 ), dim3( 256 ), 0, 0, s, a, bytes / 16 ); break;
                case 14: hipLaunchKernelGGL( ( strip3<24, false, false> ), dim3( gs.x, (rows + 23) / 24, F ), dim3( 64 ), 0, 0, s, a, b, c, stride, fstride, pieces, (int)rows ); break;
                case 15: hipLaunchKernelGGL( ( strip3<24, true, false> ), dim3( gs.x, (rows + 23) / 24, F ), dim3( 64 ), 0, 0, s, a, b, c, stride, fstride, pieces, (int)rows ); break;
                case 16: hipLaunchKernelGGL( ( strip3c<12, 62, 16> ), dim3( (pieces - 1 + 61) / 62, (rows + 11) / 12, F ), dim3( 64 ), 0, 0, s, a, b, c, stride, fstride, pieces - 1, (int)rows ); break;
                case 17: hipLaunchKernelGGL( ( strip3c<12, 56, 0> ), dim3( (pieces + 55) / 56, (rows + 11) / 12, F ), dim3( 64 ), 0, 0, s, a, b, c, stride, fstride, pieces, (int)rows ); break;
                }
            };
            for( int i = 0; i < (round ? 20 : 200); i++ )
                run();
            (void)hipEventRecord( e0 );
            for( int i = 0; i < 20; i++ )
                run();
            (void)hipEventRecord( e1 );
            (void)hipEventSynchronize( e1 );
            float ms;
            (void)hipEventElapsedTime( &ms, e0, e1 );
            if( hipGetLastError() != hipSuccess )
                return 2;
            ms_sum[v] += ms / 20;
            cnt[v]++;
        }
    for( int v = 1; v <= NV; v++ )
    {
        const double ms = ms_sum[v] / cnt[v];
        const double moved = v == 9 ? (double)bytes : v == 7 || v == 8 ? 3.0 * bytes : v == 12 || v == 13 ? 2.0 * bytes
                           : v == 10 || v == 11 ? (double)F * (1088 * 1920 + 4 * 544 * 960) : 4.0 * bytes;
        printf( "%-8s F=%d: %.4f ms, %.2f TB/s, %.3f of 8 TB/s\n", names[v], F, ms, moved / ms / 1e9,
                moved / ms / 1e9 / 8.0 );
    }
    return 0;
}
