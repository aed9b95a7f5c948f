// HBM probe for the half-pel filter's access pattern (no arithmetic): every lane
// reads one 16-byte piece per source row and writes it to three output planes,
// over the same padded 1080p plane geometry and frame count as the hpel bench
// leg.  Variants: 1 = the streaming kernel's grid (a wave per 62-piece column
// chunk x ROWS-row strip), 2 = a plain grid-stride copy of the same bytes
// (1 plane in, 3 out), 3 = a plain 1-in-1-out copy of one plane (reference), 4 = the
// frame_init_lowres pattern (three source rows per output row, four half-width planes out),
// 5 = the fused DCT+quant pattern (two planes in, 2-byte coefficients out), 6 = the
// reconstruction pattern (coefficients + prediction in, one plane out).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

template <int ROWS>
__global__ __launch_bounds__( 64 ) void strip3( const uint8_t *src, uint8_t *a, uint8_t *b, uint8_t *c, long stride,
                                                long fstride, int pieces, int rows_total )
{
    const int lane = threadIdx.x;
    const int q = blockIdx.x * 64 + lane;
    if( q >= pieces )
        return;
    const int r0 = blockIdx.y * ROWS;
    const long fo = (long)blockIdx.z * fstride + 16 * q;
    for( int r = r0; r < r0 + ROWS && r < rows_total; r++ )
    {
        const uint4 v = *(const uint4 *)(src + fo + r * stride);
        *(uint4 *)(a + fo + r * stride) = v;
        *(uint4 *)(b + fo + r * stride) = v;
        *(uint4 *)(c + fo + r * stride) = v;
    }
}

// frame_init_lowres pattern: per output row read source rows 2y, 2y+1, 2y+2 (32 bytes per
// lane each), write 16 bytes per lane to four half-width planes
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
        const uint4 x0 = *(const uint4 *)s, x1 = *(const uint4 *)(s + 16);
        const uint4 y0 = *(const uint4 *)(s + stride), y1 = *(const uint4 *)(s + stride + 16);
        const uint4 z0 = *(const uint4 *)(s + 2 * stride), z1 = *(const uint4 *)(s + 2 * stride + 16);
        const uint4 v = make_uint4( x0.x ^ x1.x ^ y0.x ^ y1.x ^ z0.x ^ z1.x, x0.y ^ x1.y ^ y0.y, x0.z ^ y1.z ^ z0.z,
                                    x1.w ^ y0.w ^ z1.w );
        const long o = blockIdx.z * dfs + (long)y * ds + 16 * k;
        *(uint4 *)(a + o) = v;
        *(uint4 *)(b + o) = v;
        *(uint4 *)(c + o) = v;
        *(uint4 *)(d + o) = v;
    }
}

// the fused DCT+quant pattern: two 1-byte planes in (fenc, pred), one 2-byte coefficient
// stream out (16 B of each input per lane -> 32 B out); and the reconstruction pattern:
// the 2-byte coefficients + pred in, one plane out
__global__ void dctpat( const uint4 *fe, const uint4 *pr, uint4 *co, long n16 )
{
    for( long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (long)gridDim.x * blockDim.x )
    {
        const uint4 a = fe[i], b = pr[i];
        co[2 * i] = make_uint4( a.x ^ b.x, a.y, b.z, a.w );
        co[2 * i + 1] = make_uint4( a.z, b.y ^ a.y, b.w, b.x );
    }
}
__global__ void recpat( const uint4 *co, const uint4 *pr, uint4 *out, long n16 )
{
    for( long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (long)gridDim.x * blockDim.x )
    {
        const uint4 a = co[2 * i], b = co[2 * i + 1], c = pr[i];
        out[i] = make_uint4( a.x ^ b.x ^ c.x, a.y ^ b.y, a.z ^ c.z, a.w ^ b.w ^ c.w );
    }
}

__global__ void flat3( const uint4 *src, uint4 *a, uint4 *b, uint4 *c, long n )
{
    for( long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x )
    {
        const uint4 v = src[i];
        a[i] = v;
        b[i] = v;
        c[i] = v;
    }
}

__global__ void flat1( const uint4 *src, uint4 *a, long n )
{
    for( long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x )
        a[i] = src[i];
}

int main( int argc, char **argv )
{
    const int F = argc > 1 ? atoi( argv[1] ) : 16;
    const long stride = 1984, rows = 1152, fstride = stride * rows;
    const long bytes = F * fstride;
    uint8_t *s, *a, *b, *c;
    hipMalloc( &s, bytes ); hipMalloc( &a, bytes ); hipMalloc( &b, bytes ); hipMalloc( &c, bytes );
    hipMemset( s, 1, bytes );
    hipEvent_t e0, e1;
    hipEventCreate( &e0 ); hipEventCreate( &e1 );
    const int pieces = (int)(stride / 16);
    uint8_t *l[4];
    const long ds = 1024, dfs = ds * (544 + 64), lbytes = F * dfs;
    for( int i = 0; i < 4; i++ )
        hipMalloc( &l[i], lbytes );
    uint8_t *co;
    hipMalloc( &co, 2 * bytes );
    for( int v = 1; v <= 6; v++ )
    {
        auto run = [&]() {
            if( v == 1 )
                hipLaunchKernelGGL( strip3<12>, dim3( (pieces + 63) / 64, (rows + 11) / 12, F ), dim3( 64 ), 0, 0, s, a,
                                    b, c, stride, fstride, pieces, (int)rows );
            else if( v == 2 )
                hipLaunchKernelGGL( flat3, dim3( 4096 ), dim3( 256 ), 0, 0, (const uint4 *)s, (uint4 *)a, (uint4 *)b,
                                    (uint4 *)c, bytes / 16 );
            else if( v == 3 )
                hipLaunchKernelGGL( flat1, dim3( 4096 ), dim3( 256 ), 0, 0, (const uint4 *)s, (uint4 *)a, bytes / 16 );
            else if( v == 5 )
                hipLaunchKernelGGL( dctpat, dim3( 4096 ), dim3( 256 ), 0, 0, (const uint4 *)s, (const uint4 *)a,
                                    (uint4 *)co, bytes / 16 );
            else if( v == 6 )
                hipLaunchKernelGGL( recpat, dim3( 4096 ), dim3( 256 ), 0, 0, (const uint4 *)co, (const uint4 *)a,
                                    (uint4 *)b, bytes / 16 );
            else
                hipLaunchKernelGGL( lowres4, dim3( 1, 272, F ), dim3( 64 ), 0, 0, s, l[0], l[1], l[2], l[3], stride,
                                    fstride, ds, dfs, 60, 544 );
        };
        for( int i = 0; i < 300; i++ )
            run();
        hipEventRecord( e0 );
        for( int i = 0; i < 100; i++ )
            run();
        hipEventRecord( e1 );
        hipEventSynchronize( e1 );
        float ms;
        hipEventElapsedTime( &ms, e0, e1 );
        ms /= 100;
        const double moved = v == 3 ? 2.0 * bytes : v == 4 ? (double)F * (1088 * 1920 + 4 * 544 * 960)
                           : v == 5 || v == 6 ? 4.0 * bytes : 4.0 * bytes;
        printf( "variant %d: %.4f ms, %.2f TB/s, %.3f of 8 TB/s\n", v, ms, moved / ms / 1e9, moved / ms / 1e9 / 8.0 );
    }
    return 0;
}
