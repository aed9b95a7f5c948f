// SSIM (reference common/pixel.c:627-714): ssim_4x4x2_core, ssim_end4 and the frame metric
// x264_pixel_ssim_wxh that x264 accumulates per filtered MB row (encoder/encoder.c:2517-2528).
//
// x264_pixel_ssim_wxh sums its per-window floats into ONE float in a fixed order (rows, then
// groups of up to four windows, each group summed first by ssim_end4), and float addition
// does not reassociate.  So the metric runs as three steps: every 4x4 block's four sums (one
// lane per block), every group's ssim_end4 (one lane per group: its <= 4 windows in order),
// then one lane adds the groups in the reference's order -- bit-identical to the scalar
// walk, with all the pixel work parallel.
#include "hipcommon.h"

namespace x264hip {

#pragma clang fp contract( off )

// ssim_end1: float arithmetic above 9 bits, int below (pixel.c:654-677)
template <int BD> __device__ __forceinline__ float ssim_end1( int s1, int s2, int ss, int s12 )
{
    if constexpr( BD > 9 )
    {
        constexpr float c1 = (float)(.01 * .01 * 1023 * 1023 * 64);
        constexpr float c2 = (float)(.03 * .03 * 1023 * 1023 * 64 * 63);
        const float fs1 = (float)s1, fs2 = (float)s2, fss = (float)ss, fs12 = (float)s12;
        const float vars = fss * 64 - fs1 * fs1 - fs2 * fs2;
        const float covar = fs12 * 64 - fs1 * fs2;
        return (2 * fs1 * fs2 + c1) * (2 * covar + c2) / ((fs1 * fs1 + fs2 * fs2 + c1) * (vars + c2));
    }
    else
    {
        constexpr int c1 = (int)(.01 * .01 * 255 * 255 * 64 + .5);
        constexpr int c2 = (int)(.03 * .03 * 255 * 255 * 64 * 63 + .5);
        const int vars = ss * 64 - s1 * s1 - s2 * s2;
        const int covar = s12 * 64 - s1 * s2;
        return (float)(2 * s1 * s2 + c1) * (float)(2 * covar + c2) /
               ((float)(s1 * s1 + s2 * s2 + c1) * (float)(vars + c2));
    }
}

// ssim_end4 over sums rows r0 / r1 (int4 per 4x4 block) from column x, n <= 4 windows
template <int BD>
__device__ __forceinline__ float ssim_end4_dev( const int4 *r0, const int4 *r1, int n )
{
    float ssim = 0.0f;
    for( int i = 0; i < n; i++ )
    {
        const int4 a = r0[i], b = r0[i + 1], c = r1[i], d = r1[i + 1];
        ssim += ssim_end1<BD>( a.x + b.x + c.x + d.x, a.y + b.y + c.y + d.y, a.z + b.z + c.z + d.z,
                               a.w + b.w + c.w + d.w );
    }
    return ssim;
}

// ssim_4x4x2_core's sums of one 4x4 block pair position: lane = block (x, z) of an nx x nz
// grid, out[z * nx + x] = (s1, s2, ss, s12) (uint32 arithmetic stored as int, as the core)
template <int BD>
__global__ __launch_bounds__( 256 ) void ssim_sums_kernel( const typename PT<BD>::pixel *__restrict__ p1,
                                                           intptr_t s1, const typename PT<BD>::pixel *__restrict__ p2,
                                                           intptr_t s2, int nx, int nz, int4 *__restrict__ out )
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if( i >= nx * nz )
        return;
    const int z = i / nx, x = i - z * nx;
    const typename PT<BD>::pixel *a = p1 + (intptr_t)4 * z * s1 + 4 * x, *b = p2 + (intptr_t)4 * z * s2 + 4 * x;
    uint32_t t1 = 0, t2 = 0, ss = 0, s12 = 0;
#pragma unroll
    for( int y = 0; y < 4; y++ )
#pragma unroll
        for( int k = 0; k < 4; k++ )
        {
            const uint32_t u = a[y * s1 + k], v = b[y * s2 + k];
            t1 += u;
            t2 += v;
            ss += u * u + v * v;
            s12 += u * v;
        }
    out[i] = make_int4( (int)t1, (int)t2, (int)ss, (int)s12 );
}

// one lane per (window row y in [1, nz), group g): ssim_end4 of windows 4g .. 4g+3
template <int BD>
__global__ __launch_bounds__( 256 ) void ssim_groups_kernel( const int4 *__restrict__ sums, int nx, int nz, int ng,
                                                             float *__restrict__ g )
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if( i >= (nz - 1) * ng )
        return;
    const int y = 1 + i / ng, x = 4 * (i % ng);
    const int n = min( 4, nx - x - 1 );
    g[i] = ssim_end4_dev<BD>( sums + (intptr_t)y * nx + x, sums + (intptr_t)(y - 1) * nx + x, n );
}

// the reference's accumulation order: row by row, group by group, into one float.  The sum is
// one dependent chain, so one lane runs it -- from LDS: the wave loads the next 1024 group
// values (coalesced, in flight while lane 0 adds the current ones) and stores them to the
// other half of a double buffer.
__global__ __launch_bounds__( 64 ) void ssim_total_kernel( const float *__restrict__ g, int n, float *__restrict__ out )
{
    constexpr int CH = 1024;
    __shared__ float4 buf[2][CH / 4];
    const int lane = threadIdx.x;
    float4 v[CH / 256];
    auto load = [&]( int c ) {
#pragma unroll
        for( int j = 0; j < CH / 256; j++ )
        {
            const int i = c * CH + 4 * (j * 64 + lane);
            v[j] = i + 3 < n ? *(const float4 *)(g + i)
                             : make_float4( i < n ? g[i] : 0.f, i + 1 < n ? g[i + 1] : 0.f,
                                            i + 2 < n ? g[i + 2] : 0.f, 0.f );
        }
    };
    float ssim = 0.0f;
    const int nc = (n + CH - 1) / CH;
    load( 0 );
    for( int c = 0; c < nc; c++ )
    {
#pragma unroll
        for( int j = 0; j < CH / 256; j++ )
            buf[c & 1][j * 64 + lane] = v[j];
        __syncthreads();
        if( c + 1 < nc )
            load( c + 1 );
        if( lane == 0 )
        {
            const int m = min( CH, n - c * CH );
            const float4 *b = buf[c & 1];
            int i = 0;
            for( ; i + 64 <= m; i += 64 )        // 16 LDS reads in flight, then 64 ordered adds
            {
                float4 t[16];
#pragma unroll
                for( int k = 0; k < 16; k++ )
                    t[k] = b[(i >> 2) + k];
#pragma unroll
                for( int k = 0; k < 16; k++ )
                {
                    ssim += t[k].x;
                    ssim += t[k].y;
                    ssim += t[k].z;
                    ssim += t[k].w;
                }
            }
            const float *bf = (const float *)b;
            for( ; i < m; i++ )
                ssim += bf[i];
        }
        __syncthreads();
    }
    if( lane == 0 )
        *out = ssim;
}

template <int BD>
hipError_t launch_ssim_wxh( const typename PT<BD>::pixel *p1, intptr_t s1, const typename PT<BD>::pixel *p2,
                            intptr_t s2, int width, int height, float *out, hipStream_t stream )
{
    const int nx = width >> 2, nz = height >> 2;
    const int ng = nx > 1 ? (nx - 1 + 3) / 4 : 0;
    const int ngroups = nz > 1 ? (nz - 1) * ng : 0;
    if( ngroups == 0 )
        return hipMemsetAsync( out, 0, sizeof( float ), stream );
    void *buf = nullptr;
    const size_t sb = sizeof( int4 ) * (size_t)nx * nz, gb = sizeof( float ) * (size_t)ngroups;
    hipError_t e = scratch_alloc( &buf, sb + gb, stream );
    if( e != hipSuccess )
        return e;
    int4 *sums = (int4 *)buf;
    float *g = (float *)((char *)buf + sb);
    hipLaunchKernelGGL( ssim_sums_kernel<BD>, dim3( (unsigned)((nx * nz + 255) / 256) ), dim3( 256 ), 0, stream, p1, s1,
                        p2, s2, nx, nz, sums );
    hipLaunchKernelGGL( ssim_groups_kernel<BD>, dim3( (unsigned)((ngroups + 255) / 256) ), dim3( 256 ), 0, stream,
                        sums, nx, nz, ng, g );
    hipLaunchKernelGGL( ssim_total_kernel, dim3( 1 ), dim3( 64 ), 0, stream, g, ngroups, out );
    e = hipGetLastError();
    const hipError_t ef = hipFreeAsync( buf, stream );
    return e != hipSuccess ? e : ef;
}
template hipError_t launch_ssim_wxh<8>( const uint8_t *, intptr_t, const uint8_t *, intptr_t, int, int, float *,
                                        hipStream_t );
template hipError_t launch_ssim_wxh<10>( const uint16_t *, intptr_t, const uint16_t *, intptr_t, int, int, float *,
                                         hipStream_t );

// The encoder's form (encoder.c:2516-2528): x264_pixel_ssim_wxh once per filtered MB-row band,
// each band's float independent of the others (the encoder adds them in double).  One
// workgroup per (band, frame) walks the band's window rows as the reference does, keeping its
// last two rows of 4x4 block sums in LDS (sum0 / sum1 of pixel.c:697-712): the workgroup
// computes a block row's sums, then every group's ssim_end4, then lane 0 adds the row's groups
// in order into the band's float -- the reference's accumulation, bit-identical, with the
// bands (68 per 1080p frame) running side by side instead of in one chain.
template <int BD>
__global__ __launch_bounds__( 256 ) void ssim_bands_kernel( const typename PT<BD>::pixel *__restrict__ p1,
                                                            intptr_t s1, intptr_t f1,
                                                            const typename PT<BD>::pixel *__restrict__ p2,
                                                            intptr_t s2, intptr_t f2, int nx,
                                                            const int2 *__restrict__ bands, int nbands,
                                                            float *__restrict__ out )
{
    extern __shared__ int4 ssim_lds[];
    const int b = blockIdx.x, f = blockIdx.y;
    const int2 bd = bands[b];
    const int nz = bd.y >> 2, ng = (nx - 1 + 3) / 4;
    float *grp = (float *)(ssim_lds + 2 * nx);             // (rows by arithmetic: an array of the two row
                                                            // pointers made them generic, flat accesses)
    const typename PT<BD>::pixel *a0 = p1 + f * f1 + (intptr_t)bd.x * s1, *b0 = p2 + f * f2 + (intptr_t)bd.x * s2;
    float ssim = 0.0f;
    for( int z = 0; z < nz; z++ )
    {
        int4 *cur = ssim_lds + (z & 1) * nx;
        for( int x = threadIdx.x; x < nx; x += blockDim.x )
        {
            const typename PT<BD>::pixel *a = a0 + (intptr_t)4 * z * s1 + 4 * x, *c = b0 + (intptr_t)4 * z * s2 + 4 * x;
            uint32_t t1 = 0, t2 = 0, ss = 0, s12 = 0;
#pragma unroll
            for( int y = 0; y < 4; y++ )
#pragma unroll
                for( int k = 0; k < 4; k++ )
                {
                    const uint32_t u = a[y * s1 + k], v = c[y * s2 + k];
                    t1 += u;
                    t2 += v;
                    ss += u * u + v * v;
                    s12 += u * v;
                }
            cur[x] = make_int4( (int)t1, (int)t2, (int)ss, (int)s12 );
        }
        __syncthreads();
        if( z == 0 )
            continue;
        for( int gi = threadIdx.x; gi < ng; gi += blockDim.x )
        {
            const int x = 4 * gi;
            // ssim_end4( sum0 = this row, sum1 = the row above ) (pixel.c:708-709)
            grp[gi] = ssim_end4_dev<BD>( cur + x, ssim_lds + ((z - 1) & 1) * nx + x, min( 4, nx - x - 1 ) );
        }
        __syncthreads();
        if( threadIdx.x == 0 )
            for( int gi = 0; gi < ng; gi++ )
                ssim += grp[gi];
        __syncthreads();
    }
    if( threadIdx.x == 0 )
        out[(intptr_t)f * nbands + b] = ssim;
}

template <int BD>
hipError_t launch_ssim_bands( const typename PT<BD>::pixel *p1, intptr_t s1, intptr_t f1,
                              const typename PT<BD>::pixel *p2, intptr_t s2, intptr_t f2, int width,
                              const int32_t *bands, int nbands, int nframes, float *out, hipStream_t stream )
{
    const int nx = width >> 2;
    if( nbands <= 0 || nframes <= 0 )
        return hipSuccess;
    if( nx > 2048 )
        return hipErrorInvalidValue;
    const size_t lds = sizeof( int4 ) * 2 * (size_t)nx + sizeof( float ) * (size_t)((nx + 2) / 4 + 1);
    hipLaunchKernelGGL( ssim_bands_kernel<BD>, dim3( (unsigned)nbands, (unsigned)nframes ), dim3( 256 ), lds, stream,
                        p1, s1, f1, p2, s2, f2, nx, (const int2 *)bands, nbands, out );
    return hipGetLastError();
}
template hipError_t launch_ssim_bands<8>( const uint8_t *, intptr_t, intptr_t, const uint8_t *, intptr_t, intptr_t, int,
                                          const int32_t *, int, int, float *, hipStream_t );
template hipError_t launch_ssim_bands<10>( const uint16_t *, intptr_t, intptr_t, const uint16_t *, intptr_t, intptr_t,
                                           int, const int32_t *, int, int, float *, hipStream_t );

// the per-call table entries' kernels: ssim_4x4x2_core of one block pair (8 ints out) and
// ssim_end4 of staged sum rows
template <int BD>
__global__ void ssim_core_kernel( const typename PT<BD>::pixel *p1, intptr_t s1, const typename PT<BD>::pixel *p2,
                                  intptr_t s2, int *out )
{
    const int z = threadIdx.x;
    if( z >= 2 )
        return;
    uint32_t t1 = 0, t2 = 0, ss = 0, s12 = 0;
    for( int y = 0; y < 4; y++ )
        for( int k = 0; k < 4; k++ )
        {
            const uint32_t u = p1[y * s1 + 4 * z + k], v = p2[y * s2 + 4 * z + k];
            t1 += u;
            t2 += v;
            ss += u * u + v * v;
            s12 += u * v;
        }
    out[4 * z] = (int)t1;
    out[4 * z + 1] = (int)t2;
    out[4 * z + 2] = (int)ss;
    out[4 * z + 3] = (int)s12;
}

template <int BD> __global__ void ssim_end4_kernel( const int4 *s0, const int4 *s1, int width, float *out )
{
    if( threadIdx.x == 0 )
        *out = ssim_end4_dev<BD>( s0, s1, width );
}

template <int BD>
hipError_t launch_ssim_core( const typename PT<BD>::pixel *p1, intptr_t s1, const typename PT<BD>::pixel *p2,
                             intptr_t s2, int *out, hipStream_t stream )
{
    hipLaunchKernelGGL( ssim_core_kernel<BD>, dim3( 1 ), dim3( 64 ), 0, stream, p1, s1, p2, s2, out );
    return hipGetLastError();
}
template <int BD>
hipError_t launch_ssim_end4( const int *s0, const int *s1, int width, float *out, hipStream_t stream )
{
    hipLaunchKernelGGL( ssim_end4_kernel<BD>, dim3( 1 ), dim3( 64 ), 0, stream, (const int4 *)s0, (const int4 *)s1,
                        width, out );
    return hipGetLastError();
}
template hipError_t launch_ssim_core<8>( const uint8_t *, intptr_t, const uint8_t *, intptr_t, int *, hipStream_t );
template hipError_t launch_ssim_core<10>( const uint16_t *, intptr_t, const uint16_t *, intptr_t, int *, hipStream_t );
template hipError_t launch_ssim_end4<8>( const int *, const int *, int, float *, hipStream_t );
template hipError_t launch_ssim_end4<10>( const int *, const int *, int, float *, hipStream_t );

} // namespace x264hip
