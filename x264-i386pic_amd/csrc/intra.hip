// Intra prediction costs: the pixel table's intra_*_x3 entries over block
// lists, and the lookahead's per-8x8 intra estimate over whole lowres frames.
//
// Semantics (reference):
//   intra_{sad,satd}_x3_{4x4,8x8c,8x16c,16x16}, intra_{sad,sa8d}_x3_8x8
//                                        common/pixel.c:518-560 (+ predict.c)
//   predict_4x4 / 8x8c / 8x16c / 16x16 V, H, DC, 8x8c P
//                                        common/predict.c:67-130, 221-308, 361-441, 495-511
//   predict_8x8_filter, predict_8x8_*    common/predict.c:632-883
//   lowres intra cost                    encoder/slicetype.c:714-757
//
// The lowres kernel is one lane per 8x8 block: fenc is held as paired columns
// (x, x+4) in 16-bit lanes, every prediction is formed in registers from the
// 25 neighbours (and the 26 filtered edge values) with compile-time indices,
// and the SATD uses the packed two-tile Hadamard of hipcommon.h.  No
// prediction touches memory.
#include "hipcommon.h"

#include <stdlib.h>

namespace x264hip {

__device__ __forceinline__ int f1( int a, int b ) { return (a + b + 1) >> 1; }
__device__ __forceinline__ int f2( int a, int b, int c ) { return (a + 2 * b + c + 2) >> 2; }

__device__ __forceinline__ x264hip_short2 mk2( int a, int b )
{
    return x264hip_short2{ (short)a, (short)b };
}

// ------------------------------------------------------------- 8x8 directional modes
// predict_8x8 modes 3..8 on the filtered edge e[] (e[7..14] = l7..l0, e[15] = lt,
// e[16..32] = t0..t15, t15) in closed form; oracle.c pred8x8_px is the same
// restatement, pinned to predict.c:741-883 by tests/golden/intra8x8_golden.npz.
template <int MODE>
__device__ __forceinline__ int pred8_dir( const int (&e)[36], int x, int y )
{
    if constexpr( MODE == 3 )   // DDL
    {
        const int z = x + y;
        return f2( e[16 + z], e[17 + z], e[16 + (z + 2 < 15 ? z + 2 : 15)] );
    }
    else if constexpr( MODE == 4 )   // DDR
    {
        const int c = x > y ? 15 + x - y : 15 - (y - x);
        return f2( e[c - 1], e[c], e[c + 1] );
    }
    else if constexpr( MODE == 5 )   // VR
    {
        const int z = 2 * x - y;
        if( z < 0 )
            return f2( e[15 + z], e[16 + z], e[17 + z] );
        if( !(z & 1) )
            return f1( e[15 + z / 2], e[16 + z / 2] );
        const int c = 15 + (z + 1) / 2;
        return f2( e[c - 1], e[c], e[c + 1] );
    }
    else if constexpr( MODE == 6 )   // HD
    {
        const int z = 2 * y - x;
        if( z < 0 )
            return f2( e[13 - z], e[14 - z], e[15 - z] );
        if( !(z & 1) )
            return f1( e[15 - z / 2], e[14 - z / 2] );
        const int c = 15 - (z + 1) / 2;
        return f2( e[c - 1], e[c], e[c + 1] );
    }
    else if constexpr( MODE == 7 )   // VL
    {
        const int c = 16 + x + (y >> 1);
        return (y & 1) ? f2( e[c], e[c + 1], e[c + 2] ) : f1( e[c], e[c + 1] );
    }
    else   // HU
    {
        const int z = x + 2 * y;
        if( z > 13 )
            return e[7];
        if( z == 13 )
            return f2( e[8], e[7], e[7] );
        const int c = 14 - (z >> 1);
        return (z & 1) ? f2( e[c], e[c - 1], e[c - 2] ) : f1( e[c], e[c - 1] );
    }
}

// cost of one 8x8 prediction given as pairs pr[y][x] = (p(x,y), p(x+4,y))
template <bool SATD>
__device__ __forceinline__ int cost8x8( const x264hip_short2 (&fe)[8][4], const x264hip_short2 (&pr)[8][4] )
{
    uint32_t s = 0;
    if constexpr( SATD )
    {
#pragma unroll
        for( int h = 0; h < 2; h++ )
        {
            x264hip_short2 d[4][4];
#pragma unroll
            for( int y = 0; y < 4; y++ )
#pragma unroll
                for( int x = 0; x < 4; x++ )
                    d[y][x] = fe[4 * h + y][x] - pr[4 * h + y][x];
            d[0][0] = sat_bias( d[0][0] );
            s = had_sad_pairs( d, s );
        }
        return (int)(s >> 1);   // satd_8x4 halves each band; every band sum is even
    }
    else
    {
#pragma unroll
        for( int y = 0; y < 8; y++ )
#pragma unroll
            for( int x = 0; x < 4; x++ )
                s = __builtin_amdgcn_sad_u16( __builtin_bit_cast( uint32_t, fe[y][x] ),
                                              __builtin_bit_cast( uint32_t, pr[y][x] ), s );
        return (int)s;
    }
}

template <int MODE, bool SATD>
__device__ __forceinline__ int dir_cost( const x264hip_short2 (&fe)[8][4], const int (&e)[36] )
{
    x264hip_short2 pr[8][4];
#pragma unroll
    for( int y = 0; y < 8; y++ )
#pragma unroll
        for( int x = 0; x < 4; x++ )
            pr[y][x] = mk2( pred8_dir<MODE>( e, x, y ), pred8_dir<MODE>( e, x + 4, y ) );
    return cost8x8<SATD>( fe, pr );
}

// --------------------------------------------------------------- lowres intra cost
// slicetype.c:716-746 for the 8x8 block at s: ((min cost + penalty) >> (BD-8)) + 4
template <int BD, bool SATD, bool ALL>
__device__ __forceinline__ int lowres_mb_cost( const typename PT<BD>::pixel *s, intptr_t stride, int penalty )
{
    // fenc as paired columns
    x264hip_short2 fe[8][4];
#pragma unroll
    for( int y = 0; y < 8; y++ )
    {
        uint32_t r[8 / PT<BD>::PPD];
        const uint32_t *rp = (const uint32_t *)(s + y * stride);
#pragma unroll
        for( int k = 0; k < 8 / PT<BD>::PPD; k++ )
            r[k] = rp[k];
#pragma unroll
        for( int x = 0; x < 4; x++ )
            fe[y][x] = pair_px<BD>( r, x );
    }
    // neighbours: t0..t15 of row -1, l0..l7 and lt of column -1
    int t[16], l[8];
    {
        const uint32_t *rp = (const uint32_t *)(s - stride);
#pragma unroll
        for( int k = 0; k < 16 / PT<BD>::PPD; k++ )
        {
            const uint32_t w = rp[k];
#pragma unroll
            for( int j = 0; j < PT<BD>::PPD; j++ )
                t[k * PT<BD>::PPD + j] = upix<BD>( w, j );
        }
    }
#pragma unroll
    for( int y = 0; y < 8; y++ )
        l[y] = s[y * stride - 1];
    const int lt = s[-stride - 1];

    // intra_mbcmp_x3_8x8c: DC, H, V of predict_8x8c (predict.c:221-281)
    int best;
    {
        const int s0 = t[0] + t[1] + t[2] + t[3], s1 = t[4] + t[5] + t[6] + t[7];
        const int s2 = l[0] + l[1] + l[2] + l[3], s3 = l[4] + l[5] + l[6] + l[7];
        const x264hip_short2 dtop = mk2( (s0 + s2 + 4) >> 3, (s1 + 2) >> 2 );
        const x264hip_short2 dbot = mk2( (s3 + 2) >> 2, (s1 + s3 + 4) >> 3 );
        x264hip_short2 pr[8][4];
#pragma unroll
        for( int y = 0; y < 8; y++ )
#pragma unroll
            for( int x = 0; x < 4; x++ )
                pr[y][x] = y < 4 ? dtop : dbot;
        best = cost8x8<SATD>( fe, pr );
#pragma unroll
        for( int y = 0; y < 8; y++ )
#pragma unroll
            for( int x = 0; x < 4; x++ )
                pr[y][x] = mk2( l[y], l[y] );
        best = min( best, cost8x8<SATD>( fe, pr ) );
#pragma unroll
        for( int y = 0; y < 8; y++ )
#pragma unroll
            for( int x = 0; x < 4; x++ )
                pr[y][x] = mk2( t[x], t[x + 4] );
        best = min( best, cost8x8<SATD>( fe, pr ) );
    }
    if constexpr( ALL )
    {
        // predict_8x8c_p (predict.c:282-308)
        {
            const int tm1 = lt;
            const int H = 1 * (t[4] - t[2]) + 2 * (t[5] - t[1]) + 3 * (t[6] - t[0]) + 4 * (t[7] - tm1);
            const int V = 1 * (l[4] - l[2]) + 2 * (l[5] - l[1]) + 3 * (l[6] - l[0]) + 4 * (l[7] - tm1);
            const int a = 16 * (l[7] + t[7]);
            const int b = (17 * H + 16) >> 5, c = (17 * V + 16) >> 5;
            const int i00 = a - 3 * b - 3 * c + 16;
            x264hip_short2 pr[8][4];
#pragma unroll
            for( int y = 0; y < 8; y++ )
#pragma unroll
                for( int x = 0; x < 4; x++ )
                    pr[y][x] = mk2( clip_pix<BD>( (i00 + b * x + c * y) >> 5 ),
                                    clip_pix<BD>( (i00 + b * (x + 4) + c * y) >> 5 ) );
            best = min( best, cost8x8<SATD>( fe, pr ) );
        }
        // predict_8x8_filter with every neighbour (predict.c:632-676)
        int e[36];
#pragma unroll
        for( int i = 0; i < 7; i++ )
            e[i] = 0;
        e[15] = f2( t[0], lt, l[0] );
        e[14] = f2( lt, l[0], l[1] );
#pragma unroll
        for( int y = 1; y < 7; y++ )
            e[14 - y] = f2( l[y - 1], l[y], l[y + 1] );
        e[6] = e[7] = (l[6] + 3 * l[7] + 2) >> 2;
        e[16] = f2( lt, t[0], t[1] );
#pragma unroll
        for( int x = 1; x < 15; x++ )
            e[16 + x] = f2( t[x - 1], t[x], t[x + 1] );
        e[31] = e[32] = (t[14] + 3 * t[15] + 2) >> 2;
        e[33] = e[34] = e[35] = 0;
        best = min( best, dir_cost<3, SATD>( fe, e ) );
        best = min( best, dir_cost<4, SATD>( fe, e ) );
        best = min( best, dir_cost<5, SATD>( fe, e ) );
        best = min( best, dir_cost<6, SATD>( fe, e ) );
        best = min( best, dir_cost<7, SATD>( fe, e ) );
        best = min( best, dir_cost<8, SATD>( fe, e ) );
    }
    return ((best + penalty) >> (BD - 8)) + 4;
}

// per-MB outputs; returns (row term, frame-score plain, frame-score aq) through refs
template <int BD, bool SATD, bool ALL>
__device__ __forceinline__ void lowres_mb( const typename PT<BD>::pixel *plane, intptr_t stride, intptr_t fstride,
                                           int mbx, int mby, int f, int mbw, int mbh, int penalty,
                                           const uint16_t *invq, uint16_t *cost, int &c_row, int &c_plain,
                                           int &c_aq )
{
    const typename PT<BD>::pixel *s = plane + f * fstride + (intptr_t)8 * mby * stride + 8 * mbx;
    const int icost = lowres_mb_cost<BD, SATD, ALL>( s, stride, penalty );
    const int mb = mbx + mby * mbw;
    const int64_t fm = (int64_t)f * mbw * mbh;
    cost[fm + mb] = (uint16_t)icost;              // i_intra_cost is uint16_t; the sums use the int
    const int aq = invq ? (icost * (int)invq[fm + mb] + 128) >> 8 : icost;
    c_row += aq;
    if( (mbx > 0 && mbx < mbw - 1 && mby > 0 && mby < mbh - 1) || mbw <= 2 || mbh <= 2 )
    {
        c_plain += icost;
        c_aq += aq;
    }
}

__device__ __forceinline__ int wave_sum( int v )
{
#pragma unroll
    for( int o = 32; o > 0; o >>= 1 )
        v += __shfl_xor( v, o );
    return v;
}

// default: grid (mb_height, n_frames), one block per MB row (blockDim = 64 * ceil(mbw/64),
// <= 256, looping for wider rows); the row sum is a plain store, the frame sums one
// atomic pair per row.
template <int BD, bool SATD, bool ALL>
__global__ __launch_bounds__( 256 ) void lowres_intra_row_kernel( const typename PT<BD>::pixel *plane,
                                                                   intptr_t stride, intptr_t fstride, int mbw,
                                                                   int mbh, int penalty, const uint16_t *invq,
                                                                   uint16_t *cost, int32_t *row_satd, int32_t *est )
{
    __shared__ int red[3][4];
    const int mby = blockIdx.x, f = blockIdx.y;
    int c_row = 0, c_plain = 0, c_aq = 0;
    for( int mbx = threadIdx.x; mbx < mbw; mbx += blockDim.x )
        lowres_mb<BD, SATD, ALL>( plane, stride, fstride, mbx, mby, f, mbw, mbh, penalty, invq, cost, c_row,
                                  c_plain, c_aq );
    c_row = wave_sum( c_row );
    c_plain = wave_sum( c_plain );
    c_aq = wave_sum( c_aq );
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if( (threadIdx.x & 63) == 0 )
    {
        red[0][w] = c_row;
        red[1][w] = c_plain;
        red[2][w] = c_aq;
    }
    __syncthreads();
    if( threadIdx.x == 0 )
    {
        int r = 0, p = 0, q = 0;
        for( int i = 0; i < nw; i++ )
        {
            r += red[0][i];
            p += red[1][i];
            q += red[2][i];
        }
        if( row_satd )
            row_satd[(int64_t)f * mbh + mby] = r;
        if( est && (p | q) )
        {
            atomicAdd( &est[2 * f], p );
            atomicAdd( &est[2 * f + 1], q );
        }
    }
}

template <int BD>
hipError_t launch_lowres_intra( const typename PT<BD>::pixel *plane, intptr_t stride, intptr_t fstride, int mbw,
                                int mbh, int nframes, int satd, int all_modes, int lambda, const uint16_t *invq,
                                uint16_t *cost, int32_t *row_satd, int32_t *est, hipStream_t st )
{
    if( mbw <= 0 || mbh <= 0 || nframes <= 0 )
        return hipSuccess;
    if( est )
    {
        hipError_t e = hipMemsetAsync( est, 0, sizeof(int32_t) * 2 * (size_t)nframes, st );
        if( e != hipSuccess )
            return e;
    }
    const int pen = 5 * lambda;
    const int bt = mbw >= 256 ? 256 : (mbw + 63) / 64 * 64;
#define L( S, A )                                                                                                    \
    do                                                                                                               \
    {                                                                                                                \
        hipLaunchKernelGGL( ( lowres_intra_row_kernel<BD, S, A> ), dim3( mbh, nframes ), dim3( bt ), 0, st,          \
                            plane, stride, fstride, mbw, mbh, pen, invq, cost, row_satd, est );                      \
    } while( 0 )
    if( satd && all_modes )
        L( true, true );
    else if( satd )
        L( true, false );
    else if( all_modes )
        L( false, true );
    else
        L( false, false );
#undef L
    return hipGetLastError();
}

// --------------------------------------------------------------- intra_*_x3 lists
// kinds (X264HIP_INTRA_*): 0 = 4x4, 1 = 8x8c, 2 = 8x16c, 3 = 16x16, 4 = 8x8 luma from edge[36]
__host__ __device__ constexpr int intra_w( int k ) { return k == 0 ? 4 : k == 3 ? 16 : 8; }
__host__ __device__ constexpr int intra_h( int k ) { return k == 0 ? 4 : k == 1 || k == 4 ? 8 : 16; }

// prediction of the 4x4 tile (tx, ty) for mode k (the x3 order of pixel.c:553-560:
// V,H,DC for 4x4 / 16x16 / 8x8; DC,H,V for chroma)
template <int BD, int KIND>
__device__ __forceinline__ void tile_pred( int k, const typename PT<BD>::pixel *d, intptr_t ds, int tx, int ty,
                                           int dc, int (&p)[4][4] )
{
    const bool chroma = KIND == 1 || KIND == 2;
    const int mv = chroma ? 2 : 0, mh = 1;
    if( k == mv )
    {
#pragma unroll
        for( int x = 0; x < 4; x++ )
        {
            const int v = KIND == 4 ? d[16 + 4 * tx + x] : d[4 * tx + x - ds];
#pragma unroll
            for( int y = 0; y < 4; y++ )
                p[y][x] = v;
        }
    }
    else if( k == mh )
    {
#pragma unroll
        for( int y = 0; y < 4; y++ )
        {
            const int v = KIND == 4 ? d[14 - 4 * ty - y] : d[(4 * ty + y) * ds - 1];
#pragma unroll
            for( int x = 0; x < 4; x++ )
                p[y][x] = v;
        }
    }
    else
    {
        int v = dc;
        if( chroma )
        {
            // predict_8x8c_dc / predict_8x16c_dc quadrant rule
            int st = 0, sl = 0;
#pragma unroll
            for( int i = 0; i < 4; i++ )
            {
                st += d[4 * tx + i - ds];
                sl += d[(4 * ty + i) * ds - 1];
            }
            v = tx == 0 && ty == 0 ? (st + sl + 4) >> 3 : tx == 1 && ty == 0 ? (st + 2) >> 2
              : tx == 0 ? (sl + 2) >> 2 : (st + sl + 4) >> 3;
        }
#pragma unroll
        for( int y = 0; y < 4; y++ )
#pragma unroll
            for( int x = 0; x < 4; x++ )
                p[y][x] = v;
    }
}

template <int BD, int KIND, int OP>
__global__ __launch_bounds__( 256 ) void intra_x3_kernel( const typename PT<BD>::pixel *fenc, intptr_t fs,
                                                          const typename PT<BD>::pixel *fdec, intptr_t ds,
                                                          const int64_t *fo, const int64_t *dof, int n,
                                                          int32_t *scores )
{
    using pixel = typename PT<BD>::pixel;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if( i >= n )
        return;
    constexpr int W = intra_w( KIND ), H = intra_h( KIND );
    const pixel *a = fenc + fo[i];
    const pixel *d = fdec + dof[i];
    int dc = 0;
    if constexpr( KIND == 4 )
    {
        int s = 8;
#pragma unroll
        for( int j = 0; j < 8; j++ )
            s += d[14 - j] + d[16 + j];
        dc = s >> 4;
    }
    else if constexpr( KIND == 0 || KIND == 3 )
    {
        int s = W;
        for( int j = 0; j < W; j++ )
            s += d[j - ds] + d[j * ds - 1];
        dc = s >> (W == 4 ? 3 : 5);
    }
#pragma unroll
    for( int k = 0; k < 3; k++ )
    {
        int total = 0;
        if constexpr( OP == 3 )   // sa8d 8x8 (KIND 4)
        {
            int m[8][8];
#pragma unroll
            for( int ty = 0; ty < 2; ty++ )
#pragma unroll
                for( int tx = 0; tx < 2; tx++ )
                {
                    int p[4][4];
                    tile_pred<BD, KIND>( k, d, ds, tx, ty, dc, p );
#pragma unroll
                    for( int y = 0; y < 4; y++ )
#pragma unroll
                        for( int x = 0; x < 4; x++ )
                            m[4 * ty + y][4 * tx + x] = (int)a[(4 * ty + y) * fs + 4 * tx + x] - p[y][x];
                }
#pragma unroll
            for( int sh = 1; sh < 8; sh <<= 1 )
#pragma unroll
                for( int y = 0; y < 8; y++ )
#pragma unroll
                    for( int x = 0; x < 8; x++ )
                        if( !(x & sh) )
                        {
                            const int u = m[y][x], v = m[y][x + sh];
                            m[y][x] = u + v;
                            m[y][x + sh] = u - v;
                        }
#pragma unroll
            for( int sh = 1; sh < 8; sh <<= 1 )
#pragma unroll
                for( int y = 0; y < 8; y++ )
#pragma unroll
                    for( int x = 0; x < 8; x++ )
                        if( !(y & sh) )
                        {
                            const int u = m[y][x], v = m[y + sh][x];
                            m[y][x] = u + v;
                            m[y + sh][x] = u - v;
                        }
#pragma unroll
            for( int y = 0; y < 8; y++ )
#pragma unroll
                for( int x = 0; x < 8; x++ )
                    total += abs( m[y][x] );
            total = (total + 2) >> 2;
        }
        else
        {
            for( int ty = 0; ty < H / 4; ty++ )
                for( int tx = 0; tx < W / 4; tx++ )
                {
                    int p[4][4];
                    tile_pred<BD, KIND>( k, d, ds, tx, ty, dc, p );
                    int m[4][4];
#pragma unroll
                    for( int y = 0; y < 4; y++ )
#pragma unroll
                        for( int x = 0; x < 4; x++ )
                            m[y][x] = (int)a[(4 * ty + y) * fs + 4 * tx + x] - p[y][x];
                    if constexpr( OP == 0 )
                    {
#pragma unroll
                        for( int y = 0; y < 4; y++ )
#pragma unroll
                            for( int x = 0; x < 4; x++ )
                                total += abs( m[y][x] );
                    }
                    else
                    {
                        int s = 0;
#pragma unroll
                        for( int y = 0; y < 4; y++ )
                        {
                            const int t0 = m[y][0] + m[y][1], t1 = m[y][0] - m[y][1];
                            const int t2 = m[y][2] + m[y][3], t3 = m[y][2] - m[y][3];
                            m[y][0] = t0 + t2; m[y][2] = t0 - t2; m[y][1] = t1 + t3; m[y][3] = t1 - t3;
                        }
#pragma unroll
                        for( int x = 0; x < 4; x++ )
                        {
                            const int t0 = m[0][x] + m[1][x], t1 = m[0][x] - m[1][x];
                            const int t2 = m[2][x] + m[3][x], t3 = m[2][x] - m[3][x];
                            s += abs( t0 + t2 ) + abs( t0 - t2 ) + abs( t1 + t3 ) + abs( t1 - t3 );
                        }
                        total += s >> 1;
                    }
                }
        }
        scores[3 * i + k] = total;
    }
}

template <int BD>
hipError_t launch_intra_x3( int kind, int op, const typename PT<BD>::pixel *fenc, intptr_t fs,
                            const typename PT<BD>::pixel *fdec, intptr_t ds, const int64_t *fo,
                            const int64_t *dof, int n, int32_t *scores, hipStream_t st )
{
    if( n <= 0 )
        return hipSuccess;
    const dim3 g( (n + 255) / 256 ), b( 256 );
#define L( K, O ) hipLaunchKernelGGL( ( intra_x3_kernel<BD, K, O> ), g, b, 0, st, fenc, fs, fdec, ds, fo, dof, n, scores )
    switch( kind * 4 + op )
    {
        case 0 * 4 + 0: L( 0, 0 ); break;
        case 0 * 4 + 2: L( 0, 2 ); break;
        case 1 * 4 + 0: L( 1, 0 ); break;
        case 1 * 4 + 2: L( 1, 2 ); break;
        case 2 * 4 + 0: L( 2, 0 ); break;
        case 2 * 4 + 2: L( 2, 2 ); break;
        case 3 * 4 + 0: L( 3, 0 ); break;
        case 3 * 4 + 2: L( 3, 2 ); break;
        case 4 * 4 + 0: L( 4, 0 ); break;
        case 4 * 4 + 3: L( 4, 3 ); break;
        default: return hipErrorInvalidValue;
    }
#undef L
    return hipGetLastError();
}

#define INST( BD )                                                                                                   \
    template hipError_t launch_lowres_intra<BD>( const PT<BD>::pixel *, intptr_t, intptr_t, int, int, int, int, int,  \
                                                 int, const uint16_t *, uint16_t *, int32_t *, int32_t *,             \
                                                 hipStream_t );                                                       \
    template hipError_t launch_intra_x3<BD>( int, int, const PT<BD>::pixel *, intptr_t, const PT<BD>::pixel *,      \
                                             intptr_t, const int64_t *, const int64_t *, int, int32_t *, hipStream_t );
INST( 8 )
INST( 10 )
#undef INST

} // namespace x264hip
