// The lookahead's lowres motion search on gfx950: slicetype_mb_cost's inter leg
// for P frames (reference encoder/slicetype.c:514-713, 758-791 with b == p1, one
// list, no weights, a fresh search) with the x264_me_search_ref /
// refine_subpel paths the lookahead runs (encoder/me.c:182-420, 774-790,
// 865-992: me = DIA or HEX, lookahead subme 2 or 4, no chroma ME).
//
// Dependencies: every block takes its MV predictors from blocks the reverse
// raster scan of slicetype_slice_cost (slicetype.c:818-833) has already
// searched -- right (x+1, y) and the row below (x-1..x+1, y+1) -- so the
// bit-exact schedule is a wavefront: block (x, y) runs at step
// t = (W-1-x) + 2(H-1-y), after all four of its predictors.  One workgroup
// walks one frame pair's W + 2H - 2 steps with a barrier between steps, one
// lane per block row; the four most recent MVs of every row sit in an LDS
// ring (the predictors of a step are at most three steps old).  Each lane
// runs the block's whole search (HEX / DIA, the hpel and qpel refinement) with
// the 8x8 SAD / SATD on fenc rows held in registers and get_ref rebuilt from
// the four lowres planes; the frame pairs of a batch run in parallel.
#include "hipcommon.h"

namespace x264hip {

__constant__ uint8_t c_lr_ref0[16] = { 0, 1, 1, 1, 0, 1, 1, 1, 2, 3, 3, 3, 0, 1, 1, 1 };   // x264_hpel_ref0
__constant__ uint8_t c_lr_ref1[16] = { 0, 0, 1, 0, 2, 2, 3, 2, 2, 2, 3, 2, 2, 2, 3, 2 };   // x264_hpel_ref1
__constant__ int8_t c_hex2[8][2] = { { -1, -2 }, { -2, 0 }, { -1, 2 }, { 1, 2 }, { 2, 0 }, { 1, -2 }, { -1, -2 }, { -2, 0 } };
__constant__ uint8_t c_mod6m1[8] = { 5, 0, 1, 2, 3, 4, 5, 0 };
__constant__ int8_t c_square1[9][2] = { { 0, 0 }, { 0, -1 }, { 0, 1 }, { -1, 0 }, { 1, 0 },
                                        { -1, -1 }, { -1, 1 }, { 1, -1 }, { 1, 1 } };

constexpr int LR_COST_MAX = 1 << 28;

__device__ __forceinline__ uint32_t lr_pack( int a, int b ) { return (uint32_t)(uint16_t)a | ((uint32_t)(uint16_t)b << 16); }
__device__ __forceinline__ int lr_clip3( int v, int lo, int hi ) { return v < lo ? lo : v > hi ? hi : v; }
__device__ __forceinline__ int lr_median( int a, int b, int c )
{
    const int mn = min( a, b ), mx = max( a, b );
    return c < mn ? mn : c > mx ? mx : c;
}

template <int BD> struct LrCtx
{
    using pixel = typename PT<BD>::pixel;
    static constexpr int NDW = 8 / PT<BD>::PPD;
    uint32_t fe[8][NDW];                    // fenc block rows (packed pixels)
    const pixel *p0, *p1, *p2, *p3;         // reference F, H, V, C at the block
    intptr_t stride;
    const uint16_t *cmx, *cmy;              // p_cost_mvx / p_cost_mvy (cost_mv - mvp)
    int satd;
    int smin0, smax0, smin1, smax1;         // h->mb.mv_min_spel / mv_max_spel
    int fmin0, fmax0, fmin1, fmax1;         // mv_limit_fpel

    // fpelcmp (SAD) at a full-pel offset of the F plane
    __device__ __forceinline__ int fpel( int mx, int my ) const
    {
        const pixel *r = p0 + (intptr_t)my * stride + mx;
        uint32_t acc = 0;
#pragma unroll
        for( int y = 0; y < 8; y++ )
        {
            uint32_t w[NDW];
            load_row_u<NDW>( r + (intptr_t)y * stride, w );
#pragma unroll
            for( int k = 0; k < NDW; k++ )
                acc = sadp<BD>( fe[y][k], w[k], acc );
        }
        return (int)acc;
    }

    // get_ref (mc.c:221-249) at a quarter-pel mv, then SAD or SATD 8x8
    __device__ __forceinline__ int qpel( int mx, int my, bool use_satd ) const
    {
        const int idx = ((my & 3) << 2) + (mx & 3);
        const intptr_t off = (intptr_t)(my >> 2) * stride + (mx >> 2);
        const int i0 = c_lr_ref0[idx], i1 = c_lr_ref1[idx];
        const pixel *s1 = (i0 == 0 ? p0 : i0 == 1 ? p1 : i0 == 2 ? p2 : p3) + off + ((my & 3) == 3) * stride;
        const pixel *s2 = (idx & 5) ? (i1 == 0 ? p0 : i1 == 1 ? p1 : i1 == 2 ? p2 : p3) + off + ((mx & 3) == 3) : s1;
        uint32_t r[8][NDW];
#pragma unroll
        for( int y = 0; y < 8; y++ )
        {
            uint32_t a[NDW], b[NDW];
            load_row_u<NDW>( s1 + (intptr_t)y * stride, a );
            load_row_u<NDW>( s2 + (intptr_t)y * stride, b );
#pragma unroll
            for( int k = 0; k < NDW; k++ )
                r[y][k] = avg_round<BD>( a[k], b[k] );
        }
        uint32_t acc = 0;
        if( use_satd )
        {
#pragma unroll
            for( int band = 0; band < 2; band++ )
            {
                uint32_t fa[4][NDW], ra[4][NDW];
#pragma unroll
                for( int y = 0; y < 4; y++ )
#pragma unroll
                    for( int k = 0; k < NDW; k++ )
                    {
                        fa[y][k] = fe[4 * band + y][k];
                        ra[y][k] = r[4 * band + y][k];
                    }
                acc += satd8x4_packed<BD>( fa, ra );
            }
            return (int)(acc >> 1);
        }
#pragma unroll
        for( int y = 0; y < 8; y++ )
#pragma unroll
            for( int k = 0; k < NDW; k++ )
                acc = sadp<BD>( fe[y][k], r[y][k], acc );
        return (int)acc;
    }

    __device__ __forceinline__ int bits_mvd( int mx, int my ) const { return cmx[mx * 4] + cmy[my * 4]; }
    __device__ __forceinline__ bool in_range( int mx, int my ) const
    {
        return mx >= fmin0 && mx <= fmax0 && my >= fmin1 && my <= fmax1;
    }
};

// x264_me_search_ref (me.c:182-420, 774-790) then refine_subpel (me.c:912-992)
template <int BD>
__device__ void lr_me_search( const LrCtx<BD> &m, int mvpx, int mvpy, const int (&mvc)[4][2], int i_mvc,
                              int me_method, int subme, int me_range, int &omvx, int &omvy, int &ocost )
{
    int bmx, bmy, bcost = LR_COST_MAX, bpred_cost = LR_COST_MAX;
    uint32_t pmv, bpred_mv = 0;
    int tmp[6][2];
#define LR_COST_MV( mx, my )                                                                                  \
    do                                                                                                        \
    {                                                                                                         \
        const int c_ = m.fpel( mx, my ) + m.bits_mvd( mx, my );                                               \
        if( c_ < bcost )                                                                                      \
        {                                                                                                     \
            bcost = c_;                                                                                       \
            bmx = (mx);                                                                                       \
            bmy = (my);                                                                                       \
        }                                                                                                     \
    } while( 0 )
    if( subme >= 3 )
    {
        int bpx = lr_clip3( mvpx, 4 * m.fmin0, 4 * m.fmax0 ), bpy = lr_clip3( mvpy, 4 * m.fmin1, 4 * m.fmax1 );
        pmv = lr_pack( bpx, bpy );
        bpred_cost = m.qpel( bpx, bpy, false ) + m.cmx[bpx] + m.cmy[bpy];            // COST_MV_HPEL
        const int pmv_cost = bpred_cost;
        int valid = 0;
        for( int i = 0; i < i_mvc; i++ )                                              // x264_predictor_clip
        {
            const uint32_t v = lr_pack( mvc[i][0], mvc[i][1] );
            if( !v || v == pmv )
                continue;
            tmp[2 + valid][0] = lr_clip3( mvc[i][0], 4 * m.fmin0, 4 * m.fmax0 );
            tmp[2 + valid][1] = lr_clip3( mvc[i][1], 4 * m.fmin1, 4 * m.fmax1 );
            valid++;
        }
        if( valid > 0 )
        {
            tmp[1][0] = bpx;
            tmp[1][1] = bpy;
            bpred_cost <<= 4;
            for( int i = 1; i <= valid; i++ )
            {
                const int mx = tmp[i + 1][0], my = tmp[i + 1][1];
                const int c = m.qpel( mx, my, false ) + m.cmx[mx] + m.cmy[my];
                if( (c << 4) + i < bpred_cost )
                    bpred_cost = (c << 4) + i;
            }
            bpx = tmp[(bpred_cost & 15) + 1][0];
            bpy = tmp[(bpred_cost & 15) + 1][1];
            bpred_cost >>= 4;
        }
        bmx = (bpx + 2) >> 2;
        bmy = (bpy + 2) >> 2;
        bpred_mv = lr_pack( bpx, bpy );
        if( bpred_mv & 0x00030003u )
            LR_COST_MV( bmx, bmy );
        else
            bcost = bpred_cost;
        if( pmv )
        {
            if( bmx | bmy )
                LR_COST_MV( 0, 0 );
        }
        else if( pmv_cost < bcost )
        {
            bcost = pmv_cost;
            bmx = bmy = 0;
        }
    }
    else
    {
        bmx = lr_clip3( (mvpx + 2) >> 2, m.fmin0, m.fmax0 );
        bmy = lr_clip3( (mvpy + 2) >> 2, m.fmin1, m.fmax1 );
        pmv = lr_pack( bmx, bmy );
        bcost = m.fpel( bmx, bmy );
        int valid = 0;
        for( int i = 0; i < i_mvc; i++ )                                              // x264_predictor_roundclip
        {
            const int mx = (mvc[i][0] + 2) >> 2, my = (mvc[i][1] + 2) >> 2;
            const uint32_t v = lr_pack( mx, my );
            if( !v || v == pmv )
                continue;
            tmp[2 + valid][0] = lr_clip3( mx, m.fmin0, m.fmax0 );
            tmp[2 + valid][1] = lr_clip3( my, m.fmin1, m.fmax1 );
            valid++;
        }
        if( valid > 0 )
        {
            tmp[1][0] = bmx;
            tmp[1][1] = bmy;
            bcost <<= 4;
            for( int i = 1; i <= valid; i++ )
            {
                const int mx = tmp[i + 1][0], my = tmp[i + 1][1];
                const int c = m.fpel( mx, my ) + m.bits_mvd( mx, my );
                if( (c << 4) + i < bcost )
                    bcost = (c << 4) + i;
            }
            bmx = tmp[(bcost & 15) + 1][0];
            bmy = tmp[(bcost & 15) + 1][1];
            bcost >>= 4;
        }
        if( pmv )
            LR_COST_MV( 0, 0 );
    }

    int costs[8];
    if( me_method == 0 )
    {
        // diamond search, radius 1 (me.c:322-342)
        bcost <<= 4;
        int i = me_range;
        do
        {
            costs[0] = m.fpel( bmx, bmy - 1 ) + m.bits_mvd( bmx, bmy - 1 );
            costs[1] = m.fpel( bmx, bmy + 1 ) + m.bits_mvd( bmx, bmy + 1 );
            costs[2] = m.fpel( bmx - 1, bmy ) + m.bits_mvd( bmx - 1, bmy );
            costs[3] = m.fpel( bmx + 1, bmy ) + m.bits_mvd( bmx + 1, bmy );
            bcost = min( bcost, (costs[0] << 4) + 1 );
            bcost = min( bcost, (costs[1] << 4) + 3 );
            bcost = min( bcost, (costs[2] << 4) + 4 );
            bcost = min( bcost, (costs[3] << 4) + 12 );
            if( !(bcost & 15) )
                break;
            bmx -= (int32_t)((uint32_t)bcost << 28) >> 30;
            bmy -= (int32_t)((uint32_t)bcost << 30) >> 30;
            bcost &= ~15;
        } while( --i && m.in_range( bmx, bmy ) );
        bcost >>= 4;
    }
    else
    {
        // hexagon search, radius 2 (me.c:344-405), then the square refine (me.c:406-420)
#define LR_X3( a, b, c, d, e, f, o )                                                                          \
    do                                                                                                        \
    {                                                                                                         \
        (o)[0] = m.fpel( bmx + (a), bmy + (b) ) + m.bits_mvd( bmx + (a), bmy + (b) );                        \
        (o)[1] = m.fpel( bmx + (c), bmy + (d) ) + m.bits_mvd( bmx + (c), bmy + (d) );                        \
        (o)[2] = m.fpel( bmx + (e), bmy + (f) ) + m.bits_mvd( bmx + (e), bmy + (f) );                        \
    } while( 0 )
        LR_X3( -2, 0, -1, 2, 1, 2, costs );
        LR_X3( 2, 0, 1, -2, -1, -2, costs + 4 );
        bcost <<= 3;
        bcost = min( bcost, (costs[0] << 3) + 2 );
        bcost = min( bcost, (costs[1] << 3) + 3 );
        bcost = min( bcost, (costs[2] << 3) + 4 );
        bcost = min( bcost, (costs[4] << 3) + 5 );
        bcost = min( bcost, (costs[5] << 3) + 6 );
        bcost = min( bcost, (costs[6] << 3) + 7 );
        if( bcost & 7 )
        {
            int dir = (bcost & 7) - 2;
            bmx += c_hex2[dir + 1][0];
            bmy += c_hex2[dir + 1][1];
            for( int i = (me_range >> 1) - 1; i > 0 && m.in_range( bmx, bmy ); i-- )
            {
                LR_X3( c_hex2[dir][0], c_hex2[dir][1], c_hex2[dir + 1][0], c_hex2[dir + 1][1], c_hex2[dir + 2][0],
                       c_hex2[dir + 2][1], costs );
                bcost &= ~7;
                bcost = min( bcost, (costs[0] << 3) + 1 );
                bcost = min( bcost, (costs[1] << 3) + 2 );
                bcost = min( bcost, (costs[2] << 3) + 3 );
                if( !(bcost & 7) )
                    break;
                dir += (bcost & 7) - 2;
                dir = c_mod6m1[dir + 1];
                bmx += c_hex2[dir + 1][0];
                bmy += c_hex2[dir + 1][1];
            }
        }
        bcost >>= 3;
#undef LR_X3
        bcost <<= 4;
#pragma unroll
        for( int k = 1; k <= 8; k++ )
        {
            const int dx = c_square1[k][0], dy = c_square1[k][1];
            const int c = m.fpel( bmx + dx, bmy + dy ) + m.bits_mvd( bmx + dx, bmy + dy );
            bcost = min( bcost, (c << 4) + k );
        }
        bmx += c_square1[bcost & 15][0];
        bmy += c_square1[bcost & 15][1];
        bcost >>= 4;
    }
#undef LR_COST_MV

    // -> qpel mv (me.c:774-790)
    int mx, my, c;
    if( subme < 3 )
    {
        c = bcost;
        if( lr_pack( bmx, bmy ) == pmv )
            c += m.bits_mvd( bmx, bmy );
        mx = 4 * bmx;
        my = 4 * bmy;
    }
    else if( bpred_cost < bcost )
    {
        mx = (int16_t)(bpred_mv & 0xffff);
        my = (int16_t)(bpred_mv >> 16);
        c = bpred_cost;
    }
    else
    {
        mx = 4 * bmx;
        my = 4 * bmy;
        c = bcost;
    }

    // refine_subpel( hpel, qpel, NULL, 0 ): subpel_iterations[subme][2..3] (me.c:38-50)
    const int hpel = subme >= 2 ? 1 : 0, qpel = subme >= 4 ? 1 : 0;
    bmx = mx;
    bmy = my;
    bcost = c;
    if( hpel )
    {
        if( subme < 3 )
        {
            const int px = lr_clip3( mvpx, m.smin0 + 2, m.smax0 - 2 ), py = lr_clip3( mvpy, m.smin1 + 2, m.smax1 - 2 );
            if( (px - bmx) | (py - bmy) )
            {
                const int cc = m.qpel( px, py, false ) + m.cmx[px] + m.cmy[py];
                if( cc < bcost )
                {
                    bcost = cc;
                    bmx = px;
                    bmy = py;
                }
            }
        }
        bcost <<= 6;
        for( int i = hpel; i > 0; i-- )
        {
            const int omx = bmx, omy = bmy;
            costs[0] = m.qpel( omx, omy - 2, false ) + m.cmx[omx] + m.cmy[omy - 2];
            costs[1] = m.qpel( omx, omy + 2, false ) + m.cmx[omx] + m.cmy[omy + 2];
            costs[2] = m.qpel( omx - 2, omy, false ) + m.cmx[omx - 2] + m.cmy[omy];
            costs[3] = m.qpel( omx + 2, omy, false ) + m.cmx[omx + 2] + m.cmy[omy];
            bcost = min( bcost, (costs[0] << 6) + 2 );
            bcost = min( bcost, (costs[1] << 6) + 6 );
            bcost = min( bcost, (costs[2] << 6) + 16 );
            bcost = min( bcost, (costs[3] << 6) + 48 );
            if( !(bcost & 63) )
                break;
            bmx -= (int32_t)((uint32_t)bcost << 26) >> 29;
            bmy -= (int32_t)((uint32_t)bcost << 29) >> 29;
            bcost &= ~63;
        }
        bcost >>= 6;
    }
    if( m.satd )
        bcost = m.qpel( bmx, bmy, true ) + m.cmx[bmx] + m.cmy[bmy];                  // COST_MV_SATD( bmx, bmy, -1 )
    int bdir = -1;
    for( int i = qpel; i > 0; i-- )
    {
        if( bmy <= m.smin1 || bmy >= m.smax1 || bmx <= m.smin0 || bmx >= m.smax0 )
            break;
        const int odir = bdir;
        const int omx = bmx, omy = bmy;
#pragma unroll
        for( int dir = 0; dir < 4; dir++ )
        {
            if( (dir ^ 1) == odir )
                continue;
            const int qx = omx + (dir == 2 ? -1 : dir == 3 ? 1 : 0), qy = omy + (dir == 0 ? -1 : dir == 1 ? 1 : 0);
            const int cc = m.qpel( qx, qy, m.satd ) + m.cmx[qx] + m.cmy[qy];
            if( cc < bcost )
            {
                bcost = cc;
                bmx = qx;
                bmy = qy;
                bdir = dir;
            }
        }
        if( bmx == omx && bmy == omy )
            break;
    }
    omvx = bmx;
    omvy = bmy;
    ocost = bcost;
}

template <int BD>
__global__ __launch_bounds__( 256 ) void lowres_inter_kernel(
    const typename PT<BD>::pixel *__restrict__ fenc, intptr_t ffs, const typename PT<BD>::pixel *r0,
    const typename PT<BD>::pixel *r1, const typename PT<BD>::pixel *r2, const typename PT<BD>::pixel *r3,
    intptr_t stride, intptr_t rfs, int mbw, int mbh, int me_method, int subme, int satd, int me_range, int mv_range,
    int lambda, const uint16_t *__restrict__ cost_mv, const uint16_t *__restrict__ intra_cost,
    const uint16_t *__restrict__ invq, int16_t *__restrict__ mvs, int32_t *__restrict__ mv_costs,
    uint16_t *__restrict__ lcosts, int32_t *__restrict__ row_satd, int32_t *__restrict__ est )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int NDW = LrCtx<BD>::NDW;
    extern __shared__ int lr_smem[];
    int *ring = lr_smem;                         // [mbh][4] packed MVs of the row's 4 latest blocks
    int *rowacc = lr_smem + 4 * mbh;             // [mbh] AQ-scaled row sums
    int *eacc = rowacc + mbh;                    // cost_est, cost_est_aq, intra_mbs
    const int f = blockIdx.x;
    const int nmb = mbw * mbh;
    fenc += (intptr_t)f * ffs;
    r0 += (intptr_t)f * rfs;
    r1 += (intptr_t)f * rfs;
    r2 += (intptr_t)f * rfs;
    r3 += (intptr_t)f * rfs;
    intra_cost += (intptr_t)f * nmb;
    if( invq )
        invq += (intptr_t)f * nmb;
    mvs += 2 * (intptr_t)f * nmb;
    mv_costs += (intptr_t)f * nmb;
    lcosts += (intptr_t)f * nmb;
    for( int i = threadIdx.x; i < mbh; i += blockDim.x )
        rowacc[i] = 0;
    if( threadIdx.x < 3 )
        eacc[threadIdx.x] = 0;
    int e0 = 0, e1 = 0, e2 = 0;
    const int mvr = 2 * mv_range;
    __syncthreads();
    const int steps = (mbw - 1) + 2 * (mbh - 1) + 1;
    for( int t = 0; t < steps; t++ )
    {
        for( int y = threadIdx.x; y < mbh; y += blockDim.x )
        {
            const int x = mbw - 1 - (t - 2 * (mbh - 1 - y));
            if( x < 0 || x >= mbw )
                continue;
            const int mb = x + y * mbw;
            const intptr_t off = 8 * (intptr_t)x + 8 * (intptr_t)y * stride;
            LrCtx<BD> m;
            const pixel *fb = fenc + off;
#pragma unroll
            for( int r = 0; r < 8; r++ )
            {
                const uint32_t *row = (const uint32_t *)(fb + (intptr_t)r * stride);
#pragma unroll
                for( int k = 0; k < NDW; k++ )
                    m.fe[r][k] = row[k];
            }
            m.p0 = r0 + off;
            m.p1 = r1 + off;
            m.p2 = r2 + off;
            m.p3 = r3 + off;
            m.stride = stride;
            m.satd = satd;
            m.smin0 = max( 4 * (-8 * x - 12), -mvr );
            m.smax0 = min( 4 * (8 * (mbw - x - 1) + 12), mvr - 1 );
            m.smin1 = max( 4 * (-8 * y - 12), -mvr );
            m.smax1 = min( 4 * (8 * (mbh - y - 1) + 12), mvr - 1 );
            m.fmin0 = m.smin0 >> 2;
            m.fmax0 = m.smax0 >> 2;
            m.fmin1 = m.smin1 >> 2;
            m.fmax1 = m.smax1 >> 2;
            // reverse-order MV prediction (slicetype.c:654-672)
            int mvc[4][2] = { { 0, 0 }, { 0, 0 }, { 0, 0 }, { 0, 0 } };
            int i_mvc = 0;
            auto add = [&]( int v ) {
                mvc[i_mvc][0] = (int16_t)(v & 0xffff);
                mvc[i_mvc][1] = (int16_t)((uint32_t)v >> 16);
                i_mvc++;
            };
            if( x < mbw - 1 )
                add( ring[4 * y + ((x + 1) & 3)] );
            if( y < mbh - 1 )
            {
                add( ring[4 * (y + 1) + (x & 3)] );
                if( x > 0 )
                    add( ring[4 * (y + 1) + ((x - 1) & 3)] );
                if( x < mbw - 1 )
                    add( ring[4 * (y + 1) + ((x + 1) & 3)] );
            }
            int mvpx, mvpy;
            if( i_mvc <= 1 )
            {
                mvpx = mvc[0][0];
                mvpy = mvc[0][1];
            }
            else
            {
                mvpx = lr_median( mvc[0][0], mvc[1][0], mvc[2][0] );
                mvpy = lr_median( mvc[0][1], mvc[1][1], mvc[2][1] );
            }
            m.cmx = cost_mv - mvpx;
            m.cmy = cost_mv - mvpy;
            int mvx = 0, mvy = 0, cost = 0;
            bool skip = false;
            if( !mvpx && !mvpy )
            {
                // fast skip of near-zero residual blocks (slicetype.c:677-686)
                cost = m.qpel( 0, 0, satd );
                skip = cost < 64;
            }
            if( !skip )
            {
                lr_me_search<BD>( m, mvpx, mvpy, mvc, i_mvc, me_method, subme, me_range, mvx, mvy, cost );
                cost -= cost_mv[0];
                if( mvx | mvy )
                    cost += 5 * lambda;
            }
            ring[4 * y + (x & 3)] = (int)lr_pack( mvx, mvy );
            mvs[2 * mb] = (int16_t)mvx;
            mvs[2 * mb + 1] = (int16_t)mvy;
            mv_costs[mb] = cost;
            // slicetype.c:758-790
            int bcost = (cost >> (BD - 8)) + 4, list_used = 1;
            const bool fsm = (x > 0 && x < mbw - 1 && y > 0 && y < mbh - 1) || mbw <= 2 || mbh <= 2;
            const int icost = intra_cost[mb];
            const bool b_intra = icost < bcost;
            if( b_intra )
            {
                bcost = icost;
                list_used = 0;
            }
            const int aq = invq ? (bcost * invq[mb] + 128) >> 8 : bcost;
            rowacc[y] += aq;
            if( fsm )
            {
                e0 += bcost;
                e1 += aq;
                e2 += b_intra;
            }
            lcosts[mb] = (uint16_t)(min( bcost, 16383 ) + (list_used << 14));
        }
        __syncthreads();
    }
    if( e0 | e1 | e2 )
    {
        atomicAdd( &eacc[0], e0 );
        atomicAdd( &eacc[1], e1 );
        atomicAdd( &eacc[2], e2 );
    }
    __syncthreads();
    if( row_satd )
        for( int i = threadIdx.x; i < mbh; i += blockDim.x )
            row_satd[(intptr_t)f * mbh + i] = rowacc[i];
    if( est && threadIdx.x < 3 )
        est[3 * f + threadIdx.x] = eacc[threadIdx.x];
}

template <int BD>
hipError_t launch_lowres_inter( const typename PT<BD>::pixel *fenc, intptr_t ffs,
                                const typename PT<BD>::pixel *const ref[4], intptr_t stride, intptr_t rfs, int mbw,
                                int mbh, int npairs, int me_method, int subme, int satd, int me_range, int mv_range,
                                int lambda, const uint16_t *cost_mv, const uint16_t *intra_cost,
                                const uint16_t *invq, int16_t *mvs, int32_t *mv_costs, uint16_t *lowres_costs,
                                int32_t *row_satd, int32_t *est, hipStream_t stream )
{
    if( npairs <= 0 || mbw <= 0 || mbh <= 0 )
        return hipSuccess;
    const int threads = min( 256, (mbh + 63) / 64 * 64 );
    const size_t lds = (size_t)(5 * mbh + 3) * sizeof( int );
    hipLaunchKernelGGL( lowres_inter_kernel<BD>, dim3( npairs ), dim3( threads ), lds, stream, fenc, ffs, ref[0],
                        ref[1], ref[2], ref[3], stride, rfs, mbw, mbh, me_method, subme, satd, me_range, mv_range,
                        lambda, cost_mv, intra_cost, invq, mvs, mv_costs, lowres_costs, row_satd, est );
    return hipGetLastError();
}

#define INST( BD )                                                                                              \
    template hipError_t launch_lowres_inter<BD>( const PT<BD>::pixel *, intptr_t, const PT<BD>::pixel *const[4], \
                                                 intptr_t, intptr_t, int, int, int, int, int, int, int, int, int, \
                                                 const uint16_t *, const uint16_t *, const uint16_t *, int16_t *, \
                                                 int32_t *, uint16_t *, int32_t *, int32_t *, hipStream_t );
INST( 8 )
INST( 10 )
#undef INST

} // namespace x264hip
