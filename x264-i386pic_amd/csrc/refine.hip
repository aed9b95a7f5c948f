// Full-resolution subpel refinement: refine_subpel (reference encoder/me.c:865-992) for a
// batch of partitions, the decision x264_me_search_ref runs after its integer search
// (me.c:791-797, hpel / qpel iterations of subpel_iterations[subme][2..3], me.c:38-50) or
// x264_me_refine_qpel runs on a winner (me.c:801-810, [0..1]).
//
// One 32-lane segment per partition, two partitions per wave: four groups of eight lanes, a
// lane per 8x4 tile of the partition (16x16: eight tiles; 16x8 / 8x16: four; 8x8: two).
// A step that scores four candidates (the hpel diamond of fpelcmp_x4, the qpel diamond of
// COST_MV_SATD) gives group g candidate g; a one-candidate step (the predictor's subpel
// component, the SATD re-score of the hpel winner) runs the same candidate in every group.
// Each lane rebuilds get_ref (mc.c:221-249: the plane pair of x264_hpel_ref0/1 and the
// rounding average) for its tile and scores it with SAD or the packed 8x4 SATD
// (satd_8x4, pixel.c:290-309, summed over tiles as PIXEL_SATD_C does); the group's tiles
// meet through DPP adds and every lane of the segment reads the four candidate costs and
// takes the reference's decisions itself (the packed bcost << 6 / << 4 codes, COPY*_IF_LT's
// strict <, the odir skip), so the segment's lanes stay in step without LDS.  Luma only:
// the chroma ME of b_chroma_me (me.c:833-861) is outside the hot path, as are the
// multi-reference early exit (p_halfpel_thresh = NULL) and weighted references.
#include "hipcommon.h"

namespace x264hip {

constexpr uint8_t c_ref0[16] = { 0, 1, 1, 1, 0, 1, 1, 1, 2, 3, 3, 3, 0, 1, 1, 1 };   // x264_hpel_ref0
constexpr uint8_t c_ref1[16] = { 0, 0, 1, 0, 2, 2, 3, 2, 2, 2, 3, 2, 2, 2, 3, 2 };   // x264_hpel_ref1

// subpel_iterations (me.c:38-50): { refine_hpel, refine_qpel, me_hpel, me_qpel }
static const uint8_t k_subpel_iterations[12][4] = { { 0, 0, 0, 0 }, { 1, 1, 0, 0 }, { 0, 1, 1, 0 }, { 0, 2, 1, 0 },
                                                    { 0, 2, 1, 1 }, { 0, 2, 1, 2 }, { 0, 0, 2, 2 }, { 0, 0, 2, 2 },
                                                    { 0, 0, 4, 10 }, { 0, 0, 4, 10 }, { 0, 0, 4, 10 },
                                                    { 0, 0, 4, 10 } };

// the lane's 8x4 tile of get_ref( mvx, mvy ) scored against its fenc tile: SAD, or the sum of
// |coef| of the tile's two 4x4 Hadamards (even; halved by the caller)
template <int BD, bool SATD>
__device__ __forceinline__ uint32_t tile_cost( const uint32_t (&fa)[4][8 / PT<BD>::PPD],
                                               const typename PT<BD>::pixel *q0, const typename PT<BD>::pixel *q1,
                                               const typename PT<BD>::pixel *q2, const typename PT<BD>::pixel *q3,
                                               intptr_t rs, int mvx, int mvy )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int HDW = 8 / PT<BD>::PPD;
    const int idx = ((mvy & 3) << 2) + (mvx & 3);
    const intptr_t off = (intptr_t)(mvy >> 2) * rs + (mvx >> 2);
    constexpr uint32_t k0 = pack_fields( c_ref0, 2 ), k1 = pack_fields( c_ref1, 2 );
    const int i0 = field( k0, 2, idx ), i1 = field( k1, 2, idx );
    // (four separate pointers, not an array: a select over an array's elements was folded into
    // an indexed load, which put the array in scratch memory)
    const pixel *s1 = (i0 == 0 ? q0 : i0 == 1 ? q1 : i0 == 2 ? q2 : q3) + off + ((mvy & 3) == 3) * rs;
    const pixel *s2 = (i1 == 0 ? q0 : i1 == 1 ? q1 : i1 == 2 ? q2 : q3) + off + ((mvx & 3) == 3);
    // rows as dword-aligned loads realigned with v_alignbyte: the address path takes a
    // byte-misaligned 8-byte lane load at ~2x the cost of an aligned 12-byte one
    // (profiles/r01d_ta_probe.txt), and it binds this kernel (TA busy ~100 %, r04d)
    uint32_t r1[4][HDW];
#pragma unroll
    for( int y = 0; y < 4; y++ )
        load_al_pad<HDW>( s1 + y * rs, r1[y] );
    if( idx & 5 )                           // two planes: the rounding average (one plane: avg( a, a ) = a)
    {
        uint32_t r2[4][HDW];
#pragma unroll
        for( int y = 0; y < 4; y++ )
            load_al_pad<HDW>( s2 + y * rs, r2[y] );
#pragma unroll
        for( int y = 0; y < 4; y++ )
#pragma unroll
            for( int k = 0; k < HDW; k++ )
                r1[y][k] = avg_round<BD>( r1[y][k], r2[y][k] );
    }
    if constexpr( SATD )
        return satd8x4_packed<BD>( fa, r1 );
    else
    {
        uint32_t acc = 0;
#pragma unroll
        for( int y = 0; y < 4; y++ )
#pragma unroll
            for( int k = 0; k < HDW; k++ )
                acc = sadp<BD>( fa[y][k], r1[y][k], acc );
        return acc;
    }
}

// the eight tiles of each group summed into the group's first lane (quad sums by quad_perm,
// then row_ror:12 brings lane 8k+4's quad sum to lane 8k)
__device__ __forceinline__ uint32_t group_sum( uint32_t v )
{
    v += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)v, 0xB1, 0xF, 0xF, false );
    v += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)v, 0x4E, 0xF, 0xF, false );
    v += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)v, 0x12C, 0xF, 0xF, false );
    return v;
}

template <int BD, int IPIX, bool FSATD>
__global__ __launch_bounds__( 256 ) void me_refine_subpel_kernel(
    const typename PT<BD>::pixel *__restrict__ fenc, intptr_t fs, intptr_t ffs, const typename PT<BD>::pixel *p0,
    const typename PT<BD>::pixel *p1, const typename PT<BD>::pixel *p2, const typename PT<BD>::pixel *p3,
    intptr_t rs, intptr_t rfs, int n, int hpel_iters, int qpel_iters, int subme, int refine_qpel,
    const int32_t *__restrict__ pos, const int16_t *__restrict__ par, const int32_t *__restrict__ init_cost,
    const uint16_t *__restrict__ cost_mv, int32_t *__restrict__ out, int32_t *__restrict__ nevals )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int HDW = 8 / PT<BD>::PPD;
    constexpr int BW = pix_w( IPIX ), BH = pix_h( IPIX ), TX = BW / 8, NT = TX * (BH / 4);
    const int lane = (int)(threadIdx.x & 63);
    const int sbase = lane & 32;                          // the segment's first lane
    const int g = (lane >> 3) & 3, u = lane & 7;
    const int64_t jo = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 5;
    const bool live = jo < n;                             // segment-uniform
    const int64_t j = live ? jo : n - 1;                  // a spare segment repeats the last job
    const bool tile = u < NT;
    const int tu = tile ? u : 0;
    const int ux = 8 * (tu % TX), uy = 4 * (tu / TX);
    const int f = pos[3 * j], bx = pos[3 * j + 1], by = pos[3 * j + 2];

    uint32_t fa[4][HDW];
    const pixel *fe = fenc + f * ffs + (intptr_t)(by + uy) * fs + bx + ux;
#pragma unroll
    for( int y = 0; y < 4; y++ )
        load_row_u<HDW>( fe + y * fs, fa[y] );
    const intptr_t qo = (intptr_t)f * rfs + (intptr_t)(by + uy) * rs + bx + ux;
    const pixel *const q0 = p0 + qo, *const q1 = p1 + qo, *const q2 = p2 + qo, *const q3 = p3 + qo;

    const int16_t *p = par + 8 * j;
    const int mvpx = p[2], mvpy = p[3];
    const int minx = p[4], miny = p[5], maxx = p[6], maxy = p[7];
    const uint16_t *cmx = cost_mv - mvpx, *cmy = cost_mv - mvpy;
    int bmx = p[0], bmy = p[1];
    int bcost = init_cost[j];
    const bool qsatd = subme > 1;                         // mbcmp_unaligned (encoder.c:1411-1413)
    int nsad = 0, nsatd = 0;                              // the reference's fpelcmp / mbcmp calls
    auto count = [&]( bool satd, int k ) {
        if( satd )
            nsatd += k;
        else
            nsad += k;
    };

    // one candidate per group: group g scores (mx[g], my[g]); every lane gets the four costs
    // (pixel cost + p_cost_mvx[mx] + p_cost_mvy[my])
    auto eval4 = [&]( const int (&mx)[4], const int (&my)[4], bool satd, int (&c)[4] ) {
        // (the group's candidate by selects: indexing the arrays with the lane's group put them
        // in scratch memory)
        const int gx = g == 0 ? mx[0] : g == 1 ? mx[1] : g == 2 ? mx[2] : mx[3];
        const int gy = g == 0 ? my[0] : g == 1 ? my[1] : g == 2 ? my[2] : my[3];
        uint32_t v = 0;
        if( tile )
            v = satd ? tile_cost<BD, true>( fa, q0, q1, q2, q3, rs, gx, gy ) >> 1
                     : tile_cost<BD, false>( fa, q0, q1, q2, q3, rs, gx, gy );
        if( u == 0 )                                      // the group's mv cost, once
            v += (uint32_t)cmx[gx] + (uint32_t)cmy[gy];
        v = group_sum( v );
#pragma unroll
        for( int k = 0; k < 4; k++ )
            c[k] = (int)__shfl( (int)v, sbase + 8 * k );
    };
    auto eval1 = [&]( int mx, int my, bool satd ) {
        const int m4x[4] = { mx, mx, mx, mx }, m4y[4] = { my, my, my, my };
        int c[4];
        eval4( m4x, m4y, satd, c );
        return c[0];
    };

    // halfpel diamond (me.c:885-923)
    if( hpel_iters )
    {
        if( subme < 3 )
        {
            // the subpel component of the predicted mv (COST_MV_SAD: fpelcmp)
            const int mx = min( max( mvpx, minx + 2 ), maxx - 2 ), my = min( max( mvpy, miny + 2 ), maxy - 2 );
            if( (mx - bmx) | (my - bmy) )
            {
                const int c = eval1( mx, my, FSATD );
                count( FSATD, 1 );
                if( c < bcost )
                {
                    bcost = c;
                    bmx = mx;
                    bmy = my;
                }
            }
        }
        bcost <<= 6;
        bool act = true;                                  // this segment still iterates
        for( int i = hpel_iters; i > 0; i-- )
        {
            if( !__any( act ) )
                break;
            const int omx = bmx, omy = bmy;
            const int mx[4] = { omx, omx, omx - 2, omx + 2 }, my[4] = { omy - 2, omy + 2, omy, omy };
            int c[4];
            eval4( mx, my, FSATD, c );
            if( act )
            {
                count( FSATD, 4 );
                if( (c[0] << 6) + 2 < bcost ) bcost = (c[0] << 6) + 2;
                if( (c[1] << 6) + 6 < bcost ) bcost = (c[1] << 6) + 6;
                if( (c[2] << 6) + 16 < bcost ) bcost = (c[2] << 6) + 16;
                if( (c[3] << 6) + 48 < bcost ) bcost = (c[3] << 6) + 48;
                if( !(bcost & 63) )
                    act = false;
                else
                {
                    bmx -= (int32_t)((uint32_t)bcost << 26) >> 29;
                    bmy -= (int32_t)((uint32_t)bcost << 29) >> 29;
                    bcost &= ~63;
                }
            }
        }
        bcost >>= 6;
    }

    // the hpel winner re-scored with mbcmp when it differs from fpelcmp (me.c:925-929)
    if( !refine_qpel && qsatd && !FSATD )
    {
        bcost = eval1( bmx, bmy, true );
        count( true, 1 );
    }

    if( subme != 1 )
    {
        // quarterpel diamond (me.c:946-963)
        int bdir = -1;
        bool act = true;
        for( int i = qpel_iters; i > 0; i-- )
        {
            if( bmy <= miny || bmy >= maxy || bmx <= minx || bmx >= maxx )
                act = false;
            if( !__any( act ) )
                break;
            const int odir = bdir;
            const int omx = bmx, omy = bmy;
            const int mx[4] = { omx, omx, omx - 1, omx + 1 }, my[4] = { omy - 1, omy + 1, omy, omy };
            int c[4];
            eval4( mx, my, qsatd, c );
            if( act )
            {
#pragma unroll
                for( int d = 0; d < 4; d++ )
                    if( (refine_qpel || (d ^ 1) != odir) )
                        count( qsatd, 1 );
#pragma unroll
                for( int d = 0; d < 4; d++ )
                    if( (refine_qpel || (d ^ 1) != odir) && c[d] < bcost )
                    {
                        bcost = c[d];
                        bmx = mx[d];
                        bmy = my[d];
                        bdir = d;
                    }
                if( bmx == omx && bmy == omy )
                    act = false;
            }
        }
    }
    else if( __any( bmy > miny && bmy < maxy && bmx > minx && bmx < maxx ) )
    {
        // subme 1 (me.c:964-986): one qpel diamond of fpelcmp over mc_luma blocks
        const bool act = bmy > miny && bmy < maxy && bmx > minx && bmx < maxx;
        const int omx = bmx, omy = bmy;
        const int mx[4] = { omx, omx, omx - 1, omx + 1 }, my[4] = { omy - 1, omy + 1, omy, omy };
        int c[4];
        eval4( mx, my, FSATD, c );
        if( act )
        {
            count( FSATD, 4 );
            bcost <<= 4;
            if( (c[0] << 4) + 1 < bcost ) bcost = (c[0] << 4) + 1;
            if( (c[1] << 4) + 3 < bcost ) bcost = (c[1] << 4) + 3;
            if( (c[2] << 4) + 4 < bcost ) bcost = (c[2] << 4) + 4;
            if( (c[3] << 4) + 12 < bcost ) bcost = (c[3] << 4) + 12;
            bmx -= (int32_t)((uint32_t)bcost << 28) >> 30;
            bmy -= (int32_t)((uint32_t)bcost << 30) >> 30;
            bcost >>= 4;
        }
    }

    if( live && lane == sbase )
    {
        *(int4 *)(out + 4 * j) = make_int4( bcost, bmx, bmy, (int)cmx[bmx] + (int)cmy[bmy] );
        if( nevals )
            nevals[j] = nsad | (nsatd << 16);
    }
}

template <int BD>
hipError_t launch_me_refine_subpel( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                                    const typename PT<BD>::pixel *const planes[4], intptr_t rs, intptr_t rfs,
                                    int i_pixel, int subme, int refine_qpel, int fpel_satd, const int32_t *pos,
                                    const int16_t *par, const int32_t *init_cost, const uint16_t *cost_mv, int n,
                                    int32_t *out, int32_t *nevals, hipStream_t stream )
{
    if( n <= 0 )
        return hipSuccess;
    if( i_pixel < 0 || i_pixel > 3 || subme < 1 || subme > 11 || ((uintptr_t)out & 15) )
        return hipErrorInvalidValue;
    const int hpel = k_subpel_iterations[subme][refine_qpel ? 0 : 2];
    const int qpel = k_subpel_iterations[subme][refine_qpel ? 1 : 3];
    // fpelcmp is SATD only under TESA with subme > 1 (encoder.c:1423-1426)
    const bool fs_satd = fpel_satd && subme > 1;
    const int64_t segs = (int64_t)n;
    dim3 blk( 256 ), g( (unsigned)((segs * 32 + 255) / 256) );
#define RS_GO( I, F )                                                                                             \
    hipLaunchKernelGGL( ( me_refine_subpel_kernel<BD, I, F> ), g, blk, 0, stream, fenc, fs, ffs, planes[0],       \
                        planes[1], planes[2], planes[3], rs, rfs, n, hpel, qpel, subme, refine_qpel ? 1 : 0, pos,   \
                        par, init_cost, cost_mv, out, nevals )
#define RS_CASE( I )                                                                                              \
    case I:                                                                                                       \
        if( fs_satd ) { RS_GO( I, true ); } else { RS_GO( I, false ); }                                           \
        break;
    switch( i_pixel )
    {
        RS_CASE( 0 ) RS_CASE( 1 ) RS_CASE( 2 ) RS_CASE( 3 )
        default: return hipErrorInvalidValue;
    }
#undef RS_CASE
#undef RS_GO
    return hipGetLastError();
}

template hipError_t launch_me_refine_subpel<8>( const uint8_t *, intptr_t, intptr_t, const uint8_t *const[4],
                                                intptr_t, intptr_t, int, int, int, int, const int32_t *,
                                                const int16_t *, const int32_t *, const uint16_t *, int, int32_t *,
                                                int32_t *, hipStream_t );
template hipError_t launch_me_refine_subpel<10>( const uint16_t *, intptr_t, intptr_t, const uint16_t *const[4],
                                                 intptr_t, intptr_t, int, int, int, int, const int32_t *,
                                                 const int16_t *, const int32_t *, const uint16_t *, int, int32_t *,
                                                 int32_t *, hipStream_t );

} // namespace x264hip
