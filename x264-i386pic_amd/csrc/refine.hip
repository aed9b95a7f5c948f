// Full-resolution subpel refinement: refine_subpel (reference encoder/me.c:865-992) for a
// batch of partitions, the decision x264_me_search_ref runs after its integer search
// (me.c:791-797, hpel / qpel iterations of subpel_iterations[subme][2..3], me.c:38-50) or
// x264_me_refine_qpel runs on a winner (me.c:801-810, [0..1]).
//
// One segment of 4 * NT lanes per partition, NT = its 8x4 tiles (16x16: eight, 16x8 / 8x16:
// four, 8x8: two), so a wave holds 2, 4 or 8 partitions: four groups of NT lanes, a lane per
// tile.  A step that scores four candidates (the hpel diamond of fpelcmp_x4, the qpel diamond
// of COST_MV_SATD) gives group g candidate g; a one-candidate step (the predictor's subpel
// component, the SATD re-score of the hpel winner) runs the same candidate in every group.
// Each lane rebuilds get_ref (mc.c:221-249: the plane pair of x264_hpel_ref0/1 and the
// rounding average) for its tile and scores it with SAD or the packed 8x4 SATD
// (satd_8x4, pixel.c:290-309, summed over tiles as PIXEL_SATD_C does); the group's tiles
// meet through DPP adds and every lane of the segment reads the four candidate costs and
// takes the reference's decisions itself (the packed bcost << 6 / << 4 codes, COPY*_IF_LT's
// strict <, the odir skip), so the segment's lanes stay in step without LDS.  The
// multi-reference early exit (p_halfpel_thresh, me.c:931-944) reads and writes a per-partition
// threshold when the caller passes one: the references of one MB chain through it, one launch
// per reference (analyse.c:1260-1314), with the caller's i_ref_cost adjustments around each
// search (analyse.c:1271, 1310) applied in the kernel from a per-partition ref_cost.
//
// The EXT forms add what x264's default preset runs on P slices (b_chroma_me at subme >= 5,
// common/macroblock.c:507-509) and weighted references (m->weight, analyse.c:1248-1250):
// every luma get_ref weighted by weight[0] (mc.c:235-242), and COST_MV_SATD's chroma branch
// (me.c:833-861) -- U's cost added when the luma cost beats the running bcost, V's when the
// sum still does.  A qpel diamond's four luma costs come first; a candidate whose luma cost
// does not beat the step's starting bcost cannot win (bcost only falls within a step), so
// the chroma pass runs only when some segment of the wave has such a candidate, and each
// segment replays the reference's sequence over the full costs (the U / V calls counted as
// the reference makes them).  4:2:0 / 4:2:2 (EXT 1): each group's eight lanes split the
// candidate's chroma 4x4 blocks of both planes (one or two per lane), each lane rebuilding
// mc_chroma (mc.c:252-283) for its block from the interleaved plane, weighting it and scoring
// it with the 4x4 Hadamard (or SAD); 4:4:4 (EXT 2): the luma tile schedule over the U and V
// hpel planes with get_ref and weight[1] / weight[2].
#include "hipcommon.h"

namespace x264hip {

constexpr uint8_t c_ref0[16] = { 0, 1, 1, 1, 0, 1, 1, 1, 2, 3, 3, 3, 0, 1, 1, 1 };   // x264_hpel_ref0
constexpr uint8_t c_ref1[16] = { 0, 0, 1, 0, 2, 2, 3, 2, 2, 2, 3, 2, 2, 2, 3, 2 };   // x264_hpel_ref1

// subpel_iterations (me.c:38-50): { refine_hpel, refine_qpel, me_hpel, me_qpel }
static const uint8_t k_subpel_iterations[12][4] = { { 0, 0, 0, 0 }, { 1, 1, 0, 0 }, { 0, 1, 1, 0 }, { 0, 2, 1, 0 },
                                                    { 0, 2, 1, 1 }, { 0, 2, 1, 2 }, { 0, 0, 2, 2 }, { 0, 0, 2, 2 },
                                                    { 0, 0, 4, 10 }, { 0, 0, 4, 10 }, { 0, 0, 4, 10 },
                                                    { 0, 0, 4, 10 } };

// explicit weight of one plane (x264_weight_t, mc.c:117-137): rnd = 1 << (denom - 1) or 0,
// offset already scaled by 1 << (BIT_DEPTH - 8)
struct RsWeight
{
    int on, scale, denom, rnd, offset;
};

// mc_weight of packed pixels: clip( ((v * scale + rnd) >> denom) + offset ) per pixel
template <int BD> __device__ __forceinline__ uint32_t weigh_packed( uint32_t w, const RsWeight &wt )
{
    constexpr int PPD = PT<BD>::PPD, SH = 32 / PPD;
    uint32_t r = 0;
#pragma unroll
    for( int k = 0; k < PPD; k++ )
    {
        const int v = upix<BD>( w, k );
        r |= (uint32_t)clip_pix<BD>( ((v * wt.scale + wt.rnd) >> wt.denom) + wt.offset ) << (SH * k);
    }
    return r;
}

// the lane's 8x4 tile of get_ref( mvx, mvy ) (weighted when WGT and wt.on) scored against its
// fenc tile: SAD, or the sum of |coef| of the tile's two 4x4 Hadamards (even; halved by the
// caller)
// LF: the lane's fenc side read from LDS (fl[256 w]: words 0-15 the tile's had8x4_biased
// coefficients, 16 + HDW y + k its words; fa unused) -- the SATD then skips the fenc unpacking
// and the difference per candidate, and the tile stays out of the kernel's registers
typedef __attribute__( ( address_space( 3 ) ) ) const uint32_t lds_cu32;
template <int BD, bool SATD, bool WGT = false, int TW = 8, bool LF = false>
__device__ __forceinline__ uint32_t tile_cost( const uint32_t (&fa)[4][8 / PT<BD>::PPD],
                                               const typename PT<BD>::pixel *q0, const typename PT<BD>::pixel *q1,
                                               const typename PT<BD>::pixel *q2, const typename PT<BD>::pixel *q3,
                                               intptr_t rs, int mvx, int mvy, const RsWeight wt = {},
                                               lds_cu32 *fl = nullptr )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int HDW = 8 / PT<BD>::PPD, LW = HDW * TW / 8;   // words of a row; of the tile's row
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
    {
        uint32_t t[LW];
        load_al_pad<LW>( s1 + y * rs, t );
#pragma unroll
        for( int k = 0; k < HDW; k++ )
            r1[y][k] = k < LW ? t[k] : 0u;
    }
    if( idx & 5 )                           // two planes: the rounding average (one plane: avg( a, a ) = a)
    {
        uint32_t r2[4][LW];
#pragma unroll
        for( int y = 0; y < 4; y++ )
            load_al_pad<LW>( s2 + y * rs, r2[y] );
#pragma unroll
        for( int y = 0; y < 4; y++ )
#pragma unroll
            for( int k = 0; k < LW; k++ )
                r1[y][k] = avg_round<BD>( r1[y][k], r2[y][k] );
    }
    if constexpr( WGT )
        if( wt.on )
#pragma unroll
            for( int y = 0; y < 4; y++ )
#pragma unroll
                for( int k = 0; k < LW; k++ )
                    r1[y][k] = weigh_packed<BD>( r1[y][k], wt );
    // a 4-wide tile (TW 4) is the 8x4 SATD's left 4x4 with zero differences on the right
    lds_cu32 *h = fl;
    if constexpr( LF )
        asm volatile( "" : "+v"( h ) );                 // read per candidate, not hoisted into registers
    if constexpr( SATD )
    {
        if constexpr( !LF )
            return satd8x4_packed<BD>( fa, r1 );
        uint32_t o[16], acc = 0;
        had8x4_biased<BD>( r1, o );
#pragma unroll
        for( int k = 0; k < 16; k++ )
            acc = __builtin_amdgcn_sad_u16( o[k], h[256 * k], acc );
        return acc;
    }
    else
    {
        uint32_t acc = 0;
#pragma unroll
        for( int y = 0; y < 4; y++ )
#pragma unroll
            for( int k = 0; k < LW; k++ )
                acc = sadp<BD>( LF ? h[256 * (16 + HDW * y + k)] : fa[y][k], r1[y][k], acc );
        return acc;
    }
}

// a partition's tiles (reference common/pixel.h:55-59): 8x4 for widths >= 8, 4x4 for the 4-wide
// sub-8x8 partitions (satd_4x4 per 4x4, pixel.c:265-288, 311-332); NT tiles, SH = log2 of the
// lanes a segment of G groups takes
template <int IPIX> constexpr int tile_w() { return pix_w( IPIX ) >= 8 ? 8 : 4; }
template <int IPIX> constexpr int tile_n() { return (pix_w( IPIX ) / tile_w<IPIX>()) * (pix_h( IPIX ) / 4); }
constexpr int ilog2( int v ) { return v <= 1 ? 0 : 1 + ilog2( v / 2 ); }
__host__ __device__ constexpr int part_tiles( int i_pixel )
{
    return (pix_w( i_pixel ) >= 8 ? pix_w( i_pixel ) / 8 : 1) * (pix_h( i_pixel ) / 4);
}
// the fenc rows of the lane's tile (4-wide: the right half zero)
template <int BD, int TW>
__device__ __forceinline__ void load_fenc_tile( const typename PT<BD>::pixel *fe, intptr_t fs,
                                                uint32_t (&fa)[4][8 / PT<BD>::PPD] )
{
    constexpr int HDW = 8 / PT<BD>::PPD, LW = HDW * TW / 8;
#pragma unroll
    for( int y = 0; y < 4; y++ )
    {
        uint32_t t[LW];
        load_row_u<LW>( fe + y * fs, t );
#pragma unroll
        for( int k = 0; k < HDW; k++ )
            fa[y][k] = k < LW ? t[k] : 0u;
    }
}

// 4x4 Hadamard sum |coef| >> 1 (satd_4x4, pixel.c:265-288) or SAD of a difference block
__device__ __forceinline__ uint32_t block4_cost( const int (&d)[4][4], bool satd )
{
    uint32_t acc = 0;
    if( !satd )
    {
#pragma unroll
        for( int y = 0; y < 4; y++ )
#pragma unroll
            for( int x = 0; x < 4; x++ )
                acc += (uint32_t)abs( d[y][x] );
        return acc;
    }
    int t[4][4];
#pragma unroll
    for( int y = 0; y < 4; y++ )
    {
        const int a0 = d[y][0] + d[y][1], a1 = d[y][0] - d[y][1], a2 = d[y][2] + d[y][3], a3 = d[y][2] - d[y][3];
        t[y][0] = a0 + a2; t[y][2] = a0 - a2; t[y][1] = a1 + a3; t[y][3] = a1 - a3;
    }
#pragma unroll
    for( int x = 0; x < 4; x++ )
    {
        const int a0 = t[0][x] + t[1][x], a1 = t[0][x] - t[1][x], a2 = t[2][x] + t[3][x], a3 = t[2][x] - t[3][x];
        acc += (uint32_t)(abs( a0 + a2 ) + abs( a0 - a2 ) + abs( a1 + a3 ) + abs( a1 - a3 ));
    }
    return acc >> 1;
}

// The chroma cost of one 4x4 position of mc_chroma (mc.c:252-283) in both planes at once, split
// over a lane pair: NV12 / NV16 interleave U and V, so a sample pair (U x, V x) is one packed
// 16-bit pair (v_perm of the bytes at 8 bit, the dword itself at 10 bit) and every step runs on
// the two planes together -- the bilinear taps as packed u16 multiply-adds (cA..cD sum to 64, so
// 64 * 1023 + 32 fits), the differences and the Hadamard as packed i16 (|coef| <= 8 * 1023).
// Lane half hh computes output rows 2hh, 2hh+1 (source rows 2hh .. 2hh+2) and their row
// transform and first column butterfly; the last butterfly is |a + b| + |a - b| = 2 max(|a|, |b|),
// so each lane takes two of the four columns, gets the partner's t of those columns by one DPP
// swap per word, and adds max(|t|, |t'|): the pair's sum is satd_4x4's sum |coef| >> 1
// (pixel.c:265-288) exactly.  The odd lane negates its columns 2, 3 of differences, which swaps
// its row transform's outputs 0, 1 with 2, 3: each lane then keeps its outputs 0, 1 and sends
// 2, 3, with no lane-dependent select.  s = the interleaved plane at the position's top-left U
// sample, row 2hh; fb = the lane's two fenc rows as (U, V) pairs.  Returns U's partial cost | V's
// << 16.
typedef unsigned short rs_us2 __attribute__( ( ext_vector_type( 2 ) ) );
__device__ __forceinline__ rs_us2 as_us2( uint32_t v ) { return __builtin_bit_cast( rs_us2, v ); }
__device__ __forceinline__ x264hip_short2 as_s2( rs_us2 v ) { return __builtin_bit_cast( x264hip_short2, v ); }
__device__ __forceinline__ uint32_t as_u32( x264hip_short2 v ) { return __builtin_bit_cast( uint32_t, v ); }

template <int BD> __device__ __forceinline__ rs_us2 nv_pair( const uint32_t *w, int x )
{
    // the (U, V) samples of pixel x of a row of interleaved words, as u16 lanes
    if constexpr( BD == 8 )
        return as_us2( __builtin_amdgcn_perm( 0u, w[x >> 1], (x & 1) ? 0x0c030c02u : 0x0c010c00u ) );
    else
        return as_us2( w[x] );
}

template <int BD>
__device__ __forceinline__ uint32_t nv_pair_cost( const typename PT<BD>::pixel *s, intptr_t rcs, int mvx, int mvyc,
                                                  const uint32_t (&fb)[2][4], const RsWeight &wu,
                                                  const RsWeight &wv, bool satd, bool hh )
{
    constexpr int NDW = BD == 8 ? 3 : 5;    // five (U, V) pairs of a source row
    const uint32_t dx = mvx & 7, dy = mvyc & 7;
    const rs_us2 kA = (rs_us2)(uint16_t)((8 - dx) * (8 - dy)), kB = (rs_us2)(uint16_t)(dx * (8 - dy));
    const rs_us2 kC = (rs_us2)(uint16_t)((8 - dx) * dy), kD = (rs_us2)(uint16_t)(dx * dy);
    s += (intptr_t)(mvyc >> 3) * rcs + (mvx >> 3) * 2;
    uint32_t w[3][NDW];
#pragma unroll
    for( int r = 0; r < 3; r++ )
        load_al_pad<NDW>( s + r * rcs, w[r] );
    x264hip_short2 d[2][4];
#pragma unroll
    for( int y = 0; y < 2; y++ )
#pragma unroll
        for( int x = 0; x < 4; x++ )
        {
            rs_us2 m = (kA * nv_pair<BD>( w[y], x ) + kB * nv_pair<BD>( w[y], x + 1 ) + kC * nv_pair<BD>( w[y + 1], x ) +
                        kD * nv_pair<BD>( w[y + 1], x + 1 ) + (rs_us2)32) >> (rs_us2)6;
            if( wu.on | wv.on )
            {
                int lo = m.x, hi = m.y;
                if( wu.on )
                    lo = clip_pix<BD>( ((lo * wu.scale + wu.rnd) >> wu.denom) + wu.offset );
                if( wv.on )
                    hi = clip_pix<BD>( ((hi * wv.scale + wv.rnd) >> wv.denom) + wv.offset );
                m = (rs_us2){ (uint16_t)lo, (uint16_t)hi };
            }
            d[y][x] = __builtin_bit_cast( x264hip_short2, fb[y][x] ) - as_s2( m );
        }
    x264hip_short2 acc = { 0, 0 };
    if( !satd )
    {
#pragma unroll
        for( int y = 0; y < 2; y++ )
#pragma unroll
            for( int x = 0; x < 4; x++ )
                acc += __builtin_elementwise_abs( d[y][x] );
        return as_u32( acc );
    }
    const x264hip_short2 sg = hh ? (x264hip_short2)-1 : (x264hip_short2)1;
    x264hip_short2 t[2][4];
#pragma unroll
    for( int y = 0; y < 2; y++ )
    {
        const x264hip_short2 a0 = d[y][0] + d[y][1], a1 = d[y][0] - d[y][1];
        const x264hip_short2 a2 = sg * (d[y][2] + d[y][3]), a3 = sg * (d[y][2] - d[y][3]);
        t[y][0] = a0 + a2; t[y][2] = a0 - a2; t[y][1] = a1 + a3; t[y][3] = a1 - a3;
    }
    // rows 0 + 1 and 0 - 1 of the lane's pair of rows; outputs 0, 1 kept, 2, 3 sent (quad_perm
    // [1,0,3,2]); max(|a|, |b|) = max(max(a, b), -min(a, b))
    x264hip_short2 own[4], snd[4];
#pragma unroll
    for( int x = 0; x < 2; x++ )
    {
        own[x] = t[0][x] + t[1][x];
        own[2 + x] = t[0][x] - t[1][x];
        snd[x] = t[0][2 + x] + t[1][2 + x];
        snd[2 + x] = t[0][2 + x] - t[1][2 + x];
    }
#pragma unroll
    for( int j = 0; j < 4; j++ )
    {
        const x264hip_short2 r = __builtin_bit_cast(
            x264hip_short2, __builtin_amdgcn_mov_dpp( (int)as_u32( snd[j] ), 0xB1, 0xF, 0xF, false ) );
        acc += __builtin_elementwise_max( __builtin_elementwise_max( own[j], r ),
                                          -__builtin_elementwise_min( own[j], r ) );
    }
    return as_u32( acc );
}

// the NT tiles of each group summed into the group's first lane (pair sums, quad sums by
// quad_perm, then for NT = 8 row_ror:12 brings lane 8k+4's quad sum to lane 8k)
template <int NT> __device__ __forceinline__ uint32_t group_sum( uint32_t v )
{
    if constexpr( NT >= 2 )
        v += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)v, 0xB1, 0xF, 0xF, false );
    if constexpr( NT >= 4 )
        v += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)v, 0x4E, 0xF, 0xF, false );
    if constexpr( NT >= 8 )
        v += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)v, 0x12C, 0xF, 0xF, false );
    return v;
}

// the EXT inputs of a launch (x264hip_refine_ext_t), by value in the kernel arguments
template <int BD> struct RsExt
{
    const typename PT<BD>::pixel *fenc_c[2];   // NV12 / NV16 plane, or U, V: pixel (0,0) of frame 0
    const typename PT<BD>::pixel *ref_c[8];    // NV12 / NV16 plane, or U's F, H, V, C then V's
    intptr_t fcs, ffcs, rcs, rfcs;
    int chroma, vs, mvy_offset;                // b_chroma_me, CHROMA_V_SHIFT, me.c:875's offset
    RsWeight wt[3];                            // m->weight[0..2]
};

template <int BD, int IPIX, bool FSATD, int EXT>
__global__ __launch_bounds__( 256 ) void me_refine_subpel_kernel(
    const typename PT<BD>::pixel *__restrict__ fenc, intptr_t fs, intptr_t ffs, const typename PT<BD>::pixel *p0,
    const typename PT<BD>::pixel *p1, const typename PT<BD>::pixel *p2, const typename PT<BD>::pixel *p3,
    intptr_t rs, intptr_t rfs, int n, int hpel_iters, int qpel_iters, int subme, int refine_qpel,
    const int32_t *__restrict__ pos, const int16_t *__restrict__ par, const int32_t *__restrict__ init_cost,
    const uint16_t *__restrict__ cost_mv, int32_t *__restrict__ out, int32_t *__restrict__ nevals, int nstride,
    int32_t *__restrict__ thr, const int32_t *__restrict__ rcost, const RsExt<BD> ext )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int HDW = 8 / PT<BD>::PPD;
    constexpr int BW = pix_w( IPIX ), BH = pix_h( IPIX ), TW = tile_w<IPIX>(), TX = BW / TW, NT = tile_n<IPIX>();
    const int lane = (int)(threadIdx.x & 63);
    constexpr int SL = 4 * NT, SH = ilog2( SL );          // segment lanes, log2
    const int sbase = lane & (64 - SL);                   // the segment's first lane
    const int g = (lane / NT) & 3, u = lane & (NT - 1);
    const int64_t jo = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> SH;
    const bool live = jo < n;                             // segment-uniform
    const int64_t j = live ? jo : n - 1;                  // a spare segment repeats the last job
    constexpr bool tile = true;                           // every lane holds a tile
    const int ux = TW * (u % TX), uy = 4 * (u / TX);
    const int f = pos[3 * j], bx = pos[3 * j + 1], by = pos[3 * j + 2];

    // the lane's fenc tile and its Hadamard coefficients in LDS, once (word-major: a word of
    // every lane is one conflict-free row; tile_cost's LF form): luma-only 0.173 -> 0.163 ms per
    // 130560 MBs.  Not with 4:2:0 / 4:2:2 chroma ME (EXT 1): 0.232 -> 0.237-0.239 ms with the
    // coefficients in LDS or in registers (profiles/r06zt_ .. r06zw_refine_*_ab.log)
    constexpr bool LF = EXT != 1;
    uint32_t fa[4][HDW];
    __shared__ uint32_t s_fl[LF ? 16 + 4 * HDW : 1][LF ? 256 : 1];
    load_fenc_tile<BD, TW>( fenc + f * ffs + (intptr_t)(by + uy) * fs + bx + ux, fs, fa );
    if constexpr( LF )
    {
        uint32_t o[16];
        had8x4_biased<BD>( fa, o );
#pragma unroll
        for( int k = 0; k < 16; k++ )
            s_fl[k][threadIdx.x] = o[k];
#pragma unroll
        for( int y = 0; y < 4; y++ )
#pragma unroll
            for( int k = 0; k < HDW; k++ )
            {
                s_fl[16 + HDW * y + k][threadIdx.x] = fa[y][k];
                fa[y][k] = 0u;                            // (unused by the LF form)
            }
    }
    lds_cu32 *const hf = LF ? (lds_cu32 *)&s_fl[0][threadIdx.x] : nullptr;
    const intptr_t qo = (intptr_t)f * rfs + (intptr_t)(by + uy) * rs + bx + ux;
    const pixel *const q0 = p0 + qo, *const q1 = p1 + qo, *const q2 = p2 + qo, *const q3 = p3 + qo;

    // ---- EXT: the weight of the luma get_ref, the lane's chroma blocks / tiles ----
    const RsWeight wt0 = ext.wt[0];
    // b_chroma_me = h->mb.b_chroma_me && (i_pixel <= PIXEL_8x8 || CHROMA444) (me.c:872)
    const bool chroma = EXT && ext.chroma && (IPIX <= 3 || EXT == 2);   // launch-uniform
    constexpr int FDW = 8 / PT<BD>::PPD;                  // words of a 4-pixel interleaved chroma row
    const pixel *cref[2] = { nullptr, nullptr };          // EXT 1: the lane's positions in the ref plane
    // their two fenc rows, in LDS (word-major: a word of every lane is one conflict-free row) --
    // in VGPRs they pushed the kernel past 128 registers, 4 -> 3 waves per SIMD
    __shared__ uint32_t s_cfb[EXT == 1 ? 2 * 2 * 4 : 1][256];
    bool has[2] = { false, false };
    const bool hh = u & 1;                                //        the lane's half of a position
    uint32_t fu[4][HDW] = {}, fv[4][HDW] = {};            // EXT 2: the fenc tiles of U and V
    const pixel *u0 = nullptr, *u1 = nullptr, *u2 = nullptr, *u3 = nullptr;   // and their hpel planes
    const pixel *v0 = nullptr, *v1 = nullptr, *v2 = nullptr, *v3 = nullptr;   // (no arrays: scratch)
    if constexpr( EXT == 1 && IPIX <= 3 )
    {
        if( chroma )
        {
            // chroma block cw x ch of the partition (luma2chroma_pixel, pixel.h:70-76) in 4x4
            // positions of both planes (at most NT of them); lane pair (2q, 2q+1) takes positions
            // q and q + NT / 2, lane 2q + hh their rows 2hh, 2hh+1
            constexpr int CW = BW / 2, BXN = CW / 4;
            const int ch = BH >> ext.vs, npos = BXN * (ch / 4);
            const intptr_t crow = by >> ext.vs;
#pragma unroll
            for( int k = 0; k < 2; k++ )
            {
                const int q = (u >> 1) + (NT / 2) * k;
                if( q < npos )
                {
                    const int cx = 4 * (q % BXN), cy = 4 * (q / BXN) + 2 * hh;
                    has[k] = true;
                    cref[k] = ext.ref_c[0] + f * ext.rfcs + (crow + cy) * ext.rcs + bx + 2 * cx;
                    const pixel *fc = ext.fenc_c[0] + f * ext.ffcs + (crow + cy) * ext.fcs + bx + 2 * cx;
#pragma unroll
                    for( int y = 0; y < 2; y++ )
                    {
                        uint32_t r[FDW];
                        load_row_u<FDW>( fc + y * ext.fcs, r );
#pragma unroll
                        for( int i = 0; i < 4; i++ )       // as (U, V) pairs
                            s_cfb[(2 * k + y) * 4 + i][threadIdx.x] = as_u32( as_s2( nv_pair<BD>( r, i ) ) );
                    }
                }
            }
        }
    }
    else if constexpr( EXT == 2 )
    {
        if( chroma )
        {
            const intptr_t fco = (intptr_t)f * ext.ffcs + (intptr_t)(by + uy) * ext.fcs + bx + ux;
            load_fenc_tile<BD, TW>( ext.fenc_c[0] + fco, ext.fcs, fu );
            load_fenc_tile<BD, TW>( ext.fenc_c[1] + fco, ext.fcs, fv );
            const intptr_t rco = (intptr_t)f * ext.rfcs + (intptr_t)(by + uy) * ext.rcs + bx + ux;
            u0 = ext.ref_c[0] + rco; u1 = ext.ref_c[1] + rco; u2 = ext.ref_c[2] + rco; u3 = ext.ref_c[3] + rco;
            v0 = ext.ref_c[4] + rco; v1 = ext.ref_c[5] + rco; v2 = ext.ref_c[6] + rco; v3 = ext.ref_c[7] + rco;
        }
    }

    const int16_t *p = par + 8 * j;
    const int mvpx = p[2], mvpy = p[3];
    const int minx = p[4], miny = p[5], maxx = p[6], maxy = p[7];
    const uint16_t *cmx = cost_mv - mvpx, *cmy = cost_mv - mvpy;
    int bmx = p[0], bmy = p[1];
    int bcost = init_cost[j];
    const bool qsatd = subme > 1;                         // mbcmp_unaligned (encoder.c:1411-1413)
    int nsad = 0, nsatd = 0, nchroma = 0;                 // the reference's fpelcmp / mbcmp calls
    auto count = [&]( bool satd, int k ) __attribute__( ( always_inline ) ) {
        if( satd )
            nsatd += k;
        else
            nsad += k;
    };

    // one candidate per group: group g scores (mx[g], my[g]); every lane gets the four costs
    // (pixel cost + p_cost_mvx[mx] + p_cost_mvy[my])
    auto eval4 = [&]( const int (&mx)[4], const int (&my)[4], bool satd, int (&c)[4] ) __attribute__( ( always_inline ) ) {
        // (the group's candidate by selects: indexing the arrays with the lane's group put them
        // in scratch memory)
        const int gx = g == 0 ? mx[0] : g == 1 ? mx[1] : g == 2 ? mx[2] : mx[3];
        const int gy = g == 0 ? my[0] : g == 1 ? my[1] : g == 2 ? my[2] : my[3];
        uint32_t v = 0;
        if( tile )
            v = satd ? tile_cost<BD, true, EXT != 0, TW, LF>( fa, q0, q1, q2, q3, rs, gx, gy, wt0, hf ) >> 1
                     : tile_cost<BD, false, EXT != 0, TW, LF>( fa, q0, q1, q2, q3, rs, gx, gy, wt0, hf );
        if( u == 0 )                                      // the group's mv cost, once
            v += (uint32_t)cmx[gx] + (uint32_t)cmy[gy];
        v = group_sum<NT>( v );
#pragma unroll
        for( int k = 0; k < 4; k++ )
            c[k] = (int)__shfl( (int)v, sbase + NT * k );
    };
    // eval4 (SATD) with the diamond's centre (cx, cy) scored beside each group's candidate in the
    // same memory round: the hpel winner's COST_MV_SATD (me.c:925-929) merged into the first
    // quarterpel diamond's round; cc = the centre's cost
    auto eval4c = [&]( const int (&mx)[4], const int (&my)[4], int cx, int cy, int (&c)[4], int &cc ) __attribute__( ( always_inline ) ) {
        const int gx = g == 0 ? mx[0] : g == 1 ? mx[1] : g == 2 ? mx[2] : mx[3];
        const int gy = g == 0 ? my[0] : g == 1 ? my[1] : g == 2 ? my[2] : my[3];
        uint32_t vc = tile_cost<BD, true, EXT != 0, TW, LF>( fa, q0, q1, q2, q3, rs, cx, cy, wt0, hf ) >> 1;
        uint32_t v = tile_cost<BD, true, EXT != 0, TW, LF>( fa, q0, q1, q2, q3, rs, gx, gy, wt0, hf ) >> 1;
        if( u == 0 )
        {
            v += (uint32_t)cmx[gx] + (uint32_t)cmy[gy];
            vc += (uint32_t)cmx[cx] + (uint32_t)cmy[cy];
        }
        v = group_sum<NT>( v );
        vc = group_sum<NT>( vc );
#pragma unroll
        for( int k = 0; k < 4; k++ )
            c[k] = (int)__shfl( (int)v, sbase + NT * k );
        cc = (int)__shfl( (int)vc, sbase );
    };
    // one candidate: group 0 scores it, the other groups' lanes stay masked off (no loads)
    auto eval1 = [&]( int mx, int my, bool satd ) __attribute__( ( always_inline ) ) {
        uint32_t v = 0;
        if( g == 0 )
        {
            v = satd ? tile_cost<BD, true, EXT != 0, TW, LF>( fa, q0, q1, q2, q3, rs, mx, my, wt0, hf ) >> 1
                     : tile_cost<BD, false, EXT != 0, TW, LF>( fa, q0, q1, q2, q3, rs, mx, my, wt0, hf );
            if( u == 0 )
                v += (uint32_t)cmx[mx] + (uint32_t)cmy[my];
        }
        v = group_sum<NT>( v );
        return (int)__shfl( (int)v, sbase );
    };
    // the chroma costs (mbcmp: SATD for subme > 1) of the diamond of step st around (ox, oy) in
    // the order (0, -st), (0, +st), (-st, 0), (+st, 0) -- st = 0: the centre in every group: U in
    // cu, V in cv.  (The group's candidate by arithmetic: the selects of eval4 became an indexed
    // scratch load here.)
    auto evalc4 = [&]( int ox, int oy, int st, int (&cu)[4], int (&cv)[4] ) __attribute__( ( always_inline ) ) {
        const int gx = ox + (g == 2 ? -st : g == 3 ? st : 0);
        const int gy = oy + (g == 0 ? -st : g == 1 ? st : 0);
        uint32_t vu = 0, vv = 0;
        const bool on = st != 0 || g == 0;               // st = 0: group 0 scores the centre alone
        if constexpr( EXT == 1 && IPIX <= 3 )
        {
            const int mvyc = (2 * (gy + ext.mvy_offset)) >> ext.vs;
            uint32_t pk = 0;                              // U | V << 16 (no carry: <= 2 * 4 * 8184)
#pragma unroll
            for( int k = 0; k < 2; k++ )
                if( on && has[k] )
                {
                    uint32_t fb[2][4];
#pragma unroll
                    for( int y = 0; y < 2; y++ )
#pragma unroll
                        for( int i = 0; i < 4; i++ )
                            fb[y][i] = s_cfb[(2 * k + y) * 4 + i][threadIdx.x];
                    pk += nv_pair_cost<BD>( cref[k], ext.rcs, gx, mvyc, fb, ext.wt[1], ext.wt[2], qsatd, hh );
                }
            vu = pk & 0xffff;
            vv = pk >> 16;
        }
        else if constexpr( EXT == 2 )
        {
            if( tile && on )
            {
                if( qsatd )
                {
                    vu = tile_cost<BD, true, true, TW>( fu, u0, u1, u2, u3, ext.rcs, gx, gy, ext.wt[1] ) >> 1;
                    vv = tile_cost<BD, true, true, TW>( fv, v0, v1, v2, v3, ext.rcs, gx, gy, ext.wt[2] ) >> 1;
                }
                else
                {
                    vu = tile_cost<BD, false, true, TW>( fu, u0, u1, u2, u3, ext.rcs, gx, gy, ext.wt[1] );
                    vv = tile_cost<BD, false, true, TW>( fv, v0, v1, v2, v3, ext.rcs, gx, gy, ext.wt[2] );
                }
            }
        }
        vu = group_sum<NT>( vu );
        vv = group_sum<NT>( vv );
#pragma unroll
        for( int k = 0; k < 4; k++ )
        {
            cu[k] = (int)__shfl( (int)vu, sbase + NT * k );
            cv[k] = (int)__shfl( (int)vv, sbase + NT * k );
        }
    };
    // evalc4 of the unit diamond around (ox, oy) with the centre's chroma in the same round (EXT 1;
    // the merged re-score, as eval4c): cuc / cvc = the centre's U / V costs
    auto evalc4c = [&]( int ox, int oy, int (&cu)[4], int (&cv)[4], int &cuc, int &cvc ) __attribute__( ( always_inline ) ) {
        const int gx = ox + (g == 2 ? -1 : g == 3 ? 1 : 0);
        const int gy = oy + (g == 0 ? -1 : g == 1 ? 1 : 0);
        uint32_t pk = 0, pc = 0;
        if constexpr( EXT == 1 && IPIX <= 3 )
        {
            const int mvyc = (2 * (gy + ext.mvy_offset)) >> ext.vs, mvyo = (2 * (oy + ext.mvy_offset)) >> ext.vs;
#pragma unroll
            for( int k = 0; k < 2; k++ )
                if( has[k] )
                {
                    uint32_t fb[2][4];
#pragma unroll
                    for( int y = 0; y < 2; y++ )
#pragma unroll
                        for( int i = 0; i < 4; i++ )
                            fb[y][i] = s_cfb[(2 * k + y) * 4 + i][threadIdx.x];
                    pc += nv_pair_cost<BD>( cref[k], ext.rcs, ox, mvyo, fb, ext.wt[1], ext.wt[2], qsatd, hh );
                    pk += nv_pair_cost<BD>( cref[k], ext.rcs, gx, mvyc, fb, ext.wt[1], ext.wt[2], qsatd, hh );
                }
        }
        const uint32_t vu = group_sum<NT>( pk & 0xffff ), vv = group_sum<NT>( pk >> 16 );
        const uint32_t wu = group_sum<NT>( pc & 0xffff ), wv = group_sum<NT>( pc >> 16 );
#pragma unroll
        for( int k = 0; k < 4; k++ )
        {
            cu[k] = (int)__shfl( (int)vu, sbase + NT * k );
            cv[k] = (int)__shfl( (int)vv, sbase + NT * k );
        }
        cuc = (int)__shfl( (int)wu, sbase );
        cvc = (int)__shfl( (int)wv, sbase );
    };
    // COST_MV_SATD's chroma branch (me.c:833-861) on a luma cost c against bcost
    auto add_chroma = [&]( int c, int cu, int cv, int bc ) __attribute__( ( always_inline ) ) {
        if( c < bc )
        {
            nchroma++;
            c += cu;
            if( c < bc )
            {
                nchroma++;
                c += cv;
            }
        }
        return c;
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

    // the hpel winner re-scored with mbcmp when it differs from fpelcmp or chroma ME is on
    // (me.c:925-929: bcost = COST_MAX, COST_MV_SATD).  With a quarterpel diamond to follow (SATD
    // mbcmp, 4:2:0 / 4:2:2 or no chroma) the re-score rides in the diamond's first round: the
    // diamond's candidates around the hpel winner do not depend on the re-scored cost, only its
    // decisions do, so every group scores its candidate and the winner together (luma, then
    // chroma) and the first iteration below takes those costs
    const bool resc = !refine_qpel && ((qsatd && !FSATD) || chroma);
    const bool merged = resc && qsatd && subme != 1 && qpel_iters > 0 && (!chroma || EXT == 1);   // uniform
    int c1[4], cu1[4] = { 0, 0, 0, 0 }, cv1[4] = { 0, 0, 0, 0 };
    if( merged )
    {
        const int mx[4] = { bmx, bmx, bmx - 1, bmx + 1 }, my[4] = { bmy - 1, bmy + 1, bmy, bmy };
        eval4c( mx, my, bmx, bmy, c1, bcost );
        count( qsatd, 1 );
        if constexpr( EXT == 1 )
            if( chroma )
            {
                int cuc, cvc;
                evalc4c( bmx, bmy, cu1, cv1, cuc, cvc );
                bcost = add_chroma( bcost, cuc, cvc, 1 << 28 );
            }
    }
    else if( resc )
    {
        bcost = eval1( bmx, bmy, qsatd );
        count( qsatd, 1 );
        if constexpr( EXT != 0 )
            if( chroma )
            {
                int cu[4], cv[4];
                evalc4( bmx, bmy, 0, cu, cv );
                bcost = add_chroma( bcost, cu[0], cv[0], 1 << 28 );
            }
    }

    // the multi-reference early exit (me.c:931-944) against *p_halfpel_thresh, which the caller
    // holds less this reference's i_ref_cost during the search (analyse.c:1271, 1310)
    bool early = false;
    if( thr )
    {
        const int rc = rcost ? rcost[j] : 0;
        int t = thr[j] - rc;
        if( (bcost * 7) >> 3 > t )
            early = true;                                 // m->cost, m->mv; m->cost_mv untouched
        else if( bcost < t )
            t = bcost;
        if( live && lane == sbase )
            thr[j] = t + rc;
    }

    if( subme != 1 )
    {
        // quarterpel diamond (me.c:946-963)
        int bdir = -1;
        bool act = !early;
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
            int cu[4] = { 0, 0, 0, 0 }, cv[4] = { 0, 0, 0, 0 };
            if( merged && i == qpel_iters )               // the first round's costs, scored with the re-score
            {
#pragma unroll
                for( int d = 0; d < 4; d++ )
                {
                    c[d] = c1[d];
                    cu[d] = cu1[d];
                    cv[d] = cv1[d];
                }
            }
            else
            {
            eval4( mx, my, qsatd, c );
            if constexpr( EXT != 0 )
                if( chroma )
                {
                    // a candidate whose luma cost does not beat the step's starting bcost never wins
                    bool need = false;
#pragma unroll
                    for( int d = 0; d < 4; d++ )
                        need |= act && (refine_qpel || (d ^ 1) != odir) && c[d] < bcost;
                    if( __any( need ) )
                        evalc4( omx, omy, 1, cu, cv );
                }
            }
            if( act )
            {
#pragma unroll
                for( int d = 0; d < 4; d++ )
                    if( refine_qpel || (d ^ 1) != odir )
                    {
                        count( qsatd, 1 );
                        const int cd = chroma ? add_chroma( c[d], cu[d], cv[d], bcost ) : c[d];
                        if( cd < bcost )
                        {
                            bcost = cd;
                            bmx = mx[d];
                            bmy = my[d];
                            bdir = d;
                        }
                    }
                if( bmx == omx && bmy == omy )
                    act = false;
            }
        }
    }
    else if( __any( !early && bmy > miny && bmy < maxy && bmx > minx && bmx < maxx ) )
    {
        // subme 1 (me.c:964-986): one qpel diamond of fpelcmp over mc_luma blocks
        const bool act = !early && bmy > miny && bmy < maxy && bmx > minx && bmx < maxx;
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
        if( early )
        {
            out[4 * j] = bcost;
            out[4 * j + 1] = bmx;
            out[4 * j + 2] = bmy;
        }
        else
            *(int4 *)(out + 4 * j) = make_int4( bcost, bmx, bmy, (int)cmx[bmx] + (int)cmy[bmy] );
        if( nevals )
            nevals[j * nstride] = nsad | (nsatd << 16) | (nchroma << 24);
    }
}

// the EXT inputs of x264hip_refine_ext_t for the kernels (mode: 0 plain, 1 weighted luma and / or
// 4:2:0 / 4:2:2 chroma ME, 2 4:4:4 chroma ME), or hipErrorInvalidValue
template <int BD> hipError_t rs_ext( const x264hip_refine_ext_t *xe, RsExt<BD> &ext, int &mode )
{
    using pixel = typename PT<BD>::pixel;
    ext = {};
    mode = 0;
    if( !xe )
        return hipSuccess;
    for( int k = 0; k < 3; k++ )
    {
        const x264hip_weight_t &w = xe->weight[k];
        if( w.weighted && (w.denom < 0 || w.denom > 7) )
            return hipErrorInvalidValue;
        ext.wt[k] = { w.weighted ? 1 : 0, w.scale, w.weighted ? w.denom : 0,
                      w.weighted && w.denom > 0 ? 1 << (w.denom - 1) : 0, w.offset * (1 << (BD - 8)) };
    }
    const int cf = xe->chroma_format;
    if( xe->b_chroma_me )
    {
        if( cf < 1 || cf > 3 || !xe->fenc_chroma[0] || !xe->ref_chroma[0] ||
            (cf == 3 && (!xe->fenc_chroma[1] || !xe->ref_chroma[1] || !xe->ref_chroma[2] || !xe->ref_chroma[3] ||
                         !xe->ref_chroma[4] || !xe->ref_chroma[5] || !xe->ref_chroma[6] || !xe->ref_chroma[7])) )
            return hipErrorInvalidValue;
        ext.chroma = 1;
        ext.vs = cf == 1;
        ext.mvy_offset = xe->mvy_offset;
        for( int k = 0; k < 2; k++ )
            ext.fenc_c[k] = (const pixel *)xe->fenc_chroma[k];
        for( int k = 0; k < 8; k++ )
            ext.ref_c[k] = (const pixel *)xe->ref_chroma[k];
        ext.fcs = xe->fenc_chroma_stride;
        ext.ffcs = xe->fenc_chroma_frame_stride;
        ext.rcs = xe->ref_chroma_stride;
        ext.rfcs = xe->ref_chroma_frame_stride;
        mode = cf == 3 ? 2 : 1;
    }
    else if( ext.wt[0].on )
        mode = 1;                                         // weighted luma, no chroma
    return hipSuccess;
}

template <int BD>
static hipError_t refine_launch( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                                 const typename PT<BD>::pixel *const planes[4], intptr_t rs, intptr_t rfs,
                                 int i_pixel, int subme, int kind, int fpel_satd, const int32_t *pos,
                                 const int16_t *par, const int32_t *init_cost, const uint16_t *cost_mv, int n,
                                 int32_t *out, int32_t *nevals, int nstride, int32_t *thr, const int32_t *rcost,
                                 const x264hip_refine_ext_t *xe, hipStream_t stream )
{
    if( n <= 0 )
        return hipSuccess;
    if( i_pixel < 0 || i_pixel > 6 || subme < 1 || subme > 11 || kind < 0 || kind > 2 || ((uintptr_t)out & 15) )
        return hipErrorInvalidValue;
    // kind 0: x264_me_search_ref's refine (me.c:794-796), 1: x264_me_refine_qpel (:801-810),
    // 2: x264_me_refine_qpel_refdupe (:812-815)
    const int refine_qpel = kind == 1;
    const int hpel = kind == 2 ? 0 : k_subpel_iterations[subme][refine_qpel ? 0 : 2];
    const int qpel = kind == 2 ? min( 2, (int)k_subpel_iterations[subme][3] )
                               : k_subpel_iterations[subme][refine_qpel ? 1 : 3];
    // fpelcmp is SATD only under TESA with subme > 1 (encoder.c:1423-1426)
    const bool fs_satd = fpel_satd && subme > 1;
    RsExt<BD> ext;
    int mode;
    if( rs_ext<BD>( xe, ext, mode ) != hipSuccess )
        return hipErrorInvalidValue;
    // 4 * (the partition's tiles) lanes per partition (me_refine_subpel_kernel's segments)
    const int64_t lanes = (int64_t)n * 4 * part_tiles( i_pixel );
    dim3 blk( 256 ), g( (unsigned)((lanes + 255) / 256) );
#define RS_GO( I, F, E )                                                                                          \
    hipLaunchKernelGGL( ( me_refine_subpel_kernel<BD, I, F, E> ), g, blk, 0, stream, fenc, fs, ffs, planes[0],    \
                        planes[1], planes[2], planes[3], rs, rfs, n, hpel, qpel, subme, refine_qpel ? 1 : 0, pos,   \
                        par, init_cost, cost_mv, out, nevals, nstride, thr, rcost, ext )
#define RS_MODE( I, F )                                                                                           \
    if( mode == 0 ) { RS_GO( I, F, 0 ); } else if( mode == 1 ) { RS_GO( I, F, 1 ); } else { RS_GO( I, F, 2 ); }
#define RS_CASE( I )                                                                                              \
    case I:                                                                                                       \
        if( fs_satd ) { RS_MODE( I, true ); } else { RS_MODE( I, false ); }                                       \
        break;
    switch( i_pixel )
    {
        RS_CASE( 0 ) RS_CASE( 1 ) RS_CASE( 2 ) RS_CASE( 3 ) RS_CASE( 4 ) RS_CASE( 5 ) RS_CASE( 6 )
        default: return hipErrorInvalidValue;
    }
#undef RS_CASE
#undef RS_MODE
#undef RS_GO
    return hipGetLastError();
}

template <int BD>
hipError_t launch_me_refine_subpel( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                                    const typename PT<BD>::pixel *const planes[4], intptr_t rs, intptr_t rfs,
                                    int i_pixel, int subme, int kind, int fpel_satd, const int32_t *pos,
                                    const int16_t *par, const int32_t *init_cost, const uint16_t *cost_mv, int n,
                                    int32_t *out, int32_t *nevals, int32_t *thr, const int32_t *rcost,
                                    const x264hip_refine_ext_t *xe, hipStream_t stream )
{
    return refine_launch<BD>( fenc, fs, ffs, planes, rs, rfs, i_pixel, subme, kind, fpel_satd, pos, par,
                              init_cost, cost_mv, n, out, nevals, 1, thr, rcost, xe, stream );
}

// ---------------------------------------------------------------------------------------------
// x264_me_search_ref's integer stage (reference encoder/me.c:182-789) for a batch of partitions:
// the predictor checks (:214-318), DIA (:322-342), HEX (:344-419) or UMH (:422-616, then its
// me_hex2), and the qpel conversion; refine_subpel follows as the kernel above (launch_me_search_ref).
// The lane layout is refine_subpel's: a segment of 4 * NT lanes per partition, four groups of NT
// tile lanes, group g scoring the step's candidate g (fpelcmp = SAD of the 8x4 tiles on p_fref_w,
// or COST_MV_HPEL's get_ref of the hpel planes weighted by m->weight[0]).  Every step's
// candidates are scored together and then taken in the reference's order with its strict-<
// updates, so a step of up to four COST_MV / COST_MV_X3 / X4 calls is one evaluation; the
// searches' control flow is per segment (each segment's lanes hold the same state), the
// segments of a wave stepping through their own paths.  Lists whose length depends on the
// state -- the predictors (x264_predictor_clip / _roundclip drop zero and pmv-equal entries),
// UMH's cross and hexagon grid (range checks) -- are walked as slots, a slot outside the mv
// range not scored (and not read: it may lie past the padding).
namespace {
constexpr int SR_MVC = 14;                                // candidates per partition (mvc_temp+2 of me.c:195)
__device__ __forceinline__ uint32_t sr_pack( int a, int b ) { return (uint32_t)(uint16_t)a | ((uint32_t)(uint16_t)b << 16); }
__device__ __forceinline__ int sr_clip( int v, int lo, int hi ) { return min( max( v, lo ), hi ); }
// hex2 (me.c:55), square1 (:56) and hex4 (:534-539) as bit fields (offset + bias)
constexpr uint8_t k_hex2x[8] = { 1, 0, 1, 3, 4, 3, 1, 0 }, k_hex2y[8] = { 0, 2, 4, 4, 2, 0, 0, 2 };   // +2
constexpr uint8_t k_sq1x[9] = { 1, 1, 1, 0, 2, 0, 0, 2, 2 }, k_sq1y[9] = { 1, 0, 2, 1, 1, 0, 2, 0, 2 };  // +1
constexpr uint8_t k_mod6m1[8] = { 5, 0, 1, 2, 3, 4, 5, 0 };
constexpr uint8_t k_hex4x0[8] = { 4, 4, 2, 6, 0, 8, 0, 8 }, k_hex4x1[8] = { 0, 8, 0, 8, 0, 8, 2, 6 };   // +4
constexpr uint8_t k_hex4y0[8] = { 0, 8, 1, 1, 2, 2, 3, 3 }, k_hex4y1[8] = { 4, 4, 5, 5, 6, 6, 7, 7 };   // +4
constexpr uint8_t k_psize_shift[7] = { 0, 1, 1, 2, 3, 3, 4 };
}

// the lane's full-pel tile SAD at four adjacent candidate columns x0 .. x0+3 of one row: one
// window load per tile row (TW + 3 pixels), each candidate's row realigned from it
template <int BD, int TW>
__device__ __forceinline__ void sad4_tile( const uint32_t (&fa)[4][8 / PT<BD>::PPD], const typename PT<BD>::pixel *q,
                                           intptr_t rs, uint32_t (&acc)[4] )
{
    constexpr int PPD = PT<BD>::PPD, LW = TW / PPD;                  // words of a tile row
    constexpr int NW = (TW + 3 + PPD - 1) / PPD;                      // words of the window
    constexpr int BPP = 4 / PPD;                                      // bytes per pixel
#pragma unroll
    for( int k = 0; k < 4; k++ )
        acc[k] = 0;
#pragma unroll
    for( int y = 0; y < 4; y++ )
    {
        uint32_t t[NW], w[NW + 1];
        load_al_pad<NW>( q + y * rs, t );
#pragma unroll
        for( int i = 0; i < NW; i++ )
            w[i] = t[i];
        w[NW] = 0;
#pragma unroll
        for( int k = 0; k < 4; k++ )
        {
            const int sh = k * BPP, o = sh / 4, sub = sh % 4;
#pragma unroll
            for( int i = 0; i < LW; i++ )
            {
                const uint32_t wk = sub ? __builtin_amdgcn_alignbyte( w[i + o + 1], w[i + o], sub ) : w[i + o];
                acc[k] = sadp<BD>( fa[y][i], wk, acc[k] );
            }
        }
    }
}

template <int BD, int IPIX, bool WGT, bool ESA>
__global__ __launch_bounds__( 256 ) void me_search_ref_kernel(
    const typename PT<BD>::pixel *__restrict__ fenc, intptr_t fs, intptr_t ffs, const typename PT<BD>::pixel *fw,
    const typename PT<BD>::pixel *p0, const typename PT<BD>::pixel *p1, const typename PT<BD>::pixel *p2,
    const typename PT<BD>::pixel *p3, intptr_t rs, intptr_t rfs, int n, int me_method, int subme, int me_range,
    const int32_t *__restrict__ pos, const int16_t *__restrict__ par, const int16_t *__restrict__ mvc,
    const uint16_t *__restrict__ cost_mv, const RsWeight wt0, int32_t *__restrict__ out,
    int16_t *__restrict__ rpar, int32_t *__restrict__ rinit, int32_t *__restrict__ nevals )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int HDW = 8 / PT<BD>::PPD;
    constexpr int BW = pix_w( IPIX ), TW = tile_w<IPIX>(), TX = BW / TW, NT = tile_n<IPIX>();
    constexpr int SL = 4 * NT, SH = ilog2( SL );
    constexpr int COST_MAX = 1 << 28;
    const int lane = (int)(threadIdx.x & 63);
    const int sbase = lane & (64 - SL);
    const int g = (lane / NT) & 3, u = lane & (NT - 1);
    const int64_t jo = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> SH;
    const bool live = jo < n;
    const int64_t j = live ? jo : n - 1;
    const int ux = TW * (u % TX), uy = 4 * (u / TX);
    const int f = pos[3 * j], bx = pos[3 * j + 1], by = pos[3 * j + 2];

    uint32_t fa[4][HDW];
    load_fenc_tile<BD, TW>( fenc + f * ffs + (intptr_t)(by + uy) * fs + bx + ux, fs, fa );
    const intptr_t qo = (intptr_t)f * rfs + (intptr_t)(by + uy) * rs + bx + ux;
    const pixel *const q0 = p0 + qo, *const q1 = p1 + qo, *const q2 = p2 + qo, *const q3 = p3 + qo;
    const pixel *const qw = fw + qo;

    const int16_t *p = par + 12 * j;
    const int mvpx = p[0], mvpy = p[1];
    const int xmin = p[2], ymin = p[3], xmax = p[4], ymax = p[5];
    const int i_mvc = min( (int)p[10], SR_MVC );
    const int16_t *mc = mvc + 2 * SR_MVC * j;
    const uint16_t *cmx = cost_mv - mvpx, *cmy = cost_mv - mvpy;
    int nf = 0, nh = 0;                                   // the reference's fpelcmp / get_ref calls

    // mode 0: fpelcmp on p_fref_w + BITS_MVD; 1: COST_MV_HPEL (get_ref + qpel mv cost); 2: fpelcmp
    // alone.  Group g scores (gx, gy) (not read when !ok); c[k] = group k's cost.
    auto evalc = [&]( int gx, int gy, int mode, bool ok, int (&c)[4] ) __attribute__( ( always_inline ) ) {
        uint32_t v = 0;
        if( ok )
        {
            if( mode == 1 )
            {
                v = tile_cost<BD, false, WGT, TW>( fa, q0, q1, q2, q3, rs, gx, gy, wt0 );
                if( u == 0 )
                    v += (uint32_t)cmx[gx] + (uint32_t)cmy[gy];
            }
            else
            {
                v = tile_cost<BD, false, false, TW>( fa, qw, qw, qw, qw, rs, 4 * gx, 4 * gy );
                if( u == 0 && mode == 0 )
                    v += (uint32_t)cmx[4 * gx] + (uint32_t)cmy[4 * gy];
            }
        }
        v = group_sum<NT>( v );
#pragma unroll
        for( int k = 0; k < 4; k++ )
            c[k] = (int)__shfl( (int)v, sbase + NT * k );
    };
    auto in_range = [&]( int mx, int my ) __attribute__( ( always_inline ) ) { return mx >= xmin && mx <= xmax && my >= ymin && my <= ymax; };

    int bmx, bmy, bcost = COST_MAX, bpred_cost = COST_MAX, pmx, pmy;
    uint32_t pmv, bpred_mv = 0;
    int c[4];
    auto upd = [&]( int cc, int mx, int my ) __attribute__( ( always_inline ) ) {
        nf++;
        if( cc < bcost )
        {
            bcost = cc;
            bmx = mx;
            bmy = my;
        }
    };
    // the want-th entry of x264_predictor_clip (qpel) / _roundclip (fpel) over the mvc list
    auto pred = [&]( int want, int &ox, int &oy ) __attribute__( ( always_inline ) ) {
        int cnt = 0;
        bool found = false;
        for( int i = 0; i < i_mvc && !found; i++ )
        {
            int mx = mc[2 * i], my = mc[2 * i + 1];
            if( subme < 3 )
            {
                mx = (mx + 2) >> 2;
                my = (my + 2) >> 2;
            }
            const uint32_t v = sr_pack( mx, my );
            if( !v || v == pmv )
                continue;
            if( cnt == want )
            {
                found = true;
                ox = subme >= 3 ? sr_clip( mx, 4 * xmin, 4 * xmax ) : sr_clip( mx, xmin, xmax );
                oy = subme >= 3 ? sr_clip( my, 4 * ymin, 4 * ymax ) : sr_clip( my, ymin, ymax );
            }
            cnt++;
        }
        return found;
    };
    auto nvalid = [&]() __attribute__( ( always_inline ) ) {
        int cnt = 0;
        for( int i = 0; i < i_mvc; i++ )
        {
            int mx = mc[2 * i], my = mc[2 * i + 1];
            if( subme < 3 )
            {
                mx = (mx + 2) >> 2;
                my = (my + 2) >> 2;
            }
            const uint32_t v = sr_pack( mx, my );
            cnt += v && v != pmv;
        }
        return cnt;
    };

    if( subme >= 3 )
    {
        int bpx = sr_clip( mvpx, 4 * xmin, 4 * xmax ), bpy = sr_clip( mvpy, 4 * ymin, 4 * ymax );
        pmv = sr_pack( bpx, bpy );
        pmx = (bpx + 2) >> 2;
        pmy = (bpy + 2) >> 2;
        evalc( bpx, bpy, 1, true, c );
        nh++;
        bpred_cost = c[0];
        const int pmv_cost = bpred_cost;
        const int nv = nvalid();
        if( nv > 0 )
        {
            bpred_cost <<= 4;
            for( int b = 0; b < nv; b += 4 )
            {
                int gx = 0, gy = 0;
                const bool ok = b + g < nv && pred( b + g, gx, gy );
                evalc( gx, gy, 1, ok, c );
#pragma unroll
                for( int k = 0; k < 4; k++ )
                    if( b + k < nv )
                    {
                        nh++;
                        if( (c[k] << 4) + b + k + 1 < bpred_cost )
                            bpred_cost = (c[k] << 4) + b + k + 1;
                    }
            }
            if( bpred_cost & 15 )
                pred( (bpred_cost & 15) - 1, bpx, bpy );
            bpred_cost >>= 4;
        }
        bmx = (bpx + 2) >> 2;
        bmy = (bpy + 2) >> 2;
        bpred_mv = sr_pack( bpx, bpy );
        // COST_MV( bmx, bmy ) of a subpel predictor and the zero vector, scored together
        const bool sub = bpred_mv & 0x00030003, zero = pmv && (bmx | bmy);
        evalc( g == 0 ? bmx : 0, g == 0 ? bmy : 0, 0, (g == 0 && sub) || (g == 1 && zero), c );
        if( sub )
            upd( c[0], bmx, bmy );
        else
            bcost = bpred_cost;
        if( pmv )
        {
            if( zero )
                upd( c[1], 0, 0 );
        }
        else if( pmv_cost < bcost )
        {
            bcost = pmv_cost;
            bmx = bmy = 0;
        }
    }
    else
    {
        bmx = pmx = sr_clip( (mvpx + 2) >> 2, xmin, xmax );
        bmy = pmy = sr_clip( (mvpy + 2) >> 2, ymin, ymax );
        pmv = sr_pack( bmx, bmy );
        evalc( bmx, bmy, 2, true, c );
        nf++;
        bcost = c[0];
        const int nv = nvalid();
        if( nv > 0 )
        {
            bcost <<= 4;
            for( int b = 0; b < nv; b += 4 )
            {
                int gx = 0, gy = 0;
                const bool ok = b + g < nv && pred( b + g, gx, gy );
                evalc( gx, gy, 0, ok, c );
#pragma unroll
                for( int k = 0; k < 4; k++ )
                    if( b + k < nv )
                    {
                        nf++;
                        if( (c[k] << 4) + b + k + 1 < bcost )
                            bcost = (c[k] << 4) + b + k + 1;
                    }
            }
            if( bcost & 15 )
                pred( (bcost & 15) - 1, bmx, bmy );
            bcost >>= 4;
        }
        if( pmv )
        {
            evalc( 0, 0, 0, true, c );
            upd( c[0], 0, 0 );
        }
    }

    // the diamond of radius 1 around (cx, cy) in COST_MV_X4's order (0,-1) (0,1) (-1,0) (1,0)
    auto dia = [&]( int cx, int cy ) __attribute__( ( always_inline ) ) {
        evalc( cx + (g == 2 ? -1 : g == 3 ? 1 : 0), cy + (g == 0 ? -1 : g == 1 ? 1 : 0), 0, true, c );
    };
    bool hex = !ESA && me_method == 1;
    int i_me_range = me_range;
    if( !ESA && me_method == 0 )
    {
        bcost <<= 4;
        int i = i_me_range;
        do
        {
            dia( bmx, bmy );
            nf += 4;
            if( (c[0] << 4) + 1 < bcost ) bcost = (c[0] << 4) + 1;
            if( (c[1] << 4) + 3 < bcost ) bcost = (c[1] << 4) + 3;
            if( (c[2] << 4) + 4 < bcost ) bcost = (c[2] << 4) + 4;
            if( (c[3] << 4) + 12 < bcost ) bcost = (c[3] << 4) + 12;
            if( !(bcost & 15) )
                break;
            bmx -= (int32_t)((uint32_t)bcost << 28) >> 30;
            bmy -= (int32_t)((uint32_t)bcost << 30) >> 30;
            bcost &= ~15;
        } while( --i && in_range( bmx, bmy ) );
        bcost >>= 4;
    }
    else if constexpr( ESA )                              // (its own instance: the other methods keep 5 waves)
    {
        // ESA (me.c:618-631, 750-768): every candidate of the window around the predictor stage's
        // (bmx, bmy), the width rounded up to a multiple of 4 (columns past max_x included), in
        // raster order with COST_MV's strict <.  The reference's successive elimination (ads on
        // the integral image) only skips candidates that cannot beat bcost, so the exhaustive
        // form it keeps under #if 0 (me.c:627-631) gives the same bcost / bmx / bmy; a round
        // scores four adjacent columns of one row (width is a multiple of 4)
        const int min_x = max( bmx - i_me_range, xmin ), min_y = max( bmy - i_me_range, ymin );
        const int max_x = min( bmx + i_me_range, xmax ), max_y = min( bmy + i_me_range, ymax );
        const int width = (max_x - min_x + 3) & ~3, nrows = width > 0 ? max( max_y - min_y + 1, 0 ) : 0;
        // the first minimum in raster order is the least (cost, raster index) key, so the
        // candidates may be scored in any order: group g takes rows g, g + 4, ..., a lane four
        // columns of its row per round (one window load per tile row)
        uint64_t best = ~0ull;
        for( int r0 = 0; __any( r0 < nrows ); r0 += 4 )
        {
            const int r = r0 + g, my = min_y + r;
            for( int cx = 0; __any( r0 < nrows && cx < width ); cx += 4 )
            {
                const bool ok = r < nrows && cx < width;
                uint32_t sa[4] = { 0, 0, 0, 0 };
                if( ok )
                    sad4_tile<BD, TW>( fa, qw + (intptr_t)my * rs + min_x + cx, rs, sa );
#pragma unroll
                for( int k = 0; k < 4; k++ )
                    sa[k] = group_sum<NT>( sa[k] );
                if( ok && u == 0 )
                {
                    const uint32_t cy = cmy[4 * my], rbase = (uint32_t)(r * width + cx);
#pragma unroll
                    for( int k = 0; k < 4; k++ )
                    {
                        const uint32_t cost = sa[k] + cmx[4 * (min_x + cx + k)] + cy;
                        const uint64_t key = ((uint64_t)cost << 32) | (rbase + k);
                        best = key < best ? key : best;
                    }
                }
            }
        }
        // the segment's groups meet (lane u == 0 of each group holds its rows' best)
        uint64_t seg = ~0ull;
#pragma unroll
        for( int k = 0; k < 4; k++ )
        {
            const int src = sbase + NT * k;
            const uint64_t o = ((uint64_t)(uint32_t)__shfl( (int)(best >> 32), src ) << 32) |
                               (uint32_t)__shfl( (int)(uint32_t)best, src );
            seg = o < seg ? o : seg;
        }
        best = seg;
        nf += width * nrows;
        if( best != ~0ull && (int)(best >> 32) < bcost )
        {
            const int ri = (int)(uint32_t)best;
            bcost = (int)(best >> 32);
            bmy = min_y + ri / width;
            bmx = min_x + ri % width;
        }
    }
    else if( me_method == 2 )
    {
        // UMH (me.c:422-616)
        auto dia1 = [&]( int cx, int cy ) __attribute__( ( always_inline ) ) {
            dia( cx, cy );
            upd( c[0], cx, cy - 1 );
            upd( c[1], cx, cy + 1 );
            upd( c[2], cx - 1, cy );
            upd( c[3], cx + 1, cy );
        };
        auto thresh = [&]( int v ) __attribute__( ( always_inline ) ) { return bcost < (v >> k_psize_shift[IPIX]); };
        int omx, omy;
        // CROSS( start, x_max, y_max ) around (omx, omy) (me.c:152-176): slot 2k / 2k+1 = +i / -i
        auto cross = [&]( int start, int x_max, int y_max ) __attribute__( ( always_inline ) ) {
            const int nhs = x_max > start ? 2 * ((x_max - start + 1) >> 1) : 0;
            const int nvs = y_max > start ? 2 * ((y_max - start + 1) >> 1) : 0;
            auto slot = [&]( int sl, int &mx, int &my ) __attribute__( ( always_inline ) ) {
                const bool v = sl >= nhs;
                const int s2 = v ? sl - nhs : sl;
                const int d = (start + 2 * (s2 >> 1)) * ((s2 & 1) ? -1 : 1);
                mx = omx + (v ? 0 : d);
                my = omy + (v ? d : 0);
                // CROSS checks the moving axis only (me.c:160-173): omx / omy may lie a step past the
                // other axis' limit (DIA1_ITER scores pmx +- 1, pmy +- 1 unchecked)
                const int a = v ? my : mx, lo = v ? ymin : xmin, hi = v ? ymax : xmax;
                return sl < nhs + nvs && (d > 0 ? a <= hi : a >= lo);
            };
            for( int b = 0; b < nhs + nvs; b += 4 )
            {
                int gx, gy;
                const bool ok = slot( b + g, gx, gy );
                evalc( gx, gy, 0, ok, c );
#pragma unroll
                for( int k = 0; k < 4; k++ )
                {
                    int mx, my;
                    if( slot( b + k, mx, my ) )
                        upd( c[k], mx, my );
                }
            }
        };
        int cross_start = 1;
        const int ucost1 = bcost;
        dia1( pmx, pmy );
        if( pmx | pmy )
            dia1( 0, 0 );
        if constexpr( IPIX == 6 )                         // PIXEL_4x4: goto me_hex2 (me.c:438-439)
            hex = true;
        else
        {
        const int ucost2 = bcost;
        if( (bmx | bmy) && ((bmx - pmx) | (bmy - pmy)) )
            dia1( bmx, bmy );
        if( bcost == ucost2 )
            cross_start = 3;
        omx = bmx;
        omy = bmy;
        bool done = false;
        if( bcost == ucost2 && thresh( 2000 ) )
        {
            // COST_MV_X4( 0,-2, -1,-1, 1,-1, -2,0 ), COST_MV_X4( 2,0, -1,1, 1,1, 0,2 )
            evalc( omx + (g == 0 ? 0 : g == 1 ? -1 : g == 2 ? 1 : -2), omy + (g == 0 ? -2 : g == 3 ? 0 : -1), 0, true,
                   c );
            upd( c[0], omx, omy - 2 );
            upd( c[1], omx - 1, omy - 1 );
            upd( c[2], omx + 1, omy - 1 );
            upd( c[3], omx - 2, omy );
            evalc( omx + (g == 0 ? 2 : g == 1 ? -1 : g == 2 ? 1 : 0), omy + (g == 0 ? 0 : g == 3 ? 2 : 1), 0, true,
                   c );
            upd( c[0], omx + 2, omy );
            upd( c[1], omx - 1, omy + 1 );
            upd( c[2], omx + 1, omy + 1 );
            upd( c[3], omx, omy + 2 );
            if( bcost == ucost1 && thresh( 500 ) )
                done = true;
            else if( bcost == ucost2 )
            {
                const int range = (i_me_range >> 1) | 1;
                cross( 3, range, range );
                // COST_MV_X4( -1,-2, 1,-2, -2,-1, 2,-1 ), COST_MV_X4( -2,1, 2,1, -1,2, 1,2 )
                evalc( omx + (g == 0 ? -1 : g == 1 ? 1 : g == 2 ? -2 : 2), omy + (g < 2 ? -2 : -1), 0, true, c );
                upd( c[0], omx - 1, omy - 2 );
                upd( c[1], omx + 1, omy - 2 );
                upd( c[2], omx - 2, omy - 1 );
                upd( c[3], omx + 2, omy - 1 );
                evalc( omx + (g == 0 ? -2 : g == 1 ? 2 : g == 2 ? -1 : 1), omy + (g < 2 ? 1 : 2), 0, true, c );
                upd( c[0], omx - 2, omy + 1 );
                upd( c[1], omx + 2, omy + 1 );
                upd( c[2], omx - 1, omy + 2 );
                upd( c[3], omx + 1, omy + 2 );
                if( bcost == ucost2 )
                    done = true;
                cross_start = range + 2;
            }
        }
        if( !done )
        {
            if( i_mvc )
            {
                // the adaptive range (me.c:469-519; x264_predictor_difference, common/base.h:248-257)
                int mvd, denom = 1;
                if( i_mvc == 1 )
                    mvd = IPIX == 0 ? 25 : abs( mvpx - mc[0] ) + abs( mvpy - mc[1] );
                else
                {
                    denom = i_mvc - 1;
                    mvd = 0;
                    if( IPIX != 0 )
                    {
                        mvd = abs( mvpx - mc[0] ) + abs( mvpy - mc[1] );
                        denom++;
                    }
                    for( int i = 0; i < i_mvc - 1; i++ )
                        mvd += abs( mc[2 * i] - mc[2 * i + 2] ) + abs( mc[2 * i + 1] - mc[2 * i + 3] );
                }
                const int sad_ctx = thresh( 1000 ) ? 0 : thresh( 2000 ) ? 1 : thresh( 4000 ) ? 2 : 3;
                const int mvd_ctx = mvd < 10 * denom ? 0 : mvd < 20 * denom ? 1 : mvd < 40 * denom ? 2 : 3;
                // range_mul[mvd_ctx][sad_ctx] (me.c:474-480) as 4-bit fields
                constexpr uint32_t rm[4] = { 0x4433u, 0x4443u, 0x5444u, 0x6544u };
                const uint32_t row = mvd_ctx == 0 ? rm[0] : mvd_ctx == 1 ? rm[1] : mvd_ctx == 2 ? rm[2] : rm[3];
                i_me_range = i_me_range * (int)((row >> (4 * sad_ctx)) & 15) >> 2;
            }
            cross( cross_start, i_me_range, i_me_range >> 1 );
            // COST_MV_X4( -2,-2, -2,2, 2,-2, 2,2 )
            evalc( omx + (g < 2 ? -2 : 2), omy + ((g & 1) ? 2 : -2), 0, true, c );
            upd( c[0], omx - 2, omy - 2 );
            upd( c[1], omx - 2, omy + 2 );
            upd( c[2], omx + 2, omy - 2 );
            upd( c[3], omx + 2, omy + 2 );
            // hexagon grid (me.c:527-612): 16 points per ring, range-checked
            omx = bmx;
            omy = bmy;
            int i = 1;
            do
            {
#pragma unroll
                for( int e = 0; e < 4; e++ )
                {
                    // ring points 4e .. 4e+3 (hex4 as 4-bit fields, +4)
                    constexpr uint32_t hx[2] = { pack_fields( k_hex4x0, 4 ), pack_fields( k_hex4x1, 4 ) };
                    constexpr uint32_t hy[2] = { pack_fields( k_hex4y0, 4 ), pack_fields( k_hex4y1, 4 ) };
                    const int gx = omx + (field( hx[e >> 1], 4, 4 * (e & 1) + g ) - 4) * i;
                    const int gy = omy + (field( hy[e >> 1], 4, 4 * (e & 1) + g ) - 4) * i;
                    evalc( gx, gy, 0, in_range( gx, gy ), c );
#pragma unroll
                    for( int k = 0; k < 4; k++ )
                    {
                        const int kx = omx + (field( hx[e >> 1], 4, 4 * (e & 1) + k ) - 4) * i;
                        const int ky = omy + (field( hy[e >> 1], 4, 4 * (e & 1) + k ) - 4) * i;
                        if( in_range( kx, ky ) )
                            upd( c[k], kx, ky );
                    }
                }
            } while( ++i <= i_me_range >> 2 );
            hex = in_range( bmx, bmy );
        }
        }
    }
    if( hex )
    {
        // hexagon (me.c:344-403): COST_MV_X3_DIR( -2,0, -1,2, 1,2 ), COST_MV_X3_DIR( 2,0, 1,-2, -1,-2 )
        constexpr uint32_t h2x = pack_fields( k_hex2x, 3 ), h2y = pack_fields( k_hex2y, 3 );
        evalc( bmx + (g == 0 ? -2 : g == 1 ? -1 : g == 2 ? 1 : 2), bmy + (g == 0 || g == 3 ? 0 : 2), 0, true, c );
        int c2[4];
        evalc( bmx + (g == 0 ? 1 : -1), bmy - 2, 0, g < 2, c2 );
        nf += 6;
        bcost <<= 3;
        if( (c[0] << 3) + 2 < bcost ) bcost = (c[0] << 3) + 2;
        if( (c[1] << 3) + 3 < bcost ) bcost = (c[1] << 3) + 3;
        if( (c[2] << 3) + 4 < bcost ) bcost = (c[2] << 3) + 4;
        if( (c[3] << 3) + 5 < bcost ) bcost = (c[3] << 3) + 5;
        if( (c2[0] << 3) + 6 < bcost ) bcost = (c2[0] << 3) + 6;
        if( (c2[1] << 3) + 7 < bcost ) bcost = (c2[1] << 3) + 7;
        if( bcost & 7 )
        {
            int dir = (bcost & 7) - 2;
            bmx += field( h2x, 3, dir + 1 ) - 2;
            bmy += field( h2y, 3, dir + 1 ) - 2;
            for( int i = (i_me_range >> 1) - 1; i > 0 && in_range( bmx, bmy ); i-- )
            {
                // COST_MV_X3_DIR( hex2[dir], hex2[dir+1], hex2[dir+2] )
                const int d = dir + (g < 3 ? g : 0);
                evalc( bmx + field( h2x, 3, d ) - 2, bmy + field( h2y, 3, d ) - 2, 0, g < 3, c );
                nf += 3;
                bcost &= ~7;
                if( (c[0] << 3) + 1 < bcost ) bcost = (c[0] << 3) + 1;
                if( (c[1] << 3) + 2 < bcost ) bcost = (c[1] << 3) + 2;
                if( (c[2] << 3) + 3 < bcost ) bcost = (c[2] << 3) + 3;
                if( !(bcost & 7) )
                    break;
                dir += (bcost & 7) - 2;
                dir = field( pack_fields( k_mod6m1, 3 ), 3, dir + 1 );
                bmx += field( h2x, 3, dir + 1 ) - 2;
                bmy += field( h2y, 3, dir + 1 ) - 2;
            }
        }
        bcost >>= 3;
        // square refine (me.c:404-418)
        bcost <<= 4;
        dia( bmx, bmy );
        if( (c[0] << 4) + 1 < bcost ) bcost = (c[0] << 4) + 1;
        if( (c[1] << 4) + 2 < bcost ) bcost = (c[1] << 4) + 2;
        if( (c[2] << 4) + 3 < bcost ) bcost = (c[2] << 4) + 3;
        if( (c[3] << 4) + 4 < bcost ) bcost = (c[3] << 4) + 4;
        evalc( bmx + (g < 2 ? -1 : 1), bmy + ((g & 1) ? 1 : -1), 0, true, c );
        if( (c[0] << 4) + 5 < bcost ) bcost = (c[0] << 4) + 5;
        if( (c[1] << 4) + 6 < bcost ) bcost = (c[1] << 4) + 6;
        if( (c[2] << 4) + 7 < bcost ) bcost = (c[2] << 4) + 7;
        if( (c[3] << 4) + 8 < bcost ) bcost = (c[3] << 4) + 8;
        nf += 8;
        constexpr uint32_t s1x = pack_fields( k_sq1x, 2 ), s1y = pack_fields( k_sq1y, 2 );
        bmx += field( s1x, 2, bcost & 15 ) - 1;
        bmy += field( s1y, 2, bcost & 15 ) - 1;
        bcost >>= 4;
    }

    // -> qpel mv (me.c:774-789)
    int mx, my, cst, cmv;
    if( subme < 3 )
    {
        cmv = (int)cmx[4 * bmx] + (int)cmy[4 * bmy];
        cst = bcost + (sr_pack( bmx, bmy ) == pmv ? cmv : 0);
        mx = 4 * bmx;
        my = 4 * bmy;
    }
    else
    {
        if( bpred_cost < bcost )
        {
            mx = (int16_t)(bpred_mv & 0xffff);
            my = (int16_t)(bpred_mv >> 16);
        }
        else
        {
            mx = 4 * bmx;
            my = 4 * bmy;
        }
        cst = min( bpred_cost, bcost );
        cmv = (int)cmx[mx] + (int)cmy[my];
    }
    if( live && lane == sbase )
    {
        if( !rpar )                                       // (with the refine, out is the refine's)
            *(int4 *)(out + 4 * j) = make_int4( cst, mx, my, cmv );
        else
        {
            *(int4 *)(rpar + 8 * j) = make_int4( (int)sr_pack( mx, my ), (int)sr_pack( mvpx, mvpy ),
                                                 (int)sr_pack( p[6], p[7] ), (int)sr_pack( p[8], p[9] ) );
            rinit[j] = cst;
        }
        if( nevals )
        {
            nevals[2 * j] = nf | (nh << 16);
            if( subme < 2 )
                nevals[2 * j + 1] = 0;                    // no refine_subpel (me.c:792)
        }
    }
}

template <int BD>
hipError_t launch_me_search_ref( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                                 const typename PT<BD>::pixel *fw, const typename PT<BD>::pixel *const planes[4],
                                 intptr_t rs, intptr_t rfs, int i_pixel, int me_method, int subme, int me_range,
                                 const int32_t *pos, const int16_t *par, const int16_t *mvc, const uint16_t *cost_mv,
                                 int n, int32_t *out, int32_t *nevals, int32_t *thr, const int32_t *rcost,
                                 const x264hip_refine_ext_t *xe, hipStream_t stream )
{
    if( n <= 0 )
        return hipSuccess;
    if( i_pixel < 0 || i_pixel > 6 || me_method < 0 || me_method > 3 || subme < 1 || subme > 11 || me_range < 4 ||
        me_range > 64 || ((uintptr_t)out & 15) )
        return hipErrorInvalidValue;
    RsExt<BD> ext;
    int mode;
    if( rs_ext<BD>( xe, ext, mode ) != hipSuccess )
        return hipErrorInvalidValue;
    const bool refine = subme >= 2;
    void *buf = nullptr;
    int16_t *rpar = nullptr;
    int32_t *rinit = nullptr;
    hipError_t e = hipSuccess;
    if( refine )
    {
        if( (e = scratch_alloc( &buf, (size_t)n * 20 + 16, stream )) != hipSuccess )
            return e;
        rpar = (int16_t *)buf;
        rinit = (int32_t *)((char *)buf + (size_t)n * 16);
    }
    const int64_t lanes = (int64_t)n * 4 * part_tiles( i_pixel );
    dim3 blk( 256 ), g( (unsigned)((lanes + 255) / 256) );
#define SR_GO( I, W )                                                                                             \
    if( me_method == 3 )                                                                                          \
        hipLaunchKernelGGL( ( me_search_ref_kernel<BD, I, W, true> ), g, blk, 0, stream, fenc, fs, ffs, fw,       \
                            planes[0], planes[1], planes[2], planes[3], rs, rfs, n, me_method, subme, me_range,   \
                            pos, par, mvc, cost_mv, ext.wt[0], out, rpar, rinit, nevals );                        \
    else                                                                                                          \
    hipLaunchKernelGGL( ( me_search_ref_kernel<BD, I, W, false> ), g, blk, 0, stream, fenc, fs, ffs, fw, planes[0], \
                        planes[1], planes[2], planes[3], rs, rfs, n, me_method, subme, me_range, pos, par, mvc,     \
                        cost_mv, ext.wt[0], out, rpar, rinit, nevals )
#define SR_CASE( I )                                                                                              \
    case I:                                                                                                       \
        if( ext.wt[0].on ) { SR_GO( I, true ); } else { SR_GO( I, false ); }                                      \
        break;
    switch( i_pixel )
    {
        SR_CASE( 0 ) SR_CASE( 1 ) SR_CASE( 2 ) SR_CASE( 3 ) SR_CASE( 4 ) SR_CASE( 5 ) SR_CASE( 6 )
        default: break;
    }
#undef SR_CASE
#undef SR_GO
    e = hipGetLastError();
    if( e == hipSuccess && refine )
        e = refine_launch<BD>( fenc, fs, ffs, planes, rs, rfs, i_pixel, subme, 0, 0, pos, rpar, rinit, cost_mv, n, out,
                               nevals ? nevals + 1 : nullptr, 2, thr, rcost, xe, stream );
    if( buf )
    {
        const hipError_t ef = hipFreeAsync( buf, stream );
        if( e == hipSuccess )
            e = ef;
    }
    return e;
}
// ---------------------------------------------------------------------------------------------
// x264_me_refine_bidir_satd (reference encoder/me.c:994-1183, rd = 0) for a batch of bipred
// partitions.  A segment of 8 groups x NT tile lanes per partition (16x16: a wave; 8x8: 16
// lanes); a pass's 33 (or 32) dia4d pairs run as rounds of eight, group g scoring pair 8r + g:
// each lane rebuilds both lists' get_ref blocks of its 8x4 tile (mc.c:221-249, unweighted),
// averages them as mc.avg[i_pixel] does (the rounding average at i_weight 32, else
// pixel_avg_weight_wxh, mc.c:77-99) and scores the tile against fenc with mbcmp; the groups meet
// by DPP and shuffles and every lane replays COPY2_IF_LT in j order.  The visited bits (one per
// (m0x, m0y, m1x, m1y) mod 8, 4096 per partition) sit in LDS: a pass never revisits a pair of
// its own (dia4d's offsets are within +-1, so two pairs of one pass never alias mod 8), so a
// round reads the bits before its own are set.
__constant__ uint8_t c_dia4d[33] = {               // me.c:1064-1075, (d + 1) in 2-bit fields
    0x55, 0x95, 0x15, 0x65, 0x45, 0x59, 0x51, 0x56, 0x54, 0xA5, 0x05, 0x69, 0x41, 0x5A, 0x50, 0x96, 0x14,
    0x99, 0x11, 0x66, 0x44, 0x85, 0x25, 0x61, 0x49, 0x58, 0x52, 0x16, 0x94, 0x91, 0x19, 0x64, 0x46 };
__device__ __forceinline__ int dia4d( int j, int c ) { return (int)((c_dia4d[j] >> (2 * c)) & 3) - 1; }

// the lane's 8x4 tile of get_ref( mvx, mvy ) (unweighted)
template <int BD>
__device__ __forceinline__ void ref_tile( const typename PT<BD>::pixel *q0, const typename PT<BD>::pixel *q1,
                                          const typename PT<BD>::pixel *q2, const typename PT<BD>::pixel *q3,
                                          intptr_t rs, int mvx, int mvy, uint32_t (&r1)[4][8 / PT<BD>::PPD] )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int HDW = 8 / PT<BD>::PPD;
    const int idx = ((mvy & 3) << 2) + (mvx & 3);
    const intptr_t off = (intptr_t)(mvy >> 2) * rs + (mvx >> 2);
    constexpr uint32_t k0 = pack_fields( c_ref0, 2 ), k1 = pack_fields( c_ref1, 2 );
    const int i0 = field( k0, 2, idx ), i1 = field( k1, 2, idx );
    const pixel *s1 = (i0 == 0 ? q0 : i0 == 1 ? q1 : i0 == 2 ? q2 : q3) + off + ((mvy & 3) == 3) * rs;
    const pixel *s2 = (i1 == 0 ? q0 : i1 == 1 ? q1 : i1 == 2 ? q2 : q3) + off + ((mvx & 3) == 3);
#pragma unroll
    for( int y = 0; y < 4; y++ )
        load_al_pad<HDW>( s1 + y * rs, r1[y] );
    if( idx & 5 )
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
}

template <int BD, int IPIX, bool SATD>
__global__ __launch_bounds__( 256 ) void me_refine_bidir_kernel(
    const typename PT<BD>::pixel *__restrict__ fenc, intptr_t fs, intptr_t ffs, const typename PT<BD>::pixel *a0,
    const typename PT<BD>::pixel *a1, const typename PT<BD>::pixel *a2, const typename PT<BD>::pixel *a3,
    const typename PT<BD>::pixel *b0, const typename PT<BD>::pixel *b1, const typename PT<BD>::pixel *b2,
    const typename PT<BD>::pixel *b3, intptr_t rs, intptr_t rfs, int n, const int32_t *__restrict__ pos,
    const int16_t *__restrict__ par, const int32_t *__restrict__ weight, const uint16_t *__restrict__ cost_mv,
    int32_t *__restrict__ out, int32_t *__restrict__ cost, int32_t *__restrict__ nevals )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int HDW = 8 / PT<BD>::PPD, PPD = PT<BD>::PPD;
    constexpr int BW = pix_w( IPIX ), TW = tile_w<IPIX>(), TX = BW / TW, NT = tile_n<IPIX>();
    constexpr int SL = 8 * NT, SH = ilog2( SL );
    constexpr int COST_MAX = 1 << 28, NONE = 0x7fffffff;
    __shared__ uint32_t s_vis[256 / SL][128];
    const int lane = (int)(threadIdx.x & 63);
    const int sbase = lane & (64 - SL), seg = (int)threadIdx.x >> SH;
    const int g = (lane / NT) & 7, u = lane & (NT - 1);
    const int64_t jo = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> SH;
    const bool live = jo < n;
    const int64_t j = live ? jo : n - 1;
    const int ux = TW * (u % TX), uy = 4 * (u / TX);
    const int f = pos[3 * j], bx = pos[3 * j + 1], by = pos[3 * j + 2];

    uint32_t fa[4][HDW];
    load_fenc_tile<BD, TW>( fenc + f * ffs + (intptr_t)(by + uy) * fs + bx + ux, fs, fa );
    uint32_t hr[16];                                      // SATD: the tile's biased Hadamards, once
    if constexpr( SATD )
        had8x4_biased<BD>( fa, hr );
    const intptr_t qo = (intptr_t)f * rfs + (intptr_t)(by + uy) * rs + bx + ux;
    const pixel *const p0 = a0 + qo, *const p1 = a1 + qo, *const p2 = a2 + qo, *const p3 = a3 + qo;
    const pixel *const r0 = b0 + qo, *const r1 = b1 + qo, *const r2 = b2 + qo, *const r3 = b3 + qo;

    const int16_t *p = par + 12 * j;
    int bm0x = p[0], bm0y = p[1], bm1x = p[2], bm1y = p[3];
    const uint16_t *c0x = cost_mv - p[4], *c0y = cost_mv - p[5], *c1x = cost_mv - p[6], *c1y = cost_mv - p[7];
    const int minx = p[8], miny = p[9], maxx = p[10], maxy = p[11];
    const int w1 = weight[j], w2 = 64 - w1;
    int bcost = COST_MAX, ncalls = 0, npass = 0;
    bool act = !(bm0y < miny + 8 || bm1y < miny + 8 || bm0y > maxy - 8 || bm1y > maxy - 8 || bm0x < minx + 8 ||
                 bm1x < minx + 8 || bm0x > maxx - 8 || bm1x > maxx - 8);
    uint32_t *vis = s_vis[seg];
#pragma unroll
    for( int i = lane - sbase; i < 128; i += SL )
        vis[i] = 0;
    for( int pass = 0; pass < 8; pass++ )
    {
        if( !__any( act ) )
            break;
        int bestj = 0;
        if( act )
            npass++;
        const int j0 = pass ? 1 : 0;
        for( int r = 0; r < (pass ? 4 : 5); r++ )
        {
            const int jj = j0 + 8 * r + g;                // this group's pair
            const int jc = jj < 33 ? jj : 0;
            const int m0x = bm0x + dia4d( jc, 0 ), m0y = bm0y + dia4d( jc, 1 );
            const int m1x = bm1x + dia4d( jc, 2 ), m1y = bm1y + dia4d( jc, 3 );
            const int key = ((m0x & 7) << 9) | ((m0y & 7) << 6) | ((m1x & 7) << 3) | (m1y & 7);
            const bool ok = act && jj < 33 && !(pass && ((vis[key >> 5] >> (key & 31)) & 1));
            uint32_t v = 0;
            if( ok )
            {
                uint32_t t0[4][HDW], t1[4][HDW];
                ref_tile<BD>( p0, p1, p2, p3, rs, m0x, m0y, t0 );
                ref_tile<BD>( r0, r1, r2, r3, rs, m1x, m1y, t1 );
                if( w1 == 32 )
                {
#pragma unroll
                    for( int y = 0; y < 4; y++ )
#pragma unroll
                        for( int k = 0; k < HDW; k++ )
                            t0[y][k] = avg_round<BD>( t0[y][k], t1[y][k] );
                }
                else
                {
#pragma unroll
                    for( int y = 0; y < 4; y++ )
#pragma unroll
                        for( int k = 0; k < HDW; k++ )
                        {
                            uint32_t o = 0;
#pragma unroll
                            for( int e = 0; e < PPD; e++ )
                                o |= (uint32_t)clip_pix<BD>( (upix<BD>( t0[y][k], e ) * w1 + upix<BD>( t1[y][k], e ) * w2 +
                                                              32) >> 6 ) << ((32 / PPD) * e);
                            t0[y][k] = o;
                        }
                }
                if constexpr( SATD )
                {
                    uint32_t o[16];
                    had8x4_biased<BD>( t0, o );
#pragma unroll
                    for( int k = 0; k < 16; k++ )
                        v = __builtin_amdgcn_sad_u16( o[k], hr[k], v );
                    v >>= 1;
                }
                else
                {
#pragma unroll
                    for( int y = 0; y < 4; y++ )
#pragma unroll
                        for( int k = 0; k < HDW; k++ )
                            v = sadp<BD>( fa[y][k], t0[y][k], v );
                }
                if( u == 0 )
                {
                    v += (uint32_t)c0x[m0x] + (uint32_t)c0y[m0y] + (uint32_t)c1x[m1x] + (uint32_t)c1y[m1y];
                    atomicOr( &vis[key >> 5], 1u << (key & 31) );
                }
            }
            else if( u == 0 )
                v = NONE;
            v = group_sum<NT>( v );
            int c[8];
#pragma unroll
            for( int k = 0; k < 8; k++ )
                c[k] = (int)__shfl( (int)v, sbase + NT * k );
            if( act )
            {
#pragma unroll
                for( int k = 0; k < 8; k++ )
                    if( c[k] != NONE )
                    {
                        ncalls++;
                        if( c[k] < bcost )
                        {
                            bcost = c[k];
                            bestj = j0 + 8 * r + k;
                        }
                    }
            }
        }
        if( act )
        {
            if( !bestj )
                act = false;
            else
            {
                bm0x += dia4d( bestj, 0 );
                bm0y += dia4d( bestj, 1 );
                bm1x += dia4d( bestj, 2 );
                bm1y += dia4d( bestj, 3 );
            }
        }
    }
    if( live && lane == sbase )
    {
        *(int4 *)(out + 4 * j) = make_int4( bm0x, bm0y, bm1x, bm1y );
        if( cost )
            cost[j] = bcost;
        if( nevals )
            nevals[j] = ncalls | (npass << 16);
    }
}

template <int BD>
hipError_t launch_me_refine_bidir( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                                   const typename PT<BD>::pixel *const planes0[4],
                                   const typename PT<BD>::pixel *const planes1[4], intptr_t rs, intptr_t rfs,
                                   int i_pixel, int satd, const int32_t *pos, const int16_t *par, const int32_t *weight,
                                   const uint16_t *cost_mv, int n, int32_t *out, int32_t *cost, int32_t *nevals,
                                   hipStream_t stream )
{
    if( n <= 0 )
        return hipSuccess;
    if( i_pixel < 0 || i_pixel > 3 || ((uintptr_t)out & 15) )
        return hipErrorInvalidValue;
    // 8 * (the partition's 8x4 tiles) lanes per partition
    const int64_t lanes = (int64_t)n * 8 * (pix_w( i_pixel ) / 8) * (pix_h( i_pixel ) / 4);
    dim3 blk( 256 ), g( (unsigned)((lanes + 255) / 256) );
#define BI_GO( I, S )                                                                                             \
    hipLaunchKernelGGL( ( me_refine_bidir_kernel<BD, I, S> ), g, blk, 0, stream, fenc, fs, ffs, planes0[0],         \
                        planes0[1], planes0[2], planes0[3], planes1[0], planes1[1], planes1[2], planes1[3], rs, rfs, \
                        n, pos, par, weight, cost_mv, out, cost, nevals )
#define BI_CASE( I )                                                                                              \
    case I:                                                                                                       \
        if( satd ) { BI_GO( I, true ); } else { BI_GO( I, false ); }                                              \
        break;
    switch( i_pixel )
    {
        BI_CASE( 0 ) BI_CASE( 1 ) BI_CASE( 2 ) BI_CASE( 3 )
        default: return hipErrorInvalidValue;
    }
#undef BI_CASE
#undef BI_GO
    return hipGetLastError();
}
template hipError_t launch_me_refine_bidir<8>( const uint8_t *, intptr_t, intptr_t, const uint8_t *const[4],
                                               const uint8_t *const[4], intptr_t, intptr_t, int, int, const int32_t *,
                                               const int16_t *, const int32_t *, const uint16_t *, int, int32_t *,
                                               int32_t *, int32_t *, hipStream_t );
template hipError_t launch_me_refine_bidir<10>( const uint16_t *, intptr_t, intptr_t, const uint16_t *const[4],
                                                const uint16_t *const[4], intptr_t, intptr_t, int, int, const int32_t *,
                                                const int16_t *, const int32_t *, const uint16_t *, int, int32_t *,
                                                int32_t *, int32_t *, hipStream_t );

template hipError_t launch_me_search_ref<8>( const uint8_t *, intptr_t, intptr_t, const uint8_t *, const uint8_t *const[4],
                                             intptr_t, intptr_t, int, int, int, int, const int32_t *, const int16_t *,
                                             const int16_t *, const uint16_t *, int, int32_t *, int32_t *, int32_t *,
                                             const int32_t *, const x264hip_refine_ext_t *, hipStream_t );
template hipError_t launch_me_search_ref<10>( const uint16_t *, intptr_t, intptr_t, const uint16_t *,
                                              const uint16_t *const[4], intptr_t, intptr_t, int, int, int, int,
                                              const int32_t *, const int16_t *, const int16_t *, const uint16_t *, int,
                                              int32_t *, int32_t *, int32_t *, const int32_t *, const x264hip_refine_ext_t *,
                                              hipStream_t );

template hipError_t launch_me_refine_subpel<8>( const uint8_t *, intptr_t, intptr_t, const uint8_t *const[4],
                                                intptr_t, intptr_t, int, int, int, int, const int32_t *,
                                                const int16_t *, const int32_t *, const uint16_t *, int, int32_t *,
                                                int32_t *, int32_t *, const int32_t *, const x264hip_refine_ext_t *,
                                                hipStream_t );
template hipError_t launch_me_refine_subpel<10>( const uint16_t *, intptr_t, intptr_t, const uint16_t *const[4],
                                                 intptr_t, intptr_t, int, int, int, int, const int32_t *,
                                                 const int16_t *, const int32_t *, const uint16_t *, int, int32_t *,
                                                 int32_t *, int32_t *, const int32_t *, const x264hip_refine_ext_t *,
                                                 hipStream_t );

// ---------------------------------------------------------------------------
// x264's P16x16 reference-0 analysis over whole frames with the encoder's own predictors
// (x264hip_*_me_analyse_p16x16).  For every MB in raster order analyse.c's
// x264_mb_analyse_inter_p16x16 takes mvp = x264_mb_predict_mv_16x16 (common/mvpred.c:129-157:
// the median of the left, top and top-right -- or top-left -- neighbours' mvs, or the only one
// with the reference) and mvc = x264_mb_predict_mv_ref16x16 (mvpred.c:519-600: the lookahead's
// lowres mv doubled, the left / top / top-left / top-right MBs' 16x16 mvs -- mv 0 off the frame,
// mvr[-1] -- and the reference's colocated / right / below mvs scaled by the POC distance), the
// mv limits of analyse.c:330-349, then x264_me_search_ref.  The raster order's dependency (a MB
// reads its left, top-left, top and top-right neighbours) is run as a wavefront: anti-diagonal d
// = x + 2y only reads diagonals d-1 .. d-3, so each diagonal of every frame is one predictor
// launch and one me_search_ref launch.  Every MB is taken as P_L0 16x16 with its searched mv (the
// neighbours' cache mvs = their mvr), i.e. the analysis of a frame none of whose MBs ends as
// intra, skip or a smaller partition.
// Entries of diagonal d: frame-major, then y from ylo(d); global entry off(d) + f L(d) + y - ylo(d).
__host__ __device__ inline int p16_ylo( int d, int mbw ) { return d - mbw + 1 > 0 ? (d - mbw + 2) / 2 : 0; }
__host__ __device__ inline int p16_len( int d, int mbw, int mbh )
{
    const int hi = min( mbh - 1, d / 2 ), lo = p16_ylo( d, mbw );
    return hi >= lo ? hi - lo + 1 : 0;
}
// MBs (of one frame) on diagonals below d
__device__ inline int p16_before( int d, int mbw, int mbh )
{
    int n = 0;
    for( int y = 0; y < mbh; y++ )
        n += min( max( d - 2 * y, 0 ), mbw );
    return n;
}
__device__ inline int p16_index( int f, int x, int y, int nf, int mbw, int mbh )
{
    const int d = x + 2 * y;
    return nf * p16_before( d, mbw, mbh ) + f * p16_len( d, mbw, mbh ) + y - p16_ylo( d, mbw );
}
__device__ inline int p16_median( int a, int b, int c )
{
    return max( min( a, b ), min( max( a, b ), c ) );
}

__global__ __launch_bounds__( 256 ) void me_p16_predict_kernel( int d, int nf, int mbw, int mbh, int fmv,
                                                                const int16_t *__restrict__ lowres,
                                                                const int16_t *__restrict__ tmv, int tscale,
                                                                const int32_t *__restrict__ outd,
                                                                int32_t *__restrict__ pos, int16_t *__restrict__ par,
                                                                int16_t *__restrict__ mvc )
{
    const int L = p16_len( d, mbw, mbh );
    const int e = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if( e >= nf * L )
        return;
    const int f = e / L, y = p16_ylo( d, mbw ) + e % L, x = d - 2 * y;
    const int nmb = mbw * mbh, mb = y * mbw + x;
    const int g = nf * p16_before( d, mbw, mbh ) + e;
    // a neighbour's 16x16 mv (the search result on an earlier diagonal), 0 off the frame
    auto nb = [&]( int nx, int ny, int &mx, int &my ) -> bool {
        if( nx < 0 || ny < 0 || nx >= mbw )
        {
            mx = my = 0;
            return false;
        }
        const int i = p16_index( f, nx, ny, nf, mbw, mbh );
        mx = outd[4 * i + 1];
        my = outd[4 * i + 2];
        return true;
    };
    int ax, ay, bx, by, cx, cy, dx, dy;
    const bool va = nb( x - 1, y, ax, ay ), vb = nb( x, y - 1, bx, by );
    const bool vd = nb( x - 1, y - 1, dx, dy );
    bool vc = x + 1 < mbw && nb( x + 1, y - 1, cx, cy );
    if( !vc )                               // mvpred.c:136-140: C unavailable -> D
    {
        cx = dx;
        cy = dy;
        vc = vd;
    }
    // x264_mb_predict_mv_16x16 with every available neighbour on reference 0 (mvpred.c:142-157)
    int px, py;
    const int cnt = va + vb + vc;
    if( cnt == 1 )
    {
        px = va ? ax : vb ? bx : cx;
        py = va ? ay : vb ? by : cy;
    }
    else if( cnt == 0 && !vb && !vc && va )
    {
        px = ax;
        py = ay;
    }
    else
    {
        px = p16_median( ax, bx, cx );
        py = p16_median( ay, by, cy );
    }
    // x264_mb_predict_mv_ref16x16 (mvpred.c:519-600), P slice, reference 0, no MBAFF
    int16_t *m = mvc + 28 * (int64_t)g;
    int i = 0;
    auto put = [&]( int vx, int vy ) {
        m[2 * i] = (int16_t)vx;
        m[2 * i + 1] = (int16_t)vy;
        i++;
    };
    if( lowres && lowres[2 * (int64_t)f * nmb] != 0x7fff )
    {
        // M32( lowres_mv ) * 2 & 0xfffeffff: each half doubled, wrapping in 16 bits
        const uint32_t w = (uint32_t)(uint16_t)lowres[2 * ((int64_t)f * nmb + mb)] |
                           ((uint32_t)(uint16_t)lowres[2 * ((int64_t)f * nmb + mb) + 1] << 16);
        const uint32_t w2 = (w * 2u) & 0xfffeffffu;
        put( (int16_t)(w2 & 0xffff), (int16_t)(w2 >> 16) );
    }
    int sx, sy;
    nb( x - 1, y, sx, sy ), put( sx, sy );
    nb( x, y - 1, sx, sy ), put( sx, sy );
    nb( x - 1, y - 1, sx, sy ), put( sx, sy );
    if( x + 1 < mbw )
        nb( x + 1, y - 1, sx, sy );
    else
        sx = sy = 0;
    put( sx, sy );
    if( tmv )
    {
        auto tput = [&]( int k ) {
            const int64_t t = (int64_t)f * nmb + k;
            put( min( max( (tmv[2 * t] * tscale + 128) >> 8, -32768 ), 32767 ),
                 min( max( (tmv[2 * t + 1] * tscale + 128) >> 8, -32768 ), 32767 ) );
        };
        tput( mb );
        if( x < mbw - 1 )
            tput( mb + 1 );
        if( y < mbh - 1 )
            tput( mb + mbw );
    }
    // the MB's limits (analyse.c:330-349)
    const int min0 = 4 * (-16 * x - 24), max0 = 4 * (16 * (mbw - x - 1) + 24);
    const int min1 = 4 * (-16 * y - 24), max1 = 4 * (16 * (mbh - y - 1) + 24);
    const int smin0 = max( min0, -fmv ), smax0 = min( max0, fmv - 1 );
    const int smin1 = max( min1, -fmv ), smax1 = min( max1, fmv - 1 );
    int16_t *q = par + 12 * (int64_t)g;
    q[0] = (int16_t)px;
    q[1] = (int16_t)py;
    q[2] = (int16_t)((smin0 >> 2) + 6);
    q[3] = (int16_t)((smin1 >> 2) + 6);
    q[4] = (int16_t)((smax0 >> 2) - 6);
    q[5] = (int16_t)((smax1 >> 2) - 6);
    q[6] = (int16_t)smin0;
    q[7] = (int16_t)smin1;
    q[8] = (int16_t)smax0;
    q[9] = (int16_t)smax1;
    q[10] = (int16_t)i;
    q[11] = 0;
    pos[3 * (int64_t)g] = f;
    pos[3 * (int64_t)g + 1] = 16 * x;
    pos[3 * (int64_t)g + 2] = 16 * y;
}

// diagonal-major results back to frame-major raster order
__global__ __launch_bounds__( 256 ) void me_p16_unscramble_kernel( int nf, int mbw, int mbh,
                                                                   const int32_t *__restrict__ outd,
                                                                   const int32_t *__restrict__ nevd,
                                                                   int32_t *__restrict__ out,
                                                                   int32_t *__restrict__ nevals )
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int nmb = mbw * mbh;
    if( t >= (int64_t)nf * nmb )
        return;
    const int f = (int)(t / nmb), mb = (int)(t - (int64_t)f * nmb), y = mb / mbw, x = mb - y * mbw;
    const int i = p16_index( f, x, y, nf, mbw, mbh );
#pragma unroll
    for( int k = 0; k < 4; k++ )
        out[4 * t + k] = outd[4 * (int64_t)i + k];
    if( nevals )
    {
        nevals[2 * t] = nevd[2 * (int64_t)i];
        nevals[2 * t + 1] = nevd[2 * (int64_t)i + 1];
    }
}

template <int BD>
hipError_t launch_me_analyse_p16x16( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                                     const typename PT<BD>::pixel *fw, const typename PT<BD>::pixel *const planes[4],
                                     intptr_t rs, intptr_t rfs, int mbw, int mbh, int nframes, int me_method,
                                     int subme, int me_range, int mv_range, const int16_t *lowres, const int16_t *tmv,
                                     int tscale, const uint16_t *cost_mv, int32_t *out, int32_t *nevals,
                                     const x264hip_refine_ext_t *ext, hipStream_t stream )
{
    const int64_t n = (int64_t)nframes * mbw * mbh;
    if( n <= 0 )
        return hipSuccess;
    if( n > (1 << 26) || mv_range < 1 || mv_range > 8192 )
        return hipErrorInvalidValue;
    // diagonal-major scratch: results, positions, call counts, par, mvc (each 256-byte aligned)
    auto al = []( size_t v ) { return (v + 255) & ~(size_t)255; };
    const size_t b_out = al( (size_t)n * 16 ), b_pos = al( (size_t)n * 12 ), b_nev = nevals ? al( (size_t)n * 8 ) : 0;
    const size_t b_par = al( (size_t)n * 24 ), b_mvc = al( (size_t)n * 56 );
    void *buf = nullptr;
    hipError_t e = scratch_alloc( &buf, b_out + b_pos + b_nev + b_par + b_mvc, stream );
    if( e != hipSuccess )
        return e;
    uint8_t *b = (uint8_t *)buf;
    int32_t *outd = (int32_t *)b, *pos = (int32_t *)(b + b_out);
    int32_t *nevd = nevals ? (int32_t *)(b + b_out + b_pos) : nullptr;
    int16_t *par = (int16_t *)(b + b_out + b_pos + b_nev), *mvc = (int16_t *)(b + b_out + b_pos + b_nev + b_par);
    const int nd = mbw + 2 * (mbh - 1);
    int64_t off = 0;
    for( int d = 0; d < nd && e == hipSuccess; d++ )
    {
        const int64_t nn = (int64_t)nframes * p16_len( d, mbw, mbh );
        if( !nn )
            continue;
        hipLaunchKernelGGL( me_p16_predict_kernel, dim3( (unsigned)((nn + 255) / 256) ), dim3( 256 ), 0, stream, d,
                            nframes, mbw, mbh, 4 * mv_range, lowres, tmv, tscale, outd, pos, par, mvc );
        if( (e = hipGetLastError()) != hipSuccess )
            break;
        e = launch_me_search_ref<BD>( fenc, fs, ffs, fw, planes, rs, rfs, 0, me_method, subme, me_range, pos + 3 * off,
                                      par + 12 * off, mvc + 28 * off, cost_mv, (int)nn, outd + 4 * off,
                                      nevd ? nevd + 2 * off : nullptr, nullptr, nullptr, ext, stream );
        off += nn;
    }
    if( e == hipSuccess )
    {
        hipLaunchKernelGGL( me_p16_unscramble_kernel, dim3( (unsigned)((n + 255) / 256) ), dim3( 256 ), 0, stream,
                            nframes, mbw, mbh, outd, nevd, out, nevals );
        e = hipGetLastError();
    }
    const hipError_t fr = hipFreeAsync( buf, stream );
    return e != hipSuccess ? e : fr;
}
template hipError_t launch_me_analyse_p16x16<8>( const uint8_t *, intptr_t, intptr_t, const uint8_t *,
                                                 const uint8_t *const[4], intptr_t, intptr_t, int, int, int, int, int,
                                                 int, int, const int16_t *, const int16_t *, int, const uint16_t *,
                                                 int32_t *, int32_t *, const x264hip_refine_ext_t *, hipStream_t );
template hipError_t launch_me_analyse_p16x16<10>( const uint16_t *, intptr_t, intptr_t, const uint16_t *,
                                                  const uint16_t *const[4], intptr_t, intptr_t, int, int, int, int,
                                                  int, int, int, const int16_t *, const int16_t *, int,
                                                  const uint16_t *, int32_t *, int32_t *, const x264hip_refine_ext_t *,
                                                  hipStream_t );

} // namespace x264hip
