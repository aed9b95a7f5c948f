// The lookahead's lowres motion search on gfx950: slicetype_mb_cost's inter leg
// for P frames (reference encoder/slicetype.c:514-713, 758-791 with b == p1, one
// list, no weights, a fresh search) and for B frames (both lists, searched or
// cached, and the TRY_BIDIR weighted averages), with the x264_me_search_ref /
// refine_subpel paths the lookahead runs (encoder/me.c:182-420, 774-790,
// 865-992: me = DIA or HEX, lookahead subme 2 or 4, no chroma ME).
//
// Dependencies: every block takes its MV predictors from blocks the reverse
// raster scan of slicetype_slice_cost (slicetype.c:818-833) has already
// searched -- right (x+1, y) and the row below (x-1..x+1, y+1) -- so the
// bit-exact schedule is a wavefront: block (x, y) runs at step
// t = (W-1-x) + 2(H-1-y), after all four of its predictors.  One workgroup
// walks one frame pair's W + 2H - 2 steps with a barrier between steps, one
// lane quad per block row (each lane two of the block's eight pixel rows, the
// metrics finished by DPP quad reductions); the four most recent MVs of every
// row sit in an LDS ring (the predictors of a step are at most three steps
// old).  Each quad runs the block's whole search (HEX / DIA, the hpel and qpel
// refinement) with fenc rows held in registers, integer patterns scored from a
// register window of the F plane and get_ref rebuilt from the four lowres
// planes; the frame pairs of a batch run in parallel.
#include "hipcommon.h"

namespace x264hip {

// The reference's small tables (tables.c hpel_ref0/1, me.c mod6m1/hex2/square1; pinned to the
// reference text by tests/test_ref_tables.py).  The searches index them with per-lane values
// on their serial chain, so the kernels read them as bit fields of compile-time words
// (an immediate shift and mask) rather than as memory: a table load was one more dependent
// memory round per hexagon step and per get_ref.
constexpr uint8_t c_lr_ref0[16] = { 0, 1, 1, 1, 0, 1, 1, 1, 2, 3, 3, 3, 0, 1, 1, 1 };   // x264_hpel_ref0
constexpr uint8_t c_lr_ref1[16] = { 0, 0, 1, 0, 2, 2, 3, 2, 2, 2, 3, 2, 2, 2, 3, 2 };   // x264_hpel_ref1
constexpr int8_t c_hex2[8][2] = { { -1, -2 }, { -2, 0 }, { -1, 2 }, { 1, 2 }, { 2, 0 }, { 1, -2 }, { -1, -2 }, { -2, 0 } };
constexpr uint8_t c_mod6m1[8] = { 5, 0, 1, 2, 3, 4, 5, 0 };
constexpr int8_t c_square1[9][2] = { { 0, 0 }, { 0, -1 }, { 0, 1 }, { -1, 0 }, { 1, 0 },
                                     { -1, -1 }, { -1, 1 }, { 1, -1 }, { 1, 1 } };
// signed entries biased by `bias`, as bit fields (pack_fields)
template <int N> constexpr uint32_t lr_pack_s( const int8_t ( &a )[N][2], int c, int b, int bias )
{
    uint32_t r = 0;
    for( int i = 0; i < N; i++ )
        r |= (uint32_t)(a[i][c] + bias) << (b * i);
    return r;
}
constexpr uint32_t k_lr_ref0 = pack_fields( c_lr_ref0, 2 ), k_lr_ref1 = pack_fields( c_lr_ref1, 2 );
constexpr uint32_t k_hex2_x = lr_pack_s( c_hex2, 0, 3, 2 ), k_hex2_y = lr_pack_s( c_hex2, 1, 3, 2 );
constexpr uint32_t k_mod6m1 = pack_fields( c_mod6m1, 3 );
constexpr uint32_t k_square1_x = lr_pack_s( c_square1, 0, 2, 1 ), k_square1_y = lr_pack_s( c_square1, 1, 2, 1 );
__device__ __forceinline__ int lr_hex2_x( int j ) { return (int)((k_hex2_x >> (3 * j)) & 7) - 2; }
__device__ __forceinline__ int lr_hex2_y( int j ) { return (int)((k_hex2_y >> (3 * j)) & 7) - 2; }
__device__ __forceinline__ int lr_mod6m1( int j ) { return (int)((k_mod6m1 >> (3 * j)) & 7); }
__device__ __forceinline__ int lr_square1_x( int k ) { return (int)((k_square1_x >> (2 * k)) & 3) - 1; }
__device__ __forceinline__ int lr_square1_y( int k ) { return (int)((k_square1_y >> (2 * k)) & 3) - 1; }

constexpr int LR_COST_MAX = 1 << 28;

__device__ __forceinline__ uint32_t lr_pack( int a, int b ) { return (uint32_t)(uint16_t)a | ((uint32_t)(uint16_t)b << 16); }
__device__ __forceinline__ int lr_clip3( int v, int lo, int hi ) { return v < lo ? lo : v > hi ? hi : v; }
__device__ __forceinline__ int lr_median( int a, int b, int c )
{
    const int mn = min( a, b ), mx = max( a, b );
    return c < mn ? mn : c > mx ? mx : c;
}

// Lanes 4y .. 4y+3 of a workgroup share block row y: lane q = lane & 3 holds rows
// 2q and 2q+1 of the 8x8 block, so every metric costs a quarter of its pixel work
// per lane and is finished by a reduction over the quad (all four lanes end with
// the same value and run the same search path).
constexpr int LR_NR = 2;

__device__ __forceinline__ uint32_t lr_swap1( uint32_t v )      // lane q ^ 1
{
    return (uint32_t)__builtin_amdgcn_mov_dpp( (int)v, 0xB1, 0xF, 0xF, true );   // quad_perm [1,0,3,2]
}
__device__ __forceinline__ uint32_t lr_quad_sum( uint32_t v )
{
    v += lr_swap1( v );
    v += (uint32_t)__builtin_amdgcn_mov_dpp( (int)v, 0x4E, 0xF, 0xF, true );      // quad_perm [2,3,0,1]
    return v;
}

// 8x8 SAD or packed SATD of fenc rows against predicted rows (this lane's two rows).
// SATD: lanes 2b and 2b+1 hold rows 0-1 and 2-3 of band b; each takes the horizontal
// Hadamard of its rows and the first vertical stage, the partner's half arrives by
// DPP and the even lane forms t0+t2 / t1+t3, the odd lane t2-t0 / t3-t1 (the
// negated t0-t2 / t1-t3: same magnitude, and the 0x8000 bias on element (0,0),
// applied by the even lane, stays 0x8000 mod 2^16 under negation).
template <int BD>
__device__ __forceinline__ int lr_cmp_rows( const uint32_t (&fe)[LR_NR][8 / PT<BD>::PPD],
                                            const uint32_t (&r)[LR_NR][8 / PT<BD>::PPD], bool use_satd, int q )
{
    constexpr int NDW = 8 / PT<BD>::PPD;
    uint32_t acc = 0;
    if( use_satd )
    {
        const bool odd = q & 1;
        x264hip_short2 d[LR_NR][4];
#pragma unroll
        for( int j = 0; j < LR_NR; j++ )
        {
            x264hip_short2 p[4];
#pragma unroll
            for( int x = 0; x < 4; x++ )
                p[x] = pair_px<BD>( fe[j], x ) - pair_px<BD>( r[j], x );
            if( j == 0 )
                p[0] = odd ? p[0] : sat_bias( p[0] );
            const x264hip_short2 t0 = p[0] + p[1], t1 = p[0] - p[1], t2 = p[2] + p[3], t3 = p[2] - p[3];
            d[j][0] = t0 + t2; d[j][2] = t0 - t2; d[j][1] = t1 + t3; d[j][3] = t1 - t3;
        }
#pragma unroll
        for( int x = 0; x < 4; x++ )
        {
            const x264hip_short2 ta = d[0][x] + d[1][x], tb = d[0][x] - d[1][x];
            const x264hip_short2 pa = __builtin_bit_cast( x264hip_short2, lr_swap1( __builtin_bit_cast( uint32_t, ta ) ) );
            const x264hip_short2 pb = __builtin_bit_cast( x264hip_short2, lr_swap1( __builtin_bit_cast( uint32_t, tb ) ) );
            const x264hip_short2 ca = odd ? ta - pa : ta + pa, cb = odd ? tb - pb : tb + pb;
            acc = __builtin_amdgcn_sad_u16( __builtin_bit_cast( uint32_t, ca ), 0x80008000u, acc );
            acc = __builtin_amdgcn_sad_u16( __builtin_bit_cast( uint32_t, cb ), 0x80008000u, acc );
        }
        return (int)(lr_quad_sum( acc ) >> 1);
    }
#pragma unroll
    for( int y = 0; y < LR_NR; y++ )
#pragma unroll
        for( int k = 0; k < NDW; k++ )
            acc = sadp<BD>( fe[y][k], r[y][k], acc );
    return (int)lr_quad_sum( acc );
}

// mc_weight (mc.c:117-137) of one dword of packed pixels: clip( ((p*scale + rnd) >> sh) + off ),
// rnd = 1 << (denom-1) and sh = denom when denom >= 1, else 0 and 0; off already scaled by
// 1 << (BD-8).  8 bit in int16 pairs: |p*scale| <= 255*128 and the sum stays inside int16.
template <int BD> __device__ __forceinline__ uint32_t lr_weight_px( uint32_t v, int sc, int rnd, int sh, int off )
{
    if constexpr( BD == 8 )
    {
        typedef short ss2 __attribute__( ( ext_vector_type( 2 ) ) );
        const ss2 scv = (ss2)(short)sc, rv = (ss2)(short)rnd, shv = (ss2)(short)sh, ov = (ss2)(short)off;
        auto f = [&]( uint32_t x ) {
            ss2 r = ((__builtin_bit_cast( ss2, x ) * scv + rv) >> shv) + ov;
            r = __builtin_elementwise_min( __builtin_elementwise_max( r, (ss2)(short)0 ), (ss2)(short)255 );
            return __builtin_bit_cast( uint32_t, r );
        };
        const uint32_t lo = f( __builtin_amdgcn_perm( 0u, v, 0x0c020c00u ) );
        const uint32_t hi = f( __builtin_amdgcn_perm( 0u, v, 0x0c030c01u ) );
        return __builtin_amdgcn_perm( hi, lo, 0x06020400u );
    }
    else
    {
        auto f = [&]( int p ) { return (uint32_t)min( max( ((p * sc + rnd) >> sh) + off, 0 ), 1023 ); };
        return f( (int)(v & 0xffff) ) | (f( (int)(v >> 16) ) << 16);
    }
}

template <int BD> struct LrCtx
{
    using pixel = typename PT<BD>::pixel;
    static constexpr int NDW = 8 / PT<BD>::PPD;
    const uint32_t (&fe)[LR_NR][NDW];       // this lane's fenc rows (packed pixels), shared by the lists
    const pixel *p0;                        // reference F at the block, row 2q (H, V, C follow at pd)
    const pixel *pw;                        // p_fref_w: the weighted F plane (p0 when unweighted)
    intptr_t pd;                            // the planes' spacing (x264's buffer_lowres, frame.c;
                                            // the launchers stage unequal planes)
    int wsc, wrnd, wsh, woff;               // m->weight (mc_weight terms)
    bool wgt;
    intptr_t stride;
    const uint16_t *cmx, *cmy;              // p_cost_mvx / p_cost_mvy (cost_mv - mvp)
    int satd, q;
    int smin0, smax0, smin1, smax1;         // h->mb.mv_min_spel / mv_max_spel
    int fmin0, fmax0, fmin1, fmax1;         // mv_limit_fpel

    __device__ __forceinline__ LrCtx( const uint32_t (&f)[LR_NR][NDW] ) : fe( f ) {}

    // per-block setup of slicetype_mb_cost (slicetype.c:539-557): the lowres mv limits
    // (the vertical ones, set at the first block of each row of the scan, depend on
    // the row only) and the reference planes at the lane's first block row
    __device__ __forceinline__ void setup( const pixel *r0, intptr_t rpd,
                                           intptr_t off, intptr_t s, int x, int y, int mbw, int mbh, int mvr,
                                           int use_satd, int lane_q )
    {
        q = lane_q;
        off += (intptr_t)(LR_NR * q) * s;
        p0 = r0 + off;
        pd = rpd;
        pw = p0;
        wgt = false;
        wsc = wrnd = wsh = woff = 0;
        stride = s;
        satd = use_satd;
        smin0 = max( 4 * (-8 * x - 12), -mvr );
        smax0 = min( 4 * (8 * (mbw - x - 1) + 12), mvr - 1 );
        smin1 = max( 4 * (-8 * y - 12), -mvr );
        smax1 = min( 4 * (8 * (mbh - y - 1) + 12), mvr - 1 );
        fmin0 = smin0 >> 2;
        fmax0 = smax0 >> 2;
        fmin1 = smin1 >> 2;
        fmax1 = smax1 >> 2;
    }

    // the weighted-reference form (slicetype.c:609-614): the integer stage on the weighted
    // F plane rw, the subpel get_refs weighted by (scale, denom, offset)
    __device__ __forceinline__ void set_weight( const pixel *rw, intptr_t off, int scale, int denom, int offset )
    {
        pw = rw + off + (intptr_t)(LR_NR * q) * stride;
        wgt = true;
        wsc = scale;
        wrnd = denom >= 1 ? 1 << (denom - 1) : 0;
        wsh = denom >= 1 ? denom : 0;
        woff = offset * (1 << (BD - 8));
    }

    // fpelcmp (SAD) at a full-pel offset of p_fref_w (me.c:63-70)
    __device__ __forceinline__ int fpel( int mx, int my ) const
    {
        const pixel *r = pw + (intptr_t)my * stride + mx;
        uint32_t acc = 0;
#pragma unroll
        for( int y = 0; y < LR_NR; y++ )
        {
            uint32_t w[NDW];
            load_al_pad<NDW>( r + (intptr_t)y * stride, w );
#pragma unroll
            for( int k = 0; k < NDW; k++ )
                acc = sadp<BD>( fe[y][k], w[k], acc );
        }
        return (int)lr_quad_sum( acc );
    }

    // The F plane's window around a full-pel centre (columns cx-2 .. cx+9; this lane's
    // rows 2q-2 .. 2q+3 of the block, i.e. the rows its two block rows meet for any
    // vertical offset in [-2, 2]): one dword-aligned load per row, realigned once by
    // the byte offset all rows share (stride * sizeof(pixel) is a multiple of 4), so
    // every integer candidate within +-2 of the centre -- a diamond, a hexagon, the
    // square refine -- is scored from registers.
    static constexpr int WR = LR_NR + 4, WD = 12 / PT<BD>::PPD;
    __device__ __forceinline__ void win( int cx, int cy, uint32_t (&w)[WR][WD] ) const
    {
        // (the aligned base by pointer arithmetic, not through an integer: the loads stay
        // global_load, where an integer round trip made them flat loads, which also count
        // against the LDS wait counter)
        const pixel *p = pw + (intptr_t)(cy - 2) * stride + (cx - 2);
        const uint32_t sh = (uint32_t)((uintptr_t)p & 3);
        const uint8_t *b = (const uint8_t *)p - sh;
        const intptr_t sb = stride * (intptr_t)sizeof( pixel );
#pragma unroll
        for( int r = 0; r < WR; r++ )
        {
            const uint32_t *row = (const uint32_t *)(b + r * sb);
            uint32_t v[WD + 1];
#pragma unroll
            for( int k = 0; k <= WD; k++ )
                v[k] = row[k];
#pragma unroll
            for( int k = 0; k < WD; k++ )
                w[r][k] = __builtin_amdgcn_alignbyte( v[k + 1], v[k], sh );
        }
    }

    // fpel( cx + DX, cy + DY ) from the window of (cx, cy), |DX|, |DY| <= 2
    template <int DX, int DY> __device__ __forceinline__ int wsad( const uint32_t (&w)[WR][WD] ) const
    {
        constexpr int B = (DX + 2) * (int)sizeof( pixel ), D = B >> 2, S = B & 3;
        uint32_t acc = 0;
#pragma unroll
        for( int y = 0; y < LR_NR; y++ )
#pragma unroll
            for( int k = 0; k < NDW; k++ )
            {
                uint32_t v;
                if constexpr( S != 0 )
                    v = __builtin_amdgcn_alignbyte( w[DY + 2 + y][D + k + 1], w[DY + 2 + y][D + k], S );
                else
                    v = w[DY + 2 + y][D + k];
                acc = sadp<BD>( fe[y][k], v, acc );
            }
        return (int)lr_quad_sum( acc );
    }

    // get_ref (mc.c:221-249) rows at N quarter-pel mvs, weighted by m->weight when W and set.
    // Branch-free: a one-plane position reads its plane twice (the rounding average of equal
    // pixels is the pixel), so every candidate's loads are issued before any is waited on --
    // N candidates cost one memory round
    template <bool W = true, int N>
    __device__ __forceinline__ void ref_rows_n( const int (&mx)[N], const int (&my)[N],
                                                uint32_t (&r)[N][LR_NR][NDW] ) const
    {
        uint32_t b[N][LR_NR][NDW];
#pragma unroll
        for( int n = 0; n < N; n++ )
        {
            const int idx = ((my[n] & 3) << 2) + (mx[n] & 3);
            const intptr_t off = (intptr_t)(my[n] >> 2) * stride + (mx[n] >> 2);
            const int i0 = (int)((k_lr_ref0 >> (2 * idx)) & 3), i1 = (int)((k_lr_ref1 >> (2 * idx)) & 3);
            // (the plane by one multiply-add: the four planes equally spaced)
            const pixel *s1 = p0 + i0 * pd + off + ((my[n] & 3) == 3) * stride;
            const pixel *s2 = (idx & 5) ? p0 + i1 * pd + off + ((mx[n] & 3) == 3) : s1;
#pragma unroll
            for( int y = 0; y < LR_NR; y++ )
            {
                load_al_pad<NDW>( s1 + (intptr_t)y * stride, r[n][y] );
                load_al_pad<NDW>( s2 + (intptr_t)y * stride, b[n][y] );
            }
        }
#pragma unroll
        for( int n = 0; n < N; n++ )
#pragma unroll
            for( int y = 0; y < LR_NR; y++ )
#pragma unroll
                for( int k = 0; k < NDW; k++ )
                {
                    r[n][y][k] = avg_round<BD>( r[n][y][k], b[n][y][k] );
                    if( W && wgt )
                        r[n][y][k] = lr_weight_px<BD>( r[n][y][k], wsc, wrnd, wsh, woff );
                }
    }
    template <bool W = true>
    __device__ __forceinline__ void ref_rows( int mx, int my, uint32_t (&r)[LR_NR][NDW] ) const
    {
        const int ax[1] = { mx }, ay[1] = { my };
        ref_rows_n<W, 1>( ax, ay, *reinterpret_cast<uint32_t( * )[1][LR_NR][NDW]>( &r ) );
    }

    // hpel plane rows addressed directly (TRY_BIDIR for subme <= 1, slicetype.c:594-600)
    __device__ __forceinline__ void hpel_rows( int mx, int my, uint32_t (&r)[LR_NR][NDW] ) const
    {
        const int i = ((mx & 2) >> 1) + (my & 2);
        const pixel *s = p0 + i * pd + (mx >> 2) + (intptr_t)(my >> 2) * stride;
#pragma unroll
        for( int y = 0; y < LR_NR; y++ )
            load_al_pad<NDW>( s + (intptr_t)y * stride, r[y] );
    }

    // get_ref at a quarter-pel mv, then SAD or SATD 8x8 (W = false: the unweighted planes)
    template <bool W = true>
    __device__ __forceinline__ int qpel( int mx, int my, bool use_satd ) const
    {
        uint32_t r[LR_NR][NDW];
        ref_rows<W>( mx, my, r );
        return lr_cmp_rows<BD>( fe, r, use_satd, q );
    }
    // two / three positions in one memory round: their SAD or SATD each (sat[n])
    template <bool W = true, int N>
    __device__ __forceinline__ void qpel_n( const int (&mx)[N], const int (&my)[N], const bool (&sat)[N],
                                            int (&c)[N] ) const
    {
        uint32_t r[N][LR_NR][NDW];
        ref_rows_n<W, N>( mx, my, r );
#pragma unroll
        for( int n = 0; n < N; n++ )
            c[n] = lr_cmp_rows<BD>( fe, r[n], sat[n], q ) + cmx[mx[n]] + cmy[my[n]];
    }

    __device__ __forceinline__ int bits_mvd( int mx, int my ) const { return cmx[mx * 4] + cmy[my * 4]; }
    __device__ __forceinline__ bool in_range( int mx, int my ) const
    {
        return mx >= fmin0 && mx <= fmax0 && my >= fmin1 && my <= fmax1;
    }
};

// x264_me_search_ref (me.c:182-420, 774-790) then refine_subpel (me.c:912-992)
// role >= 0: NG groups of the wave (lanes 64/NG apart) run this same search on the same block
// in lockstep and split each batch of (up to four) independent candidates -- the predictors,
// the hpel and qpel diamonds: with NG = 4 group r scores candidate r, with NG = 2 candidates r
// and r + 2 -- the costs are gathered from the groups and every group makes the same
// decisions.  role < 0: one group scores them in turn.
template <int NG> __device__ __forceinline__ int lr_gather( int v, int r )
{
    constexpr int S = 64 / NG;
    return __shfl( v, (int)(threadIdx.x & (S - 1)) + S * r );
}
// a batch of four candidates split over the NG groups: cand( k ) scores candidate k
template <int NG, typename F> __device__ __forceinline__ void lr_batch4( int role, F cand, int (&out)[4] )
{
    if constexpr( NG == 4 )
    {
        const int c = cand( role );
#pragma unroll
        for( int r = 0; r < 4; r++ )
            out[r] = lr_gather<4>( c, r );
    }
    else
    {
        const int c0 = cand( role ), c1 = cand( role + 2 );
        out[0] = lr_gather<2>( c0, 0 );
        out[1] = lr_gather<2>( c0, 1 );
        out[2] = lr_gather<2>( c1, 0 );
        out[3] = lr_gather<2>( c1, 1 );
    }
}

template <int BD, int NG = 4>
__device__ void lr_me_search( const LrCtx<BD> &m, int mvpx, int mvpy, const int (&mvc)[4][2], int i_mvc,
                              int me_method, int subme, int me_range, int role, int &omvx, int &omvy, int &ocost )
{
    int bmx, bmy, bcost = LR_COST_MAX, bpred_cost = LR_COST_MAX;
    uint32_t pmv, bpred_mv = 0;
    int tmp[6][2];
    // the integer search's window and its centre ((wx, wy) = the centre it was loaded at; a
    // search step whose centre is unchanged scores from it instead of loading it again)
    uint32_t w[LrCtx<BD>::WR][LrCtx<BD>::WD];
    int wx = 0x7fff, wy = 0x7fff;
    auto window = [&]() __attribute__( ( always_inline ) ) {
        if( bmx != wx || bmy != wy )
        {
            m.win( bmx, bmy, w );
            wx = bmx;
            wy = bmy;
        }
    };
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
        tmp[1][0] = bpx;
        tmp[1][1] = bpy;
        // COST_MV_HPEL of slot 0 (the clipped mvp) and of the valid predictors
        int cpred[4] = { 0, 0, 0, 0 };
        if( role >= 0 )
            lr_batch4<NG>( role, [&]( int k ) {
                const int j = k <= valid ? k : 0;
                const int mx = tmp[j + 1][0], my = tmp[j + 1][1];
                return m.qpel( mx, my, false ) + m.cmx[mx] + m.cmy[my];
            }, cpred );
        else
            cpred[0] = m.qpel( bpx, bpy, false ) + m.cmx[bpx] + m.cmy[bpy];
        bpred_cost = cpred[0];
        const int pmv_cost = bpred_cost;
        if( valid > 0 )
        {
            bpred_cost <<= 4;
            for( int i = 1; i <= valid; i++ )
            {
                const int mx = tmp[i + 1][0], my = tmp[i + 1][1];
                const int c = role >= 0 && i < 4 ? (i == 1 ? cpred[1] : i == 2 ? cpred[2] : cpred[3])
                                                 : m.qpel( mx, my, false ) + m.cmx[mx] + m.cmy[my];
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
        // the integer search's first window, at the rounded predictor, and the (0, 0)
        // candidate's rows go out together: COST_MV( bmx, bmy ) is the window's centre, and
        // the search starts from this window unless (0, 0) wins -- one memory round where
        // the candidates in turn took three
        m.win( bmx, bmy, w );
        wx = bmx;
        wy = bmy;
        const int z = m.fpel( 0, 0 );
        if( bpred_mv & 0x00030003u )
            bcost = m.template wsad<0, 0>( w ) + m.bits_mvd( bmx, bmy );
        else
            bcost = bpred_cost;
        if( pmv )
        {
            if( bmx | bmy )
            {
                const int c0 = z + m.bits_mvd( 0, 0 );
                if( c0 < bcost )
                {
                    bcost = c0;
                    bmx = bmy = 0;
                }
            }
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
            window();
            costs[0] = m.template wsad<0, -1>( w ) + m.bits_mvd( bmx, bmy - 1 );
            costs[1] = m.template wsad<0, 1>( w ) + m.bits_mvd( bmx, bmy + 1 );
            costs[2] = m.template wsad<-1, 0>( w ) + m.bits_mvd( bmx - 1, bmy );
            costs[3] = m.template wsad<1, 0>( w ) + m.bits_mvd( bmx + 1, bmy );
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
#define LR_W( DX, DY, W ) (m.template wsad<DX, DY>( W ) + m.bits_mvd( bmx + (DX), bmy + (DY) ))
        {
            window();
            costs[0] = LR_W( -2, 0, w );
            costs[1] = LR_W( -1, 2, w );
            costs[2] = LR_W( 1, 2, w );
            costs[4] = LR_W( 2, 0, w );
            costs[5] = LR_W( 1, -2, w );
            costs[6] = LR_W( -1, -2, w );
        }
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
            bmx += lr_hex2_x( dir + 1 );
            bmy += lr_hex2_y( dir + 1 );
            for( int i = (me_range >> 1) - 1; i > 0 && m.in_range( bmx, bmy ); i-- )
            {
                // the window scores all six hexagon points (c_hex2[0..5] order); the three
                // the reference evaluates in this direction, c_hex2[dir .. dir+2], are picked
                window();
                const int s6[6] = { m.template wsad<-1, -2>( w ), m.template wsad<-2, 0>( w ),
                                    m.template wsad<-1, 2>( w ), m.template wsad<1, 2>( w ),
                                    m.template wsad<2, 0>( w ), m.template wsad<1, -2>( w ) };
                auto pick = [&]( int j ) {
                    j -= j >= 6 ? 6 : 0;
                    return j == 0 ? s6[0] : j == 1 ? s6[1] : j == 2 ? s6[2] : j == 3 ? s6[3] : j == 4 ? s6[4] : s6[5];
                };
#pragma unroll
                for( int k = 0; k < 3; k++ )
                    costs[k] = pick( dir + k ) + m.bits_mvd( bmx + lr_hex2_x( dir + k ), bmy + lr_hex2_y( dir + k ) );
                bcost &= ~7;
                bcost = min( bcost, (costs[0] << 3) + 1 );
                bcost = min( bcost, (costs[1] << 3) + 2 );
                bcost = min( bcost, (costs[2] << 3) + 3 );
                if( !(bcost & 7) )
                    break;
                dir += (bcost & 7) - 2;
                dir = lr_mod6m1( dir + 1 );
                bmx += lr_hex2_x( dir + 1 );
                bmy += lr_hex2_y( dir + 1 );
            }
        }
        bcost >>= 3;
        bcost <<= 4;
        {
            window();                                    // the last hexagon step's, unless it moved
            const int c8[8] = { LR_W( 0, -1, w ), LR_W( 0, 1, w ), LR_W( -1, 0, w ), LR_W( 1, 0, w ),
                                LR_W( -1, -1, w ), LR_W( -1, 1, w ), LR_W( 1, -1, w ), LR_W( 1, 1, w ) };
#pragma unroll
            for( int k = 1; k <= 8; k++ )
                bcost = min( bcost, (c8[k - 1] << 4) + k );
        }
#undef LR_W
        bmx += lr_square1_x( bcost & 15 );
        bmy += lr_square1_y( bcost & 15 );
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
            if( role >= 0 )
            {
                int c4[4];
                lr_batch4<NG>( role, [&]( int k ) {
                    const int qx = omx + (k == 2 ? -2 : k == 3 ? 2 : 0), qy = omy + (k == 0 ? -2 : k == 1 ? 2 : 0);
                    return m.qpel( qx, qy, false ) + m.cmx[qx] + m.cmy[qy];
                }, c4 );
#pragma unroll
                for( int r = 0; r < 4; r++ )
                    costs[r] = c4[r];
            }
            else
            {
                costs[0] = m.qpel( omx, omy - 2, false ) + m.cmx[omx] + m.cmy[omy - 2];
                costs[1] = m.qpel( omx, omy + 2, false ) + m.cmx[omx] + m.cmy[omy + 2];
                costs[2] = m.qpel( omx - 2, omy, false ) + m.cmx[omx - 2] + m.cmy[omy];
                costs[3] = m.qpel( omx + 2, omy, false ) + m.cmx[omx + 2] + m.cmy[omy];
            }
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
    // COST_MV_SATD( bmx, bmy, -1 ) (me.c:925 for the lookahead's refine): with the lane groups,
    // in the first qpel iteration's memory round -- every group reads the centre beside its
    // own candidate(s); else (no qpel step, the mv limits, one group) on its own
    bool rescored = !m.satd;
    int bdir = -1;
    for( int i = qpel; i > 0; i-- )
    {
        if( bmy <= m.smin1 || bmy >= m.smax1 || bmx <= m.smin0 || bmx >= m.smax0 )
            break;
        const int odir = bdir;
        const int omx = bmx, omy = bmy;
        int cq[4] = { 0, 0, 0, 0 };
        auto qpos = [&]( int k, int &qx, int &qy ) __attribute__( ( always_inline ) ) {
            qx = omx + (k == 2 ? -1 : k == 3 ? 1 : 0);
            qy = omy + (k == 0 ? -1 : k == 1 ? 1 : 0);
        };
        if( role >= 0 && !rescored )
        {
            if constexpr( NG == 4 )
            {
                int ax[2] = { omx, 0 }, ay[2] = { omy, 0 }, c2[2];
                const bool st[2] = { true, m.satd != 0 };
                qpos( role, ax[1], ay[1] );
                m.qpel_n( ax, ay, st, c2 );
                bcost = c2[0];
#pragma unroll
                for( int r = 0; r < 4; r++ )
                    cq[r] = lr_gather<4>( c2[1], r );
            }
            else
            {
                int ax[3] = { omx, 0, 0 }, ay[3] = { omy, 0, 0 }, c3[3];
                const bool st[3] = { true, m.satd != 0, m.satd != 0 };
                qpos( role, ax[1], ay[1] );
                qpos( role + 2, ax[2], ay[2] );
                m.qpel_n( ax, ay, st, c3 );
                bcost = c3[0];
                cq[0] = lr_gather<2>( c3[1], 0 );
                cq[1] = lr_gather<2>( c3[1], 1 );
                cq[2] = lr_gather<2>( c3[2], 0 );
                cq[3] = lr_gather<2>( c3[2], 1 );
            }
            rescored = true;
        }
        else
        {
            if( !rescored )
            {
                bcost = m.qpel( bmx, bmy, true ) + m.cmx[bmx] + m.cmy[bmy];
                rescored = true;
            }
            if( role >= 0 )
                lr_batch4<NG>( role, [&]( int k ) {
                    int qx, qy;
                    qpos( k, qx, qy );
                    return m.qpel( qx, qy, m.satd ) + m.cmx[qx] + m.cmy[qy];
                }, cq );
        }
#pragma unroll
        for( int dir = 0; dir < 4; dir++ )
        {
            if( (dir ^ 1) == odir )
                continue;
            const int qx = omx + (dir == 2 ? -1 : dir == 3 ? 1 : 0), qy = omy + (dir == 0 ? -1 : dir == 1 ? 1 : 0);
            const int cc = role >= 0 ? cq[dir] : m.qpel( qx, qy, m.satd ) + m.cmx[qx] + m.cmy[qy];
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
    if( !rescored )
        bcost = m.qpel( bmx, bmy, true ) + m.cmx[bmx] + m.cmy[bmy];
    omvx = bmx;
    omvy = bmy;
    ocost = bcost;
}

// one list of slicetype_mb_cost (slicetype.c:645-702): reverse-order predictors from the
// row ring of this pass, the near-zero fast skip, x264_me_search and the cost
// adjustments.  Returns the list cost; mvx / mvy the list's mv.
template <int BD, int NG = 4>
__device__ __forceinline__ int lr_list( LrCtx<BD> &m, const uint32_t (&pred)[4], int npred, int me_method, int subme,
                                        int me_range, int lambda, const uint16_t *cost_mv, int &mvx, int &mvy,
                                        int role = -1 )
{
    int mvc[4][2] = { { 0, 0 }, { 0, 0 }, { 0, 0 }, { 0, 0 } };
    const int i_mvc = npred;
#pragma unroll
    for( int i = 0; i < 4; i++ )
    {
        mvc[i][0] = (int16_t)(pred[i] & 0xffff);
        mvc[i][1] = (int16_t)(pred[i] >> 16);
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
    int cost = 0;
    mvx = mvy = 0;
    bool skip = false;
    if( !mvpx && !mvpy )
    {
        // fast skip of near-zero residual blocks (slicetype.c:677-686): m[l].p_fref[0], the
        // unweighted F plane, even in the weighted form
        cost = m.template qpel<false>( 0, 0, m.satd );
        skip = cost < 64;
    }
    if( !skip )
    {
        lr_me_search<BD, NG>( m, mvpx, mvpy, mvc, i_mvc, me_method, subme, me_range, role, mvx, mvy, cost );
        cost -= cost_mv[0];
        if( mvx | mvy )
            cost += 5 * lambda;
    }
    return cost;
}


// ---- multi-workgroup wavefront ----
// A frame pair's block rows are split into bands of LR_BAND rows, one single-wave
// workgroup each.  A band's rows take their predictors from the LDS ring of the
// band, except the band's bottom row, whose row-below predictors (x-1, x, x+1 of
// row y1, written by the band underneath at steps t-1 .. t-3) are read from the
// mvs output itself: the launcher fills it with a sentinel no mv can take, the
// producer stores each block's mv as one 32-bit word, and the consumer waits
// until the three words it needs are no longer the sentinel.  Only bottom-up
// waits exist and the band underneath has the lower workgroup index, so it is
// dispatched first and never waits on a later workgroup.
constexpr int LR_BAND = 16;                      // max block rows per workgroup (one wave of lane quads)
constexpr uint32_t LR_SENTINEL = 0x80808080u;    // mv (-32640, -32640): outside any mv range

__device__ __forceinline__ uint32_t lr_load_mv( const uint32_t *p )
{
    return __hip_atomic_load( p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
}
__device__ __forceinline__ void lr_store_mv( uint32_t *p, uint32_t v )
{
    __hip_atomic_store( p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
}

// the predictors of block (x, y) in slicetype_mb_cost's order (slicetype.c:651-663):
// right, then below, below-left, below-right.  Returns -1 when the row-below words did
// not arrive within poll_max tries (or another band already failed): the caller's band
// then stops, and the launcher reports the failure instead of letting sentinel words
// act as predictors.
__device__ __forceinline__ int lr_preds( const int *ring, int y0, int y1, const uint32_t *gmv, int x, int y, int mbw,
                                         int send, uint32_t (&pred)[4], int poll_max, uint32_t *status )
{
    int n = 0;
#pragma unroll
    for( int i = 0; i < 4; i++ )
        pred[i] = 0;
    if( x < mbw - 1 )
        pred[n++] = (uint32_t)ring[4 * (y - y0) + ((x + 1) & 3)];
    if( y < send - 1 )                           // the slice's last row has no row below
    {
        uint32_t b = 0, bl = 0, br = 0;
        if( y + 1 < y1 )
        {
            b = (uint32_t)ring[4 * (y + 1 - y0) + (x & 3)];
            if( x > 0 )
                bl = (uint32_t)ring[4 * (y + 1 - y0) + ((x - 1) & 3)];
            if( x < mbw - 1 )
                br = (uint32_t)ring[4 * (y + 1 - y0) + ((x + 1) & 3)];
        }
        else
        {
            const uint32_t *row = gmv + (intptr_t)(y + 1) * mbw;
            bool ok = false;
            for( int it = 0; it < poll_max; it++ )   // bounded: a broken schedule ends, never hangs
            {
                b = lr_load_mv( row + x );
                bl = x > 0 ? lr_load_mv( row + x - 1 ) : 0;
                br = x < mbw - 1 ? lr_load_mv( row + x + 1 ) : 0;
                if( b != LR_SENTINEL && bl != LR_SENTINEL && br != LR_SENTINEL )
                {
                    ok = true;
                    break;
                }
                if( lr_load_mv( status ) )           // a band below gave up: so does this one
                    break;
                __builtin_amdgcn_s_sleep( 2 );
            }
            if( !ok )
            {
                __hip_atomic_fetch_or( status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
                return -1;
            }
        }
        pred[n++] = b;
        if( x > 0 )
            pred[n++] = bl;
        if( x < mbw - 1 )
            pred[n++] = br;
    }
    return n;
}


// The mv cost table staged in LDS: every candidate's cost reads p_cost_mvx/y at an index
// that depends on the previous decision, so these lookups sit on the search's serial
// chain; |index| <= 2 * (2 * mv_range) + 3 (an mv and a predictor, both within the
// lowres mv limits), the staged span keeps a margin on top.
__device__ __forceinline__ int lr_cost_span( int mv_range ) { return 4 * mv_range + 64; }
__device__ __forceinline__ const uint16_t *lr_stage_cost( uint16_t *lds, const uint16_t *cost_mv, int mv_range )
{
    const int span = lr_cost_span( mv_range );
    for( int i = threadIdx.x; i <= 2 * span; i += blockDim.x )
        lds[i] = cost_mv[i - span];
    __syncthreads();
    return lds + span;
}

template <int BD>
__device__ __forceinline__ void lr_load_fenc( const typename PT<BD>::pixel *fb, intptr_t stride,
                                              uint32_t (&fe)[LR_NR][8 / PT<BD>::PPD] )
{
#pragma unroll
    for( int r = 0; r < LR_NR; r++ )
    {
        const uint32_t *row = (const uint32_t *)(fb + (intptr_t)r * stride);
#pragma unroll
        for( int k = 0; k < 8 / PT<BD>::PPD; k++ )
            fe[r][k] = row[k];
    }
}

// The band a workgroup runs: pair f, band j.  xpairs = 0: block b is band b % nbands of pair
// b / nbands.  Else every band of a pair runs on one XCD (the dispatcher deals blocks
// round-robin over the 8 XCDs, block b on XCD b % 8): XCD x's i-th block is band i % nbands
// of pair x + 8 * (i / nbands), so the bands that share reference rows and hand mvs over
// share an L2, and a band's producer (band j - 1, block b - 8) is still dispatched first.
// Blocks past the last pair (xpairs not a multiple of 8) return.
__device__ __forceinline__ bool lr_unit( int nbands, int xpairs, int &f, int &j )
{
    if( !xpairs )
    {
        f = (int)blockIdx.x / nbands;
        j = (int)blockIdx.x % nbands;
        return true;
    }
    const int x = (int)(blockIdx.x & 7), i = (int)(blockIdx.x >> 3);
    f = x + 8 * (i / nbands);
    j = i % nbands;
    return f < xpairs;
}

// The helper wave (la_help): a second wave in the band's workgroup that reads,
// LR_AHEAD steps before the searching wave gets there, one dword of every pixel row the band's
// searches can reach in the column its blocks enter -- the reference planes (rows 8*y0 - 16 ..
// 8*y1 + 16, one per lane) and fenc -- so the search finds those lines in L2.  Its loads wait
// on its own counters, not the searching wave's.  It follows the searching wave's step
// through an LDS word (`prog`, > t1 when the band is done or has failed) and stops after
// `poll_max` polls in any case.
constexpr int LR_AHEAD = 4;
template <int BD, int NP>
__device__ __forceinline__ void lr_helper( const typename PT<BD>::pixel *const (&pl)[NP],
                                        const typename PT<BD>::pixel *fenc, intptr_t stride, int mbw, int s1, int y0,
                                        int y1, int t0, int t1, int &prog, int poll_max )
{
    const int r = 8 * y0 - 16 + (int)(threadIdx.x & 63);
    const int yb = min( max( r >> 3, y0 ), y1 - 1 );
    const bool in_band = r >= 8 * y0 && r < 8 * y1;
    // rows past the band's reach stay unread: a one-row last band (y0 = mbh - 1) would otherwise
    // read up to row 8 * mbh + 39, past the 32-row padding of the plane's last frame
    const bool in_reach = r < 8 * y1 + 16;
    uint32_t acc = 0;
    int done = t0 - 1;
    for( int it = 0; it < poll_max; it++ )
    {
        const int cur = __hip_atomic_load( &prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP );
        if( cur > t1 )
            break;
        const int target = min( cur + LR_AHEAD, t1 );
        while( done < target )
        {
            done++;
            const int x = min( max( mbw - 1 - (done - 2 * (s1 - 1 - yb)), 0 ), mbw - 1 );
            const intptr_t o = (intptr_t)r * stride + ((8 * x - 24) & ~(4 / (int)sizeof( typename PT<BD>::pixel ) - 1));
            if( in_reach )
#pragma unroll
                for( int k = 0; k < NP; k++ )
                    acc += *(const uint32_t *)(pl[k] + o);
            if( in_band )
                acc += *(const uint32_t *)(fenc + (intptr_t)r * stride + 8 * x);
        }
        __asm__ volatile( "" ::"v"( acc ) );
        __builtin_amdgcn_s_sleep( 1 );
    }
}
// the searching wave's step for the helper (an LDS word: ds_write, not a flat store)
__device__ __forceinline__ void lr_prog_set( int &prog, int v )
{
    __hip_atomic_store( &prog, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP );
}
// the searching wave's step barrier when the helper shares the workgroup: the ring is the
// one wave's own LDS, so ordering its accesses is enough
__device__ __forceinline__ void lr_wave_sync()
{
    __builtin_amdgcn_fence( __ATOMIC_SEQ_CST, "wavefront" );
    __builtin_amdgcn_wave_barrier();
}

// Lookahead slices (i_lookahead_threads, slicetype.c:901-918): slice i holds MB rows
// [(H*i + T/2)/T, (H*(i+1) + T/2)/T) and is its own wavefront (slicetype_slice_cost scans it
// alone; its row-below predictors stop at the slice end, slicetype.c:664).  Band j of a
// pair: bands are counted slice by slice, bottom band first inside a slice, so a band's
// producer (the band under it, same slice) always has the lower index.
__device__ __forceinline__ void lr_band( int j, int mbh, int nslices, int brows, int &s1, int &y0, int &y1 )
{
    s1 = y0 = y1 = 0;
    for( int i = 0; i < nslices; i++ )
    {
        const int a = (mbh * i + nslices / 2) / nslices, b = (mbh * (i + 1) + nslices / 2) / nslices;
        const int nb = (b - a + brows - 1) / brows;
        if( j < nb )
        {
            s1 = b;
            y1 = b - j * brows;
            y0 = max( a, y1 - brows );
            return;
        }
        j -= nb;
    }
}

// WGT: the weighted-reference form (rw, the scale / denom / offset); the unweighted kernel
// carries none of its code or live values
template <int BD, bool WGT, bool LAT>
__global__ __launch_bounds__( 128 ) void lowres_inter_kernel(
    const typename PT<BD>::pixel *__restrict__ fenc, intptr_t ffs, const typename PT<BD>::pixel *r0,
    intptr_t rpd,
    intptr_t stride, intptr_t rfs, int mbw, int mbh, int me_method, int subme, int satd, int me_range, int mv_range,
    int lambda, const uint16_t *__restrict__ cost_mv, const uint16_t *__restrict__ intra_cost,
    const uint16_t *__restrict__ invq, int16_t *__restrict__ mvs, int32_t *__restrict__ mv_costs,
    uint16_t *__restrict__ lcosts, int32_t *__restrict__ row_satd, int32_t *__restrict__ est, int nbands, int brows,
    int poll_max, uint32_t *status, const typename PT<BD>::pixel *rw, intptr_t wfs, int wscale, int wdenom,
    int woffset, int nslices, int help, int xpairs )
{
    constexpr int NDW = LrCtx<BD>::NDW;
    __shared__ int ring[4 * LR_BAND];            // packed MVs of each band row's 4 latest blocks
    __shared__ int prog;                         // the searching wave's step (helper wave)
    extern __shared__ uint16_t lr_cost_lds[];
    const uint16_t *cml = lr_stage_cost( lr_cost_lds, cost_mv, mv_range );
    int f, jb;
    if( !lr_unit( nbands, xpairs, f, jb ) )
        return;
    int s1, y0, y1;                               // the band's rows [y0, y1) of a slice ending at s1
    lr_band( jb, mbh, nslices, brows, s1, y0, y1 );
    const int nmb = mbw * mbh;
    fenc += (intptr_t)f * ffs;
    r0 += (intptr_t)f * rfs;
    if( WGT )
        rw += (intptr_t)f * wfs;
    intra_cost += (intptr_t)f * nmb;
    if( invq )
        invq += (intptr_t)f * nmb;
    mvs += 2 * (intptr_t)f * nmb;
    mv_costs += (intptr_t)f * nmb;
    lcosts += (intptr_t)f * nmb;
    // LAT (a launch whose bands are all resident: each step's latency is the time): the output
    // pointers, stored to once per step, held in VGPRs (an opaque per-lane zero added) --
    // scalar registers are the kernel's scarce ones (their spills go through VGPR lanes); the
    // extra VGPRs cost a wave per SIMD, which a queued (throughput) launch keeps
    if constexpr( LAT )
    {
        int z;
        asm volatile( "v_mov_b32 %0, 0" : "=v"( z ) );
        mv_costs += z;
        lcosts += z;
        intra_cost += z;
        mvs += z;
        fenc += z;
        if( invq )
            invq += z;
        if( row_satd )
            row_satd += z;
    }
    uint32_t *gmv = (uint32_t *)mvs;
    int e0 = 0, e1 = 0, e2 = 0, racc = 0;
    const int mvr = 2 * mv_range;
    const int q = threadIdx.x & 3;
    // four 16-lane groups run each row's search together and split its candidate batches
    // (lr_me_search's role); group 0 writes the results
    const int role = (int)(threadIdx.x >> 4);
    const int y = y0 + (int)((threadIdx.x & 15) >> 2);
    // steps in which this band has blocks (block (x, y) runs at (W-1-x) + 2(s1-1-y))
    const int t0 = 2 * (s1 - y1), t1 = 2 * (s1 - 1 - y0) + mbw - 1;
    if( help )
    {
        if( threadIdx.x == 0 )
            lr_prog_set( prog, t0 );
        __syncthreads();
        if( threadIdx.x >= 64 )
        {
            const typename PT<BD>::pixel *const hpl[5] = { r0, r0 + rpd, r0 + 2 * rpd, r0 + 3 * rpd, WGT ? rw : r0 };
            lr_helper<BD, 5>( hpl, fenc, stride, mbw, s1, y0, y1, t0, t1, prog, poll_max );
            return;
        }
    }
    // a row's next block is x - 1: its fenc rows, intra cost and AQ factor are fetched one
    // step ahead (read after the search, they would add a memory round to every step)
    uint32_t fnext[LR_NR][NDW];
    int inext = 0, qnext = 0;
    auto fetch = [&]( int t ) {
        const int xn = mbw - 1 - (t - 2 * (s1 - 1 - y));
        if( y < y1 && xn >= 0 && xn < mbw )
        {
            lr_load_fenc<BD>( fenc + 8 * (intptr_t)xn + (intptr_t)(8 * y + LR_NR * q) * stride, stride, fnext );
            inext = intra_cost[xn + y * mbw];
            if( invq )
                qnext = invq[xn + y * mbw];
        }
    };
    fetch( t0 );
    for( int t = t0; t <= t1; t++ )
    {
        const int x = mbw - 1 - (t - 2 * (s1 - 1 - y));
        uint32_t fe[LR_NR][NDW];
#pragma unroll
        for( int r = 0; r < LR_NR; r++ )
#pragma unroll
            for( int k = 0; k < NDW; k++ )
                fe[r][k] = fnext[r][k];
        const int icost = inext, iq = qnext;
        fetch( t + 1 );
        bool failed = false;
        if( y < y1 && x >= 0 && x < mbw )
        {
            const int mb = x + y * mbw;
            const intptr_t off = 8 * (intptr_t)x + 8 * (intptr_t)y * stride;
            LrCtx<BD> m( fe );
            m.setup( r0, rpd, off, stride, x, y, mbw, mbh, mvr, satd, q );
            if constexpr( WGT )
                m.set_weight( rw, off, wscale, wdenom, woffset );
            uint32_t pred[4];
            const int np = lr_preds( ring, y0, y1, gmv, x, y, mbw, s1, pred, poll_max, status );
            // the lanes of the band share candidate batches: a failed wait stops them all
            failed = __builtin_amdgcn_ballot_w64( np < 0 ) != 0;
            int mvx = 0, mvy = 0, cost = 0;
            if( !failed )
                cost = lr_list<BD>( m, pred, np, me_method, subme, me_range, lambda, cml, mvx, mvy, role );
            if( !failed && q == 0 && role == 0 )
            {
                ring[4 * (y - y0) + (x & 3)] = (int)lr_pack( mvx, mvy );
                lr_store_mv( gmv + mb, lr_pack( mvx, mvy ) );
                mv_costs[mb] = cost;
                // slicetype.c:758-790
                int bcost = (cost >> (BD - 8)) + 4, list_used = 1;
                const bool fsm = (x > 0 && x < mbw - 1 && y > 0 && y < mbh - 1) || mbw <= 2 || mbh <= 2;
                const bool b_intra = icost < bcost;
                if( b_intra )
                {
                    bcost = icost;
                    list_used = 0;
                }
                const int aq = invq ? (bcost * iq + 128) >> 8 : bcost;
                racc += aq;
                if( fsm )
                {
                    e0 += bcost;
                    e1 += aq;
                    e2 += b_intra;
                }
                lcosts[mb] = (uint16_t)(min( bcost, 16383 ) + (list_used << 14));
            }
        }
        if( __builtin_amdgcn_ballot_w64( failed ) )
        {
            if( help && threadIdx.x == 0 )
                lr_prog_set( prog, t1 + 1 );
            return;                                  // the launcher reports it (status word)
        }
        // one searching wave per band: ordering its own LDS ring accesses is enough (a
        // __syncthreads here also waited for the step's global stores to drain)
        lr_wave_sync();
        if( help && threadIdx.x == 0 )
            lr_prog_set( prog, t + 1 );
    }
    if( q == 0 && role == 0 && y < y1 && row_satd )
        row_satd[(intptr_t)f * mbh + y] = racc;
    if( est && (e0 | e1 | e2) )
    {
        atomicAdd( &est[3 * f], e0 );
        atomicAdd( &est[3 * f + 1], e1 );
        atomicAdd( &est[3 * f + 2], e2 );
    }
}

// pixel_avg / pixel_avg_weight_wxh (mc.c:49-87) of two packed dwords: the rounding
// average at weight 32, else (a*w + b*(64-w) + 32) >> 6 in 16-bit lanes (w in [0, 64]:
// no clipping needed, 1023*64 + 32 < 2^16)
template <int BD> __device__ __forceinline__ uint32_t lr_wavg( uint32_t a, uint32_t b, int w )
{
    if( w == 32 )
        return avg_round<BD>( a, b );
    typedef unsigned short us2 __attribute__( ( ext_vector_type( 2 ) ) );
    const us2 wa = (us2)(unsigned short)w, wb = (us2)(unsigned short)(64 - w);
    auto f = [&]( uint32_t x, uint32_t y ) {
        const us2 r = (__builtin_bit_cast( us2, x ) * wa + __builtin_bit_cast( us2, y ) * wb + (us2)32) >> (us2)6;
        return __builtin_bit_cast( uint32_t, r );
    };
    if constexpr( BD == 8 )
    {
        const uint32_t lo = f( __builtin_amdgcn_perm( 0u, a, 0x0c020c00u ), __builtin_amdgcn_perm( 0u, b, 0x0c020c00u ) );
        const uint32_t hi = f( __builtin_amdgcn_perm( 0u, a, 0x0c030c01u ), __builtin_amdgcn_perm( 0u, b, 0x0c030c01u ) );
        return __builtin_amdgcn_perm( hi, lo, 0x06020400u );
    }
    else
        return f( a, b );
}

// TRY_BIDIR (slicetype.c:589-612): the weighted average of the two lists' predictions
// scored with mbcmp; hpel = the subme <= 1 form (hpel planes addressed directly)
template <int BD>
__device__ __forceinline__ int lr_bidir( const LrCtx<BD> &m0, const LrCtx<BD> &m1, int ax, int ay, int bx, int by,
                                         bool hpel, int w )
{
    constexpr int NDW = LrCtx<BD>::NDW;
    uint32_t ra[LR_NR][NDW], rb[LR_NR][NDW];
    if( hpel )
    {
        m0.hpel_rows( ax, ay, ra );
        m1.hpel_rows( bx, by, rb );
    }
    else
    {
        m0.ref_rows( ax, ay, ra );
        m1.ref_rows( bx, by, rb );
    }
#pragma unroll
    for( int y = 0; y < LR_NR; y++ )
#pragma unroll
        for( int k = 0; k < NDW; k++ )
            ra[y][k] = lr_wavg<BD>( ra[y][k], rb[y][k], w );
    return lr_cmp_rows<BD>( m0.fe, ra, m0.satd, m0.q );
}

// B frames (p0 < b < p1): slicetype_mb_cost with b_bidir (slicetype.c:514-713, 758-791).
// A list is searched on the wavefront when search & (1 << l), else its mv / cost are read.
template <int BD>
__global__ __launch_bounds__( 128 ) void lowres_bidir_kernel(
    const typename PT<BD>::pixel *__restrict__ fenc, intptr_t ffs, const typename PT<BD>::pixel *a0, intptr_t apd,
    intptr_t afs, const typename PT<BD>::pixel *b0, intptr_t bpd, intptr_t bfs, intptr_t stride, int mbw,
    int mbh, int me_method, int subme, int satd, int me_range, int mv_range, int lambda,
    const uint16_t *__restrict__ cost_mv, int search, int16_t *__restrict__ mvs0, int32_t *__restrict__ costs0,
    int16_t *__restrict__ mvs1, int32_t *__restrict__ costs1, const int16_t *__restrict__ p1mvs, int dsf, int weight,
    const uint16_t *__restrict__ invq, uint16_t *__restrict__ lcosts, int32_t *__restrict__ row_satd,
    int32_t *__restrict__ est, int nbands, int brows, int poll_max, uint32_t *status, int nslices, int help,
    int xpairs )
{
    constexpr int NDW = LrCtx<BD>::NDW;
    __shared__ int ring0[4 * LR_BAND], ring1[4 * LR_BAND];      // per list
    __shared__ int prog;                                        // the searching wave's step
    extern __shared__ uint16_t lr_cost_lds[];
    const uint16_t *cml = lr_stage_cost( lr_cost_lds, cost_mv, mv_range );
    int f, jb;
    if( !lr_unit( nbands, xpairs, f, jb ) )
        return;
    int s1, y0, y1;                               // the band's rows [y0, y1) of a slice ending at s1
    lr_band( jb, mbh, nslices, brows, s1, y0, y1 );
    const int nmb = mbw * mbh;
    fenc += (intptr_t)f * ffs;
    a0 += (intptr_t)f * afs;
    b0 += (intptr_t)f * bfs;
    if( invq )
        invq += (intptr_t)f * nmb;
    if( p1mvs )
        p1mvs += 2 * (intptr_t)f * nmb;
    mvs0 += 2 * (intptr_t)f * nmb;
    mvs1 += 2 * (intptr_t)f * nmb;
    costs0 += (intptr_t)f * nmb;
    costs1 += (intptr_t)f * nmb;
    lcosts += (intptr_t)f * nmb;
    uint32_t *gmv0 = (uint32_t *)mvs0, *gmv1 = (uint32_t *)mvs1;
    int e0 = 0, e1 = 0, racc = 0;
    const int mvr = 2 * mv_range;
    const int q = threadIdx.x & 3;
    const bool hp = subme == 2;                  // h->param.analyse.i_subpel_refine <= 1
    // The wave's four 16-lane groups (roles) work on the same <= 4 block rows at once:
    // roles 0 / 2 run the list-0 search and roles 1 / 3 the list-1 search as one instruction
    // stream (the same code on per-lane planes, ring and mvs; each list's two groups split its
    // candidate batches), then roles 0, 1, 2 run the three TRY_BIDIR evaluations together (the
    // p1-predicted pair, (0, 0), the searched pair); role 0 gathers the values and makes
    // slicetype_mb_cost's decisions in its order.
    const int role = (int)(threadIdx.x >> 4);
    const int rl = (int)(threadIdx.x & 15);      // lane within the role: 4 * row + q
    const int y = y0 + (rl >> 2);
    const bool mine = y < y1;                    // (role 3 helps the list-1 search)
    const int t0 = 2 * (s1 - y1), t1 = 2 * (s1 - 1 - y0) + mbw - 1;
    if( help )
    {
        if( threadIdx.x == 0 )
            lr_prog_set( prog, t0 );
        __syncthreads();
        if( threadIdx.x >= 64 )
        {
            const typename PT<BD>::pixel *const hpl[8] = { a0, a0 + apd, a0 + 2 * apd, a0 + 3 * apd,
                                                           b0, b0 + bpd, b0 + 2 * bpd, b0 + 3 * bpd };
            lr_helper<BD, 8>( hpl, fenc, stride, mbw, s1, y0, y1, t0, t1, prog, poll_max );
            return;
        }
    }
    // a row's next block is x - 1: its fenc rows, p1 mv and AQ factor are fetched one step
    // ahead (read after the searches, they would add a memory round to every step)
    uint32_t fnext[LR_NR][NDW];
    uint32_t pnext = 0;
    int qnext = 0;
    auto fetch = [&]( int t ) {
        const int xn = mbw - 1 - (t - 2 * (s1 - 1 - y));
        if( mine && xn >= 0 && xn < mbw )
        {
            lr_load_fenc<BD>( fenc + 8 * (intptr_t)xn + (intptr_t)(8 * y + LR_NR * q) * stride, stride, fnext );
            if( p1mvs )
                pnext = *(const uint32_t *)(p1mvs + 2 * (xn + y * mbw));
            if( invq )
                qnext = invq[xn + y * mbw];
        }
    };
    auto from_role = [&]( int v, int r ) { return __shfl( v, rl + 16 * r ); };
    fetch( t0 );
    for( int t = t0; t <= t1; t++ )
    {
        const int x = mbw - 1 - (t - 2 * (s1 - 1 - y));
        uint32_t fe[LR_NR][NDW];
#pragma unroll
        for( int r = 0; r < LR_NR; r++ )
#pragma unroll
            for( int k = 0; k < NDW; k++ )
                fe[r][k] = fnext[r][k];
        const uint32_t p1w = pnext;
        const int iq = qnext;
        fetch( t + 1 );
        const bool act = mine && x >= 0 && x < mbw;
        const int mb = x + y * mbw;
        const intptr_t off = 8 * (intptr_t)x + 8 * (intptr_t)y * stride;
        LrCtx<BD> m0( fe ), m1( fe ), ms( fe );
        int mvx = 0, mvy = 0, lc = 0;
        bool failed = false;
        if( act )
        {
            m0.setup( a0, apd, off, stride, x, y, mbw, mbh, mvr, satd, q );
            m1.setup( b0, bpd, off, stride, x, y, mbw, mbh, mvr, satd, q );
            {
                // every role searches: list `lst` = role & 1 on groups lg = role >> 1 (two
                // groups per list split its candidate batches); the searching lanes' own
                // context: the list's planes (a per-lane choice of pointers, not of objects,
                // so nothing goes to scratch)
                const int lst = role & 1, lg = role >> 1;
                ms.setup( lst ? b0 : a0, lst ? bpd : apd, off, stride, x, y, mbw, mbh, mvr, satd, q );
                // list `lst`: searched on the wavefront (search & (1 << lst)) or read
                int *ring = lst ? ring1 : ring0;
                uint32_t *gmv = lst ? gmv1 : gmv0;
                int32_t *costs = lst ? costs1 : costs0;
                if( search & (1 << lst) )
                {
                    uint32_t pred[4];
                    const int np = lr_preds( ring, y0, y1, gmv, x, y, mbw, s1, pred, poll_max, status );
                    // the searching lanes run one instruction stream: a failed wait stops them all
                    failed = __builtin_amdgcn_ballot_w64( np < 0 ) != 0;
                    if( !failed )
                        lc = lr_list<BD, 2>( ms, pred, np, me_method, subme, me_range, lambda, cml, mvx, mvy, lg );
                    if( !failed && q == 0 && lg == 0 )
                    {
                        ring[4 * (y - y0) + (x & 3)] = (int)lr_pack( mvx, mvy );
                        lr_store_mv( gmv + mb, lr_pack( mvx, mvy ) );
                        costs[mb] = lc;
                    }
                }
                else
                {
                    const uint32_t v = gmv[mb];
                    mvx = (int16_t)(v & 0xffff);
                    mvy = (int16_t)(v >> 16);
                    lc = costs[mb];
                }
            }
        }
        if( __builtin_amdgcn_ballot_w64( failed ) )
        {
            if( help && threadIdx.x == 0 )
                lr_prog_set( prog, t1 + 1 );
            return;                                  // the launcher reports it (status word)
        }
        const int mv0x = from_role( mvx, 0 ), mv0y = from_role( mvy, 0 ), lc0 = from_role( lc, 0 );
        const int mv1x = from_role( mvx, 1 ), mv1y = from_role( mvy, 1 ), lc1 = from_role( lc, 1 );
        // the predicted bidir mvs from p1's list-0 mvs (slicetype.c:623-645)
        int d0x = 0, d0y = 0, d1x = 0, d1y = 0;
        if( act && p1mvs )
        {
            const int rx = (int16_t)(p1w & 0xffff), ry = (int16_t)(p1w >> 16);
            d0x = (rx * dsf + 128) >> 8;
            d0y = (ry * dsf + 128) >> 8;
            d1x = lr_clip3( d0x - rx, m0.smin0, m0.smax0 );
            d1y = lr_clip3( d0y - ry, m0.smin1, m0.smax1 );
            d0x = lr_clip3( d0x, m0.smin0, m0.smax0 );
            d0y = lr_clip3( d0y, m0.smin1, m0.smax1 );
            if( hp )
            {
                d0x &= ~1; d0y &= ~1; d1x &= ~1; d1y &= ~1;
            }
        }
        const bool dnz = (d0x | d0y | d1x | d1y) != 0, mvnz = (mv0x | mv0y | mv1x | mv1y) != 0;
        // TRY_BIDIR: role 0 the predicted pair, role 1 (0, 0) (when the prediction is not
        // zero), role 2 the searched pair (when not zero)
        int cb = LR_COST_MAX;
        if( act && (role == 0 || (role == 1 && dnz) || (role == 2 && mvnz)) )
        {
            const int ax = role == 0 ? d0x : role == 2 ? mv0x : 0, ay = role == 0 ? d0y : role == 2 ? mv0y : 0;
            const int bx = role == 0 ? d1x : role == 2 ? mv1x : 0, by = role == 0 ? d1y : role == 2 ? mv1y : 0;
            cb = lr_bidir<BD>( m0, m1, ax, ay, bx, by, role == 1 ? true : hp, weight );
        }
        const int cpred = from_role( cb, 0 ), czero = from_role( cb, 1 ), cmv = from_role( cb, 2 );
        if( act && role == 0 && q == 0 )
        {
            int bcost = LR_COST_MAX, list_used = 0;
            if( cpred < bcost )
            {
                bcost = cpred;
                list_used = 3;
            }
            if( dnz && czero < bcost )
            {
                bcost = czero;
                list_used = 3;
            }
            if( lc0 < bcost )
            {
                bcost = lc0;
                list_used = 1;
            }
            if( lc1 < bcost )
            {
                bcost = lc1;
                list_used = 2;
            }
            if( mvnz && 5 * lambda + cmv < bcost )
            {
                bcost = 5 * lambda + cmv;
                list_used = 3;
            }
            // slicetype.c:758-790 (no intra in B frames)
            bcost = (bcost >> (BD - 8)) + 4;
            const bool fsm = (x > 0 && x < mbw - 1 && y > 0 && y < mbh - 1) || mbw <= 2 || mbh <= 2;
            const int aq = invq ? (bcost * iq + 128) >> 8 : bcost;
            racc += aq;
            if( fsm )
            {
                e0 += bcost;
                e1 += aq;
            }
            lcosts[mb] = (uint16_t)(min( bcost, 16383 ) + (list_used << 14));
        }
        // one searching wave per band: ordering its own LDS ring accesses is enough (a
        // __syncthreads here also waited for the step's global stores to drain)
        lr_wave_sync();
        if( help && threadIdx.x == 0 )
            lr_prog_set( prog, t + 1 );
    }
    if( role == 0 && q == 0 && y < y1 && row_satd )
        row_satd[(intptr_t)f * mbh + y] = racc;
    if( est && (e0 | e1) )
    {
        atomicAdd( &est[2 * f], e0 );
        atomicAdd( &est[2 * f + 1], e1 );
    }
}

// The wavefront's status word: a per-thread, per-device device word the kernel sets when a
// band's wait for the band underneath ran out (lr_preds).  The wait can only run out if the
// schedule's premise breaks: the band a workgroup waits on has a lower index, and an XCD
// dispatches its workgroups in index order, so by induction the lowest unfinished workgroup
// is resident and never waits -- no residency bound on the batch is needed; the poll bound
// (X264HIP_LA_POLL, default 2^22 tries) turns a broken premise (preemption, a changed
// dispatcher) into this error rather than a hang.
// The launches stay asynchronous (and capturable into a graph): the word is sticky on the
// device, each launch queues a copy of it into pinned host memory behind the kernel and
// records an event, and the error is reported
//  * by the next lookahead entry on this thread and device once that copy has landed (the
//    entry then refuses with X264HIP_EDEVICE before launching anything), and
//  * by x264hip_lowres_status( stream ), which waits for the stream and reads the word.
// Reporting clears the word.  Under stream capture no copy is queued; the word is still set
// by the replayed kernels and x264hip_lowres_status reads it.
namespace {
// (no destructor: the words live as long as the process -- freeing them from a
// thread-exit destructor can run after the HIP runtime has been torn down, which
// crashed the process at exit under rocprofv3)
struct LaStatus
{
    int device = -1;
    uint32_t *dev = nullptr;
    uint32_t *host = nullptr;
    hipEvent_t ev = nullptr;
    bool pending = false;            // a copy of the word is queued behind a launch
};
// one slot per device, allocated on the device's first use and kept: a thread that alternates
// between devices keeps each device's word (and a timeout recorded on it) instead of trading
// one for the other
constexpr int LA_MAX_DEVICES = 64;
thread_local LaStatus t_la_status[LA_MAX_DEVICES];

// the status word of the stream's device for this thread (allocated on first use)
hipError_t la_status_get( hipStream_t stream, LaStatus **out )
{
    int d = 0;
    hipError_t e = stream_device( stream, &d );
    if( e != hipSuccess )
        return e;
    if( d < 0 || d >= LA_MAX_DEVICES )
        return hipErrorInvalidDevice;
    LaStatus &st = t_la_status[d];
    if( st.device != d )
    {
        int cur = 0;
        if( (e = hipGetDevice( &cur )) != hipSuccess || (cur != d && (e = hipSetDevice( d )) != hipSuccess) )
            return e;
        e = hipMalloc( (void **)&st.dev, sizeof( uint32_t ) );
        if( e == hipSuccess )
            e = hipMemset( st.dev, 0, sizeof( uint32_t ) );
        if( e == hipSuccess )
            e = hipHostMalloc( (void **)&st.host, sizeof( uint32_t ), hipHostMallocDefault );
        if( e == hipSuccess )
            e = hipEventCreateWithFlags( &st.ev, hipEventDisableTiming );
        if( cur != d )
            (void)hipSetDevice( cur );
        if( e != hipSuccess )
        {
            // (a partial allocation is released; the slot stays unset and is retried)
            if( st.dev )
                (void)hipFree( st.dev );
            if( st.host )
                (void)hipHostFree( st.host );
            st.dev = nullptr;
            st.host = nullptr;
            st.ev = nullptr;
            return e;
        }
        *st.host = 0;
        st.pending = false;
        st.device = d;
    }
    *out = &st;
    return hipSuccess;
}

// a reported timeout clears the sticky word (host and device)
hipError_t la_status_clear( LaStatus &st, hipStream_t stream )
{
    *(volatile uint32_t *)st.host = 0;
    return hipMemsetAsync( st.dev, 0, sizeof( uint32_t ), stream );
}

// before a launch: the word for the kernel, or hipErrorLaunchTimeOut when an earlier launch
// of this thread on this device is known to have timed out
hipError_t la_status_begin( hipStream_t stream, uint32_t **word )
{
    LaStatus *st = nullptr;
    hipError_t e = la_status_get( stream, &st );
    if( e != hipSuccess )
        return e;
    // no event query under capture (it would invalidate the capture): the report waits
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if( (e = hipStreamIsCapturing( stream, &cs )) != hipSuccess )
        return e;
    if( cs == hipStreamCaptureStatusNone && st->pending && hipEventQuery( st->ev ) == hipSuccess )
    {
        st->pending = false;
        if( *(volatile uint32_t *)st->host )
        {
            (void)la_status_clear( *st, stream );
            return hipErrorLaunchTimeOut;
        }
    }
    *word = st->dev;
    return hipSuccess;
}

// after the kernel: queue the word's copy behind it (not under capture)
hipError_t la_status_end( hipStream_t stream )
{
    LaStatus *stp = nullptr;
    hipError_t e = la_status_get( stream, &stp );
    if( e != hipSuccess )
        return e;
    LaStatus &st = *stp;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    e = hipStreamIsCapturing( stream, &cs );
    if( e != hipSuccess || cs != hipStreamCaptureStatusNone )
        return e;
    e = hipMemcpyAsync( st.host, st.dev, sizeof( uint32_t ), hipMemcpyDeviceToHost, stream );
    if( e == hipSuccess )
        e = hipEventRecord( st.ev, stream );
    st.pending = e == hipSuccess;
    return e;
}
} // namespace

// x264hip_lowres_status: wait for `stream`, then hipErrorLaunchTimeOut if a lookahead launch of
// this thread on the stream's device timed out since the last report (and clear it)
hipError_t lowres_status( hipStream_t stream )
{
    LaStatus *st = nullptr;
    hipError_t e = la_status_get( stream, &st );
    if( e != hipSuccess )
        return e;
    e = hipMemcpyAsync( st->host, st->dev, sizeof( uint32_t ), hipMemcpyDeviceToHost, stream );
    if( e == hipSuccess )
        e = hipStreamSynchronize( stream );
    if( e != hipSuccess )
        return e;
    st->pending = false;
    if( !*(volatile uint32_t *)st->host )
        return hipSuccess;
    if( (e = la_status_clear( *st, stream )) == hipSuccess )
        e = hipStreamSynchronize( stream );
    return e == hipSuccess ? hipErrorLaunchTimeOut : e;
}

namespace {
// bands per frame over the lookahead slices (lr_band)
int la_nbands( int mbh, int nslices, int brows )
{
    int n = 0;
    for( int i = 0; i < nslices; i++ )
        n += ((mbh * (i + 1) + nslices / 2) / nslices - (mbh * i + nslices / 2) / nslices + brows - 1) / brows;
    return n;
}


int la_poll_max()
{
    const int v = variant( V_LA_POLL );
    return v >= 0 ? v : 1 << 22;
}

// the helper wave of lr_helper: on when every band's workgroup, helper included, is resident at
// once (it rides on wave slots the launch leaves idle: the 15-pair launches; a 240-pair batch
// would double its waves and queue them), X264HIP_LA_HELPER=0 / 1 forces it off / on
// every one of nwg two-wave workgroups of `kernel` resident at once
bool la_fits( const void *kernel, int64_t nwg, size_t lds, hipStream_t stream )
{
    int dev = 0, cus = 0, per_cu = 0;
    if( stream_device( stream, &dev ) != hipSuccess ||
        hipDeviceGetAttribute( &cus, hipDeviceAttributeMultiprocessorCount, dev ) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor( &per_cu, kernel, 128, lds ) != hipSuccess )
        return false;
    return nwg <= (int64_t)cus * per_cu;
}
int la_help( const void *kernel, int64_t nwg, size_t lds, hipStream_t stream )
{
    const int v = variant( V_LA_HELPER );
    if( v >= 0 )
        return v == 1;
    return la_fits( kernel, nwg, lds, stream );
}

// The grid of n units (pairs / triplets) of nbands bands, and lr_unit's xpairs: every band of a
// unit on one XCD when that grid is resident at once (the 15-pair launches: P 1.229 -> 1.203,
// B 1.783 -> 1.752 ms, 4 slices 0.823 -> 0.790 in an interleaved A/B, profiles/r05x_la_xcd_ab.log;
// a 240-pair batch, which queues its workgroups, ran slower so: 2.25 -> 2.38 ms), else in
// block order.  X264HIP_LA_XCD=0 / 1 forces it off / on.
int64_t la_grid( const void *kernel, int n, int nbands, size_t lds, hipStream_t stream, int &xpairs )
{
    const int64_t nx = (int64_t)8 * nbands * ((n + 7) / 8);
    const int v = variant( V_LA_XCD );
    xpairs = (v == 1 || (v < 0 && la_fits( kernel, nx, lds, stream ))) ? n : 0;
    return xpairs ? nx : (int64_t)n * nbands;
}
} // namespace

// The kernels take a reference's four lowres planes (F, H, V, C) as the F plane and one
// spacing: x264 allocates them so, in one buffer_lowres (frame.c:209, 281), and one spacing
// instead of three more 64-bit pointers keeps the kernels' scalar registers (and spills) down.
// Planes that are not equally spaced are gathered first, stream-ordered, into a scratch
// buffer: per plane and frame the rows -16 .. 8 * mbh + 16 from column -32 (every row the
// search and the helper wave can reach, lr_helper), spaced evenly.
template <typename pixel>
__global__ __launch_bounds__( 256 ) void lowres_gather_kernel( const pixel *p0, const pixel *p1, const pixel *p2,
                                                               const pixel *p3, intptr_t fs, intptr_t lo,
                                                               intptr_t len, pixel *dst )
{
    const int k = blockIdx.z;
    const pixel *src = (k == 0 ? p0 : k == 1 ? p1 : k == 2 ? p2 : p3) + (intptr_t)blockIdx.y * fs - lo;
    pixel *d = dst + ((intptr_t)k * gridDim.y + blockIdx.y) * len;
    for( intptr_t i = (intptr_t)blockIdx.x * 256 + threadIdx.x; i < len; i += (intptr_t)gridDim.x * 256 )
        d[i] = src[i];
}

template <typename pixel> struct LaPlanes
{
    const pixel *base = nullptr;                 // the F plane at (0, 0) of frame 0
    intptr_t pd = 0, fs = 0;                     // plane spacing, frame stride
    pixel *scratch = nullptr;

    hipError_t init( const pixel *const p[4], intptr_t frame_stride, intptr_t stride, int nframes, int mbh,
                     hipStream_t st )
    {
        const intptr_t d = p[1] - p[0];
        fs = frame_stride;
        if( d != 0 && p[2] - p[1] == d && p[3] - p[2] == d )
        {
            base = p[0];
            pd = d;
            return hipSuccess;
        }
        const int nf = frame_stride ? nframes : 1;
        if( nf > 65535 )                          // (the gather grid's y dimension)
            return hipErrorInvalidValue;
        const intptr_t lo = 16 * stride + 32, len = (8 * (intptr_t)mbh + 33) * stride;
        hipError_t e = scratch_alloc( (void **)&scratch, (size_t)(4 * nf) * len * sizeof( pixel ), st );
        if( e != hipSuccess )
            return e;
        const int nx = (int)std::min<intptr_t>( (len + 255) / 256, 64 );
        hipLaunchKernelGGL( lowres_gather_kernel<pixel>, dim3( nx, nf, 4 ), dim3( 256 ), 0, st, p[0], p[1], p[2],
                            p[3], frame_stride, lo, len, scratch );
        base = scratch + lo;
        pd = (intptr_t)nf * len;
        fs = frame_stride ? len : 0;
        return hipGetLastError();
    }
    hipError_t done( hipStream_t st ) { return scratch ? hipFreeAsync( scratch, st ) : hipSuccess; }
};

template <int BD>
hipError_t launch_lowres_bidir( const typename PT<BD>::pixel *fenc, intptr_t ffs,
                                const typename PT<BD>::pixel *const ra[4], intptr_t afs,
                                const typename PT<BD>::pixel *const rb[4], intptr_t bfs, intptr_t stride, int mbw,
                                int mbh, int n, int me_method, int subme, int satd, int me_range, int mv_range,
                                int lambda, const uint16_t *cost_mv, int search, int16_t *mvs0, int32_t *costs0,
                                int16_t *mvs1, int32_t *costs1, const int16_t *p1mvs, int dsf, int weight,
                                const uint16_t *invq, uint16_t *lowres_costs, int32_t *row_satd, int32_t *est,
                                int nslices, hipStream_t stream )
{
    if( n <= 0 || mbw <= 0 || mbh <= 0 )
        return hipSuccess;
    // a searched list's mvs start as the sentinel the bands wait on; the frame sums
    // are accumulated by every band
    const size_t mvbytes = (size_t)n * mbw * mbh * 4;
    hipError_t e = hipSuccess;
    if( search & 1 )
        e = hipMemsetAsync( mvs0, 0x80, mvbytes, stream );
    if( e == hipSuccess && (search & 2) )
        e = hipMemsetAsync( mvs1, 0x80, mvbytes, stream );
    if( e == hipSuccess && est )
        e = hipMemsetAsync( est, 0, (size_t)n * 2 * sizeof( int32_t ), stream );
    if( e != hipSuccess )
        return e;
    // block rows per single-wave workgroup: a step costs the slowest of a wave's row
    // searches (the lanes run in lockstep), so fewer rows per wave means less divergence; 4
    // measured best (15 1080p pairs, round-2 band sweep, profiles/r02e_la_band.json: P 2.46 / 2.32 / 2.19 / 2.26 ms,
    // B 5.42 / 5.11 / 4.65 / 4.80 ms for 16 / 8 / 4 / 2 rows)
    constexpr int brows = 4;
    constexpr int brows4 = brows;                // a wave holds four roles of <= 4 rows
    const int nbands = la_nbands( mbh, nslices, brows4 );
    if( nslices < 1 || (int64_t)(n + 8) * nbands > 0x7fffffff )
        return hipErrorInvalidValue;
    const size_t lds = (size_t)(2 * (4 * mv_range + 64) + 1) * sizeof( uint16_t );
    if( mv_range < 1 || lds > 48 * 1024 )
        return hipErrorInvalidValue;
    LaPlanes<typename PT<BD>::pixel> pa, pb;
    if( (e = pa.init( ra, afs, stride, n, mbh, stream )) != hipSuccess ||
        (e = pb.init( rb, bfs, stride, n, mbh, stream )) != hipSuccess )
    {
        (void)pa.done( stream );
        (void)pb.done( stream );
        return e;
    }
    uint32_t *status = nullptr;
    if( (e = la_status_begin( stream, &status )) != hipSuccess )
    {
        (void)pa.done( stream );
        (void)pb.done( stream );
        return e;
    }
    int xp = 0;
    const int64_t nwg = la_grid( (const void *)lowres_bidir_kernel<BD>, n, nbands, lds, stream, xp );
    const int help = la_help( (const void *)lowres_bidir_kernel<BD>, nwg, lds, stream );
    hipLaunchKernelGGL( lowres_bidir_kernel<BD>, dim3( (unsigned)nwg ), dim3( help ? 128 : 64 ), lds, stream, fenc, ffs,
                        pa.base, pa.pd, pa.fs, pb.base, pb.pd, pb.fs, stride, mbw, mbh, me_method,
                        subme, satd, me_range, mv_range, lambda, cost_mv, search, mvs0, costs0, mvs1, costs1, p1mvs,
                        dsf, weight, invq, lowres_costs, row_satd, est, nbands, brows4, la_poll_max(), status,
                        nslices, help, xp );
    e = hipGetLastError();
    const hipError_t ea = pa.done( stream ), eb = pb.done( stream );
    if( e != hipSuccess || (e = ea) != hipSuccess || (e = eb) != hipSuccess )
        return e;
    return la_status_end( stream );
}

template <int BD>
hipError_t launch_lowres_inter( const typename PT<BD>::pixel *fenc, intptr_t ffs,
                                const typename PT<BD>::pixel *const ref[4], intptr_t stride, intptr_t rfs, int mbw,
                                int mbh, int npairs, int me_method, int subme, int satd, int me_range, int mv_range,
                                int lambda, const uint16_t *cost_mv, const uint16_t *intra_cost,
                                const uint16_t *invq, int16_t *mvs, int32_t *mv_costs, uint16_t *lowres_costs,
                                int32_t *row_satd, int32_t *est, const typename PT<BD>::pixel *ref_w, int wscale,
                                int wdenom, int woffset, int nslices, hipStream_t stream )
{
    if( npairs <= 0 || mbw <= 0 || mbh <= 0 )
        return hipSuccess;
    // mvs start as the sentinel the bands wait on; the frame sums are accumulated by every band
    hipError_t e = hipMemsetAsync( mvs, 0x80, (size_t)npairs * mbw * mbh * 4, stream );
    if( e == hipSuccess && est )
        e = hipMemsetAsync( est, 0, (size_t)npairs * 3 * sizeof( int32_t ), stream );
    if( e != hipSuccess )
        return e;
    // block rows per single-wave workgroup: a step costs the slowest of a wave's row
    // searches (the lanes run in lockstep), so fewer rows per wave means less divergence; 4
    // measured best (15 1080p pairs, round-2 band sweep, profiles/r02e_la_band.json: P 2.46 / 2.32 / 2.19 / 2.26 ms,
    // B 5.42 / 5.11 / 4.65 / 4.80 ms for 16 / 8 / 4 / 2 rows)
    constexpr int brows = 4;
    constexpr int brows4 = brows;                // four groups of <= 4 rows per wave
    const int nbands = la_nbands( mbh, nslices, brows4 );
    if( nslices < 1 || (int64_t)(npairs + 8) * nbands > 0x7fffffff )
        return hipErrorInvalidValue;
    const size_t lds = (size_t)(2 * (4 * mv_range + 64) + 1) * sizeof( uint16_t );
    if( mv_range < 1 || lds > 48 * 1024 )
        return hipErrorInvalidValue;
    LaPlanes<typename PT<BD>::pixel> pr;
    if( (e = pr.init( ref, rfs, stride, npairs, mbh, stream )) != hipSuccess )
    {
        (void)pr.done( stream );
        return e;
    }
    uint32_t *status = nullptr;
    if( (e = la_status_begin( stream, &status )) != hipSuccess )
    {
        (void)pr.done( stream );
        return e;
    }
    auto go = [&]( auto kernel ) {
        int xp = 0;
        const int64_t nwg = la_grid( (const void *)kernel, npairs, nbands, lds, stream, xp );
        const int help = la_help( (const void *)kernel, nwg, lds, stream );
        hipLaunchKernelGGL( kernel, dim3( (unsigned)nwg ), dim3( help ? 128 : 64 ), lds, stream, fenc, ffs, pr.base,
                            pr.pd, stride, pr.fs, mbw, mbh, me_method, subme, satd, me_range, mv_range, lambda,
                            cost_mv, intra_cost, invq, mvs, mv_costs, lowres_costs, row_satd, est, nbands, brows4,
                            la_poll_max(), status, ref_w, rfs, wscale, wdenom, woffset, nslices, help, xp );
    };
    // the latency form when its grid (bands placed by XCD) is resident at once
    const int64_t nx = (int64_t)8 * nbands * ((npairs + 7) / 8);
    if( ref_w )
    {
        if( la_fits( (const void *)lowres_inter_kernel<BD, true, true>, nx, lds, stream ) )
            go( lowres_inter_kernel<BD, true, true> );
        else
            go( lowres_inter_kernel<BD, true, false> );
    }
    else
    {
        if( la_fits( (const void *)lowres_inter_kernel<BD, false, true>, nx, lds, stream ) )
            go( lowres_inter_kernel<BD, false, true> );
        else
            go( lowres_inter_kernel<BD, false, false> );
    }
    e = hipGetLastError();
    const hipError_t ef = pr.done( stream );
    if( e != hipSuccess || (e = ef) != hipSuccess )
        return e;
    return la_status_end( stream );
}

#define INST( BD )                                                                                              \
    template hipError_t launch_lowres_inter<BD>( const PT<BD>::pixel *, intptr_t, const PT<BD>::pixel *const[4], \
                                                 intptr_t, intptr_t, int, int, int, int, int, int, int, int, int, \
                                                 const uint16_t *, const uint16_t *, const uint16_t *, int16_t *, \
                                                 int32_t *, uint16_t *, int32_t *, int32_t *,                     \
                                                 const PT<BD>::pixel *, int, int, int, int, hipStream_t );
INST( 8 )
INST( 10 )
#undef INST
#define INST( BD )                                                                                              \
    template hipError_t launch_lowres_bidir<BD>( const PT<BD>::pixel *, intptr_t, const PT<BD>::pixel *const[4], \
                                                 intptr_t, const PT<BD>::pixel *const[4], intptr_t, intptr_t, int,  \
                                                 int, int, int, int, int, int, int, int, const uint16_t *, int,     \
                                                 int16_t *, int32_t *, int16_t *, int32_t *, const int16_t *, int,  \
                                                 int, const uint16_t *, uint16_t *, int32_t *, int32_t *, int,      \
                                                 hipStream_t );
INST( 8 )
INST( 10 )
#undef INST

} // namespace x264hip
