// Exhaustive integer-pel 16x16 SAD search tables (the candidate set of the
// reference's ESA/plain exhaustive search, encoder/me.c:618-631, before the
// mv-cost term COST_MV adds, me.c:63-70), the fused ESA decision and the decision
// over a table.
//
// Table geometry (hipcommon.h full_pitch / cen_cols / cen_pitch, include/x264hip.h):
//  * a full-search table (me_search_full) is the (2R+1)^2 square around mv 0, rows at
//    pitch align4(2R+1);
//  * a centred table (me_search_centred, and the window the fused ESA decision keys) is
//    me.c's ESA window around a predictor (bmx, bmy): 2R+1 rows, and the columns the
//    window can reach -- [bmx - R, bmx + R + 2] (the width rounding (max_x - min_x + 3) & ~3
//    of me.c:626 ends up to two columns past max_x) plus the origin's alignment down to a
//    dword (3 pixels at 8 bit, 1 at 10 bit): 2R+6 columns at 8 bit, 2R+4 at 10 bit.  So a
//    template of radius me_range holds every candidate me.c evaluates, and nothing else
//    but the slack columns.
//
// Layout of the work (generic kernel, the unaligned-plane fallback): one lane owns one
// candidate COLUMN (mx) of one macroblock's window and walks the 2R+16 ref rows top to
// bottom, fetching each 16-pixel ref row ONCE and folding it into the (up to 16)
// candidates my whose 16-row footprint covers that row:
//   acc[my] += sad(fenc row (y - my), ref row y)      (v_sad_u8 / v_sad_u16)
// fenc (16 rows) stays in VGPRs for the whole lane lifetime.  Candidate my finishes at
// row my+15 and is stored then.  The grouped kernels below (four columns per lane with
// v_qsad_pk_u16_u8 at 8 bit, column pairs with v_sad_u16 at 10 bit) are the defaults.
#include "hipcommon.h"
#include <mutex>
#include <string.h>
#include <stdlib.h>
#include <atomic>
#include <utility>

namespace x264hip {

// one window row Y (compile-time): fold ref row Y into every candidate whose
// footprint covers it; candidate c uses fenc row Y - c.
template <int BD, int R, int P, int Y>
__device__ __forceinline__ void me_row( const typename PT<BD>::pixel *rb, intptr_t rs,
                                        const uint32_t (&F)[16][16 / PT<BD>::PPD], uint32_t (&acc)[16],
                                        typename PT<BD>::sadt *out )
{
    constexpr int NDW = 16 / PT<BD>::PPD;
    constexpr int C0 = Y - 15 > 0 ? Y - 15 : 0;
    constexpr int C1 = Y < 2 * R ? Y : 2 * R;
    uint32_t rr[NDW];
    load_packed<NDW>( rb + (intptr_t)Y * rs, rr );
#pragma unroll
    for( int c = C0; c <= C1; c++ )
    {
        const int r = Y - c;
        uint32_t a = r == 0 ? 0u : acc[c & 15];
#pragma unroll
        for( int k = 0; k < NDW; k++ )
            a = sadp<BD>( F[r][k], rr[k], a );
        if( r == 15 )
            out[c * P] = (typename PT<BD>::sadt)a;
        else
            acc[c & 15] = a;
    }
}

template <int BD, int R, int P, int... Ys>
__device__ __forceinline__ void me_rows( const typename PT<BD>::pixel *rb, intptr_t rs,
                                         const uint32_t (&F)[16][16 / PT<BD>::PPD], uint32_t (&acc)[16],
                                         typename PT<BD>::sadt *out, std::integer_sequence<int, Ys...> )
{
    ( me_row<BD, R, P, Ys>( rb, rs, F, acc, out ), ... );
}

// Window origin of one MB (me_search_centred; the plain search is the special case
// centre = (0, 0)): (cx, cy) - R, clamped so that every pixel a kernel fetches lies in the
// 32-pixel padded plane (x264's PADH = PADV = 32, common/frame.h:32-33) -- P columns wide,
// 2R+1 rows -- then aligned down to 4 (8 bit) / 2 (10 bit) pixels so the grouped kernels
// keep dword-aligned rows.  For centre (0, 0) and R <= 24 neither step changes anything.
// Returned relative to the MB.
template <int BD, int R, int P>
__device__ __forceinline__ void me_window( const int16_t *__restrict__ centre, int64_t mb, int mbx, int mby, int mbw,
                                           int mbh, int &ox, int &oy )
{
    constexpr int AL = BD == 8 ? 4 : 2;
    int ax = 16 * mbx - R, ay = 16 * mby - R;
    if( centre )
    {
        ax += centre[2 * mb];
        ay += centre[2 * mb + 1];
    }
    ax = min( max( ax, -32 ), 16 * mbw + 12 - P );
    ay = min( max( ay, -32 ), 16 * mbh + 16 - 2 * R );
    ax &= ~(AL - 1);
    ox = ax - 16 * mbx;
    oy = ay - 16 * mby;
}

// generic kernel: one lane per table column (NCOL columns, pitch align4(NCOL)); serves
// planes whose rows or strides are not dword aligned
template <int BD, int R, int NCOL>
__global__ __launch_bounds__( 256 ) void me_full_sad16_kernel( const typename PT<BD>::pixel *__restrict__ fenc,
                                                               intptr_t fs, intptr_t ffs,
                                                               const typename PT<BD>::pixel *__restrict__ ref,
                                                               intptr_t rs, intptr_t rfs, int mbw, int mbh,
                                                               int nframes, typename PT<BD>::sadt *__restrict__ table,
                                                               const int16_t *__restrict__ centre,
                                                               int16_t *__restrict__ origin )
{
    constexpr int W = 2 * R + 1, P = al4( NCOL );
    constexpr int NDW = 16 / PT<BD>::PPD;   // dwords per 16-pixel row
    const int64_t slot = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)nframes * mbh * mbw * NCOL;
    if( slot >= total )
        return;
    const int col = (int)(slot % NCOL);
    const int64_t mb = slot / NCOL;
    const int mbx = (int)(mb % mbw);
    const int64_t t = mb / mbw;
    const int mby = (int)(t % mbh);
    const int64_t f = t / mbh;

    // fenc rows stay resident in registers
    uint32_t F[16][NDW];
    const typename PT<BD>::pixel *fe = fenc + f * ffs + (intptr_t)16 * mby * fs + 16 * mbx;
#pragma unroll
    for( int r = 0; r < 16; r++ )
        load_packed<NDW>( fe + r * fs, F[r] );

    int ox, oy;
    me_window<BD, R, P>( centre, mb, mbx, mby, mbw, mbh, ox, oy );
    if( origin && col == 0 )
    {
        origin[2 * mb] = (int16_t)ox;
        origin[2 * mb + 1] = (int16_t)oy;
    }
    const typename PT<BD>::pixel *rb = ref + f * rfs + (intptr_t)(16 * mby + oy) * rs + 16 * mbx + ox + col;
    typename PT<BD>::sadt *out = table + mb * (W * P) + col;

    uint32_t acc[16];
    me_rows<BD, R, P>( rb, rs, F, acc, out, std::make_integer_sequence<int, 2 * R + 16>{} );
}

typedef uint64_t u64x2a4 __attribute__( ( ext_vector_type( 2 ), aligned( 4 ) ) );
typedef uint32_t u32x4a4 __attribute__( ( ext_vector_type( 4 ), aligned( 4 ) ) );
typedef uint32_t u32x2a4 __attribute__( ( ext_vector_type( 2 ), aligned( 4 ) ) );

// rows of ref-load lead in the grouped kernels: the loads of ref rows Y+1, Y+2 are issued
// before row Y's SADs (16 1080p pairs, R 16: 8 bit 0.312 -> 0.300 ms from no lead to two
// rows, 10 bit 0.653 -> 0.617 ms; a third row gained nothing, profiles of round 1-2)
constexpr int ME_LEAD = 2;

// ---------------------------------------------------------------------------
// 8 bit: one lane owns four adjacent candidate columns 4g..4g+3 and all 16 fenc rows;
// per ref row it issues two overlapping 16-byte loads (the four 8-byte windows arrive as
// aligned register pairs, no realignment) and folds the row into the <= 16 candidate rows
// whose footprint covers it, 16 byte absdiffs per v_qsad_pk_u16_u8 (a column's packed u16
// sum cannot carry: 16*16*255 < 2^16).  `sink( c, lo, hi )` receives candidate row c's four
// finished SADs as packed u16 pairs (columns 4g, 4g+1 in lo, 4g+2, 4g+3 in hi).
template <int R, int L, int Y, class Sink>
__device__ __forceinline__ void me_row7( const uint32_t *__restrict__ rbase, int rs_dw, const uint32_t (&F)[16][4],
                                         uint64_t (&acc)[16], Sink &sink, u64x2a4 (&e)[L], u64x2a4 (&o)[L] )
{
    constexpr int C0 = Y - 15 > 0 ? Y - 15 : 0;
    constexpr int C1 = Y < 2 * R ? Y : 2 * R;
    const uint64_t win[4] = { e[Y % L][0], o[Y % L][0], e[Y % L][1], o[Y % L][1] };
    if constexpr( Y + L < 2 * R + 16 )
    {
        const uint32_t *row = rbase + (Y + L) * rs_dw;
        e[Y % L] = *(const u64x2a4 *)row;
        o[Y % L] = *(const u64x2a4 *)(row + 1);
    }
#pragma unroll
    for( int c = C0; c <= C1; c++ )
    {
        const int r = Y - c;
        uint64_t a = r == 0 ? 0ull : acc[c & 15];
#pragma unroll
        for( int k = 0; k < 4; k++ )
            a = __builtin_amdgcn_qsad_pk_u16_u8( win[k], F[r][k], a );
        if( r == 15 )
            sink( c, (uint32_t)a, (uint32_t)(a >> 32) );
        else
            acc[c & 15] = a;
    }
    // keep the scheduler from hoisting later rows' loads up here
    __builtin_amdgcn_sched_barrier( 0 );
}

template <int R, int L, class Sink, int... Ys>
__device__ __forceinline__ void me_rows7( const uint32_t *__restrict__ rbase, int rs_dw, const uint32_t (&F)[16][4],
                                          uint64_t (&acc)[16], Sink &sink, std::integer_sequence<int, Ys...> )
{
    u64x2a4 e[L], o[L];
#pragma unroll
    for( int k = 0; k < L; k++ )
    {
        e[k] = *(const u64x2a4 *)(rbase + k * rs_dw);
        o[k] = *(const u64x2a4 *)(rbase + k * rs_dw + 1);
    }
    ( me_row7<R, L, Ys>( rbase, rs_dw, F, acc, sink, e, o ), ... );
}

// one lane per column group of G (full: align4(2R+1) / 4, centred: cen_pitch / 4)
template <int R, int G>
__global__ __launch_bounds__( 256 ) void me_full_sad16_v7_kernel( const uint8_t *__restrict__ fenc, intptr_t fs,
                                                                  intptr_t ffs, const uint8_t *__restrict__ ref,
                                                                  intptr_t rs, intptr_t rfs, int mbw, int mbh,
                                                                  int nframes, uint16_t *__restrict__ table,
                                                                  const int16_t *__restrict__ centre,
                                                                  int16_t *__restrict__ origin, int xcd )
{
    constexpr int P = 4 * G;                    // table row pitch
    // 32-bit index decomposition (the launcher keeps the lane count below 2^32): the
    // int64 divisions by mbw / mbh were ~150 VALU instructions of the prologue
    const uint32_t blk = xcd ? xcd_block( blockIdx.x, gridDim.x ) : blockIdx.x;
    const uint32_t slot = blk * blockDim.x + threadIdx.x;
    if( slot >= (uint32_t)nframes * (uint32_t)mbh * (uint32_t)mbw * (uint32_t)G )
        return;
    const uint32_t mb32 = slot / G, t32 = mb32 / (uint32_t)mbw, f32 = t32 / (uint32_t)mbh;
    const int grp = (int)(slot - mb32 * G);
    const int mbx = (int)(mb32 - t32 * (uint32_t)mbw);
    const int mby = (int)(t32 - f32 * (uint32_t)mbh);
    const int64_t mb = mb32, f = f32;

    uint32_t F[16][4];
    const uint32_t *fe = (const uint32_t *)(fenc + f * ffs + (intptr_t)(16 * mby) * fs + 16 * mbx);
    const int fs_dw = (int)(fs / 4);
#pragma unroll
    for( int r = 0; r < 16; r++ )
#pragma unroll
        for( int k = 0; k < 4; k++ )
            F[r][k] = fe[r * fs_dw + k];
    int ox, oy;
    me_window<8, R, P>( centre, mb, mbx, mby, mbw, mbh, ox, oy );
    if( origin && grp == 0 )
    {
        origin[2 * mb] = (int16_t)ox;
        origin[2 * mb + 1] = (int16_t)oy;
    }
    const uint32_t *rbase =
        (const uint32_t *)(ref + f * rfs + (intptr_t)(16 * mby + oy) * rs + 16 * mbx + ox + 4 * grp);
    uint64_t *out = (uint64_t *)(table + mb * ((2 * R + 1) * P) + 4 * grp);
    auto store = [out]( int c, uint32_t lo, uint32_t hi ) { out[c * (P / 4)] = ((uint64_t)hi << 32) | lo; };
    uint64_t acc[16];
    me_rows7<R, ME_LEAD>( rbase, (int)(rs / 4), F, acc, store, std::make_integer_sequence<int, 2 * R + 16>{} );
}

// ---------------------------------------------------------------------------
// X264HIP_ME_XCD (default 1): XCD-contiguous workgroup ranges (xcd_block).  Same time for
// the VALU-bound search, 2.3x fewer HBM fetches: neighbouring MBs' overlapping windows hit
// one XCD's L2 (FETCH_SIZE 160 -> 69 MB per 16 1080p pairs, profiles/r03c_*)
static int me_xcd() { return variant( V_ME_XCD ) != 0; }

// 8x8 quadrant tables (8 bit): the four-column lane with separate left (fenc dwords 0-1)
// and right (dwords 2-3) accumulators, restarted at fenc row 8: a candidate row's top
// quadrants leave at fenc row 7, its bottom ones at row 15.  The same 256 absdiffs per
// candidate as the 16x16 table -- whose SAD is the sum of the four -- and 16x8 / 8x16
// SADs are pair sums.
template <int R, int L, int Y, class Sink>
__device__ __forceinline__ void me_row8q( const uint32_t *__restrict__ rbase, int rs_dw, const uint32_t (&F)[16][4],
                                          uint64_t (&al)[16], uint64_t (&ar)[16], Sink &sink, u64x2a4 (&e)[L],
                                          u64x2a4 (&o)[L] )
{
    constexpr int C0 = Y - 15 > 0 ? Y - 15 : 0;
    constexpr int C1 = Y < 2 * R ? Y : 2 * R;
    const uint64_t win[4] = { e[Y % L][0], o[Y % L][0], e[Y % L][1], o[Y % L][1] };
    if constexpr( Y + L < 2 * R + 16 )
    {
        const uint32_t *row = rbase + (Y + L) * rs_dw;
        e[Y % L] = *(const u64x2a4 *)row;
        o[Y % L] = *(const u64x2a4 *)(row + 1);
    }
#pragma unroll
    for( int c = C0; c <= C1; c++ )
    {
        const int r = Y - c;
        uint64_t a = (r & 7) == 0 ? 0ull : al[c & 15], b = (r & 7) == 0 ? 0ull : ar[c & 15];
        a = __builtin_amdgcn_qsad_pk_u16_u8( win[0], F[r][0], a );
        a = __builtin_amdgcn_qsad_pk_u16_u8( win[1], F[r][1], a );
        b = __builtin_amdgcn_qsad_pk_u16_u8( win[2], F[r][2], b );
        b = __builtin_amdgcn_qsad_pk_u16_u8( win[3], F[r][3], b );
        if( (r & 7) == 7 )
            sink( c, r >> 3, a, b );
        else
        {
            al[c & 15] = a;
            ar[c & 15] = b;
        }
    }
    __builtin_amdgcn_sched_barrier( 0 );
}

template <int R, int L, class Sink, int... Ys>
__device__ __forceinline__ void me_rows8q( const uint32_t *__restrict__ rbase, int rs_dw, const uint32_t (&F)[16][4],
                                           uint64_t (&al)[16], uint64_t (&ar)[16], Sink &sink,
                                           std::integer_sequence<int, Ys...> )
{
    u64x2a4 e[L], o[L];
#pragma unroll
    for( int k = 0; k < L; k++ )
    {
        e[k] = *(const u64x2a4 *)(rbase + k * rs_dw);
        o[k] = *(const u64x2a4 *)(rbase + k * rs_dw + 1);
    }
    ( me_row8q<R, L, Ys>( rbase, rs_dw, F, al, ar, sink, e, o ), ... );
}

// table8[mb][q][2R+1][P]: q = 0 top-left, 1 top-right, 2 bottom-left, 3 bottom-right
template <int R>
__global__ __launch_bounds__( 256 ) void me_full_sad8q_kernel( const uint8_t *__restrict__ fenc, intptr_t fs,
                                                               intptr_t ffs, const uint8_t *__restrict__ ref,
                                                               intptr_t rs, intptr_t rfs, int mbw, int mbh,
                                                               int nframes, uint16_t *__restrict__ table8, int xcd )
{
    constexpr int P = full_pitch( R ), G = P / 4;
    const uint32_t blk = xcd ? xcd_block( blockIdx.x, gridDim.x ) : blockIdx.x;
    const uint32_t slot = blk * blockDim.x + threadIdx.x;
    if( slot >= (uint32_t)nframes * (uint32_t)mbh * (uint32_t)mbw * (uint32_t)G )
        return;
    const uint32_t mb32 = slot / G, t32 = mb32 / (uint32_t)mbw, f32 = t32 / (uint32_t)mbh;
    const int grp = (int)(slot - mb32 * G);
    const int mbx = (int)(mb32 - t32 * (uint32_t)mbw);
    const int mby = (int)(t32 - f32 * (uint32_t)mbh);
    const int64_t mb = mb32, f = f32;
    uint32_t F[16][4];
    const uint32_t *fe = (const uint32_t *)(fenc + f * ffs + (intptr_t)(16 * mby) * fs + 16 * mbx);
    const int fs_dw = (int)(fs / 4);
#pragma unroll
    for( int r = 0; r < 16; r++ )
#pragma unroll
        for( int k = 0; k < 4; k++ )
            F[r][k] = fe[r * fs_dw + k];
    const uint32_t *rbase = (const uint32_t *)(ref + f * rfs + (intptr_t)(16 * mby - R) * rs + 16 * mbx - R + 4 * grp);
    uint64_t *out = (uint64_t *)(table8 + mb * (4 * (2 * R + 1) * P) + 4 * grp);
    auto store = [out]( int c, int half, uint64_t a, uint64_t b ) {
        out[((2 * half) * (2 * R + 1) + c) * (P / 4)] = a;
        out[((2 * half + 1) * (2 * R + 1) + c) * (P / 4)] = b;
    };
    uint64_t al[16], ar[16];
    me_rows8q<R, ME_LEAD>( rbase, (int)(rs / 4), F, al, ar, store, std::make_integer_sequence<int, 2 * R + 16>{} );
}

// ---------------------------------------------------------------------------
// 10 bit: a lane owns two adjacent candidate columns (2g, 2g+1; the first is dword aligned
// for even R) and half of the fenc rows (lane pair h = 0/1: rows 8h..8h+7); per ref row it
// loads 9 dwords once (L rows ahead), forms the odd column's dwords with one
// v_alignbyte_b32 each, and folds the row into <= 8 candidates x 2 columns with v_sad_u16.
// `sink( c, a0, a1 )` receives candidate row c's two finished SADs (columns 2g, 2g+1),
// identical in both lanes of the pair after the DPP add.
template <int R, int L, int Y, class Sink>
__device__ __forceinline__ void me_row5p( const uint32_t *__restrict__ rbase, int rs_dw, const uint32_t (&F)[8][8],
                                          uint32_t (&acc)[8][2], Sink &sink, uint32_t (&ring)[L][9] )
{
    constexpr int C0 = Y - 7 > 0 ? Y - 7 : 0;
    constexpr int C1 = Y < 2 * R ? Y : 2 * R;
    uint32_t w[9], o[8];
#pragma unroll
    for( int k = 0; k < 9; k++ )
        w[k] = ring[Y % L][k];
    if constexpr( Y + L < 2 * R + 8 )
    {
        const uint32_t *row = rbase + (Y + L) * rs_dw;
#pragma unroll
        for( int k = 0; k < 9; k++ )
            ring[Y % L][k] = row[k];
    }
#pragma unroll
    for( int k = 0; k < 8; k++ )
        o[k] = __builtin_amdgcn_alignbyte( w[k + 1], w[k], 2 );
#pragma unroll
    for( int c = C0; c <= C1; c++ )
    {
        const int r = Y - c;
        uint32_t a0 = r == 0 ? 0u : acc[c & 7][0], a1 = r == 0 ? 0u : acc[c & 7][1];
#pragma unroll
        for( int k = 0; k < 8; k++ )
        {
            a0 = __builtin_amdgcn_sad_u16( F[r][k], w[k], a0 );
            a1 = __builtin_amdgcn_sad_u16( F[r][k], o[k], a1 );
        }
        if( r == 7 )
        {
            a0 += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)a0, 0xB1, 0xF, 0xF, false );
            a1 += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)a1, 0xB1, 0xF, 0xF, false );
            sink( c, a0, a1 );
        }
        else
        {
            acc[c & 7][0] = a0;
            acc[c & 7][1] = a1;
        }
    }
    __builtin_amdgcn_sched_barrier( 0 );
}

template <int R, int L, class Sink, int... Ys>
__device__ __forceinline__ void me_rows5p( const uint32_t *__restrict__ rbase, int rs_dw, const uint32_t (&F)[8][8],
                                           uint32_t (&acc)[8][2], Sink &sink, std::integer_sequence<int, Ys...> )
{
    uint32_t ring[L][9];
#pragma unroll
    for( int j = 0; j < L; j++ )
#pragma unroll
        for( int k = 0; k < 9; k++ )
            ring[j][k] = rbase[j * rs_dw + k];
    ( me_row5p<R, L, Ys>( rbase, rs_dw, F, acc, sink, ring ), ... );
}

// G column pairs per MB (full: R+1, centred: cen_cols(10, R) / 2), row pitch P
template <int R, int G, int P>
__global__ __launch_bounds__( 256 ) void me_full_sad16_v5_kernel( const uint16_t *__restrict__ fenc, intptr_t fs,
                                                                  intptr_t ffs, const uint16_t *__restrict__ ref,
                                                                  intptr_t rs, intptr_t rfs, int mbw, int mbh,
                                                                  int nframes, uint32_t *__restrict__ table,
                                                                  const int16_t *__restrict__ centre,
                                                                  int16_t *__restrict__ origin, int xcd )
{
    // 32-bit index decomposition as in v7 (the launcher keeps the lane count below 2^32)
    const uint32_t blk = xcd ? xcd_block( blockIdx.x, gridDim.x ) : blockIdx.x;
    const uint32_t slot = blk * blockDim.x + threadIdx.x;
    if( slot >= (uint32_t)nframes * (uint32_t)mbh * (uint32_t)mbw * (uint32_t)(2 * G) )
        return;
    const int h = (int)(slot & 1);
    const uint32_t mb32 = slot / (2 * G), t32 = mb32 / (uint32_t)mbw, f32 = t32 / (uint32_t)mbh;
    const int grp = (int)((slot >> 1) - mb32 * G);
    const int mbx = (int)(mb32 - t32 * (uint32_t)mbw);
    const int mby = (int)(t32 - f32 * (uint32_t)mbh);
    const int64_t mb = mb32, f = f32;

    uint32_t F[8][8];
    const uint32_t *fe = (const uint32_t *)(fenc + f * ffs + (intptr_t)(16 * mby + 8 * h) * fs + 16 * mbx);
    const int fs_dw = (int)(fs / 2);
#pragma unroll
    for( int r = 0; r < 8; r++ )
#pragma unroll
        for( int k = 0; k < 8; k++ )
            F[r][k] = fe[r * fs_dw + k];
    int ox, oy;
    me_window<10, R, P>( centre, mb, mbx, mby, mbw, mbh, ox, oy );
    if( origin && grp == 0 && h == 0 )
    {
        origin[2 * mb] = (int16_t)ox;
        origin[2 * mb + 1] = (int16_t)oy;
    }
    const uint32_t *rbase =
        (const uint32_t *)(ref + f * rfs + (intptr_t)(16 * mby + 8 * h + oy) * rs + 16 * mbx + ox + 2 * grp);
    uint32_t *out = table + mb * ((2 * R + 1) * P) + 2 * grp;
    uint32_t acc[8][2];
    // both lanes of the pair hold the sums and both store them (to the same address): with
    // the store predicated on h == 0 the compiler kept every row's sums live across the
    // branch -- 220 VGPRs and 2 waves per SIMD instead of 118 and 4, the round-4 regression
    // of 0.617 -> 0.71 ms per 16 1080p pairs
    auto store = [out]( int c, uint32_t a0, uint32_t a1 ) { *(uint2 *)(out + c * P) = make_uint2( a0, a1 ); };
    me_rows5p<R, ME_LEAD>( rbase, (int)(rs / 2), F, acc, store, std::make_integer_sequence<int, 2 * R + 8>{} );
}

// 10-bit quadrant tables: the column-pair lane of the 16x16 kernel, whose fenc row half h is
// already a quadrant row (h = 0 top, 1 bottom); the 8 dwords of a fenc row split into the
// left (dwords 0-3) and right (4-7) accumulators, so a lane's candidate row leaves as four
// 8x8 SADs (two columns x left / right) at fenc row 7 without the pair's DPP add.  An 8x8
// SAD at 10 bit is at most 64 * 1023 = 65472: the quadrant tables stay uint16.
template <int R, int L, int Y, class Sink>
__device__ __forceinline__ void me_row5q( const uint32_t *__restrict__ rbase, int rs_dw, const uint32_t (&F)[8][8],
                                          uint32_t (&acc)[8][4], Sink &sink, uint32_t (&ring)[L][9] )
{
    constexpr int C0 = Y - 7 > 0 ? Y - 7 : 0;
    constexpr int C1 = Y < 2 * R ? Y : 2 * R;
    uint32_t w[9], o[8];
#pragma unroll
    for( int k = 0; k < 9; k++ )
        w[k] = ring[Y % L][k];
    if constexpr( Y + L < 2 * R + 8 )
    {
        const uint32_t *row = rbase + (Y + L) * rs_dw;
#pragma unroll
        for( int k = 0; k < 9; k++ )
            ring[Y % L][k] = row[k];
    }
#pragma unroll
    for( int k = 0; k < 8; k++ )
        o[k] = __builtin_amdgcn_alignbyte( w[k + 1], w[k], 2 );
#pragma unroll
    for( int c = C0; c <= C1; c++ )
    {
        const int r = Y - c;
        uint32_t a[4];
#pragma unroll
        for( int j = 0; j < 4; j++ )
            a[j] = r == 0 ? 0u : acc[c & 7][j];
#pragma unroll
        for( int k = 0; k < 4; k++ )
        {
            a[0] = __builtin_amdgcn_sad_u16( F[r][k], w[k], a[0] );              // column 2g, left
            a[1] = __builtin_amdgcn_sad_u16( F[r][k], o[k], a[1] );              // column 2g+1, left
            a[2] = __builtin_amdgcn_sad_u16( F[r][k + 4], w[k + 4], a[2] );      // column 2g, right
            a[3] = __builtin_amdgcn_sad_u16( F[r][k + 4], o[k + 4], a[3] );      // column 2g+1, right
        }
        if( r == 7 )
            sink( c, a[0] | (a[1] << 16), a[2] | (a[3] << 16) );
        else
        {
#pragma unroll
            for( int j = 0; j < 4; j++ )
                acc[c & 7][j] = a[j];
        }
    }
    __builtin_amdgcn_sched_barrier( 0 );
}

template <int R, int L, class Sink, int... Ys>
__device__ __forceinline__ void me_rows5q( const uint32_t *__restrict__ rbase, int rs_dw, const uint32_t (&F)[8][8],
                                           uint32_t (&acc)[8][4], Sink &sink, std::integer_sequence<int, Ys...> )
{
    uint32_t ring[L][9];
#pragma unroll
    for( int j = 0; j < L; j++ )
#pragma unroll
        for( int k = 0; k < 9; k++ )
            ring[j][k] = rbase[j * rs_dw + k];
    ( me_row5q<R, L, Ys>( rbase, rs_dw, F, acc, sink, ring ), ... );
}

template <int R>
__global__ __launch_bounds__( 256 ) void me_full_sad8q_v5_kernel( const uint16_t *__restrict__ fenc, intptr_t fs,
                                                                  intptr_t ffs, const uint16_t *__restrict__ ref,
                                                                  intptr_t rs, intptr_t rfs, int mbw, int mbh,
                                                                  int nframes, uint16_t *__restrict__ table8, int xcd )
{
    constexpr int G = R + 1, P = full_pitch( R );
    const uint32_t blk = xcd ? xcd_block( blockIdx.x, gridDim.x ) : blockIdx.x;
    const uint32_t slot = blk * blockDim.x + threadIdx.x;
    if( slot >= (uint32_t)nframes * (uint32_t)mbh * (uint32_t)mbw * (uint32_t)(2 * G) )
        return;
    const int h = (int)(slot & 1);
    const uint32_t mb32 = slot / (2 * G), t32 = mb32 / (uint32_t)mbw, f32 = t32 / (uint32_t)mbh;
    const int grp = (int)((slot >> 1) - mb32 * G);
    const int mbx = (int)(mb32 - t32 * (uint32_t)mbw);
    const int mby = (int)(t32 - f32 * (uint32_t)mbh);
    const int64_t mb = mb32, f = f32;
    uint32_t F[8][8];
    const uint32_t *fe = (const uint32_t *)(fenc + f * ffs + (intptr_t)(16 * mby + 8 * h) * fs + 16 * mbx);
    const int fs_dw = (int)(fs / 2);
#pragma unroll
    for( int r = 0; r < 8; r++ )
#pragma unroll
        for( int k = 0; k < 8; k++ )
            F[r][k] = fe[r * fs_dw + k];
    const uint32_t *rbase =
        (const uint32_t *)(ref + f * rfs + (intptr_t)(16 * mby + 8 * h - R) * rs + 16 * mbx - R + 2 * grp);
    // quadrants 2h (left) and 2h + 1 (right), columns 2g, 2g+1 as one dword each
    uint32_t *ql = (uint32_t *)(table8 + (mb * 4 + 2 * h) * ((2 * R + 1) * P) + 2 * grp);
    uint32_t *qr = ql + (2 * R + 1) * P / 2;
    auto store = [ql, qr]( int c, uint32_t l, uint32_t r ) {
        ql[c * (P / 2)] = l;
        qr[c * (P / 2)] = r;
    };
    uint32_t acc[8][4];
    me_rows5q<R, ME_LEAD>( rbase, (int)(rs / 2), F, acc, store, std::make_integer_sequence<int, 2 * R + 8>{} );
}

template <int BD>
hipError_t launch_me_full8( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                            const typename PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs, int mbw, int mbh,
                            int nframes, int range, uint16_t *table8, hipStream_t stream )
{
    constexpr int PSZ = sizeof( typename PT<BD>::pixel );
    const int64_t lanes = (int64_t)nframes * mbh * mbw * (BD == 8 ? full_pitch( range ) / 4 : 2 * (range + 1));
    if( lanes <= 0 )
        return hipSuccess;
    if( lanes >= (1ll << 32) || (((uintptr_t)fenc | (uintptr_t)ref | (uintptr_t)(fs * PSZ) | (uintptr_t)(rs * PSZ) |
                                  (uintptr_t)table8) & 3) )
        return hipErrorInvalidValue;
    dim3 blk( 256 ), g( (unsigned)((lanes + 255) / 256) );
    const int xcd = me_xcd();
    switch( range )
    {
#define ME8_CASE( R )                                                                                           \
        case R:                                                                                                 \
            if constexpr( BD == 8 )                                                                             \
                hipLaunchKernelGGL( ( me_full_sad8q_kernel<R> ), g, blk, 0, stream, fenc, fs, ffs, ref, rs, rfs, \
                                    mbw, mbh, nframes, table8, xcd );                                           \
            else                                                                                                \
                hipLaunchKernelGGL( ( me_full_sad8q_v5_kernel<R> ), g, blk, 0, stream, fenc, fs, ffs, ref, rs,  \
                                    rfs, mbw, mbh, nframes, table8, xcd );                                      \
            break;
        ME8_CASE( 4 ) ME8_CASE( 8 ) ME8_CASE( 16 ) ME8_CASE( 24 )
#undef ME8_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
template hipError_t launch_me_full8<8>( const uint8_t *, intptr_t, intptr_t, const uint8_t *, intptr_t, intptr_t, int,
                                        int, int, int, uint16_t *, hipStream_t );
template hipError_t launch_me_full8<10>( const uint16_t *, intptr_t, intptr_t, const uint16_t *, intptr_t, intptr_t,
                                         int, int, int, int, uint16_t *, hipStream_t );

// Full-search / centred tables.  The grouped kernels need dword-aligned fenc rows,
// dword-multiple strides and a dword-aligned ref plane (and, at 8 bit, a lane count below
// 2^32); anything else runs the generic kernel (one lane per column, realigned loads).
template <int BD>
hipError_t launch_me_full( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                           const typename PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs, int mbw, int mbh,
                           int nframes, int range, typename PT<BD>::sadt *table, const int16_t *centre,
                           int16_t *origin, hipStream_t stream )
{
    constexpr int PSZ = sizeof( typename PT<BD>::pixel );
    const bool cen = centre != nullptr;
    const int64_t nmb = (int64_t)nframes * mbh * mbw;
    if( nmb <= 0 )
        return hipSuccess;
    const int ncol = cen ? cen_pitch( BD, range ) : 2 * range + 1;
    const int64_t groups = BD == 8 ? al4( ncol ) / 4 : 2 * (cen ? cen_cols( 10, range ) / 2 : range + 1);
    bool grouped = !(((uintptr_t)fenc | (uintptr_t)ref | (uintptr_t)(fs * PSZ) | (uintptr_t)(rs * PSZ)) & 3);
    if( nmb * groups >= (1ll << 32) )
        grouped = false;                        // (the grouped kernels index their lanes in 32 bits)
    const int64_t lanes = nmb * (grouped ? groups : ncol);
    dim3 blk( 256 ), g( (unsigned)((lanes + 255) / 256) );
    const int xcd = me_xcd();
    switch( range )
    {
#define ME_GO( R, CEN )                                                                                           \
    if( !grouped )                                                                                                \
        hipLaunchKernelGGL( ( me_full_sad16_kernel<BD, R, CEN ? cen_pitch( BD, R ) : 2 * R + 1> ), g, blk, 0,    \
                            stream, fenc, fs, ffs, ref, rs, rfs, mbw, mbh, nframes, table, centre, origin );      \
    else if constexpr( BD == 8 )                                                                                  \
        hipLaunchKernelGGL( ( me_full_sad16_v7_kernel<R, (CEN ? cen_pitch( 8, R ) : full_pitch( R )) / 4> ), g,   \
                            blk, 0, stream, fenc, fs, ffs, ref, rs, rfs, mbw, mbh, nframes, table, centre, origin, \
                            xcd );                                                                                \
    else                                                                                                          \
        hipLaunchKernelGGL( ( me_full_sad16_v5_kernel<R, CEN ? cen_cols( 10, R ) / 2 : R + 1,                     \
                                                      CEN ? cen_pitch( 10, R ) : full_pitch( R )> ),              \
                            g, blk, 0, stream, fenc, fs, ffs, ref, rs, rfs, mbw, mbh, nframes, table, centre,     \
                            origin, xcd );
#define ME_CASE( R )                                                                                              \
        case R:                                                                                                   \
            if( cen ) { ME_GO( R, true ) } else { ME_GO( R, false ) }                                             \
            break;
        ME_CASE( 4 ) ME_CASE( 8 ) ME_CASE( 16 ) ME_CASE( 24 )
#undef ME_CASE
#undef ME_GO
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template hipError_t launch_me_full<8>( const uint8_t *, intptr_t, intptr_t, const uint8_t *, intptr_t, intptr_t, int,
                                       int, int, int, uint16_t *, const int16_t *, int16_t *, hipStream_t );
template hipError_t launch_me_full<10>( const uint16_t *, intptr_t, intptr_t, const uint16_t *, intptr_t, intptr_t,
                                        int, int, int, int, uint32_t *, const int16_t *, int16_t *, hipStream_t );

// ---------------------------------------------------------------------------
// Fused search + ESA decision (8 bit): the four-column lanes of the centred search around
// each MB's predictor, but each finished candidate row is turned into me_esa_argmin_at's
// packed keys (cost << 12 | raster index in the clipped, width-rounded window,
// encoder/me.c:618-631, cost_mv terms me.c:60-70) and min-reduced in registers instead of
// written out: the table never leaves the chip.  Each of an MB's G lanes meets the others
// through one LDS atomicMin into the MB's key slot, and after the workgroup's barrier one lane
// per MB applies the strict-< update from the predictor cost and writes { cost, mx, my } (no
// key fill, no finishing kernel: 10 bit keeps those).  A workgroup holds whole MBs (256 / G of
// them), whose lanes first stage the MB's per-row key terms in LDS (ycost, row part of the
// raster index, row validity), so a candidate row costs one LDS read instead of a clamped
// global load and its index arithmetic.
// Column groups: an unclipped window's candidates -- width (2R + 3) & ~3 from min_x = bmx - R,
// me.c:626 -- start at most 3 columns past the dword-aligned origin, so G = ceil(((2R+3) & ~3)
// + 3) / 4) groups hold them (9 at R = 16: 36 columns, where the full centred pitch has 40).
// A window whose columns reach further (clipped on the left, so the rounded width runs up to
// two columns past max_x, or an origin clamped at the frame's right edge) needs one more
// group: the workgroup's spare lanes (256 - MPW * G of them) take those MBs' extra group, and
// an MB beyond the spare lanes has its group 0 run the extra columns after its own.
template <int R> constexpr int esa7_groups() { return ((((2 * R + 3) & ~3) + 3) + 3) / 4; }
template <int R> constexpr int esa7_mbs() { return 256 / esa7_groups<R>(); }
constexpr int esa7_groups_rt( int R ) { return ((((2 * R + 3) & ~3) + 3) + 3) / 4; }
// TAB: the same lanes write the centred table instead (the self-contained TESA's scratch table,
// launch_me_tesa): every column an MB's window can reach, the slack columns of unclipped
// windows left unwritten -- no scan reads them.
template <int R, bool TAB>
__global__ __launch_bounds__( 256 ) void me_full_esa_v7_kernel( const uint8_t *__restrict__ fenc, intptr_t fs,
                                                                intptr_t ffs, const uint8_t *__restrict__ ref,
                                                                intptr_t rs, intptr_t rfs, int mbw, int mbh,
                                                                int nframes, int me_range,
                                                                const int16_t *__restrict__ par,
                                                                const uint16_t *__restrict__ cost_mv,
                                                                uint32_t *__restrict__ keys, int xcd,
                                                                uint16_t *__restrict__ tab,
                                                                int16_t *__restrict__ torg,
                                                                const int32_t *__restrict__ init_cost )
{
    constexpr int G = esa7_groups<R>();         // column groups per MB
    constexpr int P = cen_pitch( 8, R );        // the centred template's pitch (me_window's clamp)
    constexpr int W = 2 * R + 1;                // candidate rows
    constexpr int MPW = esa7_mbs<R>();          // whole MBs per workgroup
    constexpr int NSP = 256 - MPW * G;          // spare lanes: extra groups of wide windows
    constexpr int SP = W | 1;                   // LDS row-term pitch (odd: spread banks)
    __shared__ uint32_t s_row[MPW * SP];
    __shared__ uint32_t s_need[MPW];
    __shared__ uint32_t s_key[MPW];             // the MBs' best keys (the workgroup holds whole MBs)
    const uint32_t nmb = (uint32_t)nframes * (uint32_t)mbh * (uint32_t)mbw;
    const int tid = (int)threadIdx.x;
    const bool spare = tid >= MPW * G;
    const uint32_t wg0 = (xcd ? xcd_block( blockIdx.x, gridDim.x ) : blockIdx.x) * MPW;

    // the MB-dependent terms of workgroup MB slot `slot`
    int lmb, grp, mbx, mby, bmx, bmy, min_x, min_y, max_x, max_y, width, ox, oy;
    int64_t mb, f;
    bool live;
    const uint16_t *cx, *cy;
    auto setup = [&]( int slot ) __attribute__( ( always_inline ) ) {
        lmb = slot;
        const uint32_t mbr = wg0 + (uint32_t)slot;
        live = mbr < nmb;
        const uint32_t mb32 = min( mbr, nmb - 1 ), t32 = mb32 / (uint32_t)mbw, f32 = t32 / (uint32_t)mbh;
        mbx = (int)(mb32 - t32 * (uint32_t)mbw);
        mby = (int)(t32 - f32 * (uint32_t)mbh);
        mb = mb32;
        f = f32;
        const int16_t *p = par + 8 * mb;
        bmx = p[0];
        bmy = p[1];
        min_x = max( bmx - me_range, (int)p[4] );
        min_y = max( bmy - me_range, (int)p[5] );
        max_x = min( bmx + me_range, (int)p[6] );
        max_y = min( bmy + me_range, (int)p[7] );
        width = (max_x - min_x + 3) & ~3;
        cx = cost_mv - p[2];
        cy = cost_mv - p[3];
        const int16_t cen[2] = { (int16_t)bmx, (int16_t)bmy };   // the window centre: the predictor
        me_window<8, R, P>( cen, 0, mbx, mby, mbw, mbh, ox, oy );
    };
    setup( spare ? 0 : tid / G );
    grp = spare ? G : tid - lmb * G;
    // this MB's window needs the columns past the G groups
    const bool need = live && min_x + width - 1 - ox >= 4 * G;
    if( !spare && grp == 0 )
    {
        s_need[lmb] = need;
        s_key[lmb] = 0xFFFFFFFFu;
    }
    // row terms S[c] = ycost << 12 | (my - min_y) * width for candidate row c (my = oy + c)
    // inside [min_y, max_y], all ones outside; the MB's lanes stage them together
    if( TAB && !spare && live && grp == 0 )
    {
        torg[2 * mb] = (int16_t)ox;
        torg[2 * mb + 1] = (int16_t)oy;
    }
    if( !TAB && !spare && live )
    {
        uint32_t *srow = s_row + lmb * SP;
#pragma unroll
        for( int c0 = 0; c0 < W; c0 += G )
        {
            const int c = c0 + grp, my = oy + c;
            if( c < W )
                srow[c] = my >= min_y && my <= max_y
                              ? ((uint32_t)cy[4 * my] << 12) + (uint32_t)((my - min_y) * width)
                              : 0xFFFFFFFFu;
        }
    }
    __syncthreads();
    // the extra groups: spare lane s takes the s-th MB that needs one; past the spare lanes the
    // MB's group 0 runs the extra columns itself after its own
    bool twice = false;
    if constexpr( NSP > 0 )
    {
        if( spare )
        {
            int k = tid - MPW * G, slot = -1;
            for( int i = 0; i < MPW && slot < 0; i++ )
                if( s_need[i] && k-- == 0 )
                    slot = i;
            if( slot >= 0 )
                setup( slot );
            else
                live = false;
        }
        else if( grp == 0 && need )
        {
            int rank = 0;
            for( int i = 0; i < lmb; i++ )
                rank += s_need[i] ? 1 : 0;
            twice = rank >= NSP;
        }
    }
    else
        twice = !spare && grp == 0 && need;

    uint32_t F[16][4];
    const uint32_t *fe = (const uint32_t *)(fenc + f * ffs + (intptr_t)(16 * mby) * fs + 16 * mbx);
    const int fs_dw = (int)(fs / 4);
#pragma unroll
    for( int r = 0; r < 16; r++ )
#pragma unroll
        for( int k = 0; k < 4; k++ )
            F[r][k] = fe[r * fs_dw + k];
    const uint32_t *rmb = (const uint32_t *)(ref + f * rfs + (intptr_t)(16 * mby + oy) * rs + 16 * mbx + ox);
    // key = (sad + xcost + ycost) << 12 | raster, raster = (my - min_y) * width + mx - min_x
    // < 4096, built as sat( ((sad << 12) + C[k]) + S ): C[k] = xcost << 12 | column part,
    // or 0xF0000000 outside the window (valid keys stay below 196350 << 12 + 4096 <
    // 0xF0000000, and 0xF0000000 + (65280 << 12) does not wrap); S = ycost << 12 | row
    // part, or all ones outside the window (the add saturates).  Per candidate row: one
    // extract + one shift-add + one saturating add per column and two min3.
    uint32_t ck[4];
    auto columns = [&]( int g ) __attribute__( ( always_inline ) ) {
#pragma unroll
        for( int k = 0; k < 4; k++ )
        {
            const int mx = ox + 4 * g + k;
            const bool in = mx >= min_x && mx < min_x + width;
            ck[k] = in ? ((uint32_t)cx[mx * 4] << 12) + (uint32_t)(mx - min_x) : 0xF0000000u;
        }
    };
    columns( grp );
    uint32_t key = 0xFFFFFFFFu;
    uint32_t *srow = s_row + lmb * SP;
    auto reduce = [&]( int c, uint32_t lo, uint32_t hi ) {
        // read where the row finishes, not hoisted (an LDS-typed pointer, so the pinned
        // address stays a ds_read)
        __attribute__( ( address_space( 3 ) ) ) uint32_t *q = (__attribute__( ( address_space( 3 ) ) ) uint32_t *)srow;
        asm volatile( "" : "+v"( q ) );
        const uint32_t S = q[c];
        // the fields as plain values (else the extract is folded into shift + mask and the
        // shift-add is lost): extract, v_lshl_add, saturating add
        uint32_t w0 = lo & 0xffff, w1 = lo >> 16, w2 = hi & 0xffff, w3 = hi >> 16;
        asm( "" : "+v"( w0 ), "+v"( w1 ), "+v"( w2 ), "+v"( w3 ) );
        const uint32_t k0 = __builtin_elementwise_add_sat( (w0 << 12) + ck[0], S );
        const uint32_t k1 = __builtin_elementwise_add_sat( (w1 << 12) + ck[1], S );
        const uint32_t k2 = __builtin_elementwise_add_sat( (w2 << 12) + ck[2], S );
        const uint32_t k3 = __builtin_elementwise_add_sat( (w3 << 12) + ck[3], S );
        key = min( min( key, k0 ), k1 );
        key = min( min( key, k2 ), k3 );
        asm volatile( "" : "+v"( key ) );        // fold each row where its sums finish
    };
    uint64_t acc[16];
    if constexpr( TAB )
    {
        // (a lane past the last MB rewrites the last MB's values)
        uint64_t *out = (uint64_t *)(tab + mb * ((2 * R + 1) * P) + 4 * grp);
        auto store = [&out]( int c, uint32_t lo, uint32_t hi ) { out[c * (P / 4)] = ((uint64_t)hi << 32) | lo; };
        if( live )
        {
            me_rows7<R, ME_LEAD>( rmb + grp, (int)(rs / 4), F, acc, store, std::make_integer_sequence<int, 2 * R + 16>{} );
            if( twice )
            {
                out = (uint64_t *)(tab + mb * ((2 * R + 1) * P) + 4 * G);
                me_rows7<R, ME_LEAD>( rmb + G, (int)(rs / 4), F, acc, store, std::make_integer_sequence<int, 2 * R + 16>{} );
            }
        }
    }
    else
    {
        me_rows7<R, ME_LEAD>( rmb + grp, (int)(rs / 4), F, acc, reduce, std::make_integer_sequence<int, 2 * R + 16>{} );
        if( twice )
        {
            columns( G );
            me_rows7<R, ME_LEAD>( rmb + G, (int)(rs / 4), F, acc, reduce, std::make_integer_sequence<int, 2 * R + 16>{} );
        }
        if( live && key < 0xF0000000u )
            atomicMin( &s_key[lmb], key );
        __syncthreads();
        // the strict-< update from the predictor result (COPY3_IF_LT, me.h:87-93): { cost, mx, my }
        if( tid < MPW && wg0 + (uint32_t)tid < nmb )
        {
            const int64_t i = wg0 + (uint32_t)tid;
            const int16_t *q = par + 8 * i;
            const int qx = q[0], qy = q[1];
            const int mnx = max( qx - me_range, (int)q[4] ), mny = max( qy - me_range, (int)q[5] );
            const int wd = (min( qx + me_range, (int)q[6] ) - mnx + 3) & ~3;
            const uint32_t k = s_key[tid];
            int32_t bc = init_cost[i], rx = qx, ry = qy;
            if( k != 0xFFFFFFFFu && (int32_t)(k >> 12) < bc )
            {
                const int ki = (int)(k & 4095);
                bc = (int32_t)(k >> 12);
                ry = mny + ki / wd;
                rx = mnx + ki % wd;
            }
            keys[3 * i] = (uint32_t)bc;
            keys[3 * i + 1] = (uint32_t)rx;
            keys[3 * i + 2] = (uint32_t)ry;
        }
    }
}

// out[3*mb] holds the MB's best key (0xFFFFFFFF: nothing evaluated); the strict-< update
// from the predictor result (COPY3_IF_LT, me.h:87-93) turns it into { cost, mx, my }
__global__ __launch_bounds__( 256 ) void me_esa_finish_kernel( int nmb, int me_range, const int16_t *__restrict__ par,
                                                               const int32_t *__restrict__ init_cost,
                                                               int32_t *__restrict__ out )
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if( i >= nmb )
        return;
    const int16_t *p = par + 8 * i;
    const int bmx = p[0], bmy = p[1];
    const int min_x = max( bmx - me_range, (int)p[4] ), min_y = max( bmy - me_range, (int)p[5] );
    const int max_x = min( bmx + me_range, (int)p[6] );
    const int width = (max_x - min_x + 3) & ~3;
    const uint32_t key = (uint32_t)out[3 * i];
    int32_t bcost = init_cost[i], rx = bmx, ry = bmy;
    if( key != 0xFFFFFFFFu && (int32_t)(key >> 12) < bcost )
    {
        const int k = (int)(key & 4095);
        bcost = (int32_t)(key >> 12);
        ry = min_y + k / width;
        rx = min_x + k % width;
    }
    out[3 * i] = bcost;
    out[3 * i + 1] = rx;
    out[3 * i + 2] = ry;
}

// Fused search + ESA decision (10 bit): the column-pair lanes (u32 sums) of the centred
// search around each MB's predictor; lane h of a pair keys column 2g+h.  Keys as the 8-bit
// form (cost < 2^19 at 10 bit: 261888 + two cost_mv terms).
template <int R>
__global__ __launch_bounds__( 256 ) void me_full_esa_v5_kernel( const uint16_t *__restrict__ fenc, intptr_t fs,
                                                                intptr_t ffs, const uint16_t *__restrict__ ref,
                                                                intptr_t rs, intptr_t rfs, int mbw, int mbh,
                                                                int nframes, int me_range,
                                                                const int16_t *__restrict__ par,
                                                                const uint16_t *__restrict__ cost_mv,
                                                                uint32_t *__restrict__ keys, int xcd )
{
    constexpr int G = cen_cols( 10, R ) / 2;    // column pairs per MB
    constexpr int P = cen_pitch( 10, R );
    const int64_t slot = (int64_t)(xcd ? xcd_block( blockIdx.x, gridDim.x ) : blockIdx.x) * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)nframes * mbh * mbw * (2 * G);
    if( slot >= total )
        return;
    const int h = (int)(slot & 1);
    const int grp = (int)((slot >> 1) % G);
    const int64_t mb = slot / (2 * G);
    const int mbx = (int)(mb % mbw);
    const int64_t t = mb / mbw;
    const int mby = (int)(t % mbh);
    const int64_t f = t / mbh;

    uint32_t F[8][8];
    const uint32_t *fe = (const uint32_t *)(fenc + f * ffs + (intptr_t)(16 * mby + 8 * h) * fs + 16 * mbx);
    const int fs_dw = (int)(fs / 2);
#pragma unroll
    for( int r = 0; r < 8; r++ )
#pragma unroll
        for( int k = 0; k < 8; k++ )
            F[r][k] = fe[r * fs_dw + k];
    const int16_t *p = par + 8 * mb;
    const int bmx = p[0], bmy = p[1];
    const int min_x = max( bmx - me_range, (int)p[4] ), min_y = max( bmy - me_range, (int)p[5] );
    const int max_x = min( bmx + me_range, (int)p[6] ), max_y = min( bmy + me_range, (int)p[7] );
    const int width = (max_x - min_x + 3) & ~3;
    const uint16_t *cx = cost_mv - p[2], *cy = cost_mv - p[3];
    int ox, oy;
    const int16_t cen[2] = { (int16_t)bmx, (int16_t)bmy };
    me_window<10, R, P>( cen, 0, mbx, mby, mbw, mbh, ox, oy );
    const uint32_t *rbase =
        (const uint32_t *)(ref + f * rfs + (intptr_t)(16 * mby + 8 * h + oy) * rs + 16 * mbx + ox + 2 * grp);
    const int mxc = ox + 2 * grp + h;
    const bool cin = mxc >= min_x && mxc < min_x + width;
    const uint32_t cinv = cin ? 0u : 0xFFFFFFFFu;
    const int ccost = cin ? (int)cx[mxc * 4] : 0;
    uint32_t key = 0xFFFFFFFFu;
    const int ibase = mxc - min_x - min_y * width;
    // the row cost of candidate row c + 1 is loaded while row c is folded (a row of SADs
    // ahead of its use), the first one before the rows
    uint32_t ynext = cy[4 * min( max( oy, min_y ), max_y )];
    auto reduce = [&]( int c, uint32_t a0, uint32_t a1 ) {
        const int my = oy + c;
        const uint32_t rinv = my >= min_y && my <= max_y ? 0u : 0xFFFFFFFFu;
        const uint32_t ycost = ynext;
        int yi = 4 * min( max( my + 1, min_y ), max_y );
        asm volatile( "" : "+v"( yi ) );         // issued here, not hoisted to the top
        ynext = cy[yi];
        const uint32_t sad = h ? a1 : a0;
        const uint32_t k = ((sad + (uint32_t)ccost + ycost) << 12) | (uint32_t)(my * width + ibase);
        key = min( key, k | cinv | rinv );
        asm volatile( "" : "+v"( key ) );        // fold each row where its sums finish
    };
    uint32_t acc[8][2];
    me_rows5p<R, ME_LEAD>( rbase, (int)(rs / 2), F, acc, reduce, std::make_integer_sequence<int, 2 * R + 8>{} );
    key = min( key, (uint32_t)__builtin_amdgcn_update_dpp( (int)0xFFFFFFFF, (int)key, 0xB1, 0xF, 0xF, false ) );
    if( !h && key != 0xFFFFFFFFu )
        atomicMin( keys + 3 * mb, key );
}

template <int BD>
hipError_t launch_me_search_esa( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                                 const typename PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs, int mbw, int mbh,
                                 int nframes, int range, int me_range, const int16_t *par, const int32_t *init_cost,
                                 const uint16_t *cost_mv, int32_t *out, hipStream_t stream )
{
    const int64_t nmb = (int64_t)nframes * mbw * mbh;
    if( nmb <= 0 )
        return hipSuccess;
    if( nmb > 0x7fffffff ||
        (((uintptr_t)fenc | (uintptr_t)ref | (uintptr_t)(fs * sizeof( typename PT<BD>::pixel )) |
          (uintptr_t)(rs * sizeof( typename PT<BD>::pixel ))) & 3) )
        return hipErrorInvalidValue;
    // 10 bit: the lanes meet in out[3*mb] by atomicMin, then me_esa_finish_kernel; 8 bit: in
    // the workgroup's LDS, which also applies the predictor update (no fill, no second kernel)
    if( BD != 8 )
    {
        const hipError_t e = hipMemsetAsync( out, 0xFF, (size_t)nmb * 3 * sizeof( int32_t ), stream );
        if( e != hipSuccess )
            return e;
    }
    // 8 bit: whole MBs per workgroup (esa7_mbs); 10 bit: a flat lane index over column pairs
    const int64_t mpw = range == 4 ? esa7_mbs<4>() : range == 8 ? esa7_mbs<8>() : range == 16 ? esa7_mbs<16>()
                                                                                               : esa7_mbs<24>();
    const int64_t lanes = nmb * 2 * (cen_cols( 10, range ) / 2);
    dim3 blk( 256 ), g( (unsigned)(BD == 8 ? (nmb + mpw - 1) / mpw : (lanes + 255) / 256) );
    const int xcd = me_xcd();
    switch( range )
    {
#define ESA_CASE( R )                                                                                             \
        case R:                                                                                                   \
            if constexpr( BD == 8 )                                                                               \
                hipLaunchKernelGGL( ( me_full_esa_v7_kernel<R, false> ), g, blk, 0, stream, fenc, fs, ffs, ref, rs, \
                                    rfs, mbw, mbh, nframes, me_range, par, cost_mv, (uint32_t *)out, xcd,         \
                                    nullptr, nullptr, init_cost );                                                \
            else                                                                                                  \
                hipLaunchKernelGGL( ( me_full_esa_v5_kernel<R> ), g, blk, 0, stream, fenc, fs, ffs, ref, rs, rfs, \
                                    mbw, mbh, nframes, me_range, par, cost_mv, (uint32_t *)out, xcd );            \
            break;
        ESA_CASE( 4 ) ESA_CASE( 8 ) ESA_CASE( 16 ) ESA_CASE( 24 )
#undef ESA_CASE
        default: return hipErrorInvalidValue;
    }
    if( BD != 8 )
        hipLaunchKernelGGL( me_esa_finish_kernel, dim3( (unsigned)((nmb + 255) / 256) ), dim3( 256 ), 0, stream,
                            (int)nmb, me_range, par, init_cost, out );
    return hipGetLastError();
}

template hipError_t launch_me_search_esa<8>( const uint8_t *, intptr_t, intptr_t, const uint8_t *, intptr_t, intptr_t,
                                             int, int, int, int, int, const int16_t *, const int32_t *,
                                             const uint16_t *, int32_t *, hipStream_t );
template hipError_t launch_me_search_esa<10>( const uint16_t *, intptr_t, intptr_t, const uint16_t *, intptr_t,
                                              intptr_t, int, int, int, int, int, const int16_t *, const int32_t *,
                                              const uint16_t *, int32_t *, hipStream_t );

// ---------------------------------------------------------------------------
// ESA decision over a table (reference encoder/me.c:618-631 plain exhaustive form, equal
// to its ads path :632-771): one wave per macroblock.  The MB's table rows are read as
// 4-entry chunks (8 bytes at 8 bit, 16 at 10 bit): lane l takes chunk l % NCH of rows
// y0 + l / NCH, + RPS, ... (NCH = pitch / 4 chunks per row, RPS = 64 / NCH rows per step),
// so one step's loads are one contiguous, coalesced run of the table.  A lane's columns are
// fixed, so their cost_mv terms are read once; the row term once per step.  Each entry's
// key (cost << 12 | raster index in the clipped, width-rounded window) is built as
// sat( sat( (sad << 12) + C[k] ) + S ) with C[k] = all ones outside the window or the table's
// columns, so whatever such an entry holds (a full 10-bit table's padding columns are never
// written) its key saturates (valid keys stay below 392958 << 12 + 4096), a wave min picks the lowest cost and, among equal costs, the first in raster
// order -- what the strict-< scan of the reference keeps -- and it replaces the predictor
// result only if strictly better (COPY3_IF_LT, me.h:87-93).
// Table geometry: rows = 2R+1 at `pitch`, `cols` valid columns, window origin (ox, oy)
// from `origin` (centred tables) or (-R, -R) (full tables).
// one MB's window geometry (me.c:618-626) and table position, all wave-uniform
struct EsaGeo
{
    int bmx, bmy, mvpx, mvpy, min_x, min_y, width, ox, oy, y0, y1, nsteps;
};
__device__ __forceinline__ EsaGeo esa_geo( const int16_t *par, const int16_t *origin, int mb, int R, int me_range,
                                           int rps )
{
    EsaGeo g;
    const int16_t *p = par + 8 * mb;
    g.bmx = p[0]; g.bmy = p[1]; g.mvpx = p[2]; g.mvpy = p[3];
    g.min_x = max( g.bmx - me_range, (int)p[4] );
    g.min_y = max( g.bmy - me_range, (int)p[5] );
    const int max_x = min( g.bmx + me_range, (int)p[6] ), max_y = min( g.bmy + me_range, (int)p[7] );
    g.width = (max_x - g.min_x + 3) & ~3;
    g.ox = origin ? origin[2 * mb] : -R;
    g.oy = origin ? origin[2 * mb + 1] : -R;
    g.y0 = max( g.min_y, g.oy );
    g.y1 = min( max_y, g.oy + 2 * R );
    g.nsteps = g.width > 0 && g.y1 >= g.y0 ? (g.y1 - g.y0 + rps) / rps : 0;
    return g;
}

// A wave walks MBs wave, wave + nwaves, ...: the next MB's table chunks are requested before
// the current MB is scored, so every wave keeps a table's worth of loads in flight while it
// works (one MB per wave left the loads idle through each MB's parameter fetch, cost gathers
// and reduction: 0.101 ms, 0.42 of HBM, for the 16-pair 1080p table; 0.095 ms this way).  The
// current MB's cost gathers are issued before the next MB's table loads, so waiting for them
// never waits for those (vmcnt retires in order), and the table loads are branch-free, so the
// compiler's wait counts stay exact.  (Fetching the next MB's cost gathers early too measured
// 0.0986 ms: no better.)
template <int BD, int MAXS, int E>
__global__ __launch_bounds__( 256 ) void me_esa_argmin_kernel( const typename PT<BD>::sadt *__restrict__ table, int R,
                                                               int cols, int pitch, int nmb, int me_range,
                                                               const int16_t *__restrict__ origin,
                                                               const int16_t *__restrict__ par,
                                                               const int32_t *__restrict__ init_cost,
                                                               const uint16_t *__restrict__ cost_mv,
                                                               int32_t *__restrict__ out )
{
    // a lane's chunk: E table entries (8 bit: 4 = 8 bytes, or 8 = 16 bytes when the pitch allows;
    // 10 bit: 4 = 16 bytes)
    using chunk = typename std::conditional<BD == 8 && E == 4, uint2, uint4>::type;
    const int lane = threadIdx.x & 63;
    // the MB index is wave-uniform: made a scalar, so its par / origin / init_cost words are
    // scalar loads and the address path carries only the table and cost_mv reads
    int mb = __builtin_amdgcn_readfirstlane( (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6) );
    const int nwaves = (int)(gridDim.x * (blockDim.x >> 6));
    if( mb >= nmb )
        return;
    const int W = 2 * R + 1;
    const int nch = pitch / E, rps = 64 / nch;                     // pitch <= 64: >= 4 rows per step
    const int rr = lane / nch, ch = lane - rr * nch;
    // branch-free: every lane loads every step at a row clamped into the MB's table (the
    // lanes and steps outside the window are masked where the values are used), so the
    // compiler's wait counts stay exact across the next MB's loads
    auto fetch = [&]( const EsaGeo &g, int m, chunk (&v)[MAXS] ) {
        const chunk *t = (const chunk *)(table + m * (int64_t)(W * pitch)) + ch;
#pragma unroll
        for( int st = 0; st < MAXS; st++ )
        {
            const int row = min( max( g.y0 + st * rps + rr - g.oy, 0 ), W - 1 );
            v[st] = t[row * nch];
        }
    };
    EsaGeo g = esa_geo( par, origin, mb, R, me_range, rps );
    chunk v[MAXS];
    fetch( g, mb, v );
    for( ;; )
    {
        // the MB's cost_mv terms in two gathers -- column c's in lane c, table row r's in lane r
        // -- handed to the lanes that use them by ds_bpermute: a lane's four columns once, a
        // row's term once per step
        const int cl = min( lane, pitch - 1 ), mxl = g.ox + cl;
        const bool cin = cl < cols && mxl >= g.min_x && mxl < g.min_x + g.width;
        const uint32_t ckl =
            cin ? ((uint32_t)cost_mv[mxl * 4 - g.mvpx] << 12) + (uint32_t)(mxl - g.min_x) : 0xFFFFFFFFu;
        const int myl = min( max( g.oy + lane, g.y0 ), g.y1 );
        const uint32_t Sl = ((uint32_t)cost_mv[myl * 4 - g.mvpy] << 12) + (uint32_t)((myl - g.min_y) * g.width);
        const int32_t icost = init_cost[mb];
        // the next MB's table, in flight while this one is scored (the last MB of the wave
        // re-reads its own: no branch around the loads)
        const int mbn = mb + nwaves;
        const bool has_next = mbn < nmb;
        const int mbf = has_next ? mbn : mb;
        const EsaGeo gn = esa_geo( par, origin, mbf, R, me_range, rps );
        chunk vn[MAXS];
        fetch( gn, mbf, vn );
        uint32_t ck[E];
#pragma unroll
        for( int k = 0; k < E; k++ )
            ck[k] = (uint32_t)__builtin_amdgcn_ds_bpermute( 4 * (E * ch + k), (int)ckl );
        uint32_t key = 0xFFFFFFFFu;
#pragma unroll
        for( int st = 0; st < MAXS; st++ )
        {
            const int my = g.y0 + st * rps + rr;
            const uint32_t S = (uint32_t)__builtin_amdgcn_ds_bpermute( 4 * min( max( my - g.oy, 0 ), 63 ), (int)Sl );
            if( st < g.nsteps && rr < rps && my <= g.y1 )
            {
                uint32_t s4[E];
                if constexpr( BD == 8 && E == 4 )
                {
                    s4[0] = v[st].x & 0xffff; s4[1] = v[st].x >> 16; s4[2] = v[st].y & 0xffff; s4[3] = v[st].y >> 16;
                }
                else if constexpr( BD == 8 )
                {
                    s4[0] = v[st].x & 0xffff; s4[1] = v[st].x >> 16; s4[2] = v[st].y & 0xffff; s4[3] = v[st].y >> 16;
                    s4[4] = v[st].z & 0xffff; s4[5] = v[st].z >> 16; s4[6] = v[st].w & 0xffff; s4[7] = v[st].w >> 16;
                }
                else
                {
                    s4[0] = v[st].x; s4[1] = v[st].y; s4[2] = v[st].z; s4[3] = v[st].w;
                }
#pragma unroll
                for( int k = 0; k < E; k++ )
                    key = min( key, __builtin_elementwise_add_sat(
                                        __builtin_elementwise_add_sat( s4[k] << 12, ck[k] ), S ) );
            }
        }
        // the wave minimum by DPP (row_shr 1/2/4/8, row_bcast 15/31): lane 63 ends with it
        {
            constexpr int I = (int)0xFFFFFFFF;
            key = min( key, (uint32_t)__builtin_amdgcn_update_dpp( I, (int)key, 0x111, 0xF, 0xF, false ) );
            key = min( key, (uint32_t)__builtin_amdgcn_update_dpp( I, (int)key, 0x112, 0xF, 0xF, false ) );
            key = min( key, (uint32_t)__builtin_amdgcn_update_dpp( I, (int)key, 0x114, 0xF, 0xF, false ) );
            key = min( key, (uint32_t)__builtin_amdgcn_update_dpp( I, (int)key, 0x118, 0xF, 0xF, false ) );
            key = min( key, (uint32_t)__builtin_amdgcn_update_dpp( I, (int)key, 0x142, 0xA, 0xF, false ) );
            key = min( key, (uint32_t)__builtin_amdgcn_update_dpp( I, (int)key, 0x143, 0xC, 0xF, false ) );
        }
        if( lane == 63 )
        {
            int32_t bcost = icost, rx = g.bmx, ry = g.bmy;
            if( key < 0xC0000000u && (int32_t)(key >> 12) < bcost )
            {
                const int i = (int)(key & 4095);
                bcost = (int32_t)(key >> 12);
                ry = g.min_y + i / g.width;
                rx = g.min_x + i % g.width;
            }
            out[3 * mb] = bcost;
            out[3 * mb + 1] = rx;
            out[3 * mb + 2] = ry;
        }
        if( !has_next )
            break;
        mb = mbn;
        g = gn;
#pragma unroll
        for( int st = 0; st < MAXS; st++ )
            v[st] = vn[st];
    }
}

template <int BD>
hipError_t launch_me_esa_argmin( const typename PT<BD>::sadt *table, int R, int nmb, int me_range,
                                 const int16_t *origin, const int16_t *par, const int32_t *init_cost,
                                 const uint16_t *cost_mv, int32_t *out, hipStream_t stream )
{
    if( nmb <= 0 )
        return hipSuccess;
    // centred tables (an origin given) hold the ESA window's columns, full tables the square
    const int cols = origin ? cen_cols( BD, R ) : 2 * R + 1;
    const int pitch = origin ? cen_pitch( BD, R ) : full_pitch( R );
    if( pitch > 64 || ((uintptr_t)table & (BD == 8 ? 7 : 15)) )
        return hipErrorInvalidValue;
    // steps of 64 / (pitch / E) rows cover the 2R+1 table rows (the kernel is instantiated
    // for the exact count, since it loads every step); 16 waves of every SIMD of the 256 CUs
    // walk the MBs (fewer when there are fewer MBs; 4 / 8 / 12 / 16 per SIMD: 0.100 / 0.085 /
    // 0.083 / 0.081 ms, profiles/r04w_*).  8-bit tables whose pitch is a multiple of 8 entries
    // (the centred ones) are read 16 bytes per lane (E = 8): half the load instructions, 0.094 ->
    // 0.079-0.084 ms for the 16-pair 1080p table (profiles/r04v_*).
    const bool wide = BD == 8 && pitch % 8 == 0 && !((uintptr_t)table & 15);
    const int E = wide ? 8 : 4;
    const int rps = 64 / (pitch / E), steps = (2 * R + 1 + rps - 1) / rps;
    const int waves = std::min( nmb, 256 * 4 * 16 );
    const dim3 g( (unsigned)((waves + 3) / 4) ), b( 256 );
#define ARGMIN_CASE( S, EE )                                                                                     \
    case S:                                                                                                      \
        hipLaunchKernelGGL( ( me_esa_argmin_kernel<BD, S, EE> ), g, b, 0, stream, table, R, cols, pitch, nmb,      \
                            me_range, origin, par, init_cost, cost_mv, out );                                    \
        break;
    if( wide )
    {
        switch( steps )
        {
            ARGMIN_CASE( 1, 8 ) ARGMIN_CASE( 2, 8 ) ARGMIN_CASE( 3, 8 ) ARGMIN_CASE( 4, 8 ) ARGMIN_CASE( 5, 8 )
            ARGMIN_CASE( 6, 8 ) ARGMIN_CASE( 7, 8 ) ARGMIN_CASE( 8, 8 )
            default: return hipErrorInvalidValue;
        }
    }
    else
    {
        switch( steps )
        {
            ARGMIN_CASE( 1, 4 ) ARGMIN_CASE( 2, 4 ) ARGMIN_CASE( 3, 4 ) ARGMIN_CASE( 4, 4 ) ARGMIN_CASE( 5, 4 )
            ARGMIN_CASE( 6, 4 ) ARGMIN_CASE( 7, 4 ) ARGMIN_CASE( 8, 4 ) ARGMIN_CASE( 9, 4 ) ARGMIN_CASE( 10, 4 )
            ARGMIN_CASE( 11, 4 ) ARGMIN_CASE( 12, 4 ) ARGMIN_CASE( 13, 4 ) ARGMIN_CASE( 14, 4 ) ARGMIN_CASE( 15, 4 )
            ARGMIN_CASE( 16, 4 )
            default: return hipErrorInvalidValue;
        }
    }
#undef ARGMIN_CASE
    return hipGetLastError();
}

template hipError_t launch_me_esa_argmin<8>( const uint16_t *, int, int, int, const int16_t *, const int16_t *,
                                             const int32_t *, const uint16_t *, int32_t *, hipStream_t );
template hipError_t launch_me_esa_argmin<10>( const uint32_t *, int, int, int, const int16_t *, const int16_t *,
                                              const int32_t *, const uint16_t *, int32_t *, hipStream_t );

// ---------------------------------------------------------------------------
// TESA (reference encoder/me.c:653-748) for PIXEL_16x16: one wave per macroblock.
//
// The reference walks the window row by row.  Within a row its running bsad only
// ever drops to a SAD that was appended, and every SAD below bsad is appended
// (the threshold bsad*sad_thresh>>3 >= bsad), so the bsad a candidate is tested
// against is min(row-start bsad, prefix minimum of the earlier ADS survivors'
// SADs).  A row is therefore one lane per column (width <= 64): ads4 and its
// bsad*17>>4 threshold per lane, the 16x16 SAD on the surviving lanes only, a
// wave prefix-min, and a ballot + mbcnt append into the LDS mvsads list in
// column order -- the reference's exact list.  Rows stay sequential (a row's ADS
// threshold depends on every earlier row).  The halving prune is an in-order
// LDS compaction, the drop-the-first-maximum loop a wave argmax, and the final
// COST_MV scores the <= me_range/2 survivors as 8x4 units spread over the lanes
// (satd_16x16 = the sum of eight satd_8x4, pixel.c:265-306), reduced with the
// strict-< first-index rule of COPY3_IF_LT.
template <int BD>
__device__ __forceinline__ uint32_t tesa_sad16( const uint32_t *fenc_lds, const typename PT<BD>::pixel *r,
                                                intptr_t rs )
{
    constexpr int NDW = 16 / PT<BD>::PPD;
    uint32_t acc = 0;
#pragma unroll 4
    for( int y = 0; y < 16; y++ )
    {
        uint32_t w[NDW];
        load_row_u<NDW>( r + y * rs, w );
#pragma unroll
        for( int k = 0; k < NDW; k++ )
            acc = sadp<BD>( fenc_lds[y * NDW + k], w[k], acc );
    }
    return acc;
}

// |a - b| + c of unsigned 32-bit values (v_sad_u32; clang has no builtin for it)
__device__ __forceinline__ uint32_t sad_u32( uint32_t a, uint32_t b, uint32_t c )
{
    uint32_t d;
    asm( "v_sad_u32 %0, %1, %2, %3" : "=v"( d ) : "v"( a ), "v"( b ), "v"( c ) );
    return d;
}

// inclusive min-scan over each SEG-lane segment (32 or 64) with DPP: row_shr 1/2/4/8
// inside the 16-lane rows, then row_bcast:15 (and :31 for a 64-lane segment) across
// them -- no LDS-crossbar round trips (ds_bpermute) on TESA's serial row chain
template <int SEG> __device__ __forceinline__ uint32_t seg_scan_min( uint32_t x )
{
    constexpr int I = (int)0xFFFFFFFF;
    x = min( x, (uint32_t)__builtin_amdgcn_update_dpp( I, (int)x, 0x111, 0xF, 0xF, false ) );
    x = min( x, (uint32_t)__builtin_amdgcn_update_dpp( I, (int)x, 0x112, 0xF, 0xF, false ) );
    x = min( x, (uint32_t)__builtin_amdgcn_update_dpp( I, (int)x, 0x114, 0xF, 0xF, false ) );
    x = min( x, (uint32_t)__builtin_amdgcn_update_dpp( I, (int)x, 0x118, 0xF, 0xF, false ) );
    x = min( x, (uint32_t)__builtin_amdgcn_update_dpp( I, (int)x, 0x142, 0xA, 0xF, false ) );
    if constexpr( SEG == 64 )
        x = min( x, (uint32_t)__builtin_amdgcn_update_dpp( I, (int)x, 0x143, 0xC, 0xF, false ) );
    return x;
}

// inclusive sum-scan over each SEG-lane segment, as seg_scan_min
template <int SEG> __device__ __forceinline__ uint32_t seg_scan_add( uint32_t x )
{
    x += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)x, 0x111, 0xF, 0xF, false );
    x += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)x, 0x112, 0xF, 0xF, false );
    x += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)x, 0x114, 0xF, 0xF, false );
    x += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)x, 0x118, 0xF, 0xF, false );
    x += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)x, 0x142, 0xA, 0xF, false );
    if constexpr( SEG == 64 )
        x += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)x, 0x143, 0xC, 0xF, false );
    return x;
}

// value of lane `l` of this lane's segment (l compile-time or wave-uniform), via readlane
template <int SEG> __device__ __forceinline__ uint32_t seg_lane( uint32_t v, int l, int sg )
{
    if constexpr( SEG == 64 )
        return (uint32_t)__builtin_amdgcn_readlane( (int)v, l );
    else
    {
        const uint32_t a = (uint32_t)__builtin_amdgcn_readlane( (int)v, l );
        const uint32_t b = (uint32_t)__builtin_amdgcn_readlane( (int)v, 32 + l );
        return sg ? b : a;
    }
}

// the same through the LDS crossbar (ds_bpermute, no VALU): lane l of this lane's segment.
// For the per-row broadcasts of the TESA scan, where readlane + a per-segment select cost
// four or five VALU instructions per row; `base` = (segment start lane) * 4.
template <int SEG> __device__ __forceinline__ uint32_t seg_bcast( uint32_t v, int l, int base )
{
    if constexpr( SEG == 64 )
        return (uint32_t)__builtin_amdgcn_readlane( (int)v, l );
    else
        return (uint32_t)__builtin_amdgcn_ds_bpermute( base + 4 * l, (int)v );
}

__device__ __forceinline__ uint32_t wave_min_u32( uint32_t v )
{
#pragma unroll
    for( int off = 32; off >= 1; off >>= 1 )
        v = min( v, (uint32_t)__shfl_xor( (int)v, off ) );
    return v;
}

// rows per staging chunk of the TESA scan (a build-time knob for A/B builds; divides the
// 8-row ads offset): 4 rows 0.656 ms per 16 1080p frames (128 VGPRs, 4 waves/SIMD), 2 rows
// 0.659, 8 rows 0.696 (158 VGPRs, 3 waves)
#ifndef TESA_CK
#define TESA_CK 4
#endif
// minimum waves per SIMD of the scan kernel (a build-time knob for A/B builds): at 5 (96
// VGPRs; LDS then holds ~4.5 waves per SIMD) the scan spills and runs slower -- 0.625 ms with
// 1-row chunks, 0.655 with 2-row chunks, against 0.583 for 4 waves and 4-row chunks
// (profiles/r03as/)
#ifndef TESA_WPE
#define TESA_WPE 4
#endif

// SEG lanes per MB: 64 (one MB per wave, me_range <= 32) or 32 (two MBs per wave,
// me_range <= 16: a row of <= 32 columns fits half a wave), so a wave's serial row
// chain serves two MBs.  Every per-MB value is uniform within its segment; ballots are
// masked to the segment, scans and reductions stay inside it, and loops run while any
// segment still needs them.
// The LDS a TESA scan touches (fenc rows, mvsads list) belongs to its own wave, and a
// wave's LDS operations complete in order, so the scan orders its LDS hand-offs between
// lanes with a wave-scope fence (a compiler barrier) instead of a workgroup barrier: the
// fused kernel below runs it in waves that take different numbers of MBs.
__device__ __forceinline__ void tesa_wave_sync()
{
    __builtin_amdgcn_fence( __ATOMIC_SEQ_CST, "wavefront" );
    __builtin_amdgcn_wave_barrier();
}

// NSEG mvsads lists.  64-lane segments: { cost, mx | my << 16 } in 8 bytes; 32-lane
// segments (me_range <= 16: < 32 columns, <= 33 rows, cost < 2^20) pack cost << 11 |
// row << 5 | column into 4 bytes, which halves the LDS a workgroup holds (2 -> 4 waves
// per SIMD with 128 VGPRs)
template <int SEG> using tesa_ent = typename std::conditional<SEG == 32, uint32_t, uint64_t>::type;

// One MB per SEG-lane segment of the calling wave: segment sg of the wave scans MB `mbo`
// (clamped to the last MB; it publishes only when `live` and mbo < nmb) whose table window
// starts at (ox, oy) relative to the MB.  `mvsads` / `fl` are this segment's LDS list and
// fenc rows.
template <int BD, int NR, int SEG, bool TAB, bool SPEC>
__device__ __forceinline__ void tesa_scan_mb( const typename PT<BD>::pixel *__restrict__ fenc, intptr_t fs, intptr_t ffs,
                                              const typename PT<BD>::pixel *__restrict__ ref, intptr_t rs, intptr_t rfs,
                                              const uint16_t *__restrict__ integral, intptr_t ifs, int mbw, int mbh,
                                              int nmb, int me_range, int satd,
                                              const typename PT<BD>::sadt *__restrict__ table, int R, int tcols, int tpitch,
                                              int ox, int oy,
                                              const int16_t *__restrict__ par, const int32_t *__restrict__ init_cost,
                                              const uint16_t *__restrict__ cost_mv, int32_t *__restrict__ out,
                                              int64_t mbo, bool live, int sg, int lane, tesa_ent<SEG> *mvsads,
                                              uint32_t *fl )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int NDW = 16 / PT<BD>::PPD;                     // dwords per fenc row
    using E = tesa_ent<SEG>;
    const int64_t mb = mbo < nmb ? mbo : nmb - 1;             // a spare segment repeats the last MB
    const uint64_t segmask = SEG == 64 ? ~0ull : 0xFFFFFFFFull << (32 * sg);
    auto sball = [&]( bool c ) { return (uint64_t)__ballot( c ) & segmask; };
    auto rank = [&]( uint64_t m ) {
        return (int)__builtin_amdgcn_mbcnt_hi( (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo( (uint32_t)m, 0u ) );
    };
    auto any = []( bool c ) { return __ballot( c ) != 0; };
    const int mbx = (int)(mb % mbw);
    const int64_t t = mb / mbw;
    const int mby = (int)(t % mbh);
    const int64_t f = t / mbh;
    const pixel *p_fenc = fenc + f * ffs + 16 * (mby * fs + mbx);
    const pixel *p_fref = ref + f * rfs + 16 * (mby * rs + mbx);
    const uint16_t *sums_base = integral + f * ifs + 16 * (mby * rs + mbx);
    const int16_t *p = par + 8 * mb;
    const int bmx0 = p[0], bmy0 = p[1];
    const uint16_t *cx = cost_mv - p[2], *cy = cost_mv - p[3];
    const int min_x = max( bmx0 - me_range, (int)p[4] ), min_y = max( bmy0 - me_range, (int)p[5] );
    const int max_x = min( bmx0 + me_range, (int)p[6] ), max_y = min( bmy0 + me_range, (int)p[7] );
    const int width = (max_x - min_x + 3) & ~3;
    auto ent = [&]( uint32_t cost, int ex, int ey ) -> E {
        if constexpr( SEG == 32 )
            return (cost << 11) | (uint32_t)((ey - min_y) << 5) | (uint32_t)(ex - min_x);
        else
            return (uint64_t)cost | ((uint64_t)(uint16_t)ex << 32) | ((uint64_t)(uint16_t)ey << 48);
    };
    auto ecost = []( E e ) -> uint32_t {
        if constexpr( SEG == 32 ) return (uint32_t)(e >> 11); else return (uint32_t)e;
    };
    auto emx = [&]( E e ) -> int {
        if constexpr( SEG == 32 ) return min_x + (int)(e & 31); else return (int)(int16_t)(e >> 32);
    };
    auto emy = [&]( E e ) -> int {
        if constexpr( SEG == 32 ) return min_y + (int)((e >> 5) & 63); else return (int)(int16_t)(e >> 48);
    };

    // fenc -> LDS (row-major dwords) and enc_dc (sad_x4 against x264_zero = the four 8x8 sums)
    uint32_t dcq[4] = { 0, 0, 0, 0 };
    for( int i = lane; i < 16 * NDW; i += SEG )
    {
        const int y = i / NDW, k = i % NDW;
        const uint32_t w = *(const uint32_t *)(p_fenc + y * fs + k * PT<BD>::PPD);
        fl[i] = w;
        const uint32_t s = sadp<BD>( w, 0u, 0u );
        const int q = (k * PT<BD>::PPD >= 8) + 2 * (y >= 8);
#pragma unroll
        for( int j = 0; j < 4; j++ )
            dcq[j] += q == j ? s : 0u;
    }
    int enc_dc[4];
#pragma unroll
    for( int j = 0; j < 4; j++ )                              // segment sums: DPP scan + readlane
        enc_dc[j] = (int)seg_lane<SEG>( seg_scan_add<SEG>( dcq[j] ), SEG - 1, sg );
    tesa_wave_sync();

    // table: 2R+1 rows of tcols valid columns at pitch tpitch (centred or full geometry)
    const int W = 2 * R + 1, P = tpitch;
    const typename PT<BD>::sadt *tab = TAB ? table + mb * (int64_t)(W * P) : nullptr;
    auto sad_at = [&]( int mx, int my ) -> uint32_t {
        const int tx = mx - ox, ty = my - oy;
        if( TAB && tx >= 0 && tx < tcols && ty >= 0 && ty < W )
            return (uint32_t)tab[ty * P + tx];
        return tesa_sad16<BD>( fl, p_fref + my * rs + mx, rs );
    };

    const int sad_thresh0 = me_range <= 16 ? 10 : me_range <= 24 ? 11 : 12;
    const bool active = lane < width;
    const int mx = min_x + lane;
    const int fpel = active ? (int)cx[mx * 4] : 0;           // cost_fpel_mvx[mx] (analyse.c:161-169)
    const int bsad0 = (int)sad_at( bmx0, bmy0 ) + (int)cx[bmx0 * 4] + (int)cy[bmy0 * 4];
    const int rows = max( max_y - min_y + 1, 0 );            // <= 2*me_range+1
    // ycost of row r in segment lane r (rows SEG.. in the second register)
    const int yc0 = lane < rows ? (int)cy[(min_y + lane) * 4] : 0;
    const int yc1 = lane + SEG < rows ? (int)cy[(min_y + lane + SEG) * 4] : 0;
    const int bbase = 4 * SEG * sg;                           // this segment's lane 0, in bytes
    auto ycost_of = [&]( int r ) { return (int)seg_bcast<SEG>( (uint32_t)(r < SEG ? yc0 : yc1), r % SEG, bbase ); };
    // row r's speculative ADS bound (bsad0 - ycost)*17>>4 (0 when ycost >= bsad0), per lane like
    // the ycosts and broadcast the same way
    auto ubound = [&]( int yc ) { return bsad0 > yc ? (bsad0 - yc) * 17 >> 4 : 0; };
    const int ub0 = ubound( yc0 ), ub1 = ubound( yc1 );
    auto ub_of = [&]( int r ) { return (int)seg_bcast<SEG>( (uint32_t)(r < SEG ? ub0 : ub1), r % SEG, bbase ); };

    // Staging: each row's ads4 value and -- with a table -- the cost of every candidate
    // that can still pass some row's threshold (bsad never rises, so row r's ADS threshold
    // is at most (bsad0 - ycost)*17>>4) do not depend on the scan state.  They are loaded
    // in chunks of CK rows, one chunk ahead of the scan: chunk c + 1's loads are issued
    // before chunk c's rows are scanned.  Loads are branch-free at clamped (valid)
    // addresses, the rows / lanes outside the window masked afterwards, and each integral
    // row is loaded once although row r's ads reads rows r and r + 8.
    constexpr int CK = TESA_CK, NC = (NR + CK - 1) / CK;
    const int cxm = active ? mx : min_x;
    const int tx = mx - ox, txc = min( max( tx, 0 ), tcols - 1 );
    const bool colin = tx >= 0 && tx < tcols;
    // rows as 24-bit multiplies of small offsets from per-lane bases (j <= 2*32+8 rows of a
    // stride below 2^18 elements; table rows < 66 of a pitch < 69), not 64-bit address math
    const uint16_t *ib = sums_base + cxm + (intptr_t)min_y * rs;
    const uint32_t irs = (uint32_t)rs;
    const int rmax = rows + 7, ty0 = min_y - oy;
    // (the row's two sums packed in one dword, sum at +8 in the high half: one v_sad_u16 then
    // scores both of a row's ADS terms against the packed encode sums)
    auto ldi = [&]( int j, uint32_t &pv ) {
        const uint16_t *sp = ib + __umul24( (uint32_t)min( j, rmax ), irs );
        pv = __builtin_amdgcn_perm( (uint32_t)sp[8], (uint32_t)sp[0], 0x05040100u );
    };
    const uint32_t dc01 = (uint32_t)enc_dc[0] | ((uint32_t)enc_dc[1] << 16);
    const uint32_t dc23 = (uint32_t)enc_dc[2] | ((uint32_t)enc_dc[3] << 16);
    // every candidate a lane can stage is in the table (the row / column ranges of the window
    // inside the table's): wave-uniform, so the per-row test for the rare outside candidate
    // is skipped by a scalar branch
    const bool covered = !TAB || __all( (!active || colin) && (rows == 0 || (min_y - oy >= 0 && max_y - oy < W)) );
    auto ldt = [&]( int r ) -> uint32_t {
        if constexpr( TAB )
            return (uint32_t)tab[__umul24( (uint32_t)min( max( ty0 + r, 0 ), W - 1 ), (uint32_t)P ) + txc];
        else
            return 0u;
    };
    int bsad = bsad0;
    int nmvsad = 0;
    // one row of the reference's scan (me.c:667-703) over its staged values
    auto scan_row = [&]( int r, uint32_t ads, uint32_t sr ) {
        const int my = min_y + r;
        const int ycost = ycost_of( r );
        const bool rowok = r < rows && bsad > ycost;
        const int b = bsad - ycost;
        const bool pass = rowok && ads < (uint32_t)(b * 17 >> 4);
        if( !any( pass ) )
            return;                                         // no segment's bsad changes
        // a passing lane's cost was staged (b <= bsad0 - ycost), or is computed now
        const uint32_t s = pass ? (TAB ? sr : sad_at( mx, my ) + (uint32_t)fpel) : 0xFFFFFFFFu;
        // exclusive prefix minimum over the segment's lanes (the earlier survivors of this row)
        const uint32_t incl = seg_scan_min<SEG>( s );
        uint32_t excl = (uint32_t)__builtin_amdgcn_update_dpp( (int)0xFFFFFFFF, (int)incl, 0x138, 0xF, 0xF, false );
        excl = lane ? excl : 0xFFFFFFFFu;                   // wave_shr:1 crosses into segment 1's lane 0
        const int bcur = (int)min( (uint32_t)b, excl );
        const bool app = pass && (int)s < (bcur * sad_thresh0 >> 3);
        const uint64_t m = sball( app );
        if( app )
            mvsads[nmvsad + rank( m )] = ent( s + (uint32_t)ycost, mx, my );
        nmvsad += __popcll( m );
        const uint32_t rmin = seg_lane<SEG>( incl, SEG - 1, sg );
        if( sball( pass ) )
            bsad = min( bsad, (int)rmin + ycost );            // b_final + ycost
    };
    // integral rows in a ring of D chunks: chunk c's ads reads its own rows (slot c % D) and
    // the rows 8 below (slot (c + 8 / CK) % D); table rows for the current chunk only
    static_assert( CK == 1 || CK == 2 || CK == 4 || CK == 8, "CK divides the 8-row ads offset" );
    constexpr int D = 8 / CK + 1;
    uint32_t ip[D][CK], tt[CK];
#pragma unroll
    for( int q = 0; q < D; q++ )
#pragma unroll
        for( int k = 0; k < CK; k++ )
            ldi( CK * q + k, ip[q][k] );
#pragma unroll
    for( int k = 0; k < CK; k++ )
        tt[k] = ldt( k );
#pragma unroll
    for( int c = 0; c < NC; c++ )
    {
        uint32_t n0[CK], nt[CK];
        if( c + 1 < NC )
        {
#pragma unroll
            for( int k = 0; k < CK; k++ )
            {
                ldi( CK * (c + D) + k, n0[k] );           // chunk c + D, into slot c % D after use
                nt[k] = ldt( CK * (c + 1) + k );
            }
        }
        __builtin_amdgcn_sched_barrier( 0 );
        const int st = c % D, sb = (c + 8 / CK) % D;
        uint32_t sr_k[CK], ads_k[CK];
        int ys_k[CK];                                         // the rows' ycost (TAB: read once)
#pragma unroll
        for( int k = 0; k < CK; k++ )
        {
            sr_k[k] = ads_k[k] = 0xFFFFFFFFu;
            ys_k[k] = 0;
            const int r = CK * c + k;
            if( r >= NR )
                break;
            // |dc - sum| + acc, two terms per v_sad_u16 (sums and DCs are 16-bit)
            const uint32_t av = __builtin_amdgcn_sad_u16( ip[st][k], dc01,
                                                          __builtin_amdgcn_sad_u16( ip[sb][k], dc23, (uint32_t)fpel ) );
            const uint32_t ads = r < rows && active ? av : 0xFFFFFFFFu;
            uint32_t sr = 0xFFFFFFFFu;
            if constexpr( TAB )
            {
                // with a table the SADs are reads (the rare candidate outside it computed)
                const int ycost = ycost_of( r ), ty = min_y + r - oy;
                ys_k[k] = ycost;
                const int ub = ub_of( r );
                const bool need = r < rows && ads < (uint32_t)ub;
                sr = tt[k];
                if( !covered && need && !(colin && ty >= 0 && ty < W) )
                    sr = tesa_sad16<BD>( fl, p_fref + (min_y + r) * rs + mx, rs );
                sr = need ? sr + (uint32_t)fpel : 0xFFFFFFFFu;
            }
            if constexpr( TAB && SPEC )
            {
                sr_k[k] = sr;
                ads_k[k] = ads;
            }
            else
                scan_row( r, ads, sr );
        }
        if constexpr( TAB && SPEC )
        {
            // The row scans do not wait for the running bsad.  A lane staged a cost iff it
            // can pass some row's threshold ((bsad0 - ycost)*17>>4, the speculative pass); a
            // lane that passes that but not the actual (bsad - ycost)*17>>4 has
            // s = SAD + fpel >= ads >= (b*17>>4) >= b (a SAD is at least the sum of its
            // quadrants' |DC difference|, the ads4 value), so it can neither lower bsad nor
            // the min( b, prefix ) an append is tested against.  Every row's prefix minimum
            // is therefore taken over the staged costs up front, and the serial chain per
            // row is the threshold test, the append ballot and a min.
            uint32_t excl_k[CK], rmin_k[CK];
            int yc_k[CK];
#pragma unroll
            for( int k = 0; k < CK; k++ )
            {
                const uint32_t incl = seg_scan_min<SEG>( sr_k[k] );
                uint32_t ex = (uint32_t)__builtin_amdgcn_update_dpp( (int)0xFFFFFFFF, (int)incl, 0x138, 0xF, 0xF, false );
                excl_k[k] = lane ? ex : 0xFFFFFFFFu;
                rmin_k[k] = seg_bcast<SEG>( incl, SEG - 1, bbase );
                yc_k[k] = ys_k[k];
            }
#pragma unroll
            for( int k = 0; k < CK; k++ )
            {
                const int r = CK * c + k;
                if( r >= NR )
                    break;
                const int my = min_y + r;
                const int ycost = yc_k[k];
                const bool rowok = r < rows && bsad > ycost;
                const int b = bsad - ycost;
                const bool pass = rowok && ads_k[k] < (uint32_t)(b * 17 >> 4);
                const int bcur = (int)min( (uint32_t)b, excl_k[k] );
                // costs < 2^20: a 24-bit multiply (v_mul_lo_u32 is quarter rate)
                const bool app = pass && (int)sr_k[k] < (__mul24( bcur, sad_thresh0 ) >> 3);
                const uint64_t m = sball( app );
                if( app )
                    mvsads[nmvsad + rank( m )] = ent( sr_k[k] + (uint32_t)ycost, mx, my );
                nmvsad += __popcll( m );
                if( rmin_k[k] != 0xFFFFFFFFu )
                    bsad = min( bsad, (int)rmin_k[k] + ycost );
            }
        }
        __builtin_amdgcn_sched_barrier( 0 );
        if( c + 1 < NC )
        {
#pragma unroll
            for( int k = 0; k < CK; k++ )
            {
                ip[st][k] = n0[k];
                tt[k] = nt[k];
            }
        }
    }

    // keep the best few (me.c:705-746)
    const int limit = me_range >> 1;
    int thr = bsad * sad_thresh0 >> 3;
    for( ;; )
    {
        const bool need = nmvsad > limit * 2 && thr > bsad;
        if( !any( need ) )
            break;
        if( need )
            thr = (thr + bsad) >> 1;
        int k = 0;
        for( int base = 0; any( need && base < nmvsad ); base += SEG )
        {
            const int j = base + lane;
            const bool in = need && j < nmvsad;
            const E e = in ? mvsads[j] : (E)0;
            const bool keep = in && (int)ecost( e ) <= thr;
            const uint64_t m = sball( keep );
            if( keep )
                mvsads[k + rank( m )] = e;
            k += __popcll( m );
        }
        if( need )
            nmvsad = k;
    }
    for( ;; )
    {
        const bool need = nmvsad > limit;
        if( !any( need ) )
            break;
        // first index of the largest sad: max of (sad << 32 | ~index)
        int bi;
        if constexpr( SEG == 32 )
        {
            // 32-bit keys (cost < 2^21, index < 2^11: the list holds <= 33 x 32 entries): the
            // segment's maximum as the DPP prefix minimum of the complements
            uint32_t nk = 0xFFFFFFFFu;
            for( int j = lane; any( need && j < nmvsad ); j += SEG )
                if( need && j < nmvsad )
                    nk = min( nk, ~((ecost( mvsads[j] ) << 11) | (2047u - (uint32_t)j)) );
            const uint32_t km = ~seg_lane<SEG>( seg_scan_min<SEG>( nk ), SEG - 1, sg );
            bi = 2047 - (int)(km & 2047u);
        }
        else
        {
            uint64_t key = 0;
            for( int j = lane; any( need && j < nmvsad ); j += SEG )
            {
                if( need && j < nmvsad )
                {
                    const uint64_t k = ((uint64_t)ecost( mvsads[j] ) << 32) | (uint32_t)~j;
                    key = k > key ? k : key;
                }
            }
#pragma unroll
            for( int off = SEG / 2; off >= 1; off >>= 1 )
            {
                const uint64_t o = ((uint64_t)(uint32_t)__shfl_xor( (int)(key >> 32), off ) << 32) |
                                   (uint32_t)__shfl_xor( (int)(uint32_t)key, off );
                key = o > key ? o : key;
            }
            bi = (int)~(uint32_t)key;
        }
        if( need )
        {
            nmvsad--;
            if( lane == 0 )
                mvsads[bi] = mvsads[nmvsad];
        }
        tesa_wave_sync();
    }

    // COST_MV over the survivors in list order: eight 8x4 units per candidate
    uint32_t best = 0xFFFFFFFFu;
    for( int u0 = 0; any( u0 < nmvsad * 8 ); u0 += SEG )
    {
        const int u = u0 + lane, k = u >> 3, part = u & 7;
        uint32_t v = 0;
        int cmx = 0, cmy = 0;
        if( k < nmvsad )
        {
            const E e = mvsads[k];
            cmx = emx( e );
            cmy = emy( e );
            const int bx = 8 * (part & 1), by = 4 * (part >> 1);
            constexpr int HDW = 8 / PT<BD>::PPD;
            uint32_t a[4][HDW], rr[4][HDW];
            const pixel *rp = p_fref + (intptr_t)(cmy + by) * rs + cmx + bx;
#pragma unroll
            for( int y = 0; y < 4; y++ )
            {
                load_row_u<HDW>( rp + y * rs, rr[y] );
#pragma unroll
                for( int j = 0; j < HDW; j++ )
                    a[y][j] = fl[(by + y) * NDW + bx / PT<BD>::PPD + j];
            }
            if( satd )
                v = satd8x4_packed<BD>( a, rr ) >> 1;
            else
            {
#pragma unroll
                for( int y = 0; y < 4; y++ )
#pragma unroll
                    for( int j = 0; j < HDW; j++ )
                        v = sadp<BD>( a[y][j], rr[y][j], v );
            }
        }
        // the eight units of a candidate (lanes 8k .. 8k+7): quad sums by quad_perm, then
        // row_ror:12 brings lane 8k+4's quad sum to lane 8k
        v += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)v, 0xB1, 0xF, 0xF, false );
        v += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)v, 0x4E, 0xF, 0xF, false );
        v += (uint32_t)__builtin_amdgcn_update_dpp( 0, (int)v, 0x12C, 0xF, 0xF, false );
        if( k < nmvsad && part == 0 )
        {
            const uint32_t cost = v + cx[cmx * 4] + cy[cmy * 4];
            best = min( best, (cost << 6) | (uint32_t)k );   // k < 64: first index on ties
        }
    }
    best = seg_lane<SEG>( seg_scan_min<SEG>( best ), SEG - 1, sg );
    if( lane == 0 && live && mbo < nmb )
    {
        int32_t bcost = init_cost[mb], rx = bmx0, ry = bmy0;
        if( best != 0xFFFFFFFFu && (int32_t)(best >> 6) < bcost )
        {
            const E e = mvsads[best & 63];
            bcost = (int32_t)(best >> 6);
            rx = emx( e );
            ry = emy( e );
        }
        out[4 * mb] = bcost;
        out[4 * mb + 1] = rx;
        out[4 * mb + 2] = ry;
        out[4 * mb + 3] = nmvsad;
    }
}

template <int BD, int NR, int SEG, bool TAB, bool SPEC = false>
__global__ __launch_bounds__( 64 ) __attribute__( ( amdgpu_waves_per_eu( TESA_WPE ) ) ) void me_tesa_kernel( const typename PT<BD>::pixel *__restrict__ fenc, intptr_t fs,
                                                        intptr_t ffs, const typename PT<BD>::pixel *__restrict__ ref,
                                                        intptr_t rs, intptr_t rfs,
                                                        const uint16_t *__restrict__ integral, intptr_t ifs, int mbw,
                                                        int mbh, int nmb, int me_range, int satd,
                                                        const typename PT<BD>::sadt *__restrict__ table, int R,
                                                        int tcols, int tpitch, const int16_t *__restrict__ origin,
                                                        const int16_t *__restrict__ par,
                                                        const int32_t *__restrict__ init_cost,
                                                        const uint16_t *__restrict__ cost_mv, int32_t *__restrict__ out,
                                                        int cap )
{
    constexpr int NDW = 16 / PT<BD>::PPD;
    constexpr int NSEG = 64 / SEG;
    extern __shared__ uint64_t tesa_lds[];
    __shared__ uint32_t fls[NSEG][16 * NDW];
    const int sg = (int)threadIdx.x / SEG, lane = (int)threadIdx.x % SEG;
    const int64_t mbo = (int64_t)blockIdx.x * NSEG + sg;      // this segment's MB
    const int64_t mb = mbo < nmb ? mbo : nmb - 1;
    const int ox = origin ? origin[2 * mb] : -R, oy = origin ? origin[2 * mb + 1] : -R;
    tesa_scan_mb<BD, NR, SEG, TAB, SPEC>( fenc, fs, ffs, ref, rs, rfs, integral, ifs, mbw, mbh, nmb, me_range, satd,
                                          table, R, tcols, tpitch, ox, oy, par, init_cost, cost_mv, out, mbo, true, sg,
                                          lane, (tesa_ent<SEG> *)tesa_lds + (int64_t)sg * cap, fls[sg] );
}

// the predictor pairs (par[8*mb], par[8*mb+1]) as me_window's centre array
__global__ __launch_bounds__( 256 ) void tesa_centre_kernel( int nmb, const int16_t *__restrict__ par,
                                                             int16_t *__restrict__ centre )
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if( i < nmb )
    {
        centre[2 * i] = par[8 * i];
        centre[2 * i + 1] = par[8 * i + 1];
    }
}

// stream-ordered scratch (the self-contained TESA, the weight search) from a memory pool the library owns,
// one per device (the device of the launch stream), created with an unbounded release
// threshold so a repeated call re-uses its blocks instead of mapping fresh pages; the
// application's default pool is left alone.  x264hip_trim() returns the pool's idle blocks.
static std::mutex g_pool_mu;
static hipMemPool_t g_pools[64] = {};
hipError_t scratch_alloc( void **p, size_t bytes, hipStream_t stream )
{
    int dev = 0;
    hipError_t e = stream_device( stream, &dev );
    if( e != hipSuccess )
        return e;
    if( dev < 0 || dev >= 64 )
        return hipErrorInvalidDevice;
    hipMemPool_t pool;
    {
        std::lock_guard<std::mutex> lk( g_pool_mu );
        if( !g_pools[dev] )
        {
            hipMemPoolProps props;
            memset( &props, 0, sizeof( props ) );
            props.allocType = hipMemAllocationTypePinned;
            props.handleTypes = hipMemHandleTypeNone;
            props.location.type = hipMemLocationTypeDevice;
            props.location.id = dev;
            if( (e = hipMemPoolCreate( &g_pools[dev], &props )) != hipSuccess )
            {
                g_pools[dev] = nullptr;
                return e;
            }
            uint64_t thr = UINT64_MAX;
            (void)hipMemPoolSetAttribute( g_pools[dev], hipMemPoolAttrReleaseThreshold, &thr );
        }
        pool = g_pools[dev];
    }
    return hipMallocFromPoolAsync( p, bytes, pool, stream );
}

// release the scratch pool's unused blocks of `dev` (all devices for dev < 0)
hipError_t scratch_trim( int dev )
{
    std::lock_guard<std::mutex> lk( g_pool_mu );
    for( int d = 0; d < 64; d++ )
        if( g_pools[d] && (dev < 0 || dev == d) )
        {
            const hipError_t e = hipMemPoolTrimTo( g_pools[d], 0 );
            if( e != hipSuccess )
                return e;
        }
    return hipSuccess;
}

template <int BD>
hipError_t launch_me_tesa( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                           const typename PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs, const uint16_t *integral,
                           intptr_t ifs, int mbw, int mbh, int nframes, int me_range, int satd,
                           const typename PT<BD>::sadt *table, int R, const int16_t *origin, const int16_t *par,
                           const int32_t *init_cost, const uint16_t *cost_mv, int32_t *out, hipStream_t stream )
{
    const int64_t nmb = (int64_t)nframes * mbw * mbh;
    if( nmb <= 0 )
        return hipSuccess;
    // (the scan addresses rows by 24-bit products: strides below 2^18 elements)
    if( me_range < 1 || me_range > 32 || nmb > 0x7fffffff || rs <= 0 || rs >= (1 << 18) )
        return hipErrorInvalidValue;
    // (X264HIP_TESA_VARIANT=1 forces the in-scan SADs -- the me_range > 24 kernel -- at any
    // range: a test hook for that path)
    if( !table && me_range <= 24 && variant( V_TESA ) != 1 )
    {
        // Self-contained call: the ads-filtered SADs cost a lane 16 unaligned row loads
        // each, so the kernel is address-path bound (2.6 ms per 16 1080p frames).  Every
        // window SAD from the full-search kernel around the predictors (0.3 ms) and the
        // table-reading scan give the same decisions in ~1 ms.  The table is the centred
        // (ESA-window) geometry, so every candidate the scan can reach is a read.  (The
        // in-kernel SADs remain for me_range > 24 and when no scratch can be had.)
        using sadt = typename PT<BD>::sadt;
        const int TR = me_range <= 4 ? 4 : me_range <= 8 ? 8 : me_range <= 16 ? 16 : 24;
        const size_t tab = (size_t)nmb * (2 * TR + 1) * (size_t)cen_pitch( BD, TR ) * sizeof( sadt );
        const size_t bytes = tab + (size_t)nmb * 8;
        void *buf = nullptr;
        if( scratch_alloc( &buf, bytes, stream ) == hipSuccess )
        {
            sadt *ttab = (sadt *)buf;
            int16_t *cen = (int16_t *)((uint8_t *)buf + tab), *org = cen + 2 * nmb;
            hipLaunchKernelGGL( tesa_centre_kernel, dim3( (unsigned)((nmb + 255) / 256) ), dim3( 256 ), 0, stream,
                                (int)nmb, par, cen );
            hipError_t e = hipGetLastError();
            if( e == hipSuccess )
            {
                if constexpr( BD == 8 )
                {
                    // 8 bit: the fused ESA's lanes (9 column groups at TR 16, the window's extra
                    // group only where it reaches past them) write the table: 40 -> 36 columns of
                    // work per MB against launch_me_full's whole centred template (round 4's
                    // wider template, 36 -> 40 columns, was TESA's 0.58 -> 0.62 ms)
                    switch( TR )
                    {
#define TT_CASE( RR )                                                                                             \
                        case RR:                                                                                  \
                            hipLaunchKernelGGL( ( me_full_esa_v7_kernel<RR, true> ),                              \
                                                dim3( (unsigned)((nmb + esa7_mbs<RR>() - 1) / esa7_mbs<RR>()) ),  \
                                                dim3( 256 ), 0, stream, fenc, fs, ffs, ref, rs, rfs, mbw, mbh,    \
                                                nframes, me_range, par, cost_mv, nullptr, me_xcd(), ttab, org,    \
                                                nullptr );                                                        \
                            break;
                        TT_CASE( 4 ) TT_CASE( 8 ) TT_CASE( 16 ) TT_CASE( 24 )
#undef TT_CASE
                    }
                    e = hipGetLastError();
                }
                else
                    e = launch_me_full<BD>( fenc, fs, ffs, ref, rs, rfs, mbw, mbh, nframes, TR, ttab, cen, org, stream );
            }
            if( e == hipSuccess )
                e = launch_me_tesa<BD>( fenc, fs, ffs, ref, rs, rfs, integral, ifs, mbw, mbh, nframes, me_range, satd,
                                        ttab, TR, org, par, init_cost, cost_mv, out, stream );
            const hipError_t f = hipFreeAsync( buf, stream );
            return e != hipSuccess ? e : f;
        }
        (void)hipGetLastError();                            // no scratch: the in-kernel SADs below
    }

    // the mvsads list: at most (2*me_range+1) rows x (2*me_range+3)&~3 columns per MB
    const int cap = (2 * me_range + 1) * ((2 * me_range + 3) & ~3);
    // table geometry: centred (an origin given) or full
    const int tcols = origin ? cen_cols( BD, R ) : 2 * R + 1;
    const int tpitch = origin ? cen_pitch( BD, R ) : full_pitch( R );
    if( table && (R < 1 || tpitch > 64) )
        return hipErrorInvalidValue;
    // with a table the speculative row scans (SPEC: every row's prefix minimum taken over the
    // staged costs up front), without one the SADs computed in the scan
#define TESA_GO( NR, SEG, T )                                                                                    \
    hipLaunchKernelGGL( ( me_tesa_kernel<BD, NR, SEG, T, T> ), dim3( (unsigned)((nmb + 64 / SEG - 1) / (64 / SEG)) ), \
                        dim3( 64 ), (64 / SEG) * (size_t)cap * (SEG == 32 ? 4 : 8), stream, fenc, fs, ffs, ref, rs, \
                        rfs, integral, ifs, mbw, mbh, (int)nmb, me_range, satd, table, R, tcols, tpitch, origin, par, \
                        init_cost, cost_mv, out, cap )
    if( me_range <= 16 )
    {
        if( table ) { TESA_GO( 33, 32, true ); } else { TESA_GO( 33, 32, false ); }
    }
    else
    {
        if( table ) { TESA_GO( 65, 64, true ); } else { TESA_GO( 65, 64, false ); }
    }
#undef TESA_GO
    return hipGetLastError();
}

template hipError_t launch_me_tesa<8>( const uint8_t *, intptr_t, intptr_t, const uint8_t *, intptr_t, intptr_t,
                                       const uint16_t *, intptr_t, int, int, int, int, int, const uint16_t *, int,
                                       const int16_t *, const int16_t *, const int32_t *, const uint16_t *, int32_t *,
                                       hipStream_t );
template hipError_t launch_me_tesa<10>( const uint16_t *, intptr_t, intptr_t, const uint16_t *, intptr_t, intptr_t,
                                        const uint16_t *, intptr_t, int, int, int, int, int, const uint32_t *, int,
                                        const int16_t *, const int16_t *, const int32_t *, const uint16_t *,
                                        int32_t *, hipStream_t );

// ---------------------------------------------------------------------------
// Sub-partition ESA decisions (x264hip_*_me_search_esa8): x264's ESA (encoder/me.c:618-631)
// for an MB's eight sub-partitions -- PIXEL_16x8 top / bottom, 8x16 left / right, 8x8 TL, TR,
// BL, BR (analyse.c:1425,1480,1546) -- each with its own window, mvp and predictor cost.  A
// partition's SAD is the sum of the MB's 8x8 quadrant SADs at the same mv, so one pass of
// absdiffs over a template serves all eight.
//
// Pass 1 (8 bit, me_esa8_kernel): the template of radius R around a per-MB centre -- 2R+1 rows
// and 2R columns from (cx - R, cy - R) itself, which is an unclipped window's whole width-rounded
// extent ((2R+3) & ~3 = 2R, me.c:626), so no alignment slack is computed (the origin is not
// dword aligned then, and the row loads take the address path's misaligned form) -- in R/2
// four-column groups, each split over a lane PAIR: lane
// h = 0 folds fenc rows 0-7 and h = 1 rows 8-15 (2R+8 ref rows each, 8 candidate rows in flight,
// left and right 8-column accumulators).  When a candidate row's sums finish, both lanes of the
// pair hold their two quadrants and swap one of them over DPP, so each lane keys exactly four
// partitions with the same instructions (slot 0 its left quadrant, 1 its right one, 2 their sum
// = its 16x8 half, 3 its quadrant column's 8x16 = own quadrant + the partner's): h = 0 keys
// 8x8 TL, TR, 16x8 top, 8x16 left; h = 1 8x8 BL, BR, 16x8 bottom, 8x16 right.  Keys are
// me_esa_argmin's (cost << 12 | raster index in the partition's window): v_mad_u32_u16 of the
// packed sum's half with the column term, min over the row's four columns, then the row term's
// saturating add (sat(min_k(x_k) + S) = min_k(sat(x_k + S))).  An MB's lanes meet in LDS; one
// lane per partition then applies the strict-< update from the predictor cost when the
// partition's whole window lies in the template.
// The direct pass (esa8_direct, any bit depth): the same workgroup then gives each partition
// whose window leaves the template -- centred elsewhere than its MB (x264 starts each partition
// from its own best predictor) or clipped past it -- one wave that scores the window's
// candidates outside the template with direct SADs and merges them into the template key; at
// range 0 me_esa8_direct_kernel scores every partition that way.  So the decisions are me.c's
// for any inputs; the template only decides how much is shared.  10 bit runs the same passes on
// me_row5q's column-pair lanes (R + 1 pairs from the dword-aligned origin).
__host__ __device__ constexpr int esa8_part( int h, int s ) { return s == 0 ? 4 + 2 * h : s == 1 ? 5 + 2 * h : s == 2 ? h : 2 + h; }
// 2R template columns: an unclipped window's (2R+3) & ~3 = 2R columns exactly
template <int R> constexpr int esa8_groups() { return R / 2; }
// 10 bit: column-PAIR groups (me_row5q's lane, two columns from 9 dwords a row), R + 1 of them
// from the origin aligned down to a dword (2R + 2 columns)
template <int BD, int R> constexpr int esa8_lgroups() { return BD == 8 ? esa8_groups<R>() : R + 1; }
template <int BD, int R> constexpr int esa8_mbs() { return 256 / (2 * esa8_lgroups<BD, R>()); }

// me_window's template origin with run-time R and P (the same arithmetic)
__device__ __forceinline__ void esa8_window( int R, int P, int cx, int cy, int mbx, int mby, int mbw, int mbh, int &ox,
                                             int &oy, int al = 0 )
{
    int ax = 16 * mbx - R + cx, ay = 16 * mby - R + cy;
    ax = min( max( ax, -32 ), 16 * mbw + 12 - P );
    ay = min( max( ay, -32 ), 16 * mbh + 16 - 2 * R );
    ax &= ~al;
    ox = ax - 16 * mbx;
    oy = ay - 16 * mby;
}

__device__ __forceinline__ uint32_t esa8_mad( uint32_t v, uint32_t c, uint32_t s4096, bool hi )
{
    uint32_t d;
    if( hi )
        asm( "v_mad_u32_u16 %0, %1, %2, %3 op_sel:[1,0,0,0]" : "=v"( d ) : "v"( v ), "s"( s4096 ), "v"( c ) );
    else
        asm( "v_mad_u32_u16 %0, %1, %2, %3" : "=v"( d ) : "v"( v ), "s"( s4096 ), "v"( c ) );
    return d;
}

// rbase: the dword holding the lane's first window byte, sh: that byte's offset in it.  Each row
// is six aligned dwords (the 20 bytes the lane's windows span, at any offset) realigned with
// v_alignbyte: a misaligned 16-byte load costs the address path 4x an aligned one
// (profiles/r01d_ta_probe.txt), which made the template pass address-bound off the dword grid.
template <int R, int L, int Y, class Sink>
__device__ __forceinline__ void me_row_e8( const uint32_t *__restrict__ rbase, int rs_dw, uint32_t sh,
                                           const uint32_t (&F)[8][4], uint64_t (&al)[8], uint64_t (&ar)[8],
                                           Sink &sink, u32x4a4 (&wl)[L], u32x2a4 (&wh)[L] )
{
    constexpr int C0 = Y - 7 > 0 ? Y - 7 : 0;
    constexpr int C1 = Y < 2 * R ? Y : 2 * R;
    const u32x4a4 l4 = wl[Y % L];
    const u32x2a4 h2 = wh[Y % L];
    const uint32_t d0 = __builtin_amdgcn_alignbyte( l4.y, l4.x, sh ), d1 = __builtin_amdgcn_alignbyte( l4.z, l4.y, sh );
    const uint32_t d2 = __builtin_amdgcn_alignbyte( l4.w, l4.z, sh ), d3 = __builtin_amdgcn_alignbyte( h2.x, l4.w, sh );
    const uint32_t d4 = __builtin_amdgcn_alignbyte( h2.y, h2.x, sh );
    const uint64_t win[4] = { (uint64_t)d1 << 32 | d0, (uint64_t)d2 << 32 | d1, (uint64_t)d3 << 32 | d2,
                              (uint64_t)d4 << 32 | d3 };
    if constexpr( Y + L < 2 * R + 8 )
    {
        const uint32_t *row = rbase + (Y + L) * rs_dw;
        wl[Y % L] = *(const u32x4a4 *)row;
        wh[Y % L] = *(const u32x2a4 *)(row + 4);
    }
#pragma unroll
    for( int c = C0; c <= C1; c++ )
    {
        const int r = Y - c;
        uint64_t a = r == 0 ? 0ull : al[c & 7], b = r == 0 ? 0ull : ar[c & 7];
        a = __builtin_amdgcn_qsad_pk_u16_u8( win[0], F[r][0], a );
        a = __builtin_amdgcn_qsad_pk_u16_u8( win[1], F[r][1], a );
        b = __builtin_amdgcn_qsad_pk_u16_u8( win[2], F[r][2], b );
        b = __builtin_amdgcn_qsad_pk_u16_u8( win[3], F[r][3], b );
        if( r == 7 )
            sink( c, a, b );
        else
        {
            al[c & 7] = a;
            ar[c & 7] = b;
        }
    }
    __builtin_amdgcn_sched_barrier( 0 );
}

template <int R, int L, class Sink, int... Ys>
__device__ __forceinline__ void me_rows_e8( const uint32_t *__restrict__ rbase, int rs_dw, uint32_t sh,
                                            const uint32_t (&F)[8][4], uint64_t (&al)[8], uint64_t (&ar)[8],
                                            Sink &sink, std::integer_sequence<int, Ys...> )
{
    u32x4a4 wl[L];
    u32x2a4 wh[L];
#pragma unroll
    for( int k = 0; k < L; k++ )
    {
        wl[k] = *(const u32x4a4 *)(rbase + k * rs_dw);
        wh[k] = *(const u32x2a4 *)(rbase + k * rs_dw + 4);
    }
    ( me_row_e8<R, L, Ys>( rbase, rs_dw, sh, F, al, ar, sink, wl, wh ), ... );
}

typedef uint16_t u16x2 __attribute__( ( ext_vector_type( 2 ) ) );
__device__ __forceinline__ uint64_t pk_add_u16x4( uint64_t a, uint64_t b )
{
    const u16x2 lo = __builtin_bit_cast( u16x2, (uint32_t)a ) + __builtin_bit_cast( u16x2, (uint32_t)b );
    const u16x2 hi = __builtin_bit_cast( u16x2, (uint32_t)(a >> 32) ) + __builtin_bit_cast( u16x2, (uint32_t)(b >> 32) );
    return ((uint64_t)__builtin_bit_cast( uint32_t, hi ) << 32) | __builtin_bit_cast( uint32_t, lo );
}

// The direct scan of one partition's uncovered candidates: the fenc block (NDW dwords x PH rows,
// dword aligned) held in registers for the whole scan, each candidate's ref rows (anywhere) CH at
// a time realigned from aligned loads.  Returns the lane's least key.
template <int BD, int NDW, int PH, int CH>
__device__ __forceinline__ uint32_t esa8_scan( const typename PT<BD>::pixel *fb, intptr_t fs,
                                               const typename PT<BD>::pixel *rb, intptr_t rs, const uint16_t *cx,
                                               const uint16_t *cy, int lane, int nt, int nb, int nl, int nr, int wd,
                                               int lw, int rw, int x0, int y0, int iy0, int iy1, int ix1, int min_x,
                                               int min_y, int width, uint32_t key )
{
    uint32_t a[PH][NDW];
#pragma unroll
    for( int y = 0; y < PH; y++ )
#pragma unroll
        for( int k = 0; k < NDW; k++ )
            a[y][k] = ((const uint32_t *)(fb + y * fs))[k];
    const int nc = nt + nb + nl + nr;
    for( int u = lane; u < nc; u += 64 )
    {
        int mx, my, v = u;
        if( v < nt )
            my = y0 + v / wd, mx = x0 + v % wd;
        else if( (v -= nt) < nb )
            my = iy1 + 1 + v / wd, mx = x0 + v % wd;
        else if( (v -= nb) < nl )
            my = iy0 + v / lw, mx = x0 + v % lw;
        else
            v -= nl, my = iy0 + v / rw, mx = ix1 + 1 + v % rw;
        const typename PT<BD>::pixel *r = rb + (intptr_t)my * rs + mx;
        uint32_t sad = 0;
#pragma unroll
        for( int y0r = 0; y0r < PH; y0r += CH )
        {
            uint32_t b[CH][NDW];
#pragma unroll
            for( int y = 0; y < CH; y++ )
                load_packed<NDW>( r + (y0r + y) * rs, b[y] );
#pragma unroll
            for( int y = 0; y < CH; y++ )
#pragma unroll
                for( int k = 0; k < NDW; k++ )
                    sad = sadp<BD>( a[y0r + y][k], b[y][k], sad );
        }
        const uint32_t idx = (uint32_t)((my - min_y) * width + mx - min_x);
        key = min( key, ((sad + cx[4 * mx] + cy[4 * my]) << 12) | idx );
    }
    return key;
}

// 8 bit: the uncovered candidates in runs of four columns from min_x (the width-rounded window is
// a whole number of runs): per fenc row one v_qsad_pk_u16_u8 per fenc dword scores the run's four
// candidates from realigned ref dwords, against one v_sad_u8 chain per candidate above; a run that
// also holds covered columns scores them again (the same keys: min is idempotent).  Top / bottom
// bands are whole rows of runs, the rows between them the runs holding the left / right parts.
template <int NDW, int PH>
__device__ __forceinline__ uint32_t esa8_scan4( const uint8_t *fb, intptr_t fs, const uint8_t *rb, intptr_t rs,
                                                const uint16_t *cx, const uint16_t *cy, int lane, int y0, int y1,
                                                int iy0, int iy1, int ix0, int ix1, int x0, int width, int min_x,
                                                int min_y, uint32_t key )
{
    uint32_t a[PH][NDW];
#pragma unroll
    for( int y = 0; y < PH; y++ )
#pragma unroll
        for( int k = 0; k < NDW; k++ )
            a[y][k] = ((const uint32_t *)(fb + y * fs))[k];
    if( width <= 0 || y1 < y0 )
        return key;
    const int x1 = x0 + width - 1, ng = width >> 2;
    const int gl = (ix0 - x0 + 3) >> 2, gr0 = (ix1 + 1 - x0) >> 2, gr = ix1 + 1 <= x1 ? ng - gr0 : 0;
    const int mh = iy1 - iy0 + 1;
    const int nt = (iy0 - y0) * ng, nb = (y1 - iy1) * ng, nl = mh * gl, nr = mh * gr;
    const int nu = nt + nb + nl + nr;
    for( int u = lane; u < nu; u += 64 )
    {
        int my, g, v = u;
        if( v < nt )
            my = y0 + v / ng, g = v % ng;
        else if( (v -= nt) < nb )
            my = iy1 + 1 + v / ng, g = v % ng;
        else if( (v -= nb) < nl )
            my = iy0 + v / gl, g = v % gl;
        else
            v -= nl, my = iy0 + v / gr, g = gr0 + v % gr;
        const int gx = x0 + 4 * g;
        const uint8_t *r = rb + (intptr_t)my * rs + gx;
        const uint32_t sh = (uint32_t)((uintptr_t)r & 3);
        uint64_t acc = 0;
#pragma unroll
        for( int y = 0; y < PH; y++ )
        {
            const uint32_t *base = (const uint32_t *)(r + y * rs - sh);
            uint32_t w[NDW + 2], d[NDW + 1];
#pragma unroll
            for( int k = 0; k <= NDW; k++ )
                w[k] = base[k];
            w[NDW + 1] = base[sh ? NDW + 1 : NDW];          // (aligned: no byte past the run is read)
#pragma unroll
            for( int k = 0; k <= NDW; k++ )
                d[k] = __builtin_amdgcn_alignbyte( w[k + 1], w[k], sh );
#pragma unroll
            for( int k = 0; k < NDW; k++ )
                acc = __builtin_amdgcn_qsad_pk_u16_u8( (uint64_t)d[k + 1] << 32 | d[k], a[y][k], acc );
        }
        const uint32_t rowc = cy[4 * my], rowi = (uint32_t)((my - min_y) * width + gx - min_x);
#pragma unroll
        for( int k = 0; k < 4; k++ )
        {
            const uint32_t sad = (uint32_t)(acc >> (16 * k)) & 0xffff;
            key = min( key, ((sad + cx[4 * (gx + k)] + rowc) << 12) | (rowi + k) );
        }
    }
    return key;
}

// One wave finishes partition i = 8 mb + p: the candidates of its window outside the template
// [tx0, tx1] x [ty0, ty1] (empty: all of them) by direct SADs, merged into `key` (the template
// pass's, or all ones), then the strict-< update (COPY3_IF_LT, me.h:87-93) into out[3 i].
template <int BD, int CH>
__device__ __forceinline__ void esa8_direct( const typename PT<BD>::pixel *__restrict__ fenc, intptr_t fs,
                                             intptr_t ffs, const typename PT<BD>::pixel *__restrict__ ref,
                                             intptr_t rs, intptr_t rfs, int mbw, int mbh, int me_range,
                                             const int16_t *__restrict__ par, const int32_t *__restrict__ init_cost,
                                             const uint16_t *__restrict__ cost_mv, int32_t *__restrict__ out,
                                             int64_t i, uint32_t key, int tx0, int tx1, int ty0, int ty1, int lane )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int PPD = PT<BD>::PPD;
    const int64_t mb = i >> 3;
    const int p = (int)(i & 7);
    const int64_t t = mb / mbw;
    const int mbx = (int)(mb - t * mbw), mby = (int)(t % mbh);
    const int64_t f = t / mbh;
    const int16_t *q = par + 8 * i;
    const int bmx = q[0], bmy = q[1];
    const int min_x = max( bmx - me_range, (int)q[4] ), min_y = max( bmy - me_range, (int)q[5] );
    const int max_x = min( bmx + me_range, (int)q[6] ), max_y = min( bmy + me_range, (int)q[7] );
    const int width = (max_x - min_x + 3) & ~3;
    const uint16_t *cx = cost_mv - q[2], *cy = cost_mv - q[3];
    // partition geometry: 0-1 16x8, 2-3 8x16, 4-7 8x8
    const int px = p < 2 ? 0 : p < 4 ? 8 * (p - 2) : 8 * ((p - 4) & 1);
    const int py = p < 2 ? 8 * p : p < 4 ? 0 : 8 * ((p - 4) >> 1);
    const int pw = p < 2 ? 16 : 8, ph = p >= 2 && p < 4 ? 16 : 8;
    const pixel *fb = fenc + f * ffs + (intptr_t)(16 * mby + py) * fs + 16 * mbx + px;
    const pixel *rb = ref + f * rfs + (intptr_t)(16 * mby + py) * rs + 16 * mbx + px;
    // the window [x0, x1] x [y0, y1] minus its intersection with the template: a top band
    // and a bottom band of whole rows, then the left and right parts of the rows between
    // them; every lane takes candidates of that list (none of the window's covered ones)
    const int x0 = min_x, x1 = min_x + width - 1, y0 = min_y, y1 = max_y;
    int ix0 = max( x0, tx0 ), ix1 = min( x1, tx1 ), iy0 = max( y0, ty0 ), iy1 = min( y1, ty1 );
    if( ix0 > ix1 || iy0 > iy1 )
    {
        iy0 = y1 + 1;           // no intersection: the whole window is the top band
        iy1 = y1;
        ix0 = x0;
        ix1 = x0 - 1;
    }
    const int wd = width > 0 ? width : 1;
    const int nt = width > 0 && y1 >= y0 ? (iy0 - y0) * width : 0, nb = (y1 - iy1) * width;
    const int mh = iy1 - iy0 + 1, lw = ix0 - x0, rw = x1 - ix1;
    const int nl = mh * lw, nr = mh * rw;
    if constexpr( BD == 8 )
    {
        if( pw == 16 )
            key = esa8_scan4<4, 8>( fb, fs, rb, rs, cx, cy, lane, y0, y1, iy0, iy1, ix0, ix1, x0, width, min_x, min_y,
                                    key );
        else if( ph == 16 )
            key = esa8_scan4<2, 16>( fb, fs, rb, rs, cx, cy, lane, y0, y1, iy0, iy1, ix0, ix1, x0, width, min_x, min_y,
                                     key );
        else
            key = esa8_scan4<2, 8>( fb, fs, rb, rs, cx, cy, lane, y0, y1, iy0, iy1, ix0, ix1, x0, width, min_x, min_y,
                                    key );
    }
    else if( pw == 16 )
        key = esa8_scan<BD, 16 / PPD, 8, CH < 8 ? CH : 8>( fb, fs, rb, rs, cx, cy, lane, nt, nb, nl, nr, wd, lw, rw, x0,
                                                          y0, iy0, iy1, ix1, min_x, min_y, width, key );
    else if( ph == 16 )
        key = esa8_scan<BD, 8 / PPD, 16, CH>( fb, fs, rb, rs, cx, cy, lane, nt, nb, nl, nr, wd, lw, rw, x0, y0, iy0,
                                              iy1, ix1, min_x, min_y, width, key );
    else
        key = esa8_scan<BD, 8 / PPD, 8, CH < 8 ? CH : 8>( fb, fs, rb, rs, cx, cy, lane, nt, nb, nl, nr, wd, lw, rw, x0,
                                                         y0, iy0, iy1, ix1, min_x, min_y, width, key );
#pragma unroll
    for( int off = 32; off >= 1; off >>= 1 )
        key = min( key, (uint32_t)__shfl_xor( (int)key, off, 64 ) );
    if( lane == 0 )
    {
        int32_t bc = init_cost[i], rx = bmx, ry = bmy;
        if( key != 0xFFFFFFFFu && (int32_t)(key >> 12) < bc )
        {
            const int ki = (int)(key & 4095);
            bc = (int32_t)(key >> 12);
            ry = min_y + ki / width;
            rx = min_x + ki % width;
        }
        out[3 * i] = bc;
        out[3 * i + 1] = rx;
        out[3 * i + 2] = ry;
    }
}

template <int BD, int R>
__global__ __launch_bounds__( 256 ) void me_esa8_kernel( const typename PT<BD>::pixel *__restrict__ fenc, intptr_t fs,
                                                         intptr_t ffs, const typename PT<BD>::pixel *__restrict__ ref,
                                                         intptr_t rs, intptr_t rfs,
                                                         int mbw, int mbh, int nframes, int me_range,
                                                         const int16_t *__restrict__ centre,
                                                         const int16_t *__restrict__ par,
                                                         const int32_t *__restrict__ init_cost,
                                                         const uint16_t *__restrict__ cost_mv,
                                                         int32_t *__restrict__ out, int xcd )
{
    constexpr int CPG = BD == 8 ? 4 : 2;        // candidate columns per lane
    constexpr int G = esa8_lgroups<BD, R>();    // column groups per MB
    constexpr int P = CPG * G;                  // template columns
    constexpr int W = 2 * R + 1;                // template rows
    constexpr int MPW = esa8_mbs<BD, R>();      // whole MBs per workgroup
    __shared__ __attribute__( ( aligned( 16 ) ) ) uint32_t s_row[MPW * W * 8];   // row terms [mb][c][h*4 + slot]
    __shared__ int4 s_win[MPW * 8];             // { min_x, min_y, max_y, width } per partition
    __shared__ int2 s_mvp[MPW * 8];
    __shared__ int2 s_org[MPW];
    __shared__ uint32_t s_key[MPW * 8];
    __shared__ uint16_t s_flag[MPW * 8];        // partitions left to the direct pass
    __shared__ uint32_t s_nflag;
    const uint32_t nmb = (uint32_t)nframes * (uint32_t)mbh * (uint32_t)mbw;
    const int tid = (int)threadIdx.x;
    const bool spare = tid >= MPW * 2 * G;
    if( tid == 0 )
        s_nflag = 0;
    const uint32_t wg0 = (xcd ? xcd_block( blockIdx.x, gridDim.x ) : blockIdx.x) * MPW;
    const int lmb = spare ? 0 : tid / (2 * G), lane = tid - lmb * 2 * G, grp = lane >> 1, h = lane & 1;
    const uint32_t mbr = wg0 + (uint32_t)lmb;
    const bool live = !spare && mbr < nmb;
    const uint32_t mb32 = min( mbr, nmb - 1 ), t32 = mb32 / (uint32_t)mbw, f32 = t32 / (uint32_t)mbh;
    const int mbx = (int)(mb32 - t32 * (uint32_t)mbw), mby = (int)(t32 - f32 * (uint32_t)mbh);
    const int64_t mb = mb32, f = f32;
    int ox, oy;
    esa8_window( R, P, centre ? centre[2 * mb] : 0, centre ? centre[2 * mb + 1] : 0, mbx, mby, mbw, mbh, ox, oy,
                 BD == 8 ? 0 : 1 );
    // the partitions' windows (the MB's lanes, 2G of them: 6 at R = 4), the template origin,
    // the key slots
    if( !spare )
    {
        for( int j = lane; j < 8; j += 2 * G )
        {
            const int16_t *q = par + 8 * (8 * mb + j);
            const int bmx = q[0], bmy = q[1];
            const int min_x = max( bmx - me_range, (int)q[4] ), min_y = max( bmy - me_range, (int)q[5] );
            const int max_x = min( bmx + me_range, (int)q[6] ), max_y = min( bmy + me_range, (int)q[7] );
            s_win[lmb * 8 + j] = make_int4( min_x, min_y, max_y, (max_x - min_x + 3) & ~3 );
            s_mvp[lmb * 8 + j] = make_int2( q[2], q[3] );
            s_key[lmb * 8 + j] = 0xFFFFFFFFu;
        }
        if( lane == 0 )
            s_org[lmb] = make_int2( ox, oy );
    }
    __syncthreads();
    // row terms S = ycost << 12 | (my - min_y) * width inside [min_y, max_y], all ones outside.
    // Branch-free: the cost is read at the row clamped into the window (mvd 0 for an empty
    // window) and discarded outside it.  NL = 8 k of the MB's lanes take one partition slot each
    // and every (NL / 8)-th row (R >= 8); R = 4's six lanes take the entries in turn.
    auto row_term = [&]( int c, int idx ) __attribute__( ( always_inline ) ) {
        const int p = esa8_part( idx >> 2, idx & 3 ), my = oy + c;
        const int4 w = s_win[lmb * 8 + p];
        const bool in = my >= w.y && my <= w.z;
        const int ci = w.z >= w.y && w.w > 0 ? 4 * min( max( my, w.y ), w.z ) - s_mvp[lmb * 8 + p].y : 0;
        const uint32_t t = ((uint32_t)cost_mv[ci] << 12) + (uint32_t)((my - w.y) * w.w);
        s_row[(lmb * W + c) * 8 + idx] = in ? t : 0xFFFFFFFFu;
    };
    constexpr int NL = (2 * G) / 8 * 8;
    if constexpr( NL >= 8 )
    {
        if( !spare && lane < NL )
            for( int c = lane >> 3; c < W; c += NL / 8 )
                row_term( c, lane & 7 );
    }
    else if( !spare )
        for( int e = lane; e < W * 8; e += 2 * G )
            row_term( e >> 3, e & 7 );
    // column terms C = xcost << 12 | (mx - min_x) inside the window's columns, 0xF0000000 outside
    // (the same clamped, branch-free read)
    uint32_t C[4][CPG];
#pragma unroll
    for( int sl = 0; sl < 4; sl++ )
    {
        const int p = esa8_part( h, sl );
        const int4 w = s_win[lmb * 8 + p];
        const int mvpx = s_mvp[lmb * 8 + p].x;
#pragma unroll
        for( int k = 0; k < CPG; k++ )
        {
            const int mx = ox + CPG * grp + k;
            const bool in = mx >= w.x && mx < w.x + w.w;
            const int ci = w.w > 0 ? 4 * min( max( mx, w.x ), w.x + w.w - 1 ) - mvpx : 0;
            const uint32_t t = ((uint32_t)cost_mv[ci] << 12) + (uint32_t)(mx - w.x);
            C[sl][k] = in ? t : 0xF0000000u;
        }
    }
    __syncthreads();
    uint32_t key[4] = { 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu };
    if( !spare )
    {
      if constexpr( BD == 8 )
      {
        uint32_t F[8][4];
        const uint32_t *fe = (const uint32_t *)(fenc + f * ffs + (intptr_t)(16 * mby + 8 * h) * fs + 16 * mbx);
        const int fs_dw = (int)(fs / 4);
#pragma unroll
        for( int r = 0; r < 8; r++ )
#pragma unroll
            for( int k = 0; k < 4; k++ )
                F[r][k] = fe[r * fs_dw + k];
        // (the window's first byte: 16 mbx + ox + 4 grp; its dword and offset, 16 mbx being a multiple of 4)
        const uint32_t *rbase = (const uint32_t *)(ref + f * rfs + (intptr_t)(16 * mby + 8 * h + oy) * rs + 16 * mbx +
                                                   (ox & ~3)) + grp;
        const uint32_t sh = (uint32_t)ox & 3;
        const uint32_t s4096 = 4096u;
        __attribute__( ( address_space( 3 ) ) ) uint32_t *srow =
            (__attribute__( ( address_space( 3 ) ) ) uint32_t *)(s_row + lmb * W * 8 + 4 * h);
        auto fold = [&]( uint64_t v, const uint32_t (&c)[4], uint32_t S, uint32_t &k ) __attribute__( ( always_inline ) ) {
            const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
            // (v_mad_u32_u16 with op_sel picks the 16-bit half: one instruction per candidate;
            // an extract + v_lshl_add_u32 ran 0.489 -> 0.515 ms, profiles/r06x_esa8_fold_ab.log)
            const uint32_t k0 = esa8_mad( lo, c[0], s4096, false ), k1 = esa8_mad( lo, c[1], s4096, true );
            const uint32_t k2 = esa8_mad( hi, c[2], s4096, false ), k3 = esa8_mad( hi, c[3], s4096, true );
            const uint32_t m = min( min( min( k0, k1 ), k2 ), k3 );
            k = min( k, __builtin_elementwise_add_sat( m, S ) );
        };
        auto sink = [&]( int c, uint64_t a, uint64_t b ) {
            __attribute__( ( address_space( 3 ) ) ) uint32_t *q = srow;
            asm volatile( "" : "+v"( q ) );     // read where the row finishes
            typedef uint32_t u32x4 __attribute__( ( ext_vector_type( 4 ) ) );
            const u32x4 S = *(__attribute__( ( address_space( 3 ) ) ) const u32x4 *)(q + c * 8);
            // h = 0 sends its right quadrant (TR) and receives BL; h = 1 sends BL, receives TR
            // (a lane-dependent window order instead of these selects cost more address
            // arithmetic than the selects: 0.492 -> 0.522 ms per 16 1080p pairs)
            const uint64_t send = h ? a : b, mine = h ? b : a;
            const uint32_t r0 = (uint32_t)__builtin_amdgcn_mov_dpp( (int)(uint32_t)send, 0xB1, 0xF, 0xF, false );
            const uint32_t r1 = (uint32_t)__builtin_amdgcn_mov_dpp( (int)(uint32_t)(send >> 32), 0xB1, 0xF, 0xF, false );
            const uint64_t recv = ((uint64_t)r1 << 32) | r0;
            fold( a, C[0], S.x, key[0] );
            fold( b, C[1], S.y, key[1] );
            fold( pk_add_u16x4( a, b ), C[2], S.z, key[2] );
            fold( pk_add_u16x4( mine, recv ), C[3], S.w, key[3] );
            asm volatile( "" : "+v"( key[0] ), "+v"( key[1] ), "+v"( key[2] ), "+v"( key[3] ) );
        };
        uint64_t al[8], ar[8];
        me_rows_e8<R, ME_LEAD>( rbase, (int)(rs / 4), sh, F, al, ar, sink, std::make_integer_sequence<int, 2 * R + 8>{} );
      }
      else
      {
        // 10 bit: me_row5q's lane (fenc row half h, columns 2 grp, 2 grp + 1 of the dword-aligned
        // template), its candidate row's quadrants as two packed u16 pairs; 16x8 / 8x16 sums (up to
        // 130944) and keys in 32-bit lanes
        uint32_t F[8][8];
        const uint32_t *fe = (const uint32_t *)(fenc + f * ffs + (intptr_t)(16 * mby + 8 * h) * fs + 16 * mbx);
        const int fs_dw = (int)(fs / 2);
#pragma unroll
        for( int r = 0; r < 8; r++ )
#pragma unroll
            for( int k = 0; k < 8; k++ )
                F[r][k] = fe[r * fs_dw + k];
        const uint32_t *rbase =
            (const uint32_t *)(ref + f * rfs + (intptr_t)(16 * mby + 8 * h + oy) * rs + 16 * mbx + ox + 2 * grp);
        __attribute__( ( address_space( 3 ) ) ) uint32_t *srow =
            (__attribute__( ( address_space( 3 ) ) ) uint32_t *)(s_row + lmb * W * 8 + 4 * h);
        auto fold2 = [&]( uint32_t s0, uint32_t s1, const uint32_t (&c)[CPG], uint32_t S, uint32_t &k )
            __attribute__( ( always_inline ) ) {
            const uint32_t k0 = (s0 << 12) + c[0], k1 = (s1 << 12) + c[1], m = min( k0, k1 );
            k = min( k, __builtin_elementwise_add_sat( m, S ) );
        };
        auto sink = [&]( int c, uint32_t l, uint32_t r ) {
            __attribute__( ( address_space( 3 ) ) ) uint32_t *q = srow;
            asm volatile( "" : "+v"( q ) );
            typedef uint32_t u32x4 __attribute__( ( ext_vector_type( 4 ) ) );
            const u32x4 S = *(__attribute__( ( address_space( 3 ) ) ) const u32x4 *)(q + c * 8);
            const uint32_t send = h ? l : r, mine = h ? r : l;
            const uint32_t recv = (uint32_t)__builtin_amdgcn_mov_dpp( (int)send, 0xB1, 0xF, 0xF, false );
            const uint32_t l0 = l & 0xffff, l1 = l >> 16, r0 = r & 0xffff, r1 = r >> 16;
            fold2( l0, l1, C[0], S.x, key[0] );
            fold2( r0, r1, C[1], S.y, key[1] );
            fold2( l0 + r0, l1 + r1, C[2], S.z, key[2] );
            fold2( (mine & 0xffff) + (recv & 0xffff), (mine >> 16) + (recv >> 16), C[3], S.w, key[3] );
            asm volatile( "" : "+v"( key[0] ), "+v"( key[1] ), "+v"( key[2] ), "+v"( key[3] ) );
        };
        uint32_t acc[8][4];
        me_rows5q<R, ME_LEAD>( rbase, (int)(rs / 2), F, acc, sink, std::make_integer_sequence<int, 2 * R + 8>{} );
      }
        if( live )
#pragma unroll
            for( int sl = 0; sl < 4; sl++ )
                if( key[sl] < 0xF0000000u )
                    atomicMin( &s_key[lmb * 8 + esa8_part( h, sl )], key[sl] );
    }
    __syncthreads();
    // one lane per partition: the strict-< update (COPY3_IF_LT, me.h:87-93) when the window lies
    // in the template; the others are listed for the workgroup's direct pass below
    for( int t = tid; t < MPW * 8 && wg0 + (uint32_t)(t >> 3) < nmb; t += 256 )
    {
        const int sm = t >> 3;
        const int64_t i = 8 * (int64_t)(wg0 + (uint32_t)sm) + (t & 7);
        const int4 w = s_win[t];
        const int2 org = s_org[sm];
        const uint32_t k = s_key[t];
        if( w.x >= org.x && w.x + w.w <= org.x + P && w.y >= org.y && w.z <= org.y + 2 * R )
        {
            const int16_t *q = par + 8 * i;
            int32_t bc = init_cost[i], rx = q[0], ry = q[1];
            if( k != 0xFFFFFFFFu && (int32_t)(k >> 12) < bc )
            {
                const int ki = (int)(k & 4095);
                bc = (int32_t)(k >> 12);
                ry = w.y + ki / w.w;
                rx = w.x + ki % w.w;
            }
            out[3 * i] = bc;
            out[3 * i + 1] = rx;
            out[3 * i + 2] = ry;
        }
        else
            s_flag[atomicAdd( &s_nflag, 1u )] = (uint16_t)t;
    }
    __syncthreads();
    // the direct pass over the listed partitions' windows outside the template, one wave each
    // (rows' loads four at a time: the main loop's registers are free by now, the full unroll's
    // are not)
    const uint32_t nflag = s_nflag;
    for( uint32_t e = (uint32_t)(tid >> 6); e < nflag; e += 4 )
    {
        const int t = s_flag[e], sm = t >> 3;
        const int2 org = s_org[sm];
        esa8_direct<BD, 4>( fenc, fs, ffs, ref, rs, rfs, mbw, mbh, me_range, par, init_cost, cost_mv, out,
                           8 * (int64_t)(wg0 + (uint32_t)sm) + (t & 7), s_key[t], org.x, org.x + P - 1, org.y,
                           org.y + 2 * R, tid & 63 );
    }
}

// every partition by direct SADs (10 bit, range 0, or no LDS for the template pass): one wave per
// partition
template <int BD>
__global__ __launch_bounds__( 256 ) void me_esa8_direct_kernel( const typename PT<BD>::pixel *__restrict__ fenc,
                                                                intptr_t fs, intptr_t ffs,
                                                                const typename PT<BD>::pixel *__restrict__ ref,
                                                                intptr_t rs, intptr_t rfs, int mbw, int mbh,
                                                                int me_range, const int16_t *__restrict__ par,
                                                                const int32_t *__restrict__ init_cost,
                                                                const uint16_t *__restrict__ cost_mv,
                                                                int32_t *__restrict__ out, uint32_t n )
{
    const uint32_t nw = gridDim.x * (blockDim.x >> 6);
    for( uint32_t e = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); e < n; e += nw )
        esa8_direct<BD, 16>( fenc, fs, ffs, ref, rs, rfs, mbw, mbh, me_range, par, init_cost, cost_mv, out,
                             (int64_t)e, 0xFFFFFFFFu, 1, 0, 1, 0, (int)(threadIdx.x & 63) );
}

template <int BD>
hipError_t launch_me_search_esa8( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                                  const typename PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs, int mbw, int mbh,
                                  int nframes, int range, int me_range, const int16_t *centre, const int16_t *par,
                                  const int32_t *init_cost, const uint16_t *cost_mv, int32_t *out, hipStream_t stream )
{
    const int64_t nmb = (int64_t)nframes * mbw * mbh;
    if( nmb <= 0 )
        return hipSuccess;
    if( nmb * 8 > 0x7fffffff ||
        (((uintptr_t)fenc | (uintptr_t)ref | (uintptr_t)(fs * sizeof( typename PT<BD>::pixel )) |
          (uintptr_t)(rs * sizeof( typename PT<BD>::pixel ))) & 3) )
        return hipErrorInvalidValue;
    if( range > 0 )
    {
        const int xcd = me_xcd();
        switch( range )
        {
#define E8_CASE( RR )                                                                                             \
            case RR:                                                                                              \
                hipLaunchKernelGGL( ( me_esa8_kernel<BD, RR> ),                                                   \
                                    dim3( (unsigned)((nmb + esa8_mbs<BD, RR>() - 1) / esa8_mbs<BD, RR>()) ), dim3( 256 ), \
                                    0, stream, fenc, fs, ffs, ref, rs, rfs, mbw, mbh, nframes, me_range, centre,  \
                                    par, init_cost, cost_mv, out, xcd );                                          \
                break;
            E8_CASE( 4 ) E8_CASE( 8 ) E8_CASE( 16 ) E8_CASE( 24 )
#undef E8_CASE
        }
        return hipGetLastError();
    }
    hipLaunchKernelGGL( me_esa8_direct_kernel<BD>, dim3( (unsigned)std::min<int64_t>( (nmb * 8 + 3) / 4, 2048 ) ),
                        dim3( 256 ), 0, stream, fenc, fs, ffs, ref, rs, rfs, mbw, mbh, me_range, par, init_cost,
                        cost_mv, out, (uint32_t)(nmb * 8) );
    return hipGetLastError();
}

template hipError_t launch_me_search_esa8<8>( const uint8_t *, intptr_t, intptr_t, const uint8_t *, intptr_t, intptr_t,
                                              int, int, int, int, int, const int16_t *, const int16_t *,
                                              const int32_t *, const uint16_t *, int32_t *, hipStream_t );
template hipError_t launch_me_search_esa8<10>( const uint16_t *, intptr_t, intptr_t, const uint16_t *, intptr_t,
                                               intptr_t, int, int, int, int, int, const int16_t *, const int16_t *,
                                               const int32_t *, const uint16_t *, int32_t *, hipStream_t );

} // namespace x264hip
