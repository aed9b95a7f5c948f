// Exhaustive integer-pel 16x16 SAD search tables (the candidate set of the
// reference's ESA/plain exhaustive search, encoder/me.c:618-631, before the
// mv-cost term COST_MV adds, me.c:63-70).
//
// Layout of the work: one lane owns one candidate COLUMN (mx) of one
// macroblock's (2R+1)x(2R+1) window; lanes are dealt MB-major, so the 64 lanes
// of a wave cover ~2 MBs and every lane does identical work (no idle lanes for
// any R).  The lane walks the 2R+16 window rows top to bottom, fetching each
// 16-pixel ref row ONCE (aligned dwords + v_alignbyte_b32) and folding it into
// the (up to 16) candidates my whose 16-row footprint covers that row:
//   acc[my] += sad(fenc row (y - my), ref row y)      (v_sad_u8 / v_sad_u16)
// so ref traffic is 1/16 of a per-candidate loop and the realignment cost is
// amortised over 16 candidates.  fenc (16 rows) stays in VGPRs for the whole
// lane lifetime.  Candidate my finishes at row my+15 and is stored then.
#include "hipcommon.h"
#include <utility>

namespace x264hip {

// one window row Y (compile-time): fold ref row Y into every candidate whose
// footprint covers it; candidate c uses fenc row Y - c.
template <int BD, int R, int Y>
__device__ __forceinline__ void me_row( const typename PT<BD>::pixel *rb, intptr_t rs,
                                        const uint32_t (&F)[16][16 / PT<BD>::PPD], uint32_t (&acc)[16],
                                        typename PT<BD>::sadt *out )
{
    constexpr int NDW = 16 / PT<BD>::PPD;
    constexpr int W = 2 * R + 1;
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
            out[c * W] = (typename PT<BD>::sadt)a;
        else
            acc[c & 15] = a;
    }
}

template <int BD, int R, int... Ys>
__device__ __forceinline__ void me_rows( const typename PT<BD>::pixel *rb, intptr_t rs,
                                         const uint32_t (&F)[16][16 / PT<BD>::PPD], uint32_t (&acc)[16],
                                         typename PT<BD>::sadt *out, std::integer_sequence<int, Ys...> )
{
    ( me_row<BD, R, Ys>( rb, rs, F, acc, out ), ... );
}

template <int BD, int R>
__global__ __launch_bounds__( 256 ) void me_full_sad16_kernel( const typename PT<BD>::pixel *__restrict__ fenc,
                                                               intptr_t fs, intptr_t ffs,
                                                               const typename PT<BD>::pixel *__restrict__ ref,
                                                               intptr_t rs, intptr_t rfs, int mbw, int mbh,
                                                               int nframes, typename PT<BD>::sadt *__restrict__ table )
{
    constexpr int W = 2 * R + 1;
    constexpr int NDW = 16 / PT<BD>::PPD;   // dwords per 16-pixel row
    const int64_t slot = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)nframes * mbh * mbw * W;
    if( slot >= total )
        return;
    const int col = (int)(slot % W);
    const int64_t mb = slot / W;
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

    const typename PT<BD>::pixel *rb = ref + f * rfs + (intptr_t)(16 * mby - R) * rs + 16 * mbx - R + col;
    typename PT<BD>::sadt *out = table + mb * (W * W) + col;

    uint32_t acc[16];
    me_rows<BD, R>( rb, rs, F, acc, out, std::make_integer_sequence<int, 2 * R + 16>{} );
}

template <int BD>
hipError_t launch_me_full( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                           const typename PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs, int mbw, int mbh,
                           int nframes, int range, typename PT<BD>::sadt *table, hipStream_t stream )
{
    const int64_t lanes = (int64_t)nframes * mbh * mbw * (2 * range + 1);
    if( lanes <= 0 )
        return hipSuccess;
    dim3 blk( 256 ), g( (unsigned)((lanes + 255) / 256) );
    switch( range )
    {
#define ME_CASE( R ) \
        case R: hipLaunchKernelGGL( ( me_full_sad16_kernel<BD, R> ), g, blk, 0, stream, fenc, fs, ffs, ref, rs, rfs, \
                                    mbw, mbh, nframes, table ); break;
        ME_CASE( 4 ) ME_CASE( 8 ) ME_CASE( 16 ) ME_CASE( 24 )
#undef ME_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template hipError_t launch_me_full<8>( const uint8_t *, intptr_t, intptr_t, const uint8_t *, intptr_t, intptr_t, int,
                                       int, int, int, uint16_t *, hipStream_t );
template hipError_t launch_me_full<10>( const uint16_t *, intptr_t, intptr_t, const uint16_t *, intptr_t, intptr_t,
                                        int, int, int, int, uint32_t *, hipStream_t );

} // namespace x264hip
