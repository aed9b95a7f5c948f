// Internal header shared by the gfx950 kernels and the C-ABI layer.
// Pixel/coefficient types per bit depth follow reference common/common.h:93-109.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "x264hip.h"

namespace x264hip {

// a small table (entries < 2^b) as bit fields of one word, entry i in bits [b*i, b*i + b): a
// per-lane index then reads an immediate with a shift and mask instead of a memory load on
// the dependent chain
template <int N> constexpr uint32_t pack_fields( const uint8_t ( &a )[N], int b )
{
    uint32_t r = 0;
    for( int i = 0; i < N; i++ )
        r |= (uint32_t)a[i] << (b * i);
    return r;
}
__device__ __forceinline__ int field( uint32_t k, int b, int i ) { return (int)((k >> (b * i)) & ((1u << b) - 1)); }

template <int BD> struct PT;
template <> struct PT<8>
{
    using pixel = uint8_t;
    using dctcoef = int16_t;
    using udctcoef = uint16_t;
    using sadt = uint16_t;               // 16x16 SAD <= 65280 fits
    static constexpr int PIXEL_MAX = 255;
    static constexpr int PPD = 4;        // pixels per dword
};
template <> struct PT<10>
{
    using pixel = uint16_t;
    using dctcoef = int32_t;
    using udctcoef = uint32_t;
    using sadt = uint32_t;               // 16x16 SAD <= 261888
    static constexpr int PIXEL_MAX = 1023;
    static constexpr int PPD = 2;
};

// Motion-search table geometry (me.hip; include/x264hip.h x264hip_me_table_pitch /
// x264hip_me_centred_pitch).  A full-search table is the (2R+1)^2 square around mv 0 at row
// pitch align4(2R+1).  A centred table is me.c's ESA window around a predictor: 2R+1 rows
// and the columns the window can reach past bmx + R -- the width rounding
// (max_x - min_x + 3) & ~3 (me.c:626) ends up to two columns past max_x -- plus the window
// origin's alignment down to a dword (3 pixels at 8 bit, 1 at 10 bit).
__host__ __device__ constexpr int al4( int x ) { return (x + 3) & ~3; }
__host__ __device__ constexpr int full_pitch( int R ) { return al4( 2 * R + 1 ); }
__host__ __device__ constexpr int cen_cols( int bd, int R ) { return bd == 8 ? 2 * R + 6 : 2 * R + 4; }
__host__ __device__ constexpr int cen_pitch( int bd, int R ) { return al4( cen_cols( bd, R ) ); }

// block sizes, reference common/pixel.h:55-59
__host__ __device__ constexpr int pix_w( int i ) { return i == 0 || i == 1 ? 16 : i <= 4 ? 8 : 4; }
__host__ __device__ constexpr int pix_h( int i )
{
    return i == 0 || i == 2 ? 16 : i == 1 || i == 3 || i == 5 ? 8 : i == 4 || i == 6 ? 4 : 16;
}

// ads slot -> number of DC sums (reference pixel.c:835-838 and the aliasing at :1605-1608)
__host__ __device__ constexpr int ads_nsums( int i_pixel )
{
    return i_pixel == 0 ? 4 : (i_pixel == 3 || i_pixel == 6) ? 1 : 2;
}

// Load NDW packed dwords (NDW*PPD pixels) starting at an arbitrary pixel address.
// Reads dword-aligned words only; the extra word needed for a misaligned start
// is fetched only when the start is misaligned (otherwise the last word is
// re-read), so no byte outside the dwords holding requested pixels is touched.
template <int NDW>
__device__ __forceinline__ void load_packed( const void *p, uint32_t (&out)[NDW] )
{
    // keep the pointer's provenance (global) so hipcc emits global_load, not flat_load
    uint32_t sh = (uint32_t)((uintptr_t)p & 3);
    const uint32_t *base = (const uint32_t *)((const char *)p - sh);
    uint32_t w[NDW + 1];
#pragma unroll
    for( int i = 0; i < NDW; i++ )
        w[i] = base[i];
    w[NDW] = base[sh ? NDW : NDW - 1];
#pragma unroll
    for( int i = 0; i < NDW; i++ )
        out[i] = __builtin_amdgcn_alignbyte( w[i + 1], w[i], sh );
}

// NDW packed dwords at an arbitrary pixel address from the dword-aligned words holding them
// (one vector load of NDW + 1 words; the last re-reads word NDW-1 when aligned, so no byte
// past the row's dwords is touched), realigned with v_alignbyte.  On gfx950 the address path
// takes a byte-misaligned 8-byte lane load at ~2x the cycles of an aligned 12-byte one and a
// misaligned 16-byte one at ~4x (tools/ta_probe.hip, profiles/r01d_ta_probe.txt).
template <int NDW>
__device__ __forceinline__ void load_al( const void *p, uint32_t (&out)[NDW] )
{
    typedef const __attribute__( ( address_space( 1 ) ) ) uint32_t gword;
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3);
    gword *base = (gword *)((uintptr_t)p & ~(uintptr_t)3);
    uint32_t w[NDW + 1];
#pragma unroll
    for( int i = 0; i < NDW; i++ )
        w[i] = base[i];
    w[NDW] = base[sh ? NDW : NDW - 1];
#pragma unroll
    for( int i = 0; i < NDW; i++ )
        out[i] = __builtin_amdgcn_alignbyte( w[i + 1], w[i], sh );
}

// load_al's form for padded planes: the NDW + 1 consecutive dwords from the aligned-down
// address as ONE vector load (global_load_dwordx{2,3,4,...}); the conditional re-read of
// load_al splits it into single-dword loads plus a select, which refine_subpel's address
// path measured at 0.138 -> 0.185 ms per 130560 MBs.  Reads up to 4 bytes past the pixels
// asked for: only for planes with a border (x264's 32-pixel padding).
template <int NDW>
__device__ __forceinline__ void load_al_pad( const void *p, uint32_t (&out)[NDW] )
{
    typedef const __attribute__( ( address_space( 1 ) ) ) uint32_t gword;
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3);
    gword *base = (gword *)((uintptr_t)p & ~(uintptr_t)3);
    uint32_t w[NDW + 1];
#pragma unroll
    for( int i = 0; i <= NDW; i++ )
        w[i] = base[i];
#pragma unroll
    for( int i = 0; i < NDW; i++ )
        out[i] = __builtin_amdgcn_alignbyte( w[i + 1], w[i], sh );
}

// rounding-up average of packed pixels (pixel_avg, reference common/mc.c:57): one
// v_lerp_u8 per dword at 8 bit
template <int BD> __device__ __forceinline__ uint32_t avg_round( uint32_t a, uint32_t b )
{
    if constexpr( BD == 8 )
        return __builtin_amdgcn_lerp( a, b, 0x01010101u );
    else
    {
        // 10-bit pixels: a + b <= 2046 never carries out of a 16-bit lane
        typedef unsigned short us2 __attribute__( ( ext_vector_type( 2 ) ) );
        const us2 s = __builtin_bit_cast( us2, a ) + __builtin_bit_cast( us2, b ) + (us2)1;
        return __builtin_bit_cast( uint32_t, s >> (us2)1 );
    }
}

template <int NDW> __device__ __forceinline__ void load_row_u( const void *p, uint32_t (&out)[NDW] )
{
    if constexpr( NDW == 1 )
        __builtin_memcpy( &out[0], p, 4 );
    else if constexpr( NDW == 2 )
    {
        uint2 v;
        __builtin_memcpy( &v, p, 8 );
        out[0] = v.x; out[1] = v.y;
    }
    else
    {
#pragma unroll
        for( int k = 0; k < NDW; k += 4 )
        {
            uint4 v;
            __builtin_memcpy( &v, (const char *)p + 4 * k, 16 );
            out[k] = v.x; out[k + 1] = v.y; out[k + 2] = v.z; out[k + 3] = v.w;
        }
    }
}

// packed sum of absolute differences: v_sad_u8 (4 x u8) / v_sad_u16 (2 x u16)
template <int BD> __device__ __forceinline__ uint32_t sadp( uint32_t a, uint32_t b, uint32_t acc );
template <> __device__ __forceinline__ uint32_t sadp<8>( uint32_t a, uint32_t b, uint32_t acc )
{
    return __builtin_amdgcn_sad_u8( a, b, acc );
}
template <> __device__ __forceinline__ uint32_t sadp<10>( uint32_t a, uint32_t b, uint32_t acc )
{
    return __builtin_amdgcn_sad_u16( a, b, acc );
}

// SATD of an 8x4 band as two 4x4 Hadamards in packed 16-bit lanes (the
// reference's satd_8x4 "two tiles in one sum2_t" trick of pixel.c:290-309, done
// with v_pk_add/sub_i16): pair x = (column x, column x+4) of each row.  Returns
// sum |coef| of both tiles (even, the caller halves it once).  Differences and
// all Hadamard stages fit int16 for 8 and 10 bit (|coef| <= 16 * 1023).
typedef short x264hip_short2 __attribute__( ( ext_vector_type( 2 ) ) );
template <int BD>
__device__ __forceinline__ x264hip_short2 pair_px( const uint32_t (&r)[8 / PT<BD>::PPD], int x )
{
    uint32_t v;
    if constexpr( BD == 8 )   // bytes x of r[0] and r[1] -> 16-bit lanes
        v = __builtin_amdgcn_perm( r[1], r[0], (uint32_t)x | 0x0c00u | ((uint32_t)(4 + x) << 16) | 0x0c000000u );
    else                      // 16-bit pixel x of r[0..1] and pixel x of r[2..3]
        v = __builtin_amdgcn_perm( r[2 + (x >> 1)], r[x >> 1], (x & 1) ? 0x07060302u : 0x05040100u );
    return __builtin_bit_cast( x264hip_short2, v );
}

// SATD of two 4x4 tiles held in paired columns (x, x+4) of four rows of
// differences p[y][x], accumulated onto acc.  The caller adds 0x8000 to p[0][0]
// (both halves): every Hadamard coefficient has +-1 weight on that element, so
// each coefficient then carries the same 0x8000 bias mod 2^16 and one
// v_sad_u16 against 0x8000 adds |coef| of two coefficients -- no negate / max /
// dot per output.  Exact while |coef| < 2^15 (<= 16 * 1023 here).
__device__ __forceinline__ uint32_t had_sad_pairs( const x264hip_short2 (&p)[4][4], uint32_t acc )
{
    x264hip_short2 d[4][4];
#pragma unroll
    for( int y = 0; y < 4; y++ )
    {
        const x264hip_short2 t0 = p[y][0] + p[y][1], t1 = p[y][0] - p[y][1];
        const x264hip_short2 t2 = p[y][2] + p[y][3], t3 = p[y][2] - p[y][3];
        d[y][0] = t0 + t2; d[y][2] = t0 - t2; d[y][1] = t1 + t3; d[y][3] = t1 - t3;
    }
#pragma unroll
    for( int x = 0; x < 4; x++ )
    {
        const x264hip_short2 t0 = d[0][x] + d[1][x], t1 = d[0][x] - d[1][x];
        const x264hip_short2 t2 = d[2][x] + d[3][x], t3 = d[2][x] - d[3][x];
        const x264hip_short2 c[4] = { t0 + t2, t0 - t2, t1 + t3, t1 - t3 };
#pragma unroll
        for( int k = 0; k < 4; k++ )
            acc = __builtin_amdgcn_sad_u16( __builtin_bit_cast( uint32_t, c[k] ), 0x80008000u, acc );
    }
    return acc;
}

__device__ __forceinline__ x264hip_short2 sat_bias( x264hip_short2 v )
{
    return __builtin_bit_cast( x264hip_short2, __builtin_bit_cast( uint32_t, v ) ^ 0x80008000u );
}

template <int BD>
__device__ __forceinline__ uint32_t satd8x4_packed( const uint32_t (&a)[4][8 / PT<BD>::PPD],
                                                    const uint32_t (&b)[4][8 / PT<BD>::PPD] )
{
    x264hip_short2 p[4][4];
#pragma unroll
    for( int y = 0; y < 4; y++ )
#pragma unroll
        for( int x = 0; x < 4; x++ )
            p[y][x] = pair_px<BD>( a[y], x ) - pair_px<BD>( b[y], x );
    p[0][0] = sat_bias( p[0][0] );
    return had_sad_pairs( p, 0 );
}

// the biased Hadamard coefficients of one side of satd8x4_packed: b's paired columns with 0x8000
// added to p[0][0] (so every coefficient carries it, mod 2^16), in had_sad_pairs' order (column
// pass x, output k -> o[4x + k]).  SATD is linear in the difference, so with the fenc side's
// coefficients precomputed, v_sad_u16( ref's, fenc's ) = |H(ref) - H(fenc)| per pair is
// satd8x4_packed's sum without the fenc unpacking and the difference per candidate (both sides
// lie within 0x8000 +- 16 * 1023: no wrap)
template <int BD>
__device__ __forceinline__ void had8x4_biased( const uint32_t (&b)[4][8 / PT<BD>::PPD], uint32_t (&o)[16] )
{
    x264hip_short2 p[4][4], d[4][4];
#pragma unroll
    for( int y = 0; y < 4; y++ )
#pragma unroll
        for( int x = 0; x < 4; x++ )
            p[y][x] = pair_px<BD>( b[y], x );
    p[0][0] = sat_bias( p[0][0] );
#pragma unroll
    for( int y = 0; y < 4; y++ )
    {
        const x264hip_short2 t0 = p[y][0] + p[y][1], t1 = p[y][0] - p[y][1];
        const x264hip_short2 t2 = p[y][2] + p[y][3], t3 = p[y][2] - p[y][3];
        d[y][0] = t0 + t2; d[y][2] = t0 - t2; d[y][1] = t1 + t3; d[y][3] = t1 - t3;
    }
#pragma unroll
    for( int x = 0; x < 4; x++ )
    {
        const x264hip_short2 t0 = d[0][x] + d[1][x], t1 = d[0][x] - d[1][x];
        const x264hip_short2 t2 = d[2][x] + d[3][x], t3 = d[2][x] - d[3][x];
        o[4 * x + 0] = __builtin_bit_cast( uint32_t, t0 + t2 );
        o[4 * x + 1] = __builtin_bit_cast( uint32_t, t0 - t2 );
        o[4 * x + 2] = __builtin_bit_cast( uint32_t, t1 + t3 );
        o[4 * x + 3] = __builtin_bit_cast( uint32_t, t1 - t3 );
    }
}

// value stored to a dctcoef (int16 wrap at 8 bit), read back as int
template <int BD> __device__ __forceinline__ int sto( int v ) { return (int)(typename PT<BD>::dctcoef)v; }

// x264_clip_pixel (reference common/common.h)
template <int BD> __device__ __forceinline__ int clip_pix( int v )
{
    return v < 0 ? 0 : v > PT<BD>::PIXEL_MAX ? PT<BD>::PIXEL_MAX : v;
}

// k-th pixel of a packed dword
template <int BD> __device__ __forceinline__ int upix( uint32_t w, int k )
{
    return BD == 8 ? (int)((w >> (8 * k)) & 0xff) : (int)((w >> (16 * k)) & 0xffff);
}

} // namespace x264hip

// ---- run-time switches ----
// Seeded once from the environment when the library loads and changed only through
// x264hip_set_variant(): launchers read an atomic, never the environment.  -1 = the
// launcher's default.  Every kernel a switch selects is a default kernel of some input
// (X264HIP_TESA_VARIANT=1: the in-scan SADs of me_range > 24; X264HIP_INTEGRAL_VARIANT=1: the
// unaligned-plane kernel) or a layout option within 3 % of the default in a committed A/B
// (X264HIP_ME_XCD, X264HIP_STREAM_XCD, X264HIP_STREAM_NT); X264HIP_LA_POLL is a test hook and
// X264HIP_UPLOAD_WGS the upload grid cap.
namespace x264hip {
enum VariantSlot
{
    V_TESA = 0, V_INTEGRAL, V_LA_POLL, V_UPLOAD_WGS, V_ME_XCD, V_STREAM_XCD, V_STREAM_NT, V_LA_HELPER,
    V_LA_XCD,
    V_COUNT
};
int variant( VariantSlot slot );

// Workgroup index remap that gives each XCD a contiguous range of logical workgroups:
// the dispatcher deals blocks round-robin over the 8 XCDs (MI355X_MICROARCH.md, workgroup
// dispatch; observed, for speed only), so block b runs on XCD b % 8.  Logical block
// L(b) = start of XCD b%8's range + b/8, a bijection on [0, nblocks); neighbouring logical
// blocks (neighbouring MBs, whose search windows overlap) then share one XCD's L2.
__device__ __forceinline__ uint32_t xcd_block( uint32_t b, uint32_t nblocks )
{
    const uint32_t q = nblocks >> 3, r = nblocks & 7, x = b & 7, i = b >> 3;
    return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

// the 3-D form: the grid's blocks in dispatch order (x fastest, then y, then z) remapped by
// xcd_block when `xcd`, returned as (x, y, z) block coordinates
struct Blk3
{
    uint32_t x, y, z;
};
__device__ __forceinline__ Blk3 blk3( bool xcd )
{
    if( !xcd )
        return { blockIdx.x, blockIdx.y, blockIdx.z };
    const uint32_t gx = gridDim.x, gy = gridDim.y;
    const uint32_t lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const uint32_t l = xcd_block( lin, gx * gy * gridDim.z );
    const uint32_t yz = l / gx;
    return { l - yz * gx, yz % gy, yz / gy };
}

// Store policy of the streaming frame kernels (half-pel planes, lowres planes, fused
// DCT+quant coefficients): nontemporal stores unless X264HIP_STREAM_NT=0.  With every
// wave's stores on whole 128-B lines they stream faster at any batch
// (profiles/r03r_pattern.txt: the 1-in-3-out pattern at 64 padded 1080p frames 0.575 ->
// 0.853 of 8 TB/s; r03s_nt_ab.json / r03w_stream_var.json for the kernels at 16 and 64
// frames).  Nontemporal stores of partial lines -- 62-piece chunks, every wave boundary
// mid-line -- were as slow as plain ones (0.569, the pattern `s3nt62u`).
inline bool stream_nt()
{
    return variant( V_STREAM_NT ) != 0;
}

// a 16-byte store, nontemporal when NT
template <bool NT> __device__ __forceinline__ void st16( void *p, uint4 v )
{
    typedef unsigned int v4u __attribute__( ( ext_vector_type( 4 ) ) );
    if constexpr( NT )
        __builtin_nontemporal_store( (v4u){ v.x, v.y, v.z, v.w }, (v4u *)p );
    else
        *(uint4 *)p = v;
}
} // namespace x264hip

// The device a launch runs on: the launch stream's device, or the calling thread's current
// device for the null stream.  Every launcher that keys device-side state (scratch pools,
// accumulator rings, status words) by device takes it from here, never from the thread
// alone: a stream of device 1 with device 0 current must not be handed device-0 memory.
namespace x264hip {
inline hipError_t stream_device( hipStream_t stream, int *dev )
{
    return stream ? hipStreamGetDevice( stream, dev ) : hipGetDevice( dev );
}
} // namespace x264hip

// ---- launchers implemented in the .hip files (all enqueue on `stream`) ----
namespace x264hip {
hipError_t scratch_trim( int dev );
hipError_t scratch_alloc( void **p, size_t bytes, hipStream_t stream );   // free with hipFreeAsync
hipError_t lowres_status( hipStream_t stream );
hipError_t launch_upload( void *dst, const void *src, size_t bytes, hipStream_t stream );
struct UploadPlane
{
    void *dst;
    const void *src;                    // device address of the pinned source
    intptr_t ds, ss;
    int width_bytes, height, unit, pad_x, pad_y;
};
hipError_t launch_upload_planes( int n, const UploadPlane *planes, hipStream_t stream );
template <int BD>
hipError_t launch_cmp_batch( int op, int i_pixel, const typename PT<BD>::pixel *fenc, intptr_t fs,
                             const typename PT<BD>::pixel *ref, intptr_t rs, const int64_t *fenc_off,
                             const int64_t *ref_off, int n, int32_t *scores, hipStream_t stream );
template <int BD>
hipError_t launch_me_full( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                           const typename PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs, int mbw, int mbh,
                           int nframes, int range, typename PT<BD>::sadt *table, const int16_t *centre,
                           int16_t *origin, hipStream_t stream );
template <int BD>
hipError_t launch_sub_dct( int kind, const typename PT<BD>::pixel *fenc, intptr_t fs,
                           const typename PT<BD>::pixel *fdec, intptr_t ds, const int64_t *fenc_off,
                           const int64_t *fdec_off, int n, typename PT<BD>::dctcoef *dct, hipStream_t stream );
template <int BD>
hipError_t launch_dc( int kind, typename PT<BD>::dctcoef *dct, typename PT<BD>::dctcoef *dct4x4, int n,
                      hipStream_t stream );
template <int BD>
hipError_t launch_quant( int kind, typename PT<BD>::dctcoef *dct, const typename PT<BD>::udctcoef *mf,
                         const typename PT<BD>::udctcoef *bias, int mf_dc, int bias_dc, int n, int32_t *nz,
                         hipStream_t stream );
template <int BD>
hipError_t launch_mb_dct_quant( int transform, const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                                const typename PT<BD>::pixel *pred, intptr_t ps, intptr_t pfs, int mbw, int mbh,
                                int nframes, const typename PT<BD>::udctcoef *mf,
                                const typename PT<BD>::udctcoef *bias, typename PT<BD>::dctcoef *dct, int32_t *nz,
                                hipStream_t stream );
template <int BD>
hipError_t launch_hpel_filter( const typename PT<BD>::pixel *src, typename PT<BD>::pixel *dh,
                               typename PT<BD>::pixel *dv, typename PT<BD>::pixel *dc, intptr_t stride,
                               intptr_t fstride, int width, int height, int nframes, hipStream_t stream );
template <int BD>
hipError_t launch_subpel_cmp( int op, int i_pixel, const typename PT<BD>::pixel *fenc, intptr_t fs,
                              const typename PT<BD>::pixel *const planes[4], intptr_t rs, const int64_t *fenc_off,
                              const int32_t *qxy, int n, int32_t *scores, hipStream_t stream );
template <int BD>
hipError_t launch_subpel_qpel9( int op, int i_pixel, const typename PT<BD>::pixel *fenc, intptr_t fs,
                                const typename PT<BD>::pixel *const planes[4], intptr_t rs, const int64_t *fenc_off,
                                const int32_t *cxy, int n, int32_t *scores, hipStream_t stream );
template <int BD>
hipError_t launch_me_refine_subpel( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                                    const typename PT<BD>::pixel *const planes[4], intptr_t rs, intptr_t rfs,
                                    int i_pixel, int subme, int kind, int fpel_satd, const int32_t *pos,
                                    const int16_t *par, const int32_t *init_cost, const uint16_t *cost_mv, int n,
                                    int32_t *out, int32_t *nevals, int32_t *thr, const int32_t *rcost,
                                    const x264hip_refine_ext_t *ext, hipStream_t stream );
template <int BD>
hipError_t launch_me_search_ref( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                                 const typename PT<BD>::pixel *fw, const typename PT<BD>::pixel *const planes[4],
                                 intptr_t rs, intptr_t rfs, int i_pixel, int me_method, int subme, int me_range,
                                 const int32_t *pos, const int16_t *par, const int16_t *mvc, const uint16_t *cost_mv,
                                 int n, int32_t *out, int32_t *nevals, int32_t *thr, const int32_t *rcost,
                                 const x264hip_refine_ext_t *ext, hipStream_t stream );
// x264's P16x16 reference-0 analysis with mvpred.c's predictors, as an MB wavefront (refine.hip)
template <int BD>
hipError_t launch_me_analyse_p16x16( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                                     const typename PT<BD>::pixel *fw, const typename PT<BD>::pixel *const planes[4],
                                     intptr_t rs, intptr_t rfs, int mbw, int mbh, int nframes, int me_method,
                                     int subme, int me_range, int mv_range, const int16_t *lowres, const int16_t *tmv,
                                     int tscale, const uint16_t *cost_mv, int32_t *out, int32_t *nevals,
                                     const x264hip_refine_ext_t *ext, hipStream_t stream );
template <int BD>
hipError_t launch_me_refine_bidir( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                                   const typename PT<BD>::pixel *const planes0[4],
                                   const typename PT<BD>::pixel *const planes1[4], intptr_t rs, intptr_t rfs,
                                   int i_pixel, int satd, const int32_t *pos, const int16_t *par, const int32_t *weight,
                                   const uint16_t *cost_mv, int n, int32_t *out, int32_t *cost, int32_t *nevals,
                                   hipStream_t stream );
template <int BD>
hipError_t launch_me_esa_argmin( const typename PT<BD>::sadt *table, int R, int nmb, int me_range,
                                 const int16_t *origin, const int16_t *par, const int32_t *init_cost,
                                 const uint16_t *cost_mv, int32_t *out, hipStream_t stream );
template <int BD>
hipError_t launch_me_tesa( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                           const typename PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs, const uint16_t *integral,
                           intptr_t ifs, int mbw, int mbh, int nframes, int me_range, int satd,
                           const typename PT<BD>::sadt *table, int R, const int16_t *origin, const int16_t *par,
                           const int32_t *init_cost, const uint16_t *cost_mv, int32_t *out, hipStream_t stream );
template <int BD>
hipError_t launch_plane_ssd( int nv12, const typename PT<BD>::pixel *p1, intptr_t s1, intptr_t f1,
                             const typename PT<BD>::pixel *p2, intptr_t s2, intptr_t f2, int width, int height,
                             int nframes, uint64_t *out, hipStream_t stream );
template <int BD>
hipError_t launch_me_search_esa( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                                 const typename PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs, int mbw, int mbh,
                                 int nframes, int range, int me_range, const int16_t *par, const int32_t *init_cost,
                                 const uint16_t *cost_mv, int32_t *out, hipStream_t stream );
// sub-partition ESA decisions (me.hip): x264hip_*_me_search_esa8
template <int BD>
hipError_t launch_me_search_esa8( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                                  const typename PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs, int mbw, int mbh,
                                  int nframes, int range, int me_range, const int16_t *centre, const int16_t *par,
                                  const int32_t *init_cost, const uint16_t *cost_mv, int32_t *out, hipStream_t stream );
template <int BD>
hipError_t launch_stat_batch( int op, int i_pixel, const typename PT<BD>::pixel *p1, intptr_t s1,
                              const typename PT<BD>::pixel *p2, intptr_t s2, const int64_t *off1,
                              const int64_t *off2, int height, int n, uint64_t *out, hipStream_t stream );
template <int BD>
hipError_t launch_var2_batch( int i_pixel, const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t fvd,
                              const typename PT<BD>::pixel *fdec, intptr_t ds, intptr_t dvd, const int64_t *fo,
                              const int64_t *dof, int n, int32_t *out, hipStream_t stream );
hipError_t launch_ads_batch( int i_pixel, const int32_t *enc_dc, const uint16_t *sums, int delta,
                             const int64_t *sums_off, const uint16_t *cost, const int64_t *cost_off,
                             const int32_t *width, const int32_t *thresh, int n, int16_t *mvs, int mvs_pitch,
                             int32_t *nmv, hipStream_t stream );
template <int BD>
hipError_t launch_frame_integral( const typename PT<BD>::pixel *plane, intptr_t stride, intptr_t fstride, int lines,
                                  int padh, int sub8x8, int nframes, uint16_t *integral, intptr_t ifstride,
                                  hipStream_t stream );
template <int BD>
hipError_t launch_add_idct( int kind, typename PT<BD>::pixel *dst, intptr_t ds, const int64_t *dst_off,
                            const typename PT<BD>::dctcoef *dct, int n, hipStream_t stream );
template <int BD>
hipError_t launch_dequant( int kind, typename PT<BD>::dctcoef *dct, const int32_t *dmf, const int32_t *qp, int n,
                           hipStream_t stream );
template <int BD>
hipError_t launch_idct4x4dc( typename PT<BD>::dctcoef *dct, int n, hipStream_t stream );
template <int BD>
hipError_t launch_idct_dequant_2x4( int dconly, typename PT<BD>::dctcoef *dct, typename PT<BD>::dctcoef *dct4x4,
                                    const int32_t *dmf, const int32_t *qp, int n, hipStream_t stream );
template <int BD>
hipError_t launch_optimize_chroma( int c422, typename PT<BD>::dctcoef *dct, const int32_t *dmf, int n, int32_t *nz,
                                   hipStream_t stream );
template <int BD>
hipError_t launch_denoise( typename PT<BD>::dctcoef *dct, int size, int n, uint32_t *sum,
                           const typename PT<BD>::udctcoef *offset, hipStream_t stream );
template <int BD>
hipError_t launch_coef_stat( int kind, const typename PT<BD>::dctcoef *dct, int64_t pitch, int n, int32_t *out,
                             hipStream_t stream );
template <int BD>
hipError_t launch_level_run( int num, const typename PT<BD>::dctcoef *dct, int64_t pitch, int n, int32_t *last,
                             int32_t *mask, int32_t *count, typename PT<BD>::dctcoef *level, hipStream_t stream );
template <int BD>
hipError_t launch_zigzag_scan( int size, int field, typename PT<BD>::dctcoef *level,
                               const typename PT<BD>::dctcoef *dct, int n, hipStream_t stream );
template <int BD>
hipError_t launch_zigzag_sub( int kind, int field, typename PT<BD>::dctcoef *level, typename PT<BD>::dctcoef *dc,
                              const typename PT<BD>::pixel *src, intptr_t ss, typename PT<BD>::pixel *dst,
                              intptr_t ds, const int64_t *so, const int64_t *dso, int n, int32_t *nz,
                              hipStream_t stream );
template <int BD>
hipError_t launch_interleave( typename PT<BD>::dctcoef *dst, const typename PT<BD>::dctcoef *src, uint8_t *nnz, int n,
                              hipStream_t stream );
template <int BD>
hipError_t launch_mb_recon( int transform, const typename PT<BD>::dctcoef *dct, int mbw, int mbh, int nframes,
                            const int32_t *dmf, const int32_t *qp, const typename PT<BD>::pixel *pred, intptr_t ps,
                            intptr_t pfs, typename PT<BD>::pixel *recon, intptr_t rs, intptr_t rfs,
                            hipStream_t stream );
template <int BD>
hipError_t launch_frame_init_lowres( const typename PT<BD>::pixel *src, intptr_t stride, intptr_t fstride, int width,
                                     int height, int nframes, typename PT<BD>::pixel *const dst[4], intptr_t ds,
                                     intptr_t dfs, hipStream_t stream );
template <int BD>
hipError_t launch_intra_x3( int kind, int op, const typename PT<BD>::pixel *fenc, intptr_t fs,
                            const typename PT<BD>::pixel *fdec, intptr_t ds, const int64_t *fo,
                            const int64_t *dof, int n, int32_t *scores, hipStream_t stream );
template <int BD>
hipError_t launch_lowres_intra( const typename PT<BD>::pixel *plane, intptr_t stride, intptr_t fstride, int mbw,
                                int mbh, int nframes, int satd, int all_modes, int lambda, const uint16_t *invq,
                                uint16_t *cost, int32_t *row_satd, int32_t *est, hipStream_t stream );
template <int BD>
hipError_t launch_lowres_inter( const typename PT<BD>::pixel *fenc, intptr_t ffs,
                                const typename PT<BD>::pixel *const ref[4], intptr_t stride, intptr_t rfs, int mbw,
                                int mbh, int npairs, int me_method, int subme, int satd, int me_range, int mv_range,
                                int lambda, const uint16_t *cost_mv, const uint16_t *intra_cost,
                                const uint16_t *invq, int16_t *mvs, int32_t *mv_costs, uint16_t *lowres_costs,
                                int32_t *row_satd, int32_t *est, const typename PT<BD>::pixel *ref_w, int wscale,
                                int wdenom, int woffset, int nslices, hipStream_t stream );
template <int BD>
hipError_t launch_me_full8( const typename PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,
                            const typename PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs, int mbw, int mbh,
                            int nframes, int range, uint16_t *table8, hipStream_t stream );
// x264_weights_analyse's inputs (weightp.hip; include/x264hip.h x264hip_*_weights_analyse)
template <int BD> struct WpInput
{
    const typename PT<BD>::pixel *fenc_lr;     // fenc->lowres[0] at (0,0)
    const typename PT<BD>::pixel *ref_lr[4];   // ref->lowres[0..3] at (0,0)
    intptr_t lrs;                              // i_stride_lowres
    int mbw, mbh;
    const uint16_t *intra;                     // fenc->i_intra_cost
    const int16_t *mvs;                        // fenc->lowres_mvs[0][ref0_distance] or NULL
    int cf;                                    // chroma format 0..3
    const typename PT<BD>::pixel *fenc_c[2], *ref_c[2];   // NV12 plane in [0], or the U, V planes (4:4:4)
    intptr_t cs;
    uint32_t fenc_sum[3], ref_sum[3];
    uint64_t fenc_ssd[3], ref_ssd[3];
    int b_lookahead, subme, satd, lambda, numslices, weightp_fake;
};
template <int BD>
hipError_t weights_analyse( const WpInput<BD> &in, x264hip_weight_t weights[3], float *cost_delta,
                            typename PT<BD>::pixel *wlr, hipStream_t stream );
template <int BD>
hipError_t launch_weight_cost( int kind, const typename PT<BD>::pixel *fenc, intptr_t fs,
                               const typename PT<BD>::pixel *const ref[4], intptr_t rs, int mbw, int mbh,
                               const uint16_t *intra, const int16_t *mvs, int satd, int plane, int lambda,
                               int numslices, const x264hip_weight_t *cands, int n, uint32_t *out, hipStream_t stream );
template <int BD>
hipError_t launch_frame_stats( const typename PT<BD>::pixel *y, intptr_t ys, const typename PT<BD>::pixel *u,
                               const typename PT<BD>::pixel *v, intptr_t cs, int mbw, int mbh, int cf,
                               uint64_t *stats, hipStream_t stream );
template <int BD>
hipError_t launch_ssim_wxh( const typename PT<BD>::pixel *p1, intptr_t s1, const typename PT<BD>::pixel *p2,
                            intptr_t s2, int width, int height, float *out, hipStream_t stream );
template <int BD>
hipError_t launch_ssim_bands( const typename PT<BD>::pixel *p1, intptr_t s1, intptr_t f1,
                              const typename PT<BD>::pixel *p2, intptr_t s2, intptr_t f2, int width,
                              const int32_t *bands, int nbands, int nframes, float *out, hipStream_t stream );
template <int BD>
hipError_t launch_ssim_core( const typename PT<BD>::pixel *p1, intptr_t s1, const typename PT<BD>::pixel *p2,
                             intptr_t s2, int *out, hipStream_t stream );
template <int BD>
hipError_t launch_ssim_end4( const int *s0, const int *s1, int width, float *out, hipStream_t stream );
template <int BD>
hipError_t launch_weight_plane( typename PT<BD>::pixel *dst, intptr_t ds, intptr_t dfs,
                                const typename PT<BD>::pixel *src, intptr_t ss, intptr_t sfs, int width, int height,
                                int nframes, int scale, int denom, int offset, hipStream_t stream );
template <int BD>
hipError_t launch_lowres_bidir( const typename PT<BD>::pixel *fenc, intptr_t ffs,
                                const typename PT<BD>::pixel *const ra[4], intptr_t afs,
                                const typename PT<BD>::pixel *const rb[4], intptr_t bfs, intptr_t stride, int mbw,
                                int mbh, int n, int me_method, int subme, int satd, int me_range, int mv_range,
                                int lambda, const uint16_t *cost_mv, int search, int16_t *mvs0, int32_t *costs0,
                                int16_t *mvs1, int32_t *costs1, const int16_t *p1mvs, int dsf, int weight,
                                const uint16_t *invq, uint16_t *lowres_costs, int32_t *row_satd, int32_t *est,
                                int nslices, hipStream_t stream );
} // namespace x264hip
