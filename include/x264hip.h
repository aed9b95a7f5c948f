/*****************************************************************************
 * x264hip.h: C ABI of the MI355X (gfx950) backend for x264's pixel / dct /
 *            quant function tables.
 *
 * Two layers, both plain C (no HIP or torch types in any signature):
 *
 *  1. Drop-in table initialisers.  The three structs below are
 *     layout-identical re-declarations of the reference tables
 *       x264_pixel_function_t  (reference common/pixel.h:78-144)
 *       x264_dct_function_t    (reference common/dct.h:29-59)
 *       x264_quant_function_t  (reference common/quant.h:30-70)
 *     for BIT_DEPTH 8 (pixel=uint8_t, dctcoef=int16_t, udctcoef=uint16_t) and
 *     BIT_DEPTH 10 (pixel=uint16_t, dctcoef=int32_t, udctcoef=uint32_t),
 *     reference common/common.h:93-109.  Both initialiser forms OVERRIDE
 *     entries, like x264_pixel_init_altivec() (reference common/pixel.c:
 *     1598-1603): the caller runs its C init x264_{8,10}_*_init() first, then
 *     x264hip_{8,10}_*_init(cpu, tab) (acts when cpu & X264HIP_CPU_HIP) or
 *     x264hip_{8,10}_*_init_hip(tab).  Entries this backend implements are
 *     replaced; every other entry (intra_*_x9_*, the trellis entries, the
 *     never-initialised ssim[7], the encoder's mbcmp / fpelcmp aliases) keeps the
 *     caller's.  Without a usable gfx950 device the table is left untouched
 *     (reference common/opencl.c:400-409), so no installed entry can ever
 *     reach a missing device.  Every table entry is a synchronous call that
 *     executes on the GPU (one dispatch per call).
 *
 *  2. Batched, device-resident entries (x264hip_{8,10}_*_batch, me_*, mb_*):
 *     the same kernels over whole frames / block lists already in HBM, on a
 *     caller-supplied hipStream_t passed as `void *stream` (NULL = default).
 *     These are where the GPU pays; they return 0 or a negative X264HIP_E*.
 *
 * Threading: table entries are reentrant (one HIP stream + staging buffer
 * per calling thread), as required by x264's frame/slice threads
 * (reference encoder/encoder.c:1758-1772).
 *****************************************************************************/
#ifndef X264HIP_H
#define X264HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* cpu flag selecting this backend; bits 26-31 are unused by x86
 * (reference x264.h:139-170). */
#define X264HIP_CPU_HIP (1U<<26)

/* block-size indices, reference common/pixel.h:37-53 */
enum
{
    X264HIP_PIXEL_16x16 = 0,
    X264HIP_PIXEL_16x8  = 1,
    X264HIP_PIXEL_8x16  = 2,
    X264HIP_PIXEL_8x8   = 3,
    X264HIP_PIXEL_8x4   = 4,
    X264HIP_PIXEL_4x8   = 5,
    X264HIP_PIXEL_4x4   = 6,
    X264HIP_PIXEL_4x16  = 7,
};

/* implicit strides of the per-MB caches, reference common/common.h:570-571 */
#define X264HIP_FENC_STRIDE 16
#define X264HIP_FDEC_STRIDE 32

/* error codes of the batched entries */
#define X264HIP_OK          0
#define X264HIP_EINVAL    (-1)  /* bad size / op / shape */
#define X264HIP_EDEVICE   (-2)  /* HIP runtime error (see x264hip_last_error) */
#define X264HIP_ENODEV    (-3)  /* no usable gfx950 device */

/* metric selector of x264hip_*_pixel_cmp_batch (SA8D: i_pixel 16x16 or 8x8) */
enum { X264HIP_CMP_SAD = 0, X264HIP_CMP_SSD = 1, X264HIP_CMP_SATD = 2, X264HIP_CMP_SA8D = 3 };

/* statistic selector of x264hip_*_pixel_stat_batch (uint64_t results) */
enum
{
    X264HIP_STAT_VAR         = 0,  /* var[i_pixel] (16x16, 8x16, 8x8), pixel.c:181-198      */
    X264HIP_STAT_HADAMARD_AC = 1,  /* hadamard_ac[i_pixel] (16x16..8x8), pixel.c:383-435    */
    X264HIP_STAT_SA8D_SATD   = 2,  /* sa8d_satd[16x16]: sa8d | satd << 32, checkasm.c:424-460 */
    X264HIP_STAT_VSAD        = 3,  /* vsad( pix1, stride1, height ), pixel.c:716-723          */
    X264HIP_STAT_ASD8        = 4,  /* asd8( pix1, s1, pix2, s2, height ), pixel.c:747-754     */
};

/* transform selector of x264hip_*_sub_dct_batch (one "block" = one call of
 * the named reference entry, fenc stride 16 / fdec stride 32 semantics are
 * replaced by the explicit strides) */
enum
{
    X264HIP_DCT_SUB4x4     = 0,  /* dct.c:145-189, 16 coefs  */
    X264HIP_DCT_SUB8x8     = 1,  /* dct.c:191-197, 64 coefs  */
    X264HIP_DCT_SUB16x16   = 2,  /* dct.c:199-205, 256 coefs */
    X264HIP_DCT_SUB8x8_DC  = 3,  /* dct.c:216-232, 4 coefs   */
    X264HIP_DCT_SUB8x16_DC = 4,  /* dct.c:234-270, 8 coefs   */
    X264HIP_DCT_SUB8x8_8   = 5,  /* dct.c:358-377, 64 coefs  */
    X264HIP_DCT_SUB16x16_8 = 6,  /* dct.c:379-385, 256 coefs */
};

/* coefficient-domain DC transforms of x264hip_*_dc_batch */
enum { X264HIP_DC_4x4 = 0 /* dct.c:47-76 */, X264HIP_DC_2x4 = 1 /* dct.c:109-143 */,
       X264HIP_DC_I4x4 = 2 /* idct4x4dc, dct.c:78-107 */ };

/* inverse transforms + reconstruction of x264hip_*_add_idct_batch: one "call"
 * = one call of the named reference entry (dct.c:272-476) with an explicit
 * destination stride; dct block i at dct + i*{16,64,256,4,16,64,256}. */
enum
{
    X264HIP_IDCT_ADD4x4      = 0,
    X264HIP_IDCT_ADD8x8      = 1,
    X264HIP_IDCT_ADD16x16    = 2,
    X264HIP_IDCT_ADD8x8_DC   = 3,
    X264HIP_IDCT_ADD16x16_DC = 4,
    X264HIP_IDCT_ADD8x8_8    = 5,
    X264HIP_IDCT_ADD16x16_8  = 6,
};

/* dequantisers of x264hip_*_dequant_batch, quant.c:106-162 */
enum { X264HIP_DEQUANT_4x4 = 0, X264HIP_DEQUANT_8x8 = 1, X264HIP_DEQUANT_4x4_DC = 2 };

/* coefficient statistics of x264hip_*_coef_stat_batch, quant.c:318-378
 * (DECIMATE15 reads dct+1 like decimate_score15; LASTn read dct[0..n)) */
enum
{
    X264HIP_COEF_DECIMATE15 = 0, X264HIP_COEF_DECIMATE16 = 1, X264HIP_COEF_DECIMATE64 = 2,
    X264HIP_COEF_LAST4 = 3, X264HIP_COEF_LAST8 = 4, X264HIP_COEF_LAST15 = 5,
    X264HIP_COEF_LAST16 = 6, X264HIP_COEF_LAST64 = 7,
};

/* block kinds of x264hip_*_intra_cmp_x3_batch: the pixel table's intra_*_x3
 * entries (pixel.c:518-560).  Mode order of res[3]: V,H,DC for 4x4 / 16x16 /
 * 8x8; DC,H,V for the chroma kinds. */
enum
{
    X264HIP_INTRA_4x4   = 0,   /* intra_{sad,satd}_x3_4x4   (predict.c:495-511)   */
    X264HIP_INTRA_8x8C  = 1,   /* intra_{sad,satd}_x3_8x8c  (predict.c:221-281)   */
    X264HIP_INTRA_8x16C = 2,   /* intra_{sad,satd}_x3_8x16c (predict.c:361-441)   */
    X264HIP_INTRA_16x16 = 3,   /* intra_{sad,satd}_x3_16x16 (predict.c:67-130)    */
    X264HIP_INTRA_8x8   = 4,   /* intra_{sad,sa8d}_x3_8x8 from edge[36] (predict.c:716-739) */
};

/* zigzag_sub kinds of x264hip_*_zigzag_sub_batch, dct.c:856-925 */
enum { X264HIP_ZIGZAG_SUB_4x4 = 0, X264HIP_ZIGZAG_SUB_4x4AC = 1, X264HIP_ZIGZAG_SUB_8x8 = 2 };

/* quantiser selector of x264hip_*_quant_batch, quant.c:59-104 */
enum
{
    X264HIP_QUANT_8x8   = 0,
    X264HIP_QUANT_4x4   = 1,
    X264HIP_QUANT_4x4x4 = 2,
    X264HIP_QUANT_4x4_DC = 3,
    X264HIP_QUANT_2x2_DC = 4,
};

struct x264hip_run_level_t;   /* opaque; only its pointer appears (quant.h:61-63) */

/* x264_weight_t (common/mc.h:236-245) as x264_weights_analyse leaves it: weighted = the
 * reference's weightfn != NULL (SET_WEIGHT, mc.h:249-258), the other fields whatever the
 * search wrote, weighted or not */
typedef struct x264hip_weight_t
{
    int32_t weighted, scale, denom, offset;
} x264hip_weight_t;

/* what x264hip_*_me_refine_subpel_ex adds to the luma-only refine (reference encoder/me.c:
 * 826-863, 872-875): chroma ME (h->mb.b_chroma_me, on for P slices at subme >= 5 by default,
 * common/macroblock.c:507-509) and weighted references (m->weight = h->sh.weight[i_ref],
 * encoder/analyse.c:1248-1250).  fenc_chroma / ref_chroma: device pointers at pixel (0,0) of
 * frame 0 -- 4:2:0 / 4:2:2: the frame's interleaved NV12 / NV16 plane (fenc->plane[1]) in [0];
 * 4:4:4: fenc's U, V planes in [0..1] and the reference's U planes F, H, V, C (x264_frame_filter's
 * filtered[1][0..3]) in ref_chroma[0..3], V's in [4..7].  Frame strides step the pos[] frame
 * index as the luma ones do. */
typedef struct x264hip_refine_ext_t
{
    int32_t b_chroma_me;            /* h->mb.b_chroma_me */
    int32_t chroma_format;          /* 1 = 4:2:0, 2 = 4:2:2, 3 = 4:4:4 (read when b_chroma_me) */
    int32_t mvy_offset;             /* me.c:875 (0 for progressive frames) */
    x264hip_weight_t weight[3];     /* m->weight[0..2] (weighted = 0: weightfn == NULL) */
    const void *fenc_chroma[2];
    intptr_t fenc_chroma_stride, fenc_chroma_frame_stride;
    const void *ref_chroma[8];
    intptr_t ref_chroma_stride, ref_chroma_frame_stride;
} x264hip_refine_ext_t;

/* cost kinds of x264hip_*_weight_cost_batch (slicetype.c:191-282) */
enum
{
    X264HIP_WCOST_LUMA = 0,        /* weight_cost_luma: lowres 8x8 mbcmp, min intra cost */
    X264HIP_WCOST_CHROMA420 = 1,   /* weight_cost_chroma, 8x8 asd8 of an NV12 plane */
    X264HIP_WCOST_CHROMA422 = 2,   /* weight_cost_chroma, 8x16 asd8 of an NV16 plane */
    X264HIP_WCOST_CHROMA444 = 3,   /* weight_cost_chroma444: 16x16 mbcmp of a chroma plane */
};

/*----------------------------------------------------------------------------
 * Table declarations, instantiated per bit depth.
 *--------------------------------------------------------------------------*/
#define X264HIP_DECLARE_TABLES( BD, pixel, dctcoef, udctcoef )                                   \
typedef int  (*x264hip_##BD##_pixel_cmp_t)( pixel *, intptr_t, pixel *, intptr_t );              \
typedef void (*x264hip_##BD##_pixel_cmp_x3_t)( pixel *, pixel *, pixel *, pixel *, intptr_t, int[3] ); \
typedef void (*x264hip_##BD##_pixel_cmp_x4_t)( pixel *, pixel *, pixel *, pixel *, pixel *, intptr_t, int[4] ); \
typedef struct                                                                                  \
{                                                                                               \
    x264hip_##BD##_pixel_cmp_t  sad[8];                                                         \
    x264hip_##BD##_pixel_cmp_t  ssd[8];                                                         \
    x264hip_##BD##_pixel_cmp_t satd[8];                                                         \
    x264hip_##BD##_pixel_cmp_t ssim[7];                                                         \
    x264hip_##BD##_pixel_cmp_t sa8d[4];                                                         \
    x264hip_##BD##_pixel_cmp_t mbcmp[8];                                                        \
    x264hip_##BD##_pixel_cmp_t mbcmp_unaligned[8];                                              \
    x264hip_##BD##_pixel_cmp_t fpelcmp[8];                                                      \
    x264hip_##BD##_pixel_cmp_x3_t fpelcmp_x3[7];                                                \
    x264hip_##BD##_pixel_cmp_x4_t fpelcmp_x4[7];                                                \
    x264hip_##BD##_pixel_cmp_t sad_aligned[8];                                                  \
    int (*vsad)( pixel *, intptr_t, int );                                                      \
    int (*asd8)( pixel *pix1, intptr_t stride1, pixel *pix2, intptr_t stride2, int height );    \
    uint64_t (*sa8d_satd[1])( pixel *pix1, intptr_t stride1, pixel *pix2, intptr_t stride2 );   \
    uint64_t (*var[4])( pixel *pix, intptr_t stride );                                          \
    int (*var2[4])( pixel *fenc, pixel *fdec, int ssd[2] );                                     \
    uint64_t (*hadamard_ac[4])( pixel *pix, intptr_t stride );                                  \
    void (*ssd_nv12_core)( pixel *pixuv1, intptr_t stride1, pixel *pixuv2, intptr_t stride2,    \
                           int width, int height, uint64_t *ssd_u, uint64_t *ssd_v );           \
    void (*ssim_4x4x2_core)( const pixel *pix1, intptr_t stride1,                               \
                             const pixel *pix2, intptr_t stride2, int sums[2][4] );             \
    float (*ssim_end4)( int sum0[5][4], int sum1[5][4], int width );                            \
    x264hip_##BD##_pixel_cmp_x3_t sad_x3[7];                                                    \
    x264hip_##BD##_pixel_cmp_x4_t sad_x4[7];                                                    \
    x264hip_##BD##_pixel_cmp_x3_t satd_x3[7];                                                   \
    x264hip_##BD##_pixel_cmp_x4_t satd_x4[7];                                                   \
    int (*ads[7])( int enc_dc[4], uint16_t *sums, int delta,                                    \
                   uint16_t *cost_mvx, int16_t *mvs, int width, int thresh );                   \
    void (*intra_mbcmp_x3_16x16)( pixel *fenc, pixel *fdec, int res[3] );                       \
    void (*intra_satd_x3_16x16) ( pixel *fenc, pixel *fdec, int res[3] );                       \
    void (*intra_sad_x3_16x16)  ( pixel *fenc, pixel *fdec, int res[3] );                       \
    void (*intra_mbcmp_x3_4x4)  ( pixel *fenc, pixel *fdec, int res[3] );                       \
    void (*intra_satd_x3_4x4)   ( pixel *fenc, pixel *fdec, int res[3] );                       \
    void (*intra_sad_x3_4x4)    ( pixel *fenc, pixel *fdec, int res[3] );                       \
    void (*intra_mbcmp_x3_chroma)( pixel *fenc, pixel *fdec, int res[3] );                      \
    void (*intra_satd_x3_chroma) ( pixel *fenc, pixel *fdec, int res[3] );                      \
    void (*intra_sad_x3_chroma)  ( pixel *fenc, pixel *fdec, int res[3] );                      \
    void (*intra_mbcmp_x3_8x16c) ( pixel *fenc, pixel *fdec, int res[3] );                      \
    void (*intra_satd_x3_8x16c)  ( pixel *fenc, pixel *fdec, int res[3] );                      \
    void (*intra_sad_x3_8x16c)   ( pixel *fenc, pixel *fdec, int res[3] );                      \
    void (*intra_mbcmp_x3_8x8c)  ( pixel *fenc, pixel *fdec, int res[3] );                      \
    void (*intra_satd_x3_8x8c)   ( pixel *fenc, pixel *fdec, int res[3] );                      \
    void (*intra_sad_x3_8x8c)    ( pixel *fenc, pixel *fdec, int res[3] );                      \
    void (*intra_mbcmp_x3_8x8)  ( pixel *fenc, pixel edge[36], int res[3] );                    \
    void (*intra_sa8d_x3_8x8)   ( pixel *fenc, pixel edge[36], int res[3] );                    \
    void (*intra_sad_x3_8x8)    ( pixel *fenc, pixel edge[36], int res[3] );                    \
    int (*intra_mbcmp_x9_4x4)( pixel *fenc, pixel *fdec, uint16_t *bitcosts );                  \
    int (*intra_satd_x9_4x4) ( pixel *fenc, pixel *fdec, uint16_t *bitcosts );                  \
    int (*intra_sad_x9_4x4)  ( pixel *fenc, pixel *fdec, uint16_t *bitcosts );                  \
    int (*intra_mbcmp_x9_8x8)( pixel *fenc, pixel *fdec, pixel edge[36], uint16_t *bitcosts, uint16_t *satds ); \
    int (*intra_sa8d_x9_8x8) ( pixel *fenc, pixel *fdec, pixel edge[36], uint16_t *bitcosts, uint16_t *satds ); \
    int (*intra_sad_x9_8x8)  ( pixel *fenc, pixel *fdec, pixel edge[36], uint16_t *bitcosts, uint16_t *satds ); \
} x264hip_##BD##_pixel_function_t;                                                              \
                                                                                                \
typedef struct                                                                                  \
{                                                                                               \
    void (*sub4x4_dct) ( dctcoef dct[16], pixel *pix1, pixel *pix2 );                           \
    void (*add4x4_idct)( pixel *p_dst, dctcoef dct[16] );                                       \
    void (*sub8x8_dct)    ( dctcoef dct[4][16], pixel *pix1, pixel *pix2 );                     \
    void (*sub8x8_dct_dc) ( dctcoef dct[4], pixel *pix1, pixel *pix2 );                         \
    void (*add8x8_idct)   ( pixel *p_dst, dctcoef dct[4][16] );                                 \
    void (*add8x8_idct_dc)( pixel *p_dst, dctcoef dct[4] );                                     \
    void (*sub8x16_dct_dc)( dctcoef dct[8], pixel *pix1, pixel *pix2 );                         \
    void (*sub16x16_dct)    ( dctcoef dct[16][16], pixel *pix1, pixel *pix2 );                  \
    void (*add16x16_idct)   ( pixel *p_dst, dctcoef dct[16][16] );                              \
    void (*add16x16_idct_dc)( pixel *p_dst, dctcoef dct[16] );                                  \
    void (*sub8x8_dct8) ( dctcoef dct[64], pixel *pix1, pixel *pix2 );                          \
    void (*add8x8_idct8)( pixel *p_dst, dctcoef dct[64] );                                      \
    void (*sub16x16_dct8) ( dctcoef dct[4][64], pixel *pix1, pixel *pix2 );                     \
    void (*add16x16_idct8)( pixel *p_dst, dctcoef dct[4][64] );                                 \
    void (*dct4x4dc) ( dctcoef d[16] );                                                         \
    void (*idct4x4dc)( dctcoef d[16] );                                                         \
    void (*dct2x4dc)( dctcoef dct[8], dctcoef dct4x4[8][16] );                                  \
} x264hip_##BD##_dct_function_t;                                                                \
                                                                                                \
typedef struct                                                                                  \
{                                                                                               \
    int (*quant_8x8)  ( dctcoef dct[64], udctcoef mf[64], udctcoef bias[64] );                  \
    int (*quant_4x4)  ( dctcoef dct[16], udctcoef mf[16], udctcoef bias[16] );                  \
    int (*quant_4x4x4)( dctcoef dct[4][16], udctcoef mf[16], udctcoef bias[16] );               \
    int (*quant_4x4_dc)( dctcoef dct[16], int mf, int bias );                                   \
    int (*quant_2x2_dc)( dctcoef dct[4], int mf, int bias );                                    \
    void (*dequant_8x8)( dctcoef dct[64], int dequant_mf[6][64], int i_qp );                    \
    void (*dequant_4x4)( dctcoef dct[16], int dequant_mf[6][16], int i_qp );                    \
    void (*dequant_4x4_dc)( dctcoef dct[16], int dequant_mf[6][16], int i_qp );                 \
    void (*idct_dequant_2x4_dc)( dctcoef dct[8], dctcoef dct4x4[8][16], int dequant_mf[6][16], int i_qp ); \
    void (*idct_dequant_2x4_dconly)( dctcoef dct[8], int dequant_mf[6][16], int i_qp );         \
    int (*optimize_chroma_2x2_dc)( dctcoef dct[4], int dequant_mf );                            \
    int (*optimize_chroma_2x4_dc)( dctcoef dct[8], int dequant_mf );                            \
    void (*denoise_dct)( dctcoef *dct, uint32_t *sum, udctcoef *offset, int size );             \
    int (*decimate_score15)( dctcoef *dct );                                                    \
    int (*decimate_score16)( dctcoef *dct );                                                    \
    int (*decimate_score64)( dctcoef *dct );                                                    \
    int (*coeff_last[14])( dctcoef *dct );                                                      \
    int (*coeff_last4)( dctcoef *dct );                                                         \
    int (*coeff_last8)( dctcoef *dct );                                                         \
    int (*coeff_level_run[13])( dctcoef *dct, struct x264hip_run_level_t *runlevel );           \
    int (*coeff_level_run4)( dctcoef *dct, struct x264hip_run_level_t *runlevel );              \
    int (*coeff_level_run8)( dctcoef *dct, struct x264hip_run_level_t *runlevel );              \
    int (*trellis_cabac_4x4)( const int *unquant_mf, const uint8_t *zigzag, int lambda2,        \
                              int last_nnz, dctcoef *coefs, dctcoef *quant_coefs, dctcoef *dct, \
                              uint8_t *cabac_state_sig, uint8_t *cabac_state_last,              \
                              uint64_t level_state0, uint16_t level_state1, int b_ac );         \
    int (*trellis_cabac_8x8)( const int *unquant_mf, const uint8_t *zigzag, int lambda2,        \
                              int last_nnz, dctcoef *coefs, dctcoef *quant_coefs, dctcoef *dct, \
                              uint8_t *cabac_state_sig, uint8_t *cabac_state_last,              \
                              uint64_t level_state0, uint16_t level_state1, int b_interlaced ); \
    int (*trellis_cabac_4x4_psy)( const int *unquant_mf, const uint8_t *zigzag, int lambda2,    \
                              int last_nnz, dctcoef *coefs, dctcoef *quant_coefs, dctcoef *dct, \
                              uint8_t *cabac_state_sig, uint8_t *cabac_state_last,              \
                              uint64_t level_state0, uint16_t level_state1, int b_ac,           \
                              dctcoef *fenc_dct, int psy_trellis );                             \
    int (*trellis_cabac_8x8_psy)( const int *unquant_mf, const uint8_t *zigzag, int lambda2,    \
                              int last_nnz, dctcoef *coefs, dctcoef *quant_coefs, dctcoef *dct, \
                              uint8_t *cabac_state_sig, uint8_t *cabac_state_last,              \
                              uint64_t level_state0, uint16_t level_state1, int b_interlaced,   \
                              dctcoef *fenc_dct, int psy_trellis );                             \
    int (*trellis_cabac_dc)( const int *unquant_mf, const uint8_t *zigzag, int lambda2,         \
                              int last_nnz, dctcoef *coefs, dctcoef *quant_coefs, dctcoef *dct, \
                              uint8_t *cabac_state_sig, uint8_t *cabac_state_last,              \
                              uint64_t level_state0, uint16_t level_state1, int num_coefs );    \
    int (*trellis_cabac_chroma_422_dc)( const int *unquant_mf, const uint8_t *zigzag, int lambda2, \
                              int last_nnz, dctcoef *coefs, dctcoef *quant_coefs, dctcoef *dct, \
                              uint8_t *cabac_state_sig, uint8_t *cabac_state_last,              \
                              uint64_t level_state0, uint16_t level_state1 );                   \
} x264hip_##BD##_quant_function_t;                                                             \
                                                                                                \
/* x264_zigzag_function_t, reference common/dct.h:61-70 */                                      \
typedef struct                                                                                  \
{                                                                                               \
    void (*scan_8x8)( dctcoef level[64], dctcoef dct[64] );                                     \
    void (*scan_4x4)( dctcoef level[16], dctcoef dct[16] );                                     \
    int  (*sub_8x8)  ( dctcoef level[64], const pixel *p_src, pixel *p_dst );                   \
    int  (*sub_4x4)  ( dctcoef level[16], const pixel *p_src, pixel *p_dst );                   \
    int  (*sub_4x4ac)( dctcoef level[16], const pixel *p_src, pixel *p_dst, dctcoef *dc );      \
    void (*interleave_8x8_cavlc)( dctcoef *dst, dctcoef *src, uint8_t *nnz );                   \
} x264hip_##BD##_zigzag_function_t;                                                             \
                                                                                                \
/* x264_run_level_t, reference common/bitstream.h:50-55 (level 16-byte aligned) */             \
typedef struct                                                                                  \
{                                                                                               \
    int32_t last;                                                                               \
    int32_t mask;                                                                               \
    dctcoef level[18] __attribute__((aligned(16)));                                             \
} x264hip_##BD##_run_level_t;

X264HIP_DECLARE_TABLES( 8,  uint8_t,  int16_t, uint16_t )
X264HIP_DECLARE_TABLES( 10, uint16_t, int32_t, uint32_t )

/*----------------------------------------------------------------------------
 * Runtime
 *--------------------------------------------------------------------------*/
/* Select and initialise a gfx950 device.  0 on success, X264HIP_ENODEV if no
 * gfx950 device is present (the caller then keeps its own C entries, the
 * convention of reference common/opencl.c:400-409). */
int  x264hip_init( int device );
/* last HIP error text of the calling thread ("" if none) */
const char *x264hip_last_error( void );
/* 1 if a gfx950 device is bound (x264hip_init(0) is tried when none is yet) */
int  x264hip_available( void );
/* Bind the calling thread to `device` (a gfx950 device; -1 = back to the
 * process device of x264hip_init).  Table entries called from this thread then
 * run on that device, on a stream and staging buffer owned by the thread, so
 * x264's frame / lookahead threads (reference encoder/encoder.c:1758-1772) can
 * each drive a different GPU of the node from one process.  Batched entries run
 * on the stream the caller passes, whose device they use. */
int  x264hip_set_thread_device( int device );
/* the calling thread's device (its override, else the process device; -1 if none) */
int  x264hip_thread_device( void );
/* Forward a reconstructed reference plane to the GPU encoding the next frame:
 * one asynchronous xGMI peer copy of `bytes` on `stream` (the
 * frame-per-GPU pipeline's only device-to-device transfer). */
int  x264hip_forward_ref( void *dst, int dst_device, const void *src, int src_device, size_t bytes,
                          void *stream );
/* Upload `bytes` of frame planes from page-locked host memory (hipHostMalloc /
 * hipHostRegister) to device memory: a kernel on `stream` reads the pinned pages
 * over PCIe (16-byte pieces when both pointers are 16-byte aligned), the streaming
 * form of configs[3] (H2D per frame overlapped with compute).
 * Asynchronous; the host buffer must stay untouched until `stream` passes it. */
int  x264hip_upload( void *dst, const void *host_src, size_t bytes, void *stream );
/* Upload one picture plane (width_bytes x height at host_src, rows src_stride apart, page-locked)
 * into a padded frame plane: dst = its pixel (0,0); the plane copy of x264_frame_copy_picture
 * (common/frame.c:393-521) with plane_expand_border (frame.c:535-554) fused -- the edge element of
 * `unit` bytes (1 / 2: 8 / 10-bit luma; 2 / 4: an NV12 / NV16 plane, per component) repeated over
 * pad_x bytes left and right, then rows 0 and height-1 with their pads over pad_y rows above and
 * below.  width_bytes, pad_x and both strides multiples of 16, both pointers 16-byte aligned.
 * Asynchronous on `stream`, as x264hip_upload. */
int  x264hip_upload_plane( void *dst, intptr_t dst_stride, const void *host_src, intptr_t src_stride,
                           int width_bytes, int height, int unit, int pad_x, int pad_y, void *stream );
/* the planes of one picture (luma + NV12 / NV16, or Y, U, V; 1..3) in one launch, each as
 * x264hip_upload_plane describes it, so the link does not drain between planes */
typedef struct x264hip_plane_upload_t
{
    void *dst;
    intptr_t dst_stride;
    const void *host_src;
    intptr_t src_stride;
    int32_t width_bytes, height, unit, pad_x, pad_y;
} x264hip_plane_upload_t;
int  x264hip_upload_planes( int n, const x264hip_plane_upload_t *planes, void *stream );
/* A compute / copy stream pair on complementary CU sets of the current device: *copy on
 * the first reserve_cus CUs, *compute on the others (hipExtStreamCreateWithCUMask), for
 * overlapping x264hip_upload of the next frame with the current frame's kernels.
 * x264hip_stream_destroy releases either. */
int  x264hip_stream_pair_create( int reserve_cus, void **compute, void **copy );
int  x264hip_stream_destroy( void *stream );
/* release the idle blocks of the library's scratch pools on `device` (all devices for
 * device < 0).  The self-contained me_tesa takes its table scratch (~2.6 KB per MB at
 * me_range 16, 8 bit) from a per-device pool that keeps its peak between calls, so repeated
 * calls do not map fresh pages; this returns it to the device. */
int  x264hip_trim( int device );
/* the lookahead wavefront's status: waits for `stream`, then X264HIP_EDEVICE if a
 * lowres_inter_cost / lowres_bidir_cost launch of the calling thread on the stream's device
 * timed out waiting for the band below (its outputs are then invalid; see
 * x264hip_set_variant's X264HIP_LA_POLL), else 0; reporting clears the condition.  The
 * lookahead entries themselves are asynchronous and capturable: each also reports (and
 * refuses to launch) once an earlier launch's failure has reached the host. */
int  x264hip_lowres_status( void *stream );
/* row pitch (entries) of a me_search_full table (centred = 0: align4(2*range+1)) or a
 * me_search_centred table (centred = 1: align4(2*range+6) at 8 bit, align4(2*range+4) at
 * 10 bit -- me.c's ESA window around the centre), 0 for a bad bitdepth / range */
int  x264hip_me_table_pitch( int bitdepth, int range, int centred );
/* one line naming the device and the table entries the HIP backend fills (the
 * analogue of reference encoder/encoder.c:1676-1706); also printed once to
 * stderr at the first table fill unless X264HIP_QUIET=1 */
const char *x264hip_backend_banner( void );
/* Run-time switches by environment name; the environment seeds them once, this changes one
 * at run time (-1 = default), X264HIP_EINVAL for an unknown name.  Each input has one kernel;
 * the switches select layout / store options measured within 3 % of the default
 * (X264HIP_ME_XCD, X264HIP_STREAM_XCD, X264HIP_STREAM_NT) or force a kernel that is the default
 * for other inputs (X264HIP_TESA_VARIANT=1: the in-scan SADs of me_range > 24;
 * X264HIP_INTEGRAL_VARIANT=1: the unaligned-plane integral kernel); X264HIP_UPLOAD_WGS caps
 * the upload grid; X264HIP_LA_HELPER=0 / 1 forces the lookahead's L2-warming helper wave off /
 * on (default: on when every band's workgroup fits on the GPU at once); X264HIP_LA_XCD=0 / 1
 * forces the lookahead's bands of one frame pair onto one XCD off / on (default: on under the
 * same condition).  All are bit-exact;
 * only speed differs.  One switch is a test hook:
 * X264HIP_LA_POLL bounds the lookahead wavefront's wait for the band below (default 2^22
 * tries); 0 forces the timeout path (see x264hip_lowres_status). */
int  x264hip_set_variant( const char *name, int value );

/* Table lookup mode of the drop-in 16x16 SAD entries (SURVEY.md §7 hard part 1(b)):
 * x264hip_{8,10}_me_bind registers, for the CALLING THREAD, one frame's full-search result
 * -- host pointers at pixel (0,0) of the fenc and ref luma planes (x264's padded planes,
 * common stride), and a host copy of the x264hip_*_me_search_full table of that pair
 * (range R, row pitch (2R+1+3)&~3, mb_width x mb_height MBs).  While bound,
 * sad[PIXEL_16x16] (hence fpelcmp under x264's aliasing, encoder.c:1409-1427),
 * sad_x3[PIXEL_16x16] and sad_x4[PIXEL_16x16] answer on the host, with no dispatch,
 * every call whose candidate pointer lies in the bound ref plane at a full-pel mv the
 * table holds (|mv| <= R) for an MB whose pixels equal the caller's fenc block (me.c's
 * p_fenc, FENC_STRIDE) -- the ESA / exhaustive and pattern searches of me.c:63-70,
 * 618-771 over that pair.  Every other call dispatches as before; results are identical
 * either way.  The planes and the table must stay valid and unchanged while bound.
 * x264hip_me_unbind releases the thread's binding; x264hip_me_bind_stats returns the
 * thread's hit / miss counts of bound-mode calls (reset when `reset`). */
void x264hip_me_unbind( void );
void x264hip_me_bind_stats( uint64_t *hits, uint64_t *misses, int reset );

/*----------------------------------------------------------------------------
 * Per-bit-depth entries.  BD = 8 or 10.
 *--------------------------------------------------------------------------*/
#define X264HIP_DECLARE_ENTRIES( BD, pixel, dctcoef, udctcoef, sadt )                            \
/* lookup mode of the 16x16 SAD table entries (see x264hip_me_unbind above); EINVAL for a       \
 * bad shape (range 1..29, stride >= 16*mb_width + 64) */                                        \
int x264hip_##BD##_me_bind( const pixel *fenc, const pixel *ref, intptr_t stride,               \
                            int mb_width, int mb_height, const sadt *table, int range );        \
/* the general form: a 16x16 table (or NULL) and / or 8x8 quadrant tables from                  \
 * me_search_full8 (or NULL).  With table8, sad / sad_x3 / sad_x4 of PIXEL_16x8,                 \
 * 8x16 and 8x8 answer from it as well (the partition whose pixels equal the caller's fenc       \
 * block, its SAD the sum of its quadrants), and PIXEL_16x16 from the four when table is NULL. */ \
int x264hip_##BD##_me_bind_tables( const pixel *fenc, const pixel *ref, intptr_t stride,        \
                                   int mb_width, int mb_height, const sadt *table,              \
                                   const uint16_t *table8, int range );                         \
/* drop-in table initialisers (see header comment) */                                           \
void x264hip_##BD##_pixel_init( uint32_t cpu, x264hip_##BD##_pixel_function_t *pixf );          \
void x264hip_##BD##_pixel_init_hip( x264hip_##BD##_pixel_function_t *pixf );                    \
void x264hip_##BD##_dct_init( uint32_t cpu, x264hip_##BD##_dct_function_t *dctf );              \
void x264hip_##BD##_dct_init_hip( x264hip_##BD##_dct_function_t *dctf );                        \
void x264hip_##BD##_quant_init( void *h, uint32_t cpu, x264hip_##BD##_quant_function_t *pf );   \
void x264hip_##BD##_quant_init_hip( x264hip_##BD##_quant_function_t *pf );                      \
void x264hip_##BD##_zigzag_init( uint32_t cpu, x264hip_##BD##_zigzag_function_t *pf_progressive, \
                                 x264hip_##BD##_zigzag_function_t *pf_interlaced );             \
void x264hip_##BD##_zigzag_init_hip( x264hip_##BD##_zigzag_function_t *pf_progressive,          \
                                     x264hip_##BD##_zigzag_function_t *pf_interlaced );                      \
                                                                                                \
/* quant tables: restates x264_cqm_init (reference common/set.c:73-206) for the                 \
 * mf / bias arrays the quant entries consume.  scaling_list[8] as sps->scaling_list            \
 * (4x4 lists 0..3 = CQM_4IY,4PY,4IC,4PC; 8x8 lists 4..7).  deadzone_inter/intra =              \
 * param.analyse.i_luma_deadzone[0]/[1] (defaults 21/11, reference base.c:456-457).             \
 * Output arrays are [4][qp_max_spec+1][16] and [4][qp_max_spec+1][64]; the 8x8                 \
 * ones are written only when b_transform_8x8.  Returns qp_max_spec (51 / 63). */               \
int x264hip_##BD##_cqm_init( const uint8_t *const scaling_list[8], int deadzone_inter,          \
                             int deadzone_intra, int b_transform_8x8,                           \
                             udctcoef *quant4_mf, udctcoef *quant4_bias,                        \
                             udctcoef *quant8_mf, udctcoef *quant8_bias );                      \
                                                                                                \
/* generic block metrics over device-resident planes: for i < n,                               \
 * scores[i] = op( fenc + fenc_off[i], fenc_stride, ref + ref_off[i], ref_stride )              \
 * with op the reference sad/ssd/satd of size i_pixel (pixel.c:55-110, 265-332).                \
 * Offsets and strides count pixels.  fenc_off/ref_off/scores are device arrays. */             \
int x264hip_##BD##_pixel_cmp_batch( int op, int i_pixel,                                        \
                                    const pixel *fenc, intptr_t fenc_stride,                    \
                                    const pixel *ref, intptr_t ref_stride,                      \
                                    const int64_t *fenc_off, const int64_t *ref_off,            \
                                    int n, int32_t *scores, void *stream );                     \
                                                                                                \
/* 64-bit block statistics (X264HIP_STAT_*): out[i] = the reference entry on                   \
 * pix1 + off1[i] (and pix2 + off2[i] for SA8D_SATD / ASD8; pix2/off2 unused                    \
 * otherwise), `height` used by VSAD / ASD8 only.  Device arrays. */                            \
int x264hip_##BD##_pixel_stat_batch( int op, int i_pixel,                                       \
                                     const pixel *pix1, intptr_t stride1,                       \
                                     const pixel *pix2, intptr_t stride2,                       \
                                     const int64_t *off1, const int64_t *off2,                  \
                                     int height, int n, uint64_t *out, void *stream );          \
                                                                                                \
/* var2[i_pixel] (8x16 or 8x8, pixel.c:203-227) with explicit strides: the U                    \
 * blocks at fenc + fenc_off[i] / fdec + fdec_off[i], the V blocks at +fenc_vdelta /            \
 * +fdec_vdelta (the table entry uses FENC_STRIDE/2, FDEC_STRIDE/2);                            \
 * out[3i] = return value, out[3i+1..2] = ssd[0..1]. */                                         \
int x264hip_##BD##_var2_batch( int i_pixel, const pixel *fenc, intptr_t fenc_stride,            \
                               intptr_t fenc_vdelta, const pixel *fdec, intptr_t fdec_stride,   \
                               intptr_t fdec_vdelta, const int64_t *fenc_off,                   \
                               const int64_t *fdec_off, int n, int32_t *out, void *stream );    \
                                                                                                \
/* successive elimination, n independent calls of ads[i_pixel] (pixel.c:759-803,               \
 * slots aliased as :1605-1608): call i reads enc_dc[4i..4i+3], sums +                          \
 * sums_off[i] (with the common `delta`), cost_mvx + cost_off[i], width[i] and                  \
 * thresh[i]; writes the passing candidate indices in order to                                  \
 * mvs[i*mvs_pitch ..] and their count to nmv[i].  Device arrays. */                            \
int x264hip_##BD##_ads_batch( int i_pixel, const int32_t *enc_dc, const uint16_t *sums,         \
                              int delta, const int64_t *sums_off, const uint16_t *cost_mvx,     \
                              const int64_t *cost_off, const int32_t *width,                    \
                              const int32_t *thresh, int n, int16_t *mvs, int mvs_pitch,        \
                              int32_t *nmv, void *stream );                                     \
                                                                                                \
/* n independent intra_*_x3 calls of X264HIP_INTRA_* kind: block i has fenc at                 \
 * fenc + fenc_off[i] (stride fenc_stride) and its reconstructed neighbours at                  \
 * fdec + fdec_off[i] (the block's (0,0); row -1 and column -1 are read, stride                 \
 * fdec_stride), or for X264HIP_INTRA_8x8 the 36-entry filtered edge at                          \
 * fdec + fdec_off[i].  op: X264HIP_CMP_SAD or X264HIP_CMP_SATD (X264HIP_CMP_SA8D                 \
 * for the 8x8 kind).  scores[3i..3i+2] = the reference's res[3].  The                           \
 * reference C also leaves its last prediction in fdec; this entry does not                      \
 * write fdec (as the asm versions).  Device arrays. */                                          \
int x264hip_##BD##_intra_cmp_x3_batch( int kind, int op, const pixel *fenc, intptr_t fenc_stride, \
                                       const pixel *fdec, intptr_t fdec_stride,                  \
                                       const int64_t *fenc_off, const int64_t *fdec_off, int n,  \
                                       int32_t *scores, void *stream );                          \
                                                                                                \
/* the lookahead's intra estimate (slicetype_mb_cost's lowres_intra_mb leg,                     \
 * encoder/slicetype.c:714-757) for every 8x8 block of n_frames lowres planes                    \
 * (lowres[0] of x264hip_*_frame_init_lowres; plane at (0,0), 32 pixels of border,              \
 * plane and stride 4-byte aligned).  satd = !lossless && subme > 1 (the mbcmp                   \
 * choice of encoder.c:1409-1416), all_modes = subme > 1 (planar + the six                        \
 * directional 8x8 modes over the filtered edge), lambda = x264_lambda_tab[qp].                   \
 * Outputs per frame f: intra_cost[f*mbw*mbh + mb] (fenc->i_intra_cost),                         \
 * row_satd[f*mbh + y] (i_row_satds[0][0], AQ-scaled), cost_est[2f] / [2f+1]                      \
 * (i_cost_est[0][0] / i_cost_est_aq[0][0] over the frame-score MBs).  inv_qscale                 \
 * [f*mbw*mbh + mb] (i_inv_qscale_factor) or NULL when AQ is off; row_satd and                    \
 * cost_est may be NULL.  Every MB is computed (the do_edges case of                              \
 * slicetype.c:823-828).  Device arrays. */                                                       \
int x264hip_##BD##_lowres_intra_cost( const pixel *lowres, intptr_t stride,                     \
                                      intptr_t frame_stride, int mb_width, int mb_height,        \
                                      int n_frames, int satd, int all_modes, int lambda,         \
                                      const uint16_t *inv_qscale, uint16_t *intra_cost,          \
                                      int32_t *row_satd, int32_t *cost_est, void *stream );      \
                                                                                                \
/* the lookahead's lowres motion search for P frames: slicetype_mb_cost's inter                  \
 * leg (encoder/slicetype.c:514-713, 758-791 with b == p1, one list, no weights,                 \
 * a fresh search, the do_edges scan of slicetype.c:818-833 as one lookahead                     \
 * slice) with x264_me_search_ref / refine_subpel as the lookahead runs them                     \
 * (encoder/me.c:182-420, 774-790, 865-992; lowres_context_init                                  \
 * slicetype.c:45-61): me_method 0 = DIA, 1 = HEX; subme 2 or 4 (the lookahead's                 \
 * h->mb.i_subpel_refine); satd = the mbcmp choice (!lossless && param subme > 1);               \
 * me_range = param i_me_range; mv_range = param i_mv_range; lambda =                            \
 * x264_lambda_tab[X264_LOOKAHEAD_QP]; cost_mv = device pointer at mvd 0 of                      \
 * h->cost_mv[X264_LOOKAHEAD_QP] (analyse.c:143-157, valid over +-8*mv_range).                   \
 * For n_pairs (fenc, ref) pairs of lowres frames -- fenc = lowres[0] of frame b,                \
 * ref = lowres[0..3] (F, H, V, C) of frame p0, pointers at pixel (0,0), frame                   \
 * strides apart, common stride, 32 pixels of border, (0,0) and stride 4-byte                    \
 * aligned; the four planes equally spaced as x264's buffer_lowres (frame.c:281)                 \
 * are read in place, other layouts are first gathered into a stream-ordered scratch -- \
 * and intra_cost[f*mbs + mb] from lowres_intra_cost, writes                                     \
 * fenc->lowres_mvs (mvs[2*(f*mbs + mb)]), lowres_mv_costs (mv_costs), lowres_costs               \
 * ((list_used << 14) + cost), the AQ-scaled inter row sums row_satd[f*mbh + y]                  \
 * (i_row_satds[b-p0][0]) and est[3f..3f+2] = cost_est, cost_est_aq, intra_mbs.                  \
 * inv_qscale NULL = AQ off; row_satd / est may be NULL.  Synchronous: the call waits            \
 * for the kernel and returns X264HIP_EDEVICE ("timed out", outputs invalid) if a band's         \
 * wait for the band below it ran out (a broken dispatch-order premise, never a normal run). */  \
int x264hip_##BD##_lowres_inter_cost( const pixel *fenc, intptr_t fenc_frame_stride,             \
                                      const pixel *ref_f, const pixel *ref_h,                     \
                                      const pixel *ref_v, const pixel *ref_c, intptr_t stride,   \
                                      intptr_t ref_frame_stride, int mb_width, int mb_height,    \
                                      int n_pairs, int me_method, int subme, int satd,           \
                                      int me_range, int mv_range, int lambda,                    \
                                      const uint16_t *cost_mv, const uint16_t *intra_cost,       \
                                      const uint16_t *inv_qscale, int16_t *mvs,                  \
                                      int32_t *mv_costs, uint16_t *lowres_costs,                 \
                                      int32_t *row_satd, int32_t *est, void *stream );           \
                                                                                                \
/* lowres_inter_cost with a weighted reference and lookahead slices:                              \
 * weighted reference (slicetype.c:603-614 when                                                  \
 * x264_weights_analyse( h, fenc, frames[p0], 1 ) picked fenc->weight[0][0],                     \
 * slicetype.c:859-862; weightp SMART is the default, common/base.c:452): the integer-pel        \
 * stage reads ref_w = fenc->weighted[0] (the F plane scaled by weight_scale_plane,              \
 * slicetype.c:490-499; same stride and frame stride as ref_f), the subpel get_refs weight the   \
 * unweighted hpel planes with m->weight = (w_scale, w_denom, w_offset) (mc.c:221-249,           \
 * mc_weight mc.c:117-137); the near-zero fast skip still reads ref_f (slicetype.c:680).         \
 * ref_w NULL = unweighted.  denom 0..7, scale and offset in [-128, 127].  n_slices =          \
 * param i_lookahead_threads (slicetype.c:901-918): slice i covers MB rows                        \
 * [(H*i + T/2)/T, (H*(i+1) + T/2)/T) and is scanned on its own, its last row without             \
 * row-below predictors (slicetype.c:664, i_threadslice_end); every slice runs in parallel on     \
 * the GPU (1 = lowres_inter_cost's single slice). */                                           \
int x264hip_##BD##_lowres_inter_cost_ex( const pixel *fenc, intptr_t fenc_frame_stride,          \
                                         const pixel *ref_f, const pixel *ref_h,                  \
                                         const pixel *ref_v, const pixel *ref_c, intptr_t stride, \
                                         intptr_t ref_frame_stride, int mb_width, int mb_height, \
                                         int n_pairs, int me_method, int subme, int satd,        \
                                         int me_range, int mv_range, int lambda,                 \
                                         const uint16_t *cost_mv, const uint16_t *intra_cost,    \
                                         const uint16_t *inv_qscale, int16_t *mvs,               \
                                         int32_t *mv_costs, uint16_t *lowres_costs,              \
                                         int32_t *row_satd, int32_t *est, const pixel *ref_w,    \
                                         int w_scale, int w_denom, int w_offset, int n_slices,   \
                                         void *stream );                                         \
                                                                                                \
/* x264_weight_scale_plane (common/frame.c:825-842) for n_frames planes: dst = mc_weight(src)    \
 * over the width x height region at the pointers (the reference weights 16-wide strips while   \
 * x < width-8 and one 8-wide strip after, so up to 7 columns past width are written too);      \
 * for the lookahead, src = the lowres F plane's top-left border pixel (-32, -32), width =       \
 * lowres width + 64, height = lowres height + 64.  dst != src. */                               \
int x264hip_##BD##_weight_scale_plane( pixel *dst, intptr_t dst_stride, intptr_t dst_frame_stride, \
                                       const pixel *src, intptr_t src_stride,                    \
                                       intptr_t src_frame_stride, int width, int height,         \
                                       int n_frames, int scale, int denom, int offset,           \
                                       void *stream );                                           \
                                                                                                \
/* the lookahead's B-frame costs: slicetype_mb_cost with b_bidir (p0 < b < p1,                    \
 * slicetype.c:514-713, 758-791) for n triplets: fenc = lowres[0] of frame b, ref_a /            \
 * ref_b = the four lowres planes (F, H, V, C) of p0 / p1, each with its own frame stride         \
 * (0 = one reference for the whole batch).  List l (0 = p0, 1 = p1) is searched as in          \
 * lowres_inter_cost when search & (1 << l) -- writing mvs_l / costs_l                           \
 * (fenc->lowres_mvs[l] / lowres_mv_costs[l]) -- else read from them.  p1_mvs =                   \
 * fref1->lowres_mvs[0][p1-p0-1] (NULL when p1 was not searched against p0: dmv = 0);            \
 * dist_scale_factor and bipred_weight (i_bipred_weight in [0, 64]) as slicetype.c:529,868.       \
 * Writes lowres_costs ((list_used << 14) + cost, fenc->lowres_costs[b-p0][p1-b]),               \
 * row_satd[f*mbh + y] and est[2f..2f+1] = cost_est, cost_est_aq.  Other parameters as           \
 * lowres_inter_cost. */                                                                         \
int x264hip_##BD##_lowres_bidir_cost( const pixel *fenc, intptr_t fenc_frame_stride,             \
                                      const pixel *ref_a_f, const pixel *ref_a_h,                 \
                                      const pixel *ref_a_v, const pixel *ref_a_c,                 \
                                      intptr_t ref_a_frame_stride, const pixel *ref_b_f,          \
                                      const pixel *ref_b_h, const pixel *ref_b_v,                 \
                                      const pixel *ref_b_c, intptr_t ref_b_frame_stride,          \
                                      intptr_t stride, int mb_width, int mb_height, int n,        \
                                      int me_method, int subme, int satd, int me_range,          \
                                      int mv_range, int lambda, const uint16_t *cost_mv,          \
                                      int search, int16_t *mvs0, int32_t *costs0, int16_t *mvs1,  \
                                      int32_t *costs1, const int16_t *p1_mvs,                    \
                                      int dist_scale_factor, int bipred_weight,                   \
                                      const uint16_t *inv_qscale, uint16_t *lowres_costs,         \
                                      int32_t *row_satd, int32_t *est, void *stream );           \
/* lowres_bidir_cost over n_slices lookahead slices (as lowres_inter_cost_ex) */               \
int x264hip_##BD##_lowres_bidir_cost_ex( const pixel *fenc, intptr_t fenc_frame_stride,          \
                                         const pixel *ref_a_f, const pixel *ref_a_h,              \
                                         const pixel *ref_a_v, const pixel *ref_a_c,              \
                                         intptr_t ref_a_frame_stride, const pixel *ref_b_f,       \
                                         const pixel *ref_b_h, const pixel *ref_b_v,              \
                                         const pixel *ref_b_c, intptr_t ref_b_frame_stride,       \
                                         intptr_t stride, int mb_width, int mb_height, int n,     \
                                         int me_method, int subme, int satd, int me_range,       \
                                         int mv_range, int lambda, const uint16_t *cost_mv,       \
                                         int search, int16_t *mvs0, int32_t *costs0,              \
                                         int16_t *mvs1, int32_t *costs1, const int16_t *p1_mvs,  \
                                         int dist_scale_factor, int bipred_weight,                \
                                         const uint16_t *inv_qscale, uint16_t *lowres_costs,      \
                                         int32_t *row_satd, int32_t *est, int n_slices,           \
                                         void *stream );                                          \
                                                                                                \
/* ESA integral image of n_frames luma planes (x264_frame_filter, mc.c:748-782;                 \
 * integral_init* mc.c:424-456): plane / integral point at (0,0), rows                          \
 * [-32, lines+32) with common stride; row starts at x = -padh (PADH_ALIGN,                     \
 * frame.h:34).  Writes the 8x8 box sums of rows [1-32, lines+32-8) and columns                 \
 * [-padh, stride-padh-8) -- the values the reference leaves there -- and, when                 \
 * sub8x8, the 4x4 box sums in the second plane at +stride*(lines+64). */                        \
int x264hip_##BD##_frame_integral( const pixel *plane, intptr_t stride, intptr_t frame_stride,  \
                                   int lines, int padh, int sub8x8, int n_frames,               \
                                   uint16_t *integral, intptr_t integral_frame_stride,          \
                                   void *stream );                                              \
                                                                                                \
/* exhaustive integer-pel search table (the candidate set of reference                          \
 * encoder/me.c:618-631 before mv costs).  For every 16x16 macroblock of                        \
 * n_frames (fenc, ref) pairs:                                                                  \
 *   table[((f*mb_height + mby)*mb_width + mbx)*(2*range+1)*P + j*P + i]                          \
 *     = sad_16x16( fenc_f + 16*(mby*fenc_stride + mbx), fenc_stride,                           \
 *                  ref_f + (16*mby + j - range)*ref_stride + 16*mbx + i - range, ref_stride )   \
 * for 0 <= i,j <= 2*range, i.e. mx = i - range, my = j - range, raster order                   \
 * my-major, row pitch P = (2*range+1 + 3) & ~3 (entries i > 2*range are padding;              \
 * the 8-bit kernel stores the SADs of mx = range+1.. there).  ref must be a                    \
 * padded plane (x264 PADH/PADV = 32, reference common/frame.h:32-35); every                    \
 * window row is read from x-range to x+15+range+8, so the caller keeps                        \
 * range+8 <= the horizontal padding (PADH = 32).  range is one of 4, 8, 16, 24. */             \
int x264hip_##BD##_me_search_full( const pixel *fenc, intptr_t fenc_stride,                     \
                                   intptr_t fenc_frame_stride,                                  \
                                   const pixel *ref, intptr_t ref_stride,                       \
                                   intptr_t ref_frame_stride,                                   \
                                   int mb_width, int mb_height, int n_frames, int range,        \
                                   sadt *table, void *stream );                                 \
                                                                                                \
/* 8x8 quadrant tables (uint16 at both depths: an 8x8 SAD is <= 65472 at 10 bit):               \
 * table8[mb][q][j][i] =                                                                         \
 * sad_8x8 of quadrant q of the MB (0 top-left, 1 top-right, 2 bottom-left, 3 bottom-right)      \
 * at mv (i - range, j - range), row pitch (2*range+1+3)&~3, MBs frame-major.  The 16x16         \
 * SAD is the sum of the four, PIXEL_16x8's two halves are q0+q1 / q2+q3 and PIXEL_8x16's        \
 * q0+q2 / q1+q3: the exhaustive windows of every partition me.c's ESA / TESA searches           \
 * (me.c:618-771; analyse.c:1425,1480,1546) from the absdiffs of one 16x16 search.  range       \
 * 4, 8, 16 or 24. */                                                                            \
int x264hip_##BD##_me_search_full8( const pixel *fenc, intptr_t fenc_stride,                    \
                                    intptr_t fenc_frame_stride,                                 \
                                    const pixel *ref, intptr_t ref_stride,                      \
                                    intptr_t ref_frame_stride,                                  \
                                    int mb_width, int mb_height, int n_frames, int range,       \
                                    uint16_t *table8, void *stream );                           \
                                                                                                \
/* full search of me.c's ESA window around a per-MB centre (me.c centres its window on the    \
 * best predictor, encoder/me.c:618-626): centre[2*mb..] = (cx, cy) full-pel, MBs in          \
 * frame-major raster order.  The window origin (cx - range, cy - range) is clamped so every  \
 * fetched pixel stays inside the 32-pixel padding (PADH = PADV = 32, frame.h:32-33) and      \
 * aligned down to 4 (8 bit) / 2 (10 bit) pixels; origin[2*mb..] receives it (mv of table     \
 * column 0 and row 0).  table[mb][j][i] = SAD at mv (origin + (i, j)) for j < 2*range+1 rows \
 * and i < P = x264hip_me_table_pitch( BD, range, 1 ) columns: align4(2*range+6) at 8 bit,    \
 * 2*range+4 at 10 bit -- the columns [cx - range, cx + range + 2] me.c's width-rounded       \
 * window (max_x - min_x + 3) & ~3 can reach, whatever the alignment.  So a window of radius  \
 * range = me_range holds every candidate of me.c's ESA around that centre. */              \
int x264hip_##BD##_me_search_centred( const pixel *fenc, intptr_t fenc_stride,                  \
                                      intptr_t fenc_frame_stride,                               \
                                      const pixel *ref, intptr_t ref_stride,                    \
                                      intptr_t ref_frame_stride,                                \
                                      int mb_width, int mb_height, int n_frames, int range,     \
                                      const int16_t *centre, sadt *table, int16_t *origin,      \
                                      void *stream );                                           \
                                                                                                \
/* me_esa_argmin over a me_search_centred table: origin[2*i..] as written by it.  Centred on   \
 * the predictor (bmx, bmy) with range >= me_range (else X264HIP_EINVAL) the table holds me.c's \
 * whole width-rounded window. */                                                              \
int x264hip_##BD##_me_esa_argmin_at( const sadt *table, int range, int n, int me_range,         \
                                     const int16_t *origin, const int16_t *par,                 \
                                     const int32_t *init_cost, const uint16_t *cost_mv,         \
                                     int32_t *out, void *stream );                              \
                                                                                                \
/* plane SSD of n_frames (pix1, pix2) pairs: ssd[f] = x264_pixel_ssd_wxh( pf, pix1 + f*f1,       \
 * s1, pix2 + f*f2, s2, width, height ) (reference common/pixel.c:112-151, the per-frame       \
 * PSNR sum of encoder.c:2499).  uint64 results, device pointers; strides in pixels. */        \
int x264hip_##BD##_ssd_plane_batch( const pixel *pix1, intptr_t stride1, intptr_t frame_stride1, \
                                    const pixel *pix2, intptr_t stride2, intptr_t frame_stride2, \
                                    int width, int height, int n_frames, uint64_t *ssd,         \
                                    void *stream );                                             \
                                                                                                \
/* interleaved-chroma SSD: ssd_uv[2*f], ssd_uv[2*f+1] = the ssd_u, ssd_v of                    \
 * x264_pixel_ssd_nv12( pf, pix1 + f*f1, s1, pix2 + f*f2, s2, width, height, .. )             \
 * (reference common/pixel.c:153-178, including its tail over width&7 pairs that starts at     \
 * pixel offset width&~7); width = chroma samples per plane row. */                           \
int x264hip_##BD##_ssd_nv12_batch( const pixel *pix1, intptr_t stride1, intptr_t frame_stride1, \
                                   const pixel *pix2, intptr_t stride2, intptr_t frame_stride2, \
                                   int width, int height, int n_frames, uint64_t *ssd_uv,      \
                                   void *stream );                                              \
                                                                                                \
/* Fused full search + ESA decision: me_search_centred around each MB's predictor        \
 * (centre = par[8*i+0..1]) and me_esa_argmin_at over that window in one pass, the SAD     \
 * table never written (reference encoder/me.c:618-631).  par / init_cost / cost_mv / out   \
 * as me_esa_argmin_at: out[3*i] = { cost, mx, my }.  range is 4, 8, 16 or 24 and at least  \
 * me_range (the search costs (2*range+1) rows of the centred table's columns: pick the     \
 * smallest, range = me_range for x264's default merange 16). */                            \
int x264hip_##BD##_me_search_esa( const pixel *fenc, intptr_t fenc_stride, intptr_t fenc_frame_stride, \
                                  const pixel *ref, intptr_t ref_stride, intptr_t ref_frame_stride,   \
                                  int mb_width, int mb_height, int n_frames, int range, int me_range, \
                                  const int16_t *par, const int32_t *init_cost,                       \
                                  const uint16_t *cost_mv, int32_t *out, void *stream );              \
                                                                                                \
/* ESA decisions of every MB's eight sub-partitions (reference encoder/me.c:618-631 for      \
 * PIXEL_16x8 top / bottom, 8x16 left / right, 8x8 TL / TR / BL / BR -- partition p of MB mb at \
 * index i = 8*mb + p, the block offsets of analyse.c:1425,1480,1546): par[8*i] / init_cost[i] \
 * / cost_mv / out[3*i] = { cost, mx, my } as me_esa_argmin, per partition (each its own       \
 * window, mvp and predictor).  The partitions share their absdiffs (a partition's SAD is the   \
 * sum of the MB's 8x8 quadrant SADs) over a template of radius range (4, 8, 16, 24) around     \
 * centre[2*mb..] (full-pel; NULL = mv 0) with me_search_centred's origin; a partition whose  \
 * window reaches outside it gets the rest of its window from direct SADs, so the decisions     \
 * are me.c's for any inputs, fastest when the partitions' windows are centred on the MB's      \
 * (centre = the 16x16 decision, range = me_range).  range 0 takes every candidate directly.    \
 * me_range <= 30; fenc / ref / strides dword aligned; every                                   \
 * window (width-rounded) must lie inside the padded ref plane. */                              \
int x264hip_##BD##_me_search_esa8( const pixel *fenc, intptr_t fenc_stride, intptr_t fenc_frame_stride, \
                                   const pixel *ref, intptr_t ref_stride, intptr_t ref_frame_stride,   \
                                   int mb_width, int mb_height, int n_frames, int range, int me_range, \
                                   const int16_t *centre, const int16_t *par,                          \
                                   const int32_t *init_cost, const uint16_t *cost_mv, int32_t *out,    \
                                   void *stream );                                                     \
                                                                                                \
/* TESA integer-pel search per 16x16 macroblock (reference encoder/me.c:653-748,              \
 * X264_ME_TESA with i_pixel = PIXEL_16x16): ads4 with threshold bsad*17>>4 over the ESA      \
 * integral image, the SAD threshold list (sad_thresh 10/11/12 by me_range), the halving      \
 * prune to me_range/2 candidates and COST_MV over the survivors with fpelcmp = satd          \
 * (satd != 0, mbcmp_init encoder.c:1411,1423-1424) or sad.  fenc / ref point at pixel (0,0) \
 * of frame 0 (MB-aligned fenc rows: dword-aligned); integral = frame_integral's 8x8 sums,    \
 * pixel (0,0) of frame 0, row stride = ref_stride (frame.c:273), frame stride                \
 * integral_frame_stride.  par / init_cost / cost_mv as me_esa_argmin (per MB, frame-major    \
 * raster).  table (optional, NULL = none): a me_search_full / me_search_centred table of     \
 * the same pairs (origin NULL for me_search_full); SADs inside it are read, the rest are     \
 * computed.  With no table and me_range <= 24 the call builds one around the predictors in   \
 * stream-ordered scratch (a memory pool the library owns per device; ~2.4 KB per MB at      \
 * me_range 16, 8 bit) and reads it: the same decisions, 2.6x faster than in-scan SADs.       \
 * out[4*i] = { cost, mx, my, number of COST_MV candidates }.  me_range 1..32; ref_stride     \
 * below 2^18 pixels (the scan addresses rows by 24-bit products), else X264HIP_EINVAL.       \
 * The ESA window, the width-rounded columns and their integral sums must lie inside the      \
 * padded planes (mv_limit_fpel keeps them there in the encoder). */                          \
int x264hip_##BD##_me_tesa( const pixel *fenc, intptr_t fenc_stride, intptr_t fenc_frame_stride,  \
                            const pixel *ref, intptr_t ref_stride, intptr_t ref_frame_stride,   \
                            const uint16_t *integral, intptr_t integral_frame_stride,           \
                            int mb_width, int mb_height, int n_frames, int me_range, int satd,  \
                            const sadt *table, int range, const int16_t *origin,                \
                            const int16_t *par, const int32_t *init_cost,                       \
                            const uint16_t *cost_mv, int32_t *out, void *stream );              \
                                                                                                \
/* integer-pel ESA decision per macroblock over a me_search_full table (reference            \
 * encoder/me.c:618-631, the plain exhaustive form its ads path :632-771 reproduces):           \
 * par[8*i] = { bmx, bmy (fullpel centre = best predictor), mvp_x, mvp_y (qpel),                \
 *              mv_x_min, mv_y_min, mv_x_max, mv_y_max (mv_limit_fpel, analyse.c:330-349) };    \
 * the window is [max(bmx-me_range, mv_x_min), ..] with width rounded as                        \
 * (max_x - min_x + 3) & ~3, cost = sad + cost_mv[4*mx - mvp_x] + cost_mv[4*my - mvp_y]         \
 * (cost_mv: x264's h->cost_mv[qp], pointer at mvd 0), strict-< update from                     \
 * (init_cost[i], bmx, bmy) in my-major raster order.  out[3*i] = {cost, mx, my}.               \
 * The window must lie inside the table's [-range, range + 3] square.  n = #MBs. */             \
int x264hip_##BD##_me_esa_argmin( const sadt *table, int range, int n, int me_range,            \
                                  const int16_t *par, const int32_t *init_cost,                 \
                                  const uint16_t *cost_mv, int32_t *out, void *stream );        \
                                                                                                \
/* half-pel planes (reference x264_frame_filter common/mc.c:704-726 over the                 \
 * whole frame, hpel_filter mc.c:173-196, then x264_frame_expand_border_filtered               \
 * common/frame.c:599-625): for n_frames padded planes (PAD = 32, pointers at                   \
 * pixel (0,0) of frame 0, common stride and frame stride) writes the H, V and                  \
 * centre planes over [-32, width+32) x [-32, height+32).  width, height: whole MBs. */          \
int x264hip_##BD##_hpel_filter( const pixel *src, pixel *dst_h, pixel *dst_v, pixel *dst_c,     \
                                intptr_t stride, intptr_t frame_stride, int width, int height,  \
                                int n_frames, void *stream );                                   \
                                                                                                \
/* quarter-pel candidate costs of refine_subpel (reference encoder/me.c:865-992):               \
 * scores[i] = op( fenc + fenc_off[i], fenc_stride, get_ref(qx, qy) ) with op                   \
 * X264HIP_CMP_SAD or X264HIP_CMP_SATD of size i_pixel and get_ref the unweighted               \
 * reference MC (mc.c:221-249, pixel_avg of two half-pel planes): (qx, qy) =                   \
 * qpel_xy[2i], qpel_xy[2i+1] is the block's top-left in quarter pixels of the                  \
 * plane (4*x + mvx).  planes: full-pel, H, V, centre, all with ref_stride. */                  \
int x264hip_##BD##_subpel_cmp_batch( int op, int i_pixel, const pixel *fenc,                    \
                                     intptr_t fenc_stride, const pixel *fpel,                   \
                                     const pixel *hpel_h, const pixel *hpel_v,                  \
                                     const pixel *hpel_c, intptr_t ref_stride,                  \
                                     const int64_t *fenc_off, const int32_t *qpel_xy,           \
                                     int n, int32_t *scores, void *stream );                    \
                                                                                                \
/* the 3x3 quarter-pel neighbourhood of a centre: for block i with fenc at                      \
 * fenc + fenc_off[i] and centre (cx, cy) = centre_xy[2i], centre_xy[2i+1] (quarter             \
 * pixels, as qpel_xy above), scores[9i + 3(dy+1) + (dx+1)] = op of the candidate               \
 * (cx+dx, cy+dy), dx, dy in -1..1 -- refine_subpel's quarter-pel diamond around the            \
 * half-pel winner plus its corners (reference encoder/me.c:950-963).  Equal to nine            \
 * subpel_cmp_batch candidates; a half-pel centre (even cx, cy) is the fast case                \
 * (the nine predictions from one set of register windows).  i_pixel 16x16..8x8. */             \
int x264hip_##BD##_subpel_qpel9_batch( int op, int i_pixel, const pixel *fenc,                  \
                                       intptr_t fenc_stride, const pixel *fpel,                 \
                                       const pixel *hpel_h, const pixel *hpel_v,                \
                                       const pixel *hpel_c, intptr_t ref_stride,                \
                                       const int64_t *fenc_off, const int32_t *centre_xy,       \
                                       int n, int32_t *scores, void *stream );                  \
                                                                                                \
/* refine_subpel (reference encoder/me.c:865-992) for n partitions of size i_pixel (16x16 ..   \
 * 4x4, PIXEL_16x16 .. PIXEL_4x4 = 0 .. 6) of n_frames (fenc, ref) pairs: the subpel stage      \
 * x264_me_search_ref runs                                                                      \
 * after its integer search (refine_qpel = 0: subpel_iterations[subme][2..3], me.c:791-797) or   \
 * x264_me_refine_qpel (refine_qpel = 1: [0..1], me.c:801-810) -- the halfpel diamond of         \
 * fpelcmp over get_ref blocks (SAD; SATD when fpel_satd, i.e. TESA, and subme > 1,              \
 * encoder.c:1423-1426), the SATD re-score of its winner, the quarterpel diamond of              \
 * mbcmp_unaligned (SATD for subme > 1) with the odir skip, or subme 1's single qpel diamond.   \
 * fenc: pixel (0,0) of frame 0 (frame stride fenc_frame_stride); fpel / hpel_h / hpel_v /      \
 * hpel_c: the reference's F plane and hpel_filter's planes, pixel (0,0) of frame 0, common     \
 * stride and frame stride.  pos[3*i] = { frame, x, y } (the partition's top-left pixel);        \
 * par[8*i] = { mvx, mvy (qpel start, m->mv), mvp_x, mvp_y, mv_min_spel x, y, mv_max_spel x, y  \
 * (h->mb.mv_min_spel / mv_max_spel) }; init_cost[i] = m->cost; cost_mv at mvd 0.                \
 * out[4*i] = { m->cost, m->mv[0], m->mv[1], m->cost_mv } (16-byte aligned); nevals (or NULL):  \
 * the reference's cmp calls per partition: luma SADs | luma SATDs << 16 | chroma mbcmp calls     \
 * << 24.  No multi-reference threshold (p_halfpel_thresh = NULL; see _me_search_ref_thresh /    \
 * _me_refine_qpel_refdupe).  This form is luma-only with                                        \
 * unweighted references; _ex takes x264hip_refine_ext_t (NULL = the same as this form): every  \
 * luma get_ref weighted by weight[0] (mc.c:221-249), and with b_chroma_me COST_MV_SATD's       \
 * chroma cost (mc_chroma + mbcmp[chromapix] of U then V, or get_ref + mbcmp_unaligned of the    \
 * U / V hpel planes at 4:4:4, weighted by weight[1] / weight[2]) added as the reference adds   \
 * it, including the SATD re-score of the hpel winner (me.c:925-929). */                         \
int x264hip_##BD##_me_refine_subpel( const pixel *fenc, intptr_t fenc_stride,                   \
                                     intptr_t fenc_frame_stride, const pixel *fpel,             \
                                     const pixel *hpel_h, const pixel *hpel_v,                  \
                                     const pixel *hpel_c, intptr_t ref_stride,                  \
                                     intptr_t ref_frame_stride, int i_pixel, int subme,         \
                                     int refine_qpel, int fpel_satd, const int32_t *pos,        \
                                     const int16_t *par, const int32_t *init_cost,              \
                                     const uint16_t *cost_mv, int n, int32_t *out,              \
                                     int32_t *nevals, void *stream );                           \
int x264hip_##BD##_me_refine_subpel_ex( const pixel *fenc, intptr_t fenc_stride,                \
                                        intptr_t fenc_frame_stride, const pixel *fpel,          \
                                        const pixel *hpel_h, const pixel *hpel_v,               \
                                        const pixel *hpel_c, intptr_t ref_stride,               \
                                        intptr_t ref_frame_stride, int i_pixel, int subme,      \
                                        int refine_qpel, int fpel_satd, const int32_t *pos,     \
                                        const int16_t *par, const int32_t *init_cost,           \
                                        const uint16_t *cost_mv, int n, int32_t *out,           \
                                        int32_t *nevals, const x264hip_refine_ext_t *ext,       \
                                        void *stream );                                         \
/* x264_me_refine_qpel_refdupe (reference encoder/me.c:812-815): refine_subpel with no halfpel   \
 * iterations and min(2, subpel_iterations[subme][3]) quarterpel ones, the search analyse.c:1279- \
 * 1283 runs instead of x264_me_search_ref on a reference that duplicates reference 0 (par's mv  \
 * = reference 0's result, a->l0.mvc[0][0]; init_cost = m->cost as the caller's x264_me_t holds   \
 * it).  Arguments as me_refine_subpel_ex; halfpel_thresh / ref_cost as me_search_ref_thresh. */  \
int x264hip_##BD##_me_refine_qpel_refdupe( const pixel *fenc, intptr_t fenc_stride,             \
                                           intptr_t fenc_frame_stride, const pixel *fpel,       \
                                           const pixel *hpel_h, const pixel *hpel_v,            \
                                           const pixel *hpel_c, intptr_t ref_stride,            \
                                           intptr_t ref_frame_stride, int i_pixel, int subme,   \
                                           int fpel_satd, const int32_t *pos,                   \
                                           const int16_t *par, const int32_t *init_cost,        \
                                           const uint16_t *cost_mv, int n, int32_t *out,        \
                                           int32_t *nevals, int32_t *halfpel_thresh,            \
                                           const int32_t *ref_cost,                             \
                                           const x264hip_refine_ext_t *ext, void *stream );     \
                                                                                                \
/* x264_me_search_ref (reference encoder/me.c:182-798) for n partitions of size i_pixel (16x16 ..  \
 * 4x4; UMH on PIXEL_4x4 goes to the hexagon after its predictor diamonds, me.c:438-439) with     \
 * me_method X264_ME_DIA (0), X264_ME_HEX (1, x264's default, common/base.c:439),                 \
 * X264_ME_UMH (2) or X264_ME_ESA (3: the window of me.c:618-631 around the predictor stage's      \
 * winner, every candidate scored -- the decision the successive elimination of :750-768 also     \
 * reaches; nevals then counts the exhaustive form's calls; TESA stays with me_tesa): the          \
 * predictor checks over mvp and the mvc list (x264_predictor_clip /                              \
 * _roundclip, common/common.h:774-805), the integer search (UMH with its adaptive range), the    \
 * qpel conversion (me.c:774-789), then refine_subpel when subme >= 2 as me_refine_subpel_ex      \
 * runs it (ext: chroma ME, m->weight; weight[0] also weights the predictors' get_ref).           \
 * fpel_w = m->p_fref_w (the weighted F plane, the integer search's; = fpel unweighted); fpel /    \
 * hpel_*: m->p_fref.  pos[3*i] = { frame, x, y }; par[12*i] = { mvp_x, mvp_y (qpel),              \
 * h->mb.mv_limit_fpel min x, y, max x, y, mv_min_spel x, y, mv_max_spel x, y, i_mvc, 0 };         \
 * mvc[28*i + 2*k] = candidate k (qpel, k < i_mvc <= 14).  out[4*i] = { m->cost, m->mv[0],         \
 * m->mv[1], m->cost_mv } (16-byte aligned); nevals (or NULL) = int32 [n][2]: the integer stage's  \
 * fpelcmp calls | get_ref calls << 16, then the refine's counts (me_refine_subpel's format).      \
 * p_halfpel_thresh = NULL here; me_search_ref_thresh below takes it.                           \
 * me_range 4 .. 64. */                                                                          \
int x264hip_##BD##_me_search_ref( const pixel *fenc, intptr_t fenc_stride,                      \
                                  intptr_t fenc_frame_stride, const pixel *fpel_w,              \
                                  const pixel *fpel, const pixel *hpel_h, const pixel *hpel_v,  \
                                  const pixel *hpel_c, intptr_t ref_stride,                     \
                                  intptr_t ref_frame_stride, int i_pixel, int me_method,        \
                                  int subme, int me_range, const int32_t *pos,                  \
                                  const int16_t *par, const int16_t *mvc,                       \
                                  const uint16_t *cost_mv, int n, int32_t *out,                 \
                                  int32_t *nevals, const x264hip_refine_ext_t *ext,             \
                                  void *stream );                                               \
/* x264's P16x16 reference-0 analysis of whole frames with the encoder's own predictors: for every \
 * MB in raster order (analyse.c x264_mb_analyse_inter_p16x16), mvp = x264_mb_predict_mv_16x16      \
 * (common/mvpred.c:129-157) and mvc = x264_mb_predict_mv_ref16x16 (mvpred.c:519-600, P slice,     \
 * no MBAFF: lowres_mv[mb] doubled when lowres_mv (the lookahead's field of the pair, int16        \
 * [n_frames][mb_width*mb_height][2]; 0x7fff in a frame's first entry = none) is given; the left,  \
 * top, top-left and top-right MBs' 16x16 mvs, mv 0 off the frame; then, when ref_mv (the          \
 * reference's mv16x16 field, same layout) is given, its colocated / right / below mvs scaled as   \
 * clip3((mv * ref_mv_scale + 128) >> 8) with ref_mv_scale = (curpoc - refpoc) * inv_ref_poc), the \
 * mv limits of analyse.c:330-349 (mv_range = i_mv_range in pixels), then x264_me_search_ref as   \
 * x264hip_*_me_search_ref runs it (PIXEL_16x16).  Every MB is taken as P_L0 16x16 with its       \
 * searched mv (the neighbours' mvs = their search results).  The raster dependency runs as a      \
 * wavefront of MB anti-diagonals (x + 2y): one predictor launch and one search launch per       \
 * diagonal, n_frames frames each.  out[4*(f*mb_width*mb_height + mb)] = { m->cost, mvx, mvy,       \
 * cost_mv } (raster); nevals (or NULL) as me_search_ref's.  Other arguments as me_search_ref. */  \
int x264hip_##BD##_me_analyse_p16x16( const pixel *fenc, intptr_t fenc_stride,                  \
                                      intptr_t fenc_frame_stride, const pixel *fpel_w,          \
                                      const pixel *fpel, const pixel *hpel_h,                   \
                                      const pixel *hpel_v, const pixel *hpel_c,                 \
                                      intptr_t ref_stride, intptr_t ref_frame_stride,           \
                                      int mb_width, int mb_height, int n_frames, int me_method, \
                                      int subme, int me_range, int mv_range,                    \
                                      const int16_t *lowres_mv, const int16_t *ref_mv,          \
                                      int ref_mv_scale, const uint16_t *cost_mv, int32_t *out,  \
                                      int32_t *nevals, const x264hip_refine_ext_t *ext,         \
                                      void *stream );                                           \
/* x264_me_refine_bidir_satd (reference encoder/me.c:994-1183, rd = 0) for n bipred partitions   \
 * of size i_pixel (16x16 .. 8x8) -- the 4-D diamond over (mv0, mv1) that refine_bidir runs on   \
 * every B_BI_BI / D_BI_8x8 partition at subme >= 5 (analyse.c:2692-2730): up to 8 passes over   \
 * dia4d's 33 pairs, a pair's visited bit (coordinates mod 8) skipping it in later passes, each   \
 * pair scored as mc.avg[i_pixel]( list 0 get_ref, list 1 get_ref, i_weight ) (unweighted          \
 * references; i_weight 32 the rounding average, else the implicit-weight average, mc.c:49-99)   \
 * by mbcmp (SATD when mbcmp_satd, i.e. subme > 1, else SAD) plus the four mv costs.  The        \
 * early return when a mv lies within 8 qpel of the spel limits.  l0* / l1*: the list 0 / list 1  \
 * references' F, H, V, C planes at pixel (0,0) of frame 0 (common stride and frame stride;       \
 * pos's frame index steps both and fenc's).  pos[3*i] = { frame, x, y }; par[12*i] = { m0 mv x,  \
 * y, m1 mv x, y, m0 mvp x, y, m1 mvp x, y, mv_min_spel x, y, mv_max_spel x, y }; weight[i] =       \
 * i_weight (h->mb.bipred_weight).  out[4*i] = { m0 mv x, y, m1 mv x, y } (16-byte aligned);       \
 * cost (or NULL) = the last bcost (internal in the reference; 1 << 28 after the early return);    \
 * nevals (or NULL) = mbcmp calls | passes << 16. */                                               \
int x264hip_##BD##_me_refine_bidir_satd( const pixel *fenc, intptr_t fenc_stride,                \
                                         intptr_t fenc_frame_stride, const pixel *l0_fpel,      \
                                         const pixel *l0_hpel_h, const pixel *l0_hpel_v,        \
                                         const pixel *l0_hpel_c, const pixel *l1_fpel,          \
                                         const pixel *l1_hpel_h, const pixel *l1_hpel_v,        \
                                         const pixel *l1_hpel_c, intptr_t ref_stride,           \
                                         intptr_t ref_frame_stride, int i_pixel,                \
                                         int mbcmp_satd, const int32_t *pos,                    \
                                         const int16_t *par, const int32_t *weight,             \
                                         const uint16_t *cost_mv, int n, int32_t *out,          \
                                         int32_t *cost, int32_t *nevals, void *stream );        \
/* me_search_ref with the multi-reference early exit, x264_me_search_ref( ..., p_halfpel_thresh ) \
 * (reference me.c:931-944 inside refine_subpel; x264's default ref = 3 with b_early_terminate,  \
 * common/base.c:384, encoder/analyse.c:303, 1260-1261): halfpel_thresh = int32 [n], partition i's \
 * i_halfpel_thresh (INT_MAX before its MB's first reference), read and written in place;        \
 * ref_cost = int32 [n] (or NULL = 0), the partition's i_ref_cost for this reference -- the      \
 * threshold is held less it during the search, as analyse.c:1271 / 1310 do around the call.     \
 * The caller chains one MB's references as one launch per reference.  When the exit fires the  \
 * refine returns before its quarterpel diamond with m->cost, m->mv written and m->cost_mv left   \
 * as it was: out[4*i+3] keeps what the caller stored there.  halfpel_thresh = NULL is            \
 * me_search_ref.  Only subme >= 2 runs the refine (and so reads the threshold), as me.c:792. */  \
int x264hip_##BD##_me_search_ref_thresh( const pixel *fenc, intptr_t fenc_stride,               \
                                         intptr_t fenc_frame_stride, const pixel *fpel_w,       \
                                         const pixel *fpel, const pixel *hpel_h,                \
                                         const pixel *hpel_v, const pixel *hpel_c,              \
                                         intptr_t ref_stride, intptr_t ref_frame_stride,        \
                                         int i_pixel, int me_method, int subme, int me_range,   \
                                         const int32_t *pos, const int16_t *par,                \
                                         const int16_t *mvc, const uint16_t *cost_mv, int n,    \
                                         int32_t *out, int32_t *nevals,                         \
                                         int32_t *halfpel_thresh, const int32_t *ref_cost,      \
                                         const x264hip_refine_ext_t *ext, void *stream );       \
                                                                                                \
/* block lists of the reference transforms (dct.c), device arrays;                             \
 * dct holds n consecutive outputs of the selected entry's size. */                             \
int x264hip_##BD##_sub_dct_batch( int kind, const pixel *fenc, intptr_t fenc_stride,            \
                                  const pixel *fdec, intptr_t fdec_stride,                      \
                                  const int64_t *fenc_off, const int64_t *fdec_off,             \
                                  int n, dctcoef *dct, void *stream );                          \
/* in-place DC transforms: DC_4x4 on n arrays d[16]; DC_2x4 on n pairs                          \
 * (dct[8] out, dct4x4[8][16] in/out) */                                                        \
int x264hip_##BD##_dc_batch( int kind, dctcoef *dct, dctcoef *dct4x4, int n, void *stream );    \
/* in-place quantisation of n blocks with one mf/bias set (device arrays of                     \
 * 16 or 64 udctcoef for 4x4/4x4x4/8x8; for the DC kinds mf[0]/bias[0] are the                  \
 * scalar int arguments of quant_4x4_dc / quant_2x2_dc).  nz[i] = the entry's                   \
 * return value (quant.c:59-104). */                                                            \
int x264hip_##BD##_quant_batch( int kind, dctcoef *dct, const udctcoef *mf,                     \
                                const udctcoef *bias, int n, int32_t *nz, void *stream );       \
int x264hip_##BD##_quant_dc_batch( int kind, dctcoef *dct, int mf, int bias,                    \
                                   int n, int32_t *nz, void *stream );                          \
                                                                                                \
/* fused inter-luma residual path of reference encoder/macroblock.c:806-884:                    \
 * per 16x16 macroblock, sub16x16_dct + 4x quant_4x4x4 (transform 4) or                         \
 * sub16x16_dct8 + 4x quant_8x8 (transform 8) of fenc - pred.  dct gets 256                     \
 * coefs per MB in the reference's dct4x4[16][16] / dct8x8[4][64] order; nz gets                \
 * per MB the 16-bit mask (bit 4*i8+i4 = 4x4 block nonzero, transform 4) or                     \
 * the 4-bit mask (bit i8, transform 8). */                                                     \
int x264hip_##BD##_mb_dct_quant( int transform, const pixel *fenc, intptr_t fenc_stride,        \
                                 intptr_t fenc_frame_stride,                                    \
                                 const pixel *pred, intptr_t pred_stride,                       \
                                 intptr_t pred_frame_stride,                                    \
                                 int mb_width, int mb_height, int n_frames,                     \
                                 const udctcoef *mf, const udctcoef *bias,                      \
                                 dctcoef *dct, int32_t *nz, void *stream );                     \
                                                                                                \
/* ---- inverse path (reference common/dct.c, common/quant.c), device arrays ---- */            \
/* n calls of the add*_idct* entry `kind` (X264HIP_IDCT_*) on dst + dst_off[i]                  \
 * (stride dst_stride); call i's coefficients at dct + i*size; dct is not modified. */          \
int x264hip_##BD##_add_idct_batch( int kind, pixel *dst, intptr_t dst_stride,                   \
                                   const int64_t *dst_off, const dctcoef *dct, int n,           \
                                   void *stream );                                              \
/* in-place dequant_4x4 / 8x8 / 4x4_dc (X264HIP_DEQUANT_*) of n blocks; dequant_mf is           \
 * one list's int [6][16] or [6][64] (x264hip_cqm_dequant), qp[i] per block. */                 \
int x264hip_##BD##_dequant_batch( int kind, dctcoef *dct, const int32_t *dequant_mf,            \
                                  const int32_t *qp, int n, void *stream );                     \
/* idct_dequant_2x4_dc (dconly = 0: writes dct4x4[8][16] per call, 128 coefs apart)             \
 * or _dconly (dconly = 1: in place on dct[8]) for n calls, qp[i] per call. */                   \
int x264hip_##BD##_idct_dequant_2x4_batch( int dconly, dctcoef *dct, dctcoef *dct4x4,           \
                                           const int32_t *dequant_mf, const int32_t *qp,        \
                                           int n, void *stream );                               \
/* optimize_chroma_2x2_dc (c422 = 0, 4 coefs per call) / 2x4_dc (c422 = 1, 8 coefs):            \
 * in place, dequant_mf[i] per call, nz[i] = return value. */                                   \
int x264hip_##BD##_optimize_chroma_dc_batch( int c422, dctcoef *dct, const int32_t *dequant_mf, \
                                             int n, int32_t *nz, void *stream );                \
/* denoise_dct over n consecutive blocks of `size` coefficients sharing sum[size]               \
 * (accumulated) and offset[size]. */                                                           \
int x264hip_##BD##_denoise_dct_batch( dctcoef *dct, int size, int n, uint32_t *sum,             \
                                      const udctcoef *offset, void *stream );                   \
/* decimate_score / coeff_last (X264HIP_COEF_*) of n blocks `pitch` coefs apart. */             \
int x264hip_##BD##_coef_stat_batch( int kind, const dctcoef *dct, int64_t pitch, int n,         \
                                    int32_t *out, void *stream );                               \
/* coeff_level_run4/8/15/16 (num) of n blocks `pitch` coefs apart: last[i], mask[i],             \
 * count[i] (the return value) and level[18*i ..]. */                                           \
int x264hip_##BD##_coeff_level_run_batch( int num, const dctcoef *dct, int64_t pitch, int n,    \
                                          int32_t *last, int32_t *mask, int32_t *count,         \
                                          dctcoef *level, void *stream );                       \
/* zigzag_scan_4x4 (size 4) / 8x8 (size 8), frame or field order, n blocks. */                  \
int x264hip_##BD##_zigzag_scan_batch( int size, int field, dctcoef *level, const dctcoef *dct,  \
                                      int n, void *stream );                                    \
/* zigzag_sub_4x4 / 4x4ac / 8x8 (X264HIP_ZIGZAG_SUB_*): level (16 or 64 per call),              \
 * dc[i] (4x4ac only), nz[i]; dst block is overwritten with the src block. */                   \
int x264hip_##BD##_zigzag_sub_batch( int kind, int field, dctcoef *level, dctcoef *dc,          \
                                     const pixel *src, intptr_t src_stride, pixel *dst,         \
                                     intptr_t dst_stride, const int64_t *src_off,               \
                                     const int64_t *dst_off, int n, int32_t *nz, void *stream );\
/* zigzag_interleave_8x8_cavlc of n blocks (64 coefs in/out, 16 nnz bytes per call). */         \
int x264hip_##BD##_zigzag_interleave_batch( dctcoef *dst, const dctcoef *src, uint8_t *nnz,     \
                                            int n, void *stream );                              \
/* fused reconstruction of the inter luma residual (macroblock.c dequant + add16x16_idct /     \
 * add16x16_idct8): recon = clip( pred + idct( dequant( dct ) ) ) per MB, dct[mb][256] as      \
 * written by mb_dct_quant (unchanged), qp[mb] per MB, dequant_mf the list's [6][16|64]. */     \
int x264hip_##BD##_mb_dequant_idct_add( int transform, const dctcoef *dct, int mb_width,        \
                                        int mb_height, int n_frames, const int32_t *dequant_mf, \
                                        const int32_t *qp, const pixel *pred,                   \
                                        intptr_t pred_stride, intptr_t pred_frame_stride,       \
                                        pixel *recon, intptr_t recon_stride,                    \
                                        intptr_t recon_frame_stride, void *stream );               \
                                                                                                \
/* x264_pixel_ssim_wxh (common/pixel.c:690-714) of two planes (device pointers at the region's  \
 * top-left, as encoder.c:2517-2528 passes them): *ssim (device float) = the reference's float  \
 * sum, accumulated in its order (bit-identical), *cnt (host, may be NULL) = its window count.  \
 * Reads 4x4 blocks up to column 4*(width/4) - 1 and row 4*(height/4) - 1. */                    \
int x264hip_##BD##_ssim_wxh( const pixel *pix1, intptr_t stride1, const pixel *pix2,            \
                             intptr_t stride2, int width, int height, float *ssim, int *cnt,    \
                             void *stream );                                                    \
                                                                                                \
/* the encoder's SSIM (encoder.c:2516-2528): x264_pixel_ssim_wxh of every filtered MB-row band  \
 * of n_frames frame pairs in one launch.  pix1 / pix2: the planes at the bands' left column     \
 * (plane + 2 as the encoder passes them), frame strides step the frames; bands: device int32    \
 * pairs (first row, height) relative to pix1 / pix2 -- per MB row mb_y of a thread slice         \
 * [start, end): min_y = mb_y - 1, first = 16*min_y - 4*!b_start + (b_start ? 2 : -6),           \
 * last = min( 16*mb_y - 4*!b_end, i_height ), height = last - first (encoder.c:2412-2420,       \
 * 2490, 2520) -- all of width `width` (i_width - 2).  ssim (device float[n_frames * n_bands]) =   \
 * each band's float, bit-identical to the reference's; the band's window count is              \
 * (height/4 - 1) * (width/4 - 1).  width <= 8192. */                                            \
int x264hip_##BD##_ssim_bands( const pixel *pix1, intptr_t stride1, intptr_t frame_stride1,      \
                               const pixel *pix2, intptr_t stride2, intptr_t frame_stride2,      \
                               int width, const int32_t *bands, int n_bands, int n_frames,       \
                               float *ssim, void *stream );                                      \
                                                                                                \
/* the frame statistics x264_weights_analyse reads: fenc->i_pixel_sum[3] / i_pixel_ssd[3] as    \
 * x264_adaptive_quant_frame leaves them for a progressive frame (ac_energy_mb's stores,          \
 * encoder/ratecontrol.c:225-257, 289-299, then the mean removal of :406-414; the sum wraps as    \
 * its uint32 field does).  chroma_format 0 = 4:0:0, 1 = 4:2:0, 2 = 4:2:2 (chroma_u = the        \
 * interleaved NV12 / NV16 plane, chroma_v unused), 3 = 4:4:4 (chroma_u, chroma_v).  Planes      \
 * at pixel (0,0).  stats = device uint64[6]: sum[0..2] then ssd[0..2]. */                         \
int x264hip_##BD##_frame_pixel_stats( const pixel *luma, intptr_t luma_stride,                  \
                                      const pixel *chroma_u, const pixel *chroma_v,              \
                                      intptr_t chroma_stride, int mb_width, int mb_height,       \
                                      int chroma_format, uint64_t *stats, void *stream );        \
                                                                                                \
/* weight_cost_luma / weight_cost_chroma / weight_cost_chroma444 (slicetype.c:191-282) of      \
 * n_cands candidate weights in one batch: costs[i] (device uint32) = the reference's value    \
 * with cands[i] (host array) as w, i.e. including weight_slice_header_cost when                \
 * cands[i].weighted, and the unweighted (w == NULL) cost otherwise.  kind                      \
 * X264HIP_WCOST_*: LUMA -- fenc = fenc->lowres[0], ref[0..3] = ref->lowres[0..3] (only [0]     \
 * without mvs), stride = i_stride_lowres, intra_cost = fenc->i_intra_cost; CHROMA420/422 --    \
 * fenc / ref[0] = the NV12 / NV16 planes (plane 0 = U, 1 = V); CHROMA444 -- fenc / ref[0] =    \
 * one chroma plane.  mvs = fenc->lowres_mvs[0][ref0_distance] (NULL when its first entry is     \
 * 0x7FFF): the motion-compensated reference of weight_cost_init_luma / _chroma /               \
 * _chroma444 (slicetype.c:77-168) is formed on the fly; ref planes carry expanded borders.     \
 * satd = the mbcmp choice; lambda = x264_lambda_tab[X264_LOOKAHEAD_QP]; n_slices as            \
 * weight_slice_header_cost counts them. */                                                     \
int x264hip_##BD##_weight_cost_batch( int kind, const pixel *fenc, const pixel *const ref[4],   \
                                      intptr_t stride, int mb_width, int mb_height,             \
                                      const uint16_t *intra_cost, const int16_t *mvs, int satd,  \
                                      int plane, int lambda, int n_slices,                       \
                                      const x264hip_weight_t *cands, int n_cands,                \
                                      uint32_t *costs, void *stream );                           \
                                                                                                \
/* x264_weights_analyse( h, fenc, ref, b_lookahead ) (encoder/slicetype.c:284-501): the         \
 * explicit weights of ref for fenc, luma and (outside the lookahead, after a luma weight)      \
 * chroma.  fenc_lowres / ref_lowres[0..3] / lowres_stride / intra_cost / mvs as                \
 * weight_cost_batch's LUMA (intra_cost from lowres_intra_cost: the reference computes it       \
 * first when !fenc->b_intra_calculated, slicetype.c:364-369); fenc_chroma / ref_chroma =       \
 * { NV12 plane, NULL } or { U, V } (4:4:4), chroma_stride, unused in the lookahead;            \
 * fenc_sum .. ref_ssd = the frames' i_pixel_sum / i_pixel_ssd (frame_pixel_stats); subme =     \
 * param i_subpel_refine; satd = the mbcmp choice; weightp_fake = (i_weighted_pred ==           \
 * X264_WEIGHTP_FAKE).  Writes weights[3] (fenc->weight[0][0..2]), *cost_delta                   \
 * (fenc->f_weighted_cost_delta[i_delta_index], FAKE only, may be NULL) and, in the lookahead    \
 * with a luma weight, weighted_lowres (fenc->weighted[0]: at (0,0), lowres_stride, 32-pixel     \
 * border; NULL = skip) by x264_weight_scale_plane over columns [-32, width + 32) and the rows    \
 * of the 32-row border: the reference starts at buffer_lowres (-PADH_ALIGN, i.e. -64 at 8 bit,   \
 * slicetype.c:489-497), so columns [-PADH_ALIGN, -32), which no lowres search reads, keep       \
 * whatever the caller's buffer held.  Synchronous: every candidate of a plane                   \
 * is scored in one batch on the stream and the host replays the reference's search over the   \
 * costs (one stream synchronise for luma, one for chroma); not capturable. */                  \
int x264hip_##BD##_weights_analyse( const pixel *fenc_lowres, const pixel *const ref_lowres[4], \
                                    intptr_t lowres_stride, int mb_width, int mb_height,        \
                                    const uint16_t *intra_cost, const int16_t *mvs,             \
                                    int chroma_format, const pixel *const fenc_chroma[2],       \
                                    const pixel *const ref_chroma[2], intptr_t chroma_stride,   \
                                    const uint32_t fenc_sum[3], const uint64_t fenc_ssd[3],     \
                                    const uint32_t ref_sum[3], const uint64_t ref_ssd[3],       \
                                    int b_lookahead, int subme, int satd, int lambda,           \
                                    int n_slices, int weightp_fake, pixel *weighted_lowres,     \
                                    x264hip_weight_t weights[3], float *cost_delta,             \
                                    void *stream );                                             \
                                                                                                \
/* lookahead input: x264_frame_init_lowres (mc.c:458-507, frame.c:627-631) of n_frames          \
 * luma planes of width x height (i_width[0] x i_lines[0]; src at (0,0)): the four              \
 * half-resolution planes dst[0..3] (full-pel, H, V, centre) over [-32, width/2+32) x           \
 * [-32, height/2+32) with the reference's border replication; dst points at (0,0),            \
 * dst_stride a multiple of 4 bytes, (width/2+64) a multiple of 4/sizeof(pixel). */             \
int x264hip_##BD##_frame_init_lowres( const pixel *src, intptr_t stride, intptr_t frame_stride, \
                                      int width, int height, int n_frames, pixel *const dst[4], \
                                      intptr_t dst_stride, intptr_t dst_frame_stride,           \
                                      void *stream );

/* dequant4_mf [4][6][16] and dequant8_mf [2][6][64] of x264_cqm_init (reference
 * common/set.c:124-159) for the 8 scaling lists; bit-depth independent. */
void x264hip_cqm_dequant( const uint8_t *const scaling_list[8], int b_transform_8x8,
                          int32_t *dequant4_mf, int32_t *dequant8_mf );

X264HIP_DECLARE_ENTRIES( 8,  uint8_t,  int16_t, uint16_t, uint16_t )
X264HIP_DECLARE_ENTRIES( 10, uint16_t, int32_t, uint32_t, uint32_t )

#ifdef __cplusplus
}
#endif

#endif /* X264HIP_H */
