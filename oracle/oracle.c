/*****************************************************************************
 * oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference's
 * portable C kernels on the north-star path, used as the parity checker for
 * the HIP backend.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product (x264-i386pic_amd/) never does.
 *
 * PARITY UNPINNED: the reference (xrgtn/x264-i386pic) ships no golden vectors
 * for this path (checkasm is purely differential) and its C
 * path cannot be compiled here under the round rules (common/osdep.h:39
 * includes the configure-generated config.h).  This
 * file restates the algorithm from the reference sources, line by line in
 * semantics (never in text), and is cross-checked against an independent
 * matrix-form restatement in tests/numpy_ref.py.
 *
 * Compiled twice (BIT_DEPTH=8 / 10) like the reference (Makefile:309-313);
 * symbols are prefixed oracle8_ / oracle10_.
 *****************************************************************************/
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifndef BIT_DEPTH
#error "BIT_DEPTH must be 8 or 10"
#endif

#if BIT_DEPTH > 8
typedef uint16_t pixel;
typedef int32_t  dctcoef;
typedef uint32_t udctcoef;
typedef uint32_t sum_t;      /* reference common/pixel.c:233-239 */
typedef uint64_t sum2_t;
typedef uint32_t sadt;
#else
typedef uint8_t  pixel;
typedef int16_t  dctcoef;
typedef uint16_t udctcoef;
typedef uint16_t sum_t;
typedef uint32_t sum2_t;
typedef uint16_t sadt;
#endif
#define PIXEL_MAX ((1 << BIT_DEPTH) - 1)
#define BITS_PER_SUM (8 * sizeof(sum_t))
#define QP_MAX_SPEC (51 + 6 * (BIT_DEPTH - 8))   /* reference common/common.h:58-59 */
#define FENC_STRIDE 16                            /* reference common/common.h:570-571 */
#define FDEC_STRIDE 32

#define GLUE3_(a,b,c) a##b##c
#define GLUE3(a,b,c) GLUE3_(a,b,c)
#define FN(name) GLUE3(oracle, BIT_DEPTH, _##name)

static const uint8_t pixel_w[8] = { 16, 16, 8, 8, 8, 4, 4, 4 };   /* reference common/pixel.h:55-59 */
static const uint8_t pixel_h[8] = { 16, 8, 16, 8, 4, 8, 4, 16 };

static inline pixel clip_pixel( int x )
{
    return x < 0 ? 0 : x > PIXEL_MAX ? PIXEL_MAX : x;
}

/*============================================================================
 * pixel metrics — reference common/pixel.c
 *==========================================================================*/

/* PIXEL_SAD_C, reference common/pixel.c:55-70 */
int FN(sad)( int i_pixel, const pixel *pix1, intptr_t s1, const pixel *pix2, intptr_t s2 )
{
    int lx = pixel_w[i_pixel], ly = pixel_h[i_pixel];
    int sum = 0;
    for( int y = 0; y < ly; y++, pix1 += s1, pix2 += s2 )
        for( int x = 0; x < lx; x++ )
            sum += abs( pix1[x] - pix2[x] );
    return sum;
}

/* PIXEL_SSD_C, reference common/pixel.c:85-101 */
int FN(ssd)( int i_pixel, const pixel *pix1, intptr_t s1, const pixel *pix2, intptr_t s2 )
{
    int lx = pixel_w[i_pixel], ly = pixel_h[i_pixel];
    int sum = 0;
    for( int y = 0; y < ly; y++, pix1 += s1, pix2 += s2 )
        for( int x = 0; x < lx; x++ )
        {
            int d = pix1[x] - pix2[x];
            sum += d * d;
        }
    return sum;
}

/* x264_pixel_ssd_wxh, reference common/pixel.c:112-151: 16x16 tiles when both
 * pointers and strides are 16-aligned, else 8x16, one 8x8 row band, then the
 * per-pixel right and bottom tails */
uint64_t FN(ssd_wxh)( const pixel *pix1, intptr_t i_pix1, const pixel *pix2, intptr_t i_pix2, int i_width,
                      int i_height )
{
    uint64_t i_ssd = 0;
    int y;
    int align = !(((intptr_t)pix1 | (intptr_t)pix2 | i_pix1 | i_pix2) & 15);
    for( y = 0; y < i_height - 15; y += 16 )
    {
        int x = 0;
        if( align )
            for( ; x < i_width - 15; x += 16 )
                i_ssd += FN(ssd)( 0, pix1 + y * i_pix1 + x, i_pix1, pix2 + y * i_pix2 + x, i_pix2 );
        for( ; x < i_width - 7; x += 8 )
            i_ssd += FN(ssd)( 2, pix1 + y * i_pix1 + x, i_pix1, pix2 + y * i_pix2 + x, i_pix2 );
    }
    if( y < i_height - 7 )
        for( int x = 0; x < i_width - 7; x += 8 )
            i_ssd += FN(ssd)( 3, pix1 + y * i_pix1 + x, i_pix1, pix2 + y * i_pix2 + x, i_pix2 );
    if( i_width & 7 )
        for( y = 0; y < (i_height & ~7); y++ )
            for( int x = i_width & ~7; x < i_width; x++ )
            {
                int d = pix1[y * i_pix1 + x] - pix2[y * i_pix2 + x];
                i_ssd += d * d;
            }
    if( i_height & 7 )
        for( y = i_height & ~7; y < i_height; y++ )
            for( int x = 0; x < i_width; x++ )
            {
                int d = pix1[y * i_pix1 + x] - pix2[y * i_pix2 + x];
                i_ssd += d * d;
            }
    return i_ssd;
}

/* pixel_ssd_nv12_core + x264_pixel_ssd_nv12, reference common/pixel.c:153-178 (the
 * tail starts at pixel offset i_width&~7 of the interleaved row, as written there) */
static void ssd_nv12_core( const pixel *pixuv1, intptr_t stride1, const pixel *pixuv2, intptr_t stride2, int width,
                           int height, uint64_t *ssd_u, uint64_t *ssd_v )
{
    *ssd_u = 0, *ssd_v = 0;
    for( int y = 0; y < height; y++, pixuv1 += stride1, pixuv2 += stride2 )
        for( int x = 0; x < width; x++ )
        {
            int du = pixuv1[2*x] - pixuv2[2*x];
            int dv = pixuv1[2*x+1] - pixuv2[2*x+1];
            *ssd_u += du * du;
            *ssd_v += dv * dv;
        }
}

void FN(ssd_nv12)( const pixel *pix1, intptr_t i_pix1, const pixel *pix2, intptr_t i_pix2, int i_width,
                   int i_height, uint64_t *ssd_u, uint64_t *ssd_v )
{
    ssd_nv12_core( pix1, i_pix1, pix2, i_pix2, i_width & ~7, i_height, ssd_u, ssd_v );
    if( i_width & 7 )
    {
        uint64_t tmp[2];
        ssd_nv12_core( pix1 + (i_width & ~7), i_pix1, pix2 + (i_width & ~7), i_pix2, i_width & 7, i_height,
                       &tmp[0], &tmp[1] );
        *ssd_u += tmp[0];
        *ssd_v += tmp[1];
    }
}

/* HADAMARD4 and the packed two-lane abs, reference common/pixel.c:242-259 */
#define HADAMARD4( d0, d1, d2, d3, s0, s1, s2, s3 ) {\
    sum2_t t0 = s0 + s1, t1 = s0 - s1, t2 = s2 + s3, t3 = s2 - s3;\
    d0 = t0 + t2; d2 = t0 - t2; d1 = t1 + t3; d3 = t1 - t3; }

static inline sum2_t abs2( sum2_t a )
{
    sum2_t s = ((a >> (BITS_PER_SUM - 1)) & (((sum2_t)1 << BITS_PER_SUM) + 1)) * ((sum_t)-1);
    return (a + s) ^ s;
}

/* satd 4x4, packed horizontal pairs; reference common/pixel.c:265-288 */
static int satd_4x4( const pixel *pix1, intptr_t i1, const pixel *pix2, intptr_t i2 )
{
    sum2_t tmp[4][2], a0, a1, a2, a3, b0, b1, sum = 0;
    for( int i = 0; i < 4; i++, pix1 += i1, pix2 += i2 )
    {
        a0 = (sum2_t)(pix1[0] - pix2[0]);
        a1 = (sum2_t)(pix1[1] - pix2[1]);
        b0 = (a0 + a1) + ((a0 - a1) << BITS_PER_SUM);
        a2 = (sum2_t)(pix1[2] - pix2[2]);
        a3 = (sum2_t)(pix1[3] - pix2[3]);
        b1 = (a2 + a3) + ((a2 - a3) << BITS_PER_SUM);
        tmp[i][0] = b0 + b1;
        tmp[i][1] = b0 - b1;
    }
    for( int i = 0; i < 2; i++ )
    {
        HADAMARD4( a0, a1, a2, a3, tmp[0][i], tmp[1][i], tmp[2][i], tmp[3][i] );
        a0 = abs2( a0 ) + abs2( a1 ) + abs2( a2 ) + abs2( a3 );
        sum += ((sum_t)a0) + (a0 >> BITS_PER_SUM);
    }
    return sum >> 1;
}

/* satd 8x4, two 4x4 blocks packed in the two halves; reference pixel.c:290-309 */
static int satd_8x4( const pixel *pix1, intptr_t i1, const pixel *pix2, intptr_t i2 )
{
    sum2_t tmp[4][4], a0, a1, a2, a3, sum = 0;
    for( int i = 0; i < 4; i++, pix1 += i1, pix2 += i2 )
    {
        a0 = (sum2_t)(pix1[0] - pix2[0]) + ((sum2_t)(pix1[4] - pix2[4]) << BITS_PER_SUM);
        a1 = (sum2_t)(pix1[1] - pix2[1]) + ((sum2_t)(pix1[5] - pix2[5]) << BITS_PER_SUM);
        a2 = (sum2_t)(pix1[2] - pix2[2]) + ((sum2_t)(pix1[6] - pix2[6]) << BITS_PER_SUM);
        a3 = (sum2_t)(pix1[3] - pix2[3]) + ((sum2_t)(pix1[7] - pix2[7]) << BITS_PER_SUM);
        HADAMARD4( tmp[i][0], tmp[i][1], tmp[i][2], tmp[i][3], a0, a1, a2, a3 );
    }
    for( int i = 0; i < 4; i++ )
    {
        HADAMARD4( a0, a1, a2, a3, tmp[0][i], tmp[1][i], tmp[2][i], tmp[3][i] );
        sum += abs2( a0 ) + abs2( a1 ) + abs2( a2 ) + abs2( a3 );
    }
    return (((sum_t)sum) + (sum >> BITS_PER_SUM)) >> 1;
}

/* PIXEL_SATD_C tiling, reference common/pixel.c:311-332 (8-wide sizes use the
 * 8x4 kernel, 4-wide sizes the 4x4 kernel) */
int FN(satd)( int i_pixel, const pixel *pix1, intptr_t i1, const pixel *pix2, intptr_t i2 )
{
    int w = pixel_w[i_pixel], h = pixel_h[i_pixel];
    int sum = 0;
    if( w == 4 )
    {
        for( int y = 0; y < h; y += 4 )
            sum += satd_4x4( pix1 + y*i1, i1, pix2 + y*i2, i2 );
        return sum;
    }
    for( int x = 0; x < w; x += 8 )
        for( int y = 0; y < h; y += 4 )
            sum += satd_8x4( pix1 + y*i1 + x, i1, pix2 + y*i2 + x, i2 );
    return sum;
}

/* SAD_X / SATD_X, fenc stride implicitly FENC_STRIDE; reference pixel.c:441-496 */
void FN(sad_x3)( int i_pixel, const pixel *fenc, const pixel *p0, const pixel *p1, const pixel *p2,
                 intptr_t stride, int scores[3] )
{
    scores[0] = FN(sad)( i_pixel, fenc, FENC_STRIDE, p0, stride );
    scores[1] = FN(sad)( i_pixel, fenc, FENC_STRIDE, p1, stride );
    scores[2] = FN(sad)( i_pixel, fenc, FENC_STRIDE, p2, stride );
}

void FN(sad_x4)( int i_pixel, const pixel *fenc, const pixel *p0, const pixel *p1, const pixel *p2,
                 const pixel *p3, intptr_t stride, int scores[4] )
{
    FN(sad_x3)( i_pixel, fenc, p0, p1, p2, stride, scores );
    scores[3] = FN(sad)( i_pixel, fenc, FENC_STRIDE, p3, stride );
}

void FN(satd_x3)( int i_pixel, const pixel *fenc, const pixel *p0, const pixel *p1, const pixel *p2,
                  intptr_t stride, int scores[3] )
{
    scores[0] = FN(satd)( i_pixel, fenc, FENC_STRIDE, p0, stride );
    scores[1] = FN(satd)( i_pixel, fenc, FENC_STRIDE, p1, stride );
    scores[2] = FN(satd)( i_pixel, fenc, FENC_STRIDE, p2, stride );
}

void FN(satd_x4)( int i_pixel, const pixel *fenc, const pixel *p0, const pixel *p1, const pixel *p2,
                  const pixel *p3, intptr_t stride, int scores[4] )
{
    FN(satd_x3)( i_pixel, fenc, p0, p1, p2, stride, scores );
    scores[3] = FN(satd)( i_pixel, fenc, FENC_STRIDE, p3, stride );
}

/* generic list form used to check x264hip_*_pixel_cmp_batch */
void FN(cmp_list)( int op, int i_pixel, const pixel *fenc, intptr_t fs, const pixel *ref, intptr_t rs,
                   const int64_t *fenc_off, const int64_t *ref_off, int n, int32_t *scores )
{
    for( int i = 0; i < n; i++ )
    {
        const pixel *a = fenc + fenc_off[i], *b = ref + ref_off[i];
        scores[i] = op == 0 ? FN(sad)( i_pixel, a, fs, b, rs )
                  : op == 1 ? FN(ssd)( i_pixel, a, fs, b, rs )
                  :           FN(satd)( i_pixel, a, fs, b, rs );
    }
}

/*============================================================================
 * further pixel_function_t entries — reference common/pixel.c
 *==========================================================================*/

/* sa8d_8x8 (unnormalised), packed pairs; reference common/pixel.c:334-366 */
static int sa8d_8x8_raw( const pixel *pix1, intptr_t i1, const pixel *pix2, intptr_t i2 )
{
    sum2_t tmp[8][4], a0, a1, a2, a3, a4, a5, a6, a7, b0, b1, b2, b3, sum = 0;
    for( int i = 0; i < 8; i++, pix1 += i1, pix2 += i2 )
    {
        a0 = (sum2_t)(pix1[0] - pix2[0]); a1 = (sum2_t)(pix1[1] - pix2[1]);
        b0 = (a0 + a1) + ((a0 - a1) << BITS_PER_SUM);
        a2 = (sum2_t)(pix1[2] - pix2[2]); a3 = (sum2_t)(pix1[3] - pix2[3]);
        b1 = (a2 + a3) + ((a2 - a3) << BITS_PER_SUM);
        a4 = (sum2_t)(pix1[4] - pix2[4]); a5 = (sum2_t)(pix1[5] - pix2[5]);
        b2 = (a4 + a5) + ((a4 - a5) << BITS_PER_SUM);
        a6 = (sum2_t)(pix1[6] - pix2[6]); a7 = (sum2_t)(pix1[7] - pix2[7]);
        b3 = (a6 + a7) + ((a6 - a7) << BITS_PER_SUM);
        HADAMARD4( tmp[i][0], tmp[i][1], tmp[i][2], tmp[i][3], b0, b1, b2, b3 );
    }
    for( int i = 0; i < 4; i++ )
    {
        HADAMARD4( a0, a1, a2, a3, tmp[0][i], tmp[1][i], tmp[2][i], tmp[3][i] );
        HADAMARD4( a4, a5, a6, a7, tmp[4][i], tmp[5][i], tmp[6][i], tmp[7][i] );
        b0  = abs2( a0 + a4 ) + abs2( a0 - a4 );
        b0 += abs2( a1 + a5 ) + abs2( a1 - a5 );
        b0 += abs2( a2 + a6 ) + abs2( a2 - a6 );
        b0 += abs2( a3 + a7 ) + abs2( a3 - a7 );
        sum += (sum_t)b0 + (b0 >> BITS_PER_SUM);
    }
    return (int)sum;
}

/* sa8d[PIXEL_8x8] / sa8d[PIXEL_16x16], (sum+2)>>2; reference pixel.c:368-381 */
int FN(sa8d)( int i_pixel, const pixel *pix1, intptr_t i1, const pixel *pix2, intptr_t i2 )
{
    int sum = sa8d_8x8_raw( pix1, i1, pix2, i2 );
    if( i_pixel == 0 )
        sum += sa8d_8x8_raw( pix1 + 8, i1, pix2 + 8, i2 )
             + sa8d_8x8_raw( pix1 + 8*i1, i1, pix2 + 8*i2, i2 )
             + sa8d_8x8_raw( pix1 + 8 + 8*i1, i1, pix2 + 8 + 8*i2, i2 );
    return (sum + 2) >> 2;
}

/* sa8d_satd[PIXEL_16x16]: asm-only in the reference (pixel.c:922, x86/pixel-a.asm
 * SA8D_SATD); its contract is the checkasm test (tools/checkasm.c:424-460):
 * low 32 bits = sa8d_16x16, high 32 bits = satd_16x16. */
uint64_t FN(sa8d_satd)( const pixel *pix1, intptr_t i1, const pixel *pix2, intptr_t i2 )
{
    return (uint32_t)FN(sa8d)( 0, pix1, i1, pix2, i2 ) | ((uint64_t)(uint32_t)FN(satd)( 0, pix1, i1, pix2, i2 ) << 32);
}

/* pixel_hadamard_ac, reference common/pixel.c:383-418 */
static uint64_t hadamard_ac_raw( const pixel *pix, intptr_t stride )
{
    sum2_t tmp[32], a0, a1, a2, a3, dc, sum4 = 0, sum8 = 0;
    for( int i = 0; i < 8; i++, pix += stride )
    {
        sum2_t *t = tmp + (i & 3) + (i & 4) * 4;
        a0 = (pix[0] + pix[1]) + ((sum2_t)(pix[0] - pix[1]) << BITS_PER_SUM);
        a1 = (pix[2] + pix[3]) + ((sum2_t)(pix[2] - pix[3]) << BITS_PER_SUM);
        t[0] = a0 + a1;
        t[4] = a0 - a1;
        a2 = (pix[4] + pix[5]) + ((sum2_t)(pix[4] - pix[5]) << BITS_PER_SUM);
        a3 = (pix[6] + pix[7]) + ((sum2_t)(pix[6] - pix[7]) << BITS_PER_SUM);
        t[8] = a2 + a3;
        t[12] = a2 - a3;
    }
    for( int i = 0; i < 8; i++ )
    {
        HADAMARD4( a0, a1, a2, a3, tmp[i*4+0], tmp[i*4+1], tmp[i*4+2], tmp[i*4+3] );
        tmp[i*4+0] = a0; tmp[i*4+1] = a1; tmp[i*4+2] = a2; tmp[i*4+3] = a3;
        sum4 += abs2( a0 ) + abs2( a1 ) + abs2( a2 ) + abs2( a3 );
    }
    for( int i = 0; i < 8; i++ )
    {
        HADAMARD4( a0, a1, a2, a3, tmp[i], tmp[8+i], tmp[16+i], tmp[24+i] );
        sum8 += abs2( a0 ) + abs2( a1 ) + abs2( a2 ) + abs2( a3 );
    }
    dc = (sum_t)(tmp[0] + tmp[8] + tmp[16] + tmp[24]);
    sum4 = (sum_t)sum4 + (sum4 >> BITS_PER_SUM) - dc;
    sum8 = (sum_t)sum8 + (sum8 >> BITS_PER_SUM) - dc;
    return ((uint64_t)sum8 << 32) + sum4;
}

/* HADAMARD_AC(w,h), reference common/pixel.c:420-435; i_pixel 0..3 */
uint64_t FN(hadamard_ac)( int i_pixel, const pixel *pix, intptr_t stride )
{
    int w = pixel_w[i_pixel], h = pixel_h[i_pixel];
    uint64_t sum = hadamard_ac_raw( pix, stride );
    if( w == 16 )
        sum += hadamard_ac_raw( pix + 8, stride );
    if( h == 16 )
        sum += hadamard_ac_raw( pix + 8*stride, stride );
    if( w == 16 && h == 16 )
        sum += hadamard_ac_raw( pix + 8*stride + 8, stride );
    return ((sum >> 34) << 32) + ((uint32_t)sum >> 1);
}

/* PIXEL_VAR_C, reference common/pixel.c:181-198; i_pixel 0 (16x16), 2 (8x16), 3 (8x8) */
uint64_t FN(var)( int i_pixel, const pixel *pix, intptr_t stride )
{
    int w = pixel_w[i_pixel], h = pixel_h[i_pixel];
    uint32_t sum = 0, sqr = 0;
    for( int y = 0; y < h; y++, pix += stride )
        for( int x = 0; x < w; x++ )
        {
            sum += pix[x];
            sqr += pix[x] * pix[x];
        }
    return sum + ((uint64_t)sqr << 32);
}

/* PIXEL_VAR2_C with explicit strides and U->V offsets, reference
 * common/pixel.c:203-227 (the table form uses FENC_STRIDE / FDEC_STRIDE and
 * V at +FENC_STRIDE/2, +FDEC_STRIDE/2); h 16 (shift 7) or 8 (shift 6) */
int FN(var2_s)( int h, const pixel *fenc, intptr_t fs, intptr_t fvd, const pixel *fdec, intptr_t ds,
                intptr_t dvd, int ssd[2] )
{
    int shift = h == 16 ? 7 : 6;
    int sum_u = 0, sum_v = 0, sqr_u = 0, sqr_v = 0;
    for( int y = 0; y < h; y++, fenc += fs, fdec += ds )
        for( int x = 0; x < 8; x++ )
        {
            int du = fenc[x] - fdec[x];
            int dv = fenc[x + fvd] - fdec[x + dvd];
            sum_u += du; sum_v += dv;
            sqr_u += du * du; sqr_v += dv * dv;
        }
    ssd[0] = sqr_u;
    ssd[1] = sqr_v;
    return (int)(sqr_u - ((int64_t)sum_u * sum_u >> shift) + sqr_v - ((int64_t)sum_v * sum_v >> shift));
}

int FN(var2)( int i_pixel, const pixel *fenc, const pixel *fdec, int ssd[2] )
{
    return FN(var2_s)( pixel_h[i_pixel], fenc, FENC_STRIDE, FENC_STRIDE / 2, fdec, FDEC_STRIDE, FDEC_STRIDE / 2, ssd );
}

/* pixel_vsad, reference common/pixel.c:716-723 */
int FN(vsad)( const pixel *src, intptr_t stride, int height )
{
    int score = 0;
    for( int i = 1; i < height; i++, src += stride )
        for( int j = 0; j < 16; j++ )
            score += abs( src[j] - src[j + stride] );
    return score;
}

/* pixel_asd8, reference common/pixel.c:747-754 */
int FN(asd8)( const pixel *pix1, intptr_t s1, const pixel *pix2, intptr_t s2, int height )
{
    int sum = 0;
    for( int y = 0; y < height; y++, pix1 += s1, pix2 += s2 )
        for( int x = 0; x < 8; x++ )
            sum += pix1[x] - pix2[x];
    return abs( sum );
}

/* x264_pixel_ads4/2/1 (successive elimination), reference common/pixel.c:759-803;
 * nsums selects ads4 (4), ads2 (2) or ads1 (1) */
int FN(ads)( int nsums, const int enc_dc[4], const uint16_t *sums, int delta, const uint16_t *cost_mvx,
             int16_t *mvs, int width, int thresh )
{
    int nmv = 0;
    for( int i = 0; i < width; i++, sums++ )
    {
        int ads;
        if( nsums == 4 )
            ads = abs( enc_dc[0] - sums[0] ) + abs( enc_dc[1] - sums[8] )
                + abs( enc_dc[2] - sums[delta] ) + abs( enc_dc[3] - sums[delta + 8] );
        else if( nsums == 2 )
            ads = abs( enc_dc[0] - sums[0] ) + abs( enc_dc[1] - sums[delta] );
        else
            ads = abs( enc_dc[0] - sums[0] );
        ads += cost_mvx[i];
        if( ads < thresh )
            mvs[nmv++] = (int16_t)i;
    }
    return nmv;
}

/* integral_init4h/8h/4v/8v, reference common/mc.c:424-456 */
static void integral_init4h( uint16_t *sum, const pixel *pix, intptr_t stride )
{
    int v = pix[0] + pix[1] + pix[2] + pix[3];
    for( int x = 0; x < stride - 4; x++ )
    {
        sum[x] = (uint16_t)(v + sum[x - stride]);
        v += pix[x + 4] - pix[x];
    }
}

static void integral_init8h( uint16_t *sum, const pixel *pix, intptr_t stride )
{
    int v = pix[0] + pix[1] + pix[2] + pix[3] + pix[4] + pix[5] + pix[6] + pix[7];
    for( int x = 0; x < stride - 8; x++ )
    {
        sum[x] = (uint16_t)(v + sum[x - stride]);
        v += pix[x + 8] - pix[x];
    }
}

static void integral_init4v( uint16_t *sum8, uint16_t *sum4, intptr_t stride )
{
    for( int x = 0; x < stride - 8; x++ )
        sum4[x] = (uint16_t)(sum8[x + 4*stride] - sum8[x]);
    for( int x = 0; x < stride - 8; x++ )
        sum8[x] = (uint16_t)(sum8[x + 8*stride] + sum8[x + 8*stride + 4] - sum8[x] - sum8[x + 4]);
}

static void integral_init8v( uint16_t *sum8, intptr_t stride )
{
    for( int x = 0; x < stride - 8; x++ )
        sum8[x] = (uint16_t)(sum8[x + 8*stride] - sum8[x]);
}

/* the integral-image part of x264_frame_filter over a whole progressive frame
 * (mb_y = 0 .. b_end in one pass), reference common/mc.c:748-782.  plane and
 * integral point at (0,0); both have stride `stride`, rows [-PADV, lines+PADV)
 * (the 4x4 plane follows at +stride*(lines+2*PADV) when sub8x8), and the row
 * starts at x = -padh (PADH_ALIGN, frame.h:34; 32 for this repo's frames). */
void FN(frame_integral)( const pixel *plane, intptr_t stride, int lines, int padh, int sub8x8,
                         uint16_t *integral )
{
    const int padv = 32;
    int start = -8, height = lines + 8 + padv - 9;
    memset( integral - padv*stride - padh, 0, stride * sizeof(uint16_t) );
    start = -padv;
    for( int y = start; y < height; y++ )
    {
        const pixel *pix = plane + y*stride - padh;
        uint16_t *sum8 = integral + (y + 1)*stride - padh;
        if( sub8x8 )
        {
            integral_init4h( sum8, pix, stride );
            sum8 -= 8*stride;
            uint16_t *sum4 = sum8 + stride*(lines + padv*2);
            if( y >= 8 - padv )
                integral_init4v( sum8, sum4, stride );
        }
        else
        {
            integral_init8h( sum8, pix, stride );
            if( y >= 8 - padv )
                integral_init8v( sum8 - 8*stride, stride );
        }
    }
}

/*============================================================================
 * forward transforms — reference common/dct.c
 *==========================================================================*/

/* pixel_sub_wxh, reference common/dct.c:145-155 (result stored as dctcoef) */
static void pixel_sub_wxh( dctcoef *diff, int n, const pixel *p1, intptr_t s1, const pixel *p2, intptr_t s2 )
{
    for( int y = 0; y < n; y++, p1 += s1, p2 += s2 )
        for( int x = 0; x < n; x++ )
            diff[x + y*n] = p1[x] - p2[x];
}

/* sub4x4_dct, reference common/dct.c:157-189: rows then columns, int16 temps at
 * 8 bit, transposed output dct[x*4+y]... (row i of the second pass writes dct[i*4+k]) */
static void sub4x4_dct_s( dctcoef dct[16], const pixel *p1, intptr_t s1, const pixel *p2, intptr_t s2 )
{
    dctcoef d[16], tmp[16];
    pixel_sub_wxh( d, 4, p1, s1, p2, s2 );
    for( int i = 0; i < 4; i++ )
    {
        int s03 = d[i*4+0] + d[i*4+3], s12 = d[i*4+1] + d[i*4+2];
        int d03 = d[i*4+0] - d[i*4+3], d12 = d[i*4+1] - d[i*4+2];
        tmp[0*4+i] = s03 + s12;
        tmp[1*4+i] = 2*d03 + d12;
        tmp[2*4+i] = s03 - s12;
        tmp[3*4+i] = d03 - 2*d12;
    }
    for( int i = 0; i < 4; i++ )
    {
        int s03 = tmp[i*4+0] + tmp[i*4+3], s12 = tmp[i*4+1] + tmp[i*4+2];
        int d03 = tmp[i*4+0] - tmp[i*4+3], d12 = tmp[i*4+1] - tmp[i*4+2];
        dct[i*4+0] = s03 + s12;
        dct[i*4+1] = 2*d03 + d12;
        dct[i*4+2] = s03 - s12;
        dct[i*4+3] = d03 - 2*d12;
    }
}

/* sub8x8_dct / sub16x16_dct block order, reference common/dct.c:191-205 */
static void sub8x8_dct_s( dctcoef dct[4][16], const pixel *p1, intptr_t s1, const pixel *p2, intptr_t s2 )
{
    sub4x4_dct_s( dct[0], p1,          s1, p2,          s2 );
    sub4x4_dct_s( dct[1], p1+4,        s1, p2+4,        s2 );
    sub4x4_dct_s( dct[2], p1+4*s1,     s1, p2+4*s2,     s2 );
    sub4x4_dct_s( dct[3], p1+4*s1+4,   s1, p2+4*s2+4,   s2 );
}

static void sub16x16_dct_s( dctcoef dct[16][16], const pixel *p1, intptr_t s1, const pixel *p2, intptr_t s2 )
{
    sub8x8_dct_s( &dct[ 0], p1,          s1, p2,          s2 );
    sub8x8_dct_s( &dct[ 4], p1+8,        s1, p2+8,        s2 );
    sub8x8_dct_s( &dct[ 8], p1+8*s1,     s1, p2+8*s2,     s2 );
    sub8x8_dct_s( &dct[12], p1+8*s1+8,   s1, p2+8*s2+8,   s2 );
}

/* sub4x4_dct_dc, reference common/dct.c:207-214 */
static int sub4x4_dct_dc_s( const pixel *p1, intptr_t s1, const pixel *p2, intptr_t s2 )
{
    int sum = 0;
    for( int i = 0; i < 4; i++, p1 += s1, p2 += s2 )
        sum += p1[0] + p1[1] + p1[2] + p1[3] - p2[0] - p2[1] - p2[2] - p2[3];
    return sum;
}

/* sub8x8_dct_dc with its 2x2 DC transform, reference common/dct.c:216-232.
 * The four sums are stored to dctcoef before the butterfly reads them back. */
static void sub8x8_dct_dc_s( dctcoef dct[4], const pixel *p1, intptr_t s1, const pixel *p2, intptr_t s2 )
{
    dct[0] = sub4x4_dct_dc_s( p1,        s1, p2,        s2 );
    dct[1] = sub4x4_dct_dc_s( p1+4,      s1, p2+4,      s2 );
    dct[2] = sub4x4_dct_dc_s( p1+4*s1,   s1, p2+4*s2,   s2 );
    dct[3] = sub4x4_dct_dc_s( p1+4*s1+4, s1, p2+4*s2+4, s2 );
    int d0 = dct[0] + dct[1], d1 = dct[2] + dct[3];
    int d2 = dct[0] - dct[1], d3 = dct[2] - dct[3];
    dct[0] = d0 + d1;
    dct[1] = d0 - d1;
    dct[2] = d2 + d3;
    dct[3] = d2 - d3;
}

/* sub8x16_dct_dc with its 2x4 DC transform, reference common/dct.c:234-270 */
static void sub8x16_dct_dc_s( dctcoef dct[8], const pixel *p1, intptr_t s1, const pixel *p2, intptr_t s2 )
{
    int a[8];
    for( int k = 0; k < 8; k++ )
        a[k] = sub4x4_dct_dc_s( p1 + (k>>1)*4*s1 + (k&1)*4, s1, p2 + (k>>1)*4*s2 + (k&1)*4, s2 );
    int b0 = a[0] + a[1], b1 = a[2] + a[3], b2 = a[4] + a[5], b3 = a[6] + a[7];
    int b4 = a[0] - a[1], b5 = a[2] - a[3], b6 = a[4] - a[5], b7 = a[6] - a[7];
    int c0 = b0 + b1, c1 = b2 + b3, c2 = b4 + b5, c3 = b6 + b7;
    int c4 = b0 - b1, c5 = b2 - b3, c6 = b4 - b5, c7 = b6 - b7;
    dct[0] = c0 + c1;
    dct[1] = c2 + c3;
    dct[2] = c0 - c1;
    dct[3] = c2 - c3;
    dct[4] = c4 - c5;
    dct[5] = c6 - c7;
    dct[6] = c4 + c5;
    dct[7] = c6 + c7;
}

/* DCT8_1D, reference common/dct.c:332-356 */
#define DCT8_1D {\
    int s07 = SRC(0) + SRC(7), s16 = SRC(1) + SRC(6), s25 = SRC(2) + SRC(5), s34 = SRC(3) + SRC(4);\
    int a0 = s07 + s34, a1 = s16 + s25, a2 = s07 - s34, a3 = s16 - s25;\
    int d07 = SRC(0) - SRC(7), d16 = SRC(1) - SRC(6), d25 = SRC(2) - SRC(5), d34 = SRC(3) - SRC(4);\
    int a4 = d16 + d25 + (d07 + (d07>>1));\
    int a5 = d07 - d34 - (d25 + (d25>>1));\
    int a6 = d07 + d34 - (d16 + (d16>>1));\
    int a7 = d16 - d25 + (d34 + (d34>>1));\
    DST(0) =  a0 + a1;\
    DST(1) =  a4 + (a7>>2);\
    DST(2) =  a2 + (a3>>1);\
    DST(3) =  a5 + (a6>>2);\
    DST(4) =  a0 - a1;\
    DST(5) =  a6 - (a5>>2);\
    DST(6) = (a2>>1) - a3;\
    DST(7) = (a4>>2) - a7;\
}

/* sub8x8_dct8: column pass in place (dctcoef temps), then row pass writing the
 * transposed output; reference common/dct.c:358-377 */
static void sub8x8_dct8_s( dctcoef dct[64], const pixel *p1, intptr_t s1, const pixel *p2, intptr_t s2 )
{
    dctcoef tmp[64];
    pixel_sub_wxh( tmp, 8, p1, s1, p2, s2 );
#define SRC(x) tmp[(x)*8+i]
#define DST(x) tmp[(x)*8+i]
    for( int i = 0; i < 8; i++ )
        DCT8_1D
#undef SRC
#undef DST
#define SRC(x) tmp[i*8+(x)]
#define DST(x) dct[(x)*8+i]
    for( int i = 0; i < 8; i++ )
        DCT8_1D
#undef SRC
#undef DST
}

static void sub16x16_dct8_s( dctcoef dct[4][64], const pixel *p1, intptr_t s1, const pixel *p2, intptr_t s2 )
{
    sub8x8_dct8_s( dct[0], p1,          s1, p2,          s2 );
    sub8x8_dct8_s( dct[1], p1+8,        s1, p2+8,        s2 );
    sub8x8_dct8_s( dct[2], p1+8*s1,     s1, p2+8*s2,     s2 );
    sub8x8_dct8_s( dct[3], p1+8*s1+8,   s1, p2+8*s2+8,   s2 );
}

/* entry points with the reference's implicit strides (dct.h:31-33) */
void FN(sub4x4_dct)( dctcoef dct[16], const pixel *p1, const pixel *p2 ) { sub4x4_dct_s( dct, p1, FENC_STRIDE, p2, FDEC_STRIDE ); }
void FN(sub8x8_dct)( dctcoef dct[4][16], const pixel *p1, const pixel *p2 ) { sub8x8_dct_s( dct, p1, FENC_STRIDE, p2, FDEC_STRIDE ); }
void FN(sub16x16_dct)( dctcoef dct[16][16], const pixel *p1, const pixel *p2 ) { sub16x16_dct_s( dct, p1, FENC_STRIDE, p2, FDEC_STRIDE ); }
void FN(sub8x8_dct_dc)( dctcoef dct[4], const pixel *p1, const pixel *p2 ) { sub8x8_dct_dc_s( dct, p1, FENC_STRIDE, p2, FDEC_STRIDE ); }
void FN(sub8x16_dct_dc)( dctcoef dct[8], const pixel *p1, const pixel *p2 ) { sub8x16_dct_dc_s( dct, p1, FENC_STRIDE, p2, FDEC_STRIDE ); }
void FN(sub8x8_dct8)( dctcoef dct[64], const pixel *p1, const pixel *p2 ) { sub8x8_dct8_s( dct, p1, FENC_STRIDE, p2, FDEC_STRIDE ); }
void FN(sub16x16_dct8)( dctcoef dct[4][64], const pixel *p1, const pixel *p2 ) { sub16x16_dct8_s( dct, p1, FENC_STRIDE, p2, FDEC_STRIDE ); }

/* list form for x264hip_*_sub_dct_batch; kinds as X264HIP_DCT_* */
static const int dct_kind_size[7] = { 16, 64, 256, 4, 8, 64, 256 };
void FN(sub_dct_list)( int kind, const pixel *fenc, intptr_t fs, const pixel *fdec, intptr_t ds,
                       const int64_t *fenc_off, const int64_t *fdec_off, int n, dctcoef *out )
{
    for( int i = 0; i < n; i++ )
    {
        const pixel *a = fenc + fenc_off[i], *b = fdec + fdec_off[i];
        dctcoef *o = out + (size_t)i * dct_kind_size[kind];
        switch( kind )
        {
            case 0: sub4x4_dct_s( o, a, fs, b, ds ); break;
            case 1: sub8x8_dct_s( (dctcoef(*)[16])o, a, fs, b, ds ); break;
            case 2: sub16x16_dct_s( (dctcoef(*)[16])o, a, fs, b, ds ); break;
            case 3: sub8x8_dct_dc_s( o, a, fs, b, ds ); break;
            case 4: sub8x16_dct_dc_s( o, a, fs, b, ds ); break;
            case 5: sub8x8_dct8_s( o, a, fs, b, ds ); break;
            case 6: sub16x16_dct8_s( (dctcoef(*)[64])o, a, fs, b, ds ); break;
        }
    }
}

/* dct4x4dc, reference common/dct.c:47-76 */
void FN(dct4x4dc)( dctcoef d[16] )
{
    dctcoef tmp[16];
    for( int i = 0; i < 4; i++ )
    {
        int s01 = d[i*4+0] + d[i*4+1], d01 = d[i*4+0] - d[i*4+1];
        int s23 = d[i*4+2] + d[i*4+3], d23 = d[i*4+2] - d[i*4+3];
        tmp[0*4+i] = s01 + s23;
        tmp[1*4+i] = s01 - s23;
        tmp[2*4+i] = d01 - d23;
        tmp[3*4+i] = d01 + d23;
    }
    for( int i = 0; i < 4; i++ )
    {
        int s01 = tmp[i*4+0] + tmp[i*4+1], d01 = tmp[i*4+0] - tmp[i*4+1];
        int s23 = tmp[i*4+2] + tmp[i*4+3], d23 = tmp[i*4+2] - tmp[i*4+3];
        d[i*4+0] = ( s01 + s23 + 1 ) >> 1;
        d[i*4+1] = ( s01 - s23 + 1 ) >> 1;
        d[i*4+2] = ( d01 - d23 + 1 ) >> 1;
        d[i*4+3] = ( d01 + d23 + 1 ) >> 1;
    }
}

/* dct2x4dc, reference common/dct.c:109-143 (zeroes the gathered DCs) */
void FN(dct2x4dc)( dctcoef dct[8], dctcoef dct4x4[8][16] )
{
    int a0 = dct4x4[0][0] + dct4x4[1][0], a1 = dct4x4[2][0] + dct4x4[3][0];
    int a2 = dct4x4[4][0] + dct4x4[5][0], a3 = dct4x4[6][0] + dct4x4[7][0];
    int a4 = dct4x4[0][0] - dct4x4[1][0], a5 = dct4x4[2][0] - dct4x4[3][0];
    int a6 = dct4x4[4][0] - dct4x4[5][0], a7 = dct4x4[6][0] - dct4x4[7][0];
    int b0 = a0 + a1, b1 = a2 + a3, b2 = a4 + a5, b3 = a6 + a7;
    int b4 = a0 - a1, b5 = a2 - a3, b6 = a4 - a5, b7 = a6 - a7;
    dct[0] = b0 + b1;
    dct[1] = b2 + b3;
    dct[2] = b0 - b1;
    dct[3] = b2 - b3;
    dct[4] = b4 - b5;
    dct[5] = b6 - b7;
    dct[6] = b4 + b5;
    dct[7] = b6 + b7;
    for( int k = 0; k < 8; k++ )
        dct4x4[k][0] = 0;
}

/*============================================================================
 * quantisation — reference common/quant.c:50-104
 *==========================================================================*/
#define QUANT_ONE( coef, mf, f ) \
{ \
    if( (coef) > 0 ) \
        (coef) = ((f) + (uint32_t)(coef)) * (mf) >> 16; \
    else \
        (coef) = -(int32_t)(((f) + (uint32_t)(-(coef))) * (mf) >> 16); \
    nz |= (coef); \
}

int FN(quant_8x8)( dctcoef dct[64], const udctcoef mf[64], const udctcoef bias[64] )
{
    int nz = 0;
    for( int i = 0; i < 64; i++ )
        QUANT_ONE( dct[i], mf[i], bias[i] );
    return !!nz;
}

int FN(quant_4x4)( dctcoef dct[16], const udctcoef mf[16], const udctcoef bias[16] )
{
    int nz = 0;
    for( int i = 0; i < 16; i++ )
        QUANT_ONE( dct[i], mf[i], bias[i] );
    return !!nz;
}

int FN(quant_4x4x4)( dctcoef dct[4][16], const udctcoef mf[16], const udctcoef bias[16] )
{
    int nza = 0;
    for( int j = 0; j < 4; j++ )
    {
        int nz = 0;
        for( int i = 0; i < 16; i++ )
            QUANT_ONE( dct[j][i], mf[i], bias[i] );
        nza |= (!!nz) << j;
    }
    return nza;
}

int FN(quant_4x4_dc)( dctcoef dct[16], int mf, int bias )
{
    int nz = 0;
    for( int i = 0; i < 16; i++ )
        QUANT_ONE( dct[i], mf, bias );
    return !!nz;
}

int FN(quant_2x2_dc)( dctcoef dct[4], int mf, int bias )
{
    int nz = 0;
    for( int i = 0; i < 4; i++ )
        QUANT_ONE( dct[i], mf, bias );
    return !!nz;
}

/*============================================================================
 * CQM — reference common/set.c:28-206 (quant side only)
 *==========================================================================*/
#define SHIFT(x,s) ((s)<=0 ? (x)<<-(s) : ((x)+(1<<((s)-1)))>>(s))
#define DIV(n,d) (((n) + ((d)>>1)) / (d))

/* H.264 scaling constants, reference common/set.c:31-71 */
static const uint16_t quant4_scale[6][3] =
{
    { 13107, 8066, 5243 }, { 11916, 7490, 4660 }, { 10082, 6554, 4194 },
    {  9362, 5825, 3647 }, {  8192, 5243, 3355 }, {  7282, 4559, 2893 },
};
static const uint8_t quant8_scan[16] = { 0,3,4,3, 3,1,5,1, 4,5,2,5, 3,1,5,1 };
static const uint16_t quant8_scale[6][6] =
{
    { 13107, 11428, 20972, 12222, 16777, 15481 },
    { 11916, 10826, 19174, 11058, 14980, 14290 },
    { 10082,  8943, 15978,  9675, 12710, 11985 },
    {  9362,  8228, 14913,  8931, 11984, 11259 },
    {  8192,  7346, 13159,  7740, 10486,  9777 },
    {  7282,  6428, 11570,  6830,  9118,  8640 },
};

int FN(cqm_init)( const uint8_t *const scaling_list[8], int deadzone_inter, int deadzone_intra,
                  int b_transform_8x8, udctcoef *q4_mf, udctcoef *q4_bias, udctcoef *q8_mf, udctcoef *q8_bias )
{
    /* deadzone per list: {32-dz[1], 32-dz[0], 32-11, 32-21}, reference set.c:81-83 */
    int deadzone[4] = { 32 - deadzone_intra, 32 - deadzone_inter, 32 - 11, 32 - 21 };
    int def_quant4[6][16], def_quant8[6][64];
    int quant4_mf[4][6][16], quant8_mf[4][6][64];

    for( int q = 0; q < 6; q++ )
    {
        for( int i = 0; i < 16; i++ )
            def_quant4[q][i] = quant4_scale[q][(i&1) + ((i>>2)&1)];
        for( int i = 0; i < 64; i++ )
            def_quant8[q][i] = quant8_scale[q][quant8_scan[((i>>1)&12) | (i&3)]];
    }
    for( int q = 0; q < 6; q++ )
    {
        for( int l = 0; l < 4; l++ )
            for( int i = 0; i < 16; i++ )
                quant4_mf[l][q][i] = DIV( def_quant4[q][i] * 16, scaling_list[l][i] );
        if( b_transform_8x8 )
            for( int l = 0; l < 2; l++ )   /* num_8x8_lists for 4:2:0 with 8x8dct, set.c:87-88 */
                for( int i = 0; i < 64; i++ )
                    quant8_mf[l][q][i] = DIV( def_quant8[q][i] * 16, scaling_list[4+l][i] );
    }
    for( int q = 0; q <= QP_MAX_SPEC; q++ )
    {
        for( int l = 0; l < 4; l++ )
            for( int i = 0; i < 16; i++ )
            {
                int j = SHIFT( quant4_mf[l][q%6][i], q/6 - 1 );
                size_t o = ((size_t)l*(QP_MAX_SPEC+1) + q)*16 + i;
                q4_mf[o] = (uint16_t)j;
                if( !j )
                    continue;   /* bias left untouched, as the reference does (set.c:171-175) */
                int a = DIV( deadzone[l] << 10, j ), b = (1<<15) / j;
                q4_bias[o] = a < b ? a : b;
            }
        if( b_transform_8x8 )
            for( int l = 0; l < 2; l++ )
                for( int i = 0; i < 64; i++ )
                {
                    int j = SHIFT( quant8_mf[l][q%6][i], q/6 );
                    size_t o = ((size_t)l*(QP_MAX_SPEC+1) + q)*64 + i;
                    q8_mf[o] = (uint16_t)j;
                    if( !j )
                        continue;
                    int a = DIV( deadzone[l] << 10, j ), b = (1<<15) / j;
                    q8_bias[o] = a < b ? a : b;
                }
    }
    return QP_MAX_SPEC;
}

/*============================================================================
 * inverse path — reference common/dct.c, common/quant.c
 *==========================================================================*/

/* idct4x4dc, reference common/dct.c:78-107 (tmp as dctcoef) */
void FN(idct4x4dc)( dctcoef d[16] )
{
    dctcoef tmp[16];
    for( int i = 0; i < 4; i++ )
    {
        int s01 = d[i*4+0] + d[i*4+1], d01 = d[i*4+0] - d[i*4+1];
        int s23 = d[i*4+2] + d[i*4+3], d23 = d[i*4+2] - d[i*4+3];
        tmp[0*4+i] = s01 + s23; tmp[1*4+i] = s01 - s23;
        tmp[2*4+i] = d01 - d23; tmp[3*4+i] = d01 + d23;
    }
    for( int i = 0; i < 4; i++ )
    {
        int s01 = tmp[i*4+0] + tmp[i*4+1], d01 = tmp[i*4+0] - tmp[i*4+1];
        int s23 = tmp[i*4+2] + tmp[i*4+3], d23 = tmp[i*4+2] - tmp[i*4+3];
        d[i*4+0] = s01 + s23; d[i*4+1] = s01 - s23;
        d[i*4+2] = d01 - d23; d[i*4+3] = d01 + d23;
    }
}

/* add4x4_idct with explicit dst stride, reference common/dct.c:272-309 */
static void add4x4_idct_s( pixel *p_dst, intptr_t ds, const dctcoef dct[16] )
{
    dctcoef d[16], tmp[16];
    for( int i = 0; i < 4; i++ )
    {
        int s02 = dct[0*4+i] + dct[2*4+i], d02 = dct[0*4+i] - dct[2*4+i];
        int s13 = dct[1*4+i] + (dct[3*4+i] >> 1), d13 = (dct[1*4+i] >> 1) - dct[3*4+i];
        tmp[i*4+0] = s02 + s13; tmp[i*4+1] = d02 + d13;
        tmp[i*4+2] = d02 - d13; tmp[i*4+3] = s02 - s13;
    }
    for( int i = 0; i < 4; i++ )
    {
        int s02 = tmp[0*4+i] + tmp[2*4+i], d02 = tmp[0*4+i] - tmp[2*4+i];
        int s13 = tmp[1*4+i] + (tmp[3*4+i] >> 1), d13 = (tmp[1*4+i] >> 1) - tmp[3*4+i];
        d[0*4+i] = (s02 + s13 + 32) >> 6; d[1*4+i] = (d02 + d13 + 32) >> 6;
        d[2*4+i] = (d02 - d13 + 32) >> 6; d[3*4+i] = (s02 - s13 + 32) >> 6;
    }
    for( int y = 0; y < 4; y++, p_dst += ds )
        for( int x = 0; x < 4; x++ )
            p_dst[x] = clip_pixel( p_dst[x] + d[y*4+x] );
}

static void add8x8_idct_s( pixel *p, intptr_t ds, const dctcoef dct[4][16] )
{
    add4x4_idct_s( p, ds, dct[0] );
    add4x4_idct_s( p + 4, ds, dct[1] );
    add4x4_idct_s( p + 4*ds, ds, dct[2] );
    add4x4_idct_s( p + 4*ds + 4, ds, dct[3] );
}

static void add16x16_idct_s( pixel *p, intptr_t ds, const dctcoef dct[16][16] )
{
    add8x8_idct_s( p, ds, &dct[0] );
    add8x8_idct_s( p + 8, ds, &dct[4] );
    add8x8_idct_s( p + 8*ds, ds, &dct[8] );
    add8x8_idct_s( p + 8*ds + 8, ds, &dct[12] );
}

/* IDCT8_1D and add8x8_idct8, reference common/dct.c:388-446; the reference
 * works in place on dct (dctcoef stores), so this copy does too */
#define IDCT8_1D {\
    int a0 = SRC(0) + SRC(4), a2 = SRC(0) - SRC(4);\
    int a4 = (SRC(2) >> 1) - SRC(6), a6 = (SRC(6) >> 1) + SRC(2);\
    int b0 = a0 + a6, b2 = a2 + a4, b4 = a2 - a4, b6 = a0 - a6;\
    int a1 = -SRC(3) + SRC(5) - SRC(7) - (SRC(7) >> 1);\
    int a3 =  SRC(1) + SRC(7) - SRC(3) - (SRC(3) >> 1);\
    int a5 = -SRC(1) + SRC(7) + SRC(5) + (SRC(5) >> 1);\
    int a7 =  SRC(3) + SRC(5) + SRC(1) + (SRC(1) >> 1);\
    int b1 = (a7 >> 2) + a1, b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5, b7 = a7 - (a1 >> 2);\
    DST(0, b0 + b7); DST(1, b2 + b5); DST(2, b4 + b3); DST(3, b6 + b1);\
    DST(4, b6 - b1); DST(5, b4 - b3); DST(6, b2 - b5); DST(7, b0 - b7);\
}

static void add8x8_idct8_s( pixel *dst, intptr_t ds, dctcoef dct[64] )
{
    dct[0] += 32;
#define SRC(x) dct[(x)*8+i]
#define DST(x, rhs) dct[(x)*8+i] = (rhs)
    for( int i = 0; i < 8; i++ )
        IDCT8_1D
#undef SRC
#undef DST
#define SRC(x) dct[i*8+(x)]
#define DST(x, rhs) dst[i + (x)*ds] = clip_pixel( dst[i + (x)*ds] + ((rhs) >> 6) )
    for( int i = 0; i < 8; i++ )
        IDCT8_1D
#undef SRC
#undef DST
}

static void add16x16_idct8_s( pixel *p, intptr_t ds, dctcoef dct[4][64] )
{
    add8x8_idct8_s( p, ds, dct[0] );
    add8x8_idct8_s( p + 8, ds, dct[1] );
    add8x8_idct8_s( p + 8*ds, ds, dct[2] );
    add8x8_idct8_s( p + 8*ds + 8, ds, dct[3] );
}

/* add4x4_idct_dc / add8x8_idct_dc / add16x16_idct_dc, reference dct.c:448-476 */
static void add4x4_idct_dc_s( pixel *p, intptr_t ds, dctcoef dc )
{
    dc = (dc + 32) >> 6;
    for( int i = 0; i < 4; i++, p += ds )
        for( int x = 0; x < 4; x++ )
            p[x] = clip_pixel( p[x] + dc );
}

static void add8x8_idct_dc_s( pixel *p, intptr_t ds, const dctcoef dct[4] )
{
    add4x4_idct_dc_s( p, ds, dct[0] );
    add4x4_idct_dc_s( p + 4, ds, dct[1] );
    add4x4_idct_dc_s( p + 4*ds, ds, dct[2] );
    add4x4_idct_dc_s( p + 4*ds + 4, ds, dct[3] );
}

static void add16x16_idct_dc_s( pixel *p, intptr_t ds, const dctcoef dct[16] )
{
    for( int i = 0; i < 4; i++, dct += 4, p += 4*ds )
        for( int k = 0; k < 4; k++ )
            add4x4_idct_dc_s( p + 4*k, ds, dct[k] );
}

/* table forms (p_dst stride FDEC_STRIDE) */
void FN(add4x4_idct)( pixel *p, dctcoef dct[16] ) { add4x4_idct_s( p, FDEC_STRIDE, dct ); }
void FN(add8x8_idct)( pixel *p, dctcoef dct[4][16] ) { add8x8_idct_s( p, FDEC_STRIDE, dct ); }
void FN(add16x16_idct)( pixel *p, dctcoef dct[16][16] ) { add16x16_idct_s( p, FDEC_STRIDE, dct ); }
void FN(add8x8_idct_dc)( pixel *p, dctcoef dct[4] ) { add8x8_idct_dc_s( p, FDEC_STRIDE, dct ); }
void FN(add16x16_idct_dc)( pixel *p, dctcoef dct[16] ) { add16x16_idct_dc_s( p, FDEC_STRIDE, dct ); }
void FN(add8x8_idct8)( pixel *p, dctcoef dct[64] ) { add8x8_idct8_s( p, FDEC_STRIDE, dct ); }
void FN(add16x16_idct8)( pixel *p, dctcoef dct[4][64] ) { add16x16_idct8_s( p, FDEC_STRIDE, dct ); }

/* list form of the batched add_idct entry: kind as X264HIP_IDCT_* (0 add4x4,
 * 1 add8x8, 2 add16x16, 3 add8x8_dc, 4 add16x16_dc, 5 add8x8_8, 6 add16x16_8);
 * block i reads dct + i*size (a private copy: the input is not modified) */
static const int idct_kind_size[7] = { 16, 64, 256, 4, 16, 64, 256 };
void FN(add_idct_list)( int kind, pixel *dst, intptr_t ds, const int64_t *dst_off, const dctcoef *dct, int n )
{
    dctcoef tmp[256];
    for( int i = 0; i < n; i++ )
    {
        int sz = idct_kind_size[kind];
        memcpy( tmp, dct + (size_t)i*sz, sz * sizeof(dctcoef) );
        pixel *p = dst + dst_off[i];
        switch( kind )
        {
            case 0: add4x4_idct_s( p, ds, tmp ); break;
            case 1: add8x8_idct_s( p, ds, (dctcoef(*)[16])tmp ); break;
            case 2: add16x16_idct_s( p, ds, (dctcoef(*)[16])tmp ); break;
            case 3: add8x8_idct_dc_s( p, ds, tmp ); break;
            case 4: add16x16_idct_dc_s( p, ds, tmp ); break;
            case 5: add8x8_idct8_s( p, ds, tmp ); break;
            default: add16x16_idct8_s( p, ds, (dctcoef(*)[64])tmp ); break;
        }
    }
}

/* dequant_4x4 / dequant_8x8 / dequant_4x4_dc, reference common/quant.c:106-162 */
void FN(dequant_4x4)( dctcoef dct[16], int dequant_mf[6][16], int i_qp )
{
    const int i_mf = i_qp % 6, i_qbits = i_qp / 6 - 4;
    if( i_qbits >= 0 )
        for( int i = 0; i < 16; i++ )
            dct[i] = (dct[i] * dequant_mf[i_mf][i]) * (1 << i_qbits);
    else
    {
        const int f = 1 << (-i_qbits - 1);
        for( int i = 0; i < 16; i++ )
            dct[i] = (dct[i] * dequant_mf[i_mf][i] + f) >> (-i_qbits);
    }
}

void FN(dequant_8x8)( dctcoef dct[64], int dequant_mf[6][64], int i_qp )
{
    const int i_mf = i_qp % 6, i_qbits = i_qp / 6 - 6;
    if( i_qbits >= 0 )
        for( int i = 0; i < 64; i++ )
            dct[i] = (dct[i] * dequant_mf[i_mf][i]) * (1 << i_qbits);
    else
    {
        const int f = 1 << (-i_qbits - 1);
        for( int i = 0; i < 64; i++ )
            dct[i] = (dct[i] * dequant_mf[i_mf][i] + f) >> (-i_qbits);
    }
}

void FN(dequant_4x4_dc)( dctcoef dct[16], int dequant_mf[6][16], int i_qp )
{
    const int i_qbits = i_qp / 6 - 6;
    if( i_qbits >= 0 )
    {
        const int i_dmf = dequant_mf[i_qp % 6][0] << i_qbits;
        for( int i = 0; i < 16; i++ )
            dct[i] *= i_dmf;
    }
    else
    {
        const int i_dmf = dequant_mf[i_qp % 6][0], f = 1 << (-i_qbits - 1);
        for( int i = 0; i < 16; i++ )
            dct[i] = (dct[i] * i_dmf + f) >> (-i_qbits);
    }
}

/* idct_dequant_2x4_dc / _dconly, reference common/quant.c:164-208 */
#define IDQ_2X4_START \
    int a0 = dct[0] + dct[1], a1 = dct[2] + dct[3], a2 = dct[4] + dct[5], a3 = dct[6] + dct[7]; \
    int a4 = dct[0] - dct[1], a5 = dct[2] - dct[3], a6 = dct[4] - dct[5], a7 = dct[6] - dct[7]; \
    int b0 = a0 + a1, b1 = a2 + a3, b2 = a4 + a5, b3 = a6 + a7; \
    int b4 = a0 - a1, b5 = a2 - a3, b6 = a4 - a5, b7 = a6 - a7;

void FN(idct_dequant_2x4_dc)( dctcoef dct[8], dctcoef dct4x4[8][16], int dequant_mf[6][16], int i_qp )
{
    IDQ_2X4_START
    int dmf = dequant_mf[i_qp % 6][0] << i_qp / 6;
    dct4x4[0][0] = ((b0 + b1) * dmf + 32) >> 6;
    dct4x4[1][0] = ((b2 + b3) * dmf + 32) >> 6;
    dct4x4[2][0] = ((b0 - b1) * dmf + 32) >> 6;
    dct4x4[3][0] = ((b2 - b3) * dmf + 32) >> 6;
    dct4x4[4][0] = ((b4 - b5) * dmf + 32) >> 6;
    dct4x4[5][0] = ((b6 - b7) * dmf + 32) >> 6;
    dct4x4[6][0] = ((b4 + b5) * dmf + 32) >> 6;
    dct4x4[7][0] = ((b6 + b7) * dmf + 32) >> 6;
}

void FN(idct_dequant_2x4_dconly)( dctcoef dct[8], int dequant_mf[6][16], int i_qp )
{
    IDQ_2X4_START
    int dmf = dequant_mf[i_qp % 6][0] << i_qp / 6;
    dct[0] = ((b0 + b1) * dmf + 32) >> 6;
    dct[1] = ((b2 + b3) * dmf + 32) >> 6;
    dct[2] = ((b0 - b1) * dmf + 32) >> 6;
    dct[3] = ((b2 - b3) * dmf + 32) >> 6;
    dct[4] = ((b4 - b5) * dmf + 32) >> 6;
    dct[5] = ((b6 - b7) * dmf + 32) >> 6;
    dct[6] = ((b4 + b5) * dmf + 32) >> 6;
    dct[7] = ((b6 + b7) * dmf + 32) >> 6;
}

/* optimize_chroma_2x2_dc / 2x4_dc, reference common/quant.c:210-293 */
static void oc_idq_2x4( dctcoef out[8], const dctcoef dct[8], int dmf )
{
    IDQ_2X4_START
    out[0] = ((b0 + b1) * dmf + 2080) >> 6;
    out[1] = ((b2 + b3) * dmf + 2080) >> 6;
    out[2] = ((b0 - b1) * dmf + 2080) >> 6;
    out[3] = ((b2 - b3) * dmf + 2080) >> 6;
    out[4] = ((b4 - b5) * dmf + 2080) >> 6;
    out[5] = ((b6 - b7) * dmf + 2080) >> 6;
    out[6] = ((b4 + b5) * dmf + 2080) >> 6;
    out[7] = ((b6 + b7) * dmf + 2080) >> 6;
}
#undef IDQ_2X4_START

static void oc_idq_2x2( dctcoef out[4], const dctcoef dct[4], int dmf )
{
    int d0 = dct[0] + dct[1], d1 = dct[2] + dct[3], d2 = dct[0] - dct[1], d3 = dct[2] - dct[3];
    out[0] = ((d0 + d1) * dmf >> 5) + 32;
    out[1] = ((d0 - d1) * dmf >> 5) + 32;
    out[2] = ((d2 + d3) * dmf >> 5) + 32;
    out[3] = ((d2 - d3) * dmf >> 5) + 32;
}

static int optimize_chroma_dc( dctcoef *dct, int dmf, int c422 )
{
    dctcoef orig[8], out[8];
    int n = c422 ? 8 : 4, nz = 0, sum = 0;
    if( c422 ) oc_idq_2x4( orig, dct, dmf ); else oc_idq_2x2( orig, dct, dmf );
    for( int i = 0; i < n; i++ )
        sum |= orig[i];
    if( !(sum >> 6) )
        return 0;
    for( int coeff = n - 1; coeff >= 0; coeff-- )
    {
        int level = dct[coeff];
        int sign = level >> 31 | 1;
        while( level )
        {
            dct[coeff] = level - sign;
            if( c422 ) oc_idq_2x4( out, dct, dmf ); else oc_idq_2x2( out, dct, dmf );
            int diff = 0;
            for( int i = 0; i < n; i++ )
                diff |= orig[i] ^ out[i];
            if( diff >> 6 )
            {
                nz = 1;
                dct[coeff] = level;
                break;
            }
            level -= sign;
        }
    }
    return nz;
}

int FN(optimize_chroma_2x2_dc)( dctcoef dct[4], int dmf ) { return optimize_chroma_dc( dct, dmf, 0 ); }
int FN(optimize_chroma_2x4_dc)( dctcoef dct[8], int dmf ) { return optimize_chroma_dc( dct, dmf, 1 ); }

/* denoise_dct, reference common/quant.c:295-306 */
void FN(denoise_dct)( dctcoef *dct, uint32_t *sum, const udctcoef *offset, int size )
{
    for( int i = 0; i < size; i++ )
    {
        int level = dct[i];
        int sign = level >> 31;
        level = (level + sign) ^ sign;
        sum[i] += level;
        level -= offset[i];
        dct[i] = level < 0 ? 0 : (level ^ sign) - sign;
    }
}

/* decimate_score15/16/64, reference common/quant.c:318-363, tables common/tables.c:373-383 */
static const uint8_t decimate_table4[16] = { 3,2,2,1,1,1,0,0,0,0,0,0,0,0,0,0 };
static const uint8_t decimate_table8[64] = {
    3,3,3,3,2,2,2,2,2,2,2,2,1,1,1,1, 1,1,1,1,1,1,1,1,0,0,0,0,0,0,0,0,
    0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0, 0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0 };

static int decimate_score( const dctcoef *dct, int i_max )
{
    const uint8_t *ds = i_max == 64 ? decimate_table8 : decimate_table4;
    int score = 0, idx = i_max - 1;
    while( idx >= 0 && dct[idx] == 0 )
        idx--;
    while( idx >= 0 )
    {
        if( (unsigned)(dct[idx--] + 1) > 2 )
            return 9;
        int run = 0;
        while( idx >= 0 && dct[idx] == 0 )
        {
            idx--;
            run++;
        }
        score += ds[run];
    }
    return score;
}

int FN(decimate_score15)( dctcoef *dct ) { return decimate_score( dct + 1, 15 ); }
int FN(decimate_score16)( dctcoef *dct ) { return decimate_score( dct, 16 ); }
int FN(decimate_score64)( dctcoef *dct ) { return decimate_score( dct, 64 ); }

/* coeff_last4/8/15/16/64 (the 15 form is called with dct+1 by its users via
 * coeff_last[DCT_LUMA_AC]), reference common/quant.c:365-378 */
int FN(coeff_last)( const dctcoef *l, int num )
{
    int i = num - 1;
    while( i >= 0 && l[i] == 0 )
        i--;
    return i;
}

/* coeff_level_run4/8/15/16, reference common/quant.c:380-398; out = {last, mask,
 * level[0..total)} as x264_run_level_t (common/bitstream.h:50-55) */
int FN(coeff_level_run)( const dctcoef *dct, int num, int32_t *last, int32_t *mask, dctcoef *level )
{
    int i_last = *last = FN(coeff_last)( dct, num );
    int total = 0, m = 0;
    do
    {
        level[total++] = dct[i_last];
        m |= 1 << i_last;
        while( --i_last >= 0 && dct[i_last] == 0 );
    } while( i_last >= 0 );
    *mask = m;
    return total;
}

/* zigzag scans and zigzag_sub, reference common/dct.c:768-925 */
static const uint8_t zz8_frame[64][2] = {   /* (y, x): level[i] = dct[x*8+y] */
    {0,0},{0,1},{1,0},{2,0},{1,1},{0,2},{0,3},{1,2},{2,1},{3,0},{4,0},{3,1},{2,2},{1,3},{0,4},{0,5},
    {1,4},{2,3},{3,2},{4,1},{5,0},{6,0},{5,1},{4,2},{3,3},{2,4},{1,5},{0,6},{0,7},{1,6},{2,5},{3,4},
    {4,3},{5,2},{6,1},{7,0},{7,1},{6,2},{5,3},{4,4},{3,5},{2,6},{1,7},{2,7},{3,6},{4,5},{5,4},{6,3},
    {7,2},{7,3},{6,4},{5,5},{4,6},{3,7},{4,7},{5,6},{6,5},{7,4},{7,5},{6,6},{5,7},{6,7},{7,6},{7,7} };
static const uint8_t zz8_field[64][2] = {
    {0,0},{1,0},{2,0},{0,1},{1,1},{3,0},{4,0},{2,1},{0,2},{3,1},{5,0},{6,0},{7,0},{4,1},{1,2},{0,3},
    {2,2},{5,1},{6,1},{7,1},{3,2},{1,3},{0,4},{2,3},{4,2},{5,2},{6,2},{7,2},{3,3},{1,4},{0,5},{2,4},
    {4,3},{5,3},{6,3},{7,3},{3,4},{1,5},{0,6},{2,5},{4,4},{5,4},{6,4},{7,4},{3,5},{1,6},{2,6},{4,5},
    {5,5},{6,5},{7,5},{3,6},{0,7},{1,7},{4,6},{5,6},{6,6},{7,6},{2,7},{3,7},{4,7},{5,7},{6,7},{7,7} };
static const uint8_t zz4_frame[16][2] = {
    {0,0},{0,1},{1,0},{2,0},{1,1},{0,2},{0,3},{1,2},{2,1},{3,0},{3,1},{2,2},{1,3},{2,3},{3,2},{3,3} };
static const uint8_t zz4_field[16][2] = {
    {0,0},{1,0},{0,1},{2,0},{3,0},{1,1},{2,1},{3,1},{0,2},{1,2},{2,2},{3,2},{0,3},{1,3},{2,3},{3,3} };

void FN(zigzag_scan_8x8)( int field, dctcoef level[64], const dctcoef dct[64] )
{
    const uint8_t (*t)[2] = field ? zz8_field : zz8_frame;
    for( int i = 0; i < 64; i++ )
        level[i] = dct[t[i][1]*8 + t[i][0]];
}

void FN(zigzag_scan_4x4)( int field, dctcoef level[16], const dctcoef dct[16] )
{
    const uint8_t (*t)[2] = field ? zz4_field : zz4_frame;
    for( int i = 0; i < 16; i++ )
        level[i] = dct[t[i][1]*4 + t[i][0]];
}

/* zigzag_sub_{4x4,4x4ac,8x8}: level = zigzag(src - dst), then dst = src (the
 * reference's COPY4x4 / COPY8x8); src stride FENC_STRIDE, dst FDEC_STRIDE.
 * kind 0 = 4x4, 1 = 4x4ac (dc out, level[0] = 0), 2 = 8x8 */
int FN(zigzag_sub_s)( int kind, int field, dctcoef *level, const pixel *src, intptr_t ss, pixel *dst, intptr_t ds,
                      dctcoef *dc )
{
    int n = kind == 2 ? 64 : 16, w = kind == 2 ? 8 : 4, nz = 0;
    const uint8_t (*t)[2] = kind == 2 ? (field ? zz8_field : zz8_frame) : (field ? zz4_field : zz4_frame);
    for( int i = 0; i < n; i++ )
    {
        int y = t[i][0], x = t[i][1];
        int v = src[x + y*ss] - dst[x + y*ds];
        if( kind == 1 && i == 0 )
        {
            *dc = v;
            level[0] = 0;
            continue;
        }
        level[i] = v;
        nz |= level[i];
    }
    for( int y = 0; y < w; y++ )
        for( int x = 0; x < w; x++ )
            dst[x + y*ds] = src[x + y*ss];
    return !!nz;
}

/* zigzag_interleave_8x8_cavlc, reference common/dct.c:927-940 */
void FN(zigzag_interleave_8x8_cavlc)( dctcoef *dst, const dctcoef *src, uint8_t *nnz )
{
    for( int i = 0; i < 4; i++ )
    {
        int nz = 0;
        for( int j = 0; j < 16; j++ )
        {
            nz |= src[i + j*4];
            dst[i*16 + j] = src[i + j*4];
        }
        nnz[(i & 1) + (i >> 1)*8] = !!nz;
    }
}

/* dequant4_mf / dequant8_mf of x264_cqm_init, reference common/set.c:31-39, 52-61, 124-159 */
static const uint8_t dequant4_scale[6][3] = {
    { 10, 13, 16 }, { 11, 14, 18 }, { 13, 16, 20 }, { 14, 18, 23 }, { 16, 20, 25 }, { 18, 23, 29 } };
static const uint8_t dequant8_scale[6][6] = {
    { 20, 18, 32, 19, 25, 24 }, { 22, 19, 35, 21, 28, 26 }, { 26, 23, 42, 24, 33, 31 },
    { 28, 25, 45, 26, 35, 33 }, { 32, 28, 51, 30, 40, 38 }, { 36, 32, 58, 34, 46, 43 } };

void FN(cqm_dequant)( const uint8_t *const scaling_list[8], int b_transform_8x8, int *dq4, int *dq8 )
{
    for( int q = 0; q < 6; q++ )
    {
        for( int l = 0; l < 4; l++ )
            for( int i = 0; i < 16; i++ )
                dq4[(l*6 + q)*16 + i] = dequant4_scale[q][(i&1) + ((i>>2)&1)] * scaling_list[l][i];
        if( b_transform_8x8 )
            for( int l = 0; l < 2; l++ )
                for( int i = 0; i < 64; i++ )
                    dq8[(l*6 + q)*64 + i] = dequant8_scale[q][quant8_scan[((i>>1)&12) | (i&3)]] * scaling_list[4+l][i];
    }
}

/*============================================================================
 * frame-level helpers composed from the entries above (checkers for the
 * batched HIP entries)
 *==========================================================================*/

/* exhaustive 16x16 SAD table, semantics of x264hip_*_me_search_full */
void FN(me_search_full)( const pixel *fenc, intptr_t fs, const pixel *ref, intptr_t rs,
                         int mb_width, int mb_height, int range, sadt *table )
{
    int w = 2*range + 1;
    for( int mby = 0; mby < mb_height; mby++ )
        for( int mbx = 0; mbx < mb_width; mbx++ )
        {
            const pixel *f = fenc + 16*(mby*fs + mbx);
            sadt *t = table + ((size_t)mby*mb_width + mbx) * w * w;
            for( int j = 0; j < w; j++ )
                for( int i = 0; i < w; i++ )
                    t[j*w+i] = (sadt)FN(sad)( 0, f, fs, ref + (16*mby + j - range)*rs + 16*mbx + i - range, rs );
        }
}

/* exhaustive 8x8 quadrant SAD tables, semantics of x264hip_*_me_search_full8:
 * table8[mb][q][j][i] = sad_8x8 (pixel.c:55-80, PIXEL_8x8) of quadrant q (0 = top-left,
 * 1 = top-right, 2 = bottom-left, 3 = bottom-right) of the MB at mv (i - range, j - range) */
void FN(me_search_full8)( const pixel *fenc, intptr_t fs, const pixel *ref, intptr_t rs,
                          int mb_width, int mb_height, int range, uint16_t *table8 )
{
    int w = 2*range + 1;
    for( int mby = 0; mby < mb_height; mby++ )
        for( int mbx = 0; mbx < mb_width; mbx++ )
            for( int q = 0; q < 4; q++ )
            {
                const int px = 8*(q & 1), py = 8*(q >> 1);
                const pixel *f = fenc + (16*mby + py)*fs + 16*mbx + px;
                uint16_t *t = table8 + (((size_t)mby*mb_width + mbx) * 4 + q) * w * w;
                for( int j = 0; j < w; j++ )
                    for( int i = 0; i < w; i++ )
                        t[j*w+i] = (uint16_t)FN(sad)( 3, f, fs, ref + (16*mby + py + j - range)*rs + 16*mbx + px + i - range,
                                                      rs );
            }
}

/* ESA decisions of an MB's eight sub-partitions, semantics of x264hip_*_me_search_esa8: the
 * plain exhaustive form of encoder/me.c:618-631 (what its ads path reproduces) for each of
 * PIXEL_16x8 (partitions 0, 1: rows 0 / 8), PIXEL_8x16 (2, 3: columns 0 / 8) and PIXEL_8x8
 * (4..7: (8(i&1), 8(i>>1))), at the block offsets of analyse.c:1425,1480,1546.  The window is
 * [max(bmx - me_range, mv_x_min), min(bmx + me_range, mv_x_max)] x the same in y with the width
 * rounded (max_x - min_x + 3) & ~3; cost = sad of the partition (pixel.c:55-80) +
 * cost_mv[4*mx - mvp_x] + cost_mv[4*my - mvp_y] (COST_MV, me.c:63-70), strict-< update from
 * (init_cost, bmx, bmy) in my-major raster order (COPY3_IF_LT, me.h:87-93).  par[(8*mb + p)*8]
 * as me_esa_argmin's, init_cost[8*mb + p], out[(8*mb + p)*3] = { cost, mx, my }. */
static const uint8_t esa8_part[8][3] = { { 1, 0, 0 }, { 1, 0, 8 }, { 2, 0, 0 }, { 2, 8, 0 },
                                         { 3, 0, 0 }, { 3, 8, 0 }, { 3, 0, 8 }, { 3, 8, 8 } };
void FN(me_search_esa8)( const pixel *fenc, intptr_t fs, const pixel *ref, intptr_t rs, int mb_width,
                         int mb_height, int me_range, const int16_t *par, const int32_t *init_cost,
                         const uint16_t *cost_mv, int32_t *out )
{
    for( int mb = 0; mb < mb_width * mb_height; mb++ )
        for( int p = 0; p < 8; p++ )
        {
            const int i = 8 * mb + p, ipix = esa8_part[p][0];
            const int bx = 16 * (mb % mb_width) + esa8_part[p][1], by = 16 * (mb / mb_width) + esa8_part[p][2];
            const int16_t *q = par + 8 * i;
            int bmx = q[0], bmy = q[1], bcost = init_cost[i];
            const uint16_t *cx = cost_mv - q[2], *cy = cost_mv - q[3];
            const int min_x = bmx - me_range > q[4] ? bmx - me_range : q[4];
            const int min_y = bmy - me_range > q[5] ? bmy - me_range : q[5];
            const int max_x = bmx + me_range < q[6] ? bmx + me_range : q[6];
            const int max_y = bmy + me_range < q[7] ? bmy + me_range : q[7];
            const int width = (max_x - min_x + 3) & ~3;
            for( int my = min_y; my <= max_y; my++ )
                for( int mx = min_x; mx < min_x + width; mx++ )
                {
                    int cost = FN(sad)( ipix, fenc + by * fs + bx, fs, ref + (by + my) * rs + bx + mx, rs )
                             + cx[mx * 4] + cy[my * 4];
                    if( cost < bcost )
                    {
                        bcost = cost;
                        bmx = mx;
                        bmy = my;
                    }
                }
            out[3 * i] = bcost;
            out[3 * i + 1] = bmx;
            out[3 * i + 2] = bmy;
        }
}

/* columns of a x264hip_*_me_search_centred table: me.c's ESA window around the centre,
 * [cx - range, cx + range + 2] (the width rounding (max_x - min_x + 3) & ~3, me.c:626, ends
 * up to two columns past max_x) plus the origin's alignment down to a dword (3 / 1 pixels),
 * rounded up to a multiple of 4 -- every column is a SAD */
static int cen_pitch( int range )
{
    return (2*range + (BIT_DEPTH == 8 ? 6 : 4) + 3) & ~3;
}

/* window origin of x264hip_*_me_search_centred for one MB: (cx, cy) - range,
 * clamped so every pixel the kernels fetch lies in the 32-pixel padded plane,
 * then aligned down to 4 (8 bit) / 2 (10 bit) pixels; returned relative to the MB */
static void me_window( int mbx, int mby, int mb_width, int mb_height, int range, int cx, int cy, int *ox, int *oy )
{
    const int P = cen_pitch( range ), al = BIT_DEPTH == 8 ? 4 : 2;
    int ax = 16*mbx + cx - range, ay = 16*mby + cy - range;
    int hx = 16*mb_width + 12 - P, hy = 16*mb_height + 16 - 2*range;
    ax = ax < -32 ? -32 : ax > hx ? hx : ax;
    ay = ay < -32 ? -32 : ay > hy ? hy : ay;
    ax &= ~(al - 1);
    *ox = ax - 16*mbx;
    *oy = ay - 16*mby;
}

/* semantics of x264hip_*_me_search_centred: table[mb][j][i] = SAD at mv
 * (ox + i, oy + j), j < 2*range+1, i < cen_pitch(range), with (ox, oy) = origin[mb]
 * from me_window */
void FN(me_search_centred)( const pixel *fenc, intptr_t fs, const pixel *ref, intptr_t rs, int mb_width,
                            int mb_height, int range, const int16_t *centre, sadt *table, int16_t *origin )
{
    int w = 2*range + 1, pw = cen_pitch( range );
    for( int mby = 0; mby < mb_height; mby++ )
        for( int mbx = 0; mbx < mb_width; mbx++ )
        {
            size_t mb = (size_t)mby*mb_width + mbx;
            int ox, oy;
            me_window( mbx, mby, mb_width, mb_height, range, centre[2*mb], centre[2*mb+1], &ox, &oy );
            origin[2*mb] = (int16_t)ox;
            origin[2*mb+1] = (int16_t)oy;
            const pixel *f = fenc + 16*(mby*fs + mbx);
            sadt *t = table + mb * w * pw;
            for( int j = 0; j < w; j++ )
                for( int i = 0; i < pw; i++ )
                    t[j*pw+i] = (sadt)FN(sad)( 0, f, fs, ref + (16*mby + oy + j)*rs + 16*mbx + ox + i, rs );
        }
}

/* fused inter-luma residual path, semantics of x264hip_*_mb_dct_quant
 * (reference encoder/macroblock.c:806-884 without trellis/decimation) */
void FN(mb_dct_quant)( int transform, const pixel *fenc, intptr_t fs, const pixel *pred, intptr_t ps,
                       int mb_width, int mb_height, const udctcoef *mf, const udctcoef *bias,
                       dctcoef *dct, int32_t *nz )
{
    for( int mby = 0; mby < mb_height; mby++ )
        for( int mbx = 0; mbx < mb_width; mbx++ )
        {
            size_t mb = (size_t)mby*mb_width + mbx;
            const pixel *f = fenc + 16*(mby*fs + mbx), *p = pred + 16*(mby*ps + mbx);
            dctcoef *d = dct + mb*256;
            int mask = 0;
            if( transform == 8 )
            {
                sub16x16_dct8_s( (dctcoef(*)[64])d, f, fs, p, ps );
                for( int i8 = 0; i8 < 4; i8++ )
                    mask |= FN(quant_8x8)( d + 64*i8, mf, bias ) << i8;
            }
            else
            {
                sub16x16_dct_s( (dctcoef(*)[16])d, f, fs, p, ps );
                for( int i8 = 0; i8 < 4; i8++ )
                    mask |= FN(quant_4x4x4)( (dctcoef(*)[16])(d + 64*i8), mf, bias ) << (4*i8);
            }
            nz[mb] = mask;
        }
}

/* frame-level reconstruction, semantics of x264hip_*_mb_dequant_idct_add:
 * per MB dequant_4x4 x16 + add16x16_idct, or dequant_8x8 x4 + add16x16_idct8,
 * of a copy of dct[mb][256] onto recon = pred (one frame) */
void FN(mb_dequant_idct_add)( int transform, const dctcoef *dct, int mb_width, int mb_height, const int *dmf,
                              const int32_t *qp, const pixel *pred, intptr_t ps, pixel *recon, intptr_t rs )
{
    dctcoef tmp[256];
    for( int mby = 0; mby < mb_height; mby++ )
        for( int mbx = 0; mbx < mb_width; mbx++ )
        {
            size_t mb = (size_t)mby*mb_width + mbx;
            memcpy( tmp, dct + mb*256, sizeof(tmp) );
            pixel *r = recon + 16*(mby*rs + mbx);
            const pixel *p = pred + 16*(mby*ps + mbx);
            for( int y = 0; y < 16; y++ )
                memcpy( r + y*rs, p + y*ps, 16 * sizeof(pixel) );
            if( transform == 8 )
            {
                for( int i = 0; i < 4; i++ )
                    FN(dequant_8x8)( tmp + 64*i, (int(*)[64])dmf, qp[mb] );
                add16x16_idct8_s( r, rs, (dctcoef(*)[64])tmp );
            }
            else
            {
                for( int i = 0; i < 16; i++ )
                    FN(dequant_4x4)( tmp + 16*i, (int(*)[16])dmf, qp[mb] );
                add16x16_idct_s( r, rs, (dctcoef(*)[16])tmp );
            }
        }
}

/*============================================================================
 * motion compensation inputs — reference common/mc.c
 *==========================================================================*/

/* hpel_filter, reference common/mc.c:173-196 (6-tap, clip, centre via int16
 * intermediate with the 10-bit bias `pad`) */
#define TAPFILTER(pix, d) ((pix)[x-2*d] + (pix)[x+3*d] - 5*((pix)[x-d] + (pix)[x+2*d]) + 20*((pix)[x] + (pix)[x+d]))
void FN(hpel_filter)( pixel *dsth, pixel *dstv, pixel *dstc, const pixel *src,
                      intptr_t stride, int width, int height, int16_t *buf )
{
    const int pad = (BIT_DEPTH > 9) ? (-10 * PIXEL_MAX) : 0;
    for( int y = 0; y < height; y++ )
    {
        for( int x = -2; x < width + 3; x++ )
        {
            int v = TAPFILTER( src, stride );
            dstv[x] = clip_pixel( (v + 16) >> 5 );
            buf[x+2] = v + pad;
        }
        for( int x = 0; x < width; x++ )
            dstc[x] = clip_pixel( (TAPFILTER( buf+2, 1 ) - 32*pad + 512) >> 10 );
        for( int x = 0; x < width; x++ )
            dsth[x] = clip_pixel( (TAPFILTER( src, 1 ) + 16) >> 5 );
        dsth += stride;
        dstv += stride;
        dstc += stride;
        src += stride;
    }
}

/* get_ref without weighting: qpel from two hpel planes; reference common/mc.c:221-249
 * with x264_hpel_ref0/1 of common/tables.c:183-184 */
static const uint8_t hpel_ref0[16] = {0,1,1,1,0,1,1,1,2,3,3,3,0,1,1,1};
static const uint8_t hpel_ref1[16] = {0,0,1,0,2,2,3,2,2,2,3,2,2,2,3,2};
const pixel *FN(get_ref)( pixel *dst, intptr_t *dst_stride, const pixel *const src[4], intptr_t stride,
                          int mvx, int mvy, int w, int h )
{
    int qpel_idx = ((mvy&3)<<2) + (mvx&3);
    intptr_t offset = (mvy>>2)*stride + (mvx>>2);
    const pixel *src1 = src[hpel_ref0[qpel_idx]] + offset + ((mvy&3) == 3) * stride;
    if( qpel_idx & 5 )
    {
        const pixel *src2 = src[hpel_ref1[qpel_idx]] + offset + ((mvx&3) == 3);
        for( int y = 0; y < h; y++ )
            for( int x = 0; x < w; x++ )
                dst[y * *dst_stride + x] = ( src1[y*stride + x] + src2[y*stride + x] + 1 ) >> 1;
        return dst;
    }
    *dst_stride = stride;
    return src1;
}

/* mc_weight (reference common/mc.c:117-137): explicit weighted prediction of a w x h
 * block, offset scaled by 1 << (BIT_DEPTH-8); denom 0 has no rounding term.  In place
 * is allowed (get_ref weights its own average, mc.c:235-236). */
void FN(mc_weight)( pixel *dst, intptr_t ds, const pixel *src, intptr_t ss, int scale, int denom, int offset,
                    int w, int h )
{
    const int off = offset * (1 << (BIT_DEPTH - 8));
    for( int y = 0; y < h; y++ )
        for( int x = 0; x < w; x++ )
        {
            const int v = src[y * ss + x];
            dst[y * ds + x] = (pixel)clip_pixel( denom >= 1 ? ((v * scale + (1 << (denom - 1))) >> denom) + off
                                                            : v * scale + off );
        }
}

/* get_ref with a weight (reference common/mc.c:221-249 with weight->weightfn set):
 * the qpel average (or the plane itself) then mc_weight into dst */
static const pixel *get_ref_w( pixel *dst, intptr_t *dst_stride, const pixel *const src[4], intptr_t stride,
                               int mvx, int mvy, int w, int h, const int *wt )
{
    const pixel *r = FN(get_ref)( dst, dst_stride, src, stride, mvx, mvy, w, h );
    if( !wt )
        return r;
    FN(mc_weight)( dst, 16, r, *dst_stride, wt[0], wt[1], wt[2], w, h );
    *dst_stride = 16;
    return dst;
}

/* x264_weight_scale_plane (reference common/frame.c:825-842): the plane weighted in
 * strips of 16 rows, 16-wide blocks while x < width-8 and one 8-wide block after, so
 * up to 7 columns past `width` are weighted too (pointers at the region's top-left). */
void FN(weight_scale_plane)( pixel *dst, intptr_t ds, const pixel *src, intptr_t ss, int width, int height,
                             int scale, int denom, int offset )
{
    while( height > 0 )
    {
        const int hh = height < 16 ? height : 16;
        int x;
        for( x = 0; x < width - 8; x += 16 )
            FN(mc_weight)( dst + x, ds, src + x, ss, scale, denom, offset, 16, hh );
        if( x < width )
            FN(mc_weight)( dst + x, ds, src + x, ss, scale, denom, offset, 8, hh );
        height -= 16;
        dst += 16 * ds;
        src += 16 * ss;
    }
}

/* whole-frame half-pel planes: x264_frame_filter (reference common/mc.c:704-726)
 * over every MB row (rows [-8, H+8), columns [-8, W+8) of hpel_filter) followed by
 * x264_frame_expand_border_filtered (common/frame.c:599-625: edges taken from
 * x = -4 / W+3 and y = -8 / H+7, padh 28, padv 24).  Pointers at pixel (0,0),
 * planes padded by 32. */
void FN(frame_filter)( const pixel *src, pixel *dh, pixel *dv, pixel *dc, intptr_t stride, int width, int height )
{
    int16_t *buf = malloc( (width + 48) * sizeof(int16_t) );
    intptr_t offs = -8 * stride - 8;
    FN(hpel_filter)( dh + offs, dv + offs, dc + offs, src + offs, stride, width + 16, height + 16, buf );
    free( buf );
    pixel *planes[3] = { dh, dv, dc };
    for( int p = 0; p < 3; p++ )
    {
        pixel *pl = planes[p];
        for( int y = -8; y < height + 8; y++ )
        {
            pixel *row = pl + y * stride;
            for( int x = -32; x < -4; x++ )
                row[x] = row[-4];
            for( int x = width + 4; x < width + 32; x++ )
                row[x] = row[width + 3];
        }
        for( int y = -32; y < -8; y++ )
            memcpy( pl + y * stride - 32, pl - 8 * stride - 32, (width + 64) * sizeof(pixel) );
        for( int y = height + 8; y < height + 32; y++ )
            memcpy( pl + y * stride - 32, pl + (height + 7) * stride - 32, (width + 64) * sizeof(pixel) );
    }
}

/* list form of the qpel candidate costs (get_ref then sad / satd), semantics of
 * x264hip_*_subpel_cmp_batch */
void FN(subpel_list)( int op, int i_pixel, const pixel *fenc, intptr_t fs, const pixel *p0, const pixel *p1,
                      const pixel *p2, const pixel *p3, intptr_t rs, const int64_t *fenc_off, const int32_t *qxy,
                      int n, int32_t *scores )
{
    const pixel *planes[4] = { p0, p1, p2, p3 };
    pixel tmp[16 * 16];
    for( int i = 0; i < n; i++ )
    {
        intptr_t ts = 16;
        int qx = qxy[2*i], qy = qxy[2*i+1];
        /* get_ref takes the mv relative to a block origin: use origin (0,0) and the
         * absolute qpel position as the mv */
        const pixel *r = FN(get_ref)( tmp, &ts, planes, rs, qx, qy, pixel_w[i_pixel], pixel_h[i_pixel] );
        const pixel *a = fenc + fenc_off[i];
        scores[i] = op == 0 ? FN(sad)( i_pixel, a, fs, r, ts ) : FN(satd)( i_pixel, a, fs, r, ts );
    }
}

/* exhaustive integer-pel search decision over a full-search table, restating the
 * plain exhaustive form of the ESA case of x264_me_search_ref (reference
 * encoder/me.c:618-631, which the ads successive-elimination path :632-771
 * reproduces exactly): window clipped by the mv limits, width rounded as
 * (max_x - min_x + 3) & ~3, cost = sad + p_cost_mvx[mx*4] + p_cost_mvy[my*4]
 * with p_cost_mv* = cost_mv - mvp (me.c:60-70, 230-231), strict-< update from
 * the predictor result (COPY3_IF_LT, me.h:87-93), my-major raster order.
 * par[8*i] = { bmx, bmy, mvp_x, mvp_y, mv_x_min, mv_y_min, mv_x_max, mv_y_max };
 * Without an origin the table is a full-search table (2R+1 columns at pitch align4(2R+1),
 * centred on mv (0,0)); with one, a me_search_centred table (cen_pitch(R) columns). */
void FN(me_esa_argmin)( const sadt *table, int R, int nmb, int me_range, const int16_t *origin, const int16_t *par,
                        const int32_t *init_cost, const uint16_t *cost_mv, int32_t *out )
{
    const int W = 2 * R + 1, P = origin ? cen_pitch( R ) : (W + 3) & ~3, C = origin ? P : W;
    for( int i = 0; i < nmb; i++ )
    {
        const int16_t *p = par + 8 * i;
        int bmx = p[0], bmy = p[1];
        const uint16_t *cx = cost_mv - p[2], *cy = cost_mv - p[3];
        int min_x = bmx - me_range > p[4] ? bmx - me_range : p[4];
        int min_y = bmy - me_range > p[5] ? bmy - me_range : p[5];
        int max_x = bmx + me_range < p[6] ? bmx + me_range : p[6];
        int max_y = bmy + me_range < p[7] ? bmy + me_range : p[7];
        int width = (max_x - min_x + 3) & ~3;
        int bcost = init_cost[i];
        const sadt *t = table + (size_t)i * W * P;
        const int ox = origin ? origin[2*i] : -R, oy = origin ? origin[2*i+1] : -R;
        for( int my = min_y; my <= max_y; my++ )
            for( int mx = min_x; mx < min_x + width; mx++ )
            {
                if( mx - ox < 0 || mx - ox >= C || my - oy < 0 || my - oy >= W )
                    continue;           /* outside the table: not evaluated */
                int cost = t[(my - oy) * P + mx - ox] + cx[mx * 4] + cy[my * 4];
                if( cost < bcost )
                {
                    bcost = cost;
                    bmx = mx;
                    bmy = my;
                }
            }
        out[3 * i] = bcost;
        out[3 * i + 1] = bmx;
        out[3 * i + 2] = bmy;
    }
}

/* refine_subpel (reference encoder/me.c:865-992) for a list of partitions, semantics of
 * x264hip_*_me_refine_subpel_ex (p_halfpel_thresh = NULL; refine_core below takes it, for
 * me_refine_qpel_refdupe and me_search_ref_thresh).  Iterations from subpel_iterations
 * (me.c:38-50): refine_qpel = 0 is the call of x264_me_search_ref (me.c:791-797, entries
 * 2-3), 1 the one of x264_me_refine_qpel (me.c:801-810, entries 0-1).  fpelcmp = satd iff
 * fpel_satd (TESA) and subme > 1, mbcmp / mbcmp_unaligned = satd iff subme > 1
 * (encoder.c:1409-1426).  fenc / planes point at pixel (0,0) of one frame (planes = F, H, V,
 * C); pos[2*i] = the partition's top-left pixel; par[8*i] = { mvx, mvy (qpel, m->mv), mvp_x,
 * mvp_y, mv_min_spel x, y, mv_max_spel x, y }; cost[i] = m->cost; cost_mv at mvd 0.
 * out[4*i] = { cost, mvx, mvy, cost_mv }; nevals[i] (when given) = the reference's cmp calls:
 * luma SADs | luma SATDs << 16 | chroma mbcmp calls << 24.
 * ext (NULL = luma only, unweighted) = { b_chroma_me (h->mb.b_chroma_me), chroma_format (1
 * 4:2:0, 2 4:2:2, 3 4:4:4), mvy_offset (me.c:875), then m->weight[0..2] as { weighted,
 * scale, denom, offset } }.  fenc_c = the frame's NV12 / NV16 plane in [0] or its U, V planes
 * (4:4:4), stride fcs; ref_c = the reference's NV12 / NV16 plane in [0] or (4:4:4) the F, H,
 * V, C planes of U then of V, stride rcs; all at pixel (0,0). */
static const uint8_t subpel_iterations[12][4] = { {0,0,0,0}, {1,1,0,0}, {0,1,1,0}, {0,2,1,0}, {0,2,1,1},
                                                  {0,2,1,2}, {0,0,2,2}, {0,0,2,2}, {0,0,4,10}, {0,0,4,10},
                                                  {0,0,4,10}, {0,0,4,10} };
/* x264_luma2chroma_pixel (reference common/pixel.h:70-76), partitions 16x16 .. 8x8 */
static const uint8_t luma2chroma_pixel[4][4] = { { 0 }, { 3, 4, 5, 6 }, { 2, 3, 7, 5 }, { 0, 1, 2, 3 } };
void FN(mc_chroma)( pixel *dstu, pixel *dstv, intptr_t ds, const pixel *src, intptr_t ss, int mvx, int mvy,
                    int w, int h );

typedef struct
{
    int b_chroma_me, cf, mvy_offset, satd, i_pixel, bx, by;
    const int *wt[3];                    /* { scale, denom, offset } of a weighted plane, or NULL */
    const pixel *fenc_c[2], *ref_c[8];
    intptr_t fcs, rcs;
    int nchroma;
} FN(rs_chroma_t);

/* the chroma half of COST_MV_SATD (me.c:833-861): U's cost added when the luma cost beats
 * bcost, then V's when the sum still does */
static int FN(rs_chroma)( FN(rs_chroma_t) *c, int mx, int my, int cost, int bcost )
{
    const int i_pixel = c->i_pixel, bw = pixel_w[i_pixel], bh = pixel_h[i_pixel];
    pixel pix[2][16 * 16];
    if( c->cf == 3 )
    {
        for( int p = 0; p < 2 && cost < bcost; p++ )
        {
            const pixel *q[4];
            for( int k = 0; k < 4; k++ )
                q[k] = c->ref_c[4 * p + k] + c->by * c->rcs + c->bx;
            intptr_t ts = 16;
            const pixel *r = get_ref_w( pix[p], &ts, q, c->rcs, mx, my, bw, bh, c->wt[1 + p] );
            const pixel *f = c->fenc_c[p] + c->by * c->fcs + c->bx;
            cost += c->satd ? FN(satd)( i_pixel, f, c->fcs, r, ts ) : FN(sad)( i_pixel, f, c->fcs, r, ts );
            c->nchroma++;
        }
        return cost;
    }
    const int vs = c->cf == 1, cw = bw >> 1, ch = bh >> vs, cpix = luma2chroma_pixel[c->cf][i_pixel];
    const intptr_t crow = (intptr_t)(c->by >> vs);
    FN(mc_chroma)( pix[0], pix[1], 16, c->ref_c[0] + crow * c->rcs + c->bx, c->rcs, mx,
                   2 * (my + c->mvy_offset) >> vs, cw, ch );
    pixel fe[2][16 * 16];
    for( int y = 0; y < ch; y++ )
        for( int x = 0; x < cw; x++ )
            for( int p = 0; p < 2; p++ )
                fe[p][16 * y + x] = c->fenc_c[0][(crow + y) * c->fcs + c->bx + 2 * x + p];
    for( int p = 0; p < 2 && cost < bcost; p++ )
    {
        if( c->wt[1 + p] )
            FN(mc_weight)( pix[p], 16, pix[p], 16, c->wt[1 + p][0], c->wt[1 + p][1], c->wt[1 + p][2], cw, ch );
        cost += c->satd ? FN(satd)( cpix, fe[p], 16, pix[p], 16 ) : FN(sad)( cpix, fe[p], 16, pix[p], 16 );
        c->nchroma++;
    }
    return cost;
}

/* kind 0: x264_me_search_ref's refine (me.c:794-796), 1: x264_me_refine_qpel (:801-810), 2:
 * x264_me_refine_qpel_refdupe (:812-815).  thr (or NULL): per partition *p_halfpel_thresh,
 * read and written (me.c:931-944); rcost (or NULL = 0): the i_ref_cost analyse.c:1271 / 1310
 * subtract from it before the call and add back after.  On the early exit out[4*i+3]
 * (m->cost_mv) is left as it was. */
static void FN(refine_core)( const pixel *fenc, intptr_t fs, const pixel *const planes[4], intptr_t rs,
                             int i_pixel, int subme, int kind, int fpel_satd, const int32_t *pos,
                             const int16_t *par, const int32_t *cost, const uint16_t *cost_mv, int n, int32_t *out,
                             int32_t *nevals, const int32_t *ext, const pixel *const fenc_c[2], intptr_t fcs,
                             const pixel *const ref_c[8], intptr_t rcs, int32_t *thr, const int32_t *rcost )
{
    const int bw = pixel_w[i_pixel], bh = pixel_h[i_pixel];
    const int refine_qpel = kind == 1;
    const int hpel_iters = kind == 2 ? 0 : subpel_iterations[subme][refine_qpel ? 0 : 2];
    const int qpel_iters = kind == 2 ? (subpel_iterations[subme][3] < 2 ? subpel_iterations[subme][3] : 2)
                                     : subpel_iterations[subme][refine_qpel ? 1 : 3];
    const int fsatd = fpel_satd && subme > 1, qsatd = subme > 1;
    /* me.c:872: b_chroma_me && (i_pixel <= PIXEL_8x8 || CHROMA444) */
    const int b_chroma_me = ext && ext[0] && (i_pixel <= 3 || ext[1] == 3);
    FN(rs_chroma_t) cc = { 0 };
    const int *wt0 = NULL;
    int wbuf[3][3];
    if( ext )
    {
        cc.b_chroma_me = b_chroma_me;
        cc.cf = ext[1];
        cc.mvy_offset = ext[2];
        cc.satd = qsatd;
        cc.i_pixel = i_pixel;
        for( int p = 0; p < 3; p++ )
        {
            for( int k = 0; k < 3; k++ )
                wbuf[p][k] = ext[4 + 4 * p + k];
            cc.wt[p] = ext[3 + 4 * p] ? wbuf[p] : NULL;
        }
        wt0 = cc.wt[0];
        if( b_chroma_me )
        {
            for( int p = 0; p < 2; p++ )
                cc.fenc_c[p] = fenc_c[p];
            for( int p = 0; p < 8; p++ )
                cc.ref_c[p] = ref_c[p];
            cc.fcs = fcs;
            cc.rcs = rcs;
        }
    }
    for( int i = 0; i < n; i++ )
    {
        const pixel *f = fenc + pos[2*i+1] * fs + pos[2*i];
        const pixel *q[4];
        for( int k = 0; k < 4; k++ )
            q[k] = planes[k] + pos[2*i+1] * rs + pos[2*i];
        cc.bx = pos[2*i];
        cc.by = pos[2*i+1];
        cc.nchroma = 0;
        const int16_t *p = par + 8 * i;
        const uint16_t *p_cost_mvx = cost_mv - p[2], *p_cost_mvy = cost_mv - p[3];
        const int mv_min_spel[2] = { p[4], p[5] }, mv_max_spel[2] = { p[6], p[7] };
        pixel tmp[16 * 16];
        /* get_ref with m->weight[0] (mc.c:221-249), then fpelcmp / mbcmp_unaligned */
#define RS_CMP( use_satd, mx, my ) ( ts = 16, r = get_ref_w( tmp, &ts, q, rs, mx, my, bw, bh, wt0 ), \
                                     (use_satd) ? (nsatd++, FN(satd)( i_pixel, f, fs, r, ts ))  \
                                                : (nsad++, FN(sad)( i_pixel, f, fs, r, ts )) )
        /* COST_MV_SATD's cost (me.c:826-863) against the running bcost */
#define RS_SATD( mx, my ) ( c_ = RS_CMP( qsatd, mx, my ) + p_cost_mvx[mx] + p_cost_mvy[my],           \
                            (b_chroma_me && c_ < bcost) ? FN(rs_chroma)( &cc, mx, my, c_, bcost ) : c_ )
        int nsad = 0, nsatd = 0, c_;
        intptr_t ts;
        const pixel *r;
        int bmx = p[0], bmy = p[1], bcost = cost[i];
        int odir = -1, bdir;
        int costs[4];
        if( hpel_iters )
        {
            if( subme < 3 )
            {
                int mx = p[2] < mv_min_spel[0] + 2 ? mv_min_spel[0] + 2 : p[2] > mv_max_spel[0] - 2 ? mv_max_spel[0] - 2 : p[2];
                int my = p[3] < mv_min_spel[1] + 2 ? mv_min_spel[1] + 2 : p[3] > mv_max_spel[1] - 2 ? mv_max_spel[1] - 2 : p[3];
                if( (mx - bmx) | (my - bmy) )
                {
                    int c = RS_CMP( fsatd, mx, my ) + p_cost_mvx[mx] + p_cost_mvy[my];
                    if( c < bcost ) { bcost = c; bmx = mx; bmy = my; }
                }
            }
            bcost <<= 6;
            for( int it = hpel_iters; it > 0; it-- )
            {
                int omx = bmx, omy = bmy;
                costs[0] = RS_CMP( fsatd, omx, omy - 2 ) + p_cost_mvx[omx] + p_cost_mvy[omy - 2];
                costs[1] = RS_CMP( fsatd, omx, omy + 2 ) + p_cost_mvx[omx] + p_cost_mvy[omy + 2];
                costs[2] = RS_CMP( fsatd, omx - 2, omy ) + p_cost_mvx[omx - 2] + p_cost_mvy[omy];
                costs[3] = RS_CMP( fsatd, omx + 2, omy ) + p_cost_mvx[omx + 2] + p_cost_mvy[omy];
                if( (costs[0] << 6) + 2 < bcost ) bcost = (costs[0] << 6) + 2;
                if( (costs[1] << 6) + 6 < bcost ) bcost = (costs[1] << 6) + 6;
                if( (costs[2] << 6) + 16 < bcost ) bcost = (costs[2] << 6) + 16;
                if( (costs[3] << 6) + 48 < bcost ) bcost = (costs[3] << 6) + 48;
                if( !(bcost & 63) )
                    break;
                bmx -= (int32_t)((uint32_t)bcost << 26) >> 29;
                bmy -= (int32_t)((uint32_t)bcost << 29) >> 29;
                bcost &= ~63;
            }
            bcost >>= 6;
        }
        if( !refine_qpel && (qsatd != fsatd || b_chroma_me) )
        {
            /* bcost = COST_MAX; COST_MV_SATD( bmx, bmy, -1 ) (me.c:925-929) */
            bcost = 1 << 28;
            bcost = RS_SATD( bmx, bmy );
        }
        if( thr )
        {
            /* early termination when examining multiple reference frames (me.c:931-944) */
            const int rc = rcost ? rcost[i] : 0;
            int t = thr[i] - rc;
            const int early = (bcost * 7) >> 3 > t;
            if( !early && bcost < t )
                t = bcost;
            thr[i] = t + rc;
            if( early )
            {
                out[4*i] = bcost;
                out[4*i+1] = bmx;
                out[4*i+2] = bmy;
                if( nevals )
                    nevals[i] = nsad | (nsatd << 16) | (cc.nchroma << 24);
                continue;
            }
        }
        if( subme != 1 )
        {
            bdir = -1;
            for( int it = qpel_iters; it > 0; it-- )
            {
                if( bmy <= mv_min_spel[1] || bmy >= mv_max_spel[1] || bmx <= mv_min_spel[0] || bmx >= mv_max_spel[0] )
                    break;
                odir = bdir;
                int omx = bmx, omy = bmy;
                static const int8_t qd[4][2] = { {0,-1}, {0,1}, {-1,0}, {1,0} };
                for( int dir = 0; dir < 4; dir++ )
                {
                    if( !refine_qpel && (dir ^ 1) == odir )
                        continue;
                    int mx = omx + qd[dir][0], my = omy + qd[dir][1];
                    int c = RS_SATD( mx, my );
                    if( c < bcost ) { bcost = c; bmx = mx; bmy = my; bdir = dir; }
                }
                if( bmx == omx && bmy == omy )
                    break;
            }
        }
        else if( bmy > mv_min_spel[1] && bmy < mv_max_spel[1] && bmx > mv_min_spel[0] && bmx < mv_max_spel[0] )
        {
            int omx = bmx, omy = bmy;
            costs[0] = RS_CMP( fsatd, omx, omy - 1 ) + p_cost_mvx[omx] + p_cost_mvy[omy - 1];
            costs[1] = RS_CMP( fsatd, omx, omy + 1 ) + p_cost_mvx[omx] + p_cost_mvy[omy + 1];
            costs[2] = RS_CMP( fsatd, omx - 1, omy ) + p_cost_mvx[omx - 1] + p_cost_mvy[omy];
            costs[3] = RS_CMP( fsatd, omx + 1, omy ) + p_cost_mvx[omx + 1] + p_cost_mvy[omy];
            bcost <<= 4;
            if( (costs[0] << 4) + 1 < bcost ) bcost = (costs[0] << 4) + 1;
            if( (costs[1] << 4) + 3 < bcost ) bcost = (costs[1] << 4) + 3;
            if( (costs[2] << 4) + 4 < bcost ) bcost = (costs[2] << 4) + 4;
            if( (costs[3] << 4) + 12 < bcost ) bcost = (costs[3] << 4) + 12;
            bmx -= (int32_t)((uint32_t)bcost << 28) >> 30;
            bmy -= (int32_t)((uint32_t)bcost << 30) >> 30;
            bcost >>= 4;
        }
#undef RS_SATD
#undef RS_CMP
        out[4*i] = bcost;
        out[4*i+1] = bmx;
        out[4*i+2] = bmy;
        out[4*i+3] = p_cost_mvx[bmx] + p_cost_mvy[bmy];
        if( nevals )
            nevals[i] = nsad | (nsatd << 16) | (cc.nchroma << 24);
    }
}

void FN(me_refine_subpel_ex)( const pixel *fenc, intptr_t fs, const pixel *const planes[4], intptr_t rs,
                              int i_pixel, int subme, int refine_qpel, int fpel_satd, const int32_t *pos,
                              const int16_t *par, const int32_t *cost, const uint16_t *cost_mv, int n, int32_t *out,
                              int32_t *nevals, const int32_t *ext, const pixel *const fenc_c[2], intptr_t fcs,
                              const pixel *const ref_c[8], intptr_t rcs )
{
    FN(refine_core)( fenc, fs, planes, rs, i_pixel, subme, !!refine_qpel, fpel_satd, pos, par, cost, cost_mv, n, out,
                     nevals, ext, fenc_c, fcs, ref_c, rcs, NULL, NULL );
}

/* x264_me_refine_qpel_refdupe (me.c:812-815) with p_halfpel_thresh (thr, rcost as refine_core) */
void FN(me_refine_qpel_refdupe)( const pixel *fenc, intptr_t fs, const pixel *const planes[4], intptr_t rs,
                                 int i_pixel, int subme, int fpel_satd, const int32_t *pos, const int16_t *par,
                                 const int32_t *cost, const uint16_t *cost_mv, int n, int32_t *out, int32_t *nevals,
                                 const int32_t *ext, const pixel *const fenc_c[2], intptr_t fcs,
                                 const pixel *const ref_c[8], intptr_t rcs, int32_t *thr, const int32_t *rcost )
{
    FN(refine_core)( fenc, fs, planes, rs, i_pixel, subme, 2, fpel_satd, pos, par, cost, cost_mv, n, out, nevals, ext,
                     fenc_c, fcs, ref_c, rcs, thr, rcost );
}

void FN(me_refine_subpel)( const pixel *fenc, intptr_t fs, const pixel *const planes[4], intptr_t rs, int i_pixel,
                           int subme, int refine_qpel, int fpel_satd, const int32_t *pos, const int16_t *par,
                           const int32_t *cost, const uint16_t *cost_mv, int n, int32_t *out, int32_t *nevals )
{
    FN(me_refine_subpel_ex)( fenc, fs, planes, rs, i_pixel, subme, refine_qpel, fpel_satd, pos, par, cost, cost_mv,
                             n, out, nevals, NULL, NULL, 0, NULL, 0 );
}

/* x264_me_search_ref (reference encoder/me.c:182-798) for a list of partitions of one frame
 * with me = DIA (0), HEX (1) or UMH (2) (me_search_ref_thresh: with p_halfpel_thresh as
 * refine_core reads it; me_search_ref: NULL): the predictor checks
 * (:214-318, x264_predictor_clip / _roundclip common/common.h:774-805), the integer search
 * (:320-616; UMH's adaptive range with x264_predictor_difference, common/base.h:248-257), the
 * qpel conversion (:774-789), then refine_subpel as FN(me_refine_subpel_ex) runs it when
 * subme >= 2 (:791-797).  fpelcmp = SAD (encoder.c:1421-1424 outside TESA).  fenc / planes /
 * fw at pixel (0,0) of one frame: planes = the reference's F, H, V, C (m->p_fref, for
 * COST_MV_HPEL with m->weight[0] and the refine), fw = p_fref_w (the weighted F plane; = F
 * unweighted).  pos[2*i] = the partition's top-left; par[12*i] = { mvp_x, mvp_y (qpel),
 * mv_limit_fpel min x, y, max x, y, mv_min_spel x, y, mv_max_spel x, y, i_mvc, 0 }; mvc[32*i
 * + 2*k] = candidate k (qpel, k < i_mvc <= 14).  ext / fenc_c / ref_c: as me_refine_subpel_ex
 * (weight[0] also weights COST_MV_HPEL's get_ref).  out[4*i] = { m->cost, m->mv[0], m->mv[1],
 * m->cost_mv } as x264_me_search_ref leaves them; nevals[2*i] (when given) = the integer
 * stage's fpelcmp calls on p_fref_w | its get_ref calls << 16, nevals[2*i+1] = the refine's
 * counts (me_refine_subpel_ex's format). */
#define SR_MVC_MAX 14
static inline uint32_t sr_pack( int a, int b ) { return (uint32_t)(uint16_t)a | ((uint32_t)(uint16_t)b << 16); }
static inline int sr_clip3( int v, int lo, int hi ) { return v < lo ? lo : v > hi ? hi : v; }
typedef struct
{
    const pixel *fenc, *fw;
    const pixel *q[4];
    intptr_t fs, rs;
    int i_pixel;
    const int *wt;
    int nf, nh;
} FN(sr_t);

static int FN(sr_fpel)( FN(sr_t) *c, int mx, int my )           /* fpelcmp on p_fref_w */
{
    c->nf++;
    return FN(sad)( c->i_pixel, c->fenc, c->fs, c->fw + my * c->rs + mx, c->rs );
}

static int FN(sr_hpel)( FN(sr_t) *c, int mx, int my )           /* COST_MV_HPEL's get_ref + fpelcmp */
{
    pixel tmp[16 * 16];
    intptr_t ts = 16;
    const pixel *r = get_ref_w( tmp, &ts, c->q, c->rs, mx, my, pixel_w[c->i_pixel], pixel_h[c->i_pixel], c->wt );
    c->nh++;
    return FN(sad)( c->i_pixel, c->fenc, c->fs, r, ts );
}

void FN(me_search_ref_thresh)( const pixel *fenc, intptr_t fs, const pixel *const planes[4], const pixel *fw,
                               intptr_t rs, int i_pixel, int me_method, int subme, int me_range, const int32_t *pos,
                               const int16_t *par, const int16_t *mvc_all, const uint16_t *cost_mv, int n,
                               int32_t *out, int32_t *nevals, const int32_t *ext, const pixel *const fenc_c[2],
                               intptr_t fcs, const pixel *const ref_c[8], intptr_t rcs, int32_t *thr,
                               const int32_t *rcost )
{
    static const uint8_t mod6m1[8] = { 5,0,1,2,3,4,5,0 };                                                /* me.c:53 */
    static const int8_t hex2[8][2] = { {-1,-2}, {-2,0}, {-1,2}, {1,2}, {2,0}, {1,-2}, {-1,-2}, {-2,0} }; /* me.c:55 */
    static const int8_t square1[9][2] = { {0,0}, {0,-1}, {0,1}, {-1,0}, {1,0}, {-1,-1}, {-1,1}, {1,-1}, {1,1} };
    static const int8_t hex4[16][2] = { { 0,-4}, { 0, 4}, {-2,-3}, { 2,-3}, {-4,-2}, { 4,-2}, {-4,-1}, { 4,-1},
                                        {-4, 0}, { 4, 0}, {-4, 1}, { 4, 1}, {-4, 2}, { 4, 2}, {-2, 3}, { 2, 3} };
    static const uint8_t pixel_size_shift[7] = { 0, 1, 1, 2, 3, 3, 4 };
    static const uint8_t range_mul[4][4] = { { 3, 3, 4, 4 }, { 3, 4, 4, 4 }, { 4, 4, 4, 5 }, { 4, 4, 5, 6 } };
    int wbuf[3];
    const int *wt0 = NULL;
    if( ext && ext[3] )
    {
        wbuf[0] = ext[4]; wbuf[1] = ext[5]; wbuf[2] = ext[6];
        wt0 = wbuf;
    }
    for( int j = 0; j < n; j++ )
    {
        const int bx = pos[2*j], by = pos[2*j+1];
        const int16_t *p = par + 12 * j;
        FN(sr_t) c = { fenc + by * fs + bx, fw + by * rs + bx, { NULL }, fs, rs, i_pixel, wt0, 0, 0 };
        for( int k = 0; k < 4; k++ )
            c.q[k] = planes[k] + by * rs + bx;
        const int mvp[2] = { p[0], p[1] };
        const int mv_x_min = p[2], mv_y_min = p[3], mv_x_max = p[4], mv_y_max = p[5];
        const int i_mvc = p[10];
        int16_t (*mvc)[2] = (int16_t (*)[2])(mvc_all + 2 * SR_MVC_MAX * j);
        const uint16_t *p_cost_mvx = cost_mv - mvp[0], *p_cost_mvy = cost_mv - mvp[1];
        int i_me_range = me_range;
        int bmx, bmy, bcost = 1 << 28, bpred_cost = 1 << 28;
        int omx, omy, pmx, pmy;
        uint32_t pmv, bpred_mv = 0;
        int16_t tmp[16][2];
        int costs[16];
#define SR_BITS( mx, my ) (p_cost_mvx[(mx) * 4] + p_cost_mvy[(my) * 4])
#define SR_COST_MV( mx, my ) do { int c_ = FN(sr_fpel)( &c, mx, my ) + SR_BITS( mx, my ); \
                                  if( c_ < bcost ) { bcost = c_; bmx = (mx); bmy = (my); } } while( 0 )
#define SR_IN( mx, my ) ( (mx) >= mv_x_min && (mx) <= mv_x_max && (my) >= mv_y_min && (my) <= mv_y_max )
        if( subme >= 3 )
        {
            int bpx = sr_clip3( mvp[0], 4 * mv_x_min, 4 * mv_x_max );
            int bpy = sr_clip3( mvp[1], 4 * mv_y_min, 4 * mv_y_max );
            pmv = sr_pack( bpx, bpy );
            pmx = (bpx + 2) >> 2;
            pmy = (bpy + 2) >> 2;
            bpred_cost = FN(sr_hpel)( &c, bpx, bpy ) + p_cost_mvx[bpx] + p_cost_mvy[bpy];
            const int pmv_cost = bpred_cost;
            if( i_mvc > 0 )
            {
                int valid = 0;
                for( int i = 0; i < i_mvc; i++ )
                {
                    uint32_t v = sr_pack( mvc[i][0], mvc[i][1] );
                    if( !v || v == pmv )
                        continue;
                    tmp[2 + valid][0] = sr_clip3( mvc[i][0], 4 * mv_x_min, 4 * mv_x_max );
                    tmp[2 + valid][1] = sr_clip3( mvc[i][1], 4 * mv_y_min, 4 * mv_y_max );
                    valid++;
                }
                if( valid > 0 )
                {
                    tmp[1][0] = bpx; tmp[1][1] = bpy;
                    bpred_cost <<= 4;
                    for( int i = 1; i <= valid; i++ )
                    {
                        int mx = tmp[i + 1][0], my = tmp[i + 1][1];
                        int cc = FN(sr_hpel)( &c, mx, my ) + p_cost_mvx[mx] + p_cost_mvy[my];
                        if( (cc << 4) + i < bpred_cost )
                            bpred_cost = (cc << 4) + i;
                    }
                    bpx = tmp[(bpred_cost & 15) + 1][0];
                    bpy = tmp[(bpred_cost & 15) + 1][1];
                    bpred_cost >>= 4;
                }
            }
            bmx = (bpx + 2) >> 2;
            bmy = (bpy + 2) >> 2;
            bpred_mv = sr_pack( bpx, bpy );
            if( bpred_mv & 0x00030003 )
                SR_COST_MV( bmx, bmy );
            else
                bcost = bpred_cost;
            if( pmv )
            {
                if( bmx | bmy )
                    SR_COST_MV( 0, 0 );
            }
            else if( pmv_cost < bcost )
            {
                bcost = pmv_cost;
                bmx = bmy = 0;
            }
        }
        else
        {
            bmx = pmx = sr_clip3( (mvp[0] + 2) >> 2, mv_x_min, mv_x_max );
            bmy = pmy = sr_clip3( (mvp[1] + 2) >> 2, mv_y_min, mv_y_max );
            pmv = sr_pack( bmx, bmy );
            bcost = FN(sr_fpel)( &c, bmx, bmy );
            if( i_mvc > 0 )
            {
                int valid = 0;
                for( int i = 0; i < i_mvc; i++ )
                {
                    int mx = (mvc[i][0] + 2) >> 2, my = (mvc[i][1] + 2) >> 2;
                    uint32_t v = sr_pack( mx, my );
                    if( !v || v == pmv )
                        continue;
                    tmp[2 + valid][0] = sr_clip3( mx, mv_x_min, mv_x_max );
                    tmp[2 + valid][1] = sr_clip3( my, mv_y_min, mv_y_max );
                    valid++;
                }
                if( valid > 0 )
                {
                    tmp[1][0] = bmx; tmp[1][1] = bmy;
                    bcost <<= 4;
                    for( int i = 1; i <= valid; i++ )
                    {
                        int mx = tmp[i + 1][0], my = tmp[i + 1][1];
                        int cc = FN(sr_fpel)( &c, mx, my ) + SR_BITS( mx, my );
                        if( (cc << 4) + i < bcost )
                            bcost = (cc << 4) + i;
                    }
                    bmx = tmp[(bcost & 15) + 1][0];
                    bmy = tmp[(bcost & 15) + 1][1];
                    bcost >>= 4;
                }
            }
            if( pmv )
                SR_COST_MV( 0, 0 );
        }

        int hex = me_method == 1;
        if( me_method == 0 )
        {
            bcost <<= 4;
            int i = i_me_range;
            do
            {
                costs[0] = FN(sr_fpel)( &c, bmx, bmy - 1 ) + SR_BITS( bmx, bmy - 1 );
                costs[1] = FN(sr_fpel)( &c, bmx, bmy + 1 ) + SR_BITS( bmx, bmy + 1 );
                costs[2] = FN(sr_fpel)( &c, bmx - 1, bmy ) + SR_BITS( bmx - 1, bmy );
                costs[3] = FN(sr_fpel)( &c, bmx + 1, bmy ) + SR_BITS( bmx + 1, bmy );
                if( (costs[0] << 4) + 1 < bcost ) bcost = (costs[0] << 4) + 1;
                if( (costs[1] << 4) + 3 < bcost ) bcost = (costs[1] << 4) + 3;
                if( (costs[2] << 4) + 4 < bcost ) bcost = (costs[2] << 4) + 4;
                if( (costs[3] << 4) + 12 < bcost ) bcost = (costs[3] << 4) + 12;
                if( !(bcost & 15) )
                    break;
                bmx -= (int32_t)((uint32_t)bcost << 28) >> 30;
                bmy -= (int32_t)((uint32_t)bcost << 30) >> 30;
                bcost &= ~15;
            } while( --i && SR_IN( bmx, bmy ) );
            bcost >>= 4;
        }
        else if( me_method == 3 )
        {
            /* ESA (me.c:618-631): the exhaustive form the reference keeps under #if 0 (:627-631),
             * which its successive elimination (ads, :750-768) equals in bcost / bmx / bmy: ads
             * only drops candidates whose DC bound cannot beat bcost.  The width rounds up to a
             * multiple of 4 (columns past max_x scored). */
            const int min_x = bmx - i_me_range > mv_x_min ? bmx - i_me_range : mv_x_min;
            const int min_y = bmy - i_me_range > mv_y_min ? bmy - i_me_range : mv_y_min;
            const int max_x = bmx + i_me_range < mv_x_max ? bmx + i_me_range : mv_x_max;
            const int max_y = bmy + i_me_range < mv_y_max ? bmy + i_me_range : mv_y_max;
            const int width = (max_x - min_x + 3) & ~3;
            for( int my = min_y; my <= max_y; my++ )
                for( int mx = min_x; mx < min_x + width; mx++ )
                    SR_COST_MV( mx, my );
        }
        else if( me_method == 2 )
        {
            /* UMH (me.c:422-616) */
#define SR_DIA1( cx, cy ) do { omx = (cx); omy = (cy); SR_COST_MV( omx, omy - 1 ); SR_COST_MV( omx, omy + 1 ); \
                               SR_COST_MV( omx - 1, omy ); SR_COST_MV( omx + 1, omy ); } while( 0 )
#define SR_CROSS( start, x_max, y_max ) do { \
            for( int i_ = (start); i_ < (x_max); i_ += 2 ) { \
                if( omx + i_ <= mv_x_max ) SR_COST_MV( omx + i_, omy ); \
                if( omx - i_ >= mv_x_min ) SR_COST_MV( omx - i_, omy ); } \
            for( int i_ = (start); i_ < (y_max); i_ += 2 ) { \
                if( omy + i_ <= mv_y_max ) SR_COST_MV( omx, omy + i_ ); \
                if( omy - i_ >= mv_y_min ) SR_COST_MV( omx, omy - i_ ); } } while( 0 )
#define SR_THRESH( v ) ( bcost < ((v) >> pixel_size_shift[i_pixel]) )
            int cross_start = 1;
            const int ucost1 = bcost;
            SR_DIA1( pmx, pmy );
            if( pmx | pmy )
                SR_DIA1( 0, 0 );
            if( i_pixel == 6 )                 /* PIXEL_4x4: goto me_hex2 (me.c:438-439) */
                hex = 1;
            else
            {
            const int ucost2 = bcost;
            if( (bmx | bmy) && ((bmx - pmx) | (bmy - pmy)) )
                SR_DIA1( bmx, bmy );
            if( bcost == ucost2 )
                cross_start = 3;
            omx = bmx; omy = bmy;
            int done = 0;
            if( bcost == ucost2 && SR_THRESH( 2000 ) )
            {
                static const int8_t oct[8][2] = { {0,-2}, {-1,-1}, {1,-1}, {-2,0}, {2,0}, {-1,1}, {1,1}, {0,2} };
                for( int k = 0; k < 8; k++ )
                    SR_COST_MV( omx + oct[k][0], omy + oct[k][1] );
                if( bcost == ucost1 && SR_THRESH( 500 ) )
                    done = 1;
                else if( bcost == ucost2 )
                {
                    int range = (i_me_range >> 1) | 1;
                    SR_CROSS( 3, range, range );
                    static const int8_t oct2[8][2] = { {-1,-2}, {1,-2}, {-2,-1}, {2,-1}, {-2,1}, {2,1}, {-1,2}, {1,2} };
                    for( int k = 0; k < 8; k++ )
                        SR_COST_MV( omx + oct2[k][0], omy + oct2[k][1] );
                    if( bcost == ucost2 )
                        done = 1;
                    cross_start = range + 2;
                }
            }
            if( !done )
            {
                if( i_mvc )
                {
                    int mvd, denom = 1;
                    if( i_mvc == 1 )
                        mvd = i_pixel == 0 ? 25 : abs( mvp[0] - mvc[0][0] ) + abs( mvp[1] - mvc[0][1] );
                    else
                    {
                        denom = i_mvc - 1;
                        mvd = 0;
                        if( i_pixel != 0 )
                        {
                            mvd = abs( mvp[0] - mvc[0][0] ) + abs( mvp[1] - mvc[0][1] );
                            denom++;
                        }
                        for( int i = 0; i < i_mvc - 1; i++ )
                            mvd += abs( mvc[i][0] - mvc[i + 1][0] ) + abs( mvc[i][1] - mvc[i + 1][1] );
                    }
                    const int sad_ctx = SR_THRESH( 1000 ) ? 0 : SR_THRESH( 2000 ) ? 1 : SR_THRESH( 4000 ) ? 2 : 3;
                    const int mvd_ctx = mvd < 10 * denom ? 0 : mvd < 20 * denom ? 1 : mvd < 40 * denom ? 2 : 3;
                    i_me_range = i_me_range * range_mul[mvd_ctx][sad_ctx] >> 2;
                }
                SR_CROSS( cross_start, i_me_range, i_me_range >> 1 );
                SR_COST_MV( omx - 2, omy - 2 );
                SR_COST_MV( omx - 2, omy + 2 );
                SR_COST_MV( omx + 2, omy - 2 );
                SR_COST_MV( omx + 2, omy + 2 );
                omx = bmx; omy = bmy;
                int i = 1;
                do
                {
                    for( int k = 0; k < 16; k++ )
                    {
                        const int mx = omx + hex4[k][0] * i, my = omy + hex4[k][1] * i;
                        if( SR_IN( mx, my ) )
                            SR_COST_MV( mx, my );
                    }
                } while( ++i <= i_me_range >> 2 );
                if( SR_IN( bmx, bmy ) )
                    hex = 1;
            }
            }
#undef SR_DIA1
#undef SR_CROSS
#undef SR_THRESH
        }
        if( hex )
        {
            /* hexagon (me.c:344-403), then the square refine (:404-418) */
#define SR_X3( a, b, cc, d, e, f, o ) do { \
            (o)[0] = FN(sr_fpel)( &c, bmx + (a), bmy + (b) ) + SR_BITS( bmx + (a), bmy + (b) ); \
            (o)[1] = FN(sr_fpel)( &c, bmx + (cc), bmy + (d) ) + SR_BITS( bmx + (cc), bmy + (d) ); \
            (o)[2] = FN(sr_fpel)( &c, bmx + (e), bmy + (f) ) + SR_BITS( bmx + (e), bmy + (f) ); } while( 0 )
            SR_X3( -2, 0, -1, 2, 1, 2, costs );
            SR_X3( 2, 0, 1, -2, -1, -2, costs + 4 );
            bcost <<= 3;
            if( (costs[0] << 3) + 2 < bcost ) bcost = (costs[0] << 3) + 2;
            if( (costs[1] << 3) + 3 < bcost ) bcost = (costs[1] << 3) + 3;
            if( (costs[2] << 3) + 4 < bcost ) bcost = (costs[2] << 3) + 4;
            if( (costs[4] << 3) + 5 < bcost ) bcost = (costs[4] << 3) + 5;
            if( (costs[5] << 3) + 6 < bcost ) bcost = (costs[5] << 3) + 6;
            if( (costs[6] << 3) + 7 < bcost ) bcost = (costs[6] << 3) + 7;
            if( bcost & 7 )
            {
                int dir = (bcost & 7) - 2;
                bmx += hex2[dir + 1][0];
                bmy += hex2[dir + 1][1];
                for( int i = (i_me_range >> 1) - 1; i > 0 && SR_IN( bmx, bmy ); i-- )
                {
                    SR_X3( hex2[dir][0], hex2[dir][1], hex2[dir + 1][0], hex2[dir + 1][1], hex2[dir + 2][0],
                           hex2[dir + 2][1], costs );
                    bcost &= ~7;
                    if( (costs[0] << 3) + 1 < bcost ) bcost = (costs[0] << 3) + 1;
                    if( (costs[1] << 3) + 2 < bcost ) bcost = (costs[1] << 3) + 2;
                    if( (costs[2] << 3) + 3 < bcost ) bcost = (costs[2] << 3) + 3;
                    if( !(bcost & 7) )
                        break;
                    dir += (bcost & 7) - 2;
                    dir = mod6m1[dir + 1];
                    bmx += hex2[dir + 1][0];
                    bmy += hex2[dir + 1][1];
                }
            }
            bcost >>= 3;
#undef SR_X3
            bcost <<= 4;
            for( int k = 0; k < 8; k++ )
            {
                const int cc = FN(sr_fpel)( &c, bmx + square1[k + 1][0], bmy + square1[k + 1][1] )
                             + SR_BITS( bmx + square1[k + 1][0], bmy + square1[k + 1][1] );
                if( (cc << 4) + k + 1 < bcost )
                    bcost = (cc << 4) + k + 1;
            }
            bmx += square1[bcost & 15][0];
            bmy += square1[bcost & 15][1];
            bcost >>= 4;
        }
#undef SR_COST_MV
#undef SR_IN
        /* -> qpel mv (me.c:774-789) */
        int mx, my, cst, cmv;
        if( subme < 3 )
        {
            cmv = SR_BITS( bmx, bmy );
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
            cst = bpred_cost < bcost ? bpred_cost : bcost;
            cmv = p_cost_mvx[mx] + p_cost_mvy[my];    /* (refine_subpel sets m->cost_mv) */
        }
#undef SR_BITS
        if( nevals )
        {
            nevals[2*j] = c.nf | (c.nh << 16);
            nevals[2*j+1] = 0;
        }
        if( subme >= 2 )
        {
            const int16_t rp[8] = { (int16_t)mx, (int16_t)my, (int16_t)mvp[0], (int16_t)mvp[1], p[6], p[7], p[8], p[9] };
            const int32_t rpos[2] = { bx, by };
            FN(refine_core)( fenc, fs, planes, rs, i_pixel, subme, 0, 0, rpos, rp, &cst, cost_mv, 1, out + 4 * j,
                             nevals ? nevals + 2 * j + 1 : NULL, ext, fenc_c, fcs, ref_c, rcs, thr ? thr + j : NULL,
                             rcost ? rcost + j : NULL );
        }
        else
        {
            out[4*j] = cst;
            out[4*j+1] = mx;
            out[4*j+2] = my;
            out[4*j+3] = cmv;
        }
    }
}

void FN(me_search_ref)( const pixel *fenc, intptr_t fs, const pixel *const planes[4], const pixel *fw, intptr_t rs,
                        int i_pixel, int me_method, int subme, int me_range, const int32_t *pos, const int16_t *par,
                        const int16_t *mvc_all, const uint16_t *cost_mv, int n, int32_t *out, int32_t *nevals,
                        const int32_t *ext, const pixel *const fenc_c[2], intptr_t fcs, const pixel *const ref_c[8],
                        intptr_t rcs )
{
    FN(me_search_ref_thresh)( fenc, fs, planes, fw, rs, i_pixel, me_method, subme, me_range, pos, par, mvc_all, cost_mv,
                              n, out, nevals, ext, fenc_c, fcs, ref_c, rcs, NULL, NULL );
}

/* x264_me_refine_bidir_satd (reference encoder/me.c:994-1183 with rd = 0) for a list of bipred
 * partitions of one frame: up to 8 passes over the 33 (mv0, mv1) pairs of dia4d around the
 * current pair, skipping pairs whose visited bit (m0x&7, m0y&7, m1x&7, m1y&7) an earlier pass
 * set, each scored as mc.avg[i_pixel] of the two lists' get_ref blocks (unweighted references,
 * x264_weight_none; i_weight 32: the rounding average, else pixel_avg_weight_wxh, mc.c:49-99)
 * by mbcmp (satd when `satd`, else sad) plus the four mv costs; COPY2_IF_LT in j order, then a
 * move by dia4d[bestj] or the end.  The early return when either mv lies within 8 qpel of
 * mv_min_spel / mv_max_spel (:1077-1081).  planes0 / planes1: list 0 / 1 reference F, H, V, C at
 * pixel (0,0); pos[2*i] = the partition's top-left; par[12*i] = { m0 mv x, y, m1 mv x, y, m0 mvp
 * x, y, m1 mvp x, y, mv_min_spel x, y, mv_max_spel x, y }; weight[i] = i_weight.  out[4*i] =
 * { m0 mv x, y, m1 mv x, y }; cost[i] (or NULL) = the final bcost (COST_MAX after the early
 * return; the reference keeps it internal); nevals[i] (or NULL) = mbcmp calls | passes << 16. */
void FN(me_refine_bidir)( const pixel *fenc, intptr_t fs, const pixel *const planes0[4],
                          const pixel *const planes1[4], intptr_t rs, int i_pixel, int satd, const int32_t *pos,
                          const int16_t *par, const int32_t *weight, const uint16_t *cost_mv, int n, int32_t *out,
                          int32_t *cost, int32_t *nevals )
{
    static const int8_t dia4d[33][4] = {                                                        /* me.c:1064-1075 */
        {0,0,0,0},
        {0,0,0,1}, {0,0,0,-1}, {0,0,1,0}, {0,0,-1,0},
        {0,1,0,0}, {0,-1,0,0}, {1,0,0,0}, {-1,0,0,0},
        {0,0,1,1}, {0,0,-1,-1},{0,1,1,0}, {0,-1,-1,0},
        {1,1,0,0}, {-1,-1,0,0},{1,0,0,1}, {-1,0,0,-1},
        {0,1,0,1}, {0,-1,0,-1},{1,0,1,0}, {-1,0,-1,0},
        {0,0,-1,1},{0,0,1,-1}, {0,-1,1,0},{0,1,-1,0},
        {-1,1,0,0},{1,-1,0,0}, {1,0,0,-1},{-1,0,0,1},
        {0,-1,0,1},{0,1,0,-1}, {-1,0,1,0},{1,0,-1,0},
    };
    const int bw = pixel_w[i_pixel], bh = pixel_h[i_pixel];
    for( int i = 0; i < n; i++ )
    {
        const int bx = pos[2*i], by = pos[2*i+1];
        const int16_t *p = par + 12 * i;
        const pixel *f = fenc + by * fs + bx;
        const pixel *q0[4], *q1[4];
        for( int k = 0; k < 4; k++ )
        {
            q0[k] = planes0[k] + by * rs + bx;
            q1[k] = planes1[k] + by * rs + bx;
        }
        int bm0x = p[0], bm0y = p[1], bm1x = p[2], bm1y = p[3];
        const uint16_t *c0x = cost_mv - p[4], *c0y = cost_mv - p[5], *c1x = cost_mv - p[6], *c1y = cost_mv - p[7];
        const int minx = p[8], miny = p[9], maxx = p[10], maxy = p[11];
        const int w1 = weight[i], w2 = 64 - w1;
        int bcost = 1 << 28, ncalls = 0, npass = 0;
        uint8_t visited[8][8][8];
        if( !(bm0y < miny + 8 || bm1y < miny + 8 || bm0y > maxy - 8 || bm1y > maxy - 8 ||
              bm0x < minx + 8 || bm1x < minx + 8 || bm0x > maxx - 8 || bm1x > maxx - 8) )
        {
            memset( visited, 0, sizeof(visited) );
            for( int pass = 0; pass < 8; pass++ )
            {
                int bestj = 0;
                npass++;
                for( int j = !!pass; j < 33; j++ )
                {
                    const int m0x = dia4d[j][0] + bm0x, m0y = dia4d[j][1] + bm0y;
                    const int m1x = dia4d[j][2] + bm1x, m1y = dia4d[j][3] + bm1y;
                    if( pass && (visited[m0x & 7][m0y & 7][m1x & 7] & (1 << (m1y & 7))) )
                        continue;
                    visited[m0x & 7][m0y & 7][m1x & 7] |= 1 << (m1y & 7);
                    pixel b0[16 * 16], b1[16 * 16], avg[16 * 16];
                    intptr_t s0 = 16, s1 = 16;
                    const pixel *r0 = FN(get_ref)( b0, &s0, q0, rs, m0x, m0y, bw, bh );
                    const pixel *r1 = FN(get_ref)( b1, &s1, q1, rs, m1x, m1y, bw, bh );
                    for( int y = 0; y < bh; y++ )
                        for( int x = 0; x < bw; x++ )
                            avg[16 * y + x] = w1 == 32 ? (r0[y * s0 + x] + r1[y * s1 + x] + 1) >> 1
                                                       : clip_pixel( (r0[y * s0 + x] * w1 + r1[y * s1 + x] * w2 + 32) >> 6 );
                    const int c = (satd ? FN(satd)( i_pixel, f, fs, avg, 16 ) : FN(sad)( i_pixel, f, fs, avg, 16 ))
                                + c0x[m0x] + c0y[m0y] + c1x[m1x] + c1y[m1y];
                    ncalls++;
                    if( c < bcost )
                    {
                        bcost = c;
                        bestj = j;
                    }
                }
                if( !bestj )
                    break;
                bm0x += dia4d[bestj][0];
                bm0y += dia4d[bestj][1];
                bm1x += dia4d[bestj][2];
                bm1y += dia4d[bestj][3];
            }
        }
        out[4*i] = bm0x;
        out[4*i+1] = bm0y;
        out[4*i+2] = bm1x;
        out[4*i+3] = bm1y;
        if( cost )
            cost[i] = bcost;
        if( nevals )
            nevals[i] = ncalls | (npass << 16);
    }
}

/* TESA integer-pel search of x264_me_search_ref for PIXEL_16x16, restated from
 * reference encoder/me.c:618-748 (X264_ME_TESA): enc_dc from sad_x4 against
 * x264_zero (:643-645), per row the ycost skip, ads4 with threshold bsad*17>>4
 * (:661-669, ads4 = pixel.c:759-803), the SAD threshold list with the running
 * COPY1_IF_LT (:670-701; sad_x3 scores equal three sad calls), the halving prune
 * (:705-734), the drop-the-first-maximum loop (:735-746) and COST_MV over the
 * survivors (:747-748, me.c:63-70) with fpelcmp = satd when `satd` (mbcmp_init,
 * encoder.c:1411,1423-1424) else sad.  fenc / ref / integral point at pixel (0,0)
 * of one frame; the integral image (x264_frame_filter, mc.c:748-782) shares the
 * ref stride rs (frame.c:273).  par / init_cost / cost_mv as me_esa_argmin.
 * out[4*i] = { bcost, bmx, bmy, number of COST_MV evaluations }. */
void FN(me_tesa)( const pixel *fenc, intptr_t fs, const pixel *ref, const uint16_t *integral, intptr_t rs,
                  int mb_width, int mb_height, int me_range, int satd, const int16_t *par,
                  const int32_t *init_cost, const uint16_t *cost_mv, int32_t *out )
{
    static const pixel zero[16 * 16];
    const int nmb = mb_width * mb_height;
    int16_t *xs = malloc( (4 * me_range + 8) * sizeof(int16_t) );
    uint16_t *fpel = malloc( (4 * me_range + 8) * sizeof(uint16_t) );
    struct { int sad; int16_t mv[2]; } *mvsads = malloc( (size_t)(2 * me_range + 1) * (4 * me_range + 8) * 8 );
    for( int i = 0; i < nmb; i++ )
    {
        const int mbx = i % mb_width, mby = i / mb_width;
        const int16_t *p = par + 8 * i;
        const pixel *p_fenc = fenc + 16 * (mby * fs + mbx);
        const pixel *p_fref_w = ref + 16 * (mby * rs + mbx);
        const uint16_t *sums_base = integral + 16 * (mby * rs + mbx);
        const uint16_t *p_cost_mvx = cost_mv - p[2], *p_cost_mvy = cost_mv - p[3];
        int bmx = p[0], bmy = p[1], bcost = init_cost[i], ncost = 0;
        const int min_x = bmx - me_range > p[4] ? bmx - me_range : p[4];
        const int min_y = bmy - me_range > p[5] ? bmy - me_range : p[5];
        const int max_x = bmx + me_range < p[6] ? bmx + me_range : p[6];
        const int max_y = bmy + me_range < p[7] ? bmy + me_range : p[7];
        const int width = (max_x - min_x + 3) & ~3;
        const int delta = 8 * rs;
        int enc_dc[4];
        for( int k = 0; k < 4; k++ )
            enc_dc[k] = FN(sad)( 3 /* PIXEL_8x8 */, zero, 16, p_fenc + 8 * (k & 1) + 8 * (k >> 1) * fs, fs );
        /* cost_fpel_mvx + min_x: cost_mv_fpel[qp][-mvp&3][(-mvp>>2) + x] = cost_mv[qp][4x - mvp]
         * (analyse.c:161-169) */
        for( int x = 0; x < width; x++ )
            fpel[x] = p_cost_mvx[(min_x + x) * 4];
        int nmvsad = 0, limit;
        int sad_thresh = me_range <= 16 ? 10 : me_range <= 24 ? 11 : 12;
        int bsad = FN(sad)( 0 /* PIXEL_16x16 */, p_fenc, fs, p_fref_w + bmy * rs + bmx, rs )
                 + p_cost_mvx[bmx * 4] + p_cost_mvy[bmy * 4];
        for( int my = min_y; my <= max_y; my++ )
        {
            int ycost = p_cost_mvy[my * 4];
            if( bsad <= ycost )
                continue;
            bsad -= ycost;
            int xn = FN(ads)( 4, enc_dc, sums_base + min_x + my * rs, delta, fpel, xs, width, bsad * 17 >> 4 );
            for( int k = 0; k < xn; k++ )
            {
                int mx = min_x + xs[k];
                int sad = FN(sad)( 0 /* PIXEL_16x16 */, p_fenc, fs, p_fref_w + mx + my * rs, rs ) + fpel[xs[k]];
                if( sad < bsad * sad_thresh >> 3 )
                {
                    if( sad < bsad )
                        bsad = sad;
                    mvsads[nmvsad].sad = sad + ycost;
                    mvsads[nmvsad].mv[0] = mx;
                    mvsads[nmvsad].mv[1] = my;
                    nmvsad++;
                }
            }
            bsad += ycost;
        }
        limit = me_range >> 1;
        sad_thresh = bsad * sad_thresh >> 3;
        while( nmvsad > limit * 2 && sad_thresh > bsad )
        {
            sad_thresh = (sad_thresh + bsad) >> 1;
            int k = 0;
            for( int j = 0; j < nmvsad; j++ )
                if( mvsads[j].sad <= sad_thresh )
                    mvsads[k++] = mvsads[j];
            nmvsad = k;
        }
        while( nmvsad > limit )
        {
            int bi = 0;
            for( int k = 1; k < nmvsad; k++ )
                if( mvsads[k].sad > mvsads[bi].sad )
                    bi = k;
            nmvsad--;
            mvsads[bi] = mvsads[nmvsad];
        }
        for( int k = 0; k < nmvsad; k++ )
        {
            int mx = mvsads[k].mv[0], my = mvsads[k].mv[1];
            const pixel *r = p_fref_w + my * rs + mx;
            int cost = (satd ? FN(satd)( 0 /* PIXEL_16x16 */, p_fenc, fs, r, rs ) : FN(sad)( 0 /* PIXEL_16x16 */, p_fenc, fs, r, rs ))
                     + p_cost_mvx[mx * 4] + p_cost_mvy[my * 4];
            ncost++;
            if( cost < bcost )
            {
                bcost = cost;
                bmx = mx;
                bmy = my;
            }
        }
        out[4 * i] = bcost;
        out[4 * i + 1] = bmx;
        out[4 * i + 2] = bmy;
        out[4 * i + 3] = ncost;
    }
    free( mvsads );
    free( fpel );
    free( xs );
}

/*============================================================================
 * lookahead input — reference common/mc.c:458-507, common/frame.c:535-631
 *==========================================================================*/

/* x264_frame_init_lowres on a private copy of the luma plane: duplicate the
 * last column / row (mc.c:465-468), frame_init_lowres_core (mc.c:484-507) into
 * the four half-resolution planes, then plane_expand_border with PADH = PADV =
 * 32 (frame.c:627-631).  src / dst point at (0,0); src has >= 1 pixel of
 * writable padding right and below (the copy is taken from rows [0, height]
 * and columns [0, width]). */
void FN(frame_init_lowres)( const pixel *src_in, intptr_t stride, int width, int height,
                            pixel *dst[4], intptr_t dst_stride )
{
    const int pad = 32, wl = width / 2, hl = height / 2;
    pixel *src = malloc( (size_t)(height + 1) * stride * sizeof(pixel) );
    for( int y = 0; y < height; y++ )
        memcpy( src + y*stride, src_in + y*stride, (width + 1) * sizeof(pixel) );
    for( int y = 0; y < height; y++ )
        src[width + y*stride] = src[width - 1 + y*stride];
    memcpy( src + stride*height, src + stride*(height - 1), (width + 1) * sizeof(pixel) );
#define FILTER(a,b,c,d) ((((a+b+1)>>1)+((c+d+1)>>1)+1)>>1)
    for( int y = 0; y < hl; y++ )
    {
        const pixel *s0 = src + 2*y*stride, *s1 = s0 + stride, *s2 = s1 + stride;
        pixel *d0 = dst[0] + y*dst_stride, *dh = dst[1] + y*dst_stride;
        pixel *dv = dst[2] + y*dst_stride, *dc = dst[3] + y*dst_stride;
        for( int x = 0; x < wl; x++ )
        {
            d0[x] = FILTER( s0[2*x], s1[2*x], s0[2*x+1], s1[2*x+1] );
            dh[x] = FILTER( s0[2*x+1], s1[2*x+1], s0[2*x+2], s1[2*x+2] );
            dv[x] = FILTER( s1[2*x], s2[2*x], s1[2*x+1], s2[2*x+1] );
            dc[x] = FILTER( s1[2*x+1], s2[2*x+1], s1[2*x+2], s2[2*x+2] );
        }
    }
#undef FILTER
    free( src );
    for( int i = 0; i < 4; i++ )
    {
        pixel *pix = dst[i];
        for( int y = 0; y < hl; y++ )
            for( int k = 0; k < pad; k++ )
            {
                pix[y*dst_stride - pad + k] = pix[y*dst_stride];
                pix[y*dst_stride + wl + k] = pix[y*dst_stride + wl - 1];
            }
        for( int y = 0; y < pad; y++ )
        {
            memcpy( pix + (-y-1)*dst_stride - pad, pix - pad, (wl + 2*pad) * sizeof(pixel) );
            memcpy( pix + (hl + y)*dst_stride - pad, pix + (hl - 1)*dst_stride - pad, (wl + 2*pad) * sizeof(pixel) );
        }
    }
}

/*============================================================================
 * intra prediction and the pixel table's intra_*_x3 entries — reference
 * common/predict.c, common/pixel.c:518-560; the lookahead's intra estimate of
 * encoder/slicetype.c:714-757.  Predictors work on an FDEC-layout buffer (src
 * at the block's (0,0), neighbours at x = -1 / y = -1) like the reference.
 *==========================================================================*/
#define F1(a,b)   (((a)+(b)+1)>>1)
#define F2(a,b,c) (((a)+2*(b)+(c)+2)>>2)
#define PX(x,y) src[(x) + (y)*FDEC_STRIDE]

static void fill_rect( pixel *src, int x0, int y0, int w, int h, int v )
{
    for( int y = y0; y < y0 + h; y++ )
        for( int x = x0; x < x0 + w; x++ )
            PX(x,y) = v;
}

/* predict_4x4_{v,h,dc} (predict.c:495-511), predict_16x16_{dc,h,v} (:67-130):
 * a square block of n pixels */
static void pred_sq_v( pixel *src, int n )
{
    for( int y = 0; y < n; y++ )
        for( int x = 0; x < n; x++ )
            PX(x,y) = PX(x,-1);
}
static void pred_sq_h( pixel *src, int n )
{
    for( int y = 0; y < n; y++ )
        fill_rect( src, 0, y, n, 1, PX(-1,y) );
}
static void pred_sq_dc( pixel *src, int n )
{
    int s = 0;
    for( int i = 0; i < n; i++ )
        s += PX(-1,i) + PX(i,-1);
    fill_rect( src, 0, 0, n, n, (s + n) >> (n == 4 ? 3 : 5) );
}

/* predict_8x8c_dc (predict.c:221-258) and predict_8x16c_dc (:361-419):
 * h = 8 or 16 rows of 4x4 DC quadrants */
static void pred_chroma_dc( pixel *src, int h )
{
    int s0 = 0, s1 = 0, sl[4] = { 0 };
    for( int i = 0; i < 4; i++ )
    {
        s0 += PX(i,-1);
        s1 += PX(i+4,-1);
        for( int k = 0; k < h / 4; k++ )
            sl[k] += PX(-1,i + 4*k);
    }
    fill_rect( src, 0, 0, 4, 4, (s0 + sl[0] + 4) >> 3 );
    fill_rect( src, 4, 0, 4, 4, (s1 + 2) >> 2 );
    for( int k = 1; k < h / 4; k++ )
    {
        fill_rect( src, 0, 4*k, 4, 4, (sl[k] + 2) >> 2 );
        fill_rect( src, 4, 4*k, 4, 4, (s1 + sl[k] + 4) >> 3 );
    }
}
static void pred_chroma_h( pixel *src, int h ) { for( int y = 0; y < h; y++ ) fill_rect( src, 0, y, 8, 1, PX(-1,y) ); }
static void pred_chroma_v( pixel *src, int h )
{
    for( int y = 0; y < h; y++ )
        for( int x = 0; x < 8; x++ )
            PX(x,y) = PX(x,-1);
}
/* predict_8x8c_p, predict.c:282-308 */
static void pred_8x8c_p( pixel *src )
{
    int H = 0, V = 0;
    for( int i = 0; i < 4; i++ )
    {
        H += (i + 1) * (PX(4+i,-1) - PX(2-i,-1));
        V += (i + 1) * (PX(-1,4+i) - PX(-1,2-i));
    }
    const int a = 16 * (PX(-1,7) + PX(7,-1));
    const int b = (17*H + 16) >> 5, c = (17*V + 16) >> 5;
    for( int y = 0; y < 8; y++ )
        for( int x = 0; x < 8; x++ )
            PX(x,y) = clip_pixel( (a - 3*b - 3*c + 16 + b*x + c*y) >> 5 );
}

/* predict_8x8_filter (predict.c:632-676): edge[7..14] = l7..l0, edge[15] = lt,
 * edge[16..31] = t0..t15, edge[32] = t15, low-pass filtered.  MB_LEFT = 1,
 * MB_TOP = 2, MB_TOPRIGHT = 4, MB_TOPLEFT = 8 (reference common/macroblock.h). */
void FN(predict_8x8_filter)( const pixel *src, pixel edge[36], int i_neighbor, int i_filters )
{
    const int have_lt = i_neighbor & 8;
    if( i_filters & 1 )
    {
        edge[15] = F2( PX(0,-1), PX(-1,-1), PX(-1,0) );
        edge[14] = F2( have_lt ? PX(-1,-1) : PX(-1,0), PX(-1,0), PX(-1,1) );
        for( int y = 1; y < 7; y++ )
            edge[14-y] = F2( PX(-1,y-1), PX(-1,y), PX(-1,y+1) );
        edge[6] = edge[7] = (PX(-1,6) + 3*PX(-1,7) + 2) >> 2;
    }
    if( i_filters & 2 )
    {
        const int have_tr = i_neighbor & 4;
        edge[16] = F2( have_lt ? PX(-1,-1) : PX(0,-1), PX(0,-1), PX(1,-1) );
        for( int x = 1; x < 7; x++ )
            edge[16+x] = F2( PX(x-1,-1), PX(x,-1), PX(x+1,-1) );
        edge[23] = F2( PX(6,-1), PX(7,-1), have_tr ? PX(8,-1) : PX(7,-1) );
        if( i_filters & 4 )
        {
            if( have_tr )
            {
                for( int x = 8; x < 15; x++ )
                    edge[16+x] = F2( PX(x-1,-1), PX(x,-1), PX(x+1,-1) );
                edge[31] = edge[32] = (PX(14,-1) + 3*PX(15,-1) + 2) >> 2;
            }
            else
                for( int i = 24; i < 33; i++ )
                    edge[i] = PX(7,-1);
        }
    }
}

/* predict_8x8_{v,h,dc,ddl,ddr,vr,hd,vl,hu} (predict.c:716-883) in the
 * H.264 8.3.2.2 form: with l_y = edge[14-y], lt = edge[15], t_x = edge[16+x],
 * each mode is a function of zVR = 2x-y, zHD = 2y-x or x+y walking along
 * the edge array; tests/golden/intra8x8_golden.npz pins every mode against
 * the reference's own per-pixel assignment lists. */
static int pred8x8_px( int mode, const pixel *e, int x, int y )
{
    int z, c;
    switch( mode )
    {
        case 0: return e[16+x];                                           /* V   */
        case 1: return e[14-y];                                           /* H   */
        case 3: z = x + y;                                                /* DDL */
            return F2( e[16+z], e[17+z], e[16 + (z + 2 < 15 ? z + 2 : 15)] );
        case 4:                                                           /* DDR */
            c = x > y ? 15 + x - y : 15 - (y - x);
            return F2( e[c-1], e[c], e[c+1] );
        case 5: z = 2*x - y;                                              /* VR  */
            if( z < 0 ) { c = 16 + z; return F2( e[c-1], e[c], e[c+1] ); }
            if( !(z & 1) ) return F1( e[15 + z/2], e[16 + z/2] );
            c = 15 + (z + 1)/2; return F2( e[c-1], e[c], e[c+1] );
        case 6: z = 2*y - x;                                              /* HD  */
            if( z < 0 ) { c = 14 - z; return F2( e[c-1], e[c], e[c+1] ); }
            if( !(z & 1) ) return F1( e[15 - z/2], e[14 - z/2] );
            c = 15 - (z + 1)/2; return F2( e[c-1], e[c], e[c+1] );
        case 7: c = 16 + x + (y >> 1);                                    /* VL  */
            return (y & 1) ? F2( e[c], e[c+1], e[c+2] ) : F1( e[c], e[c+1] );
        case 8: z = x + 2*y;                                              /* HU  */
            if( z > 13 ) return e[7];
            if( z == 13 ) return F2( e[8], e[7], e[7] );
            c = 14 - (z >> 1);
            return (z & 1) ? F2( e[c], e[c-1], e[c-2] ) : F1( e[c], e[c-1] );
    }
    return 0;
}
void FN(predict_8x8)( int mode, pixel *src, const pixel edge[36] )
{
    if( mode == 2 )
    {
        int s = 8;
        for( int i = 0; i < 8; i++ )
            s += edge[14-i] + edge[16+i];
        fill_rect( src, 0, 0, 8, 8, s >> 4 );
        return;
    }
    for( int y = 0; y < 8; y++ )
        for( int x = 0; x < 8; x++ )
            PX(x,y) = pred8x8_px( mode, edge, x, y );
}

/* the non-8x8 predictors by (size kind, mode); kind X264HIP_INTRA_*:
 * 0 = 4x4, 1 = 8x8c, 2 = 8x16c, 3 = 16x16; modes in the reference's I_PRED_*
 * numbering (16x16 / 4x4: 0 V, 1 H, 2 DC; chroma: 0 DC, 1 H, 2 V, 3 P) */
void FN(predict)( int kind, int mode, pixel *src )
{
    const int n = kind == 0 ? 4 : 16;
    if( kind == 0 || kind == 3 )
    {
        if( mode == 0 ) pred_sq_v( src, n );
        else if( mode == 1 ) pred_sq_h( src, n );
        else pred_sq_dc( src, n );
        return;
    }
    const int h = kind == 1 ? 8 : 16;
    if( mode == 0 ) pred_chroma_dc( src, h );
    else if( mode == 1 ) pred_chroma_h( src, h );
    else if( mode == 2 ) pred_chroma_v( src, h );
    else pred_8x8c_p( src );
}

/* intra_{sad,satd}_x3_{4x4,8x8c,8x16c,16x16} and intra_{sad,sa8d}_x3_8x8
 * (pixel.c:518-560): res[k] = cmp( prediction k, fenc ) with the mode order
 * v,h,dc (4x4, 16x16, 8x8 from edge[]) or dc,h,v (chroma).  kind 4 = 8x8 luma:
 * fdec is then the 36-entry edge array.  The reference C writes its last
 * prediction into fdec; this restatement works on a private copy. */
void FN(intra_x3)( int kind, int op, const pixel *fenc, const pixel *fdec, int res[3] )
{
    static const uint8_t ipix[5] = { 6, 3, 2, 0, 3 };
    pixel buf[17 * FDEC_STRIDE];
    pixel *src = buf + FDEC_STRIDE + 8;
    const int bw = kind == 0 ? 4 : kind == 3 ? 16 : 8, bh = kind == 0 ? 4 : kind == 1 || kind == 4 ? 8 : 16;
    if( kind != 4 )
        for( int y = -1; y < bh; y++ )
            for( int x = -1; x < bw; x++ )
                PX(x,y) = fdec[x + y*FDEC_STRIDE];
    for( int k = 0; k < 3; k++ )
    {
        if( kind == 4 )
            FN(predict_8x8)( k, src, fdec );
        else
            FN(predict)( kind, k, src );
        const int i_pixel = ipix[kind];
        res[k] = op == 0 ? FN(sad)( i_pixel, src, FDEC_STRIDE, fenc, FENC_STRIDE )
               : op == 3 ? FN(sa8d)( i_pixel, src, FDEC_STRIDE, fenc, FENC_STRIDE )
               :           FN(satd)( i_pixel, src, FDEC_STRIDE, fenc, FENC_STRIDE );
    }
}

/* slicetype_mb_cost's intra leg (encoder/slicetype.c:714-757) for every 8x8
 * block of one lowres plane (plane at (0,0), 32 pixels of border).  satd = the
 * mbcmp choice of encoder.c:1411 (!lossless && subme > 1), all_modes =
 * subme > 1: DC/H/V chroma-style, then planar and the six directional 8x8
 * modes over the filtered edge.  Costs: ((min + 5*lambda) >> (BIT_DEPTH-8)) + 4
 * into intra_cost[mb]; row_satd[y] sums the AQ-scaled cost of row y (inv_qscale
 * NULL = AQ off) and est[0] / est[1] the plain / AQ costs of the frame-score
 * MBs (slicetype.c:532-534, 751-756), every MB computed (do_edges). */
void FN(lowres_intra_cost)( const pixel *plane, intptr_t stride, int mb_width, int mb_height, int satd,
                            int all_modes, int lambda, const uint16_t *inv_qscale, uint16_t *intra_cost,
                            int32_t *row_satd, int32_t est[2] )
{
    pixel fenc[8 * FENC_STRIDE], buf[9 * FDEC_STRIDE], edge[36];
    pixel *src = buf + FDEC_STRIDE + 8;
    est[0] = est[1] = 0;
    for( int mby = 0; mby < mb_height; mby++ )
    {
        row_satd[mby] = 0;
        for( int mbx = 0; mbx < mb_width; mbx++ )
        {
            const pixel *s = plane + 8*mbx + 8*mby*stride;
            for( int y = 0; y < 8; y++ )
                memcpy( fenc + y*FENC_STRIDE, s + y*stride, 8 * sizeof(pixel) );
            for( int x = 0; x < 16; x++ )
                PX(x,-1) = s[x - stride];
            for( int y = -1; y < 8; y++ )
                PX(-1,y) = s[y*stride - 1];
            int cost = 1 << 30;
            for( int k = 0; k < 3; k++ )
            {
                FN(predict)( 1, k, src );
                const int c = satd ? FN(satd)( 3, src, FDEC_STRIDE, fenc, FENC_STRIDE )
                                   : FN(sad)( 3, src, FDEC_STRIDE, fenc, FENC_STRIDE );
                cost = c < cost ? c : cost;
            }
            if( all_modes )
            {
                pred_8x8c_p( src );
                int c = satd ? FN(satd)( 3, fenc, FENC_STRIDE, src, FDEC_STRIDE )
                             : FN(sad)( 3, fenc, FENC_STRIDE, src, FDEC_STRIDE );
                cost = c < cost ? c : cost;
                FN(predict_8x8_filter)( src, edge, 15, 15 );
                for( int m = 3; m < 9; m++ )
                {
                    FN(predict_8x8)( m, src, edge );
                    c = satd ? FN(satd)( 3, fenc, FENC_STRIDE, src, FDEC_STRIDE )
                             : FN(sad)( 3, fenc, FENC_STRIDE, src, FDEC_STRIDE );
                    cost = c < cost ? c : cost;
                }
            }
            cost = ((cost + 5 * lambda) >> (BIT_DEPTH - 8)) + 4;
            const int mb = mbx + mby * mb_width;
            intra_cost[mb] = cost;
            const int aq = inv_qscale ? (cost * inv_qscale[mb] + 128) >> 8 : cost;
            row_satd[mby] += aq;
            if( (mbx > 0 && mbx < mb_width - 1 && mby > 0 && mby < mb_height - 1) || mb_width <= 2 || mb_height <= 2 )
            {
                est[0] += cost;
                est[1] += aq;
            }
        }
    }
}
#undef PX
#undef F1
#undef F2

/*============================================================================
 * the lookahead's lowres motion search: slicetype_mb_cost's inter leg for a
 * P frame (reference encoder/slicetype.c:514-713, 758-791 with b == p1, one
 * list, no weights, a fresh search) and the x264_me_search_ref /
 * refine_subpel paths the lookahead runs (encoder/me.c:182-420, 774-790,
 * 865-992 with me = DIA or HEX, subme = 2 or 4, no chroma, no thresholds).
 *==========================================================================*/
#define LR_COST_MAX (1 << 28)
static const uint8_t lr_subpel_iters[5][4] = { {0,0,0,0}, {1,1,0,0}, {0,1,1,0}, {0,2,1,0}, {0,2,1,1} };  /* me.c:38-50 */
static const uint8_t lr_mod6m1[8] = { 5,0,1,2,3,4,5,0 };                                                /* me.c:53 */
static const int8_t lr_hex2[8][2] = { {-1,-2}, {-2,0}, {-1,2}, {1,2}, {2,0}, {1,-2}, {-1,-2}, {-2,0} }; /* me.c:55 */
static const int8_t lr_square1[9][2] = { {0,0}, {0,-1}, {0,1}, {-1,0}, {1,0}, {-1,-1}, {-1,1}, {1,-1}, {1,1} };

static inline uint32_t lr_pack( int a, int b ) { return (uint32_t)(uint16_t)a | ((uint32_t)(uint16_t)b << 16); }
static inline int lr_clip3( int v, int lo, int hi ) { return v < lo ? lo : v > hi ? hi : v; }
static inline int lr_median( int a, int b, int c )
{
    int mn = a < b ? a : b, mx = a < b ? b : a;
    return c < mn ? mn : c > mx ? mx : c;
}

typedef struct
{
    const pixel *fenc;               /* 8x8 block, FENC_STRIDE */
    const pixel *planes[4];          /* F, H, V, C of the reference at the block */
    const pixel *fw;                 /* p_fref_w: the weighted F plane (= planes[0] unweighted) */
    const int *wt;                   /* m->weight: { scale, denom, offset } or NULL */
    intptr_t stride;
    const uint16_t *cmx, *cmy;       /* p_cost_mvx / p_cost_mvy = cost_mv - mvp */
    int satd;                        /* mbcmp: satd (else sad) */
    int spel_min[2], spel_max[2];    /* h->mb.mv_min_spel / mv_max_spel */
    int fpel_min[2], fpel_max[2];    /* mv_limit_fpel */
} lrme_t;

static int lr_fpel( const lrme_t *m, int mx, int my )          /* fpelcmp on p_fref_w (me.c:63-70) */
{
    return FN(sad)( 3, m->fenc, FENC_STRIDE, m->fw + my * m->stride + mx, m->stride );
}

static int lr_qpel( const lrme_t *m, int mx, int my, int satd ) /* get_ref (mc.c:221-249, m->weight) then cmp */
{
    pixel tmp[8 * 16];
    intptr_t ts = 16;
    const pixel *r = get_ref_w( tmp, &ts, m->planes, m->stride, mx, my, 8, 8, m->wt );
    return satd ? FN(satd)( 3, m->fenc, FENC_STRIDE, r, ts ) : FN(sad)( 3, m->fenc, FENC_STRIDE, r, ts );
}

#define LR_BITS_MVD( mx, my ) (m->cmx[(mx) * 4] + m->cmy[(my) * 4])
#define LR_COST_MV( mx, my ) do { int c_ = lr_fpel( m, mx, my ) + LR_BITS_MVD( mx, my ); \
                                  if( c_ < bcost ) { bcost = c_; bmx = (mx); bmy = (my); } } while( 0 )
#define LR_CHECK_MVRANGE( mx, my ) ( (mx) >= m->fpel_min[0] && (mx) <= m->fpel_max[0] && \
                                     (my) >= m->fpel_min[1] && (my) <= m->fpel_max[1] )

/* x264_me_search_ref (me.c:182-420, 774-790) then refine_subpel (me.c:912-992) */
static void lr_me_search( const lrme_t *m, const int mvp[2], int16_t (*mvc)[2], int i_mvc, int me_method,
                          int subme, int me_range, int mv[2], int *cost )
{
    int bmx, bmy, bcost = LR_COST_MAX, bpred_cost = LR_COST_MAX;
    uint32_t pmv, bpred_mv = 0;
    int16_t tmp[16][2];
    if( subme >= 3 )
    {
        int bpx = lr_clip3( mvp[0], 4 * m->fpel_min[0], 4 * m->fpel_max[0] );
        int bpy = lr_clip3( mvp[1], 4 * m->fpel_min[1], 4 * m->fpel_max[1] );
        pmv = lr_pack( bpx, bpy );
        bpred_cost = lr_qpel( m, bpx, bpy, 0 ) + m->cmx[bpx] + m->cmy[bpy];      /* COST_MV_HPEL */
        const int pmv_cost = bpred_cost;
        if( i_mvc > 0 )
        {
            /* x264_predictor_clip (common/common.h:790-805) */
            int valid = 0;
            for( int i = 0; i < i_mvc; i++ )
            {
                uint32_t v = lr_pack( mvc[i][0], mvc[i][1] );
                if( !v || v == pmv )
                    continue;
                tmp[2 + valid][0] = lr_clip3( mvc[i][0], 4 * m->fpel_min[0], 4 * m->fpel_max[0] );
                tmp[2 + valid][1] = lr_clip3( mvc[i][1], 4 * m->fpel_min[1], 4 * m->fpel_max[1] );
                valid++;
            }
            if( valid > 0 )
            {
                tmp[1][0] = bpx; tmp[1][1] = bpy;
                bpred_cost <<= 4;
                for( int i = 1; i <= valid; i++ )
                {
                    int mx = tmp[i + 1][0], my = tmp[i + 1][1];
                    int c = lr_qpel( m, mx, my, 0 ) + m->cmx[mx] + m->cmy[my];
                    if( (c << 4) + i < bpred_cost )
                        bpred_cost = (c << 4) + i;
                }
                bpx = tmp[(bpred_cost & 15) + 1][0];
                bpy = tmp[(bpred_cost & 15) + 1][1];
                bpred_cost >>= 4;
            }
        }
        bmx = (bpx + 2) >> 2;
        bmy = (bpy + 2) >> 2;
        bpred_mv = lr_pack( bpx, bpy );
        if( bpred_mv & 0x00030003 )
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
        bmx = lr_clip3( (mvp[0] + 2) >> 2, m->fpel_min[0], m->fpel_max[0] );
        bmy = lr_clip3( (mvp[1] + 2) >> 2, m->fpel_min[1], m->fpel_max[1] );
        pmv = lr_pack( bmx, bmy );
        bcost = lr_fpel( m, bmx, bmy );
        if( i_mvc > 0 )
        {
            /* x264_predictor_roundclip (common/common.h:774-788) */
            int valid = 0;
            for( int i = 0; i < i_mvc; i++ )
            {
                int mx = (mvc[i][0] + 2) >> 2, my = (mvc[i][1] + 2) >> 2;
                uint32_t v = lr_pack( mx, my );
                if( !v || v == pmv )
                    continue;
                tmp[2 + valid][0] = lr_clip3( mx, m->fpel_min[0], m->fpel_max[0] );
                tmp[2 + valid][1] = lr_clip3( my, m->fpel_min[1], m->fpel_max[1] );
                valid++;
            }
            if( valid > 0 )
            {
                tmp[1][0] = bmx; tmp[1][1] = bmy;
                bcost <<= 4;
                for( int i = 1; i <= valid; i++ )
                {
                    int mx = tmp[i + 1][0], my = tmp[i + 1][1];
                    int c = lr_fpel( m, mx, my ) + LR_BITS_MVD( mx, my );
                    if( (c << 4) + i < bcost )
                        bcost = (c << 4) + i;
                }
                bmx = tmp[(bcost & 15) + 1][0];
                bmy = tmp[(bcost & 15) + 1][1];
                bcost >>= 4;
            }
        }
        if( pmv )
            LR_COST_MV( 0, 0 );
    }

    int costs[8];
    if( me_method == 0 )
    {
        /* diamond search, radius 1 (me.c:322-342) */
        bcost <<= 4;
        int i = me_range;
        do
        {
            costs[0] = lr_fpel( m, bmx, bmy - 1 ) + LR_BITS_MVD( bmx, bmy - 1 );
            costs[1] = lr_fpel( m, bmx, bmy + 1 ) + LR_BITS_MVD( bmx, bmy + 1 );
            costs[2] = lr_fpel( m, bmx - 1, bmy ) + LR_BITS_MVD( bmx - 1, bmy );
            costs[3] = lr_fpel( m, bmx + 1, bmy ) + LR_BITS_MVD( bmx + 1, bmy );
            if( (costs[0] << 4) + 1 < bcost ) bcost = (costs[0] << 4) + 1;
            if( (costs[1] << 4) + 3 < bcost ) bcost = (costs[1] << 4) + 3;
            if( (costs[2] << 4) + 4 < bcost ) bcost = (costs[2] << 4) + 4;
            if( (costs[3] << 4) + 12 < bcost ) bcost = (costs[3] << 4) + 12;
            if( !(bcost & 15) )
                break;
            bmx -= (int32_t)((uint32_t)bcost << 28) >> 30;
            bmy -= (int32_t)((uint32_t)bcost << 30) >> 30;
            bcost &= ~15;
        } while( --i && LR_CHECK_MVRANGE( bmx, bmy ) );
        bcost >>= 4;
    }
    else
    {
        /* hexagon search, radius 2, then the square refine (me.c:344-420) */
#define LR_X3( a, b, c, d, e, f, o ) do { \
        (o)[0] = lr_fpel( m, bmx + (a), bmy + (b) ) + LR_BITS_MVD( bmx + (a), bmy + (b) ); \
        (o)[1] = lr_fpel( m, bmx + (c), bmy + (d) ) + LR_BITS_MVD( bmx + (c), bmy + (d) ); \
        (o)[2] = lr_fpel( m, bmx + (e), bmy + (f) ) + LR_BITS_MVD( bmx + (e), bmy + (f) ); } while( 0 )
        LR_X3( -2, 0, -1, 2, 1, 2, costs );
        LR_X3( 2, 0, 1, -2, -1, -2, costs + 4 );
        bcost <<= 3;
        if( (costs[0] << 3) + 2 < bcost ) bcost = (costs[0] << 3) + 2;
        if( (costs[1] << 3) + 3 < bcost ) bcost = (costs[1] << 3) + 3;
        if( (costs[2] << 3) + 4 < bcost ) bcost = (costs[2] << 3) + 4;
        if( (costs[4] << 3) + 5 < bcost ) bcost = (costs[4] << 3) + 5;
        if( (costs[5] << 3) + 6 < bcost ) bcost = (costs[5] << 3) + 6;
        if( (costs[6] << 3) + 7 < bcost ) bcost = (costs[6] << 3) + 7;
        if( bcost & 7 )
        {
            int dir = (bcost & 7) - 2;
            bmx += lr_hex2[dir + 1][0];
            bmy += lr_hex2[dir + 1][1];
            for( int i = (me_range >> 1) - 1; i > 0 && LR_CHECK_MVRANGE( bmx, bmy ); i-- )
            {
                LR_X3( lr_hex2[dir][0], lr_hex2[dir][1], lr_hex2[dir + 1][0], lr_hex2[dir + 1][1],
                       lr_hex2[dir + 2][0], lr_hex2[dir + 2][1], costs );
                bcost &= ~7;
                if( (costs[0] << 3) + 1 < bcost ) bcost = (costs[0] << 3) + 1;
                if( (costs[1] << 3) + 2 < bcost ) bcost = (costs[1] << 3) + 2;
                if( (costs[2] << 3) + 3 < bcost ) bcost = (costs[2] << 3) + 3;
                if( !(bcost & 7) )
                    break;
                dir += (bcost & 7) - 2;
                dir = lr_mod6m1[dir + 1];
                bmx += lr_hex2[dir + 1][0];
                bmy += lr_hex2[dir + 1][1];
            }
        }
        bcost >>= 3;
#undef LR_X3
        bcost <<= 4;
        static const int8_t sq[8][2] = { {0,-1}, {0,1}, {-1,0}, {1,0}, {-1,-1}, {-1,1}, {1,-1}, {1,1} };
        for( int k = 0; k < 8; k++ )
        {
            int c = lr_fpel( m, bmx + sq[k][0], bmy + sq[k][1] ) + LR_BITS_MVD( bmx + sq[k][0], bmy + sq[k][1] );
            if( (c << 4) + k + 1 < bcost )
                bcost = (c << 4) + k + 1;
        }
        bmx += lr_square1[bcost & 15][0];
        bmy += lr_square1[bcost & 15][1];
        bcost >>= 4;
    }

    /* -> qpel mv (me.c:774-790) */
    int mx, my, c;
    if( subme < 3 )
    {
        c = bcost;
        if( lr_pack( bmx, bmy ) == pmv )
            c += LR_BITS_MVD( bmx, bmy );
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

    /* refine_subpel( hpel, qpel, NULL, 0 ) (me.c:912-992) */
    const int hpel = lr_subpel_iters[subme][2], qpel = lr_subpel_iters[subme][3];
    bmx = mx; bmy = my; bcost = c;
    if( hpel )
    {
        if( subme < 3 )
        {
            int px = lr_clip3( mvp[0], m->spel_min[0] + 2, m->spel_max[0] - 2 );
            int py = lr_clip3( mvp[1], m->spel_min[1] + 2, m->spel_max[1] - 2 );
            if( (px - bmx) | (py - bmy) )
            {
                int cc = lr_qpel( m, px, py, 0 ) + m->cmx[px] + m->cmy[py];
                if( cc < bcost ) { bcost = cc; bmx = px; bmy = py; }
            }
        }
        bcost <<= 6;
        for( int i = hpel; i > 0; i-- )
        {
            int omx = bmx, omy = bmy;
            costs[0] = lr_qpel( m, omx, omy - 2, 0 ) + m->cmx[omx] + m->cmy[omy - 2];
            costs[1] = lr_qpel( m, omx, omy + 2, 0 ) + m->cmx[omx] + m->cmy[omy + 2];
            costs[2] = lr_qpel( m, omx - 2, omy, 0 ) + m->cmx[omx - 2] + m->cmy[omy];
            costs[3] = lr_qpel( m, omx + 2, omy, 0 ) + m->cmx[omx + 2] + m->cmy[omy];
            if( (costs[0] << 6) + 2 < bcost ) bcost = (costs[0] << 6) + 2;
            if( (costs[1] << 6) + 6 < bcost ) bcost = (costs[1] << 6) + 6;
            if( (costs[2] << 6) + 16 < bcost ) bcost = (costs[2] << 6) + 16;
            if( (costs[3] << 6) + 48 < bcost ) bcost = (costs[3] << 6) + 48;
            if( !(bcost & 63) )
                break;
            bmx -= (int32_t)((uint32_t)bcost << 26) >> 29;
            bmy -= (int32_t)((uint32_t)bcost << 29) >> 29;
            bcost &= ~63;
        }
        bcost >>= 6;
    }
    if( m->satd )
        bcost = lr_qpel( m, bmx, bmy, 1 ) + m->cmx[bmx] + m->cmy[bmy];   /* COST_MV_SATD( bmx, bmy, -1 ) */
    if( subme != 1 )
    {
        int bdir = -1, odir;
        for( int i = qpel; i > 0; i-- )
        {
            if( bmy <= m->spel_min[1] || bmy >= m->spel_max[1] || bmx <= m->spel_min[0] || bmx >= m->spel_max[0] )
                break;
            odir = bdir;
            int omx = bmx, omy = bmy;
            static const int8_t qd[4][2] = { {0,-1}, {0,1}, {-1,0}, {1,0} };
            for( int dir = 0; dir < 4; dir++ )
            {
                if( (dir ^ 1) == odir )
                    continue;
                int qx = omx + qd[dir][0], qy = omy + qd[dir][1];
                int cc = lr_qpel( m, qx, qy, m->satd ) + m->cmx[qx] + m->cmy[qy];
                if( cc < bcost ) { bcost = cc; bmx = qx; bmy = qy; bdir = dir; }
            }
            if( bmx == omx && bmy == omy )
                break;
        }
    }
    mv[0] = bmx;
    mv[1] = bmy;
    *cost = bcost;
}
#undef LR_COST_MV
#undef LR_BITS_MVD
#undef LR_CHECK_MVRANGE

/* per-block setup of slicetype_mb_cost (slicetype.c:539-557): the 8x8 fenc copy and
 * the lowres mv limits (the vertical ones are set at the first block of each row of the
 * do_edges scan, x = W-1, and depend on the row only) */
static void lr_setup( lrme_t *m, pixel *fbuf, const pixel *fenc, const pixel *const ref[4], intptr_t stride,
                      int mbx, int mby, int mb_width, int mb_height, int mv_range, int satd )
{
    const intptr_t off = 8 * mbx + 8 * mby * stride;
    for( int y = 0; y < 8; y++ )
        memcpy( fbuf + y * FENC_STRIDE, fenc + off + y * stride, 8 * sizeof(pixel) );
    m->fenc = fbuf;
    for( int k = 0; k < 4; k++ )
        m->planes[k] = ref[k] + off;
    m->fw = m->planes[0];
    m->wt = NULL;
    m->stride = stride;
    m->satd = satd;
    const int mvr = 2 * mv_range;
    const int lo0 = 4 * (-8 * mbx - 12), hi0 = 4 * (8 * (mb_width - mbx - 1) + 12);
    const int lo1 = 4 * (-8 * mby - 12), hi1 = 4 * (8 * (mb_height - mby - 1) + 12);
    m->spel_min[0] = lo0 > -mvr ? lo0 : -mvr;
    m->spel_max[0] = hi0 < mvr - 1 ? hi0 : mvr - 1;
    m->spel_min[1] = lo1 > -mvr ? lo1 : -mvr;
    m->spel_max[1] = hi1 < mvr - 1 ? hi1 : mvr - 1;
    for( int k = 0; k < 2; k++ )
    {
        m->fpel_min[k] = m->spel_min[k] >> 2;
        m->fpel_max[k] = m->spel_max[k] >> 2;
    }
}

/* one list of slicetype_mb_cost (slicetype.c:645-702): reverse-order predictors from
 * this pass's mvs of the list, the near-zero fast skip, x264_me_search, the cost
 * adjustments; writes mvs[mb] and returns the list cost */
static int lr_list( lrme_t *m, int16_t *mvs, int mb, int mbx, int mby, int mb_width, int mb_height, int me_method,
                    int subme, int me_range, int lambda, const uint16_t *cost_mv )
{
    int16_t mvc[4][2] = { { 0, 0 }, { 0, 0 }, { 0, 0 }, { 0, 0 } };
    int i_mvc = 0;
#define LR_MVC( i ) do { mvc[i_mvc][0] = mvs[2 * (i)]; mvc[i_mvc][1] = mvs[2 * (i) + 1]; i_mvc++; } while( 0 )
    if( mbx < mb_width - 1 )
        LR_MVC( mb + 1 );
    if( mby < mb_height - 1 )
    {
        LR_MVC( mb + mb_width );
        if( mbx > 0 )
            LR_MVC( mb + mb_width - 1 );
        if( mbx < mb_width - 1 )
            LR_MVC( mb + mb_width + 1 );
    }
#undef LR_MVC
    int mvp[2];
    if( i_mvc <= 1 )
    {
        mvp[0] = mvc[0][0];
        mvp[1] = mvc[0][1];
    }
    else
    {
        mvp[0] = lr_median( mvc[0][0], mvc[1][0], mvc[2][0] );
        mvp[1] = lr_median( mvc[0][1], mvc[1][1], mvc[2][1] );
    }
    m->cmx = cost_mv - mvp[0];
    m->cmy = cost_mv - mvp[1];
    int mv[2] = { 0, 0 }, cost = 0, skip = 0;
    if( !mvp[0] && !mvp[1] )
    {
        cost = m->satd ? FN(satd)( 3, m->fenc, FENC_STRIDE, m->planes[0], m->stride )
                       : FN(sad)( 3, m->fenc, FENC_STRIDE, m->planes[0], m->stride );
        skip = cost < 64;
    }
    if( !skip )
    {
        lr_me_search( m, mvp, mvc, i_mvc, me_method, subme, me_range, mv, &cost );
        cost -= cost_mv[0];
        if( mv[0] | mv[1] )
            cost += 5 * lambda;
    }
    mvs[2 * mb] = mv[0];
    mvs[2 * mb + 1] = mv[1];
    return cost;
}

/* One P-frame pair: fenc = lowres[0] of frame b, ref = the four lowres planes of
 * frame p0 (all at pixel (0,0), common stride, 32 pixels of border); every MB
 * in the reverse raster order of slicetype_slice_cost (slicetype.c:818-833, the
 * do_edges case, one lookahead slice).  cost_mv = a->p_cost_mv (cost_mv[qp] of
 * analyse.c:143-157, indexable over +-4*mv_range*2) at mvd 0; intra_cost =
 * fenc->i_intra_cost (x264hip lowres_intra_cost).  Outputs lowres_mvs[mb][2],
 * lowres_mv_costs[mb], lowres_costs[mb] ((list_used << 14) + cost), row_satd[y]
 * (AQ-scaled inter row sums) and est = { cost_est, cost_est_aq, intra_mbs }. */
void FN(lowres_inter_cost_ex)( const pixel *fenc, const pixel *ref0, const pixel *ref1, const pixel *ref2,
                               const pixel *ref3, const pixel *ref_w, const int *weight, int n_slices,
                               intptr_t stride, int mb_width, int mb_height, int me_method,
                               int subme, int satd, int me_range, int mv_range, int lambda, const uint16_t *cost_mv,
                               const uint16_t *intra_cost, const uint16_t *inv_qscale, int16_t *mvs,
                               int32_t *mv_costs, uint16_t *lowres_costs, int32_t *row_satd, int32_t est[3] );

void FN(lowres_inter_cost)( const pixel *fenc, const pixel *ref0, const pixel *ref1, const pixel *ref2,
                            const pixel *ref3, intptr_t stride, int mb_width, int mb_height, int me_method,
                            int subme, int satd, int me_range, int mv_range, int lambda, const uint16_t *cost_mv,
                            const uint16_t *intra_cost, const uint16_t *inv_qscale, int16_t *mvs, int32_t *mv_costs,
                            uint16_t *lowres_costs, int32_t *row_satd, int32_t est[3] )
{
    FN(lowres_inter_cost_ex)( fenc, ref0, ref1, ref2, ref3, NULL, NULL, 1, stride, mb_width, mb_height, me_method,
                              subme, satd, me_range, mv_range, lambda, cost_mv, intra_cost, inv_qscale, mvs, mv_costs,
                              lowres_costs, row_satd, est );
}

/* The weighted-reference form (slicetype.c:603-614 with w[0].weightfn set, i.e. when
 * x264_weights_analyse( h, fenc, frames[p0], 1 ) picked a weight, slicetype.c:859-862):
 * the integer-pel stage reads fenc->weighted[0] (ref_w, the F plane scaled by
 * x264_weight_scale_plane, slicetype.c:490-499) and every get_ref of the subpel stages
 * weights the unweighted hpel planes with m->weight = weight { scale, denom, offset };
 * the near-zero fast skip still compares against the unweighted F plane
 * (slicetype.c:680).  ref_w / weight NULL: the unweighted search. */
void FN(lowres_inter_cost_ex)( const pixel *fenc, const pixel *ref0, const pixel *ref1, const pixel *ref2,
                               const pixel *ref3, const pixel *ref_w, const int *weight, int n_slices,
                               intptr_t stride, int mb_width, int mb_height, int me_method,
                               int subme, int satd, int me_range, int mv_range, int lambda, const uint16_t *cost_mv,
                               const uint16_t *intra_cost, const uint16_t *inv_qscale, int16_t *mvs,
                               int32_t *mv_costs, uint16_t *lowres_costs, int32_t *row_satd, int32_t est[3] )
{
    pixel fbuf[8 * FENC_STRIDE];
    const pixel *ref[4] = { ref0, ref1, ref2, ref3 };
    est[0] = est[1] = est[2] = 0;
    for( int y = 0; y < mb_height; y++ )
        row_satd[y] = 0;
    /* i_lookahead_threads > 1 (slicetype.c:901-918): slice i covers MB rows
     * [(H*i + T/2)/T, (H*(i+1) + T/2)/T), each scanned on its own (slicetype_slice_cost,
     * slicetype.c:813-833) with the row-below predictors only inside the slice
     * (slicetype.c:664, h->i_threadslice_end); the slices' sums add up */
    for( int sl = 0; sl < n_slices; sl++ )
    for( int mby = (mb_height * (sl + 1) + n_slices / 2) / n_slices - 1,
             s0 = (mb_height * sl + n_slices / 2) / n_slices,
             s1 = (mb_height * (sl + 1) + n_slices / 2) / n_slices; mby >= s0; mby-- )
        for( int mbx = mb_width - 1; mbx >= 0; mbx-- )
        {
            const int mb = mbx + mby * mb_width;
            lrme_t m;
            lr_setup( &m, fbuf, fenc, ref, stride, mbx, mby, mb_width, mb_height, mv_range, satd );
            if( ref_w && weight )
            {
                m.fw = ref_w + 8 * mbx + 8 * mby * stride;
                m.wt = weight;
            }
            const int cost = lr_list( &m, mvs, mb, mbx, mby, mb_width, s1, me_method, subme, me_range, lambda,
                                      cost_mv );
            mv_costs[mb] = cost;
            /* slicetype.c:758-790 */
            int bcost = (cost >> (BIT_DEPTH - 8)) + 4, list_used = 1;
            const int fsm = (mbx > 0 && mbx < mb_width - 1 && mby > 0 && mby < mb_height - 1) || mb_width <= 2 ||
                            mb_height <= 2;
            const int b_intra = intra_cost[mb] < bcost;
            if( b_intra )
            {
                bcost = intra_cost[mb];
                list_used = 0;
            }
            if( fsm )
                est[2] += b_intra;
            const int aq = inv_qscale ? (bcost * inv_qscale[mb] + 128) >> 8 : bcost;
            row_satd[mby] += aq;
            if( fsm )
            {
                est[0] += bcost;
                est[1] += aq;
            }
            lowres_costs[mb] = (uint16_t)((bcost < 16383 ? bcost : 16383) + (list_used << 14));
        }
}

/* TRY_BIDIR (slicetype.c:589-612): the weighted average of the two lists' predictions
 * (pixel_avg / pixel_avg_weight_wxh, mc.c:49-87) scored with mbcmp.  subme2 = the
 * lookahead runs subme 2 (param subme <= 1): hpel planes addressed directly. */
static int lr_bidir( const lrme_t *m0, const lrme_t *m1, const int mv0[2], const int mv1[2], int subme2, int weight )
{
    pixel a[8 * 16], b[8 * 16], avg[8 * 16];
    const pixel *s1, *s2;
    intptr_t st1 = 16, st2 = 16;
    if( subme2 )
    {
        const int i1 = ((mv0[0] & 2) >> 1) + (mv0[1] & 2), i2 = ((mv1[0] & 2) >> 1) + (mv1[1] & 2);
        s1 = m0->planes[i1] + (mv0[0] >> 2) + (mv0[1] >> 2) * m0->stride;
        s2 = m1->planes[i2] + (mv1[0] >> 2) + (mv1[1] >> 2) * m1->stride;
        st1 = m0->stride;
        st2 = m1->stride;
    }
    else
    {
        s1 = FN(get_ref)( a, &st1, m0->planes, m0->stride, mv0[0], mv0[1], 8, 8 );
        s2 = FN(get_ref)( b, &st2, m1->planes, m1->stride, mv1[0], mv1[1], 8, 8 );
    }
    for( int y = 0; y < 8; y++ )
        for( int x = 0; x < 8; x++ )
            avg[y * 16 + x] = weight == 32 ? (s1[y * st1 + x] + s2[y * st2 + x] + 1) >> 1
                                           : clip_pixel( (s1[y * st1 + x] * weight + s2[y * st2 + x] * (64 - weight) + 32) >> 6 );
    return m0->satd ? FN(satd)( 3, m0->fenc, FENC_STRIDE, avg, 16 ) : FN(sad)( 3, m0->fenc, FENC_STRIDE, avg, 16 );
}

/* One B-frame triplet p0 < b < p1: slicetype_mb_cost with b_bidir (slicetype.c:514-713,
 * 758-791): fenc = lowres[0] of frame b, ref_a / ref_b = the lowres planes of p0 / p1.
 * List l is searched when search[l] (its mvs / costs are written) or read from mvs_l /
 * costs_l (fenc->lowres_mvs[l] / lowres_mv_costs[l] of an earlier pass).  p1mvs =
 * fref1->lowres_mvs[0][p1-p0-1] (NULL: not searched, dmv = 0), dsf = dist_scale_factor,
 * weight = i_bipred_weight.  No intra in B frames.  Outputs lowres_costs[mb]
 * (fenc->lowres_costs[b-p0][p1-b]), row_satd[y] and est = { cost_est, cost_est_aq }. */
void FN(lowres_bidir_cost_ex)( const pixel *fenc, const pixel *const ref_a[4], const pixel *const ref_b[4],
                               intptr_t stride, int mb_width, int mb_height, int me_method, int subme, int satd,
                               int me_range, int mv_range, int lambda, const uint16_t *cost_mv, const int search[2],
                               int16_t *mvs0, int32_t *costs0, int16_t *mvs1, int32_t *costs1,
                               const int16_t *p1mvs, int dsf, int weight, const uint16_t *inv_qscale,
                               uint16_t *lowres_costs, int32_t *row_satd, int32_t est[2], int n_slices );

void FN(lowres_bidir_cost)( const pixel *fenc, const pixel *const ref_a[4], const pixel *const ref_b[4],
                            intptr_t stride, int mb_width, int mb_height, int me_method, int subme, int satd,
                            int me_range, int mv_range, int lambda, const uint16_t *cost_mv, const int search[2],
                            int16_t *mvs0, int32_t *costs0, int16_t *mvs1, int32_t *costs1, const int16_t *p1mvs,
                            int dsf, int weight, const uint16_t *inv_qscale, uint16_t *lowres_costs,
                            int32_t *row_satd, int32_t est[2] )
{
    FN(lowres_bidir_cost_ex)( fenc, ref_a, ref_b, stride, mb_width, mb_height, me_method, subme, satd, me_range,
                              mv_range, lambda, cost_mv, search, mvs0, costs0, mvs1, costs1, p1mvs, dsf, weight,
                              inv_qscale, lowres_costs, row_satd, est, 1 );
}

/* the B leg over n_slices lookahead slices (as lowres_inter_cost_ex) */
void FN(lowres_bidir_cost_ex)( const pixel *fenc, const pixel *const ref_a[4], const pixel *const ref_b[4],
                               intptr_t stride, int mb_width, int mb_height, int me_method, int subme, int satd,
                               int me_range, int mv_range, int lambda, const uint16_t *cost_mv, const int search[2],
                               int16_t *mvs0, int32_t *costs0, int16_t *mvs1, int32_t *costs1,
                               const int16_t *p1mvs, int dsf, int weight, const uint16_t *inv_qscale,
                               uint16_t *lowres_costs, int32_t *row_satd, int32_t est[2], int n_slices )
{
    pixel fbuf[8 * FENC_STRIDE];
    est[0] = est[1] = 0;
    for( int y = 0; y < mb_height; y++ )
        row_satd[y] = 0;
    for( int sl = 0; sl < n_slices; sl++ )
    for( int mby = (mb_height * (sl + 1) + n_slices / 2) / n_slices - 1,
             s0 = (mb_height * sl + n_slices / 2) / n_slices,
             s1 = (mb_height * (sl + 1) + n_slices / 2) / n_slices; mby >= s0; mby-- )
        for( int mbx = mb_width - 1; mbx >= 0; mbx-- )
        {
            const int mb = mbx + mby * mb_width;
            lrme_t m0, m1;
            lr_setup( &m0, fbuf, fenc, ref_a, stride, mbx, mby, mb_width, mb_height, mv_range, satd );
            lr_setup( &m1, fbuf, fenc, ref_b, stride, mbx, mby, mb_width, mb_height, mv_range, satd );
            int bcost = LR_COST_MAX, list_used = 0;
            int dmv[2][2] = { { 0, 0 }, { 0, 0 } };
            if( p1mvs )
            {
                const int mvr[2] = { p1mvs[2 * mb], p1mvs[2 * mb + 1] };
                for( int k = 0; k < 2; k++ )
                {
                    dmv[0][k] = (mvr[k] * dsf + 128) >> 8;
                    dmv[1][k] = dmv[0][k] - mvr[k];
                    dmv[0][k] = lr_clip3( dmv[0][k], m0.spel_min[k], m0.spel_max[k] );
                    dmv[1][k] = lr_clip3( dmv[1][k], m0.spel_min[k], m0.spel_max[k] );
                    if( subme == 2 )
                    {
                        dmv[0][k] &= ~1;
                        dmv[1][k] &= ~1;
                    }
                }
            }
            int c = lr_bidir( &m0, &m1, dmv[0], dmv[1], subme == 2, weight );
            if( c < bcost ) { bcost = c; list_used = 3; }
            if( dmv[0][0] | dmv[0][1] | dmv[1][0] | dmv[1][1] )
            {
                const int z[2] = { 0, 0 };
                /* h->mc.avg of the two full-pel planes at mv 0 (slicetype.c:641-645) */
                c = lr_bidir( &m0, &m1, z, z, 1, weight );
                if( c < bcost ) { bcost = c; list_used = 3; }
            }
            int mv[2][2];
            int16_t *lm[2] = { mvs0, mvs1 };
            int32_t *lc[2] = { costs0, costs1 };
            lrme_t *lmm[2] = { &m0, &m1 };
            for( int l = 0; l < 2; l++ )
            {
                int cost;
                if( search[l] )
                {
                    cost = lr_list( lmm[l], lm[l], mb, mbx, mby, mb_width, s1, me_method, subme, me_range,
                                    lambda, cost_mv );
                    lc[l][mb] = cost;
                }
                else
                    cost = lc[l][mb];
                mv[l][0] = lm[l][2 * mb];
                mv[l][1] = lm[l][2 * mb + 1];
                if( cost < bcost ) { bcost = cost; list_used = l + 1; }
            }
            if( mv[0][0] | mv[0][1] | mv[1][0] | mv[1][1] )
            {
                c = 5 * lambda + lr_bidir( &m0, &m1, mv[0], mv[1], subme == 2, weight );
                if( c < bcost ) { bcost = c; list_used = 3; }
            }
            bcost = (bcost >> (BIT_DEPTH - 8)) + 4;
            const int fsm = (mbx > 0 && mbx < mb_width - 1 && mby > 0 && mby < mb_height - 1) || mb_width <= 2 ||
                            mb_height <= 2;
            const int aq = inv_qscale ? (bcost * inv_qscale[mb] + 128) >> 8 : bcost;
            row_satd[mby] += aq;
            if( fsm )
            {
                est[0] += bcost;
                est[1] += aq;
            }
            lowres_costs[mb] = (uint16_t)((bcost < 16383 ? bcost : 16383) + (list_used << 14));
        }
}

/*============================================================================
 * weighted-prediction analysis — reference encoder/slicetype.c:63-501 (the
 * weight search), encoder/ratecontrol.c:225-257,406-414 (the frame statistics it
 * reads), common/mc.c:252-283 (mc_chroma)
 *==========================================================================*/
#include <math.h>

/* mc_chroma (common/mc.c:252-283): eighth-pel bilinear of an interleaved (NV12) plane
 * into separate U and V blocks */
void FN(mc_chroma)( pixel *dstu, pixel *dstv, intptr_t ds, const pixel *src, intptr_t ss, int mvx, int mvy,
                    int w, int h )
{
    const int dx = mvx & 7, dy = mvy & 7;
    const int cA = (8 - dx) * (8 - dy), cB = dx * (8 - dy), cC = (8 - dx) * dy, cD = dx * dy;
    src += (mvy >> 3) * ss + (mvx >> 3) * 2;
    for( int y = 0; y < h; y++, dstu += ds, dstv += ds, src += ss )
    {
        const pixel *s1 = src + ss;
        for( int x = 0; x < w; x++ )
        {
            dstu[x] = (pixel)((cA * src[2*x] + cB * src[2*x + 2] + cC * s1[2*x] + cD * s1[2*x + 2] + 32) >> 6);
            dstv[x] = (pixel)((cA * src[2*x + 1] + cB * src[2*x + 3] + cC * s1[2*x + 1] + cD * s1[2*x + 3] + 32) >> 6);
        }
    }
}

/* The frame statistics x264_weights_analyse reads (fenc->i_pixel_sum / i_pixel_ssd):
 * ac_energy_mb's stores over every MB of a progressive frame (ratecontrol.c:225-257,
 * 289-299; PIXEL_VAR_C per plane, chroma deinterleaved as load_deinterleave_chroma_fenc
 * does), the uint32 sum wrapping as the field does, then the mean removal of
 * ratecontrol.c:406-414.  chroma_format 0 = 4:0:0, 1 = 4:2:0, 2 = 4:2:2 (NV12/NV16 plane 1),
 * 3 = 4:4:4 (planes 1 and 2). */
void FN(frame_pixel_stats)( const pixel *const plane[3], const intptr_t stride[3], int mb_width, int mb_height,
                            int chroma_format, uint32_t sum[3], uint64_t ssd[3] )
{
    const int hs = chroma_format == 1 || chroma_format == 2, vs = chroma_format == 1;
    for( int i = 0; i < 3; i++ )
        sum[i] = 0, ssd[i] = 0;
    for( int mby = 0; mby < mb_height; mby++ )
        for( int mbx = 0; mbx < mb_width; mbx++ )
        {
            uint64_t v = FN(var)( 0, plane[0] + 16 * mbx + 16 * mby * stride[0], stride[0] );
            sum[0] += (uint32_t)v;
            ssd[0] += v >> 32;
            if( chroma_format == 3 )
                for( int p = 1; p <= 2; p++ )
                {
                    v = FN(var)( 0, plane[p] + 16 * mbx + 16 * mby * stride[p], stride[p] );
                    sum[p] += (uint32_t)v;
                    ssd[p] += v >> 32;
                }
            else if( chroma_format )
            {
                const int h = 16 >> vs;
                pixel buf[16 * 16];
                const pixel *s = plane[1] + 16 * mbx + h * mby * stride[1];
                for( int y = 0; y < h; y++ )
                    for( int x = 0; x < 8; x++ )
                    {
                        buf[y * 16 + x] = s[y * stride[1] + 2 * x];
                        buf[y * 16 + 8 + x] = s[y * stride[1] + 2 * x + 1];
                    }
                for( int p = 1; p <= 2; p++ )
                {
                    v = FN(var)( h == 8 ? 3 : 2, buf + 8 * (p - 1), 16 );
                    sum[p] += (uint32_t)v;
                    ssd[p] += v >> 32;
                }
            }
        }
    for( int i = 0; i < 3; i++ )
    {
        const uint64_t s = sum[i];
        const uint64_t w = (uint64_t)(16 * mb_width >> (i && hs)), h = (uint64_t)(16 * mb_height >> (i && vs));
        ssd[i] = ssd[i] - (s * s + w * h / 2) / (w * h);
    }
}

/* x264_weight_t as the search leaves it: weighted = (weightfn != NULL) */
typedef struct { int weighted, scale, denom, offset; } FN(wp_t);

static int wp_ue_tab( unsigned v )   /* x264_ue_size_tab[v] (common/bitstream.h:201-219) */
{
    int n = 0;
    while( v >> (n + 1) )
        n++;
    return v ? 2 * n + 1 : 1;
}
static int wp_size_ue( unsigned v ) { return wp_ue_tab( v + 1 ); }        /* bitstream.h:278-281 */
static int wp_size_se( int v )                                            /* bitstream.h:291-299 */
{
    int tmp = 1 - v * 2;
    if( tmp < 0 )
        tmp = v * 2;
    return tmp < 256 ? wp_ue_tab( tmp ) : wp_ue_tab( tmp >> 8 ) + 16;
}

/* weight_slice_header_cost (slicetype.c:170-189); lambda = x264_lambda_tab[X264_LOOKAHEAD_QP] */
static int wp_header_cost( const FN(wp_t) *w, int b_chroma, int lambda, int numslices )
{
    if( b_chroma )
        lambda *= 4;
    const int denom_cost = wp_size_ue( w->denom ) * (2 - b_chroma);
    return lambda * numslices * (10 + denom_cost + 2 * (wp_size_se( w->scale ) + wp_size_se( w->offset )));
}

typedef struct
{
    const pixel *fenc_lr;            /* fenc->lowres[0] at (0,0) */
    const pixel *const *ref_lr;      /* ref->lowres[0..3] at (0,0) */
    intptr_t lrs;                    /* i_stride_lowres */
    int mbw, mbh;
    const uint16_t *intra;           /* fenc->i_intra_cost */
    const int16_t *mvs;              /* fenc->lowres_mvs[0][ref0_distance], NULL = 0x7FFF (not searched) */
    int cf;                          /* chroma format */
    const pixel *const *fplane, *const *rplane;   /* full-resolution planes at (0,0) */
    const intptr_t *ps;              /* their strides */
    int satd, lambda, numslices;
} FN(wpctx_t);

/* weight_cost_luma (slicetype.c:191-222): mbcmp 8x8 of the (weighted) reference against the
 * lowres fenc, each MB capped at its intra cost, plus the header cost when weighted */
static unsigned wp_cost_luma( const FN(wpctx_t) *c, const pixel *src, intptr_t ss, const FN(wp_t) *w )
{
    unsigned cost = 0;
    pixel buf[64];
    for( int y = 0, mb = 0; y < 8 * c->mbh; y += 8 )
        for( int x = 0; x < 8 * c->mbw; x += 8, mb++ )
        {
            const pixel *r = src + y * ss + x;
            intptr_t rs = ss;
            if( w )
            {
                FN(mc_weight)( buf, 8, r, ss, w->scale, w->denom, w->offset, 8, 8 );
                r = buf;
                rs = 8;
            }
            const pixel *f = c->fenc_lr + y * c->lrs + x;
            const int cmp = c->satd ? FN(satd)( 3, r, rs, f, c->lrs ) : FN(sad)( 3, r, rs, f, c->lrs );
            cost += cmp < c->intra[mb] ? cmp : c->intra[mb];
        }
    if( w )
        cost += wp_header_cost( w, 0, c->lambda, c->numslices );
    return cost;
}

/* weight_cost_chroma (slicetype.c:224-255): asd8 (the DC difference) of 8 x (16 >> vshift)
 * blocks of the (weighted) motion-compensated reference plane against the fenc plane */
static unsigned wp_cost_chroma( const FN(wpctx_t) *c, const pixel *ref, const pixel *src, intptr_t s,
                                const FN(wp_t) *w )
{
    unsigned cost = 0;
    const int h = c->cf == 1 ? 8 : 16;
    pixel buf[8 * 16];
    for( int y = 0; y < h * c->mbh; y += h )
        for( int x = 0; x < 8 * c->mbw; x += 8 )
        {
            if( w )
            {
                FN(mc_weight)( buf, 8, ref + y * s + x, s, w->scale, w->denom, w->offset, 8, h );
                cost += FN(asd8)( buf, 8, src + y * s + x, s, h );
            }
            else
                cost += FN(asd8)( ref + y * s + x, s, src + y * s + x, s, h );
        }
    if( w )
        cost += wp_header_cost( w, 1, c->lambda, c->numslices );
    return cost;
}

/* weight_cost_chroma444 (slicetype.c:257-282): mbcmp 16x16 of the (weighted) reference plane */
static unsigned wp_cost_444( const FN(wpctx_t) *c, const pixel *ref, intptr_t rs, int p, const FN(wp_t) *w )
{
    unsigned cost = 0;
    pixel buf[256];
    const pixel *src = c->fplane[p];
    const intptr_t s = c->ps[p];
    for( int y = 0; y < 16 * c->mbh; y += 16 )
        for( int x = 0; x < 16 * c->mbw; x += 16 )
        {
            const pixel *r = ref + y * rs + x;
            intptr_t st = rs;
            if( w )
            {
                FN(mc_weight)( buf, 16, r, rs, w->scale, w->denom, w->offset, 16, 16 );
                r = buf;
                st = 16;
            }
            cost += c->satd ? FN(satd)( 0, r, st, src + y * s + x, s ) : FN(sad)( 0, r, st, src + y * s + x, s );
        }
    if( w )
        cost += wp_header_cost( w, 1, c->lambda, c->numslices );
    return cost;
}

/* the motion-compensated lowres reference of weight_cost_init_luma (slicetype.c:77-103):
 * get_ref of each 8x8 block at lowres_mvs + the block position, into a buffer of stride 8*mbw */
static pixel *wp_mc_luma( const FN(wpctx_t) *c )
{
    const intptr_t st = 8 * c->mbw;
    pixel *buf = malloc( sizeof(pixel) * 64 * c->mbw * c->mbh );
    for( int y = 0, mb = 0; y < 8 * c->mbh; y += 8 )
        for( int x = 0; x < 8 * c->mbw; x += 8, mb++ )
        {
            pixel tmp[64];
            intptr_t ts = 8;
            const pixel *r = FN(get_ref)( tmp, &ts, c->ref_lr, c->lrs, c->mvs[2 * mb] + (x << 2),
                                          c->mvs[2 * mb + 1] + (y << 2), 8, 8 );
            for( int j = 0; j < 8; j++ )
                memcpy( buf + (y + j) * st + x, r + j * ts, 8 * sizeof(pixel) );
        }
    return buf;
}

/* weight_cost_init_chroma444 (slicetype.c:142-168): 16x16 copies at lowres_mvs / 2 */
static pixel *wp_mc_444( const FN(wpctx_t) *c, int p )
{
    const intptr_t st = 16 * c->mbw;
    pixel *buf = malloc( sizeof(pixel) * 256 * c->mbw * c->mbh );
    for( int y = 0, mb = 0; y < 16 * c->mbh; y += 16 )
        for( int x = 0; x < 16 * c->mbw; x += 16, mb++ )
        {
            const int mvx = c->mvs[2 * mb] / 2, mvy = c->mvs[2 * mb + 1] / 2;
            const pixel *s = c->rplane[p] + y * c->ps[p] + x + mvx + mvy * c->ps[p];
            for( int j = 0; j < 16; j++ )
                memcpy( buf + (y + j) * st + x, s + j * c->ps[p], 16 * sizeof(pixel) );
        }
    return buf;
}

/* weight_cost_init_chroma (slicetype.c:111-140): U / V of the reference -- mc_chroma of
 * lowres_mvs (mvy scaled by 2 >> vshift) or the plane deinterleaved -- and of fenc, stride 8*mbw */
static void wp_mc_chroma( const FN(wpctx_t) *c, pixel **mcu, pixel **mcv, pixel **fu, pixel **fv )
{
    const int vs = c->cf == 1, h = 16 >> vs;
    const intptr_t st = 8 * c->mbw, ps = c->ps[1];
    const size_t n = sizeof(pixel) * 8 * c->mbw * h * c->mbh;
    *mcu = malloc( n ); *mcv = malloc( n ); *fu = malloc( n ); *fv = malloc( n );
    for( int y = 0, mb = 0; y < h * c->mbh; y += h )
        for( int x = 0; x < 8 * c->mbw; x += 8, mb++ )
        {
            if( c->mvs )
                FN(mc_chroma)( *mcu + y * st + x, *mcv + y * st + x, st, c->rplane[1] + y * ps + 2 * x, ps,
                               c->mvs[2 * mb], 2 * c->mvs[2 * mb + 1] >> vs, 8, h );
            for( int j = 0; j < h; j++ )
                for( int i = 0; i < 8; i++ )
                {
                    const intptr_t o = (y + j) * ps + 2 * (x + i);
                    if( !c->mvs )
                    {
                        (*mcu)[(y + j) * st + x + i] = c->rplane[1][o];
                        (*mcv)[(y + j) * st + x + i] = c->rplane[1][o + 1];
                    }
                    (*fu)[(y + j) * st + x + i] = c->fplane[1][o];
                    (*fv)[(y + j) * st + x + i] = c->fplane[1][o + 1];
                }
        }
}

/* weight_cost_luma / _chroma / _chroma444 of n candidates (cands[4i..4i+3] = weighted, scale,
 * denom, offset; weighted 0 = the w == NULL cost) -- the per-candidate check of
 * x264hip_*_weight_cost_batch.  kind 0: fenc / ref[0..3] lowres; 1 / 2: NV12 / NV16 planes,
 * plane 0 = U, 1 = V; 3: one 4:4:4 chroma plane. */
void FN(weight_cost_list)( int kind, const pixel *fenc, const pixel *const ref[4], intptr_t stride, int mbw,
                           int mbh, const uint16_t *intra, const int16_t *mvs, int satd, int plane, int lambda,
                           int numslices, const int *cands, int n, uint32_t *out )
{
    const pixel *fp[3] = { fenc, fenc, fenc }, *rp[3] = { ref[0], ref[0], ref[0] };
    const intptr_t ps[3] = { stride, stride, stride };
    const FN(wpctx_t) c = { fenc, ref, stride, mbw, mbh, intra, mvs, kind == 3 ? 3 : kind, fp, rp, ps, satd, lambda,
                            numslices };
    pixel *b0 = NULL, *b1 = NULL, *b2 = NULL, *b3 = NULL;
    for( int i = 0; i < n; i++ )
    {
        const FN(wp_t) w = { cands[4 * i], cands[4 * i + 1], cands[4 * i + 2], cands[4 * i + 3] };
        const FN(wp_t) *wp = w.weighted ? &w : NULL;
        if( kind == 0 )
        {
            if( mvs && !b0 )
                b0 = wp_mc_luma( &c );
            out[i] = b0 ? wp_cost_luma( &c, b0, 8 * mbw, wp ) : wp_cost_luma( &c, ref[0], stride, wp );
        }
        else if( kind == 3 )
        {
            if( mvs && !b0 )
                b0 = wp_mc_444( &c, 1 );
            out[i] = b0 ? wp_cost_444( &c, b0, 16 * mbw, 1, wp ) : wp_cost_444( &c, ref[0], stride, 1, wp );
        }
        else
        {
            if( !b0 )
                wp_mc_chroma( &c, &b0, &b1, &b2, &b3 );
            out[i] = wp_cost_chroma( &c, plane ? b1 : b0, plane ? b3 : b2, 8 * mbw, wp );
        }
    }
    free( b0 ); free( b1 ); free( b2 ); free( b3 );
}

static int wp_clip3( int v, int lo, int hi ) { return v < lo ? lo : v > hi ? hi : v; }
static double wp_clip3f( double v, double lo, double hi ) { return v < lo ? lo : v > hi ? hi : v; }

/* weight_get_h264 (slicetype.c:63-75) */
static void wp_get_h264( int weight_nonh264, int offset, FN(wp_t) *w )
{
    w->offset = offset;
    w->denom = 7;
    w->scale = weight_nonh264;
    while( w->denom > 0 && w->scale > 127 )
    {
        w->denom--;
        w->scale >>= 1;
    }
    w->scale = w->scale < 127 ? w->scale : 127;
}

#define WP_SET( w, b, s, d, o ) do { (w).scale = (s); (w).denom = (d); (w).offset = (o); (w).weighted = (b); } while( 0 )

/* x264_weights_analyse (slicetype.c:284-501) for one (fenc, ref) pair.  fsum / fssd /
 * rsum / rssd = fenc / ref i_pixel_sum / i_pixel_ssd; subme = param i_subpel_refine;
 * weightp_fake = (param i_weighted_pred == X264_WEIGHTP_FAKE).  The caller's ref planes
 * carry expanded borders (the reference expands the chroma border itself,
 * slicetype.c:124 / :151).  Writes weights[3] (fenc->weight[0][0..2]), *cost_delta
 * (fenc->f_weighted_cost_delta[i_delta_index], FAKE only) and, in the lookahead with a
 * luma weight, the weighted lowres plane (slicetype.c:490-500) at wlr (its (0,0), stride
 * lrs, 32-pixel border) when wlr is not NULL. */
void FN(weights_analyse)( const pixel *fenc_lr, const pixel *const ref_lr[4], intptr_t lrs, int mbw, int mbh,
                          const uint16_t *intra, const int16_t *mvs, int cf, const pixel *const fplane[3],
                          const pixel *const rplane[3], const intptr_t ps[3], const uint32_t fsum[3],
                          const uint64_t fssd[3], const uint32_t rsum[3], const uint64_t rssd[3], int b_lookahead,
                          int subme, int satd, int lambda, int numslices, int weightp_fake, FN(wp_t) weights[3],
                          float *cost_delta, pixel *wlr )
{
    const FN(wpctx_t) c = { fenc_lr, ref_lr, lrs, mbw, mbh, intra, mvs, cf, fplane, rplane, ps, satd, lambda,
                            numslices };
    const int hs = cf == 1 || cf == 2, vs = cf == 1;
    const float epsilon = 1.f / 128.f;
    WP_SET( weights[0], 0, 1, 0, 0 );
    WP_SET( weights[1], 0, 1, 0, 0 );
    WP_SET( weights[2], 0, 1, 0, 0 );
    int chroma_initted = 0;
    float guess_scale[3], fenc_mean[3], ref_mean[3];
    for( int plane = 0; plane <= 2 * !b_lookahead; plane++ )
    {
        if( !plane || cf )
        {
            const int zero_bias = !rssd[plane];
            const float fenc_var = fssd[plane] + zero_bias;
            const float ref_var = rssd[plane] + zero_bias;
            const int npx = (16 * mbh >> (plane ? vs : 0)) * (16 * mbw >> (plane ? hs : 0));
            guess_scale[plane] = sqrtf( fenc_var / ref_var );
            fenc_mean[plane] = (float)(fsum[plane] + zero_bias) / npx / (1 << (BIT_DEPTH - 8));
            ref_mean[plane] = (float)(rsum[plane] + zero_bias) / npx / (1 << (BIT_DEPTH - 8));
        }
        else
        {
            guess_scale[plane] = 1;
            fenc_mean[plane] = 0;
            ref_mean[plane] = 0;
        }
    }

    int chroma_denom = 7;
    if( !b_lookahead )
        while( chroma_denom > 0 )
        {
            const float thresh = 127.f / (1 << chroma_denom);
            if( guess_scale[1] < thresh && guess_scale[2] < thresh )
                break;
            chroma_denom--;
        }

    pixel *mcl = NULL, *mcu = NULL, *mcv = NULL, *fu = NULL, *fv = NULL, *mc444 = NULL;
    for( int plane = 0; plane < (cf ? 3 : 1) && !(plane && (!weights[0].weighted || b_lookahead)); plane++ )
    {
        int minoff, minscale, mindenom, found;
        unsigned minscore, origscore;
        if( fabsf( ref_mean[plane] - fenc_mean[plane] ) < 0.5f && fabsf( 1.f - guess_scale[plane] ) < epsilon )
        {
            WP_SET( weights[plane], 0, 1, 0, 0 );
            continue;
        }
        if( plane )
        {
            weights[plane].denom = chroma_denom;
            weights[plane].scale = wp_clip3( round( guess_scale[plane] * (1 << chroma_denom) ), 0, 255 );
            if( weights[plane].scale > 127 )
            {
                weights[1].weighted = weights[2].weighted = 0;
                break;
            }
        }
        else
            wp_get_h264( round( guess_scale[plane] * 128 ), 0, &weights[plane] );

        found = 0;
        mindenom = weights[plane].denom;
        minscale = weights[plane].scale;
        minoff = 0;

        /* the motion-compensated reference: weight_cost_init_luma / _chroma / _chroma444
         * (slicetype.c:77-168) */
        const pixel *mref;
        intptr_t mrs;
        if( !plane )
        {
            if( mvs )
            {
                if( !mcl )
                    mcl = wp_mc_luma( &c );
                mref = mcl;
                mrs = 8 * mbw;
            }
            else
            {
                mref = ref_lr[0];
                mrs = lrs;
            }
            origscore = minscore = wp_cost_luma( &c, mref, mrs, NULL );
        }
        else if( cf == 3 )
        {
            if( mvs )
            {
                free( mc444 );
                mc444 = wp_mc_444( &c, plane );
                mref = mc444;
                mrs = 16 * mbw;
            }
            else
            {
                mref = rplane[plane];
                mrs = ps[plane];
            }
            origscore = minscore = wp_cost_444( &c, mref, mrs, plane, NULL );
        }
        else
        {
            const intptr_t st = 8 * mbw;
            if( !chroma_initted++ )
                wp_mc_chroma( &c, &mcu, &mcv, &fu, &fv );
            mref = plane == 1 ? mcu : mcv;
            mrs = st;
            origscore = minscore = wp_cost_chroma( &c, mref, plane == 1 ? fu : fv, st, NULL );
        }

        if( !minscore )
            continue;

        static const uint8_t weight_check_distance[][2] = {
            {0,0},{0,0},{0,1},{0,1}, {0,1},{0,1},{0,1},{1,1}, {1,1},{2,1},{2,1},{4,2} };
        const int scale_dist = b_lookahead ? 0 : weight_check_distance[subme][0];
        const int offset_dist = b_lookahead ? 0 : weight_check_distance[subme][1];
        const int start_scale = wp_clip3( minscale - scale_dist, 0, 127 );
        const int end_scale = wp_clip3( minscale + scale_dist, 0, 127 );
        for( int i_scale = start_scale; i_scale <= end_scale; i_scale++ )
        {
            int cur_scale = i_scale;
            int cur_offset = fenc_mean[plane] - ref_mean[plane] * cur_scale / (1 << mindenom) + 0.5f * b_lookahead;
            if( cur_offset < -128 || cur_offset > 127 )
            {
                cur_offset = wp_clip3( cur_offset, -128, 127 );
                cur_scale = wp_clip3f( (1 << mindenom) * (fenc_mean[plane] - cur_offset) / ref_mean[plane] + 0.5f, 0,
                                       127 );
            }
            const int start_offset = wp_clip3( cur_offset - offset_dist, -128, 127 );
            const int end_offset = wp_clip3( cur_offset + offset_dist, -128, 127 );
            for( int i_off = start_offset; i_off <= end_offset; i_off++ )
            {
                WP_SET( weights[plane], 1, cur_scale, mindenom, i_off );
                unsigned s;
                if( !plane )
                    s = wp_cost_luma( &c, mref, mrs, &weights[plane] );
                else if( cf == 3 )
                    s = wp_cost_444( &c, mref, mrs, plane, &weights[plane] );
                else
                    s = wp_cost_chroma( &c, mref, plane == 1 ? fu : fv, mrs, &weights[plane] );
                if( s < minscore )
                {
                    minscore = s;
                    minscale = cur_scale;
                    minoff = i_off;
                    found = 1;
                }
                if( minoff == start_offset && i_off != start_offset )
                    break;
            }
        }

        if( !plane )
            while( mindenom > 0 && !(minscale & 1) )
            {
                mindenom--;
                minscale >>= 1;
            }

        if( !found || (minscale == 1 << mindenom && minoff == 0) || (float)minscore / origscore > 0.998f )
        {
            WP_SET( weights[plane], 0, 1, 0, 0 );
            continue;
        }
        WP_SET( weights[plane], 1, minscale, mindenom, minoff );
        if( weightp_fake && weights[0].weighted && !plane && cost_delta )
            *cost_delta = (float)minscore / origscore;
    }

    if( weights[1].weighted || weights[2].weighted )
    {
        int denom = weights[1].weighted ? weights[1].denom : weights[2].denom;
        const int both = weights[1].weighted && weights[2].weighted;
        while( (!both && denom == 7) ||
               (denom > 0 && !(weights[1].weighted && (weights[1].scale & 1)) &&
                !(weights[2].weighted && (weights[2].scale & 1))) )
        {
            denom--;
            for( int i = 1; i <= 2; i++ )
                if( weights[i].weighted )
                {
                    weights[i].scale >>= 1;
                    weights[i].denom = denom;
                }
        }
    }

    if( weights[0].weighted && b_lookahead && wlr )
        FN(weight_scale_plane)( wlr - 32 - 32 * lrs, lrs, ref_lr[0] - 32 - 32 * lrs, lrs, 8 * mbw + 64, 8 * mbh + 64,
                                weights[0].scale, weights[0].denom, weights[0].offset );
    free( mcl );
    free( mcu );
    free( mcv );
    free( fu );
    free( fv );
    free( mc444 );
}

/*============================================================================
 * SSIM — reference common/pixel.c:627-714
 *==========================================================================*/
void FN(ssim_4x4x2_core)( const pixel *pix1, intptr_t stride1, const pixel *pix2, intptr_t stride2, int sums[2][4] )
{
    for( int z = 0; z < 2; z++, pix1 += 4, pix2 += 4 )
    {
        uint32_t s1 = 0, s2 = 0, ss = 0, s12 = 0;
        for( int y = 0; y < 4; y++ )
            for( int x = 0; x < 4; x++ )
            {
                const int a = pix1[x + y * stride1], b = pix2[x + y * stride2];
                s1 += a;
                s2 += b;
                ss += a * a;
                ss += b * b;
                s12 += a * b;
            }
        sums[z][0] = s1;
        sums[z][1] = s2;
        sums[z][2] = ss;
        sums[z][3] = s12;
    }
}

/* ssim_end1: float arithmetic above 9 bits, int below (the reference's overflow note) */
static float ssim_end1( int s1, int s2, int ss, int s12 )
{
#if BIT_DEPTH > 9
    static const float c1 = .01 * .01 * PIXEL_MAX * PIXEL_MAX * 64;
    static const float c2 = .03 * .03 * PIXEL_MAX * PIXEL_MAX * 64 * 63;
    const float fs1 = s1, fs2 = s2, fss = ss, fs12 = s12;
    const float vars = fss * 64 - fs1 * fs1 - fs2 * fs2;
    const float covar = fs12 * 64 - fs1 * fs2;
    return (float)(2 * fs1 * fs2 + c1) * (float)(2 * covar + c2) / ((float)(fs1 * fs1 + fs2 * fs2 + c1) * (float)(vars + c2));
#else
    static const int c1 = (int)(.01 * .01 * PIXEL_MAX * PIXEL_MAX * 64 + .5);
    static const int c2 = (int)(.03 * .03 * PIXEL_MAX * PIXEL_MAX * 64 * 63 + .5);
    const int vars = ss * 64 - s1 * s1 - s2 * s2;
    const int covar = s12 * 64 - s1 * s2;
    return (float)(2 * s1 * s2 + c1) * (float)(2 * covar + c2) / ((float)(s1 * s1 + s2 * s2 + c1) * (float)(vars + c2));
#endif
}

float FN(ssim_end4)( int sum0[5][4], int sum1[5][4], int width )
{
    float ssim = 0.0;
    for( int i = 0; i < width; i++ )
        ssim += ssim_end1( sum0[i][0] + sum0[i + 1][0] + sum1[i][0] + sum1[i + 1][0],
                           sum0[i][1] + sum0[i + 1][1] + sum1[i][1] + sum1[i + 1][1],
                           sum0[i][2] + sum0[i + 1][2] + sum1[i][2] + sum1[i + 1][2],
                           sum0[i][3] + sum0[i + 1][3] + sum1[i][3] + sum1[i + 1][3] );
    return ssim;
}

/* x264_pixel_ssim_wxh: the two sum rows swap as the window row advances */
float FN(ssim_wxh)( const pixel *pix1, intptr_t stride1, const pixel *pix2, intptr_t stride2, int width, int height,
                    int *cnt )
{
    int z = 0;
    float ssim = 0.0;
    int (*buf)[4] = malloc( sizeof(int) * 4 * (2 * ((width >> 2) + 3)) );
    int (*sum0)[4] = buf, (*sum1)[4] = buf + (width >> 2) + 3;
    width >>= 2;
    height >>= 2;
    for( int y = 1; y < height; y++ )
    {
        for( ; z <= y; z++ )
        {
            int (*t)[4] = sum0;
            sum0 = sum1;
            sum1 = t;
            for( int x = 0; x < width; x += 2 )
                FN(ssim_4x4x2_core)( &pix1[4 * (x + z * stride1)], stride1, &pix2[4 * (x + z * stride2)], stride2,
                                     (int (*)[4])&sum0[x] );
        }
        for( int x = 0; x < width - 1; x += 4 )
            ssim += FN(ssim_end4)( sum0 + x, sum1 + x, width - x - 1 < 4 ? width - x - 1 : 4 );
    }
    *cnt = (height - 1) * (width - 1);
    free( buf );
    return ssim;
}
