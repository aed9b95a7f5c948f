/*****************************************************************************
 * cpubench.c — TEST INFRASTRUCTURE ONLY.  Multi-threaded drivers of the CPU
 * oracle, used by bench.py's cpu_baseline leg (kind "port": the reference's
 * C kernels restated in oracle.c, compiled -O3 -march=x86-64-v3).  Work is
 * split by macroblock rows, one contiguous band per thread, like the
 * per-row task split planned in BASELINE.md §3.
 *****************************************************************************/
#include <pthread.h>
#include <stdint.h>
#include <stddef.h>

void oracle8_me_search_full( const uint8_t *fenc, intptr_t fs, const uint8_t *ref, intptr_t rs,
                             int mb_width, int mb_height, int range, uint16_t *table );
void oracle8_mb_dct_quant( int transform, const uint8_t *fenc, intptr_t fs, const uint8_t *pred, intptr_t ps,
                           int mb_width, int mb_height, const uint16_t *mf, const uint16_t *bias,
                           int16_t *dct, int32_t *nz );

void oracle8_subpel_list( int op, int i_pixel, const uint8_t *fenc, intptr_t fs, const uint8_t *p0,
                          const uint8_t *p1, const uint8_t *p2, const uint8_t *p3, intptr_t rs,
                          const int64_t *fenc_off, const int32_t *qxy, int n, int32_t *scores );

typedef struct
{
    const uint8_t *fenc, *ref;
    intptr_t fs, rs;
    int mb_width, row0, rows, range, transform;
    const uint16_t *mf, *bias;
    uint16_t *table;
    int16_t *dct;
    int32_t *nz;
} job_t;

static void *me_worker( void *arg )
{
    job_t *j = arg;
    int w = 2 * j->range + 1;
    oracle8_me_search_full( j->fenc + (intptr_t)16 * j->row0 * j->fs, j->fs,
                            j->ref + (intptr_t)16 * j->row0 * j->rs, j->rs,
                            j->mb_width, j->rows, j->range,
                            j->table + (size_t)j->row0 * j->mb_width * w * w );
    return NULL;
}

static void *dq_worker( void *arg )
{
    job_t *j = arg;
    oracle8_mb_dct_quant( j->transform, j->fenc + (intptr_t)16 * j->row0 * j->fs, j->fs,
                          j->ref + (intptr_t)16 * j->row0 * j->rs, j->rs, j->mb_width, j->rows,
                          j->mf, j->bias, j->dct + (size_t)j->row0 * j->mb_width * 256,
                          j->nz + (size_t)j->row0 * j->mb_width );
    return NULL;
}

static int run( void *(*fn)( void * ), job_t base, int mb_height, int nthreads )
{
    pthread_t th[256];
    job_t jobs[256];
    if( nthreads < 1 )
        nthreads = 1;
    if( nthreads > 256 )
        nthreads = 256;
    if( nthreads > mb_height )
        nthreads = mb_height;
    int row = 0;
    for( int t = 0; t < nthreads; t++ )
    {
        int rows = mb_height / nthreads + (t < mb_height % nthreads);
        jobs[t] = base;
        jobs[t].row0 = row;
        jobs[t].rows = rows;
        row += rows;
        if( pthread_create( &th[t], NULL, fn, &jobs[t] ) )
            return -1;
    }
    for( int t = 0; t < nthreads; t++ )
        pthread_join( th[t], NULL );
    return nthreads;
}

/* more threads than MB rows (the all-CPU leg on a many-core host): each row is cut into
 * column segments and a thread takes a contiguous run of (row, segment) tasks; a segment's
 * table entries land where the whole-frame call puts them (one row's MBs are contiguous) */
typedef struct
{
    job_t b;
    int t0, t1, segs, mb_height;
} seg_job_t;

static void *me_seg_worker( void *arg )
{
    seg_job_t *j = arg;
    const int w = 2 * j->b.range + 1, W = j->b.mb_width;
    for( int t = j->t0; t < j->t1; t++ )
    {
        const int row = t / j->segs, seg = t % j->segs;
        const int c0 = W * seg / j->segs, c1 = W * (seg + 1) / j->segs;
        if( c1 > c0 )
            oracle8_me_search_full( j->b.fenc + (intptr_t)16 * row * j->b.fs + 16 * c0, j->b.fs,
                                    j->b.ref + (intptr_t)16 * row * j->b.rs + 16 * c0, j->b.rs, c1 - c0, 1,
                                    j->b.range, j->b.table + ((size_t)row * W + c0) * w * w );
    }
    return NULL;
}

/* full-search SAD tables of mb rows [0, mb_height), 8-bit; returns threads used */
int oracle8_me_search_full_mt( const uint8_t *fenc, intptr_t fs, const uint8_t *ref, intptr_t rs,
                               int mb_width, int mb_height, int range, uint16_t *table, int nthreads )
{
    job_t b = { fenc, ref, fs, rs, mb_width, 0, 0, range, 0, NULL, NULL, table, NULL, NULL };
    if( nthreads <= mb_height )
        return run( me_worker, b, mb_height, nthreads );
    if( nthreads > 256 )
        nthreads = 256;
    const int segs = (nthreads + mb_height - 1) / mb_height, tasks = segs * mb_height;
    pthread_t th[256];
    seg_job_t jobs[256];
    for( int t = 0; t < nthreads; t++ )
    {
        jobs[t].b = b;
        jobs[t].segs = segs;
        jobs[t].mb_height = mb_height;
        jobs[t].t0 = (int)((int64_t)tasks * t / nthreads);
        jobs[t].t1 = (int)((int64_t)tasks * (t + 1) / nthreads);
        if( pthread_create( &th[t], NULL, me_seg_worker, &jobs[t] ) )
            return -1;
    }
    for( int t = 0; t < nthreads; t++ )
        pthread_join( th[t], NULL );
    return nthreads;
}

/* fused dct+quant over mb rows [0, mb_height), 8-bit; returns threads used */
int oracle8_mb_dct_quant_mt( int transform, const uint8_t *fenc, intptr_t fs, const uint8_t *pred, intptr_t ps,
                             int mb_width, int mb_height, const uint16_t *mf, const uint16_t *bias,
                             int16_t *dct, int32_t *nz, int nthreads )
{
    job_t b = { fenc, pred, fs, ps, mb_width, 0, 0, 0, transform, mf, bias, NULL, dct, nz };
    return run( dq_worker, b, mb_height, nthreads );
}

typedef struct
{
    int op, i_pixel, n;
    const uint8_t *fenc, *p[4];
    intptr_t fs, rs;
    const int64_t *fenc_off;
    const int32_t *qxy;
    int32_t *scores;
} sp_job_t;

static void *sp_worker( void *arg )
{
    sp_job_t *j = arg;
    oracle8_subpel_list( j->op, j->i_pixel, j->fenc, j->fs, j->p[0], j->p[1], j->p[2], j->p[3], j->rs,
                         j->fenc_off, j->qxy, j->n, j->scores );
    return NULL;
}

/* qpel candidate list (get_ref + sad/satd), 8-bit, split into nthreads contiguous
 * slices; returns threads used */
int oracle8_subpel_list_mt( int op, int i_pixel, const uint8_t *fenc, intptr_t fs, const uint8_t *p0,
                            const uint8_t *p1, const uint8_t *p2, const uint8_t *p3, intptr_t rs,
                            const int64_t *fenc_off, const int32_t *qxy, int n, int32_t *scores, int nthreads )
{
    pthread_t th[256];
    sp_job_t jobs[256];
    if( nthreads < 1 )
        nthreads = 1;
    if( nthreads > 256 )
        nthreads = 256;
    if( nthreads > n )
        nthreads = n > 0 ? n : 1;
    int i0 = 0;
    for( int t = 0; t < nthreads; t++ )
    {
        int cnt = n / nthreads + (t < n % nthreads);
        sp_job_t j = { op, i_pixel, cnt, fenc, { p0, p1, p2, p3 }, fs, rs, fenc_off + i0, qxy + 2 * i0,
                       scores + i0 };
        jobs[t] = j;
        i0 += cnt;
        if( pthread_create( &th[t], NULL, sp_worker, &jobs[t] ) )
            return -1;
    }
    for( int t = 0; t < nthreads; t++ )
        pthread_join( th[t], NULL );
    return nthreads;
}

float oracle8_ssim_wxh( const uint8_t *pix1, intptr_t stride1, const uint8_t *pix2, intptr_t stride2, int width,
                        int height, int *cnt );

typedef struct
{
    const uint8_t *p1, *p2;
    intptr_t s1, s2;
    int width, b0, b1;
    const int32_t *bands;
    float *ssim;
    int32_t *cnt;
} ssim_job_t;

static void *ssim_worker( void *arg )
{
    ssim_job_t *j = arg;
    for( int b = j->b0; b < j->b1; b++ )
    {
        const int y = j->bands[2 * b], h = j->bands[2 * b + 1];
        int c = 0;
        j->ssim[b] = oracle8_ssim_wxh( j->p1 + (intptr_t)y * j->s1, j->s1, j->p2 + (intptr_t)y * j->s2, j->s2,
                                       j->width, h, &c );
        j->cnt[b] = c;
    }
    return NULL;
}

/* the encoder's SSIM bands (x264hip.ssim_encoder_bands: { y, h } pairs) of one frame pair, split
 * into nthreads contiguous runs of bands: one thread per run instead of one host task per band
 * (a band is ~17 us of work at 1080p, less than a thread-pool hand-off); returns threads used */
int oracle8_ssim_bands_mt( const uint8_t *pix1, intptr_t stride1, const uint8_t *pix2, intptr_t stride2, int width,
                           const int32_t *bands, int nbands, float *ssim, int32_t *cnt, int nthreads )
{
    pthread_t th[256];
    ssim_job_t jobs[256];
    if( nthreads < 1 )
        nthreads = 1;
    if( nthreads > 256 )
        nthreads = 256;
    if( nthreads > nbands )
        nthreads = nbands > 0 ? nbands : 1;
    for( int t = 0; t < nthreads; t++ )
    {
        ssim_job_t j = { pix1, pix2, stride1, stride2, width, (int)((int64_t)nbands * t / nthreads),
                         (int)((int64_t)nbands * (t + 1) / nthreads), bands, ssim, cnt };
        jobs[t] = j;
        if( pthread_create( &th[t], NULL, ssim_worker, &jobs[t] ) )
            return -1;
    }
    for( int t = 0; t < nthreads; t++ )
        pthread_join( th[t], NULL );
    return nthreads;
}
