/*****************************************************************************
 * me_bind_esa.c — TEST INFRASTRUCTURE.  A plain C99 host program that drives
 * the drop-in pixel table exactly as encoder/me.c's exhaustive integer search
 * does (me.c:618-631 window bounds and width rounding, the `#if 0` plain loop
 * of COST_MV over fpelcmp = sad, me.c:63-70, BITS_MVD of me.c:58-59), once per
 * macroblock of a frame pair, with the frame's full-search table bound
 * (x264hip_8_me_bind, lookup mode).  It writes the per-MB decisions
 * {bcost, bmx, bmy} and the timing of the search loop; the Python side
 * (tests/test_gpu_me_bind.py) compares the decisions with the oracle.
 *
 * input file (all little-endian): int64 header[12] = { magic 0x4d45424e44, W, H,
 *   stride, origin, mbw, mbh, R, me_range, c0, mb_step, bind }; then the fenc
 *   plane and the ref plane (uint8, (H+64)*stride each), the table
 *   (uint16, mbw*mbh*(2R+1)*pitch), par (int16[8] per MB: bmx, bmy, mvp x/y
 *   (qpel), mv_x_min, mv_y_min, mv_x_max, mv_y_max), init cost (int32 per MB),
 *   cost_mv (uint16[2*c0+1], mvd 0 at index c0).
 * output file: int32[3] per searched MB, then int64 { calls, hits, misses,
 *   loop_ns }.
 *****************************************************************************/
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "x264hip.h"

static void *slurp( FILE *f, size_t bytes )
{
    void *p = malloc( bytes ? bytes : 1 );
    if( !p || fread( p, 1, bytes, f ) != bytes )
    {
        fprintf( stderr, "me_bind_esa: short input\n" );
        exit( 3 );
    }
    return p;
}

static int64_t now_ns( void )
{
    struct timespec t;
    clock_gettime( CLOCK_MONOTONIC, &t );
    return (int64_t)t.tv_sec * 1000000000 + t.tv_nsec;
}

int main( int argc, char **argv )
{
    if( argc != 3 )
    {
        fprintf( stderr, "usage: me_bind_esa in.bin out.bin\n" );
        return 2;
    }
    FILE *f = fopen( argv[1], "rb" );
    if( !f )
        return 2;
    int64_t h[12];
    if( fread( h, sizeof(h), 1, f ) != 1 || h[0] != 0x4d45424e44 )
        return 3;
    const int W = (int)h[1], H = (int)h[2], mbw = (int)h[5], mbh = (int)h[6], R = (int)h[7];
    const int me_range = (int)h[8], step = (int)h[10], bind = (int)h[11];
    const intptr_t stride = (intptr_t)h[3], origin = (intptr_t)h[4], c0 = (intptr_t)h[9];
    const size_t plane = (size_t)(H + 64) * stride, pitch = (size_t)((2 * R + 1 + 3) & ~3);
    const size_t nmb = (size_t)mbw * mbh;
    uint8_t *fenc = slurp( f, plane ), *ref = slurp( f, plane );
    uint16_t *table = slurp( f, nmb * (2 * R + 1) * pitch * 2 );
    int16_t *par = slurp( f, nmb * 8 * 2 );
    int32_t *init = slurp( f, nmb * 4 );
    uint16_t *cost_mv = slurp( f, (size_t)(2 * c0 + 1) * 2 );
    fclose( f );
    (void)W;

    if( x264hip_init( 0 ) != X264HIP_OK )
    {
        fprintf( stderr, "no gfx950 device: %s\n", x264hip_last_error() );
        return 2;
    }
    x264hip_8_pixel_function_t pixf;
    memset( &pixf, 0, sizeof(pixf) );
    x264hip_8_pixel_init( X264HIP_CPU_HIP, &pixf );
    /* the encoder's alias (encoder.c:1423-1426): fpelcmp = sad unless TESA */
    int (*fpelcmp)( uint8_t *, intptr_t, uint8_t *, intptr_t ) = pixf.sad[X264HIP_PIXEL_16x16];
    const uint8_t *f0 = fenc + origin, *r0 = ref + origin;
    if( bind && x264hip_8_me_bind( f0, r0, stride, mbw, mbh, table, R ) != X264HIP_OK )
    {
        fprintf( stderr, "me_bind failed\n" );
        return 4;
    }
    x264hip_me_bind_stats( NULL, NULL, 1 );
    size_t nout = (nmb + step - 1) / step;
    int32_t *out = calloc( nout * 3, sizeof(int32_t) );
    int64_t calls = 0;
    uint8_t p_fenc[16 * X264HIP_FENC_STRIDE];
    const int64_t t0 = now_ns();
    size_t k = 0;
    for( size_t mb = 0; mb < nmb; mb += step, k++ )
    {
        const int mbx = (int)(mb % mbw), mby = (int)(mb / mbw);
        const int16_t *p = par + 8 * mb;
        /* mb.pic.p_fenc: the MB copied at FENC_STRIDE */
        for( int y = 0; y < 16; y++ )
            memcpy( p_fenc + y * X264HIP_FENC_STRIDE, f0 + (16 * mby + y) * stride + 16 * mbx, 16 );
        uint8_t *p_fref_w = (uint8_t *)r0 + 16 * mby * stride + 16 * mbx;
        const uint16_t *p_cost_mvx = cost_mv + c0 - p[2], *p_cost_mvy = cost_mv + c0 - p[3];
        int bmx = p[0], bmy = p[1], bcost = init[mb];
        /* me.c:618-626 */
        const int min_x = bmx - me_range > p[4] ? bmx - me_range : p[4];
        const int min_y = bmy - me_range > p[5] ? bmy - me_range : p[5];
        const int max_x = bmx + me_range < p[6] ? bmx + me_range : p[6];
        const int max_y = bmy + me_range < p[7] ? bmy + me_range : p[7];
        const int width = (max_x - min_x + 3) & ~3;
        /* me.c:627-631, COST_MV (me.c:63-70) */
        for( int my = min_y; my <= max_y; my++ )
            for( int mx = min_x; mx < min_x + width; mx++ )
            {
                int cost = fpelcmp( p_fenc, X264HIP_FENC_STRIDE, &p_fref_w[my * stride + mx], stride )
                         + p_cost_mvx[mx * 4] + p_cost_mvy[my * 4];
                calls++;
                if( cost < bcost )
                {
                    bcost = cost;
                    bmx = mx;
                    bmy = my;
                }
            }
        out[3 * k] = bcost;
        out[3 * k + 1] = bmx;
        out[3 * k + 2] = bmy;
    }
    const int64_t t1 = now_ns();
    uint64_t hits = 0, misses = 0;
    x264hip_me_bind_stats( &hits, &misses, 0 );
    x264hip_me_unbind();
    FILE *o = fopen( argv[2], "wb" );
    if( !o )
        return 2;
    int64_t tail[4] = { calls, (int64_t)hits, (int64_t)misses, t1 - t0 };
    fwrite( out, sizeof(int32_t), nout * 3, o );
    fwrite( tail, sizeof(tail), 1, o );
    fclose( o );
    printf( "me_bind_esa: %zu MBs, %lld calls, %llu hits, %llu misses, %.3f ms\n", nout, (long long)calls,
            (unsigned long long)hits, (unsigned long long)misses, (t1 - t0) / 1e6 );
    free( out );
    return 0;
}
