/*****************************************************************************
 * checkasm_hip.c — TEST INFRASTRUCTURE.  A plain C99 host program that uses
 * the backend exactly as x264 would after the INTEGRATION.md hook: it fills
 * the x264_*_function_t tables through x264hip_8_*_init( X264HIP_CPU_HIP ),
 * calls the entries with host pointers and the reference's implicit strides,
 * and compares every result with the oracle's C restatement (liboracle.so),
 * in the manner of the reference's tools/checkasm.c (random buffers, then
 * maxed-difference overflow patterns).  One batched device entry
 * (me_search_full) is driven through the HIP runtime API as a C caller would.
 *
 * build: gcc -std=c99 -O2 -I include -I /opt/rocm/include -D__HIP_PLATFORM_AMD__
 *        tests/c/checkasm_hip.c -L x264-i386pic_amd -lx264hip -L oracle -loracle
 *        -L /opt/rocm/lib -lamdhip64 -Wl,-rpath,...
 * prints one line per group and "checkasm_hip: all ok" on success (exit 0).
 *****************************************************************************/
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <hip/hip_runtime_api.h>

#include "x264hip.h"

/* oracle (BIT_DEPTH 8) entry points, see oracle/oracle.c */
int oracle8_sad( int, const uint8_t *, intptr_t, const uint8_t *, intptr_t );
int oracle8_ssd( int, const uint8_t *, intptr_t, const uint8_t *, intptr_t );
int oracle8_satd( int, const uint8_t *, intptr_t, const uint8_t *, intptr_t );
int oracle8_sa8d( int, const uint8_t *, intptr_t, const uint8_t *, intptr_t );
uint64_t oracle8_var( int, const uint8_t *, intptr_t );
uint64_t oracle8_hadamard_ac( int, const uint8_t *, intptr_t );
void oracle8_sad_x4( int, const uint8_t *, const uint8_t *, const uint8_t *, const uint8_t *, const uint8_t *,
                     intptr_t, int[4] );
void oracle8_sub4x4_dct( int16_t[16], const uint8_t *, const uint8_t * );
void oracle8_sub16x16_dct8( int16_t[4][64], const uint8_t *, const uint8_t * );
void oracle8_add16x16_idct( uint8_t *, int16_t[16][16] );
void oracle8_add16x16_idct8( uint8_t *, int16_t[4][64] );
int oracle8_quant_4x4( int16_t[16], const uint16_t[16], const uint16_t[16] );
void oracle8_dequant_4x4( int16_t[16], int[6][16], int );
int oracle8_cqm_init( const uint8_t *const[8], int, int, int, uint16_t *, uint16_t *, uint16_t *, uint16_t * );
void oracle8_zigzag_scan_8x8( int, int16_t[64], const int16_t[64] );
void oracle8_me_search_full( const uint8_t *, intptr_t, const uint8_t *, intptr_t, int, int, int, uint16_t * );

static uint32_t rng = 12345;
static uint32_t rnd( void ) { rng ^= rng << 13; rng ^= rng >> 17; rng ^= rng << 5; return rng; }

static int fails = 0;
#define CHECK( cond, ... ) do { if( !(cond) ) { fails++; fprintf( stderr, "FAIL: " __VA_ARGS__ ); fprintf( stderr, "\n" ); } } while( 0 )


int main( void )
{
    if( x264hip_init( 0 ) != X264HIP_OK )
    {
        fprintf( stderr, "no gfx950 device: %s\n", x264hip_last_error() );
        return 2;
    }
    static uint8_t buf1[64 * 64], buf2[64 * 64], buf3[32 * 32], buf4[32 * 32];
    for( int i = 0; i < 64 * 64; i++ )
    {
        buf1[i] = rnd() & 0xff;
        buf2[i] = rnd() & 0xff;
    }
    for( int i = 0; i < 32 * 32; i++ )   /* maxed differences (checkasm.c:368-382 style) */
    {
        buf4[i] = (rnd() & 1) ? 255 : 0;
        buf3[i] = 255 - buf4[i];
    }

    x264hip_8_pixel_function_t pf;
    memset( &pf, 0, sizeof(pf) );   /* stands for the caller's C init (the HIP init only overrides) */
    x264hip_8_pixel_init( X264HIP_CPU_HIP, &pf );
    for( int i = 0; i < 8; i++ )
        for( int j = 0; j < 16; j++ )
        {
            int s1 = (j & 7) == 7 ? 32 : 16;
            CHECK( pf.sad[i]( buf1, s1, buf2 + j, 64 ) == oracle8_sad( i, buf1, s1, buf2 + j, 64 ), "sad %d %d", i, j );
            CHECK( pf.ssd[i]( buf1, s1, buf2 + j, 64 ) == oracle8_ssd( i, buf1, s1, buf2 + j, 64 ), "ssd %d %d", i, j );
            CHECK( pf.satd[i]( buf1, s1, buf2 + j, 64 ) == oracle8_satd( i, buf1, s1, buf2 + j, 64 ), "satd %d", i );
            CHECK( pf.satd[i]( buf3, 16, buf4, 16 ) == oracle8_satd( i, buf3, 16, buf4, 16 ), "satd ovf %d", i );
        }
    for( int i = 0; i < 7; i++ )
    {
        int got[4], want[4];
        uint8_t *r = buf2 + 3;
        pf.sad_x4[i]( buf1, r, r + 6, r + 1, r + 10, 64, got );
        oracle8_sad_x4( i, buf1, r, r + 6, r + 1, r + 10, 64, want );
        CHECK( !memcmp( got, want, sizeof(got) ), "sad_x4 %d", i );
    }
    CHECK( pf.sa8d[0]( buf1, 16, buf2, 64 ) == oracle8_sa8d( 0, buf1, 16, buf2, 64 ), "sa8d 16x16" );
    CHECK( pf.sa8d[3]( buf3, 16, buf4, 16 ) == oracle8_sa8d( 3, buf3, 16, buf4, 16 ), "sa8d 8x8 ovf" );
    CHECK( pf.var[0]( buf1, 16 ) == oracle8_var( 0, buf1, 16 ), "var" );
    CHECK( pf.hadamard_ac[0]( buf1, 16 ) == oracle8_hadamard_ac( 0, buf1, 16 ), "hadamard_ac" );
    printf( "pixel: %s\n", fails ? "FAILED" : "ok" );

    /* dct / quant / dequant / idct with the implicit strides (dct.h:31-33) */
    int f0 = fails;
    x264hip_8_dct_function_t df;
    x264hip_8_quant_function_t qf;
    x264hip_8_zigzag_function_t zp, zi;
    memset( &df, 0, sizeof(df) );
    memset( &qf, 0, sizeof(qf) );
    memset( &zp, 0, sizeof(zp) );
    memset( &zi, 0, sizeof(zi) );
    x264hip_8_dct_init( X264HIP_CPU_HIP, &df );
    x264hip_8_quant_init( NULL, X264HIP_CPU_HIP, &qf );
    x264hip_8_zigzag_init( X264HIP_CPU_HIP, &zp, &zi );
    static uint8_t fenc[16 * 16], fdec[32 * 16];
    for( int i = 0; i < 16 * 16; i++ ) fenc[i] = rnd() & 0xff;
    for( int i = 0; i < 32 * 16; i++ ) fdec[i] = rnd() & 0xff;
    int16_t a4[16], b4[16];
    df.sub4x4_dct( a4, fenc, fdec );
    oracle8_sub4x4_dct( b4, fenc, fdec );
    CHECK( !memcmp( a4, b4, sizeof(a4) ), "sub4x4_dct" );
    static int16_t a8[4][64], b8[4][64];
    df.sub16x16_dct8( a8, fenc, fdec );
    oracle8_sub16x16_dct8( b8, fenc, fdec );
    CHECK( !memcmp( a8, b8, sizeof(a8) ), "sub16x16_dct8" );

    uint8_t flat[64];
    memset( flat, 16, sizeof(flat) );
    const uint8_t *sl[8] = { flat, flat, flat, flat, flat, flat, flat, flat };
    static uint16_t q4m[4][52][16], q4b[4][52][16], q8m[4][52][64], q8b[4][52][64];
    static uint16_t o4m[4][52][16], o4b[4][52][16], o8m[4][52][64], o8b[4][52][64];
    x264hip_8_cqm_init( sl, 21, 11, 1, &q4m[0][0][0], &q4b[0][0][0], &q8m[0][0][0], &q8b[0][0][0] );
    oracle8_cqm_init( sl, 21, 11, 1, &o4m[0][0][0], &o4b[0][0][0], &o8m[0][0][0], &o8b[0][0][0] );
    CHECK( !memcmp( q4m, o4m, sizeof(q4m) ) && !memcmp( q8b, o8b, sizeof(q8b) ), "cqm_init" );
    static int32_t dq4[4][6][16], dq8[2][6][64];
    x264hip_cqm_dequant( sl, 1, &dq4[0][0][0], &dq8[0][0][0] );
    for( int qp = 0; qp <= 51; qp += 3 )
    {
        int16_t x[16], y[16];
        df.sub4x4_dct( x, fenc, fdec );
        memcpy( y, x, sizeof(x) );
        CHECK( qf.quant_4x4( x, q4m[1][qp], q4b[1][qp] ) == oracle8_quant_4x4( y, o4m[1][qp], o4b[1][qp] ), "quant nz" );
        CHECK( !memcmp( x, y, sizeof(x) ), "quant_4x4 qp %d", qp );
        qf.dequant_4x4( x, dq4[1], qp );
        oracle8_dequant_4x4( y, dq4[1], qp );
        CHECK( !memcmp( x, y, sizeof(x) ), "dequant_4x4 qp %d", qp );
    }
    static int16_t c16[16][16], c16b[16][16];
    for( int i = 0; i < 256; i++ ) c16[i / 16][i % 16] = c16b[i / 16][i % 16] = (int16_t)((rnd() % 801) - 400);
    static uint8_t d1[32 * 16], d2[32 * 16];
    memcpy( d1, fdec, sizeof(d1) );
    memcpy( d2, fdec, sizeof(d2) );
    df.add16x16_idct( d1, c16 );
    oracle8_add16x16_idct( d2, c16b );
    CHECK( !memcmp( d1, d2, sizeof(d1) ), "add16x16_idct" );
    static int16_t e8[4][64], e8b[4][64];
    for( int i = 0; i < 256; i++ ) e8[i / 64][i % 64] = e8b[i / 64][i % 64] = (int16_t)((rnd() % 2001) - 1000);
    df.add16x16_idct8( d1, e8 );
    oracle8_add16x16_idct8( d2, e8b );
    CHECK( !memcmp( d1, d2, sizeof(d1) ), "add16x16_idct8" );
    int16_t lv[64], lw[64];
    zi.scan_8x8( lv, e8[1] );
    oracle8_zigzag_scan_8x8( 1, lw, e8[1] );
    CHECK( !memcmp( lv, lw, sizeof(lv) ), "zigzag_scan_8x8 field" );
    printf( "dct/quant/zigzag: %s\n", fails > f0 ? "FAILED" : "ok" );

    /* batched full search on device memory, as an encoder's frame loop would call it */
    f0 = fails;
    enum { MBW = 6, MBH = 4, R = 8, PAD = 32, W = MBW * 16, H = MBH * 16, STRIDE = 192 };
    size_t plane = (size_t)(H + 2 * PAD) * STRIDE;
    uint8_t *hf = malloc( plane ), *hr = malloc( plane );
    for( size_t i = 0; i < plane; i++ ) { hf[i] = rnd() & 0xff; hr[i] = rnd() & 0xff; }
    const int pitch = (2 * R + 1 + 3) / 4 * 4, nt = MBW * MBH * (2 * R + 1);
    uint16_t *ht = malloc( (size_t)nt * pitch * 2 ), *wt = malloc( (size_t)nt * (2 * R + 1) * 2 );
    void *df_, *dr_, *dt_;
    if( hipMalloc( &df_, plane ) || hipMalloc( &dr_, plane ) || hipMalloc( &dt_, (size_t)nt * pitch * 2 ) )
        return 3;
    hipMemcpy( df_, hf, plane, hipMemcpyHostToDevice );
    hipMemcpy( dr_, hr, plane, hipMemcpyHostToDevice );
    const size_t org = (size_t)PAD * STRIDE + PAD;
    int rc = x264hip_8_me_search_full( (uint8_t *)df_ + org, STRIDE, 0, (uint8_t *)dr_ + org, STRIDE, 0, MBW, MBH, 1,
                                       R, (uint16_t *)dt_, NULL );
    CHECK( rc == X264HIP_OK, "me_search_full rc %d", rc );
    hipDeviceSynchronize();
    hipMemcpy( ht, dt_, (size_t)nt * pitch * 2, hipMemcpyDeviceToHost );
    oracle8_me_search_full( hf + org, STRIDE, hr + org, STRIDE, MBW, MBH, R, wt );
    for( int i = 0; i < nt; i++ )
        CHECK( !memcmp( ht + (size_t)i * pitch, wt + (size_t)i * (2 * R + 1), (2 * R + 1) * 2 ), "table row %d", i );
    CHECK( x264hip_8_me_search_full( NULL, 0, 0, NULL, 0, 0, 1, 1, 1, 5, NULL, NULL ) == X264HIP_EINVAL, "bad range" );
    hipFree( df_ ); hipFree( dr_ ); hipFree( dt_ );
    free( hf ); free( hr ); free( ht ); free( wt );
    printf( "batched me_search_full: %s\n", fails > f0 ? "FAILED" : "ok" );

    if( fails )
    {
        printf( "checkasm_hip: %d failures\n", fails );
        return 1;
    }
    printf( "checkasm_hip: all ok\n" );
    return 0;
}
