// C ABI of the gfx950 backend: runtime, drop-in table initialisers, per-call
// table entries and the batched device entries.  See include/x264hip.h.
//
// Per-call table entries keep the reference's synchronous, host-pointer
// contract (reference common/pixel.h:31-35, dct.h:29-59, quant.h:30-36): the
// caller's block is staged into a per-thread pinned buffer, ONE kernel of the
// batched path runs on it (zero-copy reads over the host link) and the
// result is read back after a stream synchronise.  No metric, transform or
// quantisation is ever computed on the host here: if the GPU call fails the
// process aborts with the HIP error (there is no CPU fallback).
#include "hipcommon.h"
#include "x264hip.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <atomic>
#include <mutex>

using namespace x264hip;

// ============================================================ runtime
// The process device (x264hip_init) and an optional per-thread override
// (x264hip_set_thread_device): x264's frame / lookahead threads may each bind a
// different GPU of the node.  Per-call table entries run on the calling
// thread's device, on a stream and pinned staging buffer owned by that thread.
static std::atomic<int> g_device{ -1 };
static std::mutex g_init_mutex;
static thread_local int t_device = -1;
static thread_local char t_err[256] = "";

static int map_err( hipError_t e, const char *where );
static int set_err( hipError_t e, const char *where )
{
    snprintf( t_err, sizeof(t_err), "%s: %s", where, hipGetErrorString( e ) );
    return X264HIP_EDEVICE;
}

extern "C" const char *x264hip_last_error( void ) { return t_err; }

// 0 if `device` is a usable gfx950 device, else an X264HIP_E* code (t_err set)
static int check_device( int device )
{
    int n = 0;
    if( hipGetDeviceCount( &n ) != hipSuccess || n <= 0 )
    {
        snprintf( t_err, sizeof(t_err), "x264hip: no HIP device" );
        return X264HIP_ENODEV;
    }
    if( device < 0 || device >= n )
    {
        snprintf( t_err, sizeof(t_err), "x264hip: device %d out of range (%d devices)", device, n );
        return X264HIP_EINVAL;
    }
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties( &prop, device );
    if( e != hipSuccess )
        return set_err( e, "hipGetDeviceProperties" );
    if( strncmp( prop.gcnArchName, "gfx950", 6 ) )
    {
        snprintf( t_err, sizeof(t_err), "x264hip: device %d is %s, not gfx950", device, prop.gcnArchName );
        return X264HIP_ENODEV;
    }
    return X264HIP_OK;
}

extern "C" int x264hip_init( int device )
{
    std::lock_guard<std::mutex> lk( g_init_mutex );
    int rc = check_device( device );
    if( rc != X264HIP_OK )
        return rc;
    hipError_t e = hipSetDevice( device );
    if( e != hipSuccess )
        return set_err( e, "hipSetDevice" );
    g_device.store( device, std::memory_order_release );
    return X264HIP_OK;
}

extern "C" int x264hip_available( void )
{
    // a thread bound with x264hip_set_thread_device already has its device: the
    // implicit init below would hipSetDevice(0) over that binding
    if( t_device >= 0 || g_device.load( std::memory_order_acquire ) >= 0 )
        return 1;
    // initialise on the caller's current device (device 0 when it has none), so the device
    // x264hip_thread_device() reports is the one the entries run on and the caller's
    // current device is left as it was
    int cur = -1;
    if( hipGetDevice( &cur ) != hipSuccess || cur < 0 )
        cur = 0;
    return x264hip_init( cur ) == X264HIP_OK;
}

extern "C" int x264hip_set_thread_device( int device )
{
    if( device < 0 )
    {
        t_device = -1;
        return X264HIP_OK;
    }
    int rc = check_device( device );
    if( rc != X264HIP_OK )
        return rc;
    hipError_t e = hipSetDevice( device );
    if( e != hipSuccess )
        return set_err( e, "hipSetDevice" );
    t_device = device;
    return X264HIP_OK;
}

extern "C" int x264hip_thread_device( void )
{
    return t_device >= 0 ? t_device : g_device.load( std::memory_order_acquire );
}

// reconstructed-reference forward between the GPUs of a frame-per-GPU pipeline
// (SURVEY.md §8e): one xGMI peer copy on `stream`, asynchronous
extern "C" int x264hip_forward_ref( void *dst, int dst_device, const void *src, int src_device, size_t bytes,
                                    void *stream )
{
    if( bytes == 0 )
        return X264HIP_OK;
    if( !dst || !src || dst_device < 0 || src_device < 0 )
        return X264HIP_EINVAL;
    hipError_t e = hipMemcpyPeerAsync( dst, dst_device, src, src_device, bytes, (hipStream_t)stream );
    if( e == hipErrorInvalidValue )
    {
        snprintf( t_err, sizeof(t_err), "x264hip_forward_ref: invalid argument" );
        return X264HIP_EINVAL;
    }
    return e == hipSuccess ? X264HIP_OK : set_err( e, "hipMemcpyPeerAsync" );
}

// frame upload from page-locked host memory by a kernel reading the pinned pages
// (configs[3]'s streaming form; asynchronous on `stream`)
extern "C" int x264hip_upload( void *dst, const void *host_src, size_t bytes, void *stream )
{
    if( bytes == 0 )
        return X264HIP_OK;
    if( !dst || !host_src )
        return X264HIP_EINVAL;
    // the kernel reads the pages through their device address, which for memory
    // registered with hipHostRegister need not equal the host address; a pageable
    // range has none (XNACK is off) and is refused instead of faulting the GPU.  Both
    // ends of the range must resolve into one contiguous mapping.
    void *d0 = nullptr, *d1 = nullptr;
    if( hipHostGetDevicePointer( &d0, (void *)host_src, 0 ) != hipSuccess || !d0 ||
        hipHostGetDevicePointer( &d1, (void *)((const uint8_t *)host_src + bytes - 1), 0 ) != hipSuccess ||
        (uint8_t *)d1 != (uint8_t *)d0 + bytes - 1 )
    {
        (void)hipGetLastError();
        snprintf( t_err, sizeof(t_err), "x264hip_upload: source is not page-locked host memory" );
        return X264HIP_EINVAL;
    }
    hipError_t e = launch_upload( dst, d0, bytes, (hipStream_t)stream );
    return e == hipSuccess ? X264HIP_OK : set_err( e, "upload" );
}

// picture planes from page-locked host memory into padded planes, borders expanded
static bool pinned_range( const void *p, size_t bytes, const void **dev )
{
    void *d0 = nullptr, *d1 = nullptr;
    if( hipHostGetDevicePointer( &d0, (void *)p, 0 ) != hipSuccess || !d0 ||
        hipHostGetDevicePointer( &d1, (void *)((const uint8_t *)p + bytes - 1), 0 ) != hipSuccess ||
        (uint8_t *)d1 != (uint8_t *)d0 + bytes - 1 )
    {
        (void)hipGetLastError();
        return false;
    }
    *dev = d0;
    return true;
}

extern "C" int x264hip_upload_planes( int n, const x264hip_plane_upload_t *pl, void *stream )
{
    if( n < 1 || n > 3 || !pl )
        return X264HIP_EINVAL;
    UploadPlane q[3];
    for( int k = 0; k < n; k++ )
    {
        const x264hip_plane_upload_t &u = pl[k];
        if( !u.dst || !u.host_src || u.width_bytes <= 0 || u.height <= 0 || u.src_stride < u.width_bytes ||
            u.dst_stride < u.width_bytes + 2 * (intptr_t)u.pad_x )
            return X264HIP_EINVAL;
        const void *d = nullptr;
        if( !pinned_range( u.host_src, (size_t)u.src_stride * (u.height - 1) + u.width_bytes, &d ) )
        {
            snprintf( t_err, sizeof(t_err), "x264hip_upload_planes: source is not page-locked host memory" );
            return X264HIP_EINVAL;
        }
        q[k] = { u.dst, d, u.dst_stride, u.src_stride, u.width_bytes, u.height, u.unit, u.pad_x, u.pad_y };
    }
    hipError_t e = launch_upload_planes( n, q, (hipStream_t)stream );
    return e == hipSuccess ? X264HIP_OK : set_err( e, "upload_planes" );
}

extern "C" int x264hip_upload_plane( void *dst, intptr_t dst_stride, const void *host_src, intptr_t src_stride,
                                     int width_bytes, int height, int unit, int pad_x, int pad_y, void *stream )
{
    if( width_bytes <= 0 || height <= 0 )
        return X264HIP_OK;
    const x264hip_plane_upload_t u = { dst, dst_stride, host_src, src_stride, width_bytes, height, unit, pad_x, pad_y };
    return x264hip_upload_planes( 1, &u, stream );
}

// Two streams on complementary CU sets of the current device (hipExtStreamCreateWithCUMask):
// `copy` on the first `reserve_cus` CUs, `compute` on the rest.  The frame-streaming
// pipeline of configs[3] runs the PCIe-read upload of frame n+1 on `copy` while frame n's
// search runs on `compute`: without the split the upload's workgroups wait for CU slots the
// full-search kernel holds (0.188 vs 0.169 ms per 2160p frame, profiles/r03b_stream_probe.json).
extern "C" int x264hip_stream_pair_create( int reserve_cus, void **compute, void **copy )
{
    if( !compute || !copy || reserve_cus < 1 )
        return X264HIP_EINVAL;
    int dev = 0;
    hipError_t e = hipGetDevice( &dev );
    hipDeviceProp_t prop;
    if( e == hipSuccess )
        e = hipGetDeviceProperties( &prop, dev );
    if( e != hipSuccess )
        return set_err( e, "stream_pair_create" );
    const int ncu = prop.multiProcessorCount;
    if( reserve_cus >= ncu || ncu > 1024 )
        return X264HIP_EINVAL;
    uint32_t a[32] = { 0 }, b[32] = { 0 };
    const int nw = (ncu + 31) / 32;
    for( int i = 0; i < ncu; i++ )
        (i < reserve_cus ? b : a)[i >> 5] |= 1u << (i & 31);
    hipStream_t sc = nullptr, sk = nullptr;
    e = hipExtStreamCreateWithCUMask( &sc, (uint32_t)nw, a );
    if( e == hipSuccess )
        e = hipExtStreamCreateWithCUMask( &sk, (uint32_t)nw, b );
    if( e != hipSuccess )
    {
        if( sc )
            (void)hipStreamDestroy( sc );
        return set_err( e, "hipExtStreamCreateWithCUMask" );
    }
    *compute = sc;
    *copy = sk;
    return X264HIP_OK;
}

extern "C" int x264hip_stream_destroy( void *stream )
{
    if( !stream )
        return X264HIP_OK;
    hipError_t e = hipStreamDestroy( (hipStream_t)stream );
    return e == hipSuccess ? X264HIP_OK : set_err( e, "hipStreamDestroy" );
}

// release the idle blocks of the library's scratch pools (the self-contained TESA's tables)
// on `device`, or on every device for device < 0; the pools otherwise keep their peak
extern "C" int x264hip_trim( int device )
{
    hipError_t e = scratch_trim( device );
    return e == hipSuccess ? X264HIP_OK : set_err( e, "x264hip_trim" );
}

// the lookahead wavefront's status (lookahead.hip lowres_status): waits for `stream`
extern "C" int x264hip_lowres_status( void *stream )
{
    return map_err( lowres_status( (hipStream_t)stream ), "lowres_status" );
}

// row pitch (entries) of a me_search_full (centred = 0) or me_search_centred (centred = 1)
// table, or 0 for an unsupported bit depth / range
extern "C" int x264hip_me_table_pitch( int bitdepth, int range, int centred )
{
    if( (bitdepth != 8 && bitdepth != 10) || range < 1 || range > 29 )
        return 0;
    return centred ? cen_pitch( bitdepth, range ) : full_pitch( range );
}

[[noreturn]] static void fatal( hipError_t e, const char *where )
{
    fprintf( stderr, "x264hip: fatal HIP error in %s: %s\n", where, hipGetErrorString( e ) );
    abort();
}

#define CHECK_FATAL( call )                      \
    do {                                         \
        hipError_t e_ = ( call );                \
        if( e_ != hipSuccess )                   \
            fatal( e_, #call );                  \
    } while( 0 )

// ------------------------------------------------------------ kernel variants
namespace x264hip {
static const char *const k_variant_env[V_COUNT] = {
    "X264HIP_TESA_VARIANT", "X264HIP_INTEGRAL_VARIANT", "X264HIP_LA_POLL", "X264HIP_UPLOAD_WGS", "X264HIP_ME_XCD",
    "X264HIP_STREAM_XCD", "X264HIP_STREAM_NT", "X264HIP_LA_HELPER", "X264HIP_LA_XCD" };

struct VariantTable
{
    std::atomic<int> v[V_COUNT];
    VariantTable()
    {
        for( int i = 0; i < V_COUNT; i++ )
        {
            const char *e = getenv( k_variant_env[i] );
            v[i].store( e && *e ? atoi( e ) : -1, std::memory_order_relaxed );
        }
    }
};
static VariantTable &variants()
{
    static VariantTable t;   // seeded from the environment once, at first use
    return t;
}
int variant( VariantSlot slot ) { return variants().v[slot].load( std::memory_order_relaxed ); }
} // namespace x264hip

extern "C" int x264hip_set_variant( const char *name, int value )
{
    for( int i = 0; i < V_COUNT; i++ )
        if( name && !strcmp( name, k_variant_env[i] ) )
        {
            variants().v[i].store( value < 0 ? -1 : value, std::memory_order_relaxed );
            return X264HIP_OK;
        }
    return X264HIP_EINVAL;
}

// per-thread stream + pinned staging buffer for the per-call table entries
namespace {
struct CallCtx
{
    int device = -1;
    hipStream_t stream = nullptr;
    uint8_t *host = nullptr;   // host view
    uint8_t *dev = nullptr;    // device view of the same pinned memory
    static constexpr size_t SIZE = 64 << 10;
    void release()
    {
        // errors ignored: at process teardown the runtime may already be gone
        if( stream )
            (void)hipStreamDestroy( stream );
        if( host )
            (void)hipHostFree( host );
        stream = nullptr;
        host = dev = nullptr;
        device = -1;
    }
    ~CallCtx() { release(); }
};
thread_local CallCtx t_call;

// Entries are installed only when x264hip_available() held (see the initialisers
// below), so a device is always bound here; the thread's override wins.
CallCtx &call_ctx()
{
    const int dev = x264hip_thread_device();
    if( dev < 0 )
    {
        fprintf( stderr, "x264hip: table entry called before x264hip_init\n" );
        abort();
    }
    if( t_call.stream && t_call.device != dev )
        t_call.release();
    if( !t_call.stream )
    {
        CHECK_FATAL( hipSetDevice( dev ) );
        CHECK_FATAL( hipStreamCreateWithFlags( &t_call.stream, hipStreamNonBlocking ) );
        CHECK_FATAL( hipHostMalloc( (void **)&t_call.host, CallCtx::SIZE, hipHostMallocDefault ) );
        CHECK_FATAL( hipHostGetDevicePointer( (void **)&t_call.dev, t_call.host, 0 ) );
        t_call.device = dev;
    }
    return t_call;
}

// device view of a pointer into the staging buffer
template <typename T> T *dview( CallCtx &c, T *h ) { return (T *)(c.dev + ((uint8_t *)h - c.host)); }

// staging layout (bytes): [0,8K) block A, [8K,24K) blocks B, [24K,25K) offsets, [25K,26K) scores,
// [26K,60K) coefficients / mf / bias
constexpr size_t ST_A = 0, ST_B = 8 << 10, ST_OFF = 24 << 10, ST_SC = 25 << 10, ST_COEF = 26 << 10;

template <typename P>
void stage_block( P *dst, const P *src, intptr_t stride, int w, int h )
{
    for( int y = 0; y < h; y++ )
        memcpy( dst + y * w, src + y * stride, w * sizeof(P) );
}
} // namespace

// ============================================================ table lookup mode
// x264hip_{8,10}_me_bind: the calling thread registers one frame's full-search result
// (host copies of the fenc and ref luma planes and of the me_search_full table).  While
// bound, a 16x16 SAD entry (sad / fpelcmp / sad_x3 / sad_x4) whose candidate pointer
// lies inside the bound ref plane at a full-pel mv the table holds answers from the
// table on the host, without a dispatch (reference encoder/me.c:63-70 COST_MV over
// fpelcmp, encoder.c:1409-1427 aliases; me.c's fenc is mb.pic.p_fenc, a copy of the
// MB at FENC_STRIDE).  The MB being searched is not passed to the entry: it is the one
// of the <= 9 MBs whose window covers the candidate's offset whose pixels equal the
// caller's fenc block (MBs with equal pixels have equal SADs, so any match is exact).
// Anything else -- another plane, a stride mismatch, a window column outside the
// table, a field MB -- takes the dispatch path, so results never change.
namespace {
struct MeBind
{
    int bd = 0;                          // 0: nothing bound
    const uint8_t *fenc = nullptr;       // pixel (0, 0) of the bound planes
    const uint8_t *ref = nullptr;
    intptr_t stride = 0;                 // pixels
    int mbw = 0, mbh = 0, R = 0, pitch = 0, psz = 1;
    const void *table = nullptr;         // [mbh][mbw][2R+1][pitch] 16x16 SADs (or null)
    const uint16_t *table8 = nullptr;    // [mbh][mbw][4][2R+1][pitch] 8x8 quadrant SADs (or null)
    uint64_t hits = 0, misses = 0;
};
thread_local MeBind t_bind;
constexpr int BIND_PAD = 32;             // x264 PADH / PADV (frame.h:32-33)

// SAD of the 16x16 candidate at `cand` (stride s) for the MB whose pixels equal
// `fenc` (stride fs), from the bound table; false = not answerable here
template <int BD>
inline bool bind_lookup16( const typename PT<BD>::pixel *fenc, intptr_t fs, const typename PT<BD>::pixel *cand,
                           intptr_t s, int *out )
{
    using pixel = typename PT<BD>::pixel;
    const MeBind &b = t_bind;
    if( b.bd != BD || s != b.stride )
        return false;
    const intptr_t d = (const pixel *)cand - (const pixel *)b.ref;
    // pixel (x, y), x in [-PAD, stride - PAD): the padded rows hold stride pixels
    intptr_t y = (d + BIND_PAD) >= 0 ? (d + BIND_PAD) / s : -((-(d + BIND_PAD) + s - 1) / s);
    const intptr_t x = d - y * s;
    const int R = b.R;
    if( y < -R || y > 16 * (intptr_t)(b.mbh - 1) + R || x < -R || x > 16 * (intptr_t)(b.mbw - 1) + R )
        return false;
    const int mx0 = (int)std::max<intptr_t>( 0, (x - R + 15) >> 4 ), mx1 = (int)std::min<intptr_t>( b.mbw - 1, (x + R) >> 4 );
    const int my0 = (int)std::max<intptr_t>( 0, (y - R + 15) >> 4 ), my1 = (int)std::min<intptr_t>( b.mbh - 1, (y + R) >> 4 );
    const pixel *fp = (const pixel *)b.fenc;
    for( int my = my0; my <= my1; my++ )
        for( int mx = mx0; mx <= mx1; mx++ )
        {
            const pixel *m = fp + (intptr_t)16 * my * s + 16 * mx;
            int r = 0;
            while( r < 16 && !memcmp( fenc + r * fs, m + r * s, 16 * sizeof(pixel) ) )
                r++;
            if( r < 16 )
                continue;
            const int tx = (int)(x - 16 * mx) + R, ty = (int)(y - 16 * my) + R;
            if( b.table )
            {
                const size_t i = (((size_t)my * b.mbw + mx) * (2 * R + 1) + ty) * b.pitch + tx;
                *out = (int)((const typename PT<BD>::sadt *)b.table)[i];
            }
            else
            {
                const size_t q0 = (((size_t)my * b.mbw + mx) * 4 * (2 * R + 1) + ty) * b.pitch + tx;
                const size_t qs = (size_t)(2 * R + 1) * b.pitch;
                *out = b.table8[q0] + b.table8[q0 + qs] + b.table8[q0 + 2 * qs] + b.table8[q0 + 3 * qs];
            }
            return true;
        }
    return false;
}

// PIXEL_16x8 / 8x16 / 8x8 from the quadrant tables: the partition (W x H at (px, py) in its
// MB) is the one whose pixels equal the caller's fenc block, among the partitions of that size
// of the <= 9 MBs whose window covers the candidate; its SAD is the sum of its quadrants
template <int BD, int W, int H>
inline bool bind_lookup_part( const typename PT<BD>::pixel *fenc, intptr_t fs, const typename PT<BD>::pixel *cand,
                              intptr_t s, int *out )
{
    using pixel = typename PT<BD>::pixel;
    const MeBind &b = t_bind;
    if( b.bd != BD || !b.table8 || s != b.stride )
        return false;
    const intptr_t d = cand - (const pixel *)b.ref;
    const intptr_t y = (d + BIND_PAD) >= 0 ? (d + BIND_PAD) / s : -((-(d + BIND_PAD) + s - 1) / s);
    const intptr_t x = d - y * s;
    const int R = b.R;
    const size_t qs = (size_t)(2 * R + 1) * b.pitch;
    for( int py = 0; py < 16; py += H )
        for( int px = 0; px < 16; px += W )
        {
            const intptr_t xx = x - px, yy = y - py;     // the MB-aligned candidate position
            if( yy < -R || yy > 16 * (intptr_t)(b.mbh - 1) + R || xx < -R || xx > 16 * (intptr_t)(b.mbw - 1) + R )
                continue;
            const int mx0 = (int)std::max<intptr_t>( 0, (xx - R + 15) >> 4 );
            const int mx1 = (int)std::min<intptr_t>( b.mbw - 1, (xx + R) >> 4 );
            const int my0 = (int)std::max<intptr_t>( 0, (yy - R + 15) >> 4 );
            const int my1 = (int)std::min<intptr_t>( b.mbh - 1, (yy + R) >> 4 );
            for( int my = my0; my <= my1; my++ )
                for( int mx = mx0; mx <= mx1; mx++ )
                {
                    const pixel *m = (const pixel *)b.fenc + (intptr_t)(16 * my + py) * s + 16 * mx + px;
                    int r = 0;
                    while( r < H && !memcmp( fenc + r * fs, m + r * s, W * sizeof( pixel ) ) )
                        r++;
                    if( r < H )
                        continue;
                    const int tx = (int)(xx - 16 * mx) + R, ty = (int)(yy - 16 * my) + R;
                    const uint16_t *t = b.table8 + (((size_t)my * b.mbw + mx) * 4 * (2 * R + 1) + ty) * b.pitch + tx;
                    const int q = (py >> 3) * 2 + (px >> 3);     // the partition's first quadrant
                    int v = t[q * qs];
                    if( W == 16 )
                        v += t[(q + 1) * qs];
                    if( H == 16 )
                        v += t[(q + 2) * qs];
                    *out = v;
                    return true;
                }
        }
    return false;
}
} // namespace

#define DEFINE_BIND( BD )                                                                                            \
    extern "C" int x264hip_##BD##_me_bind_tables( const PT<BD>::pixel *fenc, const PT<BD>::pixel *ref,              \
                                                  intptr_t stride, int mb_width, int mb_height,                      \
                                                  const PT<BD>::sadt *table, const uint16_t *table8, int range )     \
    {                                                                                                                \
        if( !fenc || !ref || !( table || table8 ) || mb_width <= 0 || mb_height <= 0 ||                            \
            range < 1 || range > 29 || stride < 16 * (intptr_t)mb_width + 2 * BIND_PAD )                             \
            return X264HIP_EINVAL;                                                                                   \
        MeBind &b = t_bind;                                                                                          \
        b.table8 = table8;                                                                                           \
        b.bd = BD;                                                                                                   \
        b.fenc = (const uint8_t *)fenc;                                                                              \
        b.ref = (const uint8_t *)ref;                                                                                \
        b.stride = stride;                                                                                           \
        b.mbw = mb_width;                                                                                            \
        b.mbh = mb_height;                                                                                           \
        b.R = range;                                                                                                 \
        b.pitch = (2 * range + 1 + 3) & ~3;                                                                          \
        b.table = table;                                                                                             \
        return X264HIP_OK;                                                                                           \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_me_bind( const PT<BD>::pixel *fenc, const PT<BD>::pixel *ref, intptr_t stride,     \
                                           int mb_width, int mb_height, const PT<BD>::sadt *table, int range )       \
    {                                                                                                                \
        if( !table )                                                                                                 \
            return X264HIP_EINVAL;                                                                                   \
        return x264hip_##BD##_me_bind_tables( fenc, ref, stride, mb_width, mb_height, table, nullptr, range );      \
    }
DEFINE_BIND( 8 )
DEFINE_BIND( 10 )
#undef DEFINE_BIND

extern "C" void x264hip_me_unbind( void )
{
    const uint64_t h = t_bind.hits, m = t_bind.misses;
    t_bind = MeBind();
    t_bind.hits = h;
    t_bind.misses = m;
}

extern "C" void x264hip_me_bind_stats( uint64_t *hits, uint64_t *misses, int reset )
{
    if( hits )
        *hits = t_bind.hits;
    if( misses )
        *misses = t_bind.misses;
    if( reset )
        t_bind.hits = t_bind.misses = 0;
}

// ============================================================ per-call pixel entries
template <int BD, int OP, int IPIX>
static int cmp_call( typename PT<BD>::pixel *p1, intptr_t s1, typename PT<BD>::pixel *p2, intptr_t s2 )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int W = pix_w( IPIX ), H = pix_h( IPIX );
    if constexpr( OP == X264HIP_CMP_SAD && IPIX == X264HIP_PIXEL_16x16 )
    {
        if( t_bind.bd )
        {
            int v;
            if( bind_lookup16<BD>( p1, s1, p2, s2, &v ) )
            {
                t_bind.hits++;
                return v;
            }
            t_bind.misses++;
        }
    }
    if constexpr( OP == X264HIP_CMP_SAD &&
                  ( IPIX == X264HIP_PIXEL_16x8 || IPIX == X264HIP_PIXEL_8x16 || IPIX == X264HIP_PIXEL_8x8 ) )
    {
        if( t_bind.table8 )
        {
            int v;
            if( bind_lookup_part<BD, W, H>( p1, s1, p2, s2, &v ) )
            {
                t_bind.hits++;
                return v;
            }
            t_bind.misses++;
        }
    }
    CallCtx &c = call_ctx();
    pixel *a = (pixel *)(c.host + ST_A), *b = (pixel *)(c.host + ST_B);
    int64_t *off = (int64_t *)(c.host + ST_OFF);
    int32_t *sc = (int32_t *)(c.host + ST_SC);
    stage_block( a, p1, s1, W, H );
    stage_block( b, p2, s2, W, H );
    off[0] = off[1] = 0;
    CHECK_FATAL( launch_cmp_batch<BD>( OP, IPIX, dview( c, a ), W, dview( c, b ), W, dview( c, off ),
                                       dview( c, off + 1 ), 1, dview( c, sc ), c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    return sc[0];
}

// x3 / x4: fenc has the implicit FENC_STRIDE (reference common/pixel.c:441-456)
template <int BD, int OP, int IPIX, int N>
static void cmpx_call( typename PT<BD>::pixel *fenc, typename PT<BD>::pixel *const *refs, intptr_t stride, int *scores )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int W = pix_w( IPIX ), H = pix_h( IPIX );
    if constexpr( OP == X264HIP_CMP_SAD && IPIX == X264HIP_PIXEL_16x16 )
    {
        if( t_bind.bd )
        {
            int v[N];
            int k = 0;
            while( k < N && bind_lookup16<BD>( fenc, X264HIP_FENC_STRIDE, refs[k], stride, &v[k] ) )
                k++;
            if( k == N )
            {
                t_bind.hits += N;
                for( int j = 0; j < N; j++ )
                    scores[j] = v[j];
                return;
            }
            t_bind.misses += N;
        }
    }
    if constexpr( OP == X264HIP_CMP_SAD &&
                  ( IPIX == X264HIP_PIXEL_16x8 || IPIX == X264HIP_PIXEL_8x16 || IPIX == X264HIP_PIXEL_8x8 ) )
    {
        if( t_bind.table8 )
        {
            int v[N];
            int k = 0;
            while( k < N && bind_lookup_part<BD, W, H>( fenc, X264HIP_FENC_STRIDE, refs[k], stride, &v[k] ) )
                k++;
            if( k == N )
            {
                t_bind.hits += N;
                for( int j = 0; j < N; j++ )
                    scores[j] = v[j];
                return;
            }
            t_bind.misses += N;
        }
    }
    CallCtx &c = call_ctx();
    pixel *a = (pixel *)(c.host + ST_A), *b = (pixel *)(c.host + ST_B);
    int64_t *off = (int64_t *)(c.host + ST_OFF);
    int32_t *sc = (int32_t *)(c.host + ST_SC);
    stage_block( a, fenc, X264HIP_FENC_STRIDE, W, H );
    for( int k = 0; k < N; k++ )
    {
        stage_block( b + k * W * H, refs[k], stride, W, H );
        off[k] = 0;
        off[N + k] = (int64_t)k * W * H;
    }
    CHECK_FATAL( launch_cmp_batch<BD>( OP, IPIX, dview( c, a ), W, dview( c, b ), W, dview( c, off ),
                                       dview( c, off + N ), N, dview( c, sc ), c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    for( int k = 0; k < N; k++ )
        scores[k] = sc[k];
}

template <int BD, int OP, int IPIX>
static void cmp_x3( typename PT<BD>::pixel *fenc, typename PT<BD>::pixel *p0, typename PT<BD>::pixel *p1,
                    typename PT<BD>::pixel *p2, intptr_t stride, int scores[3] )
{
    typename PT<BD>::pixel *r[3] = { p0, p1, p2 };
    cmpx_call<BD, OP, IPIX, 3>( fenc, r, stride, scores );
}

template <int BD, int OP, int IPIX>
static void cmp_x4( typename PT<BD>::pixel *fenc, typename PT<BD>::pixel *p0, typename PT<BD>::pixel *p1,
                    typename PT<BD>::pixel *p2, typename PT<BD>::pixel *p3, intptr_t stride, int scores[4] )
{
    typename PT<BD>::pixel *r[4] = { p0, p1, p2, p3 };
    cmpx_call<BD, OP, IPIX, 4>( fenc, r, stride, scores );
}

// sa8d_satd / var / hadamard_ac / vsad / asd8: one lane of the u64 statistics kernel
template <int BD, int OP, int IPIX>
static uint64_t stat_call( typename PT<BD>::pixel *p1, intptr_t s1, typename PT<BD>::pixel *p2, intptr_t s2,
                           int w, int h, int height )
{
    using pixel = typename PT<BD>::pixel;
    CallCtx &c = call_ctx();
    pixel *a = (pixel *)(c.host + ST_A), *b = (pixel *)(c.host + ST_B);
    int64_t *off = (int64_t *)(c.host + ST_OFF);
    uint64_t *out = (uint64_t *)(c.host + ST_SC);
    if( (size_t)w * h * sizeof(pixel) > ST_B - ST_A )
    {
        fprintf( stderr, "x264hip: block of %dx%d exceeds the per-call staging buffer\n", w, h );
        abort();
    }
    stage_block( a, p1, s1, w, h );
    if( p2 )
        stage_block( b, p2, s2, w, h );
    off[0] = off[1] = 0;
    CHECK_FATAL( launch_stat_batch<BD>( OP, IPIX, dview( c, a ), w, dview( c, b ), w, dview( c, off ),
                                        dview( c, off + 1 ), height, 1, dview( c, out ), c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    return out[0];
}

template <int BD>
static uint64_t c_sa8d_satd( typename PT<BD>::pixel *p1, intptr_t s1, typename PT<BD>::pixel *p2, intptr_t s2 )
{ return stat_call<BD, X264HIP_STAT_SA8D_SATD, 0>( p1, s1, p2, s2, 16, 16, 0 ); }
template <int BD, int IPIX>
static uint64_t c_var( typename PT<BD>::pixel *p, intptr_t s )
{ return stat_call<BD, X264HIP_STAT_VAR, IPIX>( p, s, nullptr, 0, pix_w( IPIX ), pix_h( IPIX ), 0 ); }
template <int BD, int IPIX>
static uint64_t c_hadamard_ac( typename PT<BD>::pixel *p, intptr_t s )
{ return stat_call<BD, X264HIP_STAT_HADAMARD_AC, IPIX>( p, s, nullptr, 0, pix_w( IPIX ), pix_h( IPIX ), 0 ); }
template <int BD>
static int c_vsad( typename PT<BD>::pixel *p, intptr_t s, int height )
{ return height < 2 ? 0 : (int)stat_call<BD, X264HIP_STAT_VSAD, 0>( p, s, nullptr, 0, 16, height, height ); }
template <int BD>
static int c_asd8( typename PT<BD>::pixel *p1, intptr_t s1, typename PT<BD>::pixel *p2, intptr_t s2, int height )
{ return height < 1 ? 0 : (int)stat_call<BD, X264HIP_STAT_ASD8, 3>( p1, s1, p2, s2, 8, height, height ); }

// ssim_4x4x2_core (pixel.c:627-652): the two 4x4 blocks at pix1 / pix2 staged as one 8x4 block each
template <int BD>
static void c_ssim_4x4x2_core( const typename PT<BD>::pixel *p1, intptr_t s1, const typename PT<BD>::pixel *p2,
                               intptr_t s2, int sums[2][4] )
{
    using pixel = typename PT<BD>::pixel;
    CallCtx &c = call_ctx();
    pixel *a = (pixel *)(c.host + ST_A), *b = (pixel *)(c.host + ST_B);
    int32_t *out = (int32_t *)(c.host + ST_SC);
    stage_block( a, p1, s1, 8, 4 );
    stage_block( b, p2, s2, 8, 4 );
    CHECK_FATAL( launch_ssim_core<BD>( dview( c, a ), 8, dview( c, b ), 8, dview( c, out ), c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    memcpy( sums, out, 8 * sizeof( int ) );
}

// ssim_end4 (pixel.c:679-688) of the caller's two sum rows (5 x 4 ints each, width <= 4)
template <int BD>
static float c_ssim_end4( int sum0[5][4], int sum1[5][4], int width )
{
    CallCtx &c = call_ctx();
    int32_t *s = (int32_t *)(c.host + ST_A);
    float *out = (float *)(c.host + ST_SC);
    memcpy( s, sum0, 20 * sizeof( int ) );
    memcpy( s + 20, sum1, 20 * sizeof( int ) );
    CHECK_FATAL( launch_ssim_end4<BD>( dview( c, s ), dview( c, s + 20 ), width, dview( c, out ), c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    return *out;
}

// ssd_nv12_core (pixel.c:128-151; x264_pixel_ssd_nv12 hands it the width & ~7 core of whole
// chroma planes): both interleaved regions staged into a per-thread pinned buffer that grows to
// the largest region seen, copied to a device buffer of the same size in one hipMemcpyAsync (the
// kernel then reads HBM, not the host link), then the plane SSD kernel's NV12 form.  (No
// destructor, as LaStatus: a thread-exit destructor can run after the HIP runtime is torn
// down; the buffers live as long as the thread's process.)
namespace {
struct BigStage
{
    int device = -1;
    uint8_t *host = nullptr, *dev = nullptr;
    size_t size = 0;
};
thread_local BigStage t_big;
}
template <int BD>
static void c_ssd_nv12_core( typename PT<BD>::pixel *p1, intptr_t s1, typename PT<BD>::pixel *p2, intptr_t s2,
                             int width, int height, uint64_t *ssd_u, uint64_t *ssd_v )
{
    using pixel = typename PT<BD>::pixel;
    if( width <= 0 || height <= 0 )
    {
        *ssd_u = *ssd_v = 0;
        return;
    }
    CallCtx &c = call_ctx();
    const size_t plane = (size_t)2 * width * height * sizeof( pixel );
    const size_t need = 2 * plane + 64;
    if( t_big.device != c.device || t_big.size < need )
    {
        if( t_big.host )
            CHECK_FATAL( hipHostFree( t_big.host ) );
        if( t_big.dev )
            (void)hipFree( t_big.dev );         // (a buffer of the previous device: freed where it lives)
        t_big.host = t_big.dev = nullptr;
        t_big.size = 0;
        CHECK_FATAL( hipHostMalloc( (void **)&t_big.host, need, hipHostMallocDefault ) );
        CHECK_FATAL( hipMalloc( (void **)&t_big.dev, need ) );
        t_big.size = need;
        t_big.device = c.device;
    }
    pixel *a = (pixel *)t_big.host, *b = (pixel *)(t_big.host + plane);
    stage_block( a, p1, s1, 2 * width, height );
    stage_block( b, p2, s2, 2 * width, height );
    CHECK_FATAL( hipMemcpyAsync( t_big.dev, t_big.host, 2 * plane, hipMemcpyHostToDevice, c.stream ) );
    uint64_t *out = (uint64_t *)(c.host + ST_SC);
    CHECK_FATAL( launch_plane_ssd<BD>( 1, (const pixel *)t_big.dev, 2 * width, 0,
                                       (const pixel *)(t_big.dev + plane), 2 * width, 0, width, height, 1,
                                       dview( c, out ), c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    *ssd_u = out[0];
    *ssd_v = out[1];
}

// var2: U at fenc[x], V at fenc[x + FENC_STRIDE/2]; fdec stride FDEC_STRIDE (pixel.c:203-227)
template <int BD, int IPIX>
static int c_var2( typename PT<BD>::pixel *fenc, typename PT<BD>::pixel *fdec, int ssd[2] )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int H = pix_h( IPIX );
    CallCtx &c = call_ctx();
    pixel *a = (pixel *)(c.host + ST_A), *b = (pixel *)(c.host + ST_B);
    int64_t *off = (int64_t *)(c.host + ST_OFF);
    int32_t *out = (int32_t *)(c.host + ST_SC);
    stage_block( a, fenc, X264HIP_FENC_STRIDE, 16, H );
    stage_block( b, fdec, X264HIP_FDEC_STRIDE, 24, H );
    off[0] = off[1] = 0;
    CHECK_FATAL( launch_var2_batch<BD>( IPIX, dview( c, a ), 16, 8, dview( c, b ), 24, 16, dview( c, off ),
                                        dview( c, off + 1 ), 1, dview( c, out ), c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    ssd[0] = out[1];
    ssd[1] = out[2];
    return out[0];
}

// ads: the rows the reference reads (sums[0..], sums[delta..], +8 for ads4) are staged
// back to back with a compact delta (pixel.c:759-803)
template <int IPIX>
static int c_ads( int enc_dc[4], uint16_t *sums, int delta, uint16_t *cost_mvx, int16_t *mvs, int width, int thresh )
{
    constexpr int NS = ads_nsums( IPIX );
    if( width <= 0 )
        return 0;
    CallCtx &c = call_ctx();
    const int len = width + (NS == 4 ? 8 : 0);
    const int dstage = (len + 7) & ~7;
    uint16_t *sm = (uint16_t *)(c.host + ST_B);
    uint16_t *cm = (uint16_t *)(c.host + ST_COEF);
    int16_t *mv = (int16_t *)(c.host + ST_COEF + (12 << 10));
    int32_t *par = (int32_t *)(c.host + ST_SC);          // enc_dc[4], width, thresh, nmv
    int64_t *off = (int64_t *)(c.host + ST_OFF);
    if( 2 * dstage * sizeof(uint16_t) > ST_OFF - ST_B || width * sizeof(uint16_t) > (12 << 10) )
    {
        fprintf( stderr, "x264hip: ads width %d exceeds the per-call staging buffer\n", width );
        abort();
    }
    memcpy( sm, sums, len * sizeof(uint16_t) );
    if( NS > 1 )
        memcpy( sm + dstage, sums + delta, len * sizeof(uint16_t) );
    memcpy( cm, cost_mvx, width * sizeof(uint16_t) );
    for( int k = 0; k < 4; k++ )
        par[k] = k < NS ? enc_dc[k] : 0;
    par[4] = width;
    par[5] = thresh;
    off[0] = off[1] = 0;
    CHECK_FATAL( launch_ads_batch( IPIX, dview( c, par ), dview( c, sm ), dstage, dview( c, off ), dview( c, cm ),
                                   dview( c, off + 1 ), dview( c, par + 4 ), dview( c, par + 5 ), 1, dview( c, mv ),
                                   width, dview( c, par + 6 ), c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    const int n = par[6];
    memcpy( mvs, mv, n * sizeof(int16_t) );
    return n;
}

// ============================================================ per-call dct entries
// kind as X264HIP_DCT_*; fenc stride 16, fdec stride 32 (reference dct.h:31-33)
template <int BD, int KIND, int W, int H, int NOUT>
static void sub_dct_call( typename PT<BD>::dctcoef *dct, typename PT<BD>::pixel *p1, typename PT<BD>::pixel *p2 )
{
    using pixel = typename PT<BD>::pixel;
    using dctcoef = typename PT<BD>::dctcoef;
    CallCtx &c = call_ctx();
    pixel *a = (pixel *)(c.host + ST_A), *b = (pixel *)(c.host + ST_B);
    int64_t *off = (int64_t *)(c.host + ST_OFF);
    dctcoef *o = (dctcoef *)(c.host + ST_COEF);
    stage_block( a, p1, X264HIP_FENC_STRIDE, W, H );
    stage_block( b, p2, X264HIP_FDEC_STRIDE, W, H );
    off[0] = off[1] = 0;
    CHECK_FATAL( launch_sub_dct<BD>( KIND, dview( c, a ), W, dview( c, b ), W, dview( c, off ), dview( c, off + 1 ), 1,
                                     dview( c, o ), c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    memcpy( dct, o, NOUT * sizeof(dctcoef) );
}

template <int BD> static void c_sub4x4_dct( typename PT<BD>::dctcoef dct[16], typename PT<BD>::pixel *a, typename PT<BD>::pixel *b )
{ sub_dct_call<BD, X264HIP_DCT_SUB4x4, 4, 4, 16>( dct, a, b ); }
template <int BD> static void c_sub8x8_dct( typename PT<BD>::dctcoef dct[4][16], typename PT<BD>::pixel *a, typename PT<BD>::pixel *b )
{ sub_dct_call<BD, X264HIP_DCT_SUB8x8, 8, 8, 64>( &dct[0][0], a, b ); }
template <int BD> static void c_sub16x16_dct( typename PT<BD>::dctcoef dct[16][16], typename PT<BD>::pixel *a, typename PT<BD>::pixel *b )
{ sub_dct_call<BD, X264HIP_DCT_SUB16x16, 16, 16, 256>( &dct[0][0], a, b ); }
template <int BD> static void c_sub8x8_dct_dc( typename PT<BD>::dctcoef dct[4], typename PT<BD>::pixel *a, typename PT<BD>::pixel *b )
{ sub_dct_call<BD, X264HIP_DCT_SUB8x8_DC, 8, 8, 4>( dct, a, b ); }
template <int BD> static void c_sub8x16_dct_dc( typename PT<BD>::dctcoef dct[8], typename PT<BD>::pixel *a, typename PT<BD>::pixel *b )
{ sub_dct_call<BD, X264HIP_DCT_SUB8x16_DC, 8, 16, 8>( dct, a, b ); }
template <int BD> static void c_sub8x8_dct8( typename PT<BD>::dctcoef dct[64], typename PT<BD>::pixel *a, typename PT<BD>::pixel *b )
{ sub_dct_call<BD, X264HIP_DCT_SUB8x8_8, 8, 8, 64>( dct, a, b ); }
template <int BD> static void c_sub16x16_dct8( typename PT<BD>::dctcoef dct[4][64], typename PT<BD>::pixel *a, typename PT<BD>::pixel *b )
{ sub_dct_call<BD, X264HIP_DCT_SUB16x16_8, 16, 16, 256>( &dct[0][0], a, b ); }

template <int BD> static void c_dct4x4dc( typename PT<BD>::dctcoef d[16] )
{
    using dctcoef = typename PT<BD>::dctcoef;
    CallCtx &c = call_ctx();
    dctcoef *o = (dctcoef *)(c.host + ST_COEF);
    memcpy( o, d, 16 * sizeof(dctcoef) );
    CHECK_FATAL( launch_dc<BD>( X264HIP_DC_4x4, dview( c, o ), nullptr, 1, c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    memcpy( d, o, 16 * sizeof(dctcoef) );
}

template <int BD> static void c_dct2x4dc( typename PT<BD>::dctcoef dct[8], typename PT<BD>::dctcoef dct4x4[8][16] )
{
    using dctcoef = typename PT<BD>::dctcoef;
    CallCtx &c = call_ctx();
    dctcoef *o = (dctcoef *)(c.host + ST_COEF), *s = o + 16;
    memcpy( s, &dct4x4[0][0], 128 * sizeof(dctcoef) );
    CHECK_FATAL( launch_dc<BD>( X264HIP_DC_2x4, dview( c, o ), dview( c, s ), 1, c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    memcpy( dct, o, 8 * sizeof(dctcoef) );
    memcpy( &dct4x4[0][0], s, 128 * sizeof(dctcoef) );
}

// ============================================================ per-call inverse dct entries
// add*_idct*: p_dst has the implicit FDEC_STRIDE (reference dct.h:31-33); the W x W
// destination block is staged, updated by one kernel and copied back.  Unlike the
// reference C add8x8_idct8 the caller's dct[] is left unmodified (checkasm compares
// only the pixels, tools/checkasm.c:995-1013).
template <int BD, int KIND, int W, int NC>
static void idct_call( typename PT<BD>::pixel *p_dst, const typename PT<BD>::dctcoef *dct )
{
    using pixel = typename PT<BD>::pixel;
    using dctcoef = typename PT<BD>::dctcoef;
    CallCtx &c = call_ctx();
    pixel *a = (pixel *)(c.host + ST_A);
    int64_t *off = (int64_t *)(c.host + ST_OFF);
    dctcoef *o = (dctcoef *)(c.host + ST_COEF);
    stage_block( a, p_dst, X264HIP_FDEC_STRIDE, W, W );
    memcpy( o, dct, NC * sizeof(dctcoef) );
    off[0] = 0;
    CHECK_FATAL( launch_add_idct<BD>( KIND, dview( c, a ), W, dview( c, off ), dview( c, o ), 1, c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    for( int y = 0; y < W; y++ )
        memcpy( p_dst + y * X264HIP_FDEC_STRIDE, a + y * W, W * sizeof(pixel) );
}

template <int BD> static void c_add4x4_idct( typename PT<BD>::pixel *p, typename PT<BD>::dctcoef dct[16] )
{ idct_call<BD, X264HIP_IDCT_ADD4x4, 4, 16>( p, dct ); }
template <int BD> static void c_add8x8_idct( typename PT<BD>::pixel *p, typename PT<BD>::dctcoef dct[4][16] )
{ idct_call<BD, X264HIP_IDCT_ADD8x8, 8, 64>( p, &dct[0][0] ); }
template <int BD> static void c_add16x16_idct( typename PT<BD>::pixel *p, typename PT<BD>::dctcoef dct[16][16] )
{ idct_call<BD, X264HIP_IDCT_ADD16x16, 16, 256>( p, &dct[0][0] ); }
template <int BD> static void c_add8x8_idct_dc( typename PT<BD>::pixel *p, typename PT<BD>::dctcoef dct[4] )
{ idct_call<BD, X264HIP_IDCT_ADD8x8_DC, 8, 4>( p, dct ); }
template <int BD> static void c_add16x16_idct_dc( typename PT<BD>::pixel *p, typename PT<BD>::dctcoef dct[16] )
{ idct_call<BD, X264HIP_IDCT_ADD16x16_DC, 16, 16>( p, dct ); }
template <int BD> static void c_add8x8_idct8( typename PT<BD>::pixel *p, typename PT<BD>::dctcoef dct[64] )
{ idct_call<BD, X264HIP_IDCT_ADD8x8_8, 8, 64>( p, dct ); }
template <int BD> static void c_add16x16_idct8( typename PT<BD>::pixel *p, typename PT<BD>::dctcoef dct[4][64] )
{ idct_call<BD, X264HIP_IDCT_ADD16x16_8, 16, 256>( p, &dct[0][0] ); }

template <int BD> static void c_idct4x4dc( typename PT<BD>::dctcoef d[16] )
{
    using dctcoef = typename PT<BD>::dctcoef;
    CallCtx &c = call_ctx();
    dctcoef *o = (dctcoef *)(c.host + ST_COEF);
    memcpy( o, d, 16 * sizeof(dctcoef) );
    CHECK_FATAL( launch_idct4x4dc<BD>( dview( c, o ), 1, c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    memcpy( d, o, 16 * sizeof(dctcoef) );
}

// ============================================================ per-call inverse quant entries
// staging: coefficients at ST_COEF, dequant_mf at ST_COEF+4K, scalars at ST_SC
constexpr size_t ST_DMF = ST_COEF + (4 << 10);

template <int BD, int KIND, int N>
static void dequant_call( typename PT<BD>::dctcoef *dct, const int *dmf, int qp )
{
    using dctcoef = typename PT<BD>::dctcoef;
    CallCtx &c = call_ctx();
    dctcoef *o = (dctcoef *)(c.host + ST_COEF);
    int32_t *m = (int32_t *)(c.host + ST_DMF);
    int32_t *q = (int32_t *)(c.host + ST_SC);
    memcpy( o, dct, N * sizeof(dctcoef) );
    memcpy( m, dmf, 6 * (KIND == X264HIP_DEQUANT_8x8 ? 64 : 16) * sizeof(int32_t) );
    q[0] = qp;
    CHECK_FATAL( launch_dequant<BD>( KIND, dview( c, o ), dview( c, m ), dview( c, q ), 1, c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    memcpy( dct, o, N * sizeof(dctcoef) );
}
template <int BD> static void c_dequant_4x4( typename PT<BD>::dctcoef dct[16], int dmf[6][16], int qp )
{ dequant_call<BD, X264HIP_DEQUANT_4x4, 16>( dct, &dmf[0][0], qp ); }
template <int BD> static void c_dequant_8x8( typename PT<BD>::dctcoef dct[64], int dmf[6][64], int qp )
{ dequant_call<BD, X264HIP_DEQUANT_8x8, 64>( dct, &dmf[0][0], qp ); }
template <int BD> static void c_dequant_4x4_dc( typename PT<BD>::dctcoef dct[16], int dmf[6][16], int qp )
{ dequant_call<BD, X264HIP_DEQUANT_4x4_DC, 16>( dct, &dmf[0][0], qp ); }

template <int BD>
static void c_idct_dequant_2x4_dc( typename PT<BD>::dctcoef dct[8], typename PT<BD>::dctcoef dct4x4[8][16],
                                   int dmf[6][16], int qp )
{
    using dctcoef = typename PT<BD>::dctcoef;
    CallCtx &c = call_ctx();
    dctcoef *o = (dctcoef *)(c.host + ST_COEF), *s = o + 16;
    int32_t *m = (int32_t *)(c.host + ST_DMF), *q = (int32_t *)(c.host + ST_SC);
    memcpy( o, dct, 8 * sizeof(dctcoef) );
    memcpy( m, &dmf[0][0], 96 * sizeof(int32_t) );
    q[0] = qp;
    CHECK_FATAL( launch_idct_dequant_2x4<BD>( 0, dview( c, o ), dview( c, s ), dview( c, m ), dview( c, q ), 1,
                                              c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    for( int k = 0; k < 8; k++ )     // the reference writes only dct4x4[k][0]
        dct4x4[k][0] = s[k * 16];
}

template <int BD>
static void c_idct_dequant_2x4_dconly( typename PT<BD>::dctcoef dct[8], int dmf[6][16], int qp )
{
    using dctcoef = typename PT<BD>::dctcoef;
    CallCtx &c = call_ctx();
    dctcoef *o = (dctcoef *)(c.host + ST_COEF);
    int32_t *m = (int32_t *)(c.host + ST_DMF), *q = (int32_t *)(c.host + ST_SC);
    memcpy( o, dct, 8 * sizeof(dctcoef) );
    memcpy( m, &dmf[0][0], 96 * sizeof(int32_t) );
    q[0] = qp;
    CHECK_FATAL( launch_idct_dequant_2x4<BD>( 1, dview( c, o ), nullptr, dview( c, m ), dview( c, q ), 1, c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    memcpy( dct, o, 8 * sizeof(dctcoef) );
}

template <int BD, int C422>
static int c_optimize_chroma( typename PT<BD>::dctcoef *dct, int dmf )
{
    using dctcoef = typename PT<BD>::dctcoef;
    constexpr int N = C422 ? 8 : 4;
    CallCtx &c = call_ctx();
    dctcoef *o = (dctcoef *)(c.host + ST_COEF);
    int32_t *q = (int32_t *)(c.host + ST_SC);
    memcpy( o, dct, N * sizeof(dctcoef) );
    q[0] = dmf;
    CHECK_FATAL( launch_optimize_chroma<BD>( C422, dview( c, o ), dview( c, q ), 1, dview( c, q + 1 ), c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    memcpy( dct, o, N * sizeof(dctcoef) );
    return q[1];
}
template <int BD> static int c_optimize_chroma_2x2_dc( typename PT<BD>::dctcoef dct[4], int dmf )
{ return c_optimize_chroma<BD, 0>( dct, dmf ); }
template <int BD> static int c_optimize_chroma_2x4_dc( typename PT<BD>::dctcoef dct[8], int dmf )
{ return c_optimize_chroma<BD, 1>( dct, dmf ); }

template <int BD>
static void c_denoise_dct( typename PT<BD>::dctcoef *dct, uint32_t *sum, typename PT<BD>::udctcoef *offset, int size )
{
    using dctcoef = typename PT<BD>::dctcoef;
    using udctcoef = typename PT<BD>::udctcoef;
    if( size <= 0 )
        return;
    if( size > 64 )
    {
        fprintf( stderr, "x264hip: denoise_dct size %d exceeds the per-call staging buffer\n", size );
        abort();
    }
    CallCtx &c = call_ctx();
    dctcoef *o = (dctcoef *)(c.host + ST_COEF);
    uint32_t *sm = (uint32_t *)(c.host + ST_DMF);
    udctcoef *of = (udctcoef *)(c.host + ST_DMF + 1024);
    memcpy( o, dct, size * sizeof(dctcoef) );
    memcpy( sm, sum, size * sizeof(uint32_t) );
    memcpy( of, offset, size * sizeof(udctcoef) );
    CHECK_FATAL( launch_denoise<BD>( dview( c, o ), size, 1, dview( c, sm ), dview( c, of ), c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    memcpy( dct, o, size * sizeof(dctcoef) );
    memcpy( sum, sm, size * sizeof(uint32_t) );
}

template <int BD, int KIND, int N>
static int coef_stat_call( typename PT<BD>::dctcoef *dct )
{
    using dctcoef = typename PT<BD>::dctcoef;
    CallCtx &c = call_ctx();
    dctcoef *o = (dctcoef *)(c.host + ST_COEF);
    int32_t *r = (int32_t *)(c.host + ST_SC);
    memcpy( o, dct, N * sizeof(dctcoef) );
    CHECK_FATAL( launch_coef_stat<BD>( KIND, dview( c, o ), N, 1, dview( c, r ), c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    return r[0];
}

template <int BD, int NUM>
static int c_level_run( typename PT<BD>::dctcoef *dct, struct x264hip_run_level_t *rl )
{
    using dctcoef = typename PT<BD>::dctcoef;
    CallCtx &c = call_ctx();
    dctcoef *o = (dctcoef *)(c.host + ST_COEF);
    dctcoef *lv = o + 64;
    int32_t *r = (int32_t *)(c.host + ST_SC);
    memcpy( o, dct, NUM * sizeof(dctcoef) );
    CHECK_FATAL( launch_level_run<BD>( NUM, dview( c, o ), NUM, 1, dview( c, r ), dview( c, r + 1 ), dview( c, r + 2 ),
                                       dview( c, lv ), c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    // x264_run_level_t: int32 last, int32 mask, 16-byte aligned dctcoef level[18]
    // (reference common/bitstream.h:50-55)
    uint8_t *base = (uint8_t *)rl;
    memcpy( base, &r[0], 4 );
    memcpy( base + 4, &r[1], 4 );
    memcpy( base + 16, lv, r[2] * sizeof(dctcoef) );
    return r[2];
}

// ============================================================ per-call zigzag entries
template <int BD, int N>
static void c_zigzag_scan( int field, typename PT<BD>::dctcoef *level, const typename PT<BD>::dctcoef *dct )
{
    using dctcoef = typename PT<BD>::dctcoef;
    CallCtx &c = call_ctx();
    dctcoef *o = (dctcoef *)(c.host + ST_COEF), *l = o + 64;
    memcpy( o, dct, N * N * sizeof(dctcoef) );
    CHECK_FATAL( launch_zigzag_scan<BD>( N, field, dview( c, l ), dview( c, o ), 1, c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    memcpy( level, l, N * N * sizeof(dctcoef) );
}
template <int BD, int FIELD> static void c_scan_8x8( typename PT<BD>::dctcoef level[64], typename PT<BD>::dctcoef dct[64] )
{ c_zigzag_scan<BD, 8>( FIELD, level, dct ); }
template <int BD, int FIELD> static void c_scan_4x4( typename PT<BD>::dctcoef level[16], typename PT<BD>::dctcoef dct[16] )
{ c_zigzag_scan<BD, 4>( FIELD, level, dct ); }

// zigzag_sub: p_src stride FENC_STRIDE, p_dst stride FDEC_STRIDE (reference dct.c:828-840)
template <int BD, int KIND, int FIELD>
static int zigzag_sub_call( typename PT<BD>::dctcoef *level, const typename PT<BD>::pixel *src,
                            typename PT<BD>::pixel *dst, typename PT<BD>::dctcoef *dc )
{
    using pixel = typename PT<BD>::pixel;
    using dctcoef = typename PT<BD>::dctcoef;
    constexpr int W = KIND == X264HIP_ZIGZAG_SUB_8x8 ? 8 : 4;
    CallCtx &c = call_ctx();
    pixel *a = (pixel *)(c.host + ST_A), *b = (pixel *)(c.host + ST_B);
    int64_t *off = (int64_t *)(c.host + ST_OFF);
    dctcoef *l = (dctcoef *)(c.host + ST_COEF), *d = l + 64;
    int32_t *nz = (int32_t *)(c.host + ST_SC);
    stage_block( a, src, X264HIP_FENC_STRIDE, W, W );
    stage_block( b, (const pixel *)dst, X264HIP_FDEC_STRIDE, W, W );
    off[0] = 0;
    CHECK_FATAL( launch_zigzag_sub<BD>( KIND, FIELD, dview( c, l ), dview( c, d ), dview( c, a ), W, dview( c, b ), W,
                                        dview( c, off ), dview( c, off ), 1, dview( c, nz ), c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    memcpy( level, l, W * W * sizeof(dctcoef) );
    for( int y = 0; y < W; y++ )
        memcpy( dst + y * X264HIP_FDEC_STRIDE, b + y * W, W * sizeof(pixel) );
    if( dc )
        *dc = d[0];
    return nz[0];
}
template <int BD, int FIELD>
static int c_sub_8x8( typename PT<BD>::dctcoef level[64], const typename PT<BD>::pixel *s, typename PT<BD>::pixel *d )
{ return zigzag_sub_call<BD, X264HIP_ZIGZAG_SUB_8x8, FIELD>( level, s, d, nullptr ); }
template <int BD, int FIELD>
static int c_sub_4x4( typename PT<BD>::dctcoef level[16], const typename PT<BD>::pixel *s, typename PT<BD>::pixel *d )
{ return zigzag_sub_call<BD, X264HIP_ZIGZAG_SUB_4x4, FIELD>( level, s, d, nullptr ); }
template <int BD, int FIELD>
static int c_sub_4x4ac( typename PT<BD>::dctcoef level[16], const typename PT<BD>::pixel *s, typename PT<BD>::pixel *d,
                        typename PT<BD>::dctcoef *dc )
{ return zigzag_sub_call<BD, X264HIP_ZIGZAG_SUB_4x4AC, FIELD>( level, s, d, dc ); }

template <int BD>
static void c_interleave_8x8_cavlc( typename PT<BD>::dctcoef *dst, typename PT<BD>::dctcoef *src, uint8_t *nnz )
{
    using dctcoef = typename PT<BD>::dctcoef;
    CallCtx &c = call_ctx();
    dctcoef *s = (dctcoef *)(c.host + ST_COEF), *d = s + 64;
    uint8_t *nn = (uint8_t *)(c.host + ST_SC);
    memcpy( s, src, 64 * sizeof(dctcoef) );
    CHECK_FATAL( launch_interleave<BD>( dview( c, d ), dview( c, s ), dview( c, nn ), 1, c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    memcpy( dst, d, 64 * sizeof(dctcoef) );
    // the reference writes nnz[0], nnz[1], nnz[8], nnz[9] only (dct.c:927-940)
    nnz[0] = nn[0]; nnz[1] = nn[1]; nnz[8] = nn[8]; nnz[9] = nn[9];
}

// ============================================================ per-call quant entries
template <int BD, int KIND, int N, int NMF>
static int quant_call( typename PT<BD>::dctcoef *dct, const typename PT<BD>::udctcoef *mf,
                       const typename PT<BD>::udctcoef *bias, int mf_dc, int bias_dc )
{
    using dctcoef = typename PT<BD>::dctcoef;
    using udctcoef = typename PT<BD>::udctcoef;
    CallCtx &c = call_ctx();
    dctcoef *o = (dctcoef *)(c.host + ST_COEF);
    udctcoef *m = (udctcoef *)(c.host + ST_COEF + 1024), *f = m + 64;
    int32_t *nz = (int32_t *)(c.host + ST_SC);
    memcpy( o, dct, N * sizeof(dctcoef) );
    if( NMF )
    {
        memcpy( m, mf, NMF * sizeof(udctcoef) );
        memcpy( f, bias, NMF * sizeof(udctcoef) );
    }
    CHECK_FATAL( launch_quant<BD>( KIND, dview( c, o ), dview( c, m ), dview( c, f ), mf_dc, bias_dc, 1,
                                   dview( c, nz ), c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    memcpy( dct, o, N * sizeof(dctcoef) );
    return nz[0];
}

template <int BD> static int c_quant_8x8( typename PT<BD>::dctcoef dct[64], typename PT<BD>::udctcoef mf[64], typename PT<BD>::udctcoef bias[64] )
{ return quant_call<BD, X264HIP_QUANT_8x8, 64, 64>( dct, mf, bias, 0, 0 ); }
template <int BD> static int c_quant_4x4( typename PT<BD>::dctcoef dct[16], typename PT<BD>::udctcoef mf[16], typename PT<BD>::udctcoef bias[16] )
{ return quant_call<BD, X264HIP_QUANT_4x4, 16, 16>( dct, mf, bias, 0, 0 ); }
template <int BD> static int c_quant_4x4x4( typename PT<BD>::dctcoef dct[4][16], typename PT<BD>::udctcoef mf[16], typename PT<BD>::udctcoef bias[16] )
{ return quant_call<BD, X264HIP_QUANT_4x4x4, 64, 16>( &dct[0][0], mf, bias, 0, 0 ); }
template <int BD> static int c_quant_4x4_dc( typename PT<BD>::dctcoef dct[16], int mf, int bias )
{ return quant_call<BD, X264HIP_QUANT_4x4_DC, 16, 0>( dct, nullptr, nullptr, mf, bias ); }
template <int BD> static int c_quant_2x2_dc( typename PT<BD>::dctcoef dct[4], int mf, int bias )
{ return quant_call<BD, X264HIP_QUANT_2x2_DC, 4, 0>( dct, nullptr, nullptr, mf, bias ); }

// ============================================================ table initialisers
// intra_*_x3 (pixel.c:518-560): fenc (FENC_STRIDE) and the block's row -1 /
// column -1 neighbours (FDEC_STRIDE) staged into one (W+1)x(H+1) tile, or the
// 36-entry edge for the 8x8 luma kind
template <int BD, int KIND, int OP>
static void c_intra_x3( typename PT<BD>::pixel *fenc, typename PT<BD>::pixel *fdec, int res[3] )
{
    using pixel = typename PT<BD>::pixel;
    constexpr int W = KIND == 0 ? 4 : KIND == 3 ? 16 : 8, H = KIND == 0 ? 4 : KIND == 1 || KIND == 4 ? 8 : 16;
    CallCtx &c = call_ctx();
    pixel *a = (pixel *)(c.host + ST_A), *b = (pixel *)(c.host + ST_B);
    int64_t *off = (int64_t *)(c.host + ST_OFF);
    int32_t *sc = (int32_t *)(c.host + ST_SC);
    stage_block( a, fenc, X264HIP_FENC_STRIDE, W, H );
    const intptr_t ds = W + 1;
    if( KIND == 4 )
    {
        memcpy( b, fdec, 36 * sizeof(pixel) );
        off[1] = 0;
    }
    else
    {
        stage_block( b, fdec - X264HIP_FDEC_STRIDE - 1, X264HIP_FDEC_STRIDE, W + 1, H + 1 );
        off[1] = ds + 1;
    }
    off[0] = 0;
    CHECK_FATAL( launch_intra_x3<BD>( KIND, OP, dview( c, a ), W, dview( c, b ), ds, dview( c, off ),
                                      dview( c, off + 1 ), 1, dview( c, sc ), c.stream ) );
    CHECK_FATAL( hipStreamSynchronize( c.stream ) );
    res[0] = sc[0];
    res[1] = sc[1];
    res[2] = sc[2];
}

template <int BD, typename Tab>
static void fill_pixel( Tab *pf )
{
#define SIZES8( field, OP )                                           \
    pf->field[0] = cmp_call<BD, OP, 0>; pf->field[1] = cmp_call<BD, OP, 1>; \
    pf->field[2] = cmp_call<BD, OP, 2>; pf->field[3] = cmp_call<BD, OP, 3>; \
    pf->field[4] = cmp_call<BD, OP, 4>; pf->field[5] = cmp_call<BD, OP, 5>; \
    pf->field[6] = cmp_call<BD, OP, 6>; pf->field[7] = cmp_call<BD, OP, 7>;
#define SIZES7( field, FN, OP )                                       \
    pf->field[0] = FN<BD, OP, 0>; pf->field[1] = FN<BD, OP, 1>;       \
    pf->field[2] = FN<BD, OP, 2>; pf->field[3] = FN<BD, OP, 3>;       \
    pf->field[4] = FN<BD, OP, 4>; pf->field[5] = FN<BD, OP, 5>;       \
    pf->field[6] = FN<BD, OP, 6>;
    // entries filled by the reference's C init, common/pixel.c:844-851
    SIZES8( sad, 0 )
    SIZES8( sad_aligned, 0 )
    SIZES8( ssd, 1 )
    SIZES8( satd, 2 )
    SIZES7( sad_x3, cmp_x3, 0 )
    SIZES7( sad_x4, cmp_x4, 0 )
    SIZES7( satd_x3, cmp_x3, 2 )
    SIZES7( satd_x4, cmp_x4, 2 )
    // pixel.c:852-867 (sa8d, var, var2, hadamard_ac, vsad, asd8, ads) and the
    // asm-only merged sa8d_satd (pixel.c:922)
    pf->sa8d[0] = cmp_call<BD, X264HIP_CMP_SA8D, 0>;
    pf->sa8d[3] = cmp_call<BD, X264HIP_CMP_SA8D, 3>;
    pf->sa8d_satd[0] = c_sa8d_satd<BD>;
    pf->var[0] = c_var<BD, 0>;
    pf->var[2] = c_var<BD, 2>;
    pf->var[3] = c_var<BD, 3>;
    pf->var2[2] = c_var2<BD, 2>;
    pf->var2[3] = c_var2<BD, 3>;
    pf->hadamard_ac[0] = c_hadamard_ac<BD, 0>;
    pf->hadamard_ac[1] = c_hadamard_ac<BD, 1>;
    pf->hadamard_ac[2] = c_hadamard_ac<BD, 2>;
    pf->hadamard_ac[3] = c_hadamard_ac<BD, 3>;
    pf->vsad = c_vsad<BD>;
    pf->asd8 = c_asd8<BD>;
    // ssim and the NV12 SSD core (pixel.c:861-865)
    pf->ssd_nv12_core = c_ssd_nv12_core<BD>;
    pf->ssim_4x4x2_core = c_ssim_4x4x2_core<BD>;
    pf->ssim_end4 = c_ssim_end4<BD>;
    // ads slots with the reference's aliasing (pixel.c:835-838, 1605-1608)
    pf->ads[0] = c_ads<0>;
    pf->ads[1] = c_ads<1>;
    pf->ads[2] = c_ads<2>;
    pf->ads[3] = c_ads<3>;
    pf->ads[4] = c_ads<4>;
    pf->ads[5] = c_ads<5>;
    pf->ads[6] = c_ads<6>;
    // intra_*_x3, pixel.c:869-878 (the intra_mbcmp_* aliases are the encoder's, encoder.c:1409-1420)
    pf->intra_sad_x3_4x4 = c_intra_x3<BD, X264HIP_INTRA_4x4, X264HIP_CMP_SAD>;
    pf->intra_satd_x3_4x4 = c_intra_x3<BD, X264HIP_INTRA_4x4, X264HIP_CMP_SATD>;
    pf->intra_sad_x3_8x8 = c_intra_x3<BD, X264HIP_INTRA_8x8, X264HIP_CMP_SAD>;
    pf->intra_sa8d_x3_8x8 = c_intra_x3<BD, X264HIP_INTRA_8x8, X264HIP_CMP_SA8D>;
    pf->intra_sad_x3_8x8c = c_intra_x3<BD, X264HIP_INTRA_8x8C, X264HIP_CMP_SAD>;
    pf->intra_satd_x3_8x8c = c_intra_x3<BD, X264HIP_INTRA_8x8C, X264HIP_CMP_SATD>;
    pf->intra_sad_x3_8x16c = c_intra_x3<BD, X264HIP_INTRA_8x16C, X264HIP_CMP_SAD>;
    pf->intra_satd_x3_8x16c = c_intra_x3<BD, X264HIP_INTRA_8x16C, X264HIP_CMP_SATD>;
    pf->intra_sad_x3_16x16 = c_intra_x3<BD, X264HIP_INTRA_16x16, X264HIP_CMP_SAD>;
    pf->intra_satd_x3_16x16 = c_intra_x3<BD, X264HIP_INTRA_16x16, X264HIP_CMP_SATD>;
#undef SIZES8
#undef SIZES7
}

template <int BD, typename Tab>
static void fill_dct( Tab *d )
{
    d->sub4x4_dct = c_sub4x4_dct<BD>;
    d->sub8x8_dct = c_sub8x8_dct<BD>;
    d->sub8x8_dct_dc = c_sub8x8_dct_dc<BD>;
    d->sub8x16_dct_dc = c_sub8x16_dct_dc<BD>;
    d->sub16x16_dct = c_sub16x16_dct<BD>;
    d->sub8x8_dct8 = c_sub8x8_dct8<BD>;
    d->sub16x16_dct8 = c_sub16x16_dct8<BD>;
    d->dct4x4dc = c_dct4x4dc<BD>;
    d->dct2x4dc = c_dct2x4dc<BD>;
    // inverse entries, reference dct.c:479-502
    d->add4x4_idct = c_add4x4_idct<BD>;
    d->add8x8_idct = c_add8x8_idct<BD>;
    d->add8x8_idct_dc = c_add8x8_idct_dc<BD>;
    d->add16x16_idct = c_add16x16_idct<BD>;
    d->add16x16_idct_dc = c_add16x16_idct_dc<BD>;
    d->add8x8_idct8 = c_add8x8_idct8<BD>;
    d->add16x16_idct8 = c_add16x16_idct8<BD>;
    d->idct4x4dc = c_idct4x4dc<BD>;
}

// zigzag tables, reference dct.c:938-951 (field scans for the interlaced table)
template <int BD, typename Tab>
static void fill_zigzag( Tab *p, Tab *i )
{
    p->scan_8x8 = c_scan_8x8<BD, 0>;
    i->scan_8x8 = c_scan_8x8<BD, 1>;
    p->scan_4x4 = c_scan_4x4<BD, 0>;
    i->scan_4x4 = c_scan_4x4<BD, 1>;
    p->sub_8x8 = c_sub_8x8<BD, 0>;
    i->sub_8x8 = c_sub_8x8<BD, 1>;
    p->sub_4x4 = c_sub_4x4<BD, 0>;
    i->sub_4x4 = c_sub_4x4<BD, 1>;
    p->sub_4x4ac = c_sub_4x4ac<BD, 0>;
    i->sub_4x4ac = c_sub_4x4ac<BD, 1>;
    p->interleave_8x8_cavlc = i->interleave_8x8_cavlc = c_interleave_8x8_cavlc<BD>;
}

template <int BD, typename Tab>
static void fill_quant( Tab *q )
{
    q->quant_8x8 = c_quant_8x8<BD>;
    q->quant_4x4 = c_quant_4x4<BD>;
    q->quant_4x4x4 = c_quant_4x4x4<BD>;
    q->quant_4x4_dc = c_quant_4x4_dc<BD>;
    q->quant_2x2_dc = c_quant_2x2_dc<BD>;
    // reference quant.c:422-445 and the category aliasing at the end of x264_quant_init
    q->dequant_4x4 = c_dequant_4x4<BD>;
    q->dequant_4x4_dc = c_dequant_4x4_dc<BD>;
    q->dequant_8x8 = c_dequant_8x8<BD>;
    q->idct_dequant_2x4_dc = c_idct_dequant_2x4_dc<BD>;
    q->idct_dequant_2x4_dconly = c_idct_dequant_2x4_dconly<BD>;
    q->optimize_chroma_2x2_dc = c_optimize_chroma_2x2_dc<BD>;
    q->optimize_chroma_2x4_dc = c_optimize_chroma_2x4_dc<BD>;
    q->denoise_dct = c_denoise_dct<BD>;
    q->decimate_score15 = coef_stat_call<BD, X264HIP_COEF_DECIMATE15, 16>;
    q->decimate_score16 = coef_stat_call<BD, X264HIP_COEF_DECIMATE16, 16>;
    q->decimate_score64 = coef_stat_call<BD, X264HIP_COEF_DECIMATE64, 64>;
    q->coeff_last4 = coef_stat_call<BD, X264HIP_COEF_LAST4, 4>;
    q->coeff_last8 = coef_stat_call<BD, X264HIP_COEF_LAST8, 8>;
    // block categories, reference common/macroblock.h:273-289
    for( int cat : { 1, 4, 7, 11 } )
    {
        q->coeff_last[cat] = coef_stat_call<BD, X264HIP_COEF_LAST15, 15>;
        q->coeff_level_run[cat] = c_level_run<BD, 15>;
    }
    for( int cat : { 0, 2, 6, 8, 10, 12 } )
    {
        q->coeff_last[cat] = coef_stat_call<BD, X264HIP_COEF_LAST16, 16>;
        q->coeff_level_run[cat] = c_level_run<BD, 16>;
    }
    for( int cat : { 5, 9, 13 } )
        q->coeff_last[cat] = coef_stat_call<BD, X264HIP_COEF_LAST64, 64>;
    q->coeff_level_run4 = c_level_run<BD, 4>;
    q->coeff_level_run8 = c_level_run<BD, 8>;
}

// ============================================================ CQM (quant side)
// Restates x264_cqm_init, reference common/set.c:28-206, for the mf/bias
// tables the quant entries take as inputs.
static const uint16_t k_quant4_scale[6][3] = {
    { 13107, 8066, 5243 }, { 11916, 7490, 4660 }, { 10082, 6554, 4194 },
    { 9362, 5825, 3647 },  { 8192, 5243, 3355 },  { 7282, 4559, 2893 } };
static const uint8_t k_quant8_scan[16] = { 0, 3, 4, 3, 3, 1, 5, 1, 4, 5, 2, 5, 3, 1, 5, 1 };
static const uint16_t k_quant8_scale[6][6] = {
    { 13107, 11428, 20972, 12222, 16777, 15481 }, { 11916, 10826, 19174, 11058, 14980, 14290 },
    { 10082, 8943, 15978, 9675, 12710, 11985 },   { 9362, 8228, 14913, 8931, 11984, 11259 },
    { 8192, 7346, 13159, 7740, 10486, 9777 },     { 7282, 6428, 11570, 6830, 9118, 8640 } };

static inline int cqm_div( int n, int d ) { return (n + (d >> 1)) / d; }
static inline int cqm_shift( int x, int s ) { return s <= 0 ? x << -s : (x + (1 << (s - 1))) >> s; }

template <int BD>
static int cqm_init( const uint8_t *const sl[8], int dz_inter, int dz_intra, int b8, typename PT<BD>::udctcoef *q4m,
                     typename PT<BD>::udctcoef *q4b, typename PT<BD>::udctcoef *q8m, typename PT<BD>::udctcoef *q8b )
{
    const int qmax = 51 + 6 * (BD - 8);
    const int dz[4] = { 32 - dz_intra, 32 - dz_inter, 32 - 11, 32 - 21 };
    for( int q = 0; q <= qmax; q++ )
    {
        for( int l = 0; l < 4; l++ )
            for( int i = 0; i < 16; i++ )
            {
                int base = cqm_div( k_quant4_scale[q % 6][(i & 1) + ((i >> 2) & 1)] * 16, sl[l][i] );
                int j = cqm_shift( base, q / 6 - 1 );
                size_t o = ((size_t)l * (qmax + 1) + q) * 16 + i;
                q4m[o] = (uint16_t)j;
                if( j )
                {
                    int a = cqm_div( dz[l] << 10, j ), b = (1 << 15) / j;
                    q4b[o] = a < b ? a : b;
                }
            }
        if( b8 )
            for( int l = 0; l < 2; l++ )
                for( int i = 0; i < 64; i++ )
                {
                    int base = cqm_div( k_quant8_scale[q % 6][k_quant8_scan[((i >> 1) & 12) | (i & 3)]] * 16, sl[4 + l][i] );
                    int j = cqm_shift( base, q / 6 );
                    size_t o = ((size_t)l * (qmax + 1) + q) * 64 + i;
                    q8m[o] = (uint16_t)j;
                    if( j )
                    {
                        int a = cqm_div( dz[l] << 10, j ), b = (1 << 15) / j;
                        q8b[o] = a < b ? a : b;
                    }
                }
    }
    return qmax;
}

// ============================================================ exported entries
// a centred window's origin is aligned down by up to 3 (8 bit) / 1 (10 bit) pixels and

static int map_err( hipError_t e, const char *where )
{
    if( e == hipSuccess )
        return X264HIP_OK;
    if( e == hipErrorLaunchTimeOut )
    {
        // the lookahead wavefront's status word (lookahead.hip la_status_end)
        snprintf( t_err, sizeof(t_err), "%s: a band's wait for the band below timed out; outputs are invalid",
                  where );
        return X264HIP_EDEVICE;
    }
    if( e == hipErrorInvalidValue )
    {
        snprintf( t_err, sizeof(t_err), "%s: invalid argument", where );
        return X264HIP_EINVAL;
    }
    return set_err( e, where );
}

// ------------------------------------------------------------ backend banner
// The analogue of the encoder's "using cpu capabilities" line (reference
// encoder/encoder.c:1676-1706): which device serves the tables and which entries
// the HIP backend filled.  Printed once to stderr at the first table fill
// (X264HIP_QUIET=1 silences it); x264hip_backend_banner() returns the text.
static char g_banner[768];
static std::once_flag g_banner_once;
static std::mutex g_banner_mutex;

static void build_banner()
{
    std::lock_guard<std::mutex> lk( g_banner_mutex );
    const int dev = x264hip_thread_device();
    hipDeviceProp_t prop;
    char name[160] = "no device";
    if( dev >= 0 && hipGetDeviceProperties( &prop, dev ) == hipSuccess )
        snprintf( name, sizeof(name), "device %d %s (%s, %d CUs)", dev, prop.name, prop.gcnArchName,
                  prop.multiProcessorCount );
    snprintf( g_banner, sizeof(g_banner),
              "x264hip: %s; HIP entries: pixel sad/sad_aligned/ssd/satd[8] sad_x3/x4 satd_x3/x4[7] sa8d[2] "
              "sa8d_satd var[3] var2[2] hadamard_ac[4] vsad asd8 ads[7] intra_*_x3[10] ssd_nv12_core "
              "ssim_4x4x2_core ssim_end4; dct 17/17; "
              "quant quant[5] dequant[3] idct_dequant_2x4[2] optimize_chroma[2] denoise decimate[3] coeff_last[16] "
              "coeff_level_run[15]; zigzag 6+6; kept from the caller's C init: intra_*_x9 trellis_cabac_* "
              "(ssim[7] is never set by the reference)",
              name );
}

static void note_fill()
{
    std::call_once( g_banner_once, [] {
        build_banner();
        const char *q = getenv( "X264HIP_QUIET" );
        if( !(q && *q && *q != '0') )
            fprintf( stderr, "%s\n", g_banner );
    } );
}

extern "C" const char *x264hip_backend_banner( void )
{
    build_banner();
    return g_banner;
}

// Table initialisers.  Both forms only OVERRIDE: the entries this backend
// implements are replaced, every other entry (the trellis entries, intra_*_x9_*, the
// never-initialised ssim[7], and the encoder's mbcmp / fpelcmp aliases) keeps what the caller's
// C init put there.  Without a usable gfx950 device (or without X264HIP_CPU_HIP in
// `cpu` for the flag form) the table is left untouched, so a host without the GPU
// keeps its C entries, the convention of reference common/opencl.c:400-409; no
// entry that could reach a missing device is ever installed.
#define DEFINE_ENTRIES( BD )                                                                                         \
    extern "C" void x264hip_##BD##_pixel_init_hip( x264hip_##BD##_pixel_function_t *pixf )                         \
    {                                                                                                                \
        if( pixf && x264hip_available() )                                                                            \
        {                                                                                                            \
            fill_pixel<BD>( pixf );                                                                                  \
            note_fill();                                                                                             \
        }                                                                                                            \
    }                                                                                                                \
    extern "C" void x264hip_##BD##_pixel_init( uint32_t cpu, x264hip_##BD##_pixel_function_t *pixf )                \
    {                                                                                                                \
        if( cpu & X264HIP_CPU_HIP )                                                                                  \
            x264hip_##BD##_pixel_init_hip( pixf );                                                                   \
    }                                                                                                                \
    extern "C" void x264hip_##BD##_dct_init_hip( x264hip_##BD##_dct_function_t *d )                                 \
    {                                                                                                                \
        if( d && x264hip_available() )                                                                               \
            fill_dct<BD>( d );                                                                                       \
    }                                                                                                                \
    extern "C" void x264hip_##BD##_dct_init( uint32_t cpu, x264hip_##BD##_dct_function_t *d )                       \
    {                                                                                                                \
        if( cpu & X264HIP_CPU_HIP )                                                                                  \
            x264hip_##BD##_dct_init_hip( d );                                                                        \
    }                                                                                                                \
    extern "C" void x264hip_##BD##_quant_init_hip( x264hip_##BD##_quant_function_t *q )                             \
    {                                                                                                                \
        if( q && x264hip_available() )                                                                               \
            fill_quant<BD>( q );                                                                                     \
    }                                                                                                                \
    extern "C" void x264hip_##BD##_quant_init( void *h, uint32_t cpu, x264hip_##BD##_quant_function_t *q )          \
    {                                                                                                                \
        (void)h;                                                                                                     \
        if( cpu & X264HIP_CPU_HIP )                                                                                  \
            x264hip_##BD##_quant_init_hip( q );                                                                      \
    }                                                                                                                \
    extern "C" void x264hip_##BD##_zigzag_init_hip( x264hip_##BD##_zigzag_function_t *p,                            \
                                                    x264hip_##BD##_zigzag_function_t *i )                            \
    {                                                                                                                \
        if( p && i && x264hip_available() )                                                                          \
            fill_zigzag<BD>( p, i );                                                                                 \
    }                                                                                                                \
    extern "C" void x264hip_##BD##_zigzag_init( uint32_t cpu, x264hip_##BD##_zigzag_function_t *p,                  \
                                                x264hip_##BD##_zigzag_function_t *i )                                \
    {                                                                                                                \
        if( cpu & X264HIP_CPU_HIP )                                                                                  \
            x264hip_##BD##_zigzag_init_hip( p, i );                                                                  \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_cqm_init( const uint8_t *const sl[8], int dz_inter, int dz_intra, int b8,         \
                                            PT<BD>::udctcoef *q4m, PT<BD>::udctcoef *q4b, PT<BD>::udctcoef *q8m,     \
                                            PT<BD>::udctcoef *q8b )                                                  \
    {                                                                                                                \
        return cqm_init<BD>( sl, dz_inter, dz_intra, b8, q4m, q4b, q8m, q8b );                                       \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_pixel_cmp_batch( int op, int i_pixel, const PT<BD>::pixel *fenc, intptr_t fs,     \
                                                   const PT<BD>::pixel *ref, intptr_t rs, const int64_t *fo,         \
                                                   const int64_t *ro, int n, int32_t *scores, void *stream )        \
    {                                                                                                                \
        if( op < 0 || op > 3 || i_pixel < 0 || i_pixel > 7 || n < 0 )                                                \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_cmp_batch<BD>( op, i_pixel, fenc, fs, ref, rs, fo, ro, n, scores,                     \
                                              (hipStream_t)stream ), "pixel_cmp_batch" );                            \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_pixel_stat_batch( int op, int i_pixel, const PT<BD>::pixel *p1, intptr_t s1,      \
                                                    const PT<BD>::pixel *p2, intptr_t s2, const int64_t *o1,        \
                                                    const int64_t *o2, int height, int n, uint64_t *out,            \
                                                    void *stream )                                                   \
    {                                                                                                                \
        if( op < 0 || op > 4 || n < 0 || ( (op == 3 || op == 4) && height < 0 ) )                                    \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_stat_batch<BD>( op, i_pixel, p1, s1, p2, s2, o1, o2, height, n, out,                  \
                                               (hipStream_t)stream ), "pixel_stat_batch" );                          \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_var2_batch( int i_pixel, const PT<BD>::pixel *fenc, intptr_t fs, intptr_t fvd,    \
                                              const PT<BD>::pixel *fdec, intptr_t ds, intptr_t dvd,                  \
                                              const int64_t *fo, const int64_t *dof, int n, int32_t *out,            \
                                              void *stream )                                                         \
    {                                                                                                                \
        if( n < 0 )                                                                                                  \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_var2_batch<BD>( i_pixel, fenc, fs, fvd, fdec, ds, dvd, fo, dof, n, out,               \
                                               (hipStream_t)stream ), "var2_batch" );                                \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_ads_batch( int i_pixel, const int32_t *enc_dc, const uint16_t *sums, int delta,   \
                                             const int64_t *sums_off, const uint16_t *cost, const int64_t *cost_off, \
                                             const int32_t *width, const int32_t *thresh, int n, int16_t *mvs,       \
                                             int mvs_pitch, int32_t *nmv, void *stream )                             \
    {                                                                                                                \
        if( i_pixel < 0 || i_pixel > 6 || n < 0 || mvs_pitch < 0 )                                                   \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_ads_batch( i_pixel, enc_dc, sums, delta, sums_off, cost, cost_off, width, thresh, n,  \
                                          mvs, mvs_pitch, nmv, (hipStream_t)stream ), "ads_batch" );                 \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_intra_cmp_x3_batch( int kind, int op, const PT<BD>::pixel *fenc, intptr_t fs,     \
                                                      const PT<BD>::pixel *fdec, intptr_t ds, const int64_t *fo,    \
                                                      const int64_t *dof, int n, int32_t *scores, void *stream )    \
    {                                                                                                                \
        const bool ok = kind >= 0 && kind <= 4 &&                                                                    \
                        ( op == X264HIP_CMP_SAD || ( kind == 4 ? op == X264HIP_CMP_SA8D : op == X264HIP_CMP_SATD ) ); \
        if( !ok || n < 0 || ( n > 0 && ( !fenc || !fdec || !fo || !dof || !scores ) ) )                             \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_intra_x3<BD>( kind, op, fenc, fs, fdec, ds, fo, dof, n, scores,                       \
                                             (hipStream_t)stream ), "intra_cmp_x3_batch" );                          \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_lowres_intra_cost( const PT<BD>::pixel *plane, intptr_t stride, intptr_t fstride, \
                                                     int mbw, int mbh, int nframes, int satd, int all_modes,        \
                                                     int lambda, const uint16_t *invq, uint16_t *cost,              \
                                                     int32_t *row_satd, int32_t *est, void *stream )                \
    {                                                                                                                \
        if( mbw < 0 || mbh < 0 || nframes < 0 || lambda < 0 || ( (uintptr_t)plane & 3 ) ||                          \
            ( ( stride * (intptr_t)sizeof(PT<BD>::pixel) ) & 3 ) ||                                                 \
            ( ( fstride * (intptr_t)sizeof(PT<BD>::pixel) ) & 3 ) || stride < 8 * mbw + 64 ||                      \
            ( (int64_t)mbw * mbh * nframes > 0 && ( !plane || !cost ) ) )                                            \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_lowres_intra<BD>( plane, stride, fstride, mbw, mbh, nframes, satd, all_modes, lambda, \
                                                 invq, cost, row_satd, est, (hipStream_t)stream ),                   \
                        "lowres_intra_cost" );                                                                       \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_lowres_inter_cost_ex(                                                            \
        const PT<BD>::pixel *fenc, intptr_t ffs, const PT<BD>::pixel *rf, const PT<BD>::pixel *rh,                  \
        const PT<BD>::pixel *rv, const PT<BD>::pixel *rc, intptr_t stride, intptr_t rfs, int mbw, int mbh,          \
        int npairs, int me_method, int subme, int satd, int me_range, int mv_range, int lambda,                     \
        const uint16_t *cost_mv, const uint16_t *intra_cost, const uint16_t *invq, int16_t *mvs, int32_t *mv_costs,   \
        uint16_t *lowres_costs, int32_t *row_satd, int32_t *est, const PT<BD>::pixel *ref_w, int w_scale,           \
        int w_denom, int w_offset, int n_slices, void *stream )                                                      \
    {                                                                                                                \
        if( n_slices < 1 || n_slices > 256 )                                                                         \
            return X264HIP_EINVAL;                                                                                   \
        const intptr_t pb = (intptr_t)sizeof( PT<BD>::pixel );                                                       \
        if( mbw < 0 || mbh < 0 || npairs < 0 || ( me_method != 0 && me_method != 1 ) ||                              \
            ( subme != 2 && subme != 4 ) || me_range < 1 || mv_range < 1 || lambda < 0 ||                            \
            ( (uintptr_t)fenc & 3 ) || ( ( stride * pb ) & 3 ) || ( ( ffs * pb ) & 3 ) ||                            \
            stride < 8 * mbw + 64 ||                                                                                 \
            ( ref_w && ( w_denom < 0 || w_denom > 7 || w_scale < -128 || w_scale > 127 || w_offset < -128 ||         \
                         w_offset > 127 ) ) ||                                                                       \
            ( (int64_t)mbw * mbh * npairs > 0 &&                                                                     \
              ( !fenc || !rf || !rh || !rv || !rc || !cost_mv || !intra_cost || !mvs || !mv_costs ||                 \
                !lowres_costs ) ) )                                                                                  \
            return X264HIP_EINVAL;                                                                                   \
        const PT<BD>::pixel *ref[4] = { rf, rh, rv, rc };                                                            \
        return map_err( launch_lowres_inter<BD>( fenc, ffs, ref, stride, rfs, mbw, mbh, npairs, me_method, subme,    \
                                                 satd, me_range, mv_range, lambda, cost_mv, intra_cost, invq, mvs,   \
                                                 mv_costs, lowres_costs, row_satd, est, ref_w, w_scale, w_denom,     \
                                                 w_offset, n_slices, (hipStream_t)stream ),                          \
                        "lowres_inter_cost" );                                                                       \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_lowres_inter_cost(                                                               \
        const PT<BD>::pixel *fenc, intptr_t ffs, const PT<BD>::pixel *rf, const PT<BD>::pixel *rh,                  \
        const PT<BD>::pixel *rv, const PT<BD>::pixel *rc, intptr_t stride, intptr_t rfs, int mbw, int mbh,          \
        int npairs, int me_method, int subme, int satd, int me_range, int mv_range, int lambda,                     \
        const uint16_t *cost_mv, const uint16_t *intra_cost, const uint16_t *invq, int16_t *mvs, int32_t *mv_costs,   \
        uint16_t *lowres_costs, int32_t *row_satd, int32_t *est, void *stream )                                      \
    {                                                                                                                \
        return x264hip_##BD##_lowres_inter_cost_ex( fenc, ffs, rf, rh, rv, rc, stride, rfs, mbw, mbh, npairs,         \
                                                    me_method, subme, satd, me_range, mv_range, lambda, cost_mv,     \
                                                    intra_cost, invq, mvs, mv_costs, lowres_costs, row_satd, est,    \
                                                    nullptr, 0, 0, 0, 1, stream );                                   \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_weight_scale_plane( PT<BD>::pixel *dst, intptr_t ds, intptr_t dfs,               \
                                                      const PT<BD>::pixel *src, intptr_t ss, intptr_t sfs,          \
                                                      int width, int height, int nframes, int scale, int denom,     \
                                                      int offset, void *stream )                                    \
    {                                                                                                                \
        if( width < 0 || height < 0 || nframes < 0 || denom < 0 || denom > 7 || scale < -128 || scale > 127 ||      \
            offset < -128 || offset > 127 ||                                                                         \
            ( (int64_t)width * height * nframes > 0 && ( !dst || !src || dst == src ) ) )                            \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_weight_plane<BD>( dst, ds, dfs, src, ss, sfs, width, height, nframes, scale, denom,  \
                                                 offset, (hipStream_t)stream ),                                      \
                        "weight_scale_plane" );                                                                      \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_lowres_bidir_cost_ex(                                                            \
        const PT<BD>::pixel *fenc, intptr_t ffs, const PT<BD>::pixel *af, const PT<BD>::pixel *ah,                  \
        const PT<BD>::pixel *av, const PT<BD>::pixel *ac, intptr_t afs, const PT<BD>::pixel *bf,                    \
        const PT<BD>::pixel *bh, const PT<BD>::pixel *bv, const PT<BD>::pixel *bc, intptr_t bfs, intptr_t stride,   \
        int mbw, int mbh, int n, int me_method, int subme, int satd, int me_range, int mv_range, int lambda,        \
        const uint16_t *cost_mv, int search, int16_t *mvs0, int32_t *costs0, int16_t *mvs1, int32_t *costs1,       \
        const int16_t *p1mvs, int dsf, int weight, const uint16_t *invq, uint16_t *lowres_costs, int32_t *row_satd,  \
        int32_t *est, int n_slices, void *stream )                                                                   \
    {                                                                                                                \
        const intptr_t pb = (intptr_t)sizeof( PT<BD>::pixel );                                                       \
        if( n_slices < 1 || n_slices > 256 )                                                                         \
            return X264HIP_EINVAL;                                                                                   \
        if( mbw < 0 || mbh < 0 || n < 0 || ( me_method != 0 && me_method != 1 ) || ( subme != 2 && subme != 4 ) ||   \
            me_range < 1 || mv_range < 1 || lambda < 0 || search < 0 || search > 3 || weight < 0 || weight > 64 ||   \
            ( (uintptr_t)fenc & 3 ) || ( ( stride * pb ) & 3 ) || ( ( ffs * pb ) & 3 ) || stride < 8 * mbw + 64 ||   \
            ( (int64_t)mbw * mbh * n > 0 && ( !fenc || !af || !ah || !av || !ac || !bf || !bh || !bv || !bc ||       \
                                              !cost_mv || !mvs0 || !costs0 || !mvs1 || !costs1 || !lowres_costs ) ) ) \
            return X264HIP_EINVAL;                                                                                   \
        const PT<BD>::pixel *ra[4] = { af, ah, av, ac }, *rb[4] = { bf, bh, bv, bc };                                \
        return map_err( launch_lowres_bidir<BD>( fenc, ffs, ra, afs, rb, bfs, stride, mbw, mbh, n, me_method, subme, \
                                                 satd, me_range, mv_range, lambda, cost_mv, search, mvs0, costs0,    \
                                                 mvs1, costs1, p1mvs, dsf, weight, invq, lowres_costs, row_satd,     \
                                                 est, n_slices, (hipStream_t)stream ),                               \
                        "lowres_bidir_cost" );                                                                       \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_lowres_bidir_cost(                                                               \
        const PT<BD>::pixel *fenc, intptr_t ffs, const PT<BD>::pixel *af, const PT<BD>::pixel *ah,                  \
        const PT<BD>::pixel *av, const PT<BD>::pixel *ac, intptr_t afs, const PT<BD>::pixel *bf,                    \
        const PT<BD>::pixel *bh, const PT<BD>::pixel *bv, const PT<BD>::pixel *bc, intptr_t bfs, intptr_t stride,   \
        int mbw, int mbh, int n, int me_method, int subme, int satd, int me_range, int mv_range, int lambda,        \
        const uint16_t *cost_mv, int search, int16_t *mvs0, int32_t *costs0, int16_t *mvs1, int32_t *costs1,       \
        const int16_t *p1mvs, int dsf, int weight, const uint16_t *invq, uint16_t *lowres_costs, int32_t *row_satd,  \
        int32_t *est, void *stream )                                                                                 \
    {                                                                                                                \
        return x264hip_##BD##_lowres_bidir_cost_ex( fenc, ffs, af, ah, av, ac, afs, bf, bh, bv, bc, bfs, stride,     \
                                                    mbw, mbh, n, me_method, subme, satd, me_range, mv_range,         \
                                                    lambda, cost_mv, search, mvs0, costs0, mvs1, costs1, p1mvs, dsf, \
                                                    weight, invq, lowres_costs, row_satd, est, 1, stream );          \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_frame_integral( const PT<BD>::pixel *plane, intptr_t stride, intptr_t fstride,    \
                                                  int lines, int padh, int sub8x8, int nframes, uint16_t *integral,  \
                                                  intptr_t ifstride, void *stream )                                  \
    {                                                                                                                \
        if( lines <= 0 || nframes < 0 || padh < 0 || stride < padh + 16 )                                            \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_frame_integral<BD>( plane, stride, fstride, lines, padh, sub8x8, nframes, integral,   \
                                                   ifstride, (hipStream_t)stream ), "frame_integral" );              \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_me_search_full( const PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,             \
                                                  const PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs, int mbw,      \
                                                  int mbh, int nframes, int range, PT<BD>::sadt *table,             \
                                                  void *stream )                                                     \
    {                                                                                                                \
        if( mbw < 0 || mbh < 0 || nframes < 0 || !( range == 4 || range == 8 || range == 16 || range == 24 ) )        \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_me_full<BD>( fenc, fs, ffs, ref, rs, rfs, mbw, mbh, nframes, range, table, nullptr,  \
                                            nullptr, (hipStream_t)stream ), "me_search_full" );                      \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_me_search_centred( const PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,          \
                                                     const PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs, int mbw,   \
                                                     int mbh, int nframes, int range, const int16_t *centre,         \
                                                     PT<BD>::sadt *table, int16_t *origin, void *stream )            \
    {                                                                                                                \
        if( mbw < 0 || mbh < 0 || nframes < 0 || !centre || !origin ||                                               \
            !( range == 4 || range == 8 || range == 16 || range == 24 ) )                                            \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_me_full<BD>( fenc, fs, ffs, ref, rs, rfs, mbw, mbh, nframes, range, table, centre,   \
                                            origin, (hipStream_t)stream ), "me_search_centred" );                    \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_me_search_full8( const PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,           \
                                                   const PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs, int mbw,     \
                                                   int mbh, int nframes, int range, uint16_t *table8,                \
                                                   void *stream )                                                    \
    {                                                                                                                \
        if( mbw < 0 || mbh < 0 || nframes < 0 ||                                                                     \
            !( range == 4 || range == 8 || range == 16 || range == 24 ) ||                                           \
            ( (int64_t)mbw * mbh * nframes > 0 && ( !fenc || !ref || !table8 ) ) )                                   \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_me_full8<BD>( fenc, fs, ffs, ref, rs, rfs, mbw, mbh, nframes, range, table8,          \
                                             (hipStream_t)stream ), "me_search_full8" );                             \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_me_esa_argmin( const PT<BD>::sadt *table, int range, int n, int me_range,         \
                                                 const int16_t *par, const int32_t *init_cost,                       \
                                                 const uint16_t *cost_mv, int32_t *out, void *stream )               \
    {                                                                                                                \
        if( range < 1 || range > 29 || n < 0 || me_range < 0 || 2 * me_range + 4 > 64 )                              \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_me_esa_argmin<BD>( table, range, n, me_range, nullptr, par, init_cost, cost_mv, out,  \
                                                  (hipStream_t)stream ), "me_esa_argmin" );                          \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_me_esa_argmin_at( const PT<BD>::sadt *table, int range, int n, int me_range,      \
                                                    const int16_t *origin, const int16_t *par,                       \
                                                    const int32_t *init_cost, const uint16_t *cost_mv, int32_t *out, \
                                                    void *stream )                                                   \
    {                                                                                                                \
        if( range < 1 || range > 29 || n < 0 || me_range < 0 || 2 * me_range + 4 > 64 || !origin ||                  \
            range < me_range )                                                                                       \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_me_esa_argmin<BD>( table, range, n, me_range, origin, par, init_cost, cost_mv, out,   \
                                                  (hipStream_t)stream ), "me_esa_argmin_at" );                       \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_ssd_plane_batch( const PT<BD>::pixel *pix1, intptr_t s1, intptr_t f1,             \
                                                   const PT<BD>::pixel *pix2, intptr_t s2, intptr_t f2, int width,   \
                                                   int height, int nframes, uint64_t *ssd, void *stream )            \
    {                                                                                                                \
        if( width < 0 || height < 0 || nframes < 0 || (nframes && (!pix1 || !pix2 || !ssd)) )                       \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_plane_ssd<BD>( 0, pix1, s1, f1, pix2, s2, f2, width, height, nframes, ssd,            \
                                              (hipStream_t)stream ), "ssd_plane_batch" );                            \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_ssd_nv12_batch( const PT<BD>::pixel *pix1, intptr_t s1, intptr_t f1,              \
                                                  const PT<BD>::pixel *pix2, intptr_t s2, intptr_t f2, int width,    \
                                                  int height, int nframes, uint64_t *ssd_uv, void *stream )          \
    {                                                                                                                \
        if( width < 0 || height < 0 || nframes < 0 || (nframes && (!pix1 || !pix2 || !ssd_uv)) )                    \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_plane_ssd<BD>( 1, pix1, s1, f1, pix2, s2, f2, width, height, nframes, ssd_uv,         \
                                              (hipStream_t)stream ), "ssd_nv12_batch" );                             \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_me_search_esa( const PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,           \
                                                 const PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs, int mbw,       \
                                                 int mbh, int nframes, int range, int me_range, const int16_t *par,  \
                                                 const int32_t *init_cost, const uint16_t *cost_mv, int32_t *out,    \
                                                 void *stream )                                                      \
    {                                                                                                                \
        if( mbw < 0 || mbh < 0 || nframes < 0 || !( range == 4 || range == 8 || range == 16 || range == 24 ) ||       \
            me_range < 0 || 2 * me_range + 4 > 64 || range < me_range ||                                            \
            ((int64_t)nframes * mbw * mbh && (!par || !init_cost || !cost_mv || !out)) )                             \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_me_search_esa<BD>( fenc, fs, ffs, ref, rs, rfs, mbw, mbh, nframes, range, me_range,   \
                                                  par, init_cost, cost_mv, out, (hipStream_t)stream ),               \
                        "me_search_esa" );                                                                           \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_me_search_esa8( const PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,          \
                                                  const PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs, int mbw,      \
                                                  int mbh, int nframes, int range, int me_range,                     \
                                                  const int16_t *centre, const int16_t *par,                         \
                                                  const int32_t *init_cost, const uint16_t *cost_mv, int32_t *out,   \
                                                  void *stream )                                                     \
    {                                                                                                                \
        if( mbw < 0 || mbh < 0 || nframes < 0 ||                                                                     \
            !( range == 0 || range == 4 || range == 8 || range == 16 || range == 24 ) || me_range < 0 ||             \
            2 * me_range + 4 > 64 || ((int64_t)nframes * mbw * mbh && (!fenc || !ref || !par || !init_cost ||        \
                                                                       !cost_mv || !out)) )                          \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_me_search_esa8<BD>( fenc, fs, ffs, ref, rs, rfs, mbw, mbh, nframes, range, me_range,  \
                                                   centre, par, init_cost, cost_mv, out, (hipStream_t)stream ),      \
                        "me_search_esa8" );                                                                          \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_me_tesa( const PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,                    \
                                           const PT<BD>::pixel *ref, intptr_t rs, intptr_t rfs,                      \
                                           const uint16_t *integral, intptr_t ifs, int mbw, int mbh, int nframes,    \
                                           int me_range, int satd, const PT<BD>::sadt *table, int range,             \
                                           const int16_t *origin, const int16_t *par, const int32_t *init_cost,      \
                                           const uint16_t *cost_mv, int32_t *out, void *stream )                     \
    {                                                                                                                \
        if( mbw < 0 || mbh < 0 || nframes < 0 || me_range < 1 || me_range > 32 || !fenc || !ref || !integral ||      \
            !par || !init_cost || !cost_mv || !out || ((uintptr_t)fenc & 3) || ((fs * sizeof( PT<BD>::pixel )) & 3) || \
            (table && (range < 1 || range > 29)) )                                                                   \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_me_tesa<BD>( fenc, fs, ffs, ref, rs, rfs, integral, ifs, mbw, mbh, nframes, me_range, \
                                            satd, table, range, origin, par, init_cost, cost_mv, out,               \
                                            (hipStream_t)stream ), "me_tesa" );                                      \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_hpel_filter( const PT<BD>::pixel *src, PT<BD>::pixel *dh, PT<BD>::pixel *dv,       \
                                               PT<BD>::pixel *dc, intptr_t stride, intptr_t fstride, int width,     \
                                               int height, int nframes, void *stream )                              \
    {                                                                                                                \
        if( width <= 0 || height <= 0 || nframes < 0 || (width | height) & 15 )                                      \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_hpel_filter<BD>( src, dh, dv, dc, stride, fstride, width, height, nframes,            \
                                                (hipStream_t)stream ), "hpel_filter" );                              \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_subpel_cmp_batch( int op, int i_pixel, const PT<BD>::pixel *fenc, intptr_t fs,    \
                                                    const PT<BD>::pixel *p0, const PT<BD>::pixel *p1,                \
                                                    const PT<BD>::pixel *p2, const PT<BD>::pixel *p3, intptr_t rs,   \
                                                    const int64_t *fo, const int32_t *qxy, int n, int32_t *scores,   \
                                                    void *stream )                                                   \
    {                                                                                                                \
        if( ( op != X264HIP_CMP_SAD && op != X264HIP_CMP_SATD ) || i_pixel < 0 || i_pixel > 7 || n < 0 )             \
            return X264HIP_EINVAL;                                                                                   \
        const PT<BD>::pixel *planes[4] = { p0, p1, p2, p3 };                                                         \
        return map_err( launch_subpel_cmp<BD>( op, i_pixel, fenc, fs, planes, rs, fo, qxy, n, scores,                \
                                               (hipStream_t)stream ), "subpel_cmp_batch" );                          \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_subpel_qpel9_batch( int op, int i_pixel, const PT<BD>::pixel *fenc, intptr_t fs,  \
                                                      const PT<BD>::pixel *p0, const PT<BD>::pixel *p1,              \
                                                      const PT<BD>::pixel *p2, const PT<BD>::pixel *p3, intptr_t rs, \
                                                      const int64_t *fo, const int32_t *cxy, int n, int32_t *scores, \
                                                      void *stream )                                                 \
    {                                                                                                                \
        if( ( op != X264HIP_CMP_SAD && op != X264HIP_CMP_SATD ) || i_pixel < 0 || i_pixel > 3 || n < 0 ||             \
            ( n > 0 && ( !fenc || !p0 || !p1 || !p2 || !p3 || !fo || !cxy || !scores ) ) )                           \
            return X264HIP_EINVAL;                                                                                   \
        const PT<BD>::pixel *planes[4] = { p0, p1, p2, p3 };                                                         \
        return map_err( launch_subpel_qpel9<BD>( op, i_pixel, fenc, fs, planes, rs, fo, cxy, n, scores,              \
                                                 (hipStream_t)stream ), "subpel_qpel9_batch" );                      \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_me_refine_subpel( const PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,          \
                                                    const PT<BD>::pixel *p0, const PT<BD>::pixel *p1,                \
                                                    const PT<BD>::pixel *p2, const PT<BD>::pixel *p3, intptr_t rs,   \
                                                    intptr_t rfs, int i_pixel, int subme, int refine_qpel,           \
                                                    int fpel_satd, const int32_t *pos, const int16_t *par,           \
                                                    const int32_t *init_cost, const uint16_t *cost_mv, int n,        \
                                                    int32_t *out, int32_t *nevals, void *stream )                    \
    {                                                                                                                \
        if( i_pixel < 0 || i_pixel > 6 || subme < 1 || subme > 11 || n < 0 ||                                        \
            ( n > 0 && ( !fenc || !p0 || !p1 || !p2 || !p3 || !pos || !par || !init_cost || !cost_mv || !out ) ) )   \
            return X264HIP_EINVAL;                                                                                   \
        const PT<BD>::pixel *planes[4] = { p0, p1, p2, p3 };                                                         \
        return map_err( launch_me_refine_subpel<BD>( fenc, fs, ffs, planes, rs, rfs, i_pixel, subme, !!refine_qpel,  \
                                                     fpel_satd, pos, par, init_cost, cost_mv, n, out, nevals,       \
                                                     nullptr, nullptr, nullptr, (hipStream_t)stream ),               \
                        "me_refine_subpel" );                                                                        \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_me_refine_subpel_ex( const PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,       \
                                                       const PT<BD>::pixel *p0, const PT<BD>::pixel *p1,             \
                                                       const PT<BD>::pixel *p2, const PT<BD>::pixel *p3,             \
                                                       intptr_t rs, intptr_t rfs, int i_pixel, int subme,            \
                                                       int refine_qpel, int fpel_satd, const int32_t *pos,           \
                                                       const int16_t *par, const int32_t *init_cost,                 \
                                                       const uint16_t *cost_mv, int n, int32_t *out,                 \
                                                       int32_t *nevals, const x264hip_refine_ext_t *ext,             \
                                                       void *stream )                                                \
    {                                                                                                                \
        if( i_pixel < 0 || i_pixel > 6 || subme < 1 || subme > 11 || n < 0 ||                                        \
            ( n > 0 && ( !fenc || !p0 || !p1 || !p2 || !p3 || !pos || !par || !init_cost || !cost_mv || !out ) ) )   \
            return X264HIP_EINVAL;                                                                                   \
        const PT<BD>::pixel *planes[4] = { p0, p1, p2, p3 };                                                         \
        return map_err( launch_me_refine_subpel<BD>( fenc, fs, ffs, planes, rs, rfs, i_pixel, subme, !!refine_qpel,  \
                                                     fpel_satd, pos, par, init_cost, cost_mv, n, out, nevals,       \
                                                     nullptr, nullptr, ext, (hipStream_t)stream ),                   \
                        "me_refine_subpel_ex" );                                                                     \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_me_refine_qpel_refdupe( const PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,    \
                                                          const PT<BD>::pixel *p0, const PT<BD>::pixel *p1,          \
                                                          const PT<BD>::pixel *p2, const PT<BD>::pixel *p3,          \
                                                          intptr_t rs, intptr_t rfs, int i_pixel, int subme,         \
                                                          int fpel_satd, const int32_t *pos, const int16_t *par,     \
                                                          const int32_t *init_cost, const uint16_t *cost_mv, int n,  \
                                                          int32_t *out, int32_t *nevals, int32_t *halfpel_thresh,    \
                                                          const int32_t *ref_cost, const x264hip_refine_ext_t *ext,  \
                                                          void *stream )                                             \
    {                                                                                                                \
        if( i_pixel < 0 || i_pixel > 6 || subme < 1 || subme > 11 || n < 0 ||                                        \
            ( n > 0 && ( !fenc || !p0 || !p1 || !p2 || !p3 || !pos || !par || !init_cost || !cost_mv || !out ) ) )   \
            return X264HIP_EINVAL;                                                                                   \
        const PT<BD>::pixel *planes[4] = { p0, p1, p2, p3 };                                                         \
        return map_err( launch_me_refine_subpel<BD>( fenc, fs, ffs, planes, rs, rfs, i_pixel, subme, 2, fpel_satd,   \
                                                     pos, par, init_cost, cost_mv, n, out, nevals, halfpel_thresh,  \
                                                     ref_cost, ext, (hipStream_t)stream ),                           \
                        "me_refine_qpel_refdupe" );                                                                  \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_me_search_ref( const PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,              \
                                                 const PT<BD>::pixel *fw, const PT<BD>::pixel *p0,                   \
                                                 const PT<BD>::pixel *p1, const PT<BD>::pixel *p2,                   \
                                                 const PT<BD>::pixel *p3, intptr_t rs, intptr_t rfs, int i_pixel,    \
                                                 int me_method, int subme, int me_range, const int32_t *pos,         \
                                                 const int16_t *par, const int16_t *mvc, const uint16_t *cost_mv,    \
                                                 int n, int32_t *out, int32_t *nevals,                               \
                                                 const x264hip_refine_ext_t *ext, void *stream )                     \
    {                                                                                                                \
        if( n < 0 || ( n > 0 && ( !fenc || !fw || !p0 || !p1 || !p2 || !p3 || !pos || !par || !mvc || !cost_mv ||   \
                                  !out ) ) )                                                                         \
            return X264HIP_EINVAL;                                                                                   \
        const PT<BD>::pixel *planes[4] = { p0, p1, p2, p3 };                                                         \
        return map_err( launch_me_search_ref<BD>( fenc, fs, ffs, fw, planes, rs, rfs, i_pixel, me_method, subme,     \
                                                  me_range, pos, par, mvc, cost_mv, n, out, nevals, nullptr,         \
                                                  nullptr, ext, (hipStream_t)stream ), "me_search_ref" );            \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_me_analyse_p16x16(                                                              \
        const PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs, const PT<BD>::pixel *fw, const PT<BD>::pixel *p0,       \
        const PT<BD>::pixel *p1, const PT<BD>::pixel *p2, const PT<BD>::pixel *p3, intptr_t rs, intptr_t rfs,         \
        int mbw, int mbh, int nframes, int me_method, int subme, int me_range, int mv_range,                         \
        const int16_t *lowres_mv, const int16_t *ref_mv, int ref_mv_scale, const uint16_t *cost_mv, int32_t *out,    \
        int32_t *nevals, const x264hip_refine_ext_t *ext, void *stream )                                             \
    {                                                                                                                \
        if( mbw < 0 || mbh < 0 || nframes < 0 || mv_range < 1 || mv_range > 8192 ||                                  \
            ( (int64_t)mbw * mbh * nframes > 0 && ( !fenc || !fw || !p0 || !p1 || !p2 || !p3 || !cost_mv || !out ) ) ) \
            return X264HIP_EINVAL;                                                                                   \
        const PT<BD>::pixel *planes[4] = { p0, p1, p2, p3 };                                                         \
        return map_err( launch_me_analyse_p16x16<BD>( fenc, fs, ffs, fw, planes, rs, rfs, mbw, mbh, nframes,         \
                                                      me_method, subme, me_range, mv_range, lowres_mv, ref_mv,       \
                                                      ref_mv_scale, cost_mv, out, nevals, ext, (hipStream_t)stream ), \
                        "me_analyse_p16x16" );                                                                       \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_me_refine_bidir_satd(                                                           \
        const PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs, const PT<BD>::pixel *l0f, const PT<BD>::pixel *l0h,     \
        const PT<BD>::pixel *l0v, const PT<BD>::pixel *l0c, const PT<BD>::pixel *l1f, const PT<BD>::pixel *l1h,       \
        const PT<BD>::pixel *l1v, const PT<BD>::pixel *l1c, intptr_t rs, intptr_t rfs, int i_pixel, int mbcmp_satd,   \
        const int32_t *pos, const int16_t *par, const int32_t *weight, const uint16_t *cost_mv, int n, int32_t *out,  \
        int32_t *cost, int32_t *nevals, void *stream )                                                               \
    {                                                                                                                \
        if( i_pixel < 0 || i_pixel > 3 || n < 0 ||                                                                   \
            ( n > 0 && ( !fenc || !l0f || !l0h || !l0v || !l0c || !l1f || !l1h || !l1v || !l1c || !pos || !par ||     \
                         !weight || !cost_mv || !out ) ) )                                                           \
            return X264HIP_EINVAL;                                                                                   \
        const PT<BD>::pixel *p0[4] = { l0f, l0h, l0v, l0c }, *p1[4] = { l1f, l1h, l1v, l1c };                        \
        return map_err( launch_me_refine_bidir<BD>( fenc, fs, ffs, p0, p1, rs, rfs, i_pixel, mbcmp_satd, pos, par,   \
                                                    weight, cost_mv, n, out, cost, nevals, (hipStream_t)stream ),    \
                        "me_refine_bidir_satd" );                                                                    \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_me_search_ref_thresh( const PT<BD>::pixel *fenc, intptr_t fs, intptr_t ffs,       \
                                                        const PT<BD>::pixel *fw, const PT<BD>::pixel *p0,            \
                                                        const PT<BD>::pixel *p1, const PT<BD>::pixel *p2,            \
                                                        const PT<BD>::pixel *p3, intptr_t rs, intptr_t rfs,          \
                                                        int i_pixel, int me_method, int subme, int me_range,         \
                                                        const int32_t *pos, const int16_t *par, const int16_t *mvc,  \
                                                        const uint16_t *cost_mv, int n, int32_t *out,                \
                                                        int32_t *nevals, int32_t *halfpel_thresh,                    \
                                                        const int32_t *ref_cost, const x264hip_refine_ext_t *ext,    \
                                                        void *stream )                                               \
    {                                                                                                                \
        if( n < 0 || ( n > 0 && ( !fenc || !fw || !p0 || !p1 || !p2 || !p3 || !pos || !par || !mvc || !cost_mv ||   \
                                  !out ) ) )                                                                         \
            return X264HIP_EINVAL;                                                                                   \
        const PT<BD>::pixel *planes[4] = { p0, p1, p2, p3 };                                                         \
        return map_err( launch_me_search_ref<BD>( fenc, fs, ffs, fw, planes, rs, rfs, i_pixel, me_method, subme,     \
                                                  me_range, pos, par, mvc, cost_mv, n, out, nevals, halfpel_thresh,  \
                                                  ref_cost, ext, (hipStream_t)stream ), "me_search_ref_thresh" );    \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_sub_dct_batch( int kind, const PT<BD>::pixel *fenc, intptr_t fs,                  \
                                                 const PT<BD>::pixel *fdec, intptr_t ds, const int64_t *fo,          \
                                                 const int64_t *dofs, int n, PT<BD>::dctcoef *dct, void *stream )    \
    {                                                                                                                \
        if( kind < 0 || kind > 6 || n < 0 )                                                                          \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_sub_dct<BD>( kind, fenc, fs, fdec, ds, fo, dofs, n, dct, (hipStream_t)stream ),      \
                        "sub_dct_batch" );                                                                           \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_dc_batch( int kind, PT<BD>::dctcoef *dct, PT<BD>::dctcoef *dct4x4, int n,         \
                                            void *stream )                                                           \
    {                                                                                                                \
        if( kind < 0 || kind > 2 || n < 0 || ( kind == 1 && !dct4x4 ) )                                              \
            return X264HIP_EINVAL;                                                                                   \
        if( kind == X264HIP_DC_I4x4 )                                                                                \
            return map_err( launch_idct4x4dc<BD>( dct, n, (hipStream_t)stream ), "dc_batch" );                       \
        return map_err( launch_dc<BD>( kind, dct, dct4x4, n, (hipStream_t)stream ), "dc_batch" );                  \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_add_idct_batch( int kind, PT<BD>::pixel *dst, intptr_t ds, const int64_t *doff,    \
                                                  const PT<BD>::dctcoef *dct, int n, void *stream )                  \
    {                                                                                                                \
        if( kind < 0 || kind > 6 || n < 0 )                                                                          \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_add_idct<BD>( kind, dst, ds, doff, dct, n, (hipStream_t)stream ), "add_idct_batch" ); \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_dequant_batch( int kind, PT<BD>::dctcoef *dct, const int32_t *dmf,                 \
                                                 const int32_t *qp, int n, void *stream )                            \
    {                                                                                                                \
        if( kind < 0 || kind > 2 || n < 0 )                                                                          \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_dequant<BD>( kind, dct, dmf, qp, n, (hipStream_t)stream ), "dequant_batch" );         \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_idct_dequant_2x4_batch( int dconly, PT<BD>::dctcoef *dct,                           \
                                                          PT<BD>::dctcoef *dct4x4, const int32_t *dmf,               \
                                                          const int32_t *qp, int n, void *stream )                   \
    {                                                                                                                \
        if( n < 0 || ( !dconly && !dct4x4 ) )                                                                        \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_idct_dequant_2x4<BD>( dconly, dct, dct4x4, dmf, qp, n, (hipStream_t)stream ),         \
                        "idct_dequant_2x4_batch" );                                                                  \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_optimize_chroma_dc_batch( int c422, PT<BD>::dctcoef *dct, const int32_t *dmf,      \
                                                            int n, int32_t *nz, void *stream )                       \
    {                                                                                                                \
        if( n < 0 )                                                                                                  \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_optimize_chroma<BD>( c422, dct, dmf, n, nz, (hipStream_t)stream ),                    \
                        "optimize_chroma_dc_batch" );                                                                \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_denoise_dct_batch( PT<BD>::dctcoef *dct, int size, int n, uint32_t *sum,           \
                                                     const PT<BD>::udctcoef *offset, void *stream )                  \
    {                                                                                                                \
        if( n < 0 || size < 0 )                                                                                      \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_denoise<BD>( dct, size, n, sum, offset, (hipStream_t)stream ), "denoise_dct_batch" ); \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_coef_stat_batch( int kind, const PT<BD>::dctcoef *dct, int64_t pitch, int n,       \
                                                   int32_t *out, void *stream )                                      \
    {                                                                                                                \
        if( kind < 0 || kind > 7 || n < 0 )                                                                          \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_coef_stat<BD>( kind, dct, pitch, n, out, (hipStream_t)stream ), "coef_stat_batch" );  \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_coeff_level_run_batch( int num, const PT<BD>::dctcoef *dct, int64_t pitch, int n,  \
                                                         int32_t *last, int32_t *mask, int32_t *count,               \
                                                         PT<BD>::dctcoef *level, void *stream )                      \
    {                                                                                                                \
        if( !( num == 4 || num == 8 || num == 15 || num == 16 ) || n < 0 )                                           \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_level_run<BD>( num, dct, pitch, n, last, mask, count, level, (hipStream_t)stream ),    \
                        "coeff_level_run_batch" );                                                                   \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_zigzag_scan_batch( int size, int field, PT<BD>::dctcoef *level,                    \
                                                     const PT<BD>::dctcoef *dct, int n, void *stream )               \
    {                                                                                                                \
        if( !( size == 4 || size == 8 ) || n < 0 )                                                                   \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_zigzag_scan<BD>( size, field ? 1 : 0, level, dct, n, (hipStream_t)stream ),          \
                        "zigzag_scan_batch" );                                                                       \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_zigzag_sub_batch( int kind, int field, PT<BD>::dctcoef *level,                     \
                                                    PT<BD>::dctcoef *dc, const PT<BD>::pixel *src, intptr_t ss,      \
                                                    PT<BD>::pixel *dst, intptr_t ds, const int64_t *so,              \
                                                    const int64_t *dso, int n, int32_t *nz, void *stream )           \
    {                                                                                                                \
        if( kind < 0 || kind > 2 || n < 0 || ( kind == 1 && !dc ) )                                                  \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_zigzag_sub<BD>( kind, field ? 1 : 0, level, dc, src, ss, dst, ds, so, dso, n, nz,      \
                                               (hipStream_t)stream ), "zigzag_sub_batch" );                          \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_zigzag_interleave_batch( PT<BD>::dctcoef *dst, const PT<BD>::dctcoef *src,         \
                                                           uint8_t *nnz, int n, void *stream )                       \
    {                                                                                                                \
        if( n < 0 )                                                                                                  \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_interleave<BD>( dst, src, nnz, n, (hipStream_t)stream ), "zigzag_interleave_batch" ); \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_frame_init_lowres( const PT<BD>::pixel *src, intptr_t stride, intptr_t fstride,   \
                                                     int width, int height, int nframes,                             \
                                                     PT<BD>::pixel *const dst[4], intptr_t ds, intptr_t dfs,         \
                                                     void *stream )                                                  \
    {                                                                                                                \
        if( width < 2 || height < 2 || nframes < 0 || !dst || ( (width / 2 + 64) % PT<BD>::PPD ) ||                 \
            ( (ds * (intptr_t)sizeof(PT<BD>::pixel)) & 3 ) || ( ( (uintptr_t)dst[0] | (uintptr_t)dst[1] |             \
                                                                    (uintptr_t)dst[2] | (uintptr_t)dst[3] ) & 3 ) )  \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_frame_init_lowres<BD>( src, stride, fstride, width, height, nframes, dst, ds, dfs,     \
                                                      (hipStream_t)stream ), "frame_init_lowres" );                  \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_ssim_bands( const PT<BD>::pixel *p1, intptr_t s1, intptr_t f1,                    \
                                              const PT<BD>::pixel *p2, intptr_t s2, intptr_t f2, int width,          \
                                              const int32_t *bands, int n_bands, int n_frames, float *ssim,          \
                                              void *stream )                                                         \
    {                                                                                                                \
        if( width < 0 || width > 8192 || n_bands < 0 || n_frames < 0 ||                                             \
            ( n_bands > 0 && n_frames > 0 && ( !p1 || !p2 || !bands || !ssim ) ) )                                   \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_ssim_bands<BD>( p1, s1, f1, p2, s2, f2, width, bands, n_bands, n_frames, ssim,        \
                                               (hipStream_t)stream ), "ssim_bands" );                                \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_ssim_wxh( const PT<BD>::pixel *p1, intptr_t s1, const PT<BD>::pixel *p2,          \
                                            intptr_t s2, int width, int height, float *ssim, int *cnt,              \
                                            void *stream )                                                           \
    {                                                                                                                \
        if( width < 0 || height < 0 || !ssim || ( width >= 8 && height >= 8 && ( !p1 || !p2 ) ) )                   \
            return X264HIP_EINVAL;                                                                                   \
        if( cnt )                                                                                                    \
            *cnt = ( (height >> 2) - 1 ) * ( (width >> 2) - 1 );                                                     \
        return map_err( launch_ssim_wxh<BD>( p1, s1, p2, s2, width, height, ssim, (hipStream_t)stream ),             \
                        "ssim_wxh" );                                                                                \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_frame_pixel_stats( const PT<BD>::pixel *luma, intptr_t ls,                        \
                                                     const PT<BD>::pixel *cu, const PT<BD>::pixel *cv, intptr_t cs,  \
                                                     int mbw, int mbh, int cf, uint64_t *stats, void *stream )       \
    {                                                                                                                \
        if( mbw < 0 || mbh < 0 || cf < 0 || cf > 3 || !stats || ( mbw * mbh > 0 && !luma ) ||                        \
            ( mbw * mbh > 0 && cf && !cu ) || ( mbw * mbh > 0 && cf == 3 && !cv ) )                                  \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_frame_stats<BD>( luma, ls, cu, cv, cs, mbw, mbh, cf, stats, (hipStream_t)stream ),   \
                        "frame_pixel_stats" );                                                                       \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_weight_cost_batch( int kind, const PT<BD>::pixel *fenc,                           \
                                                     const PT<BD>::pixel *const ref[4], intptr_t stride, int mbw,    \
                                                     int mbh, const uint16_t *intra, const int16_t *mvs, int satd,   \
                                                     int plane, int lambda, int n_slices,                            \
                                                     const x264hip_weight_t *cands, int n, uint32_t *costs,          \
                                                     void *stream )                                                  \
    {                                                                                                                \
        if( kind < 0 || kind > 3 || mbw < 0 || mbh < 0 || n < 0 || lambda < 0 || n_slices < 1 ||                     \
            ( (kind == 1 || kind == 2) && ( plane < 0 || plane > 1 ) ) )                                             \
            return X264HIP_EINVAL;                                                                                   \
        if( n > 0 && ( !cands || !costs ) )                                                                          \
            return X264HIP_EINVAL;                                                                                   \
        for( int i = 0; i < n; i++ )                                                                                 \
            if( cands[i].weighted && ( cands[i].scale < 0 || cands[i].scale > 255 || cands[i].denom < 0 ||          \
                                       cands[i].denom > 7 || cands[i].offset < -128 || cands[i].offset > 127 ) )     \
                return X264HIP_EINVAL;                                                                               \
        if( n > 0 && mbw * mbh > 0 &&                                                                                \
            ( !fenc || !ref || !ref[0] || ( kind == 0 && !intra ) ||                                                 \
              ( kind == 0 && mvs && ( !ref[1] || !ref[2] || !ref[3] ) ) ) )                                          \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_weight_cost<BD>( kind, fenc, stride, ref, stride, mbw, mbh, intra, mvs, satd,        \
                                                kind == 1 || kind == 2 ? plane : 0, lambda, n_slices, cands, n,      \
                                                costs, (hipStream_t)stream ), "weight_cost_batch" );                 \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_weights_analyse(                                                                 \
        const PT<BD>::pixel *fenc_lr, const PT<BD>::pixel *const ref_lr[4], intptr_t lrs, int mbw, int mbh,          \
        const uint16_t *intra, const int16_t *mvs, int cf, const PT<BD>::pixel *const fenc_c[2],                     \
        const PT<BD>::pixel *const ref_c[2], intptr_t cs, const uint32_t fsum[3], const uint64_t fssd[3],            \
        const uint32_t rsum[3], const uint64_t rssd[3], int b_lookahead, int subme, int satd, int lambda,            \
        int n_slices, int weightp_fake, PT<BD>::pixel *wlr, x264hip_weight_t weights[3], float *cost_delta,          \
        void *stream )                                                                                               \
    {                                                                                                                \
        if( mbw <= 0 || mbh <= 0 || cf < 0 || cf > 3 || subme < 0 || subme > 11 || lambda < 0 || n_slices < 1 ||     \
            !fenc_lr || !ref_lr || !ref_lr[0] || !intra || !fsum || !fssd || !rsum || !rssd || !weights ||           \
            ( mvs && ( !ref_lr[1] || !ref_lr[2] || !ref_lr[3] ) ) ||                                                 \
            ( !b_lookahead && cf && ( !fenc_c || !ref_c || !fenc_c[0] || !ref_c[0] ||                                \
                                      ( cf == 3 && ( !fenc_c[1] || !ref_c[1] ) ) ) ) )                               \
            return X264HIP_EINVAL;                                                                                   \
        WpInput<BD> in;                                                                                              \
        memset( &in, 0, sizeof( in ) );                                                                              \
        in.fenc_lr = fenc_lr;                                                                                        \
        for( int i = 0; i < 4; i++ )                                                                                 \
            in.ref_lr[i] = ref_lr[i];                                                                                \
        in.lrs = lrs; in.mbw = mbw; in.mbh = mbh; in.intra = intra; in.mvs = mvs; in.cf = cf;                        \
        if( !b_lookahead && cf )                                                                                     \
            for( int i = 0; i < 2; i++ )                                                                             \
            {                                                                                                        \
                in.fenc_c[i] = fenc_c[i];                                                                            \
                in.ref_c[i] = ref_c[i];                                                                              \
            }                                                                                                        \
        in.cs = cs;                                                                                                  \
        for( int i = 0; i < 3; i++ )                                                                                 \
        {                                                                                                            \
            in.fenc_sum[i] = fsum[i]; in.ref_sum[i] = rsum[i];                                                       \
            in.fenc_ssd[i] = fssd[i]; in.ref_ssd[i] = rssd[i];                                                       \
        }                                                                                                            \
        in.b_lookahead = !!b_lookahead; in.subme = subme; in.satd = satd; in.lambda = lambda;                        \
        in.numslices = n_slices; in.weightp_fake = weightp_fake;                                                     \
        return map_err( weights_analyse<BD>( in, weights, cost_delta, wlr, (hipStream_t)stream ),                    \
                        "weights_analyse" );                                                                         \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_mb_dequant_idct_add( int transform, const PT<BD>::dctcoef *dct, int mbw, int mbh,  \
                                                       int nframes, const int32_t *dmf, const int32_t *qp,           \
                                                       const PT<BD>::pixel *pred, intptr_t ps, intptr_t pfs,         \
                                                       PT<BD>::pixel *recon, intptr_t rs, intptr_t rfs,              \
                                                       void *stream )                                                \
    {                                                                                                                \
        if( !( transform == 4 || transform == 8 ) || mbw < 0 || mbh < 0 || nframes < 0 )                             \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_mb_recon<BD>( transform, dct, mbw, mbh, nframes, dmf, qp, pred, ps, pfs, recon, rs,   \
                                             rfs, (hipStream_t)stream ), "mb_dequant_idct_add" );                    \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_quant_batch( int kind, PT<BD>::dctcoef *dct, const PT<BD>::udctcoef *mf,          \
                                               const PT<BD>::udctcoef *bias, int n, int32_t *nz, void *stream )      \
    {                                                                                                                \
        if( kind < 0 || kind > 2 || n < 0 )                                                                          \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_quant<BD>( kind, dct, mf, bias, 0, 0, n, nz, (hipStream_t)stream ), "quant_batch" ); \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_quant_dc_batch( int kind, PT<BD>::dctcoef *dct, int mf, int bias, int n,          \
                                                  int32_t *nz, void *stream )                                        \
    {                                                                                                                \
        if( kind < 3 || kind > 4 || n < 0 )                                                                          \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_quant<BD>( kind, dct, nullptr, nullptr, mf, bias, n, nz, (hipStream_t)stream ),      \
                        "quant_dc_batch" );                                                                          \
    }                                                                                                                \
    extern "C" int x264hip_##BD##_mb_dct_quant( int transform, const PT<BD>::pixel *fenc, intptr_t fs,              \
                                                intptr_t ffs, const PT<BD>::pixel *pred, intptr_t ps, intptr_t pfs,  \
                                                int mbw, int mbh, int nframes, const PT<BD>::udctcoef *mf,          \
                                                const PT<BD>::udctcoef *bias, PT<BD>::dctcoef *dct, int32_t *nz,     \
                                                void *stream )                                                       \
    {                                                                                                                \
        if( ( transform != 4 && transform != 8 ) || mbw < 0 || mbh < 0 || nframes < 0 )                              \
            return X264HIP_EINVAL;                                                                                   \
        return map_err( launch_mb_dct_quant<BD>( transform, fenc, fs, ffs, pred, ps, pfs, mbw, mbh, nframes, mf,    \
                                                 bias, dct, nz, (hipStream_t)stream ), "mb_dct_quant" );            \
    }

DEFINE_ENTRIES( 8 )
DEFINE_ENTRIES( 10 )

// dequant4_mf / dequant8_mf of x264_cqm_init, reference common/set.c:31-39,
// 52-61, 124-159 (host-side table set-up, the input of the dequant entries)
static const uint8_t k_dequant4_scale[6][3] = {
    { 10, 13, 16 }, { 11, 14, 18 }, { 13, 16, 20 }, { 14, 18, 23 }, { 16, 20, 25 }, { 18, 23, 29 } };
static const uint8_t k_dequant8_scale[6][6] = {
    { 20, 18, 32, 19, 25, 24 }, { 22, 19, 35, 21, 28, 26 }, { 26, 23, 42, 24, 33, 31 },
    { 28, 25, 45, 26, 35, 33 }, { 32, 28, 51, 30, 40, 38 }, { 36, 32, 58, 34, 46, 43 } };
static const uint8_t k_quant8_scan16[16] = { 0, 3, 4, 3, 3, 1, 5, 1, 4, 5, 2, 5, 3, 1, 5, 1 };

extern "C" void x264hip_cqm_dequant( const uint8_t *const sl[8], int b8, int32_t *dq4, int32_t *dq8 )
{
    for( int q = 0; q < 6; q++ )
    {
        for( int l = 0; l < 4; l++ )
            for( int i = 0; i < 16; i++ )
                dq4[(l * 6 + q) * 16 + i] = k_dequant4_scale[q][(i & 1) + ((i >> 2) & 1)] * sl[l][i];
        if( b8 )
            for( int l = 0; l < 2; l++ )
                for( int i = 0; i < 64; i++ )
                    dq8[(l * 6 + q) * 64 + i] =
                        k_dequant8_scale[q][k_quant8_scan16[((i >> 1) & 12) | (i & 3)]] * sl[4 + l][i];
    }
}
