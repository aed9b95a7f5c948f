// Probe of the vector-memory address path on gfx950: time per wave-instruction of
// global loads whose 64 lanes read consecutive 8-byte pieces (the qpel list kernel's
// row loads), by load width and alignment.  L1-resident footprint (16 KiB), 8 waves
// per SIMD on every CU.  Prints ns and CU-cycles (at the measured-under-load
// 2.1 GHz) per wave-instruction per CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

// plain loads at 16 distinct row addresses per iteration (nothing to merge or CSE);
// the ISA of every mode is checked to hold exactly the intended load width
template <int MODE> __device__ __forceinline__ uint32_t ld( const uint8_t *p )
{
    if constexpr (MODE == 0 || MODE == 7) {
        const uint2 v = *(const uint2 *)p; return v.x + v.y;
    } else if constexpr (MODE == 1) {
        uint2 v; __builtin_memcpy(&v, p, 8); return v.x + v.y;
    } else if constexpr (MODE == 2) {
        const uint32_t *q = (const uint32_t *)p;
        typedef uint32_t u3 __attribute__((ext_vector_type(3)));
        const u3 v = *(const u3 *)q; return v.x + v.y + v.z;
    } else if constexpr (MODE == 3 || MODE == 5) {
        const uint4 v = *(const uint4 *)p; return v.x + v.y + v.z + v.w;
    } else if constexpr (MODE == 6) {
        uint4 v; __builtin_memcpy(&v, p, 16); return v.x + v.y + v.z + v.w;
    } else {
        return *(const uint32_t *)p;
    }
}

template <int MODE>
__global__ __launch_bounds__(256) void probe(const uint8_t *buf, uint32_t *out, int iters)
{
    const int lane = threadIdx.x & 63;
    // per-lane byte offset inside a 1 KiB row: 0 dwordx2 aligned (8 B apart), 1 dwordx2 +1,
    // 2 dwordx3 dword-aligned (8 B apart), 3 dwordx4 dword-aligned (8 B apart), 4 dword (4 B apart),
    // 5 dwordx4 aligned (16 B apart), 6 dwordx4 +1 (16 B apart), 7 dwordx2 with 9 lanes per address
    const int off = MODE == 0 ? 8 * lane : MODE == 1 ? 8 * lane + 1 : MODE == 2 || MODE == 3 ? 8 * lane
                  : MODE == 4 ? 4 * lane : MODE == 5 ? 16 * lane : MODE == 6 ? 16 * lane + 1 : 8 * (lane / 9);
    uint32_t acc = 0;
    for (int it = 0; it < iters; it++) {
        uint32_t v[16];
#pragma unroll
        for (int r = 0; r < 16; r++)
            v[r] = ld<MODE>(buf + (((r + it) & 15) << 10) + off);
#pragma unroll
        for (int r = 0; r < 16; r++)
            acc += v[r];
    }
    if (acc == 0x9e3779b9u) out[0] = acc;
}

template <int MODE>
static void run(const uint8_t *buf, uint32_t *out, const char *name)
{
    const int blocks = 256 * 8, iters = 200;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int w = 0; w < 3; w++) hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, buf, out, iters);
    hipEventRecord(a);
    const int reps = 5;
    for (int w = 0; w < reps; w++) hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, buf, out, iters);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    const double instr_per_cu = (double)blocks * 4 * iters * 16 / 256;
    printf("%-40s %8.3f ms  %6.2f ns  %6.1f cyc@2.1GHz per wave-load per CU\n", name, ms,
           ms * 1e6 / instr_per_cu, ms * 1e-3 * 2.1e9 / instr_per_cu);
}

int main()
{
    uint8_t *buf; uint32_t *out;
    hipMalloc(&buf, 1 << 20); hipMalloc(&out, 64);
    hipMemset(buf, 7, 1 << 20);
    run<0>(buf, out, "dwordx2 aligned, 8 B/lane contiguous");
    run<1>(buf, out, "dwordx2 +1 misaligned");
    run<2>(buf, out, "dwordx3 dword-aligned + alignbyte");
    run<3>(buf, out, "dwordx4 dword-aligned + alignbyte");
    run<4>(buf, out, "dword aligned, 4 B/lane");
    run<5>(buf, out, "dwordx4 aligned, 16 B/lane");
    run<6>(buf, out, "dwordx4 +1 misaligned, 16 B/lane");
    run<7>(buf, out, "dwordx2, 9 lanes per address");
    return 0;
}
