// Measures the chip-wide issue rate of v_sad_u8 / v_sad_u16 / v_add_u32 on
// gfx950 (the denominator of the SAD roofline in bench.py).  8 independent
// accumulation chains per lane, 4096 iterations, every CU busy.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t seed, uint32_t *out, int iters)
{
    uint32_t a = seed ^ threadIdx.x, b = seed * 2654435761u + blockIdx.x;
    uint32_t acc[8];
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = i;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int j = 0; j < 16; j++)
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (OP == 0) acc[i] = __builtin_amdgcn_sad_u8(a + i, b + j, acc[i]);
                else if (OP == 1) acc[i] = __builtin_amdgcn_sad_u16(a + i, b + j, acc[i]);
                else acc[i] = acc[i] + (a ^ (b + j + i));
            }
        a = a * 1664525u + 1013904223u;
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s += acc[i];
    if (s == 0x12345678) out[0] = s;
}

int main()
{
    uint32_t *out; hipMalloc(&out, 4);
    int blocks = 256 * 8, iters = 4096;
    const char *names[3] = {"v_sad_u8", "v_sad_u16", "v_add+xor(ref)"};
    for (int op = 0; op < 3; op++) {
        hipEvent_t s, e; hipEventCreate(&s); hipEventCreate(&e);
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(s);
            if (op == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, 1u, out, iters);
            if (op == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, 1u, out, iters);
            if (op == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, 1u, out, iters);
            hipEventRecord(e); hipEventSynchronize(e);
            float ms; hipEventElapsedTime(&ms, s, e);
            double ops = (double)blocks * 256 * iters * 16 * 8;
            if (rep == 2) printf("%-16s %.1f T lane-ops/s (%.3f ms)\n", names[op], ops / (ms * 1e-3) / 1e12, ms);
        }
    }
    return 0;
}
