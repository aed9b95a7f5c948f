// Probe of v_qsad_pk_u16_u8 / v_mqsad_u32_u8 on gfx950: exact semantics
// (compared on the host with a model) and chip-wide issue rate.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

__global__ void sem(const uint64_t *s0, const uint32_t *s1, const uint64_t *s2, uint64_t *o, uint32_t *mo, int n)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    o[i] = __builtin_amdgcn_qsad_pk_u16_u8(s0[i], s1[i], s2[i]);
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    u4 acc = {(uint32_t)s2[i], (uint32_t)(s2[i] >> 32), 7u, 9u};
    u4 r = __builtin_amdgcn_mqsad_u32_u8(s0[i], s1[i], acc);
    mo[4 * i + 0] = r.x; mo[4 * i + 1] = r.y; mo[4 * i + 2] = r.z; mo[4 * i + 3] = r.w;
}

template <int OP>
__global__ __launch_bounds__(256) void rate(uint32_t seed, uint32_t *out, int iters)
{
    uint64_t a = seed ^ threadIdx.x;
    uint32_t b = seed * 2654435761u + blockIdx.x;
    uint64_t acc[8];
    for (int i = 0; i < 8; i++) acc[i] = i;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int j = 0; j < 16; j++)
#pragma unroll
            for (int i = 0; i < 8; i++)
                acc[i] = __builtin_amdgcn_qsad_pk_u16_u8(a + i, b + j, acc[i]);
        a = a * 1664525u + 1013904223u;
    }
    uint64_t s = 0;
    for (int i = 0; i < 8; i++) s += acc[i];
    if (s == 0x12345678) out[0] = (uint32_t)s;
}

static uint64_t model_qsad(uint64_t s0, uint32_t s1, uint64_t s2)
{
    uint64_t d = 0;
    for (int k = 0; k < 4; k++) {
        uint32_t acc = (s2 >> (16 * k)) & 0xffff;
        for (int b = 0; b < 4; b++) {
            int x = (s0 >> (8 * (k + b))) & 0xff, y = (s1 >> (8 * b)) & 0xff;
            acc += abs(x - y);
        }
        d |= (uint64_t)(acc & 0xffff) << (16 * k);
    }
    return d;
}

int main()
{
    const int n = 1 << 16;
    uint64_t *s0, *s2, *o; uint32_t *s1, *mo;
    hipMallocManaged(&s0, n * 8); hipMallocManaged(&s2, n * 8); hipMallocManaged(&o, n * 8);
    hipMallocManaged(&s1, n * 4); hipMallocManaged(&mo, n * 16);
    srand(1);
    for (int i = 0; i < n; i++) {
        s0[i] = ((uint64_t)rand() << 40) ^ ((uint64_t)rand() << 20) ^ rand();
        s1[i] = rand() ^ (rand() << 16);
        uint64_t acc = 0;
        for (int k = 0; k < 4; k++) acc |= (uint64_t)(rand() % (i < n / 2 ? 60000 : 65536)) << (16 * k);
        s2[i] = acc;
        if (i % 7 == 0) { s0[i] = 0; }
        if (i % 11 == 0) { s1[i] = 0xffffffffu; }
    }
    hipLaunchKernelGGL(sem, dim3(n / 256), dim3(256), 0, 0, s0, s1, s2, o, mo, n);
    hipDeviceSynchronize();
    int bad = 0, badhi = 0;
    for (int i = 0; i < n; i++) {
        uint64_t m = model_qsad(s0[i], s1[i], s2[i]);
        if (m != o[i]) { if (i < n / 2) bad++; else badhi++; if (bad + badhi < 4) printf("mismatch %d: s0=%016llx s1=%08x s2=%016llx hw=%016llx model=%016llx\n", i, (unsigned long long)s0[i], s1[i], (unsigned long long)s2[i], (unsigned long long)o[i], (unsigned long long)m); }
    }
    printf("qsad_pk_u16_u8 vs wrap model: %d mismatches (acc<60000), %d mismatches (any acc)\n", bad, badhi);
    printf("mqsad sample: s0=%016llx s1=%08x -> %u %u %u %u\n", (unsigned long long)s0[1], s1[1], mo[4], mo[5], mo[6], mo[7]);
    uint32_t *out; hipMalloc(&out, 4);
    int blocks = 256 * 8, iters = 2048;
    hipEvent_t s, e; hipEventCreate(&s); hipEventCreate(&e);
    for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(s);
        hipLaunchKernelGGL(rate<0>, dim3(blocks), dim3(256), 0, 0, 1u, out, iters);
        hipEventRecord(e); hipEventSynchronize(e);
        float ms; hipEventElapsedTime(&ms, s, e);
        double ops = (double)blocks * 256 * iters * 16 * 8;
        if (rep == 2) printf("v_qsad_pk_u16_u8 %.1f T lane-ops/s = %.1f T absdiff/s (%.3f ms)\n", ops / (ms * 1e-3) / 1e12, 16 * ops / (ms * 1e-3) / 1e12, ms);
    }
    return 0;
}
