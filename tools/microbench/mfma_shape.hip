// MFMA shape/data microbenchmark on gfx950: FLOP rate of 32x32x16 vs 16x16x32 f16 MFMA chains with
// NV independent VALU per MFMA, random vs zero operands, 2 and 4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

template <int SHAPE, int NV>
__global__ __launch_bounds__(256) void k(const h8* __restrict__ in, float* out, int iters) {
    h8 a = in[threadIdx.x], b = in[threadIdx.x + 256];
    constexpr int CH = SHAPE == 32 ? 4 : 8;  // equal FLOP per iteration
    f16v acc[4];
    f4v acc2[8];
    for (int c = 0; c < 4; ++c) acc[c] = f16v{};
    for (int c = 0; c < 8; ++c) acc2[c] = f4v{};
    float v[8];
    for (int j = 0; j < 8; ++j) v[j] = (float)(threadIdx.x + j);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            if (SHAPE == 32) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[c], 0, 0, 0);
            else acc2[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc2[c], 0, 0, 0);
            constexpr int nv = SHAPE == 32 ? NV : NV / 2;
#pragma unroll
            for (int j = 0; j < nv; ++j) v[j & 7] = __builtin_fmaf(v[j & 7], 1.0001f, 0.5f);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if (nv) __builtin_amdgcn_sched_group_barrier(0x002, nv, 0);
        }
    }
    float s = 0.f;
    for (int c = 0; c < 4; ++c) s += acc[c][0];
    for (int c = 0; c < 8; ++c) s += acc2[c][0];
    for (int j = 0; j < 8; ++j) s += v[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int SHAPE, int NV>
float run(const h8* in, float* out, int blocks, int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k<SHAPE, NV>), dim3(blocks), dim3(256), 0, 0, in, out, iters);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k<SHAPE, NV>), dim3(blocks), dim3(256), 0, 0, in, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    std::vector<_Float16> h(512 * 8), z(512 * 8, (_Float16)0.0f);
    unsigned s = 1;
    for (auto& x : h) { s = s * 1664525u + 1013904223u; x = (_Float16)(((s >> 9) & 0xffff) / 65536.0f - 0.5f); }
    h8 *in, *inz;
    float* out;
    (void)hipMalloc(&in, h.size() * 2);
    (void)hipMalloc(&inz, h.size() * 2);
    (void)hipMalloc(&out, 4 * 256 * cus * 8);
    (void)hipMemcpy(in, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(inz, z.data(), z.size() * 2, hipMemcpyHostToDevice);
    const int iters = 2000;
    printf("{\"rows\": [\n");
    bool first = true;
    for (int data = 0; data < 2; ++data)
        for (int wps : {2, 4}) {
            const int blocks = cus * wps;
            const h8* src = data ? inz : in;
#define RUN(SH, NV)                                                                                   \
    {                                                                                                 \
        float ms = run<SH, NV>(src, out, blocks, iters);                                              \
        double flop = 2.0 * 32 * 32 * 16 * 4 * (double)iters * blocks * 256 / 64;                     \
        printf("%s{\"shape\": %d, \"data\": \"%s\", \"waves_per_simd\": %d, \"valu_per_32x32_equiv\": %d, " \
               "\"tflops\": %.1f}\n",                                                                 \
               first ? "" : ",", SH, data ? "zero" : "random", wps, NV, flop / (ms * 1e-3) / 1e12);    \
        first = false;                                                                                \
    }
            RUN(32, 0) RUN(16, 0) RUN(32, 4) RUN(16, 4) RUN(32, 8) RUN(16, 8) RUN(32, 16) RUN(16, 16)
        }
    printf("]}\n");
    return 0;
}
