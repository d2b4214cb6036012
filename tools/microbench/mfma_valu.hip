// Microbenchmark: how much independent VALU work hides between v_mfma_f32_32x32x16_f16 issues on
// gfx950, at 1/2/4 waves per SIMD. Random (non-zero) f16 operands (DVFS depends on data).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

template <int NV, int CHAINS>
__global__ __launch_bounds__(256) void k(const h8* __restrict__ in, float* out, int iters) {
    h8 a = in[threadIdx.x], b = in[threadIdx.x + 256];
    f16v acc[CHAINS];
    for (int c = 0; c < CHAINS; ++c) acc[c] = f16v{};
    float v[8];
    for (int j = 0; j < 8; ++j) v[j] = (float)(threadIdx.x + j);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[c], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < NV; ++j) v[j & 7] = __builtin_fmaf(v[j & 7], 1.0001f, 0.5f);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if (NV) __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
        }
    }
    float s = 0.f;
    for (int c = 0; c < CHAINS; ++c) s += acc[c][0];
    for (int j = 0; j < 8; ++j) s += v[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int NV, int CHAINS>
float run(const h8* in, float* out, int blocks, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((k<NV, CHAINS>), dim3(blocks), dim3(256), 0, 0, in, out, iters);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k<NV, CHAINS>), dim3(blocks), dim3(256), 0, 0, in, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    std::vector<_Float16> h(512 * 8);
    unsigned s = 1;
    for (auto& x : h) { s = s * 1664525u + 1013904223u; x = (_Float16)(((s >> 9) & 0xffff) / 65536.0f - 0.5f); }
    h8* in;
    float* out;
    hipMalloc(&in, h.size() * 2);
    hipMalloc(&out, 4 * 256 * cus * 8);
    hipMemcpy(in, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    const int iters = 2000;
    printf("{\"cus\": %d, \"rows\": [\n", cus);
    bool first = true;
    for (int wps : {1, 2, 4}) {
        const int blocks = cus * wps;  // 256-thread blocks: one wave per SIMD per block
#define RUN(NV)                                                                                        \
    {                                                                                                  \
        float ms = run<NV, 4>(in, out, blocks, iters);                                                 \
        double mfma_per_simd = (double)iters * 4 * wps;                                                \
        printf("%s{\"waves_per_simd\": %d, \"valu_per_mfma\": %d, \"us\": %.2f, \"ns_per_mfma_per_simd\": %.4f}\n", \
               first ? "" : ",", wps, NV, ms * 1e3, ms * 1e6 / mfma_per_simd);                          \
        first = false;                                                                                 \
    }
        RUN(0) RUN(2) RUN(4) RUN(6) RUN(8) RUN(12) RUN(16) RUN(24)
    }
    printf("]}\n");
    return 0;
}
