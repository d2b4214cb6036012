// MFMA shape microbenchmark, round 2: v_mfma_f32_32x32x16_f16 vs v_mfma_f32_16x16x32_f16 at equal FLOP per
// iteration, random vs zero operands, with NV independent VALU per 32 cycles of MFMA pipe (per 32x32x16, or per
// two 16x16x32), 4 waves per SIMD, and an in-kernel clock (s_memtime / s_memrealtime).
//
// Why a second version: tools/microbench/mfma_shape.hip kept eight f4v accumulators in C++ and the compiler
// shuffled them through v_accvgpr_read/write/mov every iteration (≈40 extra VALU per 8 MFMAs, see the ISA of
// k<16, *>), so its 16x16x32 rows measured the shuffles, not the MFMA. Here every MFMA and every filler is
// inline asm on VGPR accumulators ("+v"), so the loop body is exactly the instructions listed.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

template <int NV>
__device__ __forceinline__ void filler(float (&v)[8]) {
#pragma unroll
    for (int j = 0; j < NV; ++j) asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(v[j & 7]) : "v"(v[(j + 3) & 7]));
}

// SHAPE 32: 4 accumulators x 32x32x16 per iteration; SHAPE 16: 8 accumulators x 16x16x32 (same FLOP).
template <int SHAPE, int NV>
__global__ __launch_bounds__(256) void k(const h8* __restrict__ in, float* out, unsigned long long* clk, int iters) {
    h8 a = in[threadIdx.x], b = in[threadIdx.x + 256];
    f16v acc[4] = {};
    f4v acc2[8] = {};
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)(threadIdx.x + j) * 1e-3f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        if constexpr (SHAPE == 32) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b));
                filler<NV>(v);
            }
        } else {
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc2[c]) : "v"(a), "v"(b));
                filler<NV / 2>(v);
                if ((NV & 1) && (c & 1)) filler<1>(v);
            }
        }
    }
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    for (int c = 0; c < 4; ++c) s += acc[c][0] + acc[c][15];
    for (int c = 0; c < 8; ++c) s += acc2[c][0] + acc2[c][3];
    for (int j = 0; j < 8; ++j) s += v[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

struct Res {
    float ms;
    double ghz;
};

template <int SHAPE, int NV>
Res run(const h8* in, float* out, unsigned long long* clk, int blocks, int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int r = 0; r < 20; ++r)  // >= 2 s-equivalent warm-up is not needed for a ranking, but settle the clock
        hipLaunchKernelGGL((k<SHAPE, NV>), dim3(blocks), dim3(256), 0, 0, in, out, clk, iters);
    (void)hipEventRecord(e0);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k<SHAPE, NV>), dim3(blocks), dim3(256), 0, 0, in, out, clk, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> c(2 * blocks);
    (void)hipMemcpy(c.data(), clk, 16 * blocks, hipMemcpyDeviceToHost);
    std::vector<double> g;
    for (int i = 0; i < blocks; ++i) g.push_back((double)c[2 * i] / (double)c[2 * i + 1] * 0.1);  // realtime 100 MHz
    std::sort(g.begin(), g.end());
    return {ms / reps, g[g.size() / 2]};
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    std::vector<_Float16> h(512 * 8), z(512 * 8, (_Float16)0.0f);
    unsigned s = 1;
    for (auto& x : h) {
        s = s * 1664525u + 1013904223u;
        x = (_Float16)(((s >> 9) & 0xffff) / 65536.0f - 0.5f);
    }
    h8 *in, *inz;
    float* out;
    unsigned long long* clk;
    (void)hipMalloc(&in, h.size() * 2);
    (void)hipMalloc(&inz, h.size() * 2);
    (void)hipMalloc(&out, 4 * 256 * cus * 8);
    (void)hipMalloc(&clk, 16 * cus * 8);
    (void)hipMemcpy(in, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(inz, z.data(), z.size() * 2, hipMemcpyHostToDevice);
    const int iters = 4000;
    printf("{\"rows\": [\n");
    bool first = true;
    for (int data = 0; data < 2; ++data) {
        const int wps = 4;
        const int blocks = cus * wps;
        const h8* src = data ? inz : in;
#define RUN(SH, NV)                                                                                         \
    {                                                                                                       \
        Res r = run<SH, NV>(src, out, clk, blocks, iters);                                                  \
        double flop = 2.0 * 32 * 32 * 16 * 4 * (double)iters * blocks * 256 / 64;                           \
        double cyc_per_32 = r.ms * 1e-3 * r.ghz * 1e9 / ((double)iters * 4 * wps);                          \
        printf("%s{\"shape\": %d, \"data\": \"%s\", \"waves_per_simd\": %d, \"valu_per_32cyc\": %d, "          \
               "\"tflops\": %.1f, \"clock_ghz\": %.3f, \"simd_cycles_per_32x32_equiv\": %.2f}\n",                \
               first ? "" : ",", SH, data ? "zero" : "random", wps, NV, flop / (r.ms * 1e-3) / 1e12, r.ghz,  \
               cyc_per_32);                                                                                 \
        fflush(stdout);                                                                                     \
        first = false;                                                                                      \
    }
        RUN(32, 0) RUN(16, 0) RUN(32, 2) RUN(16, 2) RUN(32, 4) RUN(16, 4) RUN(32, 6) RUN(16, 6) RUN(32, 8)
        RUN(16, 8)
    }
    printf("]}\n");
    return 0;
}
