// Issue cost of v_mfma_f32_4x4x4_16b_f16 (16 independent 4x4x4 blocks) against v_mfma_f32_32x32x16_f16 on gfx950:
// back-to-back independent MFMAs of one wave per SIMD, s_memtime cycles per MFMA (median over waves). Decides
// whether an accumulator re-entry by four 4x4x4 identity MFMAs (the tcnn-numerics kernel) is cheaper than two 32x32x16.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/mfma_4x4.hip -o tools/microbench/mfma_4x4 && ./tools/microbench/mfma_4x4
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

template <int SHAPE>
__global__ __launch_bounds__(256) void k(const h8* __restrict__ in, float* out, unsigned long long* cyc, int iters) {
    const h8 a8 = in[threadIdx.x], b8 = in[threadIdx.x + 256];
    const h4 a4 = {a8[0], a8[1], a8[2], a8[3]}, b4 = {b8[0], b8[1], b8[2], b8[3]};
    f4 acc4[8];
    f16v acc32[4];
    for (int c = 0; c < 8; ++c) acc4[c] = f4{};
    for (int c = 0; c < 4; ++c) acc32[c] = f16v{};
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if constexpr (SHAPE == 4) {
#pragma unroll
            for (int c = 0; c < 8; ++c) acc4[c] = __builtin_amdgcn_mfma_f32_4x4x4f16(a4, b4, acc4[c], 0, 0, 0);
        } else {
#pragma unroll
            for (int c = 0; c < 4; ++c) acc32[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, b8, acc32[c], 0, 0, 0);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.0f;
    for (int c = 0; c < 8; ++c) s += acc4[c][0];
    for (int c = 0; c < 4; ++c) s += acc32[c][0];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <int SHAPE>
double run(const h8* in, float* out, unsigned long long* cyc, int blocks, int iters) {
    k<SHAPE><<<blocks, 256>>>(in, out, cyc, iters);
    if (hipDeviceSynchronize() != hipSuccess) return -1.0;
    std::vector<unsigned long long> h(blocks * 4);
    if (hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1.0;
    std::sort(h.begin(), h.end());
    const double per = SHAPE == 4 ? 8.0 * iters : 4.0 * iters;
    return (double)h[h.size() / 2] / per;
}

int main() {
    const int blocks = 256, iters = 4096;
    h8* in;
    float* out;
    unsigned long long* cyc;
    std::vector<_Float16> hin(512 * 8);
    for (size_t i = 0; i < hin.size(); ++i) hin[i] = (_Float16)((float)((i * 37) % 101) / 101.0f - 0.5f);
    if (hipMalloc(&in, hin.size() * 2) != hipSuccess || hipMalloc(&out, blocks * 256 * 4) != hipSuccess ||
        hipMalloc(&cyc, blocks * 4 * 8) != hipSuccess)
        return 1;
    if (hipMemcpy(in, hin.data(), hin.size() * 2, hipMemcpyHostToDevice) != hipSuccess) return 1;
    for (int rep = 0; rep < 3; ++rep) {
        const double c4 = run<4>(in, out, cyc, blocks, iters);
        const double c32 = run<32>(in, out, cyc, blocks, iters);
        printf("s_memtime cycles per MFMA (one wave per SIMD, independent accumulators): 4x4x4_16b_f16 %.2f, "
               "32x32x16_f16 %.2f\n", c4, c32);
    }
    return hipFree(in) != hipSuccess || hipFree(out) != hipSuccess || hipFree(cyc) != hipSuccess;
}
