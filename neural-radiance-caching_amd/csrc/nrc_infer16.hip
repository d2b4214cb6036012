// nrc_infer16.hip — Frequency inference on v_mfma_f32_16x16x32_f16 (the "t16" layout of the training kernel,
// nrc_internal.h), A/B candidate against the 32x32x16 kernel (infer_kernel_v2, variant 39). Reference:
// Network::infer -> network->inference (nrc/src/NRCNetwork.cu:64-77), tcnn FullyFusedMLP forward.
//
// Why: at equal MFMA work the 16x16x32 shape runs at a higher clock under the power limit (MI355X_MICROARCH.md DVFS
// item 7; profiles/r02_microbench/mfma_shape2.json), and the output layer computes 16 rows instead of 32. Cost: every
// MFMA holds vector issue for the same 8 cycles for half the FLOPs, and the 96-slot encoder evaluates 4 OneBlob dims
// per lane per 32 queries instead of 3.
//
// Block = 1024 threads (16 waves, 4 per SIMD) per CU with the 46-KiB forward image in LDS; the block owns a contiguous
// range of 32-query tiles that its waves draw from an LDS counter (as variant 39). A wave's tile is two 16-query
// groups u; lane l = (g = l >> 4, c = l & 15) encodes the 24 K slots of group g for query 16 u + c, and every weight
// fragment read from LDS feeds both groups' MFMAs. Per tile: 24 + 4 x 16 + 4 = 92 MFMAs (= 46 of 32x32x16).
#include "nrc_t16.h"

namespace nrc_amd {
namespace {

using t16::f4;
using t16::mfma16;
using t16::relu_b;
using t16::encode16;

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f3v __attribute__((ext_vector_type(3)));

constexpr int kThreads = 1024, kWaves = kThreads / 64;

typedef __attribute__((address_space(3))) const h8 lds_h8;
// hide the LDS image base from loop-invariant code motion: fragments are re-read per layer, not hoisted into VGPRs
__device__ __forceinline__ lds_h8* launder16(lds_h8* p) {
    asm volatile("" : "+v"(p));
    return p;
}

struct Q16 {
    f3v p[2];
    f2v b[2], i[2];
};

// the tile's queries for this lane: rows 16 u + c, position + OneBlob dims 3 + 2gg, 4 + 2gg + Identity 9 + 2gg,
// 10 + 2gg; raw buffer loads whose descriptor covers the tile's valid rows (past n they return 0)
__device__ __forceinline__ Q16 load_q16(const float* __restrict__ q, int64_t n, int64_t tile, int c, int gg) {
    const int64_t s0 = tile * 32;
    const __amdgpu_buffer_rsrc_t rs = buffer_rsrc(q + s0 * NRC_INPUT_DIMS, tile_rows(n, s0) * (NRC_INPUT_DIMS * 4));
    Q16 Q;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int o = (16 * u + c) * (NRC_INPUT_DIMS * 4);
        // whole-vector bit_casts (clang 22 element bit_cast bug)
        Q.p[u] = __builtin_bit_cast(f3v, __builtin_amdgcn_raw_buffer_load_b96(rs, o, 0, 0));
        Q.b[u] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs, o + 12 + 8 * gg, 0, 0));
        Q.i[u] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rs, o + 36 + 8 * gg, 0, 0));
    }
    return Q;
}

// one hidden layer (L = 1..4) for both groups: 8 fragments x 2 groups
__device__ __forceinline__ void hidden16(lds_h8* wl, int L, const h8 (&in)[2][2], h8 (&y)[2][2]) {
    h8 w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = wl[t16_fwd_frag(L, i >> 1, i & 1) * 64];
    f4 cc[2][4];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int u = 0; u < 2; ++u) cc[u][mb] = mfma16(w[2 * mb], in[u][0], f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int u = 0; u < 2; ++u) cc[u][mb] = mfma16(w[2 * mb + 1], in[u][1], cc[u][mb]);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        y[u][0] = relu_b(cc[u][0], cc[u][1]);
        y[u][1] = relu_b(cc[u][2], cc[u][3]);
    }
}

__global__ __launch_bounds__(kThreads, 1) void infer16_kernel(const float* __restrict__ q, float* __restrict__ out,
                                                               int64_t n, const h8* __restrict__ wf) {
    __shared__ __attribute__((aligned(16))) h8 lw[kT16FwdFrags * 64];
    __shared__ uint32_t wq_next;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // forward image -> LDS by LDS-DMA: fragment f from wave f % 16
#pragma unroll
    for (int k = 0; k < (kT16FwdFrags + kWaves - 1) / kWaves; ++k) {
        const int f = wave + kWaves * k;
        if (f < kT16FwdFrags)
            __builtin_amdgcn_global_load_lds((const void*)(wf + f * 64 + lane),
                                             (__attribute__((address_space(3))) void*)(lw + f * 64), 16, 0, 0);
    }
    if (threadIdx.x == 0) wq_next = 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    const int g = lane >> 4, c = lane & 15, gg = g < 3 ? g : 0;
    const int64_t ntiles = (n + 31) >> 5;
    const int64_t gbase = (int64_t)blockIdx.x * ntiles / gridDim.x;
    const int64_t gend = (int64_t)(blockIdx.x + 1) * ntiles / gridDim.x;
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(&wq_next, 1u);
    int64_t tile = gbase + (int64_t)__builtin_amdgcn_readfirstlane(t);
    if (tile >= gend) return;
    // the draw for the next tile is issued one iteration ahead, so its latency hides under a whole tile
    uint32_t nn_raw = 0;
    if (lane == 0) nn_raw = atomicAdd(&wq_next, 1u);
    Q16 Q = load_q16(q, n, tile, c, gg);
    lds_h8* const lwl = (lds_h8*)(lw + lane);
    while (tile < gend) {
        uint32_t tn;
        asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(tn) : "v"(nn_raw));
        const int64_t next = gbase + (int64_t)tn;
        if (lane == 0) nn_raw = atomicAdd(&wq_next, 1u);
        h8 x[2][3];
#pragma unroll
        for (int u = 0; u < 2; ++u) encode16(Q.p[u].x, Q.p[u].y, Q.p[u].z, Q.b[u].x, Q.b[u].y, Q.i[u].x, Q.i[u].y, g, x[u]);
        Q = load_q16(q, n, next, c, gg);  // prefetch (a tile past gend is a harmless read, or returns 0 past n)

        lds_h8* wl = launder16(lwl);
        h8 a[2][2], b[2][2];
        {
            f4 cc[2][4];
#pragma unroll
            for (int ks = 0; ks < 3; ++ks) {
                h8 w[4];
#pragma unroll
                for (int mb = 0; mb < 4; ++mb) w[mb] = wl[t16_fwd_frag(0, mb, ks) * 64];
#pragma unroll
                for (int mb = 0; mb < 4; ++mb)
#pragma unroll
                    for (int u = 0; u < 2; ++u)
                        cc[u][mb] = mfma16(w[mb], x[u][ks], ks ? cc[u][mb] : f4{0.f, 0.f, 0.f, 0.f});
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                a[u][0] = relu_b(cc[u][0], cc[u][1]);
                a[u][1] = relu_b(cc[u][2], cc[u][3]);
            }
        }
        hidden16(launder16(lwl), 1, a, b);
        hidden16(launder16(lwl), 2, b, a);
        hidden16(launder16(lwl), 3, a, b);
        hidden16(launder16(lwl), 4, b, a);
        f4 o[2];
        {
            lds_h8* w5 = launder16(lwl);
            const h8 w0 = w5[t16_fwd_frag(5, 0, 0) * 64], w1 = w5[t16_fwd_frag(5, 0, 1) * 64];
#pragma unroll
            for (int u = 0; u < 2; ++u) o[u] = mfma16(w1, a[u][1], mfma16(w0, a[u][0], f4{0.f, 0.f, 0.f, 0.f}));
        }
        // rows 0..2 of column c are registers 0..2 of lane group 0; the other groups' stores are dropped
        const int64_t s0 = tile * 32;
        const __amdgpu_buffer_rsrc_t rs = buffer_rsrc(out + s0 * NRC_OUTPUT_DIMS, tile_rows(n, s0) * 12);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const h2 z = {};
            const h2 lo = __builtin_elementwise_max(__builtin_bit_cast(h2, pk2(o[u][0], o[u][1])), z);
            const h2 hi = __builtin_elementwise_max(__builtin_bit_cast(h2, pk2(o[u][2], 0.0f)), z);
            const u3 ov = {__builtin_bit_cast(uint32_t, (float)lo[0]), __builtin_bit_cast(uint32_t, (float)lo[1]),
                           __builtin_bit_cast(uint32_t, (float)hi[0])};
            __builtin_amdgcn_raw_buffer_store_b96(ov, rs, g == 0 ? (16 * u + c) * 12 : kBufferOff, 0, 0);
        }
        tile = next;
    }
}

}  // namespace

hipError_t launch_infer16(const float* queries, float* out, int64_t n, const _Float16* wf16, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    static int cus = 0;
    if (!cus) {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
            v = 256;
        cus = v;
    }
    const int64_t ntiles = (n + 31) / 32;
    const int64_t want = (ntiles + kWaves - 1) / kWaves;
    const int grid = (int)(want < cus ? want : cus);
    hipLaunchKernelGGL(infer16_kernel, dim3(grid), dim3(kThreads), 0, s, queries, out, n, (const h8*)wf16);
    return hipGetLastError();
}

}  // namespace nrc_amd
