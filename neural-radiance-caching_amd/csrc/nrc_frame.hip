// nrc_frame.hip — the per-frame kernels around the network (include/nrc/frame.h).
//
// All four are HBM/latency-bound integer-and-copy work on a few MB: one thread per pixel,
// tile or output dword, coalesced where the layout allows, no LDS, no MFMA. Float arithmetic is written with
// explicit fmaf where the reference's nvcc --use_fast_math build contracts `a += b * c`
// (CMakeLists.txt:256-257), so results are bit-identical to the oracle (oracle/nrc_frame_oracle.c).
#include <hip/hip_runtime.h>

#include "nrc_internal.h"

namespace nrc_amd {

namespace {

struct F3 {
    float x, y, z;
};
struct TrainRecord {  // neural_radiance_caching.h:57-75
    int prop_to;
    F3 lt;
    int pixel, tile, len;
};
struct EndVertex {  // neural_radiance_caching.h:78-94
    int start;
    float mask;
    int pixel, tile;
};
static_assert(sizeof(TrainRecord) == 28 && sizeof(EndVertex) == 16, "reference record sizes");

// accumulate_render_radiance (nrc_helpers.cu:77-129), one pixel per lane; MODE is the RenderMode.
// w = 1/(iterationIndex+1) comes from the host (correctly rounded).
template <int MODE>
__global__ __launch_bounds__(256) void accumulate_kernel(const F3* __restrict__ rad, const F3* __restrict__ thr,
                                                         float4* __restrict__ rgba, uint32_t n, float w) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    float4 o;
    if constexpr (MODE == 0) {  // Full: dst += (T * L) * w
        const F3 L = rad[i], T = thr[i];
        o = rgba[i];
        o.x = __builtin_fmaf(T.x * L.x, w, o.x);
        o.y = __builtin_fmaf(T.y * L.y, w, o.y);
        o.z = __builtin_fmaf(T.z * L.z, w, o.z);
    } else if constexpr (MODE == 2) {  // CacheOnly
        const F3 L = rad[i], T = thr[i];
        o.x = L.x * T.x;
        o.y = L.y * T.y;
        o.z = L.z * T.z;
    } else if constexpr (MODE == 4) {  // DebugCacheNoThroughputModulation / copy_radiance_to_output_buffer
        const F3 L = rad[i];
        o.x = L.x;
        o.y = L.y;
        o.z = L.z;
    } else {  // 5: DebugThroughputOnly
        const F3 T = thr[i];
        o.x = T.x;
        o.y = T.y;
        o.z = T.z;
    }
    o.w = 1.0f;
    rgba[i] = o;
}

// propagate_train_radiance (nrc_helpers.cu:131-224), one tile per lane walking its own record chain.
// Chains are disjoint (one train path per tile), so the read-modify-write of targets needs no atomics.
// Every lane exits: an index outside [0, nrec) ends the chain, and a chain is cut after nrec steps.
__global__ __launch_bounds__(256) void propagate_kernel(const EndVertex* __restrict__ ends,
                                                        const F3* __restrict__ end_rad, uint32_t tiles,
                                                        const TrainRecord* __restrict__ rec, F3* targets,
                                                        uint32_t nrec) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= tiles) return;
    const EndVertex ev = ends[t];
    const F3 er = end_rad[t];
    F3 last = {er.x * ev.mask, er.y * ev.mask, er.z * ev.mask};  // :154
    int i = ev.start;
    for (uint32_t steps = 0; i >= 0 && (uint32_t)i < nrec && steps < nrec; ++steps) {
        const int next = rec[i].prop_to;
        const F3 lt = rec[i].lt;
        F3 v = targets[i];
        v.x = __builtin_fmaf(lt.x, last.x, v.x);  // :199 radianceTo += localThroughput * lastRadiance
        v.y = __builtin_fmaf(lt.y, last.y, v.y);
        v.z = __builtin_fmaf(lt.z, last.z, v.z);
        targets[i] = v;  // :205
        last = v;        // :213
        i = next;        // :214
    }
}

// ---- shuffle permutation: keyed 4-round Feistel network on [0, 2^(2h)) with cycle walking into [0, n).
// Spec in DESIGN.md §9 (restated independently in oracle/nrc_frame_oracle.c).
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

struct FeistelKey {
    uint32_t k[4];
    uint32_t h, n;
};

__device__ __forceinline__ uint32_t feistel_perm(uint32_t d, const FeistelKey& fk) {
    const uint32_t mask = (1u << fk.h) - 1u;
    uint32_t x = d;
    do {
        uint32_t L = x >> fk.h, R = x & mask;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t nl = R;
            R = L ^ (mix32(R ^ fk.k[r]) & mask);
            L = nl;
        }
        x = (L << fk.h) | R;
    } while (x >= fk.n);  // terminates: the walk stays on d's cycle, which contains d < n
    return x;
}

__global__ __launch_bounds__(256) void permutation_kernel(FeistelKey fk, int* __restrict__ perm) {
    const uint32_t d = blockIdx.x * 256u + threadIdx.x;
    if (d >= fk.n) return;
    perm[d] = (int)feistel_perm(d, fk);
}

// permute_train_data (nrc_helpers.cu:226-249) as a dword copy: threads [0, 15 n) write the query array,
// threads [15 n, 18 n) the target array, so every wave's stores are contiguous; each lane re-derives its
// record's source index (a few dozen integer ops, cheaper than a second pass through HBM).
__global__ __launch_bounds__(256) void permute_kernel(const uint32_t* __restrict__ qs, const uint32_t* __restrict__ ts,
                                                      const int* __restrict__ perm, FeistelKey fk, uint32_t nrec,
                                                      uint32_t* __restrict__ qd, uint32_t* __restrict__ td) {
    const uint32_t g = blockIdx.x * 256u + threadIdx.x;
    const uint32_t nq = fk.n * 15u;
    if (g >= nq + fk.n * 3u) return;
    const bool is_q = g < nq;
    const uint32_t gg = is_q ? g : g - nq;
    const uint32_t d = is_q ? gg / 15u : gg / 3u;  // constant divisors: mul-hi, no integer division
    const uint32_t k = gg - d * (is_q ? 15u : 3u);
    const uint32_t p = perm ? (uint32_t)perm[d] : feistel_perm(d, fk);
    const uint32_t s = p % nrec;  // :245 (a negative caller entry reads as unsigned: never out of bounds)
    if (is_q)
        qd[gg] = qs[(size_t)s * 15u + k];
    else
        td[gg] = ts[(size_t)s * 3u + k];
}

FeistelKey make_key(uint64_t seed, uint32_t frame, uint32_t n) {
    auto mix = [](uint32_t x) {
        x ^= x >> 16;
        x *= 0x7feb352du;
        x ^= x >> 15;
        x *= 0x846ca68bu;
        x ^= x >> 16;
        return x;
    };
    FeistelKey fk{};
    for (uint32_t r = 0; r < 4; ++r)
        fk.k[r] = mix((uint32_t)seed ^ mix((uint32_t)(seed >> 32) ^ mix(frame + 0x9e3779b9u * (r + 1))));
    uint32_t b = 2;
    while (b < 32 && (1ull << b) < (uint64_t)n) ++b;
    if (b & 1) ++b;
    fk.h = b / 2;
    fk.n = n;
    return fk;
}

inline dim3 grid_for(uint64_t threads) { return dim3((unsigned)((threads + 255) / 256)); }

}  // namespace

hipError_t launch_accumulate(const float* rad, const float* thr, float* rgba, uint32_t n, int mode, float w,
                             hipStream_t s) {
    if (n == 0) return hipSuccess;
    const F3* r = reinterpret_cast<const F3*>(rad);
    const F3* t = reinterpret_cast<const F3*>(thr);
    float4* o = reinterpret_cast<float4*>(rgba);
    switch (mode) {
    case 0: hipLaunchKernelGGL(accumulate_kernel<0>, grid_for(n), dim3(256), 0, s, r, t, o, n, w); break;
    case 2: hipLaunchKernelGGL(accumulate_kernel<2>, grid_for(n), dim3(256), 0, s, r, t, o, n, w); break;
    case 4: hipLaunchKernelGGL(accumulate_kernel<4>, grid_for(n), dim3(256), 0, s, r, t, o, n, w); break;
    case 5: hipLaunchKernelGGL(accumulate_kernel<5>, grid_for(n), dim3(256), 0, s, r, t, o, n, w); break;
    default: return hipSuccess;  // NoCache / CacheFirstVertex: nothing to accumulate (nrc_helpers.cu:104-107)
    }
    return hipGetLastError();
}

hipError_t launch_propagate(const void* ends, const float* end_rad, uint32_t tiles, const void* records,
                            float* targets, uint32_t nrec, hipStream_t s) {
    if (tiles == 0 || nrec == 0) return hipSuccess;
    hipLaunchKernelGGL(propagate_kernel, grid_for(tiles), dim3(256), 0, s, reinterpret_cast<const EndVertex*>(ends),
                       reinterpret_cast<const F3*>(end_rad), tiles, reinterpret_cast<const TrainRecord*>(records),
                       reinterpret_cast<F3*>(targets), nrec);
    return hipGetLastError();
}

hipError_t launch_permutation(uint64_t seed, uint32_t frame, int* perm, uint32_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(permutation_kernel, grid_for(n), dim3(256), 0, s, make_key(seed, frame, n), perm);
    return hipGetLastError();
}

hipError_t launch_permute(const float* qs, const float* ts, const int* perm, uint64_t seed, uint32_t frame,
                          uint32_t nrec, float* qd, float* td, uint32_t n_out, hipStream_t s) {
    if (n_out == 0 || nrec == 0) return hipSuccess;
    hipLaunchKernelGGL(permute_kernel, grid_for((uint64_t)n_out * 18u), dim3(256), 0, s,
                       reinterpret_cast<const uint32_t*>(qs), reinterpret_cast<const uint32_t*>(ts), perm,
                       make_key(seed, frame, n_out), nrec, reinterpret_cast<uint32_t*>(qd),
                       reinterpret_cast<uint32_t*>(td));
    return hipGetLastError();
}

}  // namespace nrc_amd
