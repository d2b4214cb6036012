// nrc_hash.h — HashGrid lookup shared by the inference kernels (nrc_kernels.hip) and the t16 training kernel
// (nrc_train16.hip): tcnn GridEncoding's corner addressing and interpolation of one level (NRCNetworkConfigs.h:84-103,
// SURVEY.md Appendix A; restated in oracle/nrc_hash_oracle.c).
#pragma once

#include "nrc_device.h"

namespace nrc_amd {

// element i (0..3) of a 16-byte load, by named components (see the bit_cast note in infer_v2_body)
__device__ __forceinline__ uint32_t pick4(const u4& q, uint32_t i) {
    const uint32_t lo = (i & 1u) ? q.y : q.x, hi = (i & 1u) ? q.w : q.z;
    return (i & 2u) ? hi : lo;
}

struct HashCorners {
    uint32_t entry[8];  // global table entries
    float w[8];         // trilinear weights, tcnn order ((1 * wx) * wy) * wz
};

// tcnn pos_fract + grid_index for level l. DENSE_OK: the level may be dense (l <= 1 possible); dense = l <= 1.
template <bool DENSE_OK>
__device__ __forceinline__ void hash_corners(float px, float py, float pz, int l, HashCorners& C) {
    const float scale = (float)(16 << l) - 1.0f;  // exact: 16 * 2^l - 1 < 2^24
    const uint32_t res = 16u << l;
    const float xs[3] = {px, py, pz};
    float fr[3];
    uint32_t cell[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const float pos = __builtin_fmaf(scale, xs[d], 0.5f);
        const float fl = floorf(pos);
        cell[d] = (uint32_t)(int)fl;
        fr[d] = pos - fl;
    }
    const bool dense = DENSE_OK && l <= 1;
    const uint32_t mask = l == 0 ? 4095u : 32767u;
    const uint32_t off = l == 0 ? 0u : 4096u + (uint32_t)(l - 1) * 32768u;
    // per-dimension corner terms: dense x + y*res + z*res^2, hashed x ^ y*P1 ^ z*P2 (uint32 wrap-around)
    const uint32_t ym = dense ? res : NRC_HASH_PRIME1, zm = dense ? res * res : NRC_HASH_PRIME2;
    const uint32_t X[2] = {cell[0], cell[0] + 1u};
    const uint32_t Y[2] = {cell[1] * ym, cell[1] * ym + ym};
    const uint32_t Z[2] = {cell[2] * zm, cell[2] * zm + zm};
    const float wx[2] = {1.0f - fr[0], fr[0]}, wy[2] = {1.0f - fr[1], fr[1]}, wz[2] = {1.0f - fr[2], fr[2]};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const int bx = c & 1, by = (c >> 1) & 1, bz = c >> 2;
        uint32_t i;
        if (DENSE_OK)
            i = dense ? X[bx] + Y[by] + Z[bz] : X[bx] ^ Y[by] ^ Z[bz];
        else
            i = X[bx] ^ Y[by] ^ Z[bz];
        C.entry[c] = (i & mask) + off;
        C.w[c] = (wx[bx] * wy[by]) * wz[bz];
    }
}

// tcnn kernel_grid's interpolation of one level: result = fma((half)w, value, result) over corners 0..7, packed half2
__device__ __forceinline__ uint32_t hash_interp(const HashCorners& C, const uint32_t (&v)[8]) {
    h2v acc = {(_Float16)0.0f, (_Float16)0.0f};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        // (half)weight must be rounded before the FMA: the launder stops the compiler from folding the f32->f16
        // conversion into a mixed-precision v_fma_mix (which would skip that rounding)
        uint32_t w2 = pk2(C.w[c], C.w[c]);
        asm volatile("" : "+v"(w2));
        acc = __builtin_elementwise_fma(__builtin_bit_cast(h2v, w2), __builtin_bit_cast(h2v, v[c]), acc);
    }
    return __builtin_bit_cast(uint32_t, acc);
}

// One level's two features as a packed half2: tcnn kernel_grid result = fma((half)w, value, result), corners 0..7.
template <bool DENSE_OK>
__device__ __forceinline__ uint32_t hash_level_feature(float px, float py, float pz, int l,
                                                        const uint32_t* __restrict__ table) {
    HashCorners C;
    hash_corners<DENSE_OK>(px, py, pz, l, C);
    // Corners 2p and 2p+1 differ only in x: their entries share an aligned group of 4 unless the x carry leaves
    // it (hashed: cell x = 3 mod 4; dense: entry = 3 mod 4), i.e. for 1 lane in 4. One 16-byte load of the
    // group serves both; the partner gets its own 4-byte load only when it lies outside (the buffer load of the
    // other lanes is dropped by the descriptor bound and touches no cache line): 1.25 cache-line accesses per
    // corner pair instead of 2 — the random gathers run at the L1 line rate.
    const __amdgpu_buffer_rsrc_t rs = buffer_rsrc(table, NRC_HASH_ENTRIES * 4);
    uint32_t v[8];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const uint32_t e0 = C.entry[2 * p], e1 = C.entry[2 * p + 1];
        const u4 quad = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((e0 & ~3u) * 4u), 0, 0);
        const bool same = (e1 >> 2) == (e0 >> 2);
        const uint32_t far = __builtin_amdgcn_raw_buffer_load_b32(rs, same ? kBufferOff : (int)(e1 * 4u), 0, 0);
        v[2 * p] = pick4(quad, e0 & 3u);
        v[2 * p + 1] = same ? pick4(quad, e1 & 3u) : far;
    }
    return hash_interp(C, v);
}


}  // namespace nrc_amd
