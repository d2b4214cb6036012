// nrc_t16.h — device pieces of the "t16" layout (v_mfma_f32_16x16x32_f16, nrc_internal.h) shared by the training
// kernel (nrc_train16.hip) and the 16x16x32 inference kernel (nrc_infer16.hip): the MFMA wrapper, the packed ReLU,
// accumulator -> B-operand conversion and the 96-slot encoder (t16_slot_feature).
#pragma once

#include "nrc_device.h"
#include "nrc_hash.h"

namespace nrc_amd {
namespace t16 {

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mfma16(h8 a, h8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }

// Values that an MFMA reads are never produced by inline asm here: LLVM's hazard recognizer does not look inside
// inline asm, so an asm VALU def read by an MFMA within 2 wait states gets no s_nop and the MFMA reads the stale
// register (tools/asm_hazard_check.py; tests/test_asm_hazards.py checks every product kernel).
typedef short s2v __attribute__((ext_vector_type(2)));

// f16 ReLU of a packed pair as an integer max (v_pk_max_i16): negative halves (sign bit set, -0 included) become +0,
// so an activation is +0 or has positive bits, and RNE conversion commuting with ReLU makes this f16(max(x, 0)).
__device__ __forceinline__ uint32_t relu_pk(uint32_t x) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s2v, x), s2v{0, 0}));
}
// pk2(|a|, |b|) for an MFMA operand: RNE convert, then clear both sign bits (the compiler-visible form of
// pk2_abs)
__device__ __forceinline__ uint32_t pk2_abs_v(float a, float b) { return pk2(a, b) & 0x7FFF7FFFu; }

// accumulators of M-blocks 2s, 2s + 1 -> B operand of k-step s (rows t16_row(s, g, j)), ReLU applied
__device__ __forceinline__ h8 relu_b(const f4& lo, const f4& hi) {
    const u4 w = {relu_pk(pk2(lo[0], lo[1])), relu_pk(pk2(lo[2], lo[3])), relu_pk(pk2(hi[0], hi[1])),
                  relu_pk(pk2(hi[2], hi[3]))};
    return __builtin_bit_cast(h8, w);
}

// Encoded input of sample c in lane group g: 24 K slots (t16_slot_feature) as three B-operand k-steps.
// TriangleWave by the tent map (as encode_v3, octaves 3g .. 3g + 2 of each position dim), OneBlob in closed form
// with the clamped wrap (blob_v3), Identity, padding 1.0.
// pad: the value of slot 11 of lane group 0 -- canonical feature 66, the first constant-one column -- which is 1.0
// for compact queries and the query's pad_ for padded ones (nrc_config.query_layout, the reference's Identity(1))
__device__ __forceinline__ void encode16(float p0, float p1, float p2, float bA, float bB, float iA, float iB, int g,
                                         h8 (&x)[3], float pad = 1.0f) {
    const float sc = (float)(1 << (3 * g));
    float t[9];
    const float p[3] = {p0, p1, p2};
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        float v = fmaf(__builtin_amdgcn_fractf(__builtin_fabsf(p[d]) * sc), 2.0f, -1.0f);
        t[3 * d] = v;
        v = tent_step(v);
        t[3 * d + 1] = v;
        v = tent_step(v);
        t[3 * d + 2] = v;
    }
    uint32_t w[12];
    w[0] = pk2_abs_v(t[0], t[1]);
    w[1] = pk2_abs_v(t[2], t[3]);
    w[2] = pk2_abs_v(t[4], t[5]);
    w[3] = pk2_abs_v(t[6], t[7]);
    w[4] = pk2(__builtin_fabsf(t[8]), iA);
    w[5] = pk2(iB, g == 0 ? pad : 1.0f);
    blob_v3(bA, w[6], w[7]);
    blob_v3(bB, w[8], w[9]);
    w[10] = w[11] = 0x3C003C00u;
#pragma unroll
    for (int s = 0; s < 3; ++s) x[s] = __builtin_bit_cast(h8, u4{w[4 * s], w[4 * s + 1], w[4 * s + 2], w[4 * s + 3]});
}

// InputEncoding::Hash in the same 24 slots per lane group (t16_hash_slot_feature): the 4 grid levels 4g .. 4g + 3 of the
// sample (hash_level_feature: tcnn's corners and f16 interpolation, gathers from the f16 training table), pad 1.0,
// Identity, pad, OneBlob as encode16, pads. Levels 0 and 1 (group 0) are dense: the first two levels of every group
// take the dense/hashed select.
// pad: the value of slot 8 of lane group 0 -- canonical feature 62, the first constant-one column -- 1.0 for compact
// queries and the query's pad_ for padded ones
__device__ __forceinline__ void encode16_hash(float p0, float p1, float p2, float bA, float bB, float iA, float iB, int g,
                                              const uint32_t* __restrict__ table, h8 (&x)[3], float pad = 1.0f) {
    uint32_t w[12];
    const int l0 = 4 * g;
    w[0] = hash_level_feature<true>(p0, p1, p2, l0, table);
    w[1] = hash_level_feature<true>(p0, p1, p2, l0 + 1, table);
    w[2] = hash_level_feature<false>(p0, p1, p2, l0 + 2, table);
    w[3] = hash_level_feature<false>(p0, p1, p2, l0 + 3, table);
    w[4] = pk2(g == 0 ? pad : 1.0f, iA);
    w[5] = pk2(iB, 1.0f);
    blob_v3(bA, w[6], w[7]);
    blob_v3(bB, w[8], w[9]);
    w[10] = w[11] = 0x3C003C00u;
#pragma unroll
    for (int s = 0; s < 3; ++s) x[s] = __builtin_bit_cast(h8, u4{w[4 * s], w[4 * s + 1], w[4 * s + 2], w[4 * s + 3]});
}

// The same slots with the 4 level features already computed (hash_feature_kernel's workspace): F[i] = level 4g + i.
__device__ __forceinline__ void encode16_hashf(const uint32_t (&F)[4], float bA, float bB, float iA, float iB, int g,
                                               h8 (&x)[3], float pad = 1.0f) {
    uint32_t w[12];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = F[i];
    w[4] = pk2(g == 0 ? pad : 1.0f, iA);
    w[5] = pk2(iB, 1.0f);
    blob_v3(bA, w[6], w[7]);
    blob_v3(bB, w[8], w[9]);
    w[10] = w[11] = 0x3C003C00u;
#pragma unroll
    for (int s = 0; s < 3; ++s) x[s] = __builtin_bit_cast(h8, u4{w[4 * s], w[4 * s + 1], w[4 * s + 2], w[4 * s + 3]});
}

// ---- training-side pieces shared by nrc_train16.hip and nrc_train_dc.hip ----
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f4 mfma16k16(h4 a, h4 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0); }

// [sample r][64 features] image, 128-B rows of 16 quads (4 features = 8 B). Quad Q of row r sits at slot
// Q ^ swz(r), swz a bijection of r's low 4 bits (bit 0 -> 0, 2 -> 1, 1 -> 2, 3 -> 3). Row writes (ds_write_b64, banks
// (a / 4) mod 32 in 16-lane groups = 16 samples x one quad) see 16 distinct slots; transposed reads (banks (a / 4)
// mod 64 in 32-lane halves = samples 8G + q, G = 0..1, q = 0..3, x quads 4t + p) get 32 distinct 8-byte bank pairs
// because bit 0 of r picks the 256-B half and bits 1, 3 the quad group (tests/test_layouts.py checks both).
__device__ __forceinline__ int swz64(int r) {
    return (r & 1) | (((r >> 2) & 1) << 1) | (((r >> 1) & 1) << 2) | (((r >> 3) & 1) << 3);
}
__device__ __forceinline__ int off64(int r, int Q) { return r * 128 + 8 * (Q ^ swz64(r)); }
// [sample][32 features] image (layer-0 slots 64..95), 64-B rows of 8 quads, swizzled by r's bits 1..3
__device__ __forceinline__ int swz32(int r) { return ((r >> 1) & 1) | (((r >> 2) & 1) << 1) | (((r >> 3) & 1) << 2); }
__device__ __forceinline__ int off32(int r, int Q) { return r * 64 + 8 * (Q ^ swz32(r)); }

__device__ __forceinline__ h4 tr16(const char* p) {
    const s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)p);
    return __builtin_bit_cast(h4, v);
}
__device__ __forceinline__ h8 tr_pair(const char* p0, const char* p1) {
    const h4 a = tr16(p0), b = tr16(p1);
    return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

// backward ReLU gate on packed halves: d where the activation m > 0, else +0. m is +0 or positive bits (relu_pk),
// so min_u16(m, 1) is the 0/1 mask and an integer multiply selects (2 VALU per dword). The min is inline asm (the
// compiler turns a visible min-and-multiply into compares and selects); the multiply, whose result MFMAs read, is
// compiler-visible so that the hazard recognizer sees it.
typedef unsigned short u2h __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t gate_pk(uint32_t d, uint32_t m) {
    uint32_t mask;
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(mask) : "v"(m), "s"(0x00010001u));
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u2h, mask) * __builtin_bit_cast(u2h, d));
}

// the same rows as a delta, gated by the forward activation (B-operand form, same rows)
__device__ __forceinline__ h8 gate_b(const f4& lo, const f4& hi, const h8& a) {
    const u4 m = __builtin_bit_cast(u4, a);
    const u4 w = {gate_pk(pk2(lo[0], lo[1]), m.x), gate_pk(pk2(lo[2], lo[3]), m.y), gate_pk(pk2(hi[0], hi[1]), m.z),
                  gate_pk(pk2(hi[2], hi[3]), m.w)};
    return __builtin_bit_cast(h8, w);
}

// B-operand rows of a 64-row operand (2 k-steps) -> its image row: k-step s elements 4h .. 4h + 3 are quad
// 8s + 4h + g, at the lane's precomputed offsets wo[2s + h] (row_offsets)
__device__ __forceinline__ void put_rows64(char* img, const int (&wo)[4], const h8 (&v)[2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const u4 w = __builtin_bit_cast(u4, v[s]);
        *(u2*)(img + wo[2 * s]) = u2{w.x, w.y};
        *(u2*)(img + wo[2 * s + 1]) = u2{w.z, w.w};
    }
}
__device__ __forceinline__ void row_offsets(int r, int g, int (&wo)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) wo[k] = off64(r, 8 * (k >> 1) + 4 * (k & 1) + g);
}

// dW tiles into a slab as f16 (t16_slab_pos: column pairs, one 16-byte store per lane for both tiles of a pair)
__device__ __forceinline__ u4 pack_pair(const f4& e, const f4& o) {
    return u4{pk2(e[0], e[1]), pk2(e[2], e[3]), pk2(o[0], o[1]), pk2(o[2], o[3])};
}
// raw buffer stores with an explicit cache policy AUX (gfx950 cpol bits: 1 sc0, 2 nt, 16 sc1)
template <int AUX>
__device__ __forceinline__ void slab_pair_b(_Float16* __restrict__ slab, int L, int tm, int tn_even, int lane, const u4& v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, buffer_rsrc(slab, slab_floats(0) * 2),
                                           t16_slab_base(L, tm, tn_even) * 2 + lane * 16, 0, AUX);
}
template <int AUX>
__device__ __forceinline__ void slab_single_b(_Float16* __restrict__ slab, int L, int tm, int tn, int lane, const f4& v) {
    const u2 w = {pk2(v[0], v[1]), pk2(v[2], v[3])};
    __builtin_amdgcn_raw_buffer_store_b64(w, buffer_rsrc(slab, slab_floats(0) * 2), t16_slab_pos(L, tm, tn, lane, 0) * 2,
                                          0, AUX);
}

// DPP sum over a 16-lane row (row_ror 8, 4, 2, 1): every lane of the row ends with the row's total
__device__ __forceinline__ float row_sum16(float v) {
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x122, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x121, 0xF, 0xF, false));
    return v;
}

// delta_{L-1} = (W_L^T delta_L) * [a_{L-1} > 0] for G 16-sample groups of a wave (W: 4 M-blocks x 2 k-steps)
template <int G>
__device__ __forceinline__ void chain_groups(const h8 (&W)[4][2], const h8 (&d)[G][2], const h8 (&a)[G][2],
                                             h8 (&dn)[G][2]) {
    f4 cc[G][4];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int u = 0; u < G; ++u) {
            cc[u][mb] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 2; ++s) cc[u][mb] = mfma16(W[mb][s], d[u][s], cc[u][mb]);
        }
#pragma unroll
    for (int u = 0; u < G; ++u)
#pragma unroll
        for (int s = 0; s < 2; ++s) dn[u][s] = gate_b(cc[u][2 * s], cc[u][2 * s + 1], a[u][s]);
}

// RelativeL2Luminance of one 16-sample group on the f16 prediction (rows 0..2 = registers 0..2 of lane
// group 0): adds this lane's loss terms to lossv and returns the loss-scaled f16 gradient delta_5 as a 16x16x16 B
// operand (rows 4g .. 4g + 3). One division per sample (1 / (denom * n_total)) instead of two per channel.
__device__ __forceinline__ h4 loss_delta5(const f4& o, const float (&tg)[3], bool valid, int g, float n_total,
                                          float loss_scale, float& lossv) {
    h4 d5 = h4{};
    if (g == 0) {
        float y[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) y[k] = (float)(_Float16)fmaxf(o[k], 0.0f);
        const float lum = 0.299f * y[0] + 0.587f * y[1] + 0.114f * y[2];
        const float inv = 1.0f / ((lum * lum + NRC_LUM_EPS) * n_total);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float diff = y[k] - tg[k];
            lossv += valid ? diff * diff * inv : 0.0f;
            d5[k] = (valid && y[k] > 0.0f) ? (_Float16)(loss_scale * 2.0f * diff * inv) : (_Float16)0.0f;
        }
    }
    return d5;
}

}  // namespace t16
}  // namespace nrc_amd
