// nrc_t16.h — device pieces of the "t16" layout (v_mfma_f32_16x16x32_f16, nrc_internal.h) shared by the training
// kernel (nrc_train16.hip) and the 16x16x32 inference kernel (nrc_infer16.hip): the MFMA wrapper, the packed ReLU,
// accumulator -> B-operand conversion and the 96-slot encoder (t16_slot_feature).
#pragma once

#include "nrc_device.h"

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
__device__ __forceinline__ void encode16(float p0, float p1, float p2, float bA, float bB, float iA, float iB, int g,
                                         h8 (&x)[3]) {
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
    w[5] = pk2(iB, 1.0f);
    blob_v3(bA, w[6], w[7]);
    blob_v3(bB, w[8], w[9]);
    w[10] = w[11] = 0x3C003C00u;
#pragma unroll
    for (int s = 0; s < 3; ++s) x[s] = __builtin_bit_cast(h8, u4{w[4 * s], w[4 * s + 1], w[4 * s + 2], w[4 * s + 3]});
}

}  // namespace t16
}  // namespace nrc_amd
