// nrc_device.h — device-side helpers shared by the gfx950 kernel translation units (nrc_kernels.hip,
// nrc_train16.hip): operand types, the RadianceQuery lane loads, f16 packing, the encoder pieces (tent-map triangle
// wave, closed-form OneBlob), raw buffer descriptors and the LDS-only barrier.
#pragma once

#include "nrc_internal.h"

namespace nrc_amd {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f16v mfma(h8 a, h8 b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f16v zero16() {
    f16v z = {};
    return z;
}

// ------------------------------------------------------------------------------------------------
// Composite encoding (NRCNetworkConfigs.h:51-81), computed in f32 per lane, 40 K slots per lane half.
// ------------------------------------------------------------------------------------------------
struct QLane {
    float p0, p1, p2;  // position (both halves)
    float b0, b1, b2;  // OneBlob inputs 3+3h .. 5+3h (FrequencySH: direction theta, phi, OneBlob input 5+2h)
    float i0, i1, i2;  // Identity inputs 9+3h .. 11+3h
    float x3;          // FrequencySH only: OneBlob input 6+2h
};

// PADQ: padded 16-float records (nrc_config.query_layout = NRC_QUERY_PADDED): pad_ at float 3 (into x3), the rest one
// float further
template <bool PADQ = false>
__device__ __forceinline__ QLane load_q(const float* __restrict__ q, int64_t s, int h) {
    constexpr int X = PADQ ? 1 : 0;
    const float* r = q + s * (NRC_INPUT_DIMS + X);
    QLane Q;
    Q.p0 = r[0];
    Q.p1 = r[1];
    Q.p2 = r[2];
    Q.x3 = PADQ ? r[3] : 0.0f;
    const float* rb = r + 3 + X + 3 * h;
    Q.b0 = rb[0];
    Q.b1 = rb[1];
    Q.b2 = rb[2];
    const float* ri = r + 9 + X + 3 * h;
    Q.i0 = ri[0];
    Q.i1 = ri[1];
    Q.i2 = ri[2];
    return Q;
}

// FrequencySH extension: both halves need the direction (dims 3, 4); OneBlob dims 5+2h, 6+2h.
__device__ __forceinline__ QLane load_q_sh(const float* __restrict__ q, int64_t s, int h) {
    const float* r = q + s * NRC_INPUT_DIMS;
    QLane Q;
    Q.p0 = r[0];
    Q.p1 = r[1];
    Q.p2 = r[2];
    Q.b0 = r[3];
    Q.b1 = r[4];
    Q.b2 = r[5 + 2 * h];
    Q.x3 = r[6 + 2 * h];
    const float* ri = r + 9 + 3 * h;
    Q.i0 = ri[0];
    Q.i1 = ri[1];
    Q.i2 = ri[2];
    return Q;
}

template <int ENC, bool PADQ = false>
__device__ __forceinline__ QLane load_q_enc(const float* __restrict__ q, int64_t s, int h) {
    static_assert(!(PADQ && ENC == 2), "FrequencySH has no padded layout");
    if constexpr (ENC == 2) return load_q_sh(q, s, h);
    else return load_q<PADQ>(q, s, h);
}

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk2(float a, float b) {
    const f2 v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, h2));  // v_cvt_pk_f16_f32 (RNE)
}

// pk2(|a|, |b|) with the absolute values as input modifiers of v_cvt_pk_f16_f32 (the compiler otherwise masks the
// f16 result with a separate v_and).
__device__ __forceinline__ uint32_t pk2_abs(float a, float b) {
    uint32_t r;
    asm("v_cvt_pk_f16_f32 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// Output modifiers (omod mul:2) are ignored by the hardware while MODE.IEEE is set or f32 output denormals are
// enabled (both are the HIP kernel defaults), which is why the CHAIN encoder failed on hardware. A kernel that
// uses it first clears MODE.IEEE (bit 9) and switches MODE.FP_DENORM[f32] (bits 5:4) to "allow input denormals,
// flush output denormals". Inference results are unchanged: every f32 value that could be flushed (< 1.2e-38)
// becomes the same f16 anyway, and the only min/max in the kernel (v_pk_max_f16 ReLU against 0) returns the
// non-NaN operand for a quiet NaN in both modes.
__device__ __forceinline__ void fp32_flush_output_denorms() {
    __builtin_amdgcn_s_setreg((1 << 11) | (4 << 6) | 1 /* hwreg(HW_REG_MODE, 4, 2) */, 1u);
    __builtin_amdgcn_s_setreg((0 << 11) | (9 << 6) | 1 /* hwreg(HW_REG_MODE, 9, 1) = IEEE */, 0u);
}

// 2 * frac(x) via v_fract_f32's mul:2 output modifier (needs fp32_flush_output_denorms, see above).
__device__ __forceinline__ float fract2(float x) {
    float r;
    asm("v_fract_f32_e64 %0, %1 mul:2" : "=v"(r) : "v"(x));
    return r;
}
// 2 * frac(|x|): the triangle wave is even, tri(-u) = tri(u), and frac of a non-negative value is exact, so the
// doubling chain started from |x| is exact in every octave (frac(x) of a negative x rounds x + 1, and doubling
// would amplify that rounding 2^5-fold).
__device__ __forceinline__ float fract2_abs(float x) {
    float r;
    asm("v_fract_f32_e64 %0, |%1| mul:2" : "=v"(r) : "v"(x));
    return r;
}

__device__ __forceinline__ float tent_step(float x) { return __builtin_fmaf(__builtin_fabsf(x), 2.0f, -1.0f); }

__device__ __forceinline__ float step01(float t, float edge) {  // 1 for t >= edge, else 0 (t, edge on the 2^-21 grid)
    return __builtin_amdgcn_fmed3f(__builtin_fmaf(t, 0x1p21f, 1.0f - edge * 0x1p21f), 0.0f, 1.0f);
}

__device__ __forceinline__ void blob_v3(float x, uint32_t& lo, uint32_t& hi) {
    const float t = __builtin_amdgcn_fmed3f(x * 4.0f, -5.0f, 8.0f);
    const float fr = __builtin_amdgcn_fractf(t);
    uint32_t sh;  // 16 * ((floor(t) - 1) & 3) in the low 6 bits: v_cvt_flr_i32_f32 + v_lshl_add_u32 (the compiler
                  // emits floor + cvt + shift + add for the C form)
    asm("v_cvt_flr_i32_f32 %0, %1\n\tv_lshl_add_u32 %0, %0, 4, 48" : "=&v"(sh) : "v"(t));
    const float fr2 = fr * fr;
    float A = fmaf(-fr, fmaf(fr2, fmaf(fr2, 3.0f / 16.0f, -10.0f / 16.0f), 15.0f / 16.0f), 0.5f);
    const float w = 1.0f - fr;
    const float w2 = w * w;
    float B = fmaf(w, fmaf(w2, fmaf(w2, 3.0f / 16.0f, -10.0f / 16.0f), 15.0f / 16.0f), 0.5f);
    A = __builtin_amdgcn_fmed3f(A, step01(t, 8.0f), step01(t, -4.0f));
    B = fmaxf(B, step01(t, 7.0f));
    const float M1 = B - A, M2 = 1.0f - B;
    const uint64_t v = (uint64_t)pk2(A, M1) | ((uint64_t)pk2(M2, 0.0f) << 32);
    const uint64_t r = (v << (sh & 63u)) | (v >> ((64u - sh) & 63u));
    lo = (uint32_t)r;
    hi = (uint32_t)(r >> 32);
}

typedef _Float16 h2v __attribute__((ext_vector_type(2)));

// Raw buffer descriptors (gfx9 dword3 = 0x00020000, stride 0): loads past num_records return 0 and stores past it
// are dropped by the hardware, which lets a tile's tail and inactive lanes go without branches.
typedef uint32_t u3 __attribute__((ext_vector_type(3)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
constexpr int kBufferOff = 0x40000000;  // an offset past every descriptor below: the access is dropped
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_rsrc(const void* base, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}
// valid rows of the 32-row tile starting at s0 in an array of n rows (0..32)
__device__ __forceinline__ int tile_rows(int64_t n, int64_t s0) {
    const int64_t left = n - s0;
    return (int)(left >= 32 ? 32 : left > 0 ? left : 0);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops (lgkmcnt) but not for its
// outstanding global stores (the weight-gradient slab writes drain in the background) — __syncthreads()
// would emit s_waitcnt vmcnt(0) first. The asm "memory" clobber keeps the compiler's memory ops on
// their side of the barrier.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---- tcnn Adam + EMA (optimizers/adam.h, exponential_moving_average.h) of one parameter with its f16
// image packs, shared by reduce_adam_kernel (nrc_kernels.hip) and the fused optimizer phase of nrc_train16.hip.
// adam_pack_one (mode kReduceFused) split into its loads and the rest, same float operations
struct AdamIn {
    float w, m, v, ema;
    int fp, ft, bp;
};
__device__ __forceinline__ AdamIn adam_load(int p, const ModelBuffers& mb) {
    return AdamIn{mb.params[p], mb.m[p], mb.v[p], mb.ema[p], mb.fwd_pos[p], mb.fwdt_pos[p], mb.bwd_pos[p]};
}
__device__ __forceinline__ void adam_pack_pre(int p, float gsum, const AdamIn& in, const ModelBuffers& mb,
                                              const OptimArgs& oa, float lr_t, float ema_debias) {
#pragma clang fp contract(off)
    float gradient = gsum / oa.loss_scale;
    float w = in.w;
    gradient += oa.l2_reg * w;
    const float gsq = gradient * gradient;
    const float m1 = oa.beta1 * in.m + (1.0f - oa.beta1) * gradient;
    const float v1 = oa.beta2 * in.v + (1.0f - oa.beta2) * gsq;
    mb.m[p] = m1;
    mb.v[p] = v1;
    const float eff = lr_t / (sqrtf(v1) + oa.eps);
    w = w - eff * m1;
    mb.params[p] = w;
    const float e = in.ema * oa.ema_decay + w * (1.0f - oa.ema_decay);
    mb.ema[p] = e;
    const float inf = e / ema_debias;
    mb.infer[p] = inf;
    mb.wf_train[in.ft] = (_Float16)w;
    mb.wf_infer[in.fp] = (_Float16)inf;
    if (mb.wf_infer16) mb.wf_infer16[in.ft] = (_Float16)inf;
    if (in.bp >= 0) mb.wb_train[in.bp] = (_Float16)w;
}

}  // namespace nrc_amd
