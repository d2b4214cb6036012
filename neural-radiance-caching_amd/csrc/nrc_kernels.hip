// nrc_kernels.hip — gfx950 (CDNA4) kernels of the NRC query/train hot path.
//
// Replaces the tiny-cuda-nn calls the reference makes from /root/reference/nrc/src/NRCNetwork.cu:
//   network->inference      (:76)    -> infer_kernel       (fused Composite encode + 64x5 MLP + cast)
//   trainer->training_step  (:53)   -> train_kernel        (encode + fwd + RelativeL2Luminance + bwd +
//                                                           per-block weight-gradient partials)
//                                     reduce_adam_kernel  (fixed-order dW reduce + Adam + EMA + f16 repack)
//   trainer->loss           (:55)   -> loss partials reduced in reduce_adam_kernel
//
// Design: every matmul is a chain of v_mfma_f32_32x32x16_f16 with samples on the MFMA
// column (lane) axis and features on the row axis, so each layer's f32 accumulator converts in
// registers into the next layer's B operand (no LDS round trip between layers). Weights live in LDS
// as pre-swizzled A-operand "fragment images" (one ds_read_b128 per MFMA), packed by
// reduce_adam_kernel after every optimizer step. Weight gradients (a contraction over samples) go
// through a per-block LDS transpose read with ds_read_b64_tr_b16.
#include <cstdlib>
#include <type_traits>

#include "nrc_device.h"
#include "nrc_hash.h"

namespace nrc_amd {

// TriangleWave [L spec choice, SURVEY A.2]: |2 frac(u) - 1|.
__device__ __forceinline__ float tri(float u) {
    const float fr = u - floorf(u);
    return fabsf(2.0f * fr - 1.0f);
}

// OneBlob quartic CDF with inv_radius = n_bins = 4.
__device__ __forceinline__ float qcdf(float x) {
    const float u = x * 4.0f;
    const float u2 = u * u;
    const float u4 = u2 * u2;
    const float v = (1.0f / 16.0f) * u * (15.0f - 10.0f * u2 + 3.0f * u4) + 0.5f;
    return fminf(fmaxf(v, 0.0f), 1.0f);
}

__device__ __forceinline__ void one_blob(float x, float* o) {
    float left[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const float d = 0.25f * (float)b - x;
        left[b] = qcdf(d) + qcdf(d - 1.0f) + qcdf(d + 1.0f);
    }
    o[0] = left[1] - left[0];
    o[1] = left[2] - left[1];
    o[2] = left[3] - left[2];
    o[3] = left[0] + 1.0f - left[3];
}

// v[n] = value of K slot n (n = 8*kk + j) for lane half h, see slot_feature().
__device__ __forceinline__ void encode_f32(const QLane& Q, int h, float (&v)[40]) {
    const float hs = h ? 64.0f : 1.0f;  // octaves 6..11 for the upper half
    const float p[3] = {Q.p0 * hs, Q.p1 * hs, Q.p2 * hs};
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int k = 0; k < 6; ++k) v[d * 6 + k] = tri(p[d] * (float)(1 << k));
    one_blob(Q.b0, &v[18]);
    one_blob(Q.b1, &v[22]);
    one_blob(Q.b2, &v[26]);
    v[30] = Q.i0;
    v[31] = Q.i1;
    v[32] = Q.i2;
#pragma unroll
    for (int n = 33; n < 40; ++n) v[n] = 1.0f;
}

__device__ __forceinline__ void encode(const QLane& Q, int h, h8 (&x)[5]) {
    float v[40];
    encode_f32(Q, h, v);
#pragma unroll
    for (int kk = 0; kk < 5; ++kk)
#pragma unroll
        for (int j = 0; j < 8; ++j) x[kk][j] = (_Float16)v[8 * kk + j];
}

// Accumulator rows 8s..8s+7 -> f16 B fragment of the next layer, ReLU applied (ReLU commutes with
// round-to-nearest, so this equals f16(relu(acc))).
__device__ __forceinline__ void relu_pack(const f16v& a, h8& lo, h8& hi) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        lo[j] = (_Float16)fmaxf(a[j], 0.0f);
        hi[j] = (_Float16)fmaxf(a[8 + j], 0.0f);
    }
}

// Backward ReLU: delta = f16(acc) where the forward activation a > 0, else 0.
__device__ __forceinline__ void mask_pack(const f16v& a, const h8& m_lo, const h8& m_hi, h8& lo, h8& hi) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        lo[j] = m_lo[j] > (_Float16)0.0f ? (_Float16)a[j] : (_Float16)0.0f;
        hi[j] = m_hi[j] > (_Float16)0.0f ? (_Float16)a[8 + j] : (_Float16)0.0f;
    }
}

template <int KK>
__device__ __forceinline__ void mlp_layer(const h8* __restrict__ lw, int frag0, const h8 (&x)[KK], int lane,
                                          f16v& a0, f16v& a1) {
    a0 = zero16();
    a1 = zero16();
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
        a0 = mfma(lw[(frag0 + kk) * 64 + lane], x[kk], a0);
        a1 = mfma(lw[(frag0 + KK + kk) * 64 + lane], x[kk], a1);
    }
}

// Forward through the five hidden-producing layers; a[l][*] = input of layer l+1 (B fragments).
__device__ __forceinline__ void mlp_hidden(const h8* __restrict__ lw, const h8 (&x)[5], int lane, h8 (&a)[5][4]) {
    f16v c0, c1;
    mlp_layer<5>(lw, fwd_frag(0, 0, 0), x, lane, c0, c1);
    relu_pack(c0, a[0][0], a[0][1]);
    relu_pack(c1, a[0][2], a[0][3]);
#pragma unroll
    for (int l = 1; l < 5; ++l) {
        mlp_layer<4>(lw, fwd_frag(l, 0, 0), a[l - 1], lane, c0, c1);
        relu_pack(c0, a[l][0], a[l][1]);
        relu_pack(c1, a[l][2], a[l][3]);
    }
}

__device__ __forceinline__ f16v mlp_out(const h8* __restrict__ lw, const h8 (&a5)[4], int lane) {
    f16v o = zero16();
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) o = mfma(lw[fwd_frag(5, 0, kk) * 64 + lane], a5[kk], o);
    return o;
}

// Global -> LDS copy of a fragment image with every load in flight before the first LDS store
// (a plain strided loop waits one round trip per iteration: ~7k cycles for 80 KiB).
template <int THREADS, int COUNT>
__device__ __forceinline__ void copy_to_lds(h8* __restrict__ dst, const h8* __restrict__ src) {
    constexpr int PER = (COUNT + THREADS - 1) / THREADS;
    h8 v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int i = threadIdx.x + k * THREADS;
        if (i < COUNT) v[k] = src[i];
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int i = threadIdx.x + k * THREADS;
        if (i < COUNT) dst[i] = v[k];
    }
}

#if NRC_DEBUG_KERNELS  // round-1 reference kernel (debug library only)
// ------------------------------------------------------------------------------------------------
// Inference: persistent waves, 32 queries per wave-iteration.
// ------------------------------------------------------------------------------------------------
constexpr int kInferThreads = 256;

__global__ __launch_bounds__(kInferThreads) void infer_kernel(const float* __restrict__ q, float* __restrict__ out,
                                                              int64_t n, const h8* __restrict__ wf) {
    __shared__ __attribute__((aligned(16))) h8 lw[kFwdFrags * 64];
    copy_to_lds<kInferThreads, kFwdFrags * 64>(lw, wf);
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int h = lane >> 5, r = lane & 31;
    const int64_t ntiles = (n + 31) >> 5;
    const int64_t wstride = (int64_t)gridDim.x * (kInferThreads / 64);
    int64_t tile = (int64_t)blockIdx.x * (kInferThreads / 64) + (threadIdx.x >> 6);
    if (tile >= ntiles) return;
    const int64_t last = n - 1;

    QLane Q = load_q(q, min(tile * 32 + r, last), h);
    for (; tile < ntiles; tile += wstride) {
        const int64_t s = tile * 32 + r;
        h8 x[5];
        encode(Q, h, x);
        const int64_t nt = tile + wstride;
        if (nt < ntiles) Q = load_q(q, min(nt * 32 + r, last), h);

        h8 a[5][4];
        mlp_hidden(lw, x, lane, a);
        const f16v o = mlp_out(lw, a[4], lane);
        // Output rows 0..2 sit in registers 0..2 of lanes 0..31 (C/D map row = (reg&3)+8(reg>>2)+4h).
        // tcnn casts the f16 network output to f32 (trim_and_cast).
        if (h == 0 && s < n) {
            float* dst = out + s * NRC_OUTPUT_DIMS;
            dst[0] = (float)(_Float16)fmaxf(o[0], 0.0f);
            dst[1] = (float)(_Float16)fmaxf(o[1], 0.0f);
            dst[2] = (float)(_Float16)fmaxf(o[2], 0.0f);
        }
    }
}

#endif

// ------------------------------------------------------------------------------------------------
// Inference v2: VALU-lean encoding, packed-f16 ReLU, LDS-resident weights, TILES x 32 queries per
// wave iteration (each weight fragment read from LDS feeds TILES MFMAs).
// ------------------------------------------------------------------------------------------------
// OneBlob(4 bins) of one input in closed form. tcnn's formula sums 12 quartic-CDF terms;
// at most two are unsaturated: with t = 4x, fl = floor(t), fr = t - fl the kernel mass falls into the
// unit intervals j = fl-1, fl, fl+1 as A, B-A, 1-B (A = K(-fr), B = K(1-fr)); interval j lands in bin
// j & 3 when -4 <= j <= 7 and in bin 3 otherwise (the period-1 wrap of the formula). Returns the four
// bins as packed f16 pairs (bins 0,1 | bins 2,3). IN_RANGE: the caller guarantees -3 <= t < 7, where all
// three intervals land in bins j & 3 and the wrap bookkeeping (selects, the bin-3 surplus) drops out.
template <bool IN_RANGE = false>
__device__ __forceinline__ void blob_fast(float x, uint32_t& lo, uint32_t& hi) {
    const float t = x * 4.0f;
    const float fl = floorf(t);
    const float fr = t - fl;
    const float fr2 = fr * fr;
    const float A = fmaf(-fr, fmaf(fr2, fmaf(fr2, 3.0f / 16.0f, -10.0f / 16.0f), 15.0f / 16.0f), 0.5f);
    const float w = 1.0f - fr;
    const float w2 = w * w;
    const float B = fmaf(w, fmaf(w2, fmaf(w2, 3.0f / 16.0f, -10.0f / 16.0f), 15.0f / 16.0f), 0.5f);
    const float M1 = B - A, M2 = 1.0f - B;
    const int j0 = (int)fl - 1;
    const uint32_t s = (uint32_t)(j0 & 3) << 4;
    if constexpr (IN_RANGE) {
        uint64_t v = (uint64_t)pk2(A, M1) | ((uint64_t)pk2(M2, 0.0f) << 32);
        v = (v << s) | (v >> ((64u - s) & 63u));
        lo = (uint32_t)v;
        hi = (uint32_t)(v >> 32);
    } else {
        const bool in0 = (unsigned)(j0 + 4) <= 11u;
        const bool in1 = (unsigned)(j0 + 5) <= 11u;
        const bool in2 = (unsigned)(j0 + 6) <= 11u;
        const float m0 = in0 ? A : 0.0f, m1 = in1 ? M1 : 0.0f, m2 = in2 ? M2 : 0.0f;
        const float extra = (in0 ? 0.0f : A) + (in1 ? 0.0f : M1) + (in2 ? 0.0f : M2);
        uint64_t v = (uint64_t)pk2(m0, m1) | ((uint64_t)pk2(m2, 0.0f) << 32);
        v = (v << s) | (v >> ((64u - s) & 63u));
        lo = (uint32_t)v;
        h2 hv = __builtin_bit_cast(h2, (uint32_t)(v >> 32));
        hv[1] = hv[1] + (_Float16)extra;
        hi = __builtin_bit_cast(uint32_t, hv);
    }
}

// OneBlob of N inputs of this lane into words (w[2i], w[2i+1]). A wave whose inputs all satisfy -3 <= 4x < 7
// (every query of a renderer stream: OneBlob inputs are in [0, 1]) takes the branch without the wrap
// bookkeeping (~17 VALU less per input); bit-identical to the general branch for those inputs.
template <int N>
__device__ __forceinline__ void blob_many(const float (&xs)[N], uint32_t (&lo)[N], uint32_t (&hi)[N]) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const float t = xs[i] * 4.0f;
        ok = ok && (t >= -3.0f) && (t < 7.0f);
    }
    if (__all(ok)) {
#pragma unroll
        for (int i = 0; i < N; ++i) blob_fast<true>(xs[i], lo[i], hi[i]);
    } else {
        asm volatile("; OneBlob wrap path");  // a side effect: keeps this a branch instead of both arms + selects
#pragma unroll
        for (int i = 0; i < N; ++i) blob_fast<false>(xs[i], lo[i], hi[i]);
    }
}

__device__ __forceinline__ float tri_fast(float u) {
    return fabsf(fmaf(__builtin_amdgcn_fractf(u), 2.0f, -1.0f));
}

// 40 K slots of lane half h as 20 packed f16 pairs = 5 B fragments (same slot map as encode()).
// CHAIN: triangle-wave octaves by doubling through v_fract's mul:2 output modifier (1 VALU per octave instead
// of mul + fract + half an fma); only valid after fp32_flush_output_denorms().
template <bool CHAIN = false>
__device__ __forceinline__ void encode_fast(const QLane& Q, int h, h8 (&x)[5]) {
    uint32_t w[20];
    const float hs = h ? 64.0f : 1.0f;
    const float p[3] = {Q.p0 * hs, Q.p1 * hs, Q.p2 * hs};
    if (CHAIN) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            float g[6];
            g[0] = fract2_abs(p[d]);
#pragma unroll
            for (int k = 1; k < 6; ++k) g[k] = fract2(g[k - 1]);
#pragma unroll
            for (int k = 0; k < 6; k += 2) w[(d * 6 + k) >> 1] = pk2_abs(g[k] - 1.0f, g[k + 1] - 1.0f);
        }
    } else {
#pragma unroll
        for (int d = 0; d < 3; ++d)
#pragma unroll
            for (int k = 0; k < 6; k += 2)
                w[(d * 6 + k) >> 1] = pk2(tri_fast(p[d] * (float)(1 << k)), tri_fast(p[d] * (float)(2 << k)));
    }
    {
        const float xb[3] = {Q.b0, Q.b1, Q.b2};
        uint32_t lo[3], hi[3];
        blob_many<3>(xb, lo, hi);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            w[9 + 2 * i] = lo[i];
            w[9 + 2 * i + 1] = hi[i];
        }
    }
    w[15] = pk2(Q.i0, Q.i1);
    w[16] = pk2(Q.i2, 1.0f);
    w[17] = w[18] = w[19] = 0x3C003C00u;  // pad features = 1.0
#pragma unroll
    for (int kk = 0; kk < 5; ++kk) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        u4 t4 = {w[4 * kk], w[4 * kk + 1], w[4 * kk + 2], w[4 * kk + 3]};
        x[kk] = __builtin_bit_cast(h8, t4);
    }
}

// ------------------------------------------------------------------------------------------------
// Encoder v3 (round 2): fewer VALU for the same 40 K slots per lane half (slot map unchanged, slot_feature()).
//
// TriangleWave by the tent map. With x_k = 2 frac(2^k u) - 1, tri_k = |x_k| and x_{k+1} = 2 |x_k| - 1 (doubling a
// point of the period-1 triangle wave folds it: frac(2^(k+1) u) = 2 frac(2^k u) - [frac(2^k u) >= 1/2]), so each
// further octave is ONE v_fma_f32 with an |.| input modifier, and |x_k| is the cvt's input modifier: 1.5 VALU per
// feature instead of 2.5 (fract, subtract, half a cvt). x_0 = 2 frac(|u|) - 1 (the wave is even). Rounding: 2|x| - 1
// is exact unless |x| < 1/4, where it rounds by <= 2^-25; the doubling carries an error e to 2e, so after the five
// steps of a lane half the features are within 2^-19 (1.9e-6) absolute of the directly evaluated wave.
//
// OneBlob with the wrap folded into two clamps. The closed form of blob_fast puts the masses A, B - A, 1 - B of the
// intervals j0 = floor(4x) - 1 .. j0 + 2 into bins (j0 + i) & 3; tcnn's formula sends an interval outside
// [-4, 7] to bin 3 instead. For t = 4x clamped to [-5, 8] that is exactly: A -> 0 when t < -4, A -> 1 when t >= 8,
// B -> 1 when t >= 7 (every other out-of-range case is equivalent to one of these at the clamp ends), i.e. a med3 of
// A and a max of B against step functions of t; the masses are rotated into place as before. The reference feeds
// raw angles (theta in [0, pi], phi in (-pi, pi]) to OneBlob, so Cornell waves always take the wrap: this replaces
// blob_many's wave-uniform branch (~25 extra VALU per input on the wrap side) by ~6 VALU per input on one path.
// ------------------------------------------------------------------------------------------------
// PADQ (padded RadianceQuery, nrc_config.query_layout): slot 33 of lane half 0 -- the first constant-one column,
// canonical feature 66 -- carries the query's pad_ (Q.x3) instead: the reference's Identity(1) of pad_ (layout.h)
template <bool PADQ = false>
__device__ __forceinline__ void encode_v3(const QLane& Q, int h, h8 (&x)[5]) {
    uint32_t w[20];
    const float hs = h ? 64.0f : 1.0f;  // octaves 6..11 for the upper half
    const float p[3] = {Q.p0 * hs, Q.p1 * hs, Q.p2 * hs};
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        float g[6];
        g[0] = fmaf(__builtin_amdgcn_fractf(__builtin_fabsf(p[d])), 2.0f, -1.0f);
#pragma unroll
        for (int k = 1; k < 6; ++k) g[k] = tent_step(g[k - 1]);
#pragma unroll
        for (int k = 0; k < 6; k += 2) w[(d * 6 + k) >> 1] = pk2_abs(g[k], g[k + 1]);
    }
    blob_v3(Q.b0, w[9], w[10]);
    blob_v3(Q.b1, w[11], w[12]);
    blob_v3(Q.b2, w[13], w[14]);
    w[15] = pk2(Q.i0, Q.i1);
    w[16] = pk2(Q.i2, PADQ && h == 0 ? Q.x3 : 1.0f);
    w[17] = w[18] = w[19] = 0x3C003C00u;  // pad features = 1.0
#pragma unroll
    for (int kk = 0; kk < 5; ++kk) {
        typedef uint32_t w4 __attribute__((ext_vector_type(4)));
        w4 t4 = {w[4 * kk], w[4 * kk + 1], w[4 * kk + 2], w[4 * kk + 3]};
        x[kk] = __builtin_bit_cast(h8, t4);
    }
}

// Diagnostic clock of the inference kernels (ABL & 512): per wave (s_memtime cycles of the persistent loop, the
// s_memrealtime 100 MHz ticks at loop start, loop end and wave start, HW_ID and XCC_ID), read back by
// nrc_debug_read_infer_clock.
#if NRC_DEBUG_KERNELS
constexpr int kInferClockWavesMax = 8192;
__device__ uint64_t g_infer_clock[6 * kInferClockWavesMax];
#endif

// ------------------------------------------------------------------------------------------------
// HashGrid (InputEncoding::Hash, NRCNetworkConfigs.h:94-103; spec in oracle/nrc_hash_oracle.c): lane half h
// encodes levels 8h..8h+7 of its query. Table: f16 [entry][2] (one 4-B half2 gather per corner).
// ------------------------------------------------------------------------------------------------
// A tile's 32 RadianceQuery rows (60 B each) through raw buffer loads: the descriptor (scalar: tile base, valid rows)
// returns 0 past n, so there is no per-lane clamp or 64-bit address arithmetic; vo = this lane's constant byte
// offsets of its three 12-byte pieces (position, OneBlob inputs 3+3h.., Identity inputs 9+3h..).
struct QOffsets {
    int p, b, i;
};
// PADQ (padded 64-B records, vo from q_offsets<true>): the position and pad_ as one 16-byte load, pad_ in Q.x3.
template <bool PADQ = false>
__device__ __forceinline__ QLane load_q_tile(const float* __restrict__ q, int64_t n, int64_t tile, const QOffsets& vo) {
    typedef float f3 __attribute__((ext_vector_type(3)));
    typedef float f4 __attribute__((ext_vector_type(4)));
    constexpr int kQD = PADQ ? NRC_INPUT_DIMS_PADDED : NRC_INPUT_DIMS;
    const int64_t s0 = tile * 32;
    const __amdgpu_buffer_rsrc_t rs = buffer_rsrc(q + s0 * kQD, tile_rows(n, s0) * (kQD * 4));
    // whole-vector bit_casts (clang 22 element bit_cast bug, see infer_v2_body)
    QLane Q;
    if constexpr (PADQ) {
        const f4 a = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo.p, 0, 0));
        Q.p0 = a.x; Q.p1 = a.y; Q.p2 = a.z;
        Q.x3 = a.w;
    } else {
        const f3 a = __builtin_bit_cast(f3, __builtin_amdgcn_raw_buffer_load_b96(rs, vo.p, 0, 0));
        Q.p0 = a.x; Q.p1 = a.y; Q.p2 = a.z;
        Q.x3 = 0.0f;
    }
    const f3 b = __builtin_bit_cast(f3, __builtin_amdgcn_raw_buffer_load_b96(rs, vo.b, 0, 0));
    const f3 c = __builtin_bit_cast(f3, __builtin_amdgcn_raw_buffer_load_b96(rs, vo.i, 0, 0));
    Q.b0 = b.x; Q.b1 = b.y; Q.b2 = b.z;
    Q.i0 = c.x; Q.i1 = c.y; Q.i2 = c.z;
    return Q;
}
// lane (r, h)'s byte offsets in a tile of records: position (+ pad_), OneBlob inputs 3+3h.., Identity inputs 9+3h..
// (padded records: one float further each)
template <bool PADQ>
__device__ __forceinline__ QOffsets q_offsets(int r, int h) {
    constexpr int R = PADQ ? 64 : 60, X = PADQ ? 4 : 0;
    return QOffsets{r * R, r * R + 12 + X + 12 * h, r * R + 36 + X + 12 * h};
}

// 32 K slots of lane half h (see hash_slot_feature): 8 hash levels (16 features), 3 OneBlob dims, 3 identity,
// one pad; as 4 B fragments.
// PADQ: slot 31 of lane half 0 carries pad_ (Q.x3), as encode_hashf
template <bool PADQ = false>
__device__ __forceinline__ void encode_hash(const QLane& Q, int h, const uint32_t* __restrict__ table, h8 (&x)[4]) {
    uint32_t w[16];
    // levels in two groups of 4 with a scheduling fence between them: the compiler otherwise hoists every
    // level's gathers (8 x 4 x 20 B per lane) ahead of the interpolation and runs out of registers
    w[0] = hash_level_feature<true>(Q.p0, Q.p1, Q.p2, 8 * h + 0, table);
    w[1] = hash_level_feature<true>(Q.p0, Q.p1, Q.p2, 8 * h + 1, table);
#pragma unroll
    for (int i = 2; i < 8; ++i) {
        if (i == 4) asm volatile("" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]) : : "memory");
        w[i] = hash_level_feature<false>(Q.p0, Q.p1, Q.p2, 8 * h + i, table);
    }
    // OneBlob as encoder v3 (clamped wrap, one path): the reference's raw-angle inputs send every Cornell wave down
    // blob_many's wrap branch (~25 VALU more per input)
    blob_v3(Q.b0, w[8], w[9]);
    blob_v3(Q.b1, w[10], w[11]);
    blob_v3(Q.b2, w[12], w[13]);
    w[14] = pk2(Q.i0, Q.i1);
    w[15] = pk2(Q.i2, PADQ && h == 0 ? Q.x3 : 1.0f);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        u4 t4 = {w[4 * kk], w[4 * kk + 1], w[4 * kk + 2], w[4 * kk + 3]};
        x[kk] = __builtin_bit_cast(h8, t4);
    }
}

// encode_hash with the 8 level features of lane half h already computed (hash_feature_kernel): F[i] = level 8h + i
// PADQ: slot 31 of lane half 0 (canonical feature 62, the first constant-one column) carries pad_ (Q.x3)
template <bool PADQ = false>
__device__ __forceinline__ void encode_hashf(const QLane& Q, const uint32_t (&F)[8], int h, h8 (&x)[4]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = F[i];
    // OneBlob as encoder v3 (clamped wrap, one path): the reference's raw-angle inputs send every Cornell wave down
    // blob_many's wrap branch (~25 VALU more per input)
    blob_v3(Q.b0, w[8], w[9]);
    blob_v3(Q.b1, w[10], w[11]);
    blob_v3(Q.b2, w[12], w[13]);
    w[14] = pk2(Q.i0, Q.i1);
    w[15] = pk2(Q.i2, PADQ && h == 0 ? Q.x3 : 1.0f);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        u4 t4 = {w[4 * kk], w[4 * kk + 1], w[4 * kk + 2], w[4 * kk + 3]};
        x[kk] = __builtin_bit_cast(h8, t4);
    }
}

// HashGrid features of a chunk of queries, one level per block with the level's table in LDS (round 3). The gather
// kernel above reads 128 random 4-byte table entries per query from L1/L2 -- one cache line each, the L1 line rate
// bounds it -- while one level's table (32,768 entries x 4 B = 128 KiB, level 0: 16 KiB) fits a CU's LDS, where a
// random 4-byte read costs a bank access instead of a line. Block b: level (b / 8) % 16, query range sub = b % 8 +
// 8 * (b / 128) of P: the 16 level blocks of a range are dispatched to the same XCD (round-robin b % 8), so they share
// its L2 for the positions. feat[level * kHashFeatStride + s] = the same half2 as hash_level_feature (same corners,
// same interpolation), for s in [0, n).
// hash_corners for one level whose table sits alone in LDS: the corners' LDS byte offsets instead of global entries.
// (index & mask) * 4 == (4 index) & (4 mask) for the hashed x ^ y P1 ^ z P2 and the dense x + y res + z res^2 alike
// (uint32 wrap-around), so the cell coordinates and multipliers carry the factor 4 and one v_bitop3 per corner
// ((x ^ yz) & mask) gives the offset; positions, fractions and weights are hash_corners' float operations.
struct LdsCorners {
    uint32_t off[8];
    float w[8];
};
// round-3 form (scalar f32 products; A/B: hash_feature_kernel ablation bit 8)
template <bool DENSE>
__device__ __forceinline__ void hash_corners_lds_r3(float px, float py, float pz, int l, LdsCorners& C) {
    const float scale = (float)(16 << l) - 1.0f;
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
    const uint32_t mask4 = (l == 0 ? 4095u : 32767u) << 2;
    const uint32_t ym = 4u * (DENSE ? res : NRC_HASH_PRIME1), zm = 4u * (DENSE ? res * res : NRC_HASH_PRIME2);
    const uint32_t X[2] = {4u * cell[0], 4u * cell[0] + 4u};
    const uint32_t Y[2] = {cell[1] * ym, cell[1] * ym + ym};
    const uint32_t Z[2] = {cell[2] * zm, cell[2] * zm + zm};
    const float wx[2] = {1.0f - fr[0], fr[0]}, wy[2] = {1.0f - fr[1], fr[1]}, wz[2] = {1.0f - fr[2], fr[2]};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const int bx = c & 1, by = (c >> 1) & 1, bz = c >> 2;
        const uint32_t i = DENSE ? X[bx] + (Y[by] + Z[bz]) : X[bx] ^ (Y[by] ^ Z[bz]);
        C.off[c] = i & mask4;
        C.w[c] = (wx[bx] * wy[by]) * wz[bz];
    }
}

template <bool DENSE>
__device__ __forceinline__ void hash_corners_lds(float px, float py, float pz, int l, LdsCorners& C) {
    const float scale = (float)(16 << l) - 1.0f;
    const uint32_t res = 16u << l;
    // round 4: the per-dimension and per-corner f32 products as packed pairs (v_pk_fma_f32 / v_pk_add_f32 /
    // v_pk_mul_f32: two IEEE operations per instruction, the same roundings), since the feature pass is VALU-bound
    const f2 p01 = __builtin_elementwise_fma(f2{scale, scale}, f2{px, py}, f2{0.5f, 0.5f});
    const float pos[3] = {p01[0], p01[1], __builtin_fmaf(scale, pz, 0.5f)};
    float fr[3];
    uint32_t cell[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const float fl = floorf(pos[d]);
        cell[d] = (uint32_t)(int)fl;
        fr[d] = pos[d] - fl;
    }
    const uint32_t mask4 = (l == 0 ? 4095u : 32767u) << 2;
    const uint32_t ym = 4u * (DENSE ? res : NRC_HASH_PRIME1), zm = 4u * (DENSE ? res * res : NRC_HASH_PRIME2);
    const uint32_t X[2] = {4u * cell[0], 4u * cell[0] + 4u};
    const uint32_t Y[2] = {cell[1] * ym, cell[1] * ym + ym};
    const uint32_t Z[2] = {cell[2] * zm, cell[2] * zm + zm};
    const f2 om01 = f2{1.0f, 1.0f} - f2{fr[0], fr[1]};  // 1 - fr for x, y
    const f2 wx = {om01[0], fr[0]};                       // (wx0, wx1)
    const float wy[2] = {om01[1], fr[1]}, wz[2] = {1.0f - fr[2], fr[2]};
    // (wx[bx] * wy[by]) * wz[bz] for bx = 0, 1 in one packed multiply each
    f2 wxy[2], w[4];
#pragma unroll
    for (int by = 0; by < 2; ++by) wxy[by] = wx * f2{wy[by], wy[by]};
#pragma unroll
    for (int bz = 0; bz < 2; ++bz)
#pragma unroll
        for (int by = 0; by < 2; ++by) w[bz * 2 + by] = wxy[by] * f2{wz[bz], wz[bz]};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const int bx = c & 1, by = (c >> 1) & 1, bz = c >> 2;
        const uint32_t i = DENSE ? X[bx] + (Y[by] + Z[bz]) : X[bx] ^ (Y[by] ^ Z[bz]);
        C.off[c] = i & mask4;
        C.w[c] = w[bz * 2 + by][bx];
    }
}

// hash_interp with the corner weights converted two at a time (corners 2k, 2k + 1 in one v_cvt_pk_f16_f32) and each
// half broadcast into the packed FMA (op_sel): the same f16 roundings and FMA order, half the conversions
__device__ __forceinline__ uint32_t hash_interp_pk(const float (&w)[8], const uint32_t (&v)[8]) {
    h2v acc = {(_Float16)0.0f, (_Float16)0.0f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t w2 = pk2(w[2 * k], w[2 * k + 1]);
        asm volatile("" : "+v"(w2));  // (half)w rounded before the FMA (no v_fma_mix folding)
        const h2v wp = __builtin_bit_cast(h2v, w2);
        acc = __builtin_elementwise_fma(h2v{wp[0], wp[0]}, __builtin_bit_cast(h2v, v[2 * k]), acc);
        acc = __builtin_elementwise_fma(h2v{wp[1], wp[1]}, __builtin_bit_cast(h2v, v[2 * k + 1]), acc);
    }
    return __builtin_bit_cast(uint32_t, acc);
}

template <int ABL = 0>  // ablations (timing only, knob hash_feat_abl): 1 no LDS gathers, 2 no position loads, 4 no stores,
                        // 128 positions 5 steps ahead (same results);
                        // 8 the round-3 scalar arithmetic, 16 the round-3 unpipelined loop (same results), 32 hashed
                        // synthetic positions instead of the position loads
__global__ __launch_bounds__(1024, 1) void hash_feature_kernel(const float* __restrict__ q, int64_t n, int P,
                                                               const uint32_t* __restrict__ table,
                                                               uint32_t* __restrict__ feat) {
    __shared__ __attribute__((aligned(16))) uint32_t lt[NRC_HASH_T];
    const int b = blockIdx.x;
    const int level = (b >> 3) & 15, sub = (b & 7) + 8 * (b >> 7);
    if (sub >= P) return;
    const uint32_t entries = level == 0 ? 4096u : (uint32_t)NRC_HASH_T;
    const uint32_t off = level == 0 ? 0u : 4096u + (uint32_t)(level - 1) * (uint32_t)NRC_HASH_T;
    {
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const u4* src = reinterpret_cast<const u4*>(table + off);
        for (int c = wave; c < (int)(entries / 256u); c += 16)
            __builtin_amdgcn_global_load_lds((const void*)(src + c * 64 + lane),
                                             (__attribute__((address_space(3))) void*)(lt + c * 256), 16, 0, 0);
    }
    const int64_t s0 = (int64_t)sub * n / P, s1 = (int64_t)(sub + 1) * n / P;
    const int cnt = (int)(s1 - s0);  // <= kHashFeatStride: 32-bit byte offsets below
    // raw buffer descriptors over this block's range: position loads past it return 0, feature stores past it are
    // dropped, so the loop has no branch around a memory op (a conditional store made the compiler wait vmcnt(0),
    // i.e. for the store's acknowledgement, before the next iteration's prefetched position). All memory operations
    // stay compiler-visible: an inline-asm load that the compiler cannot see in flight lets it reuse the destination
    // registers before the data lands.
    constexpr int kQD = (ABL & 64) != 0 ? NRC_INPUT_DIMS_PADDED : NRC_INPUT_DIMS;  // ABL 64: padded RadianceQuery
    const __amdgpu_buffer_rsrc_t rq = buffer_rsrc(q + s0 * kQD, cnt * (kQD * 4));
    const __amdgpu_buffer_rsrc_t rf = buffer_rsrc(feat + (int64_t)level * kHashFeatStride + s0, cnt * 4);
    typedef float f3 __attribute__((ext_vector_type(3)));
    auto load_pos = [&](int k) -> f3 {
        if constexpr ((ABL & 2) != 0) {
            const float u = (float)(k & 1023) * (1.0f / 1024.0f);
            return f3{u, 1.0f - u, u * u};
        }
        if constexpr ((ABL & 32) != 0) {  // no position loads, but scattered positions (the gathers keep their conflicts)
            uint32_t hsh = (uint32_t)k * 0x9E3779B1u + (uint32_t)level;
            float c[3];
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                hsh ^= hsh >> 15;
                hsh *= 0x2C1B3C6Du;
                hsh ^= hsh >> 12;
                c[d] = (float)(hsh >> 8) * (1.0f / 16777216.0f);
            }
            return f3{c[0], c[1], c[2]};
        }
        return __builtin_bit_cast(f3, __builtin_amdgcn_raw_buffer_load_b96(rq, k * (kQD * 4), 0, 0));
    };
    // two queries per lane per step (i, i + 1024), their positions two steps ahead in two register sets used
    // alternately
    int i = threadIdx.x;
    f3 PB[2][2] = {{load_pos(i), load_pos(i + 1024)}, {load_pos(i + 2048), load_pos(i + 3072)}};
    // the table DMA is counted on vmcnt, and a workgroup barrier does not wait for it: every wave's copy must have
    // landed before any wave reads the table (the other LDS-copy sites wait the same way)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const char* const ltb = reinterpret_cast<const char*>(lt);
    auto corners = [&](const f3& p, LdsCorners& C, auto dense_c) {
        constexpr bool kDense = decltype(dense_c)::value;
        if constexpr ((ABL & 8) != 0) hash_corners_lds_r3<kDense>(p.x, p.y, p.z, level, C);
        else hash_corners_lds<kDense>(p.x, p.y, p.z, level, C);
    };
    auto gather = [&](const LdsCorners& C, uint32_t (&v)[8]) {
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = (ABL & 1) ? C.off[c] : *reinterpret_cast<const uint32_t*>(ltb + C.off[c]);
    };
    auto interp = [&](const LdsCorners& C, const uint32_t (&v)[8]) -> uint32_t {
        if constexpr ((ABL & 8) != 0) {
            HashCorners W;
#pragma unroll
            for (int c = 0; c < 8; ++c) W.w[c] = C.w[c];
            return hash_interp(W, v);
        } else {
            return hash_interp_pk(C.w, v);
        }
    };
    // Round 4 (default): software-pipelined steps. PMC of the round-3 loop: LDS 47 % and VALU 43 % busy, waves waiting
    // on their own dependencies 62 % of their cycles -- each step ran hash -> 16 gathers -> wait -> interpolate in
    // series. Here a step is one query per lane, and step s + 1's corners are computed and its 8 gathers issued before
    // step s's 8 are consumed: 16 gathers in flight per wave (the wait for the older 8 is lgkmcnt(8): gfx950's LDS
    // counter field holds at most 15, so a 2-query step's 16 + 16 could not be waited for exactly) and the hashing
    // overlaps the LDS latency. Same arithmetic per query.
    auto body_pipe = [&](auto dense_c) {
        f3 PP[2] = {PB[0][0], PB[0][1]};  // positions of steps 0, 1 (queries i, i + 1024), loaded above
        LdsCorners C[2];
        uint32_t v[2][8];
        corners(PP[0], C[0], dense_c);
        PP[0] = load_pos(i + 2048);  // step 2
        gather(C[0], v[0]);
        // step 0's gathers land before the loop (a compiler-visible s_waitcnt lgkmcnt(0), vmcnt/expcnt untouched): the
        // waitcnt pass merges the loop entry with the back edge, and gathers still in flight on the entry edge (into
        // other registers than the back edge's) made it wait lgkmcnt(0) at the top of every other phase
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        // phase cur: step s (set cur, gathers in flight) -> prepare step s + 1 in set nxt, then finish step s
        auto phase = [&](auto cur_c) -> bool {
            constexpr int cur = decltype(cur_c)::value, nxt = 1 - cur;
            if (i - (int)threadIdx.x >= cnt) return false;  // block-uniform
            // step s + 1 (positions past the range read 0: valid LDS offsets, results never stored)
            corners(PP[nxt], C[nxt], dense_c);
            PP[nxt] = load_pos(i + 3072);  // step s + 3
            gather(C[nxt], v[nxt]);
            __builtin_amdgcn_raw_buffer_store_b32(interp(C[cur], v[cur]), rf, (ABL & 4) ? kBufferOff : i * 4, 0, 0);
            i += 1024;
            return true;
        };
        while (phase(std::integral_constant<int, 0>{}) && phase(std::integral_constant<int, 1>{})) {
        }
    };
    // ABL & 128 (round 6, A/B): the positions 5 steps ahead instead of 3 (a ring of 4 position sets): step s prepares step
    // s + 1 from set (s + 1) % 4 and reloads that set with step s + 5's positions
    auto body_deep = [&](auto dense_c) {
        f3 PP[4] = {PB[0][0], PB[0][1], PB[1][0], PB[1][1]};  // steps 0..3
        LdsCorners C[2];
        uint32_t v[2][8];
        corners(PP[0], C[0], dense_c);
        PP[0] = load_pos(i + 4096);  // step 4
        gather(C[0], v[0]);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        auto phase = [&](auto cur_c, auto slot_c) -> bool {
            constexpr int cur = decltype(cur_c)::value, nxt = 1 - cur, slot = decltype(slot_c)::value;
            if (i - (int)threadIdx.x >= cnt) return false;  // block-uniform
            corners(PP[slot], C[nxt], dense_c);
            PP[slot] = load_pos(i + 5120);  // step s + 5
            gather(C[nxt], v[nxt]);
            __builtin_amdgcn_raw_buffer_store_b32(interp(C[cur], v[cur]), rf, (ABL & 4) ? kBufferOff : i * 4, 0, 0);
            i += 1024;
            return true;
        };
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        using I3 = std::integral_constant<int, 3>;
        while (phase(I0{}, I1{}) && phase(I1{}, I2{}) && phase(I0{}, I3{}) && phase(I1{}, I0{})) {
        }
    };
    if constexpr ((ABL & 128) != 0) {
        if (level <= 1) body_deep(std::integral_constant<bool, true>{});
        else body_deep(std::integral_constant<bool, false>{});
        return;
    }
    if constexpr ((ABL & 16) == 0) {
        if (level <= 1) body_pipe(std::integral_constant<bool, true>{});
        else body_pipe(std::integral_constant<bool, false>{});
        return;
    }
    // ABL & 16: the round-3 loop (A/B)
    auto body = [&](auto dense_c) {
        constexpr bool kDense = decltype(dense_c)::value;
        auto step = [&](auto cur_c) -> bool {
            constexpr int cur = decltype(cur_c)::value;
            if (i - (int)threadIdx.x >= cnt) return false;  // block-uniform
            LdsCorners C[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                if constexpr ((ABL & 8) != 0) hash_corners_lds_r3<kDense>(PB[cur][u].x, PB[cur][u].y, PB[cur][u].z, level, C[u]);
                else hash_corners_lds<kDense>(PB[cur][u].x, PB[cur][u].y, PB[cur][u].z, level, C[u]);
            }
            PB[cur][0] = load_pos(i + 4096);
            PB[cur][1] = load_pos(i + 5120);
            uint32_t v[2][8];
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int c = 0; c < 8; ++c)
                    v[u][c] = (ABL & 1) ? C[u].off[c] : *reinterpret_cast<const uint32_t*>(ltb + C[u].off[c]);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                uint32_t f;
                if constexpr ((ABL & 8) != 0) {
                    HashCorners W;
#pragma unroll
                    for (int c = 0; c < 8; ++c) W.w[c] = C[u].w[c];
                    f = hash_interp(W, v[u]);
                } else {
                    f = hash_interp_pk(C[u].w, v[u]);
                }
                __builtin_amdgcn_raw_buffer_store_b32(f, rf, (ABL & 4) ? kBufferOff : (i + 1024 * u) * 4, 0, 0);
            }
            i += 2048;
            return true;
        };
        while (step(std::integral_constant<int, 0>{}) && step(std::integral_constant<int, 1>{})) {
        }
    };
    if (level <= 1) body(std::integral_constant<bool, true>{});
    else body(std::integral_constant<bool, false>{});
}

// ------------------------------------------------------------------------------------------------
// FrequencySH extension (NRC_ENCODING_FREQUENCY_SH; oracle/nrc_oracle.c orc_encode_sh): TriangleWave as the
// Frequency composite, the direction's degree-4 real SH (tcnn SphericalHarmonics basis) with lane half h
// producing coefficients 8h..8h+7, OneBlob of dims 5+2h, 6+2h, Identity 9+3h.., 3 pad slots.
// ------------------------------------------------------------------------------------------------
template <bool CHAIN = false>
__device__ __forceinline__ void encode_sh(const QLane& Q, int h, h8 (&x)[5]) {
    uint32_t w[20];
    {
        h8 t[5];
        encode_fast<CHAIN>(Q, h, t);  // slots 0..17 (words 0..8) are the triangle wave; the rest is replaced
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            w[k] = __builtin_bit_cast(u4, t[k >> 2])[k & 3];
        }
    }
    const float st = sinf(Q.b0), ct = cosf(Q.b0), sp = sinf(Q.b1), cp = cosf(Q.b1);
    const float X = st * cp, Y = st * sp, Z = ct;
    const float xy = X * Y, xz = X * Z, yz = Y * Z, x2 = X * X, y2 = Y * Y, z2 = Z * Z;
    float o[8];
    if (h == 0) {
        o[0] = 0.28209479177387814f;
        o[1] = -0.48860251190291987f * Y;
        o[2] = 0.48860251190291987f * Z;
        o[3] = -0.48860251190291987f * X;
        o[4] = 1.0925484305920792f * xy;
        o[5] = -1.0925484305920792f * yz;
        o[6] = 0.94617469575755997f * z2 - 0.31539156525251999f;
        o[7] = -1.0925484305920792f * xz;
    } else {
        o[0] = 0.54627421529603959f * x2 - 0.54627421529603959f * y2;
        o[1] = 0.59004358992664352f * Y * (-3.0f * x2 + y2);
        o[2] = 2.8906114426405538f * xy * Z;
        o[3] = 0.45704579946446572f * Y * (1.0f - 5.0f * z2);
        o[4] = 0.3731763325901154f * Z * (5.0f * z2 - 3.0f);
        o[5] = 0.45704579946446572f * X * (1.0f - 5.0f * z2);
        o[6] = 1.4453057213202769f * Z * (x2 - y2);
        o[7] = 0.59004358992664352f * X * (-x2 + 3.0f * y2);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) w[9 + k] = pk2(o[2 * k], o[2 * k + 1]);
    {
        const float xb[2] = {Q.b2, Q.x3};
        uint32_t lo[2], hi[2];
        blob_many<2>(xb, lo, hi);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            w[13 + 2 * i] = lo[i];
            w[13 + 2 * i + 1] = hi[i];
        }
    }
    w[17] = pk2(Q.i0, Q.i1);
    w[18] = pk2(Q.i2, 1.0f);
    w[19] = 0x3C003C00u;
#pragma unroll
    for (int kk = 0; kk < 5; ++kk) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        u4 t4 = {w[4 * kk], w[4 * kk + 1], w[4 * kk + 2], w[4 * kk + 3]};
        x[kk] = __builtin_bit_cast(h8, t4);
    }
}

// s_memtime between scheduling fences (diagnostic builds only)
__device__ __forceinline__ uint64_t stamp_now() {
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t t = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
constexpr int kInferPhases = 8;  // encode+prefetch, layers 0..4, output layer, epilogue

template <int ABL = 0>
__device__ __forceinline__ h8 relu_h8(const f16v& a, int base) {
    h8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (_Float16)a[base + j];
    if (ABL & 2) return r;
    const h8 z = {};
    return __builtin_elementwise_max(r, z);
}

// Hide the LDS weight base from loop-invariant code motion so fragments are re-read per layer
// instead of being hoisted into ~184 registers (which pins the kernel at one wave per SIMD).
typedef __attribute__((address_space(3))) const h8 lds_h8;
__device__ __forceinline__ lds_h8* launder(lds_h8* p) {
    asm volatile("" : "+v"(p));
    return p;
}

template <int KK, int ABL = 0>
__device__ __forceinline__ void load_frags(lds_h8* lw_lane, int layer, h8 (&a)[2][KK]) {
    if (ABL & 4) {
        h8 v = {};
        v[0] = (_Float16)(float)layer;
        asm volatile("" : "+v"(v));
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) a[0][kk] = a[1][kk] = v;
        return;
    }
    lds_h8* wl = launder(lw_lane);
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
        a[0][kk] = wl[fwd_frag(layer, 0, kk) * 64];
        a[1][kk] = wl[fwd_frag(layer, 1, kk) * 64];
    }
}

template <int TILES, int KK, int ABL = 0>
__device__ __forceinline__ void layer_mfma(const h8 (&a)[2][KK], const h8 (&in)[TILES][KK], h8 (&y)[TILES][4]) {
    f16v c[TILES][2];
#pragma unroll
    for (int t = 0; t < TILES; ++t) c[t][0] = c[t][1] = zero16();
    if constexpr ((ABL & 262144) != 0) {
        // tile-major order (round 4, 2-tile A/B): tile 0's MFMAs of the layer, then tile 1's, so that tile 0's ReLU/pack
        // VALU can issue beside tile 1's MFMAs and tile 1's beside tile 0's next layer
#pragma unroll
        for (int t = 0; t < TILES; ++t)
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) {
                c[t][0] = mfma(a[0][kk], in[t][kk], c[t][0]);
                c[t][1] = mfma(a[1][kk], in[t][kk], c[t][1]);
            }
    } else if constexpr ((ABL & 131072) != 0) {
        // A-major order (round 4, energy A/B): consecutive MFMAs share the A operand (weight fragment) across tiles
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int t = 0; t < TILES; ++t) c[t][m] = mfma(a[m][kk], in[t][kk], c[t][m]);
    } else {
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
#pragma unroll
            for (int t = 0; t < TILES; ++t) {
                c[t][0] = mfma(a[0][kk], in[t][kk], c[t][0]);
                c[t][1] = mfma(a[1][kk], in[t][kk], c[t][1]);
            }
    }
#pragma unroll
    for (int t = 0; t < TILES; ++t) {
        y[t][0] = relu_h8<ABL>(c[t][0], 0);
        y[t][1] = relu_h8<ABL>(c[t][0], 8);
        y[t][2] = relu_h8<ABL>(c[t][1], 0);
        y[t][3] = relu_h8<ABL>(c[t][1], 8);
    }
}

// PREFETCH: issue layer l+1's weight-fragment reads before layer l's MFMAs (double-buffered
// fragment registers) instead of at the head of layer l+1.
template <int TILES, bool PREFETCH, int ABL = 0, int KK0 = 5>
__device__ __forceinline__ void mlp_tiles(lds_h8* lw_lane, const h8 (&x)[TILES][KK0], f16v (&o)[TILES],
                                          uint64_t* ph = nullptr, uint64_t* tprev = nullptr) {
    auto mark = [&](int k) {  // ABL & 256: add the time since the previous mark to phase k
        if constexpr ((ABL & 256) != 0) {
            const uint64_t t = stamp_now();
            ph[k] += t - *tprev;
            *tprev = t;
        }
    };
    static_assert(KK0 == 5 || !PREFETCH, "the prefetch schedule is written for the 80-wide input layer");
    h8 y[TILES][4], z[TILES][4];
    if constexpr (PREFETCH) {
        h8 a0[2][5];
        load_frags<5>(lw_lane, 0, a0);
        h8 aA[2][4], aB[2][4];
        load_frags<4>(lw_lane, 1, aA);
        layer_mfma<TILES, 5>(a0, x, y);
        load_frags<4>(lw_lane, 2, aB);
        layer_mfma<TILES, 4>(aA, y, z);
        load_frags<4>(lw_lane, 3, aA);
        layer_mfma<TILES, 4>(aB, z, y);
        load_frags<4>(lw_lane, 4, aB);
        layer_mfma<TILES, 4>(aA, y, z);
        lds_h8* wl = launder(lw_lane);
        h8 a5[4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) a5[kk] = wl[fwd_frag(5, 0, kk) * 64];
        layer_mfma<TILES, 4>(aB, z, y);
#pragma unroll
        for (int t = 0; t < TILES; ++t) o[t] = zero16();
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int t = 0; t < TILES; ++t) o[t] = mfma(a5[kk], y[t][kk], o[t]);
    } else {
        {
            h8 a0[2][KK0];
            load_frags<KK0, ABL & 7>(lw_lane, 0, a0);
            layer_mfma<TILES, KK0, ABL & (7 | 131072 | 262144)>(a0, x, y);
        }
        mark(1);
#pragma unroll
        for (int l = 1; l < 5; ++l) {
            h8 a[2][4];
            load_frags<4, ABL & 7>(lw_lane, l, a);
            layer_mfma<TILES, 4, ABL & (7 | 131072 | 262144)>(a, y, z);
#pragma unroll
            for (int t = 0; t < TILES; ++t)
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) y[t][kk] = z[t][kk];
            mark(1 + l);
        }
        if constexpr ((ABL & 65536) != 0) {
            // Output layer on v_mfma_f32_4x4x4_16b_f16 (16 independent 4x4x4 blocks): block b = lane / 4 takes the
            // samples of lanes 4b..4b+3 and the hidden half (lane / 32) those lanes hold, so the h8 activations feed
            // the B operand as they are; the A operand of lane l is output row l % 4 of that half's weights, i.e. the
            // 32x32x16 fragment of lane (l & 3) | (l & 32). 8 of these (4 rows, 3 used) replace 4 32x32x16 (32 rows);
            // o[t][0..3] = rows 0..3 of sample lane % 32 summed over hidden half lane / 32 (the epilogue adds halves).
            const int ln = threadIdx.x & 63;
            lds_h8* w4 = launder(lw_lane + (((ln & 3) | (ln & 32)) - ln));
            f4v c4[TILES];
#pragma unroll
            for (int t = 0; t < TILES; ++t) c4[t] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const h8 a = w4[fwd_frag(5, 0, kk) * 64];
#pragma unroll
                for (int t = 0; t < TILES; ++t) {
                    c4[t] = __builtin_amdgcn_mfma_f32_4x4x4f16(__builtin_shufflevector(a, a, 0, 1, 2, 3),
                                                                __builtin_shufflevector(y[t][kk], y[t][kk], 0, 1, 2, 3),
                                                                c4[t], 0, 0, 0);
                    c4[t] = __builtin_amdgcn_mfma_f32_4x4x4f16(__builtin_shufflevector(a, a, 4, 5, 6, 7),
                                                                __builtin_shufflevector(y[t][kk], y[t][kk], 4, 5, 6, 7),
                                                                c4[t], 0, 0, 0);
                }
            }
#pragma unroll
            for (int t = 0; t < TILES; ++t) {
                o[t] = zero16();
#pragma unroll
                for (int i = 0; i < 4; ++i) o[t][i] = c4[t][i];
            }
        } else {
            lds_h8* wl = launder(lw_lane);
#pragma unroll
            for (int t = 0; t < TILES; ++t) o[t] = zero16();
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const h8 a = wl[fwd_frag(5, 0, kk) * 64];
#pragma unroll
                for (int t = 0; t < TILES; ++t) o[t] = mfma(a, y[t][kk], o[t]);
            }
        }
        if constexpr ((ABL & 256) != 0) {
            // make the output MFMAs complete inside their own phase
#pragma unroll
            for (int t = 0; t < TILES; ++t) asm volatile("" : "+v"(o[t]));
        }
        mark(6);
    }
}

// Options of the production kernels: 16 = omod doubling-chain triangle wave (variant 22), 32 = branch-free
// prefetch and buffer load/store epilogue (variant 23).
constexpr int kDefaultAbl = 48;
constexpr int kAblPadQ = 1 << 20;  // padded RadianceQuery records (nrc_config.query_layout = NRC_QUERY_PADDED)
// Round 6 (with the per-block LDS queue, ABL & 2048): a wave's first tile is block range start + its wave index, not a
// queue draw, so its query loads issue before the weight copy and their latency overlaps the copy's (the queue counter
// starts past the first tiles). The same tiles, so the same rows: outputs are unchanged.
constexpr int kAblEarlyQ = 1 << 21;

// Optional epilogue: accumulate_render_radiance (nrc_helpers.cu:77-129) fused into inference for the render
// queries [0, n_acc) (EPI = RenderMode Full 0 / CacheOnly 2); their radiance is consumed in registers and never
// written. Queries [n_acc, n) (the train-suffix ends) are written to out as usual. Same float operations as
// accumulate_kernel (nrc_frame.hip), so the frame buffer is bit-identical to the unfused path.
struct InferEpilogue {
    const float* thr;  // [n_acc] float3 lastRenderThroughput
    float4* rgba;      // [n_acc] frame buffer
    int64_t n_acc;
    float w;           // 1 / (iterationIndex + 1)
    uint64_t* stamps = nullptr;  // diagnostic build only (ABL & 256): per-wave phase cycle sums
    uint32_t* wq = nullptr;      // ABL & 16384: the handle's work-pool counters (kPoolSets sets of kPools)
    int parity = 0;              // ABL & 16384: this launch's counter set; it zeroes the other one for the next launch
};
// ABL & 16384: the launch's tiles split into kPools contiguous pools, each a device-scope atomic counter; a block starts
// on pool blockIdx % kPools and, once that pool is dry, steals from the others (a per-block LDS mask of the pools seen
// dry keeps the walk short). Counters are 128 B apart; two sets alternate between launches on the stream.
constexpr int kPools = 32, kPoolStride = 32, kPoolSetWords = kPools * kPoolStride;


// ENC: 0 = Frequency composite (80-wide input), 1 = Hash composite (64-wide; grid = f16x2 table),
// 2 = FrequencySH extension (80-wide)
template <int TILES, int THREADS, bool PREFETCH, int ABL, int EPI, int ENC = 0>
__device__ __forceinline__ void infer_v2_body(const float* __restrict__ q, float* __restrict__ out, int64_t n,
                                              const h8* __restrict__ wf, const InferEpilogue& epi,
                                              const uint32_t* __restrict__ grid = nullptr) {
    constexpr int KK0 = ENC == 1 || ENC == 3 ? 4 : 5;  // ENC 3: Hash from hash_feature_kernel's features (grid = feat)
    [[maybe_unused]] uint64_t rstart = 0;
    if constexpr ((ABL & 512) != 0) rstart = __builtin_amdgcn_s_memrealtime();
    __shared__ __attribute__((aligned(16))) h8 lw[kFwdFrags * 64];
    // ABL & 8: per-wave staging of a tile's 32 x 12-B results so they leave as 24 contiguous 16-B stores
    __shared__ __attribute__((aligned(16))) float ostage[(ABL & 8) ? THREADS / 64 : 1][96];
    // ABL & 2048: a per-block work queue in LDS. With a fixed share of tiles per wave, the waves that share a SIMD do
    // not progress at the same rate (the oldest wave issues first): at 2^21 queries the first waves finished their 16
    // tiles at 36 us and the last at 82 us, the SIMDs running the tail at 1-2 waves. The block takes a contiguous
    // range of tiles and its waves draw the next tile from an LDS counter, so every SIMD stays loaded to the end.
    __shared__ uint32_t wq_next;
    __shared__ uint32_t pool_dry;
    if constexpr ((ABL & 16) != 0) fp32_flush_output_denorms();
    if constexpr ((ABL & 2048) != 0) {
        if (threadIdx.x == 0) wq_next = 0;
    }
    if constexpr ((ABL & 16384) != 0) {
        if (threadIdx.x == 0) pool_dry = 0;
        // block 0 zeroes the other counter set: the launch before this one (same stream) used it and has completed
        if (blockIdx.x == 0 && threadIdx.x < kPools)
            epi.wq[(1 - epi.parity) * kPoolSetWords + threadIdx.x * kPoolStride] = 0u;
    }
    // ABL & 32768: the block's tile range as with the LDS queue (2048), but its counter in global memory (one per block,
    // 64 B apart, two sets alternating by launch parity), so that waves whose block has drained its range steal tiles
    // from other blocks' ranges. Every tile of a range is taken by exactly one atomic add on that range's counter and
    // every block drains its own counter, so stealing only moves work; each launch zeroes the other set for the next.
    [[maybe_unused]] uint32_t* const scnt = epi.wq + (ABL & 32768 ? 2 * kPoolSetWords + epi.parity * kStealSetWords : 0);
    if constexpr ((ABL & 32768) != 0) {
        uint32_t* const other = epi.wq + 2 * kPoolSetWords + (1 - epi.parity) * kStealSetWords;
        for (int b = blockIdx.x + gridDim.x * (int)threadIdx.x; b < kStealMaxBlocks; b += gridDim.x * THREADS)
            __hip_atomic_store(other + b * kStealStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    constexpr bool kEarly = (ABL & kAblEarlyQ) != 0;
    static_assert(!kEarly || ((ABL & 2048) != 0 && (ABL & (4096 | 16384 | 32768)) == 0 && (ABL & 8192) != 0 && TILES == 1),
                  "early first-tile loads: the per-block LDS queue with buffer-loaded queries");
    if constexpr (kEarly) {
        if (threadIdx.x == 0) wq_next = THREADS / 64;  // the first tiles are taken by wave index (below)
    }
    // kEarly: the first tile's loads, issued before the weight copy (declared here, used by the loop below)
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5, r = lane & 31;
    const int64_t ngroups_all = (((n + 31) >> 5) + TILES - 1) / TILES;
    constexpr bool kBufQ = (ABL & 8192) != 0 && (ENC == 0 || ENC == 3) && TILES == 1;
    constexpr bool kPadQ = (ABL & kAblPadQ) != 0;
    static_assert(!kPadQ || kBufQ, "padded queries: the buffer-load prefetch path");
    const QOffsets vo = q_offsets<kPadQ>(r, h);
    [[maybe_unused]] uint32_t F[8];
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t rfeat =
        buffer_rsrc(grid, ENC == 3 ? (int)(NRC_HASH_LEVELS * kHashFeatStride * 4) : 0);
    auto load_f = [&](int64_t tile) {
        if constexpr (ENC == 3) {
            const int vo = (8 * h * (int)kHashFeatStride + (int)tile * 32 + r) * 4;
#pragma unroll
            for (int i = 0; i < 8; ++i)
                F[i] = __builtin_amdgcn_raw_buffer_load_b32(rfeat, vo, i * (int)kHashFeatStride * 4, 0);
        }
    };
    QLane Q[TILES];
    [[maybe_unused]] int64_t g_early = 0;
    if constexpr (kEarly) {
        // a tile past the launch reads zeros (empty buffer descriptor) and is never used
        g_early = (int64_t)blockIdx.x * ngroups_all / gridDim.x + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        load_f(g_early);
        Q[0] = load_q_tile<kPadQ>(q, n, g_early, vo);
    }
    copy_to_lds<THREADS, kFwdFrags * 64>(lw, wf);
    __syncthreads();

    const bool out16 = (reinterpret_cast<uintptr_t>(out) & 15) == 0;
    int64_t ngroups = ngroups_all, wstride = (int64_t)gridDim.x * (THREADS / 64), gbase = 0;
    // wave-uniform tile index (readfirstlane: scalar address arithmetic, scalar buffer descriptors)
    int64_t g = (int64_t)blockIdx.x * (THREADS / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    auto draw = [&]() -> int64_t {  // next tile of this block's range (ABL & 2048) / of the launch (ABL & 4096)
        uint32_t t = 0;
        if constexpr ((ABL & 4096) != 0) {
            if (lane == 0) t = __hip_atomic_fetch_add(epi.wq, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0) t = atomicAdd(&wq_next, 1u);
        }
        return gbase + (int64_t)__builtin_amdgcn_readfirstlane(t);
    };
    // ABL & 4096: one queue for the whole launch (tiles balance across CUs and XCDs too). Every wave draws until its
    // draw fails, then counts itself finished; the last wave to finish (all draws of the launch are done by then)
    // zeroes both counters, so the next launch on the stream starts from an empty queue.
    auto finish = [&]() {
        if constexpr ((ABL & 4096) != 0) {
            if (lane == 0) {
                const uint32_t total = gridDim.x * (THREADS / 64);
                if (__hip_atomic_fetch_add(epi.wq + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == total - 1) {
                    __hip_atomic_store(epi.wq, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(epi.wq + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
    };
    if constexpr ((ABL & 2048) != 0 && (ABL & 4096) == 0) {
        gbase = (int64_t)blockIdx.x * ngroups_all / gridDim.x;
        ngroups = (int64_t)(blockIdx.x + 1) * ngroups_all / gridDim.x;  // end of this block's range
        if constexpr (kEarly) g = g_early;
        else g = draw();
    }
    // steal state (ABL & 32768): the range the wave draws from (own block first)
    [[maybe_unused]] int scur = blockIdx.x;
    __shared__ uint32_t steal_dry;  // some wave of this block found every range drained
    if constexpr ((ABL & 32768) != 0) {
        if (threadIdx.x == 0) steal_dry = 0;
        __syncthreads();
    }
    auto rbeg = [&](int v) -> int64_t { return (int64_t)v * ngroups_all / gridDim.x; };
    auto sissue = [&]() -> uint32_t {
        uint32_t t = 0;
        if (lane == 0) t = __hip_atomic_fetch_add(scnt + scur * kStealStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return t;
    };
    // the tile of a draw from range scur that returned t; a drained range sends the wave looking for a range with tiles
    // left: every other block's counter read at once (lane i: candidates i, i + 64, ..., sc1 loads; the blocks of this
    // block's XCD first under round-robin placement), atomic claims on those that showed tiles left, in order;
    // ngroups_all = nothing left
    auto sresolve = [&](uint32_t t) -> int64_t {
        int64_t idx = rbeg(scur) + (int64_t)t;
        if (idx < rbeg(scur + 1)) return idx;
        if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&steal_dry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)))
            return ngroups_all;
        const int G = gridDim.x;
        constexpr int kProbe = kStealMaxBlocks / 64;
        int vs[kProbe];
        uint32_t cs[kProbe];
#pragma unroll
        for (int k = 0; k < kProbe; ++k) {
            const int i = 1 + lane + 64 * k;
            vs[k] = i < G ? (int)(((int64_t)blockIdx.x + 8 * (int64_t)i + (8 * (int64_t)i) / G) % G) : -1;
            cs[k] = vs[k] >= 0 ? __hip_atomic_load(scnt + vs[k] * kStealStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : 0u;
        }
#pragma unroll
        for (int k = 0; k < kProbe; ++k) {
            uint64_t m = __ballot(vs[k] >= 0 && (int64_t)cs[k] < rbeg(vs[k] + 1) - rbeg(vs[k]));
            while (m) {
                const int src = __builtin_ctzll(m);
                m &= m - 1;
                const int cand = __builtin_amdgcn_readlane(vs[k], src);
                uint32_t tt = 0;
                if (lane == 0)
                    tt = __hip_atomic_fetch_add(scnt + cand * kStealStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                tt = __builtin_amdgcn_readfirstlane(tt);
                if (rbeg(cand) + (int64_t)tt < rbeg(cand + 1)) {
                    scur = cand;
                    return rbeg(cand) + tt;
                }
            }
        }
        if (lane == 0) __hip_atomic_store(&steal_dry, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return ngroups_all;
    };
    if constexpr ((ABL & 32768) != 0) {
        uint32_t traw = sissue(), tt;
        asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(tt) : "v"(traw));
        g = sresolve(tt);
        ngroups = ngroups_all;
    }
    if constexpr ((ABL & 4096) != 0) g = draw();
    // ABL & 16384: pooled draws (see kPools)
    [[maybe_unused]] int cur = blockIdx.x % kPools;
    [[maybe_unused]] uint32_t* const pools = epi.wq + epi.parity * kPoolSetWords;
    auto pool_begin = [&](int k) -> int64_t { return (int64_t)k * ngroups_all / kPools; };
    auto pool_issue = [&](int k) -> uint32_t {
        uint32_t t = 0;
        if (lane == 0) t = __hip_atomic_fetch_add(pools + k * kPoolStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return t;
    };
    // the tile of a draw from pool cur that returned t (wave-uniform); a dry pool sends the wave to the next pool not
    // yet seen dry by its block (blocking draws; only at pool transitions); ngroups_all = nothing left anywhere
    auto pool_resolve = [&](uint32_t t) -> int64_t {
        int64_t idx = pool_begin(cur) + (int64_t)t;
        if (idx < pool_begin(cur + 1)) return idx;
        for (;;) {
            if (lane == 0) atomicOr(&pool_dry, 1u << cur);
            uint32_t m = 0;
            if (lane == 0) m = __hip_atomic_load(&pool_dry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            m = __builtin_amdgcn_readfirstlane(m);
            if (m == 0xFFFFFFFFu) return ngroups_all;
            const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
            const uint32_t rot = (uint32_t)((cur + 1 + wv) % kPools);
            const uint32_t free_rot = ~((m >> rot) | (m << ((32u - rot) & 31u)));  // bit i: pool (rot + i) % 32 free
            cur = (int)((rot + (uint32_t)__builtin_ctz(free_rot)) % kPools);
            uint32_t traw = pool_issue(cur), tt;
            asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(tt) : "v"(traw));
            idx = pool_begin(cur) + (int64_t)tt;
            if (idx < pool_begin(cur + 1)) return idx;
        }
    };
    if constexpr ((ABL & 16384) != 0) {
        uint32_t traw = pool_issue(cur), tt;
        asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(tt) : "v"(traw));
        g = pool_resolve(tt);
    }
    if (g >= ngroups) {
        finish();
        return;
    }
    const int64_t last = n - 1;

    // ABL & 8192 (ENC 0 / 3, TILES 1): queries through raw buffer loads (load_q_tile); ABL kAblPadQ: padded
    // RadianceQuery records (nrc_config.query_layout), through load_q_tile only. ENC 3: the lane's 8 level features of
    // the tile's query (levels 8h .. 8h + 7), prefetched with the query, as raw buffer loads (load_f): one 32-bit lane
    // offset per tile and the level stride in the scalar offset (instead of 8 64-bit addresses); rows past the
    // workspace read 0, rows past n are never stored
    static_assert(ENC != 3 || TILES == 1, "ENC 3 prefetches one tile");
    if constexpr (kEarly) {
        // loaded before the weight copy
    } else if constexpr (kBufQ) {
        load_f(g);
        Q[0] = load_q_tile<kPadQ>(q, n, g, vo);
    } else {
        load_f(g);
#pragma unroll
        for (int t = 0; t < TILES; ++t) Q[t] = load_q_enc<ENC>(q, min((g * TILES + t) * 32 + r, last), h);
    }
    if constexpr ((ABL & 32) != 0) {
        // stores that the hardware drops (empty descriptors): the loop is then entered with the same "prefetch
        // loads, then the epilogue's stores" vmcnt pattern as the back-edge, so the waits inside stay exact
        if constexpr (EPI >= 0)
            __builtin_amdgcn_raw_buffer_store_b128(u4{0u, 0u, 0u, 0u}, buffer_rsrc(out, 0), 0, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b96(u3{0u, 0u, 0u}, buffer_rsrc(out, 0), 0, 0, 0);
    }
    if constexpr ((ABL & (64 | 128)) != 0) {
        // stagger the waves that share a SIMD (wave slot from HW_ID) so that their encoders do not run in lockstep:
        // ABL 64: slot & 3 quarter-tile steps, ABL 128: odd slots half a tile
        const uint32_t slot = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 4 /* hwreg(HW_REG_HW_ID, 0, 4) */);
        const uint32_t steps = (ABL & 64) ? (slot & 3u) : 2u * (slot & 1u);
        for (uint32_t i = 0; i < steps; ++i) __builtin_amdgcn_s_sleep(25);
    }
    uint64_t ph[kInferPhases] = {};
    uint64_t tprev = 0;
    if constexpr ((ABL & 256) != 0) tprev = stamp_now();
    [[maybe_unused]] uint64_t clk0 = 0, rclk0 = 0;
    if constexpr ((ABL & 512) != 0) {
        clk0 = __builtin_amdgcn_s_memtime();
        rclk0 = __builtin_amdgcn_s_memrealtime();
    }
    bool first_iter = true;
    // queue variants draw one tile ahead: the draw for the tile after next is issued before this iteration's
    // prefetch loads, so its (atomic) latency hides under a whole tile and the prefetch never waits for it
    int64_t ng = 0;
    uint32_t nn_raw = 0;  // the pending draw: lane 0's atomic result, read (readfirstlane) one iteration later
    if constexpr ((ABL & (2048 | 4096)) != 0 && (ABL & 32768) == 0) ng = draw();
    if constexpr ((ABL & 32768) != 0) {
        uint32_t traw = g < ngroups_all ? sissue() : 0u, tt;
        asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(tt) : "v"(traw));
        ng = g < ngroups_all ? sresolve(tt) : ngroups_all;
    }
    if constexpr ((ABL & 16384) != 0) {
        uint32_t traw = pool_issue(cur), tt;
        asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(tt) : "v"(traw));
        ng = pool_resolve(tt);
    }
    for (int64_t nn = 0; g < ngroups; g = ng, ng = nn) {
        if constexpr ((ABL & (2048 | 4096 | 16384 | 32768)) != 0) {
            if (!first_iter) {
                // an asm readfirstlane stays here; the builtin is hoisted to the atomic and the wave then waits for it
                uint32_t t;
                asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(t) : "v"(nn_raw));
                if constexpr ((ABL & 16384) != 0) ng = pool_resolve(t);
                else if constexpr ((ABL & 32768) != 0) ng = sresolve(t);
                else ng = gbase + (int64_t)t;
            }
        }
        if constexpr ((ABL & 256) != 0) {  // the previous iteration's epilogue (stores, loop overhead)
            const uint64_t tn = stamp_now();
            if (!first_iter) ph[7] += tn - tprev;
            tprev = tn;
            first_iter = false;
        }
        h8 x[TILES][KK0];
#pragma unroll
        for (int t = 0; t < TILES; ++t) {
            if constexpr (ENC == 1) {
                encode_hash(Q[t], h, grid, x[t]);
            } else if constexpr (ENC == 3) {
                encode_hashf<kPadQ>(Q[t], F, h, x[t]);
            } else if constexpr (ENC == 2) {
                encode_sh<(ABL & 16) != 0>(Q[t], h, x[t]);
            } else if constexpr ((ABL & 1) != 0) {
                typedef float f4 __attribute__((ext_vector_type(4)));
                const f4 a = {Q[t].p0, Q[t].p1, Q[t].b0, Q[t].b1}, b = {Q[t].b2, Q[t].i0, Q[t].i1, Q[t].i2};
#pragma unroll
                for (int kk = 0; kk < 5; ++kk) x[t][kk] = __builtin_bit_cast(h8, (kk & 1) ? a : b);
            } else if constexpr ((ABL & 1024) != 0) {
                encode_v3<kPadQ>(Q[t], h, x[t]);
                if constexpr ((ABL & 524288) != 0) {
                    // energy probe (timing only, wrong outputs): 12 of the 14 constant-one pad slots (34..39 of both
                    // halves) fed as zeros, i.e. what folding the pad weights into one bias slot per half would feed
                    x[t][4] = h8{x[t][4][0], x[t][4][1], (_Float16)0, (_Float16)0, (_Float16)0, (_Float16)0,
                                 (_Float16)0, (_Float16)0};
                }
            } else {
                encode_fast<(ABL & 16) != 0>(Q[t], h, x[t]);
            }
        }
        if constexpr ((ABL & 16384) != 0) {
            nn_raw = ng < ngroups_all ? pool_issue(cur) : 0u;  // wave-uniform condition: no draw once everything is dry
            first_iter = false;
        } else if constexpr ((ABL & 32768) != 0) {
            nn_raw = ng < ngroups_all ? sissue() : 0u;
            first_iter = false;
        } else if constexpr ((ABL & (2048 | 4096)) != 0) {
            if constexpr ((ABL & 4096) != 0) {
                // every lane issues the buffer atomic; the descriptor covers lane 0's counter only, the other lanes'
                // adds are dropped by the hardware (no branch around the atomic)
                nn_raw = (uint32_t)__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, buffer_rsrc(epi.wq, 4), lane ? kBufferOff : 0, 0, 0);
            } else {
                if (lane == 0) nn_raw = atomicAdd(&wq_next, 1u);
            }
            first_iter = false;
        } else {
            ng = g + wstride;
            nn = ng;
        }
        load_f(ng);  // ENC 3 (after the encoder has consumed F)
        if constexpr (kBufQ) {
            Q[0] = load_q_tile<kPadQ>(q, n, ng, vo);
        } else if constexpr ((ABL & 32) != 0) {
            // unconditional (clamped) prefetch: no branch around the loads, so the compiler's vmcnt bookkeeping
            // stays exact across the loop back-edge
#pragma unroll
            for (int t = 0; t < TILES; ++t) Q[t] = load_q_enc<ENC>(q, min((ng * TILES + t) * 32 + r, last), h);
        } else if (ng < ngroups) {
#pragma unroll
            for (int t = 0; t < TILES; ++t) Q[t] = load_q_enc<ENC>(q, min((ng * TILES + t) * 32 + r, last), h);
        }
        // epilogue operands are fetched before the MLP so their latency hides under the MFMAs
        float tr[TILES][3];
        float4 acc[TILES];
        if constexpr (EPI >= 0 && (ABL & 32) != 0) {
            // branch-free: buffer loads whose descriptors end at n_acc return 0 past it (and for the h = 1 lanes)
#pragma unroll
            for (int t = 0; t < TILES; ++t) {
                const int64_t s0 = (g * TILES + t) * 32;
                const int rows = tile_rows(epi.n_acc, s0);
                const u3 tv = __builtin_amdgcn_raw_buffer_load_b96(
                    buffer_rsrc(epi.thr + s0 * 3, rows * 12), h ? kBufferOff : r * 12, 0, 0);
                // whole-vector bit_cast: clang 22 (ROCm 7.2) miscompiles __builtin_bit_cast(float, tv[i]) on a
                // buffer-load result into tv[0] for every i
                typedef float f3 __attribute__((ext_vector_type(3)));
                const f3 tf = __builtin_bit_cast(f3, tv);
                tr[t][0] = tf.x;
                tr[t][1] = tf.y;
                tr[t][2] = tf.z;
                if constexpr (EPI == 0) {
                    const u4 av = __builtin_amdgcn_raw_buffer_load_b128(
                        buffer_rsrc(epi.rgba + s0, rows * 16), h ? kBufferOff : r * 16, 0, 0);
                    acc[t] = __builtin_bit_cast(float4, av);
                }
            }
        } else if constexpr (EPI >= 0) {
#pragma unroll
            for (int t = 0; t < TILES; ++t) {
                const int64_t s = (g * TILES + t) * 32 + r;
                if (h == 0 && s < epi.n_acc) {
                    const float* T = epi.thr + s * 3;
                    tr[t][0] = T[0];
                    tr[t][1] = T[1];
                    tr[t][2] = T[2];
                    if constexpr (EPI == 0) acc[t] = epi.rgba[s];
                }
            }
        }
        f16v o[TILES];
        if constexpr ((ABL & 256) != 0) {
#pragma unroll
            for (int t = 0; t < TILES; ++t)
#pragma unroll
                for (int kk = 0; kk < KK0; ++kk) asm volatile("" : "+v"(x[t][kk]));
            const uint64_t tn = stamp_now();
            ph[0] += tn - tprev;
            tprev = tn;
        }
        mlp_tiles<TILES, PREFETCH, ABL & (7 | 256 | 65536 | 131072 | 262144), KK0>((lds_h8*)(lw + lane), x, o, ph, &tprev);
        if constexpr ((ABL & 8) && EPI < 0) {
            const int64_t s0 = g * TILES * 32;
            if (out16 && s0 + TILES * 32 <= n) {
                float* st = ostage[threadIdx.x >> 6];
#pragma unroll
                for (int t = 0; t < TILES; ++t) {
                    if (h == 0) {
                        st[3 * r + 0] = (float)(_Float16)fmaxf(o[t][0], 0.0f);
                        st[3 * r + 1] = (float)(_Float16)fmaxf(o[t][1], 0.0f);
                        st[3 * r + 2] = (float)(_Float16)fmaxf(o[t][2], 0.0f);
                    }
                    __builtin_amdgcn_wave_barrier();  // LDS is in order within a wave; keep the compiler in order too
                    if (lane < 24)
                        reinterpret_cast<float4*>(out + (s0 + t * 32) * NRC_OUTPUT_DIMS)[lane] =
                            reinterpret_cast<const float4*>(st)[lane];
                    __builtin_amdgcn_wave_barrier();
                }
                continue;
            }
        }
        if constexpr ((ABL & 32) != 0) {
            // every lane issues its stores: raw buffer stores whose descriptors cover only this tile's valid rows
            // drop the tail, the h = 1 lanes and the rows that belong to the other destination in hardware, so
            // there is no branch around a store (a conditional store leaves the next iteration's vmcnt wait at
            // 0, i.e. waiting for the store's acknowledgement)
#pragma unroll
            for (int t = 0; t < TILES; ++t) {
                const int64_t s0 = (g * TILES + t) * 32, sq = s0 + r;
                float L0, L1, L2;
                if constexpr ((ABL & 65536) != 0) {
                    // halves of the 4x4x4 output layer: swapping lanes 32..63 of rows 0 / 2 with lanes 0..31 of rows
                    // 1 / 3 lines up both halves of a row in one lane pair; the sums are row 0 (lanes 0..31), row 1
                    // (lanes 32..63), row 2 (lanes 0..31) of sample lane % 32
                    // (a whole-vector bit_cast: clang 22 turns __builtin_bit_cast(uint32_t, v[i]) into element 0, §8)
                    typedef uint32_t u16v __attribute__((ext_vector_type(16)));
                    const u16v ob = __builtin_bit_cast(u16v, o[t]);
                    const auto s01 = __builtin_amdgcn_permlane32_swap(ob[0], ob[1], false, false);
                    const auto s23 = __builtin_amdgcn_permlane32_swap(ob[2], ob[3], false, false);
                    const f2 p01 = __builtin_bit_cast(f2, s01), p23 = __builtin_bit_cast(f2, s23);
                    const float A = p01[0] + p01[1];
                    const float B = p23[0] + p23[1];
                    const h2 z = {};
                    const h2 ab = __builtin_elementwise_max(__builtin_bit_cast(h2, pk2(A, B)), z);
                    const float LA = (float)ab[0], LB = (float)ab[1];
                    if constexpr (EPI < 0) {
                        const auto rs = buffer_rsrc(out + s0 * NRC_OUTPUT_DIMS, tile_rows(n, s0) * 12);
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, LA), rs, r * 12 + h * 4, 0, 0);
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, LB), rs,
                                                              h ? kBufferOff : r * 12 + 8, 0, 0);
                        continue;
                    }
                    const uint32_t la = __builtin_bit_cast(uint32_t, LA);
                    const auto s11 = __builtin_amdgcn_permlane32_swap(la, la, false, false);
                    L0 = LA;
                    L1 = __builtin_bit_cast(f2, s11)[1];
                    L2 = LB;
                } else if constexpr ((ABL & 8192) != 0) {
                    // f16(max(x, 0)) == max(f16(x), 0): two packed converts + two packed maxes + three widenings
                    const h2 z = {};
                    const h2 a = __builtin_elementwise_max(__builtin_bit_cast(h2, pk2(o[t][0], o[t][1])), z);
                    const h2 b = __builtin_elementwise_max(__builtin_bit_cast(h2, pk2(o[t][2], 0.0f)), z);
                    L0 = (float)a[0];
                    L1 = (float)a[1];
                    L2 = (float)b[0];
                } else {
                    L0 = (float)(_Float16)fmaxf(o[t][0], 0.0f);
                    L1 = (float)(_Float16)fmaxf(o[t][1], 0.0f);
                    L2 = (float)(_Float16)fmaxf(o[t][2], 0.0f);
                }
                bool to_out = h == 0;
                if constexpr (EPI >= 0) {
                    float4 v;
                    if constexpr (EPI == 0) {  // Full: dst += (T * L) * w
                        v = acc[t];
                        v.x = __builtin_fmaf(tr[t][0] * L0, epi.w, v.x);
                        v.y = __builtin_fmaf(tr[t][1] * L1, epi.w, v.y);
                        v.z = __builtin_fmaf(tr[t][2] * L2, epi.w, v.z);
                    } else {  // CacheOnly
                        v.x = L0 * tr[t][0];
                        v.y = L1 * tr[t][1];
                        v.z = L2 * tr[t][2];
                    }
                    v.w = 1.0f;
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v),
                                                           buffer_rsrc(epi.rgba + s0, tile_rows(epi.n_acc, s0) * 16),
                                                           h ? kBufferOff : r * 16, 0, 0);
                    to_out = to_out && sq >= epi.n_acc;
                }
                const u3 ov = {__builtin_bit_cast(uint32_t, L0), __builtin_bit_cast(uint32_t, L1),
                               __builtin_bit_cast(uint32_t, L2)};
                __builtin_amdgcn_raw_buffer_store_b96(ov, buffer_rsrc(out + s0 * NRC_OUTPUT_DIMS, tile_rows(n, s0) * 12),
                                                      to_out ? r * 12 : kBufferOff, 0, 0);
            }
            continue;
        }
        if (h == 0) {
#pragma unroll
            for (int t = 0; t < TILES; ++t) {
                const int64_t s = (g * TILES + t) * 32 + r;
                if (s < n) {
                    const float L0 = (float)(_Float16)fmaxf(o[t][0], 0.0f);
                    const float L1 = (float)(_Float16)fmaxf(o[t][1], 0.0f);
                    const float L2 = (float)(_Float16)fmaxf(o[t][2], 0.0f);
                    if (EPI >= 0 && s < epi.n_acc) {
                        float4 v;
                        if constexpr (EPI == 0) {  // Full: dst += (T * L) * w
                            v = acc[t];
                            v.x = __builtin_fmaf(tr[t][0] * L0, epi.w, v.x);
                            v.y = __builtin_fmaf(tr[t][1] * L1, epi.w, v.y);
                            v.z = __builtin_fmaf(tr[t][2] * L2, epi.w, v.z);
                        } else {  // CacheOnly
                            v.x = L0 * tr[t][0];
                            v.y = L1 * tr[t][1];
                            v.z = L2 * tr[t][2];
                        }
                        v.w = 1.0f;
                        epi.rgba[s] = v;
                    } else {
                        float* dst = out + s * NRC_OUTPUT_DIMS;
                        dst[0] = L0;
                        dst[1] = L1;
                        dst[2] = L2;
                    }
                }
            }
        }
    }
    finish();
#if NRC_DEBUG_KERNELS
    if constexpr ((ABL & 512) != 0) {
        const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        const int64_t wid = (int64_t)blockIdx.x * (THREADS / 64) + (threadIdx.x >> 6);
        if (lane == 0 && wid < kInferClockWavesMax) {
            g_infer_clock[6 * wid] = c1 - clk0;
            g_infer_clock[6 * wid + 1] = rclk0;
            g_infer_clock[6 * wid + 2] = r1;
            g_infer_clock[6 * wid + 3] = rstart;
            g_infer_clock[6 * wid + 4] = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // hwreg(HW_REG_HW_ID)
            g_infer_clock[6 * wid + 5] = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);  // hwreg(HW_REG_XCC_ID)
        }
    }
#endif
    if constexpr ((ABL & 256) != 0) {
        const uint64_t tn = stamp_now();
        ph[7] += tn - tprev;
        const int64_t wid = (int64_t)blockIdx.x * (THREADS / 64) + (threadIdx.x >> 6);
        if (lane == 0)
#pragma unroll
            for (int k = 0; k < kInferPhases; ++k) epi.stamps[wid * kInferPhases + k] = ph[k];
    }
}

template <int TILES, int WAVES_PER_EU, int THREADS, bool PREFETCH, int ABL = 0>
__global__ __launch_bounds__(THREADS, WAVES_PER_EU) void infer_kernel_v2(const float* __restrict__ q,
                                                                         float* __restrict__ out, int64_t n,
                                                                         const h8* __restrict__ wf) {
    infer_v2_body<TILES, THREADS, PREFETCH, ABL, -1>(q, out, n, wf, InferEpilogue{});
}

#if NRC_DEBUG_KERNELS
// variant 41 (A/B, rejected: 89.3 vs 81.0 us): variant 39's body with pooled cross-CU draws
// (ABL & 16384) instead of the per-block LDS queue
template <int ABL>
__global__ __launch_bounds__(1024, 4) void infer_pooled_kernel(const float* __restrict__ q, float* __restrict__ out,
                                                              int64_t n, const h8* __restrict__ wf, InferEpilogue epi) {
    infer_v2_body<1, 1024, false, ABL, -1>(q, out, n, wf, epi);
}

// Diagnostic build of the default inference kernel (variant 23) with per-wave phase stamps (ABL & 256).
__global__ __launch_bounds__(512, 4) void infer_stamp_kernel(const float* __restrict__ q, float* __restrict__ out,
                                                             int64_t n, const h8* __restrict__ wf,
                                                             uint64_t* __restrict__ stamps) {
    InferEpilogue e{};
    e.stamps = stamps;
    infer_v2_body<1, 512, false, kDefaultAbl | 256, -1>(q, out, n, wf, e);
}

#endif

// the default inference configuration with the accumulation epilogue: THREADS 1024 + XABL 2048 = variant 39's
// shape (one block per CU, LDS work queue); THREADS 512, XABL 0 = the round-1 shape
template <int EPI, int THREADS = 512, int XABL = 0>
__global__ __launch_bounds__(THREADS, 4) void infer_accumulate_kernel(const float* __restrict__ q, float* __restrict__ out,
                                                                      int64_t n, const h8* __restrict__ wf,
                                                                      InferEpilogue epi) {
    infer_v2_body<1, THREADS, false, kDefaultAbl | 1024 | 8192 | XABL, EPI>(q, out, n, wf, epi);  // encoder v3, buffer-load prefetch
    // (XABL 2048 | 65536: the product inference kernel's shape and output layer, so the fused frame is bit-identical)
}

// InputEncoding::Hash inference (EPI -1: plain infer; 0 / 2: fused accumulation as above)
template <int EPI, int XABL = 0>
__global__ __launch_bounds__(512, 2) void infer_hash_kernel(const float* __restrict__ q, float* __restrict__ out,
                                                            int64_t n, const h8* __restrict__ wf, InferEpilogue epi,
                                                            const uint32_t* __restrict__ grid) {
    // ABL 0: the buffer-store epilogue (32) measured 2 % slower here (536 vs 524 us; gather-bound kernel)
    infer_v2_body<1, 512, false, XABL, EPI, 1>(q, out, n, wf, epi, grid);
}

// InputEncoding::Hash inference from hash_feature_kernel's level features (round 3): variant 47's shape, queue and
// 4x4x4 output layer (the gather kernel below takes the same output layer, so the two stay bitwise equal)
template <int EPI, int XABL = 0>
__global__ __launch_bounds__(1024, 4) void infer_hashf_kernel(const float* __restrict__ q, float* __restrict__ out,
                                                              int64_t n, const h8* __restrict__ wf, InferEpilogue epi,
                                                              const uint32_t* __restrict__ feat) {
    infer_v2_body<1, 1024, false, 32 | 2048 | 8192 | 65536 | XABL, EPI, 3>(q, out, n, wf, epi, feat);
}

// FrequencySH extension inference (EPI -1 plain; 0 / 2 fused accumulation)
template <int EPI, int THREADS = 512, int XABL = 0>
__global__ __launch_bounds__(THREADS, 4) void infer_sh_kernel(const float* __restrict__ q, float* __restrict__ out,
                                                              int64_t n, const h8* __restrict__ wf, InferEpilogue epi) {
    infer_v2_body<1, THREADS, false, kDefaultAbl | XABL, EPI, 2>(q, out, n, wf, epi);
}

// The production FrequencySH encoder unpacked to canonical order as f32 (parity tests): [n][80].
__global__ void encode_sh_kernel(const float* __restrict__ q, float* __restrict__ enc, int64_t n) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t s = gid >> 1;
    const int h = (int)(gid & 1);
    if (s >= n) return;
    const QLane Q = load_q_sh(q, s, h);
    h8 x[5];
    encode_sh(Q, h, x);
#pragma unroll
    for (int k = 0; k < 40; ++k) enc[s * NRC_ENC_WIDTH + sh_slot_feature(k, h)] = (float)x[k >> 3][k & 7];
}

// The production hash encoder unpacked to canonical order as f32 (parity tests): [n][64].
__global__ void encode_hash_kernel(const float* __restrict__ q, const uint32_t* __restrict__ grid,
                                   float* __restrict__ enc, int64_t n) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t s = gid >> 1;
    const int h = (int)(gid & 1);
    if (s >= n) return;
    const QLane Q = load_q(q, s, h);
    h8 x[4];
    encode_hash(Q, h, grid, x);
#pragma unroll
    for (int k = 0; k < 32; ++k) enc[s * NRC_HASH_ENC_WIDTH + hash_slot_feature(k, h)] = (float)x[k >> 3][k & 7];
}

// ------------------------------------------------------------------------------------------------
// Width-128 MLP inference (BASELINE.json configs[4] / SURVEY §8 C5; oracle/nrc_wide_oracle.c).
// Same structure as the 64-wide kernel: one wave = 32 queries on the MFMA column axis, the encoder's f16 output as
// layer 0's B operand, every layer's accumulators converted in registers into the next layer's B operand.
//   PREC 0 (f16): 4 M-blocks x 8 k-steps of v_mfma_f32_32x32x16_f16 per hidden layer; 156 KiB of fragments in LDS.
//   PREC 1 (FP8): layer 0 f16; layers 1..5 on v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 x e4m3, 2x the f16 rate), the
//   weights e4m3 with one E8M0 scale per output row (the MX scale-A operand: byte mb of the lane's scale word via
//   op_sel), activations converted with v_cvt_scalef32_pk_fp8_f32 (RNE, saturating at +-448 under MODE.FP16_OVFL)
//   and ReLU'd on the e4m3 bytes (pack_fp8; round 5 clamped every value with a med3 first); 88 KiB of fragments in LDS.
// ------------------------------------------------------------------------------------------------
typedef int i8v __attribute__((ext_vector_type(8)));  // 32 e4m3 bytes: one operand of the 32x32x64 MX MFMA

template <int OPSEL>
__device__ __forceinline__ f16v mfma_fp8(const i8v& a, const i8v& b, const f16v& c, uint32_t scale_a) {
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, OPSEL, (int)scale_a, 0, 127);
}
__device__ __forceinline__ f16v mfma_fp8_mb(int mb, const i8v& a, const i8v& b, const f16v& c, uint32_t scale_a) {
    switch (mb) {  // mb is a constant after unrolling: the switch folds
        case 0: return mfma_fp8<0>(a, b, c, scale_a);
        case 1: return mfma_fp8<1>(a, b, c, scale_a);
        case 2: return mfma_fp8<2>(a, b, c, scale_a);
        default: return mfma_fp8<3>(a, b, c, scale_a);
    }
}

// e4m3 bytes of ReLU(accumulator registers 4q .. 4q+3), saturated at 448: the round-5 form (debug variant 2),
// one med3 per value before the convert.
__device__ __forceinline__ uint32_t relu_fp8x4_med3(const f16v& c, int q) {
    const float a0 = __builtin_amdgcn_fmed3f(c[4 * q + 0], 0.0f, 448.0f);
    const float a1 = __builtin_amdgcn_fmed3f(c[4 * q + 1], 0.0f, 448.0f);
    const float a2 = __builtin_amdgcn_fmed3f(c[4 * q + 2], 0.0f, 448.0f);
    const float a3 = __builtin_amdgcn_fmed3f(c[4 * q + 3], 0.0f, 448.0f);
    // the first convert writes bytes 0..1 and keeps bytes 2..3 of its "old" operand, which the second overwrites: old =
    // a0's own bits (a0 dies here, so the destination takes its register) instead of 0, which cost one v_mov_b32 per
    // 4 values (80 per tile)
    const uint32_t lo = __builtin_amdgcn_cvt_pk_fp8_f32(a0, a1, (int)__builtin_bit_cast(uint32_t, a0), false);
    return __builtin_amdgcn_cvt_pk_fp8_f32(a2, a3, lo, true);
}

// MODE.FP16_OVFL (bit 23): overflowing f16 / FP8 results clamp to the largest finite value instead of inf / NaN
__device__ __forceinline__ void fp8_saturating_converts() {
    __builtin_amdgcn_s_setreg((0 << 11) | (23 << 6) | 1 /* hwreg(HW_REG_MODE, 23, 1) */, 1u);
}
// two e4m3 bytes into word half `hi` of `old` (scale 1), saturating under fp8_saturating_converts()
template <bool HI>
__device__ __forceinline__ uint32_t cvt_sat_fp8(float a, float b, uint32_t old) {
    typedef short s2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(__builtin_bit_cast(s2, old), a, b,
                                                                                  1.0f, HI));
}

// Zero every e4m3 byte of w whose sign bit is set (a negative value or -0): v_perm_b32's selectors 8..11 replicate the
// sign bits of bytes 1, 3 of its second source and bytes 1, 3 of its first, so (w << 8, w) with 0x090B080A gives 0xFF
// for each such byte.
__device__ __forceinline__ uint32_t relu_e4m3x4(uint32_t w, uint32_t sh) {
    return w & ~__builtin_amdgcn_perm(sh, w, 0x090B080Au);
}

// next layer's fp8 B operands from the 4 accumulator blocks: k-step s byte j = row f8_row(s, h, j)
template <bool MED3 = false>
__device__ __forceinline__ void pack_fp8(const f16v (&c)[4], i8v (&y)[2]) {
    if constexpr (!MED3) {
        // round 6: ReLU on the converted bytes. Under MODE.FP16_OVFL (set at kernel start,
        // fp8_saturating_converts) the scaled convert saturates at +-448, infinities included, as the med3 clamp does
        // (tools/probe_fp8_cvt.hip: without the mode bit a finite value past 464 becomes 0x7F, a NaN), then
        // relu_e4m3x4: 3 VALU per 4 values instead of 4 med3 (FP8 width-128 kernel 632.7 -> 590.2 us per 2^23
        // queries, bitwise equal, profiles/r06_wide/).
        // The first convert's "old" operand (bytes 2..3 kept, then overwritten by the second convert) must be a register
        // that dies there: an accumulator element would be copied first (its tuple is still live), so it is the
        // previous group's shifted word
        uint32_t spare = 0;
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int d = 0; d < 8; ++d) {
                const f16v& cc = c[2 * s + (d >> 2)];
                const int q = d & 3;
                const uint32_t lo = cvt_sat_fp8<false>(cc[4 * q + 0], cc[4 * q + 1], spare);
                const uint32_t w = cvt_sat_fp8<true>(cc[4 * q + 2], cc[4 * q + 3], lo);
                const uint32_t sh = w << 8;
                y[s][d] = (int)relu_e4m3x4(w, sh);
                spare = sh;
            }
        return;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int d = 0; d < 8; ++d) y[s][d] = (int)relu_fp8x4_med3(c[2 * s + (d >> 2)], d & 3);
}

// wait for LDS reads at this point only (the image copy) — a full __syncthreads() would also wait for the
// prefetched query loads
template <int THREADS, int COUNT>
__device__ __forceinline__ void copy_to_lds_chunked(h8* __restrict__ dst, const h8* __restrict__ src) {
    constexpr int PER = (COUNT + THREADS - 1) / THREADS;
    constexpr int CH = 5;
#pragma unroll
    for (int k0 = 0; k0 < PER; k0 += CH) {
        h8 v[CH];
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int i = threadIdx.x + (k0 + k) * THREADS;
            if (k0 + k < PER && i < COUNT) v[k] = src[i];
        }
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int i = threadIdx.x + (k0 + k) * THREADS;
            if (k0 + k < PER && i < COUNT) dst[i] = v[k];
        }
    }
}

// The width-128 images span 88 / 156 KiB of LDS, past the 64-KiB reach of a ds_read's immediate offset: a fragment read
// through one laundered base pointer cost a v_add_u32 per read beyond it (108 per tile f16, 40 FP8). WideLds holds one
// laundered base per 64 KiB (the launder keeps the reads inside the tile loop, as in the 64-wide kernel), so every
// fragment read is base k + an immediate.
struct WideLds {
    lds_h8* b[3];
    __device__ __forceinline__ explicit WideLds(lds_h8* lane_base) {
#pragma unroll
        for (int k = 0; k < 3; ++k) b[k] = launder(lane_base + 4096 * k);
    }
    // h8 offset o (a compile-time constant after unrolling) from the lane's base
    __device__ __forceinline__ h8 at(int o) const { return b[o >> 12][o & 4095]; }
};

template <int PREC, bool MED3 = false>
__device__ __forceinline__ f16v wide_mlp(lds_h8* lw_lane, const h8 (&x)[5], const uint32_t (&sc)[5]) {
    f16v c[4];
    {
        const WideLds wl(lw_lane);
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) c[mb] = zero16();
#pragma unroll
        for (int kk = 0; kk < 5; ++kk)
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) c[mb] = mfma(wl.at(wide_frag(0, mb, kk) * 64), x[kk], c[mb]);
    }
    if constexpr (PREC == 0) {
        h8 y[8];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) y[kk] = relu_h8(c[kk >> 1], 8 * (kk & 1));
#pragma unroll
        for (int l = 1; l < 5; ++l) {
            const WideLds wl(lw_lane);
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) c[mb] = zero16();
#pragma unroll
            for (int kk = 0; kk < 8; ++kk)
#pragma unroll
                for (int mb = 0; mb < 4; ++mb) c[mb] = mfma(wl.at(wide_frag(l, mb, kk) * 64), y[kk], c[mb]);
#pragma unroll
            for (int kk = 0; kk < 8; ++kk) y[kk] = relu_h8(c[kk >> 1], 8 * (kk & 1));
        }
        const WideLds wl(lw_lane);
        f16v o = zero16();
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) o = mfma(wl.at(wide_frag(5, 0, kk) * 64), y[kk], o);
        return o;
    } else {
        i8v y[2];
        pack_fp8<MED3>(c, y);
        // fp8 fragment f: planes at h8 offsets (20 + 2 f) * 64 and (21 + 2 f) * 64 from the lane's base
        auto frag8 = [&](const WideLds& wl, int f) {
            const h8 lo = wl.at((20 + 2 * f) * 64), hi = wl.at((21 + 2 * f) * 64);
            typedef int i4v __attribute__((ext_vector_type(4)));
            // one shuffle of the two 16-byte reads (element-wise construction made the compiler copy both halves into a
            // fresh register octet: 96 v_mov_b32 per tile)
            return (i8v)__builtin_shufflevector(__builtin_bit_cast(i4v, lo), __builtin_bit_cast(i4v, hi), 0, 1, 2, 3, 4, 5,
                                                6, 7);
        };
#pragma unroll
        for (int l = 1; l < 5; ++l) {
            const WideLds wl(lw_lane);
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) c[mb] = zero16();
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int mb = 0; mb < 4; ++mb)
                    c[mb] = mfma_fp8_mb(mb, frag8(wl, wide8_frag(l, mb, s)), y[s], c[mb], sc[l - 1]);
            pack_fp8<MED3>(c, y);
        }
        const WideLds wl(lw_lane);
        f16v o = zero16();
#pragma unroll
        for (int s = 0; s < 2; ++s) o = mfma_fp8<0>(frag8(wl, wide8_frag(5, 0, s)), y[s], o, sc[4]);
        return o;
    }
}

// ENC 0 = Frequency, 2 = FrequencySH (both 80-wide); EPI -1 plain, 0 / 2 fused accumulate_render_radiance.
// Persistent waves, 2 per SIMD (one 512-thread block per CU: the f16 image takes 156 KiB of LDS).
// THREADS 1024 (debug variant 1): 4 waves per SIMD within 128 VGPRs.
// QUEUE (round 2, default): the block owns a contiguous range of tiles and its waves draw from an LDS counter (as the
// 64-wide variant 39) instead of a fixed tile sequence per wave.
// MED3 (debug variant 2): the FP8 activations clamped by one med3 per value before the convert (round 5).
template <int ENC, int PREC, int EPI, int THREADS = 512, bool QUEUE = false, bool MED3 = false>
__global__ __launch_bounds__(THREADS, THREADS / 256) void infer_wide_kernel(const float* __restrict__ q,
                                                                            float* __restrict__ out, int64_t n,
                                                                            const h8* __restrict__ img,
                                                                            InferEpilogue epi,
                                                                            const uint32_t* __restrict__ wscale) {
    constexpr int NH8 = (PREC == 0 ? kWideF16Bytes : kWide8Bytes) / 16;
    __shared__ __attribute__((aligned(16))) h8 lw[NH8];
    __shared__ uint32_t wq_next;
    fp32_flush_output_denorms();  // the omod doubling-chain encoder
    if constexpr (PREC == 1 && !MED3) fp8_saturating_converts();  // pack_fp8
    copy_to_lds_chunked<THREADS, NH8>(lw, img);
    if (QUEUE && threadIdx.x == 0) wq_next = 0;
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int h = lane >> 5, r = lane & 31;
    uint32_t sc[5] = {};
    if constexpr (PREC == 1) {
#pragma unroll
        for (int l = 0; l < 5; ++l) sc[l] = wscale[l * 32 + r];
    }
    const int64_t ntiles = (n + 31) >> 5;
    const int64_t wstride = (int64_t)gridDim.x * (THREADS / 64);
    int64_t g, ngroups = ntiles, gbase = 0, ng = 0;
    uint32_t nn_raw = 0;
    if constexpr (QUEUE) {
        gbase = (int64_t)blockIdx.x * ntiles / gridDim.x;
        ngroups = (int64_t)(blockIdx.x + 1) * ntiles / gridDim.x;  // end of this block's range
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(&wq_next, 1u);
        g = gbase + (int64_t)__builtin_amdgcn_readfirstlane(t);
        if (g >= ngroups) return;
        if (lane == 0) t = atomicAdd(&wq_next, 1u);
        ng = gbase + (int64_t)__builtin_amdgcn_readfirstlane(t);
    } else {
        g = (int64_t)blockIdx.x * (THREADS / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        if (g >= ngroups) return;
    }
    const int64_t last = n - 1;
    QLane Q = load_q_enc<ENC>(q, min(g * 32 + r, last), h);
    if constexpr (EPI >= 0) __builtin_amdgcn_raw_buffer_store_b128(u4{0u, 0u, 0u, 0u}, buffer_rsrc(out, 0), 0, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b96(u3{0u, 0u, 0u}, buffer_rsrc(out, 0), 0, 0, 0);
    for (bool first = true; g < ngroups; first = false) {
        if constexpr (QUEUE) {
            if (!first) {
                // the draw issued one iteration ago (an asm readfirstlane stays here; the builtin would be hoisted
                // to the atomic and the wave would wait for it there)
                uint32_t t;
                asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(t) : "v"(nn_raw));
                ng = gbase + (int64_t)t;
            }
        } else {
            ng = g + wstride;
        }
        h8 x[5];
        // round 6: the 64-wide kernel's encoder v3 (tent-map wave, OneBlob wrap as two clamps: one path) instead of
        // round 1's encode_fast, whose OneBlob wrap branch the Cornell stream's raw angles always take (-61 VALU per tile)
        if constexpr (ENC == 2) encode_sh<true>(Q, h, x);
        else encode_v3(Q, h, x);
        if constexpr (QUEUE) {
            if (lane == 0) nn_raw = atomicAdd(&wq_next, 1u);  // the tile after next
        }
        Q = load_q_enc<ENC>(q, min(ng * 32 + r, last), h);  // clamped, branch-free prefetch
        const int64_t s0 = g * 32, sq = s0 + r;
        float tr[3] = {};
        float4 acc = {};
        if constexpr (EPI >= 0) {
            const int rows = tile_rows(epi.n_acc, s0);
            const u3 tv = __builtin_amdgcn_raw_buffer_load_b96(buffer_rsrc(epi.thr + s0 * 3, rows * 12),
                                                               h ? kBufferOff : r * 12, 0, 0);
            typedef float f3 __attribute__((ext_vector_type(3)));
            const f3 tf = __builtin_bit_cast(f3, tv);  // whole-vector bit_cast (see infer_v2_body)
            tr[0] = tf.x;
            tr[1] = tf.y;
            tr[2] = tf.z;
            if constexpr (EPI == 0) {
                const u4 av = __builtin_amdgcn_raw_buffer_load_b128(buffer_rsrc(epi.rgba + s0, rows * 16),
                                                                    h ? kBufferOff : r * 16, 0, 0);
                acc = __builtin_bit_cast(float4, av);
            }
        }
        const f16v o = wide_mlp<PREC, MED3>((lds_h8*)(lw + lane), x, sc);
        const float L0 = (float)(_Float16)fmaxf(o[0], 0.0f);
        const float L1 = (float)(_Float16)fmaxf(o[1], 0.0f);
        const float L2 = (float)(_Float16)fmaxf(o[2], 0.0f);
        bool to_out = h == 0;
        if constexpr (EPI >= 0) {
            float4 v;
            if constexpr (EPI == 0) {  // Full: dst += (T * L) * w
                v = acc;
                v.x = __builtin_fmaf(tr[0] * L0, epi.w, v.x);
                v.y = __builtin_fmaf(tr[1] * L1, epi.w, v.y);
                v.z = __builtin_fmaf(tr[2] * L2, epi.w, v.z);
            } else {  // CacheOnly
                v.x = L0 * tr[0];
                v.y = L1 * tr[1];
                v.z = L2 * tr[2];
            }
            v.w = 1.0f;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v),
                                                   buffer_rsrc(epi.rgba + s0, tile_rows(epi.n_acc, s0) * 16),
                                                   h ? kBufferOff : r * 16, 0, 0);
            to_out = to_out && sq >= epi.n_acc;
        }
        const u3 ov = {__builtin_bit_cast(uint32_t, L0), __builtin_bit_cast(uint32_t, L1),
                       __builtin_bit_cast(uint32_t, L2)};
        __builtin_amdgcn_raw_buffer_store_b96(ov, buffer_rsrc(out + s0 * NRC_OUTPUT_DIMS, tile_rows(n, s0) * 12),
                                              to_out ? r * 12 : kBufferOff, 0, 0);
        g = ng;
    }
}

// width-128 training layout helpers: backward-image fragment, workspace rows, parameter offsets
__host__ __device__ constexpr int wide_bwd_frag(int layer, int mb, int kk) {
    return layer == 5 ? mb : 4 + (layer - 1) * 32 + mb * 8 + kk;
}
__host__ __device__ constexpr int64_t wide_in_row(int layer) { return layer == 0 ? 0 : 80 + (layer - 1) * 128; }
__host__ __device__ constexpr int64_t wide_d_row(int layer) { return (int64_t)layer * 128; }
__host__ __device__ constexpr int wide_off(int layer) {
    return layer == 0 ? NRC_WIDE_W0_OFFSET : layer <= 4 ? NRC_WIDE_W1_OFFSET + (layer - 1) * 16384 : NRC_WIDE_W5_OFFSET;
}

// e4m3 conversion as the FP8 kernels do it (diagnostic entry for the exhaustive conversion test)
__global__ void fp8_convert_kernel(const float* __restrict__ x, uint8_t* __restrict__ y, int64_t n, int relu) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fp8_saturating_converts();  // the FP8 inference kernel's conversion (pack_fp8)
    uint32_t w = cvt_sat_fp8<false>(x[i], 0.0f, 0u);
    if (relu) w = relu_e4m3x4(w, w << 8);
    y[i] = (uint8_t)(w & 0xffu);
}

// Standalone encoding kernel (HBM-bound; used by the parity tests of the encoding): writes the f32
// features in canonical tcnn order, [n][80].
__global__ void encode_kernel(const float* __restrict__ q, float* __restrict__ enc, int64_t n) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t s = gid >> 1;
    const int h = (int)(gid & 1);
    if (s >= n) return;
    const QLane Q = load_q(q, s, h);
    float v[40];
    encode_f32(Q, h, v);
#pragma unroll
    for (int k = 0; k < 40; ++k) enc[s * NRC_ENC_WIDTH + slot_feature(k, h)] = v[k];
}

// The production encoder (encode_fast: f16 B fragments) unpacked to canonical order as f32 — lets the
// parity tests check the exact code path the MLP kernels run.
template <int VARIANT>  // 0: encode_fast, 1: encode_fast<CHAIN>, 2: encode_v3
__global__ void encode_fast_kernel(const float* __restrict__ q, float* __restrict__ enc, int64_t n) {
    if (VARIANT >= 1) fp32_flush_output_denorms();
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t s = gid >> 1;
    const int h = (int)(gid & 1);
    if (s >= n) return;
    const QLane Q = load_q(q, s, h);
    h8 x[5];
    if constexpr (VARIANT == 2) encode_v3(Q, h, x);
    else encode_fast<VARIANT == 1>(Q, h, x);
#pragma unroll
    for (int k = 0; k < 40; ++k) enc[s * NRC_ENC_WIDTH + slot_feature(k, h)] = (float)x[k >> 3][k & 7];
}

hipError_t launch_encode_fast(const float* queries, float* enc, int64_t n, hipStream_t s, int variant) {
    if (n <= 0) return hipSuccess;
    const int grid = (int)((2 * n + 255) / 256);
    if (variant == 2)
        hipLaunchKernelGGL(encode_fast_kernel<2>, dim3(grid), dim3(256), 0, s, queries, enc, n);
    else if (variant == 1)
        hipLaunchKernelGGL(encode_fast_kernel<1>, dim3(grid), dim3(256), 0, s, queries, enc, n);
    else
        hipLaunchKernelGGL(encode_fast_kernel<0>, dim3(grid), dim3(256), 0, s, queries, enc, n);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Training: one block = 4 waves = 128 samples.
// ------------------------------------------------------------------------------------------------
// LDS images of activations / deltas for the weight-gradient GEMMs: [128 samples][64 features] f16, 128-B rows.
// A lane holds 8 features of one sample per fragment, as two 4-feature quads 8 features apart (acc_row), so the
// quads of a row are stored permuted (bits 0 and 1 of the quad index swapped within each group of 4) to make
// those two quads one 16-byte slot, and the 8 slots of a row are XOR-swizzled by a bijection of (s mod 8) in
// which s and s + 2 differ in bit 2. Then the row writes are one ds_write_b128 per fragment (8 contiguous
// lanes = 8 samples hit 8 distinct slots) and the transposed reads (ds_read_b64_tr_b16: 4 samples x 8 quads
// per 32 lanes; samples s, s+2 share a bank half and get disjoint slot groups) are conflict-free. At one wave
// per SIMD the 16-byte stores reach the LDS store rate where 8-byte ones do not (MI355X_MICROARCH.md §LDS):
// 16 ds_write_b64 per wave and layer took ~1,100 cycles.
__device__ __forceinline__ int img_off(int s, int c) {
    const int lq = c >> 2;
    const int pq = (lq & ~3) | ((lq & 1) << 1) | ((lq >> 1) & 1);
    const int hs = (s & 1) | (((s >> 2) & 1) << 1) | (((s >> 1) & 1) << 2);
    return s * 128 + (((pq >> 1) ^ hs) << 4) + ((pq & 1) << 3) + ((c & 3) << 1);
}

__device__ __forceinline__ h4 tr_read(const char* p) {
    const s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)p);
    return __builtin_bit_cast(h4, v);
}

__device__ __forceinline__ h8 cat(h4 a, h4 b) {
    h8 r;
    r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
    r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
    return r;
}

// MFMA operand with samples on k: lane (row = 32*fb + (lane&31), half hh) gets samples 16kk+8hh+0..7
// of that feature, from a [sample][feature] image (cdna_hip_programming.md T10).
__device__ __forceinline__ h8 tr_frag(const char* img, int fb, int kk, int lane) {
    const int g = lane >> 4, idx = lane & 15, q = idx >> 2, p = idx & 3;
    const int c = 32 * fb + 16 * (g & 1) + 4 * p;
    const int s0 = 16 * kk + 8 * (g >> 1) + q;
    return cat(tr_read(img + img_off(s0, c)), tr_read(img + img_off(s0 + 4, c)));
}

// Same for the 16-wide x_hi image ([128][16] f16, 32-B rows); lanes for features >= 16 read the same
// addresses as their partners (results discarded).
__device__ __forceinline__ h8 tr_frag_xhi(const char* img, int kk, int lane) {
    const int g = lane >> 4, idx = lane & 15, q = idx >> 2, p = idx & 3;
    const int s0 = 16 * kk + 8 * (g >> 1) + q;
    return cat(tr_read(img + s0 * 32 + 8 * p), tr_read(img + (s0 + 4) * 32 + 8 * p));
}

__device__ __forceinline__ void store_h4(char* img, int off, h8 v, int j0) {
    h4 t;
    t[0] = v[j0]; t[1] = v[j0 + 1]; t[2] = v[j0 + 2]; t[3] = v[j0 + 3];
    *(h4*)(img + off) = t;
}

// Write a 64-row activation/delta held as 4 B fragments (rows acc_row(kk,h,j)) into the image: fragment kk is
// one 16-byte slot (see img_off).
__device__ __forceinline__ void write_rows64(char* img, int sl, int h, const h8 (&f)[4]) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) *(h8*)(img + img_off(sl, acc_row(kk, h, 0))) = f[kk];
}

constexpr int kLdsWf = kFwdHalves * 2;   // 47104
constexpr int kLdsWb = kBwdHalvesHash * 2;  // 38912 (the Frequency config uses the first 34816)
constexpr int kLdsImg = 128 * 128;       // 16384
constexpr int kLdsXhi = 128 * 32;        // 4096
constexpr int kLdsTrain = kLdsWf + kLdsWb + 4 * kLdsImg + kLdsXhi + 16;

// canonical offset of W_L in the parameter blob of encoding ENC (layout.h)
template <int L, int ENC>
__host__ __device__ constexpr int w_offset() {
    return ENC == 1 ? (L == 0 ? NRC_HASH_W0_OFFSET : L <= 4 ? NRC_HASH_W1_OFFSET + (L - 1) * 4096 : NRC_HASH_W5_OFFSET)
                    : (L == 0   ? NRC_W0_OFFSET
                       : L == 1 ? NRC_W1_OFFSET
                       : L == 2 ? NRC_W2_OFFSET
                       : L == 3 ? NRC_W3_OFFSET
                       : L == 4 ? NRC_W4_OFFSET
                                : NRC_W5_OFFSET);
}

// Lane offsets of the transposed reads. tr_frag(img, fb, kk) reads img + img_off(s0, c) and img + img_off(s0 + 4, c)
// with s0 = 16 kk + (lane part): the k step only adds 16 rows = 2048 bytes (the swizzle uses s mod 8), and the x_hi
// image's rows are 32 bytes, so every read of a layer step is a per-lane base plus an immediate offset. Computed once
// per kernel and hidden from the optimiser, which otherwise rebuilds each address with 3-4 VALU (v_or does not fold
// into the ds_read offset field).
struct TrOffs {
    int a[2][2];  // feature block fb, read 0/1
    int x[2];     // x_hi image, read 0/1
};
__device__ __forceinline__ TrOffs make_tr_offs(int lane) {
    const int g = lane >> 4, idx = lane & 15, q = idx >> 2, p = idx & 3;
    const int s0 = 8 * (g >> 1) + q;
    TrOffs o;
#pragma unroll
    for (int fb = 0; fb < 2; ++fb) {
        const int c = 32 * fb + 16 * (g & 1) + 4 * p;
        o.a[fb][0] = img_off(s0, c);
        o.a[fb][1] = img_off(s0 + 4, c);
        asm volatile("" : "+v"(o.a[fb][0]), "+v"(o.a[fb][1]));
    }
    o.x[0] = s0 * 32 + 8 * p;
    o.x[1] = (s0 + 4) * 32 + 8 * p;
    asm volatile("" : "+v"(o.x[0]), "+v"(o.x[1]));
    return o;
}
__device__ __forceinline__ h8 tr_frag_o(const char* img, int o0, int o1, int kk) {
    return cat(tr_read(img + o0 + 2048 * kk), tr_read(img + o1 + 2048 * kk));
}

// dW output block (mb, nb) of layer L: A = delta image (features = output rows), B = activation image.
// Split into the MFMA chain and the slab store so that a layer step can issue the delta chain between them: the
// wave issues in order, and a store placed right after the dW MFMAs would hold it until their results are out.
// All 32 transposed reads are issued before the first MFMA, so the chain waits on them once instead of once per k step.
template <int L, int ENC = 0>
__device__ __forceinline__ f16v dw_block_mfma(const char* img_d, const char* img_a, const char* img_xh, int mb, int nb,
                                              int lane, const TrOffs& to) {
    const bool zero_a = (L == 5) && (lane & 16);  // rows 16..31 of the 16-row output delta do not exist
    const bool xhi = ENC != 1 && L == 0 && nb == 2;
    const int da0 = mb ? to.a[1][0] : to.a[0][0], da1 = mb ? to.a[1][1] : to.a[0][1];
    const int db0 = nb ? to.a[1][0] : to.a[0][0], db1 = nb ? to.a[1][1] : to.a[0][1];
    h8 A[8], B[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
        A[kk] = tr_frag_o(img_d, da0, da1, kk);
        if (L == 0 && ENC != 1 && xhi)
            B[kk] = cat(tr_read(img_xh + to.x[0] + 512 * kk), tr_read(img_xh + to.x[1] + 512 * kk));
        else
            B[kk] = tr_frag_o(img_a, db0, db1, kk);
    }
    f16v acc = zero16();
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) acc = mfma(zero_a ? h8{} : A[kk], B[kk], acc);
    return acc;
}

template <int L, int ENC = 0>
__device__ __forceinline__ void dw_block_store(const f16v& acc, int mb, int nb, int lane, float* __restrict__ slab) {
    // fragment-major slab block (slab_block_base): 4 (layer 5: 2) lane-contiguous 16-byte stores per lane
    typedef float f4 __attribute__((ext_vector_type(4)));
    constexpr int J = L == 5 ? 2 : 4;  // layer 5: registers 0..7 hold the 16 real rows
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const f4 v = {acc[4 * j], acc[4 * j + 1], acc[4 * j + 2], acc[4 * j + 3]};
#if defined(NRC_SLAB_NT)
        // streamed: nontemporal (plain stores measured 18.8 -> 20.7 us per step)
        __builtin_nontemporal_store(v, (f4*)(slab + slab_block_base(ENC, L, mb, nb)) + j * 64 + lane);
#else
        // sc1: write through, the line dropped from the XCD's L2 (no end-of-launch write-back of the slabs; the
        // reduce reads them from memory on every XCD anyway; round 2, as nrc_train16.hip's slab stores)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), buffer_rsrc(slab, slab_floats(ENC) * 4),
                                               (slab_block_base(ENC, L, mb, nb) + (j * 64 + lane) * 4) * 4, 0, 16);
#endif
    }
}

// The dW blocks of layer L for this wave: 64x64 layers = 2x2 blocks (one per wave); layer 5 = 1x2 (waves 0,1);
// Frequency layer 0 = 2x3 blocks (the third column block is the 16-wide x_hi image; waves 0,1 take two).
template <int L, int ENC = 0>
struct DwAcc {
    f16v a0, a1;
    __device__ __forceinline__ void mfma_all(const char* img_d, const char* img_a, const char* img_xh, int wave,
                                             int lane, const TrOffs& to) {
        if (L == 5) {
            if (wave < 2) a0 = dw_block_mfma<5, ENC>(img_d, img_a, img_xh, 0, wave, lane, to);
        } else if (L == 0 && ENC != 1) {
            a0 = dw_block_mfma<0, ENC>(img_d, img_a, img_xh, wave / 3, wave % 3, lane, to);
            if (wave < 2) a1 = dw_block_mfma<0, ENC>(img_d, img_a, img_xh, (wave + 4) / 3, (wave + 4) % 3, lane, to);
        } else {
            a0 = dw_block_mfma<L, ENC>(img_d, img_a, img_xh, wave >> 1, wave & 1, lane, to);
        }
    }
    __device__ __forceinline__ void store_all(int wave, int lane, float* __restrict__ slab) const {
        if (L == 5) {
            if (wave < 2) dw_block_store<5, ENC>(a0, 0, wave, lane, slab);
        } else if (L == 0 && ENC != 1) {
            dw_block_store<0, ENC>(a0, wave / 3, wave % 3, lane, slab);
            if (wave < 2) dw_block_store<0, ENC>(a1, (wave + 4) / 3, (wave + 4) % 3, lane, slab);
        } else {
            dw_block_store<L, ENC>(a0, wave >> 1, wave & 1, lane, slab);
        }
    }
};


// Backward ReLU on packed halves: d = f16(acc) where the forward activation a > 0, else +0. One dword (two
// features) costs v_cvt_pk_f16_f32 + v_pk_max_i16 + v_pk_min_i16 + v_pk_mul_lo_u16: the activation bits as i16
// are positive exactly for a > 0 (+0, -0 and negatives are not; a ReLU output is never negative), clamped to
// 0/1 they select the delta bits by an integer multiply. Same values as mask_pack (7 VALU per dword there)
// except for a NaN activation, which this keeps and a > 0 drops.
__device__ __forceinline__ uint32_t relu_gate_pk(uint32_t d, uint32_t m) {
    // written out: the compiler folds clamp-to-0/1-and-multiply back into per-half compares and selects
    uint32_t r;
    asm("v_pk_max_i16 %0, %1, 0\n\t"
        "v_pk_min_i16 %0, %0, %3\n\t"
        "v_pk_mul_lo_u16 %0, %0, %2"
        : "=&v"(r)
        : "v"(m), "v"(d), "s"(0x00010001u));
    return r;
}

__device__ __forceinline__ void mask_pack_pk(const f16v& a, const h8& m_lo, const h8& m_hi, h8& lo, h8& hi) {
    typedef uint32_t u4v __attribute__((ext_vector_type(4)));
    const u4v ml = __builtin_bit_cast(u4v, m_lo), mh = __builtin_bit_cast(u4v, m_hi);
    u4v ol, oh;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        ol[k] = relu_gate_pk(pk2(a[2 * k], a[2 * k + 1]), ml[k]);
        oh[k] = relu_gate_pk(pk2(a[8 + 2 * k], a[8 + 2 * k + 1]), mh[k]);
    }
    lo = __builtin_bit_cast(h8, ol);
    hi = __builtin_bit_cast(h8, oh);
}

// delta_{L-1} = (W_L^T delta_L) * [a_L > 0]
// W(i) returns backward fragment i of this lane (register-resident or LDS image).
template <int L, class W>
__device__ __forceinline__ void bwd_chain(W wfrag, const h8 (&d)[4], const h8 (&a)[4], h8 (&dn)[4]) {
    constexpr int KK = (L == 5) ? 1 : 4;
    f16v c0 = zero16(), c1 = zero16();
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
        c0 = mfma(wfrag(bwd_frag(L, 0, kk)), d[kk], c0);
        c1 = mfma(wfrag(bwd_frag(L, 1, kk)), d[kk], c1);
    }
    mask_pack_pk(c0, a[0], a[1], dn[0], dn[1]);
    mask_pack_pk(c1, a[2], a[3], dn[2], dn[3]);
}

// The same with the layer's backward fragments read ahead (before the step's dW operand reads), so the chain's
// MFMAs do not each wait on their own ds_read_b128.
template <int L, class W>
__device__ __forceinline__ void load_bwd(W wfrag, h8 (&w)[2][4]) {
    constexpr int KK = (L == 5) ? 1 : 4;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
        w[0][kk] = wfrag(bwd_frag(L, 0, kk));
        w[1][kk] = wfrag(bwd_frag(L, 1, kk));
    }
}
template <int L>
__device__ __forceinline__ void bwd_chain_pre(const h8 (&w)[2][4], const h8 (&d)[4], const h8 (&a)[4], h8 (&dn)[4]) {
    bwd_chain<L>([&](int i) { return i < 2 ? w[i][0] : w[((i - 2) >> 2) & 1][(i - 2) & 3]; }, d, a, dn);
}

// grid_grad[e] += (half2){a, b}: each product rounded to f16, accumulated in f16 at the memory side
__device__ __forceinline__ void grid_atomic(h2v* __restrict__ grid_grad, uint32_t e, float a, float b) {
    const h2v v = {(_Float16)a, (_Float16)b};
    __builtin_amdgcn_global_atomic_fadd_v2f16((__attribute__((address_space(1))) h2v*)(grid_grad + e), v);
}

// STAMP (diagnostic build only): wave 0 of every block records s_memtime at phase boundaries into
// stamps[block][16]; the product instantiation (STAMP = false) executes no stamp.
// ENC 1 (InputEncoding::Hash): 64-wide layer 0, grid table `grid` (f16x2, training weights); the grid-feature
// gradient W0^T delta_0 is scattered into grid_grad (f16x2 per entry) with packed-half atomics, as tcnn's
// kernel_grid_backward does (half2 atomicAdd): one 4-byte atomic per corner for both features.
// PADQ: padded RadianceQuery records (Hash only in the product: nrc_config.query_layout = NRC_QUERY_PADDED)
template <bool STAMP, int ENC = 0, bool PADQ = false>
__global__ __launch_bounds__(256, 1) void train_kernel(const float* __restrict__ q, const float* __restrict__ t,
                                                       int64_t b, float n_total, float loss_scale,
                                                       const h8* __restrict__ wf, const h8* __restrict__ wb,
                                                       float* __restrict__ slabs, float* __restrict__ loss_partials,
                                                       uint64_t* __restrict__ stamps,
                                                       const uint32_t* __restrict__ grid = nullptr,
                                                       h2v* __restrict__ grid_grad = nullptr,
                                                       float4* __restrict__ gpos = nullptr,
                                                       uint32_t* __restrict__ gdy = nullptr, int64_t bcap = 0) {
    constexpr int KK0 = ENC == 1 ? 4 : 5;
    constexpr int NBF = ENC == 1 ? kBwdFragsHash : kBwdFrags;
    constexpr int SLAB = slab_floats(ENC);
    int nst = 0;
    auto stamp = [&]() {
        if (STAMP) {
            __builtin_amdgcn_sched_barrier(0);
            const uint64_t tt = __builtin_amdgcn_s_memtime();
            __builtin_amdgcn_sched_barrier(0);
            if (threadIdx.x == 0) stamps[blockIdx.x * 16 + nst] = tt;
            ++nst;
        }
    };
    stamp();
    __shared__ __attribute__((aligned(16))) char smem[kLdsTrain];
    h8* lwf = (h8*)smem;
    h8* lwb = (h8*)(smem + kLdsWf);
    // double-buffered [sample][feature] images: buffer p holds (delta_l, a_l) for layers l with l & 1 == p
    char* img_a[2] = {smem + kLdsWf + kLdsWb, smem + kLdsWf + kLdsWb + kLdsImg};
    char* img_d[2] = {smem + kLdsWf + kLdsWb + 2 * kLdsImg, smem + kLdsWf + kLdsWb + 3 * kLdsImg};
    char* img_xh = smem + kLdsWf + kLdsWb + 4 * kLdsImg;
    float* red = (float*)(img_xh + kLdsXhi);

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, r = lane & 31;
    const int sl = wave * 32 + r;
    const TrOffs to = make_tr_offs(lane);
    const int64_t s = (int64_t)blockIdx.x * kTrainSamplesPerBlock + sl;
    const bool valid = s < b;
    const int64_t sc = valid ? s : b - 1;
    const QLane Q = load_q_enc<ENC, PADQ>(q, sc, h);
    float tgt[3] = {0.f, 0.f, 0.f};
    if (h == 0) {
        tgt[0] = t[sc * 3 + 0];
        tgt[1] = t[sc * 3 + 1];
        tgt[2] = t[sc * 3 + 2];
    }
    // weight images: the sample loads go first, then every weight load; the forward images are stored to LDS
    // after the encoder, the backward images only after the forward pass (their transfer overlaps it)
    constexpr int PF = (kFwdFrags * 64 + 255) / 256, PB = (NBF * 64 + 255) / 256;
    h8 vf[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) {
        const int i = threadIdx.x + k * 256;
        if (i < kFwdFrags * 64) vf[k] = wf[i];
    }
    h8 vb[PB];
#pragma unroll
    for (int k = 0; k < PB; ++k) {
        const int i = threadIdx.x + k * 256;
        if (i < NBF * 64) vb[k] = wb[i];
    }
    auto wfrag = [&](int i) { return lwb[i * 64 + lane]; };
    if constexpr (STAMP) {  // diagnostic: wait for the sample loads here, so the encoder is timed on its own
        asm volatile("" ::"v"(Q.p0), "v"(Q.p1), "v"(Q.p2), "v"(Q.b0), "v"(Q.b1), "v"(Q.b2), "v"(Q.i0), "v"(Q.i1),
                     "v"(Q.i2));
        stamp();
    }
    h8 x[KK0];
    static_assert(!PADQ || ENC == 1, "train_kernel: padded queries for the Hash encoding");
    if constexpr (ENC == 1) encode_hash<PADQ>(Q, h, grid, x);
    else if constexpr (ENC == 2) encode_sh(Q, h, x);
    else encode_fast(Q, h, x);
    // pin the encoder here (the asm consumes x) and keep the image stores and their vmcnt waits behind it, so
    // the encoder overlaps the weight loads instead of being sunk past the barrier
#pragma unroll
    for (int kk = 0; kk < KK0; ++kk) asm volatile("" : "+v"(x[kk]));
    __builtin_amdgcn_sched_barrier(0);
    stamp();
#pragma unroll
    for (int k = 0; k < PF; ++k) {
        const int i = threadIdx.x + k * 256;
        if (i < kFwdFrags * 64) lwf[i] = vf[k];
    }
    lds_barrier();  // forward weight images in LDS
    stamp();

    h8 a[5][4];
    {
        lds_h8* wl = (lds_h8*)(lwf + lane);
        h8 w0[2][KK0];
        load_frags<KK0>(wl, 0, w0);
        h8 xx[1][KK0];
#pragma unroll
        for (int kk = 0; kk < KK0; ++kk) xx[0][kk] = x[kk];
        h8 yy[1][4];
        layer_mfma<1, KK0>(w0, xx, yy);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) a[0][kk] = yy[0][kk];
#pragma unroll
        for (int l = 1; l < 5; ++l) {
            h8 wlay[2][4];
            load_frags<4>(wl, l, wlay);
            h8 in[1][4] = {{a[l - 1][0], a[l - 1][1], a[l - 1][2], a[l - 1][3]}};
            layer_mfma<1, 4>(wlay, in, yy);
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) a[l][kk] = yy[0][kk];
        }
    }
    const f16v o = mlp_out(lwf, a[4], lane);
#pragma unroll
    for (int k = 0; k < PB; ++k) {
        const int i = threadIdx.x + k * 256;
        if (i < NBF * 64) lwb[i] = vb[k];
    }
    stamp();

    // RelativeL2Luminance on the f16 prediction, loss-scaled f16 gradient, ReLU-masked.
    float lossv = 0.0f;
    h8 g[4] = {h8{}, h8{}, h8{}, h8{}};
    if (h == 0) {
        float y[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) y[c] = (float)(_Float16)fmaxf(o[c], 0.0f);
        const float lum = 0.299f * y[0] + 0.587f * y[1] + 0.114f * y[2];
        const float denom = lum * lum + NRC_LUM_EPS;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float diff = y[c] - tgt[c];
            const float lv = diff * diff / denom / n_total;
            const float gv = loss_scale * 2.0f * diff / denom / n_total;
            lossv += valid ? lv : 0.0f;
            g[0][c] = (valid && y[c] > 0.0f) ? (_Float16)gv : (_Float16)0.0f;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) lossv += __shfl_xor(lossv, off);
    if (lane == 0) red[wave] = lossv;

    float* slab = slabs + (int64_t)blockIdx.x * SLAB;

    // layer 5 operands (buffer 1): delta_5 = g (16 rows, k-step 0 only), a_5
    *(h8*)(img_d[1] + img_off(sl, acc_row(0, h, 0))) = g[0];
    write_rows64(img_a[1], sl, h, a[4]);
    lds_barrier();
    if (threadIdx.x == 0) loss_partials[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
    stamp();

    // One barrier per layer: step l reads buffer l&1 and writes layer l-1's operands into the other
    // buffer, whose previous readers (step l+1) all passed the barrier that ended step l+1. The dW GEMM of
    // layer l comes first in program order: its operand reads are independent of the delta chain, so the
    // compiler can interleave the two MFMA streams without an LDS write in between.
    h8 d4[4], d3[4], d2[4], d1[4], d0[4];
    {
        DwAcc<5, ENC> dw;
        h8 wbf[2][4];
        load_bwd<5>(wfrag, wbf);
        dw.mfma_all(img_d[1], img_a[1], img_xh, wave, lane, to);
        bwd_chain_pre<5>(wbf, g, a[4], d4);
        write_rows64(img_d[0], sl, h, d4);
        write_rows64(img_a[0], sl, h, a[3]);
        dw.store_all(wave, lane, slab);
    }
    lds_barrier();
    stamp();
    {
        DwAcc<4, ENC> dw;
        h8 wbf[2][4];
        load_bwd<4>(wfrag, wbf);
        dw.mfma_all(img_d[0], img_a[0], img_xh, wave, lane, to);
        bwd_chain_pre<4>(wbf, d4, a[3], d3);
        write_rows64(img_d[1], sl, h, d3);
        write_rows64(img_a[1], sl, h, a[2]);
        dw.store_all(wave, lane, slab);
    }
    lds_barrier();
    stamp();
    {
        DwAcc<3, ENC> dw;
        h8 wbf[2][4];
        load_bwd<3>(wfrag, wbf);
        dw.mfma_all(img_d[1], img_a[1], img_xh, wave, lane, to);
        bwd_chain_pre<3>(wbf, d3, a[2], d2);
        write_rows64(img_d[0], sl, h, d2);
        write_rows64(img_a[0], sl, h, a[1]);
        dw.store_all(wave, lane, slab);
    }
    lds_barrier();
    stamp();
    {
        DwAcc<2, ENC> dw;
        h8 wbf[2][4];
        load_bwd<2>(wfrag, wbf);
        dw.mfma_all(img_d[0], img_a[0], img_xh, wave, lane, to);
        bwd_chain_pre<2>(wbf, d2, a[1], d1);
        write_rows64(img_d[1], sl, h, d1);
        write_rows64(img_a[1], sl, h, a[0]);
        dw.store_all(wave, lane, slab);
    }
    lds_barrier();
    stamp();
    DwAcc<1, ENC> dw1;
    h8 wbf[2][4];
    load_bwd<1>(wfrag, wbf);
    dw1.mfma_all(img_d[1], img_a[1], img_xh, wave, lane, to);
    bwd_chain_pre<1>(wbf, d1, a[0], d0);
    // layer-0 operands: delta_0 and the encoded input x (K order; x_lo -> img_a[0], x_hi -> img_xh)
    write_rows64(img_d[0], sl, h, d0);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int jg = 0; jg < 2; ++jg) store_h4(img_a[0], img_off(sl, 16 * kk + 8 * h + 4 * jg), x[kk], 4 * jg);
    if constexpr (ENC != 1) *(h8*)(img_xh + sl * 32 + 16 * h) = x[KK0 - 1];
    // Grid gradient (Hash): dL/d(grid feature 16h + r) = (W0^T delta_0)[.] for sample s. The trilinear scatter of
    // tcnn's kernel_grid_backward (grad[entry][f] += w_corner * dy_f) runs afterwards in grid_scatter_kernel: here
    // each sample leaves its position and its 16 levels' (dy0, dy1) as f16 pairs, level-major [level][sample]
    // (zeros for the padding samples).
    if constexpr (ENC == 1) {
        f16v c = zero16();
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) c = mfma(wfrag(kBwdFrags + kk), d0[kk], c);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const h2v dv = {valid ? (_Float16)c[2 * i] : (_Float16)0.0f, valid ? (_Float16)c[2 * i + 1] : (_Float16)0.0f};
            gdy[(int64_t)(8 * h + i) * bcap + s] = __builtin_bit_cast(uint32_t, dv);
        }
        if (h == 0) gpos[s] = float4{Q.p0, Q.p1, Q.p2, 0.0f};
    }
    dw1.store_all(wave, lane, slab);
    lds_barrier();
    stamp();
    {
        DwAcc<0, ENC> dw0;
        dw0.mfma_all(img_d[0], img_a[0], img_xh, wave, lane, to);
        dw0.store_all(wave, lane, slab);
    }
    stamp();
}

// ------------------------------------------------------------------------------------------------
// Fixed-order weight-gradient reduction + tcnn Adam + EMA + f16 fragment-image repack.
// ------------------------------------------------------------------------------------------------
// Block = 16 lanes x float4 = 64 parameters x 16 slab groups (352 blocks for the Frequency config, so the
// whole chip shares the 11.5 MB of slabs); each thread sums every 16th slab with all of its loads in flight,
// the groups are combined in LDS in a fixed tree: the result is bitwise reproducible for a given slab count.
constexpr int kRedParams = 16, kRedGroups = 16, kRedThreads = kRedParams * kRedGroups;
constexpr int kRedVec = 4;  // floats per thread: one 16-byte load per slab
static_assert(NRC_NUM_PARAMS % (kRedParams * 4) == 0 && NRC_HASH_MLP_PARAMS % (kRedParams * 4) == 0 &&
                  slab_floats(0) % (kRedParams * 4) == 0 && slab_floats(1) % (kRedParams * 4) == 0,
              "parameter counts and slab sizes must tile the reduction");

__device__ __forceinline__ void adam_pack_one(int mode, int p, float gsum, const ModelBuffers& mb, const OptimArgs& oa,
                                              float lr_t, float ema_debias) {
#pragma clang fp contract(off)
    float w, inf;
    if (mode == kPackOnly) {
        w = mb.params[p];
        inf = mb.infer[p];
    } else {
        // tcnn Adam (optimizers/adam.h); lr_t and the EMA debias come from the host in f32.
        float gradient = gsum / oa.loss_scale;
        w = mb.params[p];
        gradient += oa.l2_reg * w;
        const float gsq = gradient * gradient;
        const float m1 = oa.beta1 * mb.m[p] + (1.0f - oa.beta1) * gradient;
        const float v1 = oa.beta2 * mb.v[p] + (1.0f - oa.beta2) * gsq;
        mb.m[p] = m1;
        mb.v[p] = v1;
        const float eff = lr_t / (sqrtf(v1) + oa.eps);
        w = w - eff * m1;
        mb.params[p] = w;
        const float e = mb.ema[p] * oa.ema_decay + w * (1.0f - oa.ema_decay);
        mb.ema[p] = e;
        inf = e / ema_debias;
        mb.infer[p] = inf;
    }
    mb.wf_train[mb.fwdt_pos[p]] = (_Float16)w;
    mb.wf_infer[mb.fwd_pos[p]] = (_Float16)inf;
    if (mb.wf_infer16) mb.wf_infer16[mb.fwdt_pos[p]] = (_Float16)inf;
    const int bp = mb.bwd_pos[p];
    if (bp >= 0) mb.wb_train[bp] = (_Float16)w;
}

// Sum of the loss partials p[lane], p[lane + 64], ... (in that order) for one wave: the loads of each batch of 8 issue
// together (branch-free: clamped index, masked add), instead of one round trip per partial
__device__ __forceinline__ float lane_partial_sum(const float* __restrict__ p, int n, int lane) {
    float L = 0.0f;
    for (int base = lane; base < n; base += 8 * 64) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[min(base + 64 * u, n - 1)];
#pragma unroll
        for (int u = 0; u < 8; ++u) L += base + 64 * u < n ? v[u] : 0.0f;
    }
    return L;
}

// The per-slab loss partials are summed by wave 0 of block 0: a strided per-lane sum and a fixed xor
// butterfly (one load latency instead of a serial chain of nslabs loads).
// H: f16 slabs (the t16 training kernel's), converted to f32 before the same fixed-order f32 sums
template <bool H>
__device__ __forceinline__ void reduce_adam_body(const int blk, int mode, const float* __restrict__ slabs, int nslabs,
                                                 const float* __restrict__ loss_partials, float* __restrict__ grad_io,
                                                 float* __restrict__ loss_out, const ModelBuffers& mb,
                                                 const OptimArgs& oa, float lr_t, float ema_debias) {
#pragma clang fp contract(off)
    typedef float f4 __attribute__((ext_vector_type(4)));
    __shared__ f4 part[kRedGroups][kRedParams];
    const int pl = threadIdx.x & (kRedParams - 1), grp = threadIdx.x / kRedParams;
    const int p0 = (blk * kRedParams + pl) * kRedVec;  // slab position (reduce modes) / parameter (apply, pack)
    // diagnostic build: per-block s_memrealtime stamps of thread 0 (entry, slab sums done, after the combine barrier,
    // Adam issued) in g_infer_clock, read back by nrc_debug_read_infer_clock (tools/reduce_stamps.py)
    auto stamp = [&](int k) {
#if NRC_DEBUG_KERNELS
        if (threadIdx.x == 0 && mode == kReduceFused && blk < kInferClockWavesMax)
            g_infer_clock[6 * blk + k] = __builtin_amdgcn_s_memrealtime();
        if (k == 0 && threadIdx.x == 0 && mode == kReduceFused && blk < kInferClockWavesMax) {
            g_infer_clock[6 * blk + 4] = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
            g_infer_clock[6 * blk + 5] = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);
        }
#else
        (void)k;
#endif
    };
    stamp(0);
    if (blk == 0 && threadIdx.x < 64) {
        if (mode == kReduceFused || mode == kReduceOnly) {
            float L = 0.0f;
            L = lane_partial_sum(loss_partials, nslabs, threadIdx.x);
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) L += __shfl_xor(L, off, 64);
            if (threadIdx.x == 0) {
                if (mode == kReduceOnly) grad_io[mb.n_total] = L;
                else if (loss_out) loss_out[0] = L;
            }
        } else if (mode == kApplyOnly && loss_out && threadIdx.x == 0) {
            loss_out[0] = grad_io[mb.n_total];
        }
    }
    if (mode == kReduceFused || mode == kReduceOnly) {
        // Load order (round 3): the parameter-map load, then the first batch of up to 8 slab loads, then the Adam
        // state of the mapped parameter -- so that the slab loads do not wait a round trip for the map (the in-order
        // vmcnt lets the map's value be used with the slab loads still in flight), and a short last batch is issued
        // in one go (the remainder used to be a serial loop: 4 round trips for the 64 slabs of a 2,048-sample step).
        // the slab position this thread combines (threads < 64): t16 slabs map it in closed form, the 32x32 slabs
        // through the map (one branch-free load, every thread)
        const int mypos = blk * kRedParams * kRedVec + (threadIdx.x & (kRedParams * kRedVec - 1));
        int pp_raw;
        if constexpr (H) pp_raw = mb.slab_closed == 2 ? t16_hash_slab_param(mypos) : t16_slab_param(mypos);
        else pp_raw = mb.slab_param[mypos];
        f4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
        auto ld = [&](int slab) -> f4 {
            if constexpr (H) {
                const h4 v = *(const h4*)((const _Float16*)slabs + (int64_t)slab * mb.n_slab + p0);
                return f4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
            } else {
                return *(const f4*)&slabs[(int64_t)slab * mb.n_slab + p0];
            }
        };
        // slabs grp, grp + G, ... (G = kRedGroups), in batches of 8 loads; element k of the sequence goes to a0 for
        // even k, a1 for odd k (the same float sums as the round-2 loop)
        // loads are branch-free (a slab index past the last is clamped to it and its value not added): a load under a
        // branch made the compiler wait for it at the join
        const int nmine = grp < nslabs ? (nslabs - grp + kRedGroups - 1) / kRedGroups : 0;
        auto ldc = [&](int k) -> f4 { return ld(min(grp + k * kRedGroups, nslabs - 1)); };
        // the combining threads' Adam state first (t16: its address needs no load), then the slabs: all in flight at once
        const int pp = threadIdx.x < kRedParams * kRedVec ? pp_raw : -1;
        AdamIn ain{};
        if (mode == kReduceFused && pp >= 0) ain = adam_load(pp, mb);
        f4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = ldc(u);
        // the image positions are first used here: otherwise the compiler computes the 64-bit store addresses right
        // after their loads and waits for them before issuing the slab loads
        asm volatile("" : "+v"(ain.fp), "+v"(ain.ft), "+v"(ain.bp));
        for (int base = 0;;) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const bool in = base + u < nmine;
                if (u & 1) a1 += in ? v[u] : f4{0.f, 0.f, 0.f, 0.f};
                else a0 += in ? v[u] : f4{0.f, 0.f, 0.f, 0.f};
            }
            base += 8;
            if (base >= nmine) break;
            // plain loads (0.4 us per step faster than nontemporal ones here)
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = ldc(base + u);
        }
        part[grp][pl] = a0 + a1;
        stamp(1);
        __syncthreads();
        stamp(2);
        // one parameter per thread for the combine + Adam (threads 0..63 of the block)
        if (threadIdx.x >= kRedParams * kRedVec) return;
        const int lp = threadIdx.x / kRedVec, comp = threadIdx.x % kRedVec;
        float t8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t8[u] = part[2 * u][lp][comp] + part[2 * u + 1][lp][comp];
        const float g1 = ((t8[0] + t8[1]) + (t8[2] + t8[3])) + ((t8[4] + t8[5]) + (t8[6] + t8[7]));
        const int p = pp;
        if (p < 0) return;  // padding position (x_hi block lanes past the 80 inputs)
        if (mode == kReduceOnly) {
            grad_io[p] = g1;
            return;
        }
        adam_pack_pre(p, g1, ain, mb, oa, lr_t, ema_debias);
        stamp(3);
        return;
    }
    if (threadIdx.x >= kRedParams * kRedVec) return;
    const int p = blk * kRedParams * kRedVec + threadIdx.x;
    adam_pack_one(mode, p, mode == kApplyOnly ? grad_io[p] : 0.0f, mb, oa, lr_t, ema_debias);
}

template <bool H>
__global__ __launch_bounds__(kRedThreads) void reduce_adam_kernel(int mode, const float* __restrict__ slabs, int nslabs,
                                                          const float* __restrict__ loss_partials,
                                                          float* __restrict__ grad_io, float* __restrict__ loss_out,
                                                          ModelBuffers mb, OptimArgs oa, float lr_t, float ema_debias) {
    reduce_adam_body<H>(blockIdx.x, mode, slabs, nslabs, loss_partials, grad_io, loss_out, mb, oa, lr_t, ema_debias);
}

// ------------------------------------------------------------------------------------------------
// Width-128 training step (BASELINE configs[4]; oracle/nrc_wide_oracle.c orc_wide_grad + orc_adam_ema):
//   wide_fwd_bwd_lds_kernel  two waves (64 samples) per block: encode, forward (f16 MFMA chain, A fragments from the
//                        LDS-staged training images), RelativeL2Luminance, delta chain through W_l^T; stores every
//                        layer's input and delta as f16 [feature][sample] rows of a workspace (row stride wide_ld);
//   wide_dw_kernel       dW_l = sum_s delta_l in_l^T as 32x32 tiles x 512-sample chunks (A and B fragments are
//                        16-byte loads of those rows), partial sums per chunk in canonical parameter order;
//   wide_adam_pack_kernel fixed-order chunk sum + tcnn Adam + EMA per parameter (same float operations as
//                        adam_pack_one) and, in the same launch, every f16 / FP8 weight image.
// ------------------------------------------------------------------------------------------------
// f16 B fragments (rows acc_row(kk, h, j), sample s) -> ws[row * ld + s] with 4-byte stores: adjacent lanes
// (samples 2p, 2p + 1) swap half of their 8 rows (one DPP quad_perm [1,0,3,2] per dword), so each lane holds 4 rows x
// 2 samples and writes 4 words instead of 8 halves (wide_fwd_bwd_lds_kernel 67.4 -> 64.4 us per training step in
// A/B; 8-byte stores after a second exchange with lane ^ 2: 65.1)
__device__ __forceinline__ void store_frag_rows(_Float16* __restrict__ ws, int64_t ld, int64_t s, int h,
                                                const h8 (&y)[8]) {
    const bool odd = threadIdx.x & 1;
    const int64_t s0 = s & ~(int64_t)1;
    const int jb = odd ? 4 : 0;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
        const u4 d = __builtin_bit_cast(u4, y[kk]);  // (j0, j1), (j2, j3), (j4, j5), (j6, j7)
        const uint32_t give0 = odd ? d.x : d.z, give1 = odd ? d.y : d.w;
        const uint32_t keep0 = odd ? d.z : d.x, keep1 = odd ? d.w : d.y;
        const uint32_t got0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)give0, 0xB1, 0xF, 0xF, false);
        const uint32_t got1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)give1, 0xB1, 0xF, 0xF, false);
        // sample s0 in the low half of each word, s0 + 1 in the high half
        const uint32_t lo0 = odd ? got0 : keep0, hi0 = odd ? keep0 : got0;
        const uint32_t lo1 = odd ? got1 : keep1, hi1 = odd ? keep1 : got1;
        const uint32_t w[4] = {__builtin_amdgcn_perm(hi0, lo0, 0x05040100u), __builtin_amdgcn_perm(hi0, lo0, 0x07060302u),
                               __builtin_amdgcn_perm(hi1, lo1, 0x05040100u), __builtin_amdgcn_perm(hi1, lo1, 0x07060302u)};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t* const dst = reinterpret_cast<uint32_t*>(ws + (int64_t)acc_row(kk, h, jb + i) * ld + s0);
#if defined(NRC_WIDE_PLAIN_STORES)
            *dst = w[i];
#else
            __hip_atomic_store(dst, w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1, as the slab stores
#endif
        }
    }
}

// Copy COUNT h8 (1-KiB fragments of 64 lanes) global -> LDS with LDS-DMA (global_load_lds_dwordx4: no VGPRs, all
// of a thread's copies in flight at once); fragment c goes to wave c % W's instruction c / W. The caller waits
// (s_waitcnt vmcnt(0)) and synchronises before reading.
template <int W, int FRAGS>
__device__ __forceinline__ void dma_frags_to_lds(h8* lds, const h8* __restrict__ src) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
#pragma unroll 4
    for (int c = wave; c < FRAGS; c += W)
        __builtin_amdgcn_global_load_lds((const void*)(src + c * 64 + lane),
                                         (__attribute__((address_space(3))) void*)(lds + c * 64), 16, 0, 0);
}

// Width-128 forward + loss + delta chain, the weight images staged in LDS: a block of 2 waves (64 samples, one wave
// per 32) per CU stages the 156-KiB forward image by LDS-DMA, encodes, runs the forward pass and the loss, then
// stages the 132-KiB backward image over it for the delta chain. Every layer's input and delta go to the workspace
// as f16 [feature][sample] rows for wide_dw_kernel. (The first version ran one wave per block and read every A
// fragment from L2 -- 288 KiB per wave, a round trip per layer: 39.5 us per 16,384-sample step; this one 26.5 us.)
template <int ENC>
__global__ __launch_bounds__(128, 1) void wide_fwd_bwd_lds_kernel(const float* __restrict__ q,
                                                                  const float* __restrict__ t, int64_t b,
                                                                  int64_t bpad, int64_t ld, float n_total,
                                                                  float loss_scale, const h8* __restrict__ wf,
                                                                  const h8* __restrict__ wb,
                                                                  _Float16* __restrict__ ws_in,
                                                                  _Float16* __restrict__ ws_d,
                                                                  float* __restrict__ loss_partials) {
    __shared__ __attribute__((aligned(16))) h8 lw[kWideF16Bytes / 16];
    static_assert(kWideBwdBytes <= kWideF16Bytes, "backward image reuses the forward image's LDS");
    dma_frags_to_lds<2, kWideF16Frags>(lw, wf);
    fp32_flush_output_denorms();  // the omod doubling-chain encoder (as the inference kernels)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, r = lane & 31;
    const int64_t tile = (int64_t)blockIdx.x * 2 + wave;
    const bool live = tile * 32 < bpad;        // the last block's second wave may have no samples (bpad % 64 == 32)
    const int64_t s = tile * 32 + r;           // < bpad + 32 <= ld: a dead wave's stores land in the row padding
    const bool valid = s < b;
    const int64_t sc = valid ? s : b - 1;
    const QLane Q = load_q_enc<ENC>(q, sc, h);
    float tgt[3] = {0.f, 0.f, 0.f};
    if (h == 0) {
        tgt[0] = t[sc * 3 + 0];
        tgt[1] = t[sc * 3 + 1];
        tgt[2] = t[sc * 3 + 2];
    }
    h8 x[5];
    if constexpr (ENC == 2) encode_sh<true>(Q, h, x);
    else encode_v3(Q, h, x);  // the inference kernel's encoder (round 6)
#pragma unroll
    for (int kk = 0; kk < 5; ++kk)
#pragma unroll
        for (int j = 0; j < 8; ++j) ws_in[(int64_t)enc_k0_feature(ENC, 16 * kk + 8 * h + j) * ld + s] = x[kk][j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    h8 a[5][8];
    f16v c[4];
    {
        lds_h8* wl = launder((lds_h8*)(lw + lane));
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) c[mb] = zero16();
#pragma unroll
        for (int kk = 0; kk < 5; ++kk)
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) c[mb] = mfma(wl[wide_frag(0, mb, kk) * 64], x[kk], c[mb]);
    }
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) a[0][kk] = relu_h8(c[kk >> 1], 8 * (kk & 1));
    store_frag_rows(ws_in + wide_in_row(1) * ld, ld, s, h, a[0]);
#pragma unroll
    for (int l = 1; l < 5; ++l) {
        lds_h8* wl = launder((lds_h8*)(lw + lane));
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) c[mb] = zero16();
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) c[mb] = mfma(wl[wide_frag(l, mb, kk) * 64], a[l - 1][kk], c[mb]);
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) a[l][kk] = relu_h8(c[kk >> 1], 8 * (kk & 1));
        store_frag_rows(ws_in + wide_in_row(l + 1) * ld, ld, s, h, a[l]);
    }
    f16v o = zero16();
    {
        lds_h8* wl = launder((lds_h8*)(lw + lane));
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) o = mfma(wl[wide_frag(5, 0, kk) * 64], a[4][kk], o);
    }
    // every wave is past its last forward-image read: stage the backward image while the loss is computed
    __syncthreads();
    dma_frags_to_lds<2, kWideBwdFrags>(lw, wb);

    // RelativeL2Luminance on the f16 prediction, loss-scaled f16 gradient, ReLU-masked (as train_kernel)
    float lossv = 0.0f;
    h8 g = {};
    if (h == 0) {
        float y[3];
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) y[cc] = (float)(_Float16)fmaxf(o[cc], 0.0f);
        const float lum = 0.299f * y[0] + 0.587f * y[1] + 0.114f * y[2];
        const float denom = lum * lum + NRC_LUM_EPS;
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) {
            const float diff = y[cc] - tgt[cc];
            const float lv = diff * diff / denom / n_total;
            const float gv = loss_scale * 2.0f * diff / denom / n_total;
            lossv += valid ? lv : 0.0f;
            g[cc] = (valid && y[cc] > 0.0f) ? (_Float16)gv : (_Float16)0.0f;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) lossv += __shfl_xor(lossv, off);
    if (lane == 0 && live) loss_partials[tile] = lossv;
#pragma unroll
    for (int j = 0; j < 8; ++j) ws_d[(wide_d_row(5) + acc_row(0, h, j)) * ld + s] = g[j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // delta chain: d_{l-1} = relu'(a_{l-1}) (W_l^T d_l); accumulator block mb regs 0-7 / 8-15 are the rows of the
    // B fragments 2 mb / 2 mb + 1, so the gate takes the activation fragments as they are
    h8 d[8];
    {
        lds_h8* bl = launder((lds_h8*)(lw + lane));
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) c[mb] = mfma(bl[wide_bwd_frag(5, mb, 0) * 64], g, zero16());
    }
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) mask_pack_pk(c[mb], a[4][2 * mb], a[4][2 * mb + 1], d[2 * mb], d[2 * mb + 1]);
    store_frag_rows(ws_d + wide_d_row(4) * ld, ld, s, h, d);
#pragma unroll
    for (int l = 4; l >= 1; --l) {
        lds_h8* bl = launder((lds_h8*)(lw + lane));
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) c[mb] = zero16();
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) c[mb] = mfma(bl[wide_bwd_frag(l, mb, kk) * 64], d[kk], c[mb]);
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
            mask_pack_pk(c[mb], a[l - 1][2 * mb], a[l - 1][2 * mb + 1], d[2 * mb], d[2 * mb + 1]);
        store_frag_rows(ws_d + wide_d_row(l - 1) * ld, ld, s, h, d);
    }
}

// dW_l = sum_s delta_l in_l^T per (layer, chunk of kWideChunk samples): one block of 4 waves per pair, 6 layers x
// nchunks blocks. The chunk's input rows (<= 128 rows x 512 samples f16 = 128 KiB) are staged in LDS by LDS-DMA, each
// 1-KiB row's 16-byte slots XOR-swizzled by the row (slot s of row i at s ^ (i & 31): the 32 lanes of a B-fragment read
// hit 32 distinct slots); wave w holds the delta rows 32 w .. 32 w + 31 of the chunk in registers (A operands, all 32
// k steps loaded at once) and computes the row block's 32x32 tiles against every 32-row block of the inputs (layer 5:
// 16 delta rows, wave w takes input block w). Every load of the block is in flight at once: one memory round trip per
// block instead of one per 8 k steps (round 2's wave-per-tile kernel: 23.9 us per 16,384-sample step, every input row
// read from L2 by 4 waves). Partial sums per chunk in canonical parameter order, written through (sc1).
constexpr int kWideChunk = 512;
__global__ __launch_bounds__(256, 1) void wide_dw_kernel(const _Float16* __restrict__ ws_in, const _Float16* __restrict__ ws_d,
                                                         int64_t bpad, int64_t ld, int nchunks, float* __restrict__ slabs) {
    constexpr int KS = kWideChunk / 16;  // k steps per chunk
    __shared__ __attribute__((aligned(16))) h8 lb[128 * (kWideChunk / 8)];
    const int layer = blockIdx.x % 6, chunk = blockIdx.x / 6;
    if (chunk >= nchunks) return;
    const int in_dim = layer == 0 ? NRC_ENC_WIDTH : 128, out_dim = layer == 5 ? NRC_OUT_PADDED : 128;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, h = lane >> 5, r = lane & 31;
    const int64_t k0 = (int64_t)chunk * kWideChunk;
    const int nk = (int)min<int64_t>(KS, (bpad - k0) / 16);  // bpad % 32 == 0
    // input rows -> LDS: one DMA instruction per row (64 lanes x 16 B), lane L fetches the slot that lands at L
    for (int i = wave; i < in_dim; i += 4) {
        const int src_slot = lane ^ (i & 31);
        if (src_slot < 2 * nk)
            __builtin_amdgcn_global_load_lds((const void*)(ws_in + (wide_in_row(layer) + i) * ld + k0 + 8 * src_slot),
                                             (__attribute__((address_space(3))) void*)(lb + i * (kWideChunk / 8)), 16, 0, 0);
    }
    // delta rows -> registers
    const int mb = layer == 5 ? 0 : wave;
    const int o = 32 * mb + r;
    const bool oa = o < out_dim;
    const h8* pa = reinterpret_cast<const h8*>(ws_d + (wide_d_row(layer) + (oa ? o : 0)) * ld + k0 + 8 * h);
    const h8 z = {};
    h8 A[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) A[ks] = (oa && ks < nk) ? pa[2 * ks] : z;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int nb0 = layer == 5 ? wave : 0, nb1 = layer == 5 ? wave + 1 : (in_dim + 31) / 32;
    lds_h8* lbl = launder((lds_h8*)lb);
    for (int nb = nb0; nb < nb1; ++nb) {
        f16v acc = zero16();
        const int i = 32 * nb + r;  // this lane's B column (input row); rows past in_dim read stale LDS, never stored
        lds_h8* row = lbl + i * (kWideChunk / 8);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
            if (ks < nk) acc = mfma(A[ks], row[(2 * ks + h) ^ r], acc);
        if (i >= in_dim) continue;
        float* slab = slabs + (int64_t)chunk * NRC_WIDE_NUM_PARAMS + wide_off(layer);
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int orow = 32 * mb + (reg & 3) + 8 * (reg >> 2) + 4 * h;
            // sc1: written through, not left dirty in this XCD's L2 (wide_adam_pack_kernel reads the chunks on every XCD)
            if (orow < out_dim)
                __hip_atomic_store(&slab[orow * in_dim + i], acc[reg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Width-128 optimizer step with every weight image packed in the same launch (round 3; replaced wide_adam_kernel +
// wide_pack_all_kernel, 6.3 + 9.5 us per step: the pack's FP8 part was 17 waves each gathering 64 scattered weights).
// One row of one layer per 32 lanes, 4 consecutive parameters per lane (16-byte loads / stores of the f32 arrays):
//   modes kReduceFused / kReduceOnly: the chunk partials summed in chunk order (as the oracle's f32 loop); kApplyOnly: the
//   all-reduced gradient; then tcnn Adam + EMA, the same float operations as adam_pack_one (kReduceOnly stops at the sum);
//   kPackOnly: no step, the images from the current params / infer;
//   images: f16 inference image (img16, and img8's f16 layer-0 fragments) from the debiased EMA weights, training
//   forward (fwd16) and backward W_l^T (bwd16) images from the master weights, and the FP8 image with its per-row E8M0
//   exponent: max |w| of the row is a max over the row's 32 lanes (orc_fp8_row_exponent).
// The loss partials are summed by wave 0 of block 0.
struct K0Inverse {
    int8_t k[2][NRC_ENC_WIDTH];  // [FrequencySH][canonical feature] -> layer-0 K slot
};
constexpr K0Inverse make_k0_inverse() {
    K0Inverse t{};
    for (int e = 0; e < 2; ++e)
        for (int K = 0; K < NRC_ENC_WIDTH; ++K) t.k[e][enc_k0_feature(e ? 2 : 0, K)] = (int8_t)K;
    return t;
}
__constant__ K0Inverse kK0Inv = make_k0_inverse();
constexpr int kWideRowUnits = 128 + 4 * 128 + 32;  // layer 0, layers 1-4, layer 5 incl. the 16 zero rows of its images

__global__ __launch_bounds__(256) void wide_adam_pack_kernel(int mode, const float* __restrict__ slabs, int nchunks,
                                                             const float* __restrict__ loss_partials, int nlp,
                                                             float* __restrict__ grad_io, float* __restrict__ loss_out,
                                                             ModelBuffers mb, OptimArgs oa, float lr_t, float ema_debias,
                                                             WideImages im) {
#pragma clang fp contract(off)
    typedef float f4 __attribute__((ext_vector_type(4)));
    if (blockIdx.x == 0 && threadIdx.x < 64) {
        if (mode == kReduceFused || mode == kReduceOnly) {
            float L = 0.0f;
            L = lane_partial_sum(loss_partials, nlp, threadIdx.x);
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) L += __shfl_xor(L, off, 64);
            if (threadIdx.x == 0) {
                if (mode == kReduceOnly) grad_io[mb.n_total] = L;
                else if (loss_out) loss_out[0] = L;
            }
        } else if (mode == kApplyOnly && loss_out && threadIdx.x == 0) {
            loss_out[0] = grad_io[mb.n_total];
        }
    }
    const int unit = (int)((blockIdx.x * 256u + threadIdx.x) >> 5), c4 = threadIdx.x & 31;
    if (unit >= kWideRowUnits) return;  // whole half-waves
    const int layer = unit < 128 ? 0 : unit < 640 ? 1 + (unit - 128) / 128 : 5;
    const int row = unit < 128 ? unit : unit < 640 ? (unit - 128) % 128 : unit - 640;
    const int in_dim = layer == 0 ? NRC_ENC_WIDTH : 128, c = 4 * c4;
    const bool live = (layer < 5 || row < NRC_OUT_PADDED) && c < in_dim;
    const int p = wide_off(layer) + row * in_dim + c;  // this lane's first parameter
    f4 w = {0.f, 0.f, 0.f, 0.f}, inf = {0.f, 0.f, 0.f, 0.f};
    if (live) {
        if (mode == kPackOnly) {
            w = *(const f4*)(mb.params + p);
            inf = *(const f4*)(mb.infer + p);
        } else {
            const f4 w0 = *(const f4*)(mb.params + p);
            f4 g = {0.f, 0.f, 0.f, 0.f}, m0 = {}, v0 = {}, e0 = {};
            if (mode != kReduceOnly) {
                m0 = *(const f4*)(mb.m + p);
                v0 = *(const f4*)(mb.v + p);
                e0 = *(const f4*)(mb.ema + p);
            }
            if (mode == kApplyOnly) {
                // the caller's all-reduced buffer: 4-byte aligned only
                for (int i = 0; i < 4; ++i) g[i] = grad_io[p + i];
            } else {
                // 16 chunk loads in flight per batch, summed in chunk order (+0 for absent chunks leaves the sum unchanged)
                for (int c0 = 0; c0 < nchunks; c0 += 16) {
                    f4 v[16];
#pragma unroll
                    for (int j = 0; j < 16; ++j)
                        v[j] = c0 + j < nchunks ? *(const f4*)(slabs + (int64_t)(c0 + j) * NRC_WIDE_NUM_PARAMS + p)
                                                : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int j = 0; j < 16; ++j) g += v[j];
                }
                if (mode == kReduceOnly) {
                    for (int i = 0; i < 4; ++i) grad_io[p + i] = g[i];
                    return;
                }
            }
            f4 m1, v1, e1;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float gradient = g[i] / oa.loss_scale;
                float wi = w0[i];
                gradient += oa.l2_reg * wi;
                const float gsq = gradient * gradient;
                m1[i] = oa.beta1 * m0[i] + (1.0f - oa.beta1) * gradient;
                v1[i] = oa.beta2 * v0[i] + (1.0f - oa.beta2) * gsq;
                const float eff = lr_t / (sqrtf(v1[i]) + oa.eps);
                wi = wi - eff * m1[i];
                w[i] = wi;
                e1[i] = e0[i] * oa.ema_decay + wi * (1.0f - oa.ema_decay);
                inf[i] = e1[i] / ema_debias;
            }
            *(f4*)(mb.m + p) = m1;
            *(f4*)(mb.v + p) = v1;
            *(f4*)(mb.params + p) = w;
            *(f4*)(mb.ema + p) = e1;
            *(f4*)(mb.infer + p) = inf;
        }
    } else if (mode == kReduceOnly) {
        return;
    }
    // ---- images
    const int mbk = row >> 5, r = row & 31;
    if (layer == 0) {
        if (c >= in_dim) return;
        for (int i = 0; i < 4; ++i) {
            const int K = kK0Inv.k[im.enc == 2][c + i];
            const int idx = (wide_frag(0, mbk, K >> 4) * 64 + r + 32 * ((K >> 3) & 1)) * 8 + (K & 7);
            im.img16[idx] = (_Float16)inf[i];
            reinterpret_cast<_Float16*>(im.img8)[idx] = (_Float16)inf[i];
            im.fwd16[idx] = (_Float16)w[i];
        }
        return;
    }
    {
        // forward layout: column c -> (k-step kk, lane half h, element j) of acc_row; 4 columns = 4 consecutive halves
        const int kk = ((c >> 5) << 1) | ((c >> 4) & 1), h = (c >> 2) & 1, j = ((c >> 3) & 1) * 4;
        const int idx = (wide_frag(layer, mbk, kk) * 64 + r + 32 * h) * 8 + j;
        const h4 hi = {(_Float16)inf[0], (_Float16)inf[1], (_Float16)inf[2], (_Float16)inf[3]};
        const h4 hw = {(_Float16)w[0], (_Float16)w[1], (_Float16)w[2], (_Float16)w[3]};
        *(h4*)(im.img16 + idx) = hi;
        *(h4*)(im.fwd16 + idx) = hw;
    }
    if (layer < 5 || row < NRC_OUT_PADDED) {
        // backward image W_l^T: element (row, col) at lane (col % 32, half (row >> 2) & 1) of fragment (col / 32, kk(row))
        const int kk = ((row >> 5) << 1) | ((row >> 4) & 1), h = (row >> 2) & 1, j = ((row >> 3) & 1) * 4 + (row & 3);
        for (int i = 0; i < 4; ++i) {
            const int col = c + i;
            im.bwd16[(wide_bwd_frag(layer, col >> 5, kk) * 64 + (col & 31) + 32 * h) * 8 + j] = (_Float16)w[i];
        }
    }
    // FP8 image: the row's exponent, then bytes k .. k + 3 of (k-step s, plane, lane r + 32 h)
    float amax = fmaxf(fmaxf(fabsf(inf[0]), fabsf(inf[1])), fmaxf(fabsf(inf[2]), fabsf(inf[3])));
#pragma unroll
    for (int off = 16; off >= 1; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off, 64));
    int e = 0;
    if (amax > 0.0f) {
        int E = 0;
        const float M = frexpf(amax, &E);
        e = M <= 0.875f ? E - 9 : E - 8;
        e = max(-127, min(127, e));
    }
    float a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = __builtin_amdgcn_fmed3f(ldexpf(inf[i], -e), -448.0f, 448.0f);
    const uint32_t lo = __builtin_amdgcn_cvt_pk_fp8_f32(a[0], a[1], 0, false);
    const uint32_t wd = __builtin_amdgcn_cvt_pk_fp8_f32(a[2], a[3], lo, true);
    {
        const int s = c >> 6, plane = (c >> 5) & 1, h = (c >> 2) & 1, k = 4 * ((c >> 3) & 3);
        const int f = wide8_frag(layer, mbk, s);
        *reinterpret_cast<uint32_t*>(im.img8 + 20 * 1024 + (f * 128 + plane * 64 + r + 32 * h) * 16 + k) = wd;
    }
    if (c4 == 0) {
        if (layer < 5) reinterpret_cast<uint8_t*>(im.scales)[((layer - 1) * 32 + r) * 4 + mbk] = (uint8_t)(e + 127);
        else im.scales[4 * 32 + r] = (uint32_t)(e + 127) | (127u << 8) | (127u << 16) | (127u << 24);
    }
}


// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
static int num_cus() {
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (dev < 0 || dev >= 64) dev = 0;
    if (!cached[dev]) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        cached[dev] = v;
    }
    return cached[dev];
}

template <class K>
static int blocks_per_cu(K kernel, int threads) {
    int v = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, kernel, threads, 0) != hipSuccess || v <= 0) v = 1;
    return v;
}

template <class K, class... Extra>
static hipError_t launch_persistent_infer(K kernel, int threads, int& cache_bpc, int64_t groups, const float* queries,
                                          float* out, int64_t n, const _Float16* wf, hipStream_t s, Extra... extra) {
    if (!cache_bpc) cache_bpc = blocks_per_cu(kernel, threads);
    const int wpb = threads / 64;
    const int64_t want = (groups + wpb - 1) / wpb;
    const int64_t cap = (int64_t)num_cus() * cache_bpc;
    const int grid = (int)(want < cap ? want : cap);
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(threads), 0, s, queries, out, n, (const h8*)wf, extra...);
    return hipGetLastError();
}

#if NRC_DEBUG_KERNELS
static int64_t g_last_clock_waves = 0;
template <class K, class... Extra>
static hipError_t launch_clocked(K kernel, int threads, int& cache_bpc, int64_t groups, const float* queries, float* out,
                                 int64_t n, const _Float16* wf, hipStream_t s, Extra... extra) {
    if (!cache_bpc) cache_bpc = blocks_per_cu(kernel, threads);
    const int64_t want = (groups + threads / 64 - 1) / (threads / 64);
    const int64_t grid = std::min<int64_t>(want, (int64_t)num_cus() * cache_bpc);
    g_last_clock_waves = std::min<int64_t>(grid * (threads / 64), kInferClockWavesMax);
    return launch_persistent_infer(kernel, threads, cache_bpc, groups, queries, out, n, wf, s, extra...);
}

hipError_t read_infer_clock(uint64_t* host, int64_t cap_waves, int64_t* waves) {
    const int64_t w = std::min(cap_waves, g_last_clock_waves);
    *waves = w;
    if (w <= 0) return hipSuccess;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_infer_clock), sizeof(uint64_t) * 6 * w, 0, hipMemcpyDeviceToHost);
}

#else
hipError_t read_infer_clock(uint64_t*, int64_t, int64_t*) { return hipErrorNotSupported; }
#endif

// Inference kernel variants (A/B-able in one process through nrc_debug_infer_variant):
//   0: v1 (weights hoisted into registers, one wave per SIMD)
//   1: v2, 1 tile (32 queries) per wave iteration, up to 3 waves per SIMD
//   2: v2, 2 tiles (64 queries) per wave iteration, 2 waves per SIMD
//   3: v2, 1 tile, 512-thread blocks, 4 waves per SIMD
//   4: v2, 1 tile, next-layer fragment prefetch, 3 waves per SIMD
//   5: v2, 1 tile, 512-thread blocks, 4 waves per SIMD, prefetch
//   6: v2, 2 tiles, 512-thread blocks, 2 waves per SIMD, prefetch
//   7-9, 14-16: ablations (timing only); 10-13: v3 register-resident weights; 17-20: v4 asm prefetch
//   21: variant 3 + LDS-staged 16-B result stores;  22: variant 3 + omod doubling-chain encoder
//   23: variant 22 + branch-free prefetch and buffer-store epilogue (default)
// round 2: variant 39 (encoder v3, per-CU LDS work queue on 1024-thread blocks, buffer-load prefetch, packed epilogue);
// in-process A/B at 2^21 queries: 75.1 vs 86.5 us for variant 23 (profiles/r02_infer/). round 3: variant 47 (below)
static int g_default_infer_variant = 47;

hipError_t launch_infer_variant(int variant, const float* queries, float* out, int64_t n, const _Float16* wf,
                                hipStream_t s, uint32_t* pools, int* parity) {
    if (n <= 0) return hipSuccess;
    const int64_t ntiles = (n + 31) / 32;
    static int bpc[kNumInferVariants] = {};
#if NRC_DEBUG_KERNELS
    if (variant == 41 || variant == 42) {  // 42: 41 with the in-kernel clock
        if (!pools || !parity) return hipErrorInvalidValue;
        InferEpilogue e{};
        e.wq = pools;
        e.parity = (*parity ^= 1) & 1;  // only pooled launches flip it: the set they skip is the one they zero
        if (variant == 41)
            return launch_persistent_infer(infer_pooled_kernel<48 | 1024 | 8192 | 16384>, 1024, bpc[41], ntiles, queries, out, n, wf, s, e);
        return launch_clocked(infer_pooled_kernel<48 | 1024 | 8192 | 16384 | 512>, 1024, bpc[42], ntiles, queries, out, n, wf, s, e);
    }
    if (variant == 45 || variant == 46) {  // 46: 45 with the in-kernel clock
        if (!pools || !parity) return hipErrorInvalidValue;
        InferEpilogue e{};
        e.wq = pools;
        *parity ^= 2;  // the steal sets' own parity bit (the pooled variants flip bit 0)
        e.parity = (*parity >> 1) & 1;
        if (variant == 45)
            return launch_persistent_infer(infer_pooled_kernel<48 | 1024 | 8192 | 32768>, 1024, bpc[45], ntiles, queries, out, n, wf, s, e);
        return launch_clocked(infer_pooled_kernel<48 | 1024 | 8192 | 32768 | 512>, 1024, bpc[46], ntiles, queries, out, n, wf, s, e);
    }
#endif
    switch (variant) {
        // The kernels kept for in-process A/B (tools/ab_infer.py). The rejected ones of rounds 1-2 (register-resident
        // weights, explicit layer-ahead prefetch, ping-pong tiles, 2-tile waves, SIMD-staggered starts, launch-wide
        // work queue, ablations) were measured, recorded in DESIGN.md §13 / profiles/r02_infer, and removed.
#if NRC_DEBUG_KERNELS
        // 0: round-1 reference kernel (32-query tiles, one tile per wave iteration)
        case 0: return launch_persistent_infer(infer_kernel, kInferThreads, bpc[0], ntiles, queries, out, n, wf, s);
        // 23: round-1 production (1 tile / 4 waves per SIMD, omod triangle chain, branch-free prefetch, buffer stores)
        case 23: return launch_persistent_infer(infer_kernel_v2<1, 4, 512, false, 48>, 512, bpc[23], ntiles, queries, out, n, wf, s);
        // 30: 23 with encoder v3 (tent-map triangle wave, clamped OneBlob wrap)
        case 30: return launch_persistent_infer(infer_kernel_v2<1, 4, 512, false, 48 | 1024>, 512, bpc[30], ntiles, queries, out, n, wf, s);
        // 39 (default): 30 with 1024-thread blocks (one per CU) drawing tiles from an LDS work queue, buffer-load query
        // prefetch and the packed output epilogue; 40: 39 with the in-kernel clock (nrc_debug_read_infer_clock)
        case 40: return launch_clocked(infer_kernel_v2<1, 4, 1024, false, 48 | 1024 | 2048 | 8192 | 512>, 1024, bpc[40], ntiles, queries, out, n, wf, s);
        case 39: return launch_persistent_infer(infer_kernel_v2<1, 4, 1024, false, 48 | 1024 | 2048 | 8192>, 1024, bpc[39], ntiles, queries, out, n, wf, s);
        // 48: 47 with the in-kernel clock
        case 48: return launch_clocked(infer_kernel_v2<1, 4, 1024, false, 48 | 1024 | 2048 | 8192 | 65536 | 512>, 1024, bpc[48], ntiles, queries, out, n, wf, s);
        // round 4 (energy per query): 47's body with two 32-query tiles per wave iteration, every
        // weight-fragment read from LDS feeding both tiles (23.5 instead of 47 ds_read_b128 per tile); 52: 512-thread
        // blocks at 2 waves per SIMD, 53: 52 with A-major MFMA order (consecutive MFMAs share the weight operand), 54:
        // 768-thread blocks at 3 waves per SIMD (<= 168 VGPRs), 55: 54 A-major. Groups of 2 tiles: ntiles / 2 groups.
        case 52: return launch_persistent_infer(infer_kernel_v2<2, 2, 512, false, 48 | 1024 | 2048 | 65536>, 512, bpc[52], (ntiles + 1) / 2, queries, out, n, wf, s);
        case 53: return launch_persistent_infer(infer_kernel_v2<2, 2, 512, false, 48 | 1024 | 2048 | 65536 | 131072>, 512, bpc[53], (ntiles + 1) / 2, queries, out, n, wf, s);
        case 54: return launch_persistent_infer(infer_kernel_v2<2, 3, 768, false, 48 | 1024 | 2048 | 65536>, 768, bpc[54], (ntiles + 1) / 2, queries, out, n, wf, s);
        case 55: return launch_persistent_infer(infer_kernel_v2<2, 3, 768, false, 48 | 1024 | 2048 | 65536 | 131072>, 768, bpc[55], (ntiles + 1) / 2, queries, out, n, wf, s);
        // 56 / 58: 52 / 54 with tile-major MFMA order; 57 / 59: 2 / 3 waves per SIMD with the layer-ahead fragment
        // prefetch (PREFETCH; 32x32x16 output layer)
        case 56: return launch_persistent_infer(infer_kernel_v2<2, 2, 512, false, 48 | 1024 | 2048 | 65536 | 262144>, 512, bpc[56], (ntiles + 1) / 2, queries, out, n, wf, s);
        case 57: return launch_persistent_infer(infer_kernel_v2<2, 2, 512, true, 48 | 1024 | 2048>, 512, bpc[57], (ntiles + 1) / 2, queries, out, n, wf, s);
        case 58: return launch_persistent_infer(infer_kernel_v2<2, 3, 768, false, 48 | 1024 | 2048 | 65536 | 262144>, 768, bpc[58], (ntiles + 1) / 2, queries, out, n, wf, s);
        case 59: return launch_persistent_infer(infer_kernel_v2<2, 3, 768, true, 48 | 1024 | 2048>, 768, bpc[59], (ntiles + 1) / 2, queries, out, n, wf, s);
        // round 4 (the C4 per-rank shard's one-tile tail): 47's body with fewer waves per CU, one persistent block per
        // CU -- 61: 512 threads (2 waves per SIMD), 62: 768 threads (3 per SIMD) -- so that the last tile of a CU takes
        // about half / three quarters of the 4-wave tile time
        case 61: bpc[61] = 1; return launch_persistent_infer(infer_kernel_v2<1, 2, 512, false, 48 | 1024 | 2048 | 8192 | 65536>, 512, bpc[61], ntiles, queries, out, n, wf, s);
        case 62: bpc[62] = 1; return launch_persistent_infer(infer_kernel_v2<1, 3, 768, false, 48 | 1024 | 2048 | 8192 | 65536>, 768, bpc[62], ntiles, queries, out, n, wf, s);
        // round 6: 63 / 64 = 47 / 62 with the first tile's loads issued before the weight copy (kAblEarlyQ)
        case 63: return launch_persistent_infer(infer_kernel_v2<1, 4, 1024, false, 48 | 1024 | 2048 | 8192 | 65536 | kAblEarlyQ>, 1024, bpc[63], ntiles, queries, out, n, wf, s);
        case 64: bpc[64] = 1; return launch_persistent_infer(infer_kernel_v2<1, 3, 768, false, 48 | 1024 | 2048 | 8192 | 65536 | kAblEarlyQ>, 768, bpc[64], ntiles, queries, out, n, wf, s);
        // 60: energy probe (wrong outputs): 47 with 12 of the 14 pad slots of layer 0 fed as zeros
        case 60: return launch_persistent_infer(infer_kernel_v2<1, 4, 1024, false, 48 | 1024 | 2048 | 8192 | 65536 | 524288>, 1024, bpc[60], ntiles, queries, out, n, wf, s);
#endif
        // 47 (default, round 3): 39 with the output layer on 4x4x4 16-block MFMAs (65536); in-process A/B at 2^21
        // queries 82.3-82.6 vs 82.7-83.4 us (profiles/r03_infer/ab_out4x4_v47.json)
        case 47: return launch_persistent_infer(infer_kernel_v2<1, 4, 1024, false, 48 | 1024 | 2048 | 8192 | 65536>, 1024, bpc[47], ntiles, queries, out, n, wf, s);
        default: return hipErrorInvalidValue;
    }
}

#if NRC_DEBUG_KERNELS
// Diagnostic: the default kernel with phase stamps; stamps gets kInferPhases sums per wave of the persistent grid.
hipError_t launch_infer_stamped(const float* queries, float* out, int64_t n, const _Float16* wf, uint64_t* stamps,
                                int64_t* waves, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t ntiles = (n + 31) / 32;
    const int bpc = blocks_per_cu(infer_stamp_kernel, 512);
    const int64_t blocks = std::min<int64_t>((int64_t)num_cus() * bpc, (ntiles + 7) / 8);
    *waves = blocks * 8;
    hipLaunchKernelGGL(infer_stamp_kernel, dim3((unsigned)blocks), dim3(512), 0, s, queries, out, n,
                       (const h8*)wf, stamps);
    return hipGetLastError();
}

#else
hipError_t launch_infer_stamped(const float*, float*, int64_t, const _Float16*, uint64_t*, int64_t*, hipStream_t) {
    return hipErrorNotSupported;
}
#endif

// Launches of at most kInferSmallN queries (a data-parallel rank's shard: 2^19 at 8 ranks) run variant 47's body with
// 768-thread blocks, one per CU (3 waves per SIMD): the CU's last tile then takes three quarters of the 4-wave tile
// time, and the tail after the queue runs dry is the per-launch cost that dominates a small launch (DESIGN.md §8:
// 22.6 vs 24.1 us at 2^19 in-process, 33.9 vs 34.9 at 3 * 2^18; 44.6 vs 43.2 at 2^20 and 79.7 vs 78.9 at 2^21, where
// the 4-wave shape stays: profiles/r04_tail/).
constexpr int64_t kInferSmallN = (int64_t)3 << 18;

hipError_t launch_infer(const float* queries, float* out, int64_t n, const _Float16* wf, hipStream_t s, uint32_t* pools,
                        int* parity, bool padq) {
    if (n <= 0) return hipSuccess;
    constexpr int A47 = 48 | 1024 | 2048 | 8192 | 65536;
    const int64_t ntiles = (n + 31) / 32;
    if (n <= kInferSmallN) {
        static int bpc = 1, bpc_p = 1;  // one persistent block per CU
        if (padq)
            return launch_persistent_infer(infer_kernel_v2<1, 3, 768, false, A47 | kAblPadQ>, 768, bpc_p, ntiles, queries,
                                           out, n, wf, s);
        return launch_persistent_infer(infer_kernel_v2<1, 3, 768, false, A47>, 768, bpc, ntiles, queries, out, n, wf, s);
    }
    if (padq) {  // variant 47 over padded RadianceQuery records
        static int bpc = 0;
        return launch_persistent_infer(infer_kernel_v2<1, 4, 1024, false, A47 | kAblPadQ>, 1024, bpc, ntiles, queries, out,
                                       n, wf, s);
    }
    return launch_infer_variant(g_default_infer_variant, queries, out, n, wf, s, pools, parity);
}

// Round 5: a training step's level features by gathers from the f16 table (2 MB, L2-resident) instead of the LDS
// pass: at 16,384 samples the LDS pass is 128 blocks each staging a 128-KiB level table into one CU (≈5 us of LDS-DMA
// per block, half the chip idle), while the 2 M gathers of the step spread over every CU. Thread = (level, sample);
// block k sits on XCD k % 8, which holds levels x and x + 8 (two level tables per XCD L2). Bitwise the LDS pass's
// features (hash_level_feature: the same corners, weights and half-FMA order).
template <int QD>
__global__ __launch_bounds__(256) void hash_feature_gather_kernel(const float* __restrict__ q, int64_t n, int nchunk,
                                                                  const uint32_t* __restrict__ table,
                                                                  uint32_t* __restrict__ feat) {
    const int k = (int)blockIdx.x, x = k & 7, j = k >> 3;
    const int level = x + (j >= nchunk ? 8 : 0), chunk = j >= nchunk ? j - nchunk : j;
    const int64_t s = (int64_t)chunk * 256 + threadIdx.x;
    if (s >= n) return;
    const float* r = q + s * QD;
    const float px = r[0], py = r[1], pz = r[2];
    feat[(int64_t)level * kHashFeatStride + s] = level <= 1 ? hash_level_feature<true>(px, py, pz, level, table)
                                                            : hash_level_feature<false>(px, py, pz, level, table);
}

static void launch_hash_feature_gather(const float* q, int64_t n, const uint32_t* g, uint32_t* feat, bool padq,
                                       hipStream_t s) {
    const int nchunk = (int)((n + 255) / 256);
    if (padq)
        hipLaunchKernelGGL(hash_feature_gather_kernel<NRC_INPUT_DIMS_PADDED>, dim3(16 * nchunk), dim3(256), 0, s, q, n,
                           nchunk, g, feat);
    else
        hipLaunchKernelGGL(hash_feature_gather_kernel<NRC_INPUT_DIMS>, dim3(16 * nchunk), dim3(256), 0, s, q, n, nchunk,
                           g, feat);
}

// One feature pass of hash_feature_kernel over cnt <= kHashFeatStride queries (the launch shape of launch_infer_hash).
// p_default: query ranges per level when the knob is unset (0: the inference choice below)
static void launch_hash_feature_pass(const float* qc0, int64_t cnt, const uint32_t* g, uint32_t* feat, bool padq,
                                     hipStream_t s, int p_default = 0) {
    // query ranges per level (multiple of the 8 XCDs); knob hash_feat_p overrides (A/B). Round 4: 32 above 2^19
    // queries (4 blocks per CU, two ranges' positions per XCD L2 at a time): 179.7 vs 185.3 us (P = 16) per 2^21
    // queries in-process, 24 / 48 / 64 / 128 slower (profiles/r04_hash/ab_hash_feat_p*.json)
    const int kp = knob(kKnobHashFeatP);
    const int P = kp > 0 ? kp : p_default > 0 ? p_default : cnt > ((int64_t)1 << 19) ? 32 : 8;
#if NRC_DEBUG_KERNELS
    const int fa = knob(kKnobHashFeatAbl);
    if (fa > 0) {
        auto k = fa == 1   ? hash_feature_kernel<1>
                 : fa == 2 ? hash_feature_kernel<2>
                 : fa == 4 ? hash_feature_kernel<4>
                 : fa == 8 ? hash_feature_kernel<8>  // round-3 arithmetic (A/B of the packed form)
                 : fa == 16 ? hash_feature_kernel<16>  // round-3 loop (A/B of the pipelined steps)
                 : fa == 32 ? hash_feature_kernel<32>  // no position loads, scattered positions
                 : fa == 33 ? hash_feature_kernel<33>  // 32 without the gathers
                 : fa == 36 ? hash_feature_kernel<36>  // 32 without the stores
                 : fa == 128 ? hash_feature_kernel<128>  // positions 5 steps ahead (round 6)
                           : hash_feature_kernel<7>;
        hipLaunchKernelGGL(k, dim3(16 * P), dim3(1024), 0, s, qc0, cnt, P, g, feat);
        return;
    }
#endif
    if (padq) hipLaunchKernelGGL(hash_feature_kernel<64>, dim3(16 * P), dim3(1024), 0, s, qc0, cnt, P, g, feat);
    else hipLaunchKernelGGL(hash_feature_kernel<0>, dim3(16 * P), dim3(1024), 0, s, qc0, cnt, P, g, feat);
}

hipError_t launch_infer_hash(const float* queries, float* out, int64_t n, const _Float16* wf, const _Float16* grid,
                             const float* thr, float* rgba, int64_t n_acc, int mode, float w, hipStream_t s,
                             uint32_t* feat, bool padq) {
    if (n <= 0) return hipSuccess;
    if (mode != -1 && mode != 0 && mode != 2) return hipErrorInvalidValue;
    if (padq && !feat) return hipErrorInvalidValue;  // padded queries: the feature-pass path only
    const int qd = padq ? NRC_INPUT_DIMS_PADDED : NRC_INPUT_DIMS;
    const uint32_t* g = reinterpret_cast<const uint32_t*>(grid);
    if (feat) {
        // round 3: per pass of <= kHashFeatStride queries, the LDS-table feature kernel, then the MLP kernel reading them
        static int bpf[3] = {};
        for (int64_t c0 = 0; c0 < n; c0 += kHashFeatStride) {
            const int64_t cnt = std::min<int64_t>(kHashFeatStride, n - c0);
            launch_hash_feature_pass(queries + c0 * qd, cnt, g, feat, padq, s);
            const int64_t acc = std::min<int64_t>(std::max<int64_t>(n_acc - c0, 0), cnt);
            const InferEpilogue e{thr ? thr + c0 * 3 : nullptr, rgba ? reinterpret_cast<float4*>(rgba) + c0 : nullptr, acc, w};
            const float* qc = queries + c0 * qd;
            float* oc = out ? out + c0 * NRC_OUTPUT_DIMS : nullptr;
            const int64_t nt = (cnt + 31) / 32;
            hipError_t err;
            const uint32_t* fc = feat;
            if (padq) {
                static int bpp[3] = {};
                if (mode == -1) err = launch_persistent_infer(infer_hashf_kernel<-1, kAblPadQ>, 1024, bpp[0], nt, qc, oc, cnt, wf, s, e, fc);
                else if (mode == 0) err = launch_persistent_infer(infer_hashf_kernel<0, kAblPadQ>, 1024, bpp[1], nt, qc, oc, cnt, wf, s, e, fc);
                else err = launch_persistent_infer(infer_hashf_kernel<2, kAblPadQ>, 1024, bpp[2], nt, qc, oc, cnt, wf, s, e, fc);
            } else if (mode == -1) err = launch_persistent_infer(infer_hashf_kernel<-1>, 1024, bpf[0], nt, qc, oc, cnt, wf, s, e, fc);
            else if (mode == 0) err = launch_persistent_infer(infer_hashf_kernel<0>, 1024, bpf[1], nt, qc, oc, cnt, wf, s, e, fc);
            else err = launch_persistent_infer(infer_hashf_kernel<2>, 1024, bpf[2], nt, qc, oc, cnt, wf, s, e, fc);
            if (err != hipSuccess) return err;
        }
        return hipGetLastError();
    }
    const int64_t ntiles = (n + 31) / 32;
    const InferEpilogue epi{thr, reinterpret_cast<float4*>(rgba), n_acc, w};
    static int bpq[3] = {};
    switch (mode) {
        case -1: return launch_persistent_infer(infer_hash_kernel<-1, 2048 | 32 | 65536>, 512, bpq[0], ntiles, queries, out, n, wf, s, epi, g);
        case 0: return launch_persistent_infer(infer_hash_kernel<0, 2048 | 32 | 65536>, 512, bpq[1], ntiles, queries, out, n, wf, s, epi, g);
        case 2: return launch_persistent_infer(infer_hash_kernel<2, 2048 | 32 | 65536>, 512, bpq[2], ntiles, queries, out, n, wf, s, epi, g);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_infer_sh(const float* queries, float* out, int64_t n, const _Float16* wf, const float* thr,
                           float* rgba, int64_t n_acc, int mode, float w, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t ntiles = (n + 31) / 32;
    const InferEpilogue epi{thr, reinterpret_cast<float4*>(rgba), n_acc, w};
    static int bpq[3] = {};
    switch (mode) {
        case -1: return launch_persistent_infer(infer_sh_kernel<-1, 1024, 2048>, 1024, bpq[0], ntiles, queries, out, n, wf, s, epi);
        case 0: return launch_persistent_infer(infer_sh_kernel<0, 1024, 2048>, 1024, bpq[1], ntiles, queries, out, n, wf, s, epi);
        case 2: return launch_persistent_infer(infer_sh_kernel<2, 1024, 2048>, 1024, bpq[2], ntiles, queries, out, n, wf, s, epi);
        default: return hipErrorInvalidValue;
    }
}

// ------------------------------------------------------------------------------------------------
// tcnn-numerics inference (round 4, opt-in: nrc_config.infer_precision = NRC_PRECISION_F16_ACC16).
// tiny-cuda-nn's FullyFusedMLP forward keeps its accumulators in f16 (NRCNetworkConfigs.h:26-33; SURVEY App. A.5 [M]):
// every 16-wide K chunk of every layer is added to an f16 accumulator, in K order, and rounded to f16 -- the oracle's
// ORC_TCNN mode (oracle/nrc_oracle.c matvec). The production kernel accumulates a whole layer in f32 instead, which sits
// 1.7-2.1e-3 from ORC_TCNN on random weights. Here:
//   * chunk kk of a layer must hold the features 16 kk .. 16 kk + 15 in tcnn's order. Hidden layers already do (the
//     accumulator-as-operand chain: chunk kk = rows 16 kk.. of the previous layer, acc_row); layer 0 does not (the
//     encoder's lane slots mix features, slot_feature), so each wave writes its tile's encoded features to an LDS row per
//     query in canonical order ([32][80] f16, the 14 pad features 1.0 written once) and reads chunk kk back as the
//     B operand (lane half h: features 16 kk + 8 h ..), and the layer-0 A fragments are rebuilt in that order from the
//     f32 inference weights at block start;
//   * per chunk: acc = f16(MFMA(W_kk, x_kk, acc)) (the MFMA adds the chunk's 16 exact products to the f16-valued
//     accumulator in f32, then one rounding to f16: the oracle's f16(acc + part) up to f32 double rounding);
//   * output layer: the 32x32x16 form (rows 0..2 of lane half 0), the same chunking.
// Same encoder (encode_v3) and output format as the production kernel; about 4x its VALU (the per-chunk roundings).
// Round 6: the round-4/5 kernel ran 2.95x the production kernel's time. PMC of it and of a first
// rework (profiles/r06_tcnn/): VALU-issue-bound -- 85 % of every SIMD's vector issue, at 3x the production kernel's
// VALU per tile, the matrix pipe at 21 % -- because every chunk's f32 result was rounded to f16 and widened back to f32
// for the next chunk's MFMA (1.5 VALU per element; v_fma_mixlo/hi_f16 in its place costs 2 issue slots per element and
// measured no faster). Now:
//   * the widening is done by the matrix cores (TcnnId below): 0.5 VALU per element and chunk;
//   * 1024-thread blocks (16 waves, 4 per SIMD) over one copy of the weights, each wave drawing its tiles from the
//     block's LDS queue and fetching the next tile's inputs one tile ahead (as the production kernel); a branch-free
//     buffer store (a conditional store, and the wavefront-scope fences around the row hand-off, made every tile wait
//     vmcnt(0));
//   * 176-byte query rows (44 dwords = 4 x 11): the chunk reads (ds_read_b128) of 16 consecutive lanes hit 16 distinct
//     bank quads (the 160-byte rows had 48 % of the LDS cycles in bank conflicts).
constexpr int kTcnnRowHalves = 88;  // one query's 80 encoded features + 8 unused halves (176 B)
constexpr int kTcnnWaves = 16;

// acc = f16(part): one v_cvt_pk_f16_f32 per pair
__device__ __forceinline__ void first16(uint32_t (&a)[8], const f16v& p) {
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = pk2(p[2 * i], p[2 * i + 1]);
}
// accumulator words 4b .. 4b + 3 -> B operand, ReLU on the packed halves (f16(relu(x)) == relu(f16(x))) as a signed
// 16-bit max with 0 (v_pk_max_i16): a negative half has its sign bit set and becomes +0. (An f16 max of words that come
// out of inline asm gets a canonicalising v_pk_max_f16 in front of it: twice the instructions.)
__device__ __forceinline__ h8 relu_words(const uint32_t (&a)[8], int b) {
    typedef short s8v __attribute__((ext_vector_type(8)));
    const u4 w = {a[4 * b], a[4 * b + 1], a[4 * b + 2], a[4 * b + 3]};
    const s8v z = {};
    return __builtin_bit_cast(h8, __builtin_elementwise_max(__builtin_bit_cast(s8v, w), z));
}

// The f16 accumulator back into f32 by the matrix cores (round 6, second form): the packed accumulator words 0..3 /
// 4..7 are B operands (the accumulator-as-operand layout, acc_row), and two constant 0/1 A fragments Id0 / Id1 route
// them back to rows 0..15 / 16..31 of an f32 accumulator -- products with 1.0 and sums with zeros, exact. The chunk's own
// MFMA then adds its 16 products to that C, and one v_cvt_pk_f16_f32 per pair rounds: acc = f16(acc + chunk), tcnn's
// per-chunk f16 accumulation, with 0.5 VALU per element instead of 1.5 (convert down, widen both halves back) or 2
// issue slots (v_fma_mix). The kernel was VALU-issue-bound (85 % of the SIMDs' vector issue, PMC); the identity MFMAs
// move that work to the matrix pipe, which ran at 21 %.
// Second form (round 6, RE 1, the default): v_mfma_f32_4x4x4_16b_f16 runs 16 independent 4x4x4 products, block
// b = lane / 4 taking its B columns from lanes 4b..4b+3 and writing column lane % 4 of its 4-row result into that lane's
// 4 registers. With A = the 4x4 identity (lane l: a one at element l % 4) the result is the lane's own 4 B halves as
// f32, in order: one such MFMA widens accumulator words 2q, 2q + 1 into registers 4q .. 4q + 3, four of them the whole
// 32x32 block -- about 12.5 cycles each against 34 for a 32x32x16 (tools/microbench/mfma_4x4.hip), so 4 x 4x4x4 instead
// of 2 x 32x32x16 per block and chunk. (An infinite f16 accumulator element -- an overflow of tcnn's f16 accumulation --
// makes the other elements that share its identity product NaN, 0 x inf: those are the same query's other neurons,
// whose output is then not finite in tcnn's arithmetic either; no other query is touched.)
typedef _Float16 h4v __attribute__((ext_vector_type(4)));
struct TcnnId {
    h8 lo, hi;  // A fragments: lane (i, h) element e is 1 where row i == 8 (e / 4) + 4 h + e % 4 (+ 16 for hi)
    h4v q;      // 4x4x4 identity: element lane % 4 is 1
    __device__ __forceinline__ explicit TcnnId(int lane) {
        const int i = lane & 31, h = lane >> 5;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int row = 8 * (e >> 2) + 4 * h + (e & 3);
            lo[e] = (_Float16)(i == row ? 1.0f : 0.0f);
            hi[e] = (_Float16)(i == 16 + row ? 1.0f : 0.0f);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) q[e] = (_Float16)((lane & 3) == e ? 1.0f : 0.0f);
    }
};
__device__ __forceinline__ h8 acc_words(const uint32_t (&a)[8], int b) {
    const u4 w = {a[4 * b], a[4 * b + 1], a[4 * b + 2], a[4 * b + 3]};
    return __builtin_bit_cast(h8, w);
}
// accumulator words 0..7 widened to the f32 32x32 accumulator by four 4x4x4 identity MFMAs
__device__ __forceinline__ f16v widen4(const TcnnId& id, const uint32_t (&a)[8]) {
    typedef uint32_t u2v __attribute__((ext_vector_type(2)));
    typedef float f4 __attribute__((ext_vector_type(4)));
    typedef float f8v __attribute__((ext_vector_type(8)));
    f4 d[4];
#pragma unroll
    for (int qq = 0; qq < 4; ++qq)
        d[qq] = __builtin_amdgcn_mfma_f32_4x4x4f16(id.q, __builtin_bit_cast(h4v, u2v{a[2 * qq], a[2 * qq + 1]}),
                                                   f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    const f8v lo = __builtin_shufflevector(d[0], d[1], 0, 1, 2, 3, 4, 5, 6, 7);
    const f8v hi = __builtin_shufflevector(d[2], d[3], 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
}

// One layer's KK chunks of both M-blocks into the packed-f16 accumulators: chunk 0 rounds the MFMA result, every
// further chunk re-enters the accumulator first (RE 0: through Id0 / Id1, RE 1: widen4). The two M-blocks' chains are
// independent.
template <int KK, int RE>
__device__ __forceinline__ void tcnn_layer(lds_h8* wl, const TcnnId& id, int layer, const h8 (&in)[KK],
                                           uint32_t (&acc)[2][8]) {
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
        const h8 w0 = wl[fwd_frag(layer, 0, kk) * 64], w1 = wl[fwd_frag(layer, 1, kk) * 64];
        f16v c0 = zero16(), c1 = zero16();
        if (kk > 0) {
            if constexpr (RE == 1) {
                c0 = widen4(id, acc[0]);
                c1 = widen4(id, acc[1]);
            } else {
                c0 = mfma(id.lo, acc_words(acc[0], 0), c0);
                c1 = mfma(id.lo, acc_words(acc[1], 0), c1);
                c0 = mfma(id.hi, acc_words(acc[0], 1), c0);
                c1 = mfma(id.hi, acc_words(acc[1], 1), c1);
            }
        }
        c0 = mfma(w0, in[kk], c0);
        c1 = mfma(w1, in[kk], c1);
        first16(acc[0], c0);
        first16(acc[1], c1);
    }
}

// ENC 0: Frequency (K = 80, 5 chunks, pad features 66..79); ENC 3: Hash (round 5) from hash_feature_kernel's level features
// (K = 64, 4 chunks: grid 0..31, OneBlob 32..55, Identity 56..61, pad 62, 63; feat = the pass's workspace), the same MLP
// chunking -- tcnn runs the same FullyFusedMLP behind either encoding (NRCNetworkConfigs.h:84-128).
template <int ENC, int RE = 1>
__global__ __launch_bounds__(64 * kTcnnWaves, 1) void infer_tcnn_kernel(const float* __restrict__ q,
                                                                        float* __restrict__ out, int64_t n,
                                                                        const h8* __restrict__ wf,
                                                                        const float* __restrict__ w0,
                                                                        const uint32_t* __restrict__ feat) {
    static_assert(ENC == 0 || ENC == 3, "Frequency or Hash-from-features");
    constexpr int W = kTcnnWaves, T = 64 * W;
    constexpr int KK0 = ENC == 3 ? 4 : 5, IN = ENC == 3 ? NRC_HASH_ENC_WIDTH : NRC_ENC_WIDTH;
    constexpr int PAD0 = ENC == 3 ? 62 : 66;  // first constant-one feature
    __shared__ __attribute__((aligned(16))) h8 lw[kFwdFrags * 64];
    __shared__ __attribute__((aligned(16))) _Float16 enc[W][32 * kTcnnRowHalves];
    __shared__ uint32_t wq_next;
    if (threadIdx.x == 0) wq_next = 0;
    copy_to_lds<T, kFwdFrags * 64>(lw, wf);
    __syncthreads();
    // layer-0 fragments in canonical K order: fragment (mb, kk), lane L, element j = W0[32 mb + L % 32][16 kk + 8 (L / 32) + j]
    for (int i = threadIdx.x; i < 2 * KK0 * 64; i += T) {
        const int frag = i >> 6, L = i & 63, mb = frag / KK0, kk = frag % KK0;
        const float* src = w0 + (32 * mb + (L & 31)) * IN + 16 * kk + 8 * (L >> 5);
        h8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (_Float16)src[j];
        lw[fwd_frag(0, mb, kk) * 64 + L] = v;
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, r = lane & 31;
    const TcnnId id(lane);
    _Float16* const row = &enc[wave][r * kTcnnRowHalves];
    // pad features (never rewritten)
    if (h == 0)
#pragma unroll
        for (int f = PAD0; f < IN; ++f) row[f] = (_Float16)1.0f;
    __syncthreads();
    char* const rowb = reinterpret_cast<char*>(row);
    // the block's contiguous range of tiles, drawn one at a time by its waves (the production kernel's LDS queue)
    const int64_t ntiles = (n + 31) / 32;
    const int64_t gbase = (int64_t)blockIdx.x * ntiles / gridDim.x, gend = (int64_t)(blockIdx.x + 1) * ntiles / gridDim.x;
    auto draw = [&]() -> int64_t {
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(&wq_next, 1u);
        return gbase + (int64_t)__builtin_amdgcn_readfirstlane(t);
    };
    // the next tile's queries (and level features) and the tile after it are fetched one tile ahead, as in the production
    // kernel (clamped rows: a fetch past the range reads a valid row that is never used)
    int64_t g = draw();
    if (g >= gend) return;
    auto fetch = [&](int64_t tile, QLane& Q, uint32_t (&F)[8]) {
        const int64_t sc = min(tile * 32 + r, n - 1);
        Q = load_q(q, sc, h);
        if constexpr (ENC == 3) {
#pragma unroll
            for (int i = 0; i < 8; ++i) F[i] = feat[(int64_t)(8 * h + i) * kHashFeatStride + sc];
        }
    };
    QLane Q;
    uint32_t F[8] = {};
    fetch(g, Q, F);
    int64_t gn = draw();
    for (; g < gend; g = gn, gn = draw()) {
        uint32_t w[20];
        if constexpr (ENC == 3) {
            // encode_hashf's slots: levels 8h.. (features 16h.., one half2 per level), OneBlob dims 3h.. (features
            // 32 + 12h..), Identity dims 3h.. (features 56 + 3h..)
#pragma unroll
            for (int i = 0; i < 8; ++i) w[i] = F[i];
            blob_v3(Q.b0, w[8], w[9]);
            blob_v3(Q.b1, w[10], w[11]);
            blob_v3(Q.b2, w[12], w[13]);
            w[14] = pk2(Q.i0, Q.i1);
            w[15] = pk2(Q.i2, 1.0f);
        } else {
            h8 x[5];
            encode_v3(Q, h, x);
#pragma unroll
            for (int kk = 0; kk < 5; ++kk) {
                const u4 t = __builtin_bit_cast(u4, x[kk]);
                w[4 * kk] = t.x;
                w[4 * kk + 1] = t.y;
                w[4 * kk + 2] = t.z;
                w[4 * kk + 3] = t.w;
            }
        }
        fetch(gn, Q, F);                // the next tile's inputs, in flight under this tile's MLP
        asm volatile("" ::: "memory");  // the previous tile's chunk reads of this row stay above these writes
        if constexpr (ENC == 3) {
#pragma unroll
            for (int i = 0; i < 8; ++i) *(uint32_t*)(rowb + 2 * (16 * h) + 4 * i) = w[i];
#pragma unroll
            for (int i = 0; i < 6; ++i) *(uint32_t*)(rowb + 2 * (32 + 12 * h) + 4 * i) = w[8 + i];
            const h2 id01 = __builtin_bit_cast(h2, w[14]), id2 = __builtin_bit_cast(h2, w[15]);
            row[56 + 3 * h] = id01[0];
            row[57 + 3 * h] = id01[1];
            row[58 + 3 * h] = id2[0];
        } else {
            // slots -> canonical features (slot_feature): TriangleWave slots 6d.. -> 12 d + 6 h.., OneBlob slots 18.. ->
            // 36 + 12 h.., Identity slots 30..32 -> 60 + 3 h..
#pragma unroll
            for (int d = 0; d < 3; ++d)
#pragma unroll
                for (int i = 0; i < 3; ++i) *(uint32_t*)(rowb + 2 * (12 * d + 6 * h) + 4 * i) = w[3 * d + i];
#pragma unroll
            for (int i = 0; i < 6; ++i) *(uint32_t*)(rowb + 2 * (36 + 12 * h) + 4 * i) = w[9 + i];
            const h2 id01 = __builtin_bit_cast(h2, w[15]), id2 = __builtin_bit_cast(h2, w[16]);
            row[60 + 3 * h] = id01[0];
            row[61 + 3 * h] = id01[1];
            row[62 + 3 * h] = id2[0];
        }
        // the wave's writes of every row land before its lanes read other lanes' rows: LDS executes one wave's operations
        // in order, so only the compiler must keep the reads below the writes (the "memory" clobbers). (Round 6: the
        // wavefront-scope release/acquire fences that stood here made the compiler wait vmcnt(0) -- for the prefetched
        // queries and the previous tile's stores -- on every tile.)
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        h8 in0[KK0];
#pragma unroll
        for (int kk = 0; kk < KK0; ++kk) in0[kk] = *(const h8*)(rowb + 32 * kk + 16 * h);
        asm volatile("" ::: "memory");
        lds_h8* const wl = (lds_h8*)(lw + lane);
        uint32_t acc[2][8];
        h8 y[4];
        // layer 0 (K = 80 / 64: 5 / 4 chunks) and the hidden layers (K = 64, 4 chunks)
        tcnn_layer<KK0, RE>(wl, id, 0, in0, acc);
#pragma unroll
        for (int l = 1; l < 5; ++l) {
            // k-step kk of the next layer = accumulator rows 16 kk.. = M-block kk / 2, registers 8 (kk % 2)..
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                y[b] = relu_words(acc[0], b);
                y[2 + b] = relu_words(acc[1], b);
            }
            tcnn_layer<4, RE>(launder(wl), id, l, y, acc);
        }
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            y[b] = relu_words(acc[0], b);
            y[2 + b] = relu_words(acc[1], b);
        }
        // output layer (rows 0..2 of lane half 0 = elements 0..2), the same chunking; RE 0: rows 0..3 re-enter through
        // Id0 (accumulator elements 4..7, rows 8..11, are fed as zeros); RE 1: elements 0..3 through one 4x4x4 identity
        // MFMA, elements 4..15 (rows no output reads) keep the previous chunk's values
        uint32_t o[2];
        {
            lds_h8* const wll = launder(wl);
            f16v c = zero16();
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                if constexpr (RE == 1) {
                    if (kk > 0) {
                        typedef uint32_t u2v __attribute__((ext_vector_type(2)));
                        typedef float f4 __attribute__((ext_vector_type(4)));
                        const f4 d = __builtin_amdgcn_mfma_f32_4x4x4f16(id.q, __builtin_bit_cast(h4v, u2v{o[0], o[1]}),
                                                                        f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
                        for (int e = 0; e < 4; ++e) c[e] = d[e];
                    }
                } else {
                    c = zero16();
                    if (kk > 0) c = mfma(id.lo, __builtin_bit_cast(h8, u4{o[0], o[1], 0u, 0u}), c);
                }
                c = mfma(wll[fwd_frag(5, 0, kk) * 64], y[kk], c);
                o[0] = pk2(c[0], c[1]);
                o[1] = pk2(c[2], c[3]);
            }
        }
        {
            // the output ReLU (NRCNetworkConfigs.h:29) of the f16 result; branch-free raw buffer store whose descriptor
            // covers the tile's valid rows (the h = 1 lanes and the tail are dropped by the hardware, as in the
            // production kernel: a conditional store made the next tile wait for its acknowledgement)
            const h2 o01 = __builtin_bit_cast(h2, o[0]), o23 = __builtin_bit_cast(h2, o[1]);
            const u3 ov = {__builtin_bit_cast(uint32_t, fmaxf((float)o01[0], 0.0f)),
                           __builtin_bit_cast(uint32_t, fmaxf((float)o01[1], 0.0f)),
                           __builtin_bit_cast(uint32_t, fmaxf((float)o23[0], 0.0f))};
            const int64_t s0 = g * 32;
            __builtin_amdgcn_raw_buffer_store_b96(ov, buffer_rsrc(out + s0 * NRC_OUTPUT_DIMS, tile_rows(n, s0) * 12),
                                                  h ? kBufferOff : r * 12, 0, 0);
        }
    }
}

hipError_t launch_infer_tcnn(const float* queries, float* out, int64_t n, const _Float16* wf, const float* w0,
                             hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (!wf || !w0) return hipErrorInvalidValue;
    static int bpc[2] = {};
    if (knob(kKnobTcnnReentry) == 0)
        return launch_persistent_infer(infer_tcnn_kernel<0, 0>, 64 * kTcnnWaves, bpc[0], (n + 31) / 32, queries, out, n,
                                       wf, s, w0, (const uint32_t*)nullptr);
    return launch_persistent_infer(infer_tcnn_kernel<0, 1>, 64 * kTcnnWaves, bpc[1], (n + 31) / 32, queries, out, n, wf,
                                   s, w0, (const uint32_t*)nullptr);
}

// tcnn-numerics Hash inference (NRC_PRECISION_F16_ACC16, round 5): the feature pass, then infer_tcnn_kernel<3> per pass
hipError_t launch_infer_hash_tcnn(const float* queries, float* out, int64_t n, const _Float16* wf, const float* w0,
                                  const _Float16* grid, uint32_t* feat, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (!wf || !w0 || !grid || !feat) return hipErrorInvalidValue;
    static int bpc[2] = {};
    const int re = knob(kKnobTcnnReentry) == 0 ? 0 : 1;
    for (int64_t c0 = 0; c0 < n; c0 += kHashFeatStride) {
        const int64_t cnt = std::min<int64_t>(kHashFeatStride, n - c0);
        const float* qc = queries + c0 * NRC_INPUT_DIMS;
        launch_hash_feature_pass(qc, cnt, reinterpret_cast<const uint32_t*>(grid), feat, false, s);
        const hipError_t e =
            re == 0 ? launch_persistent_infer(infer_tcnn_kernel<3, 0>, 64 * kTcnnWaves, bpc[0], (cnt + 31) / 32, qc,
                                              out + c0 * NRC_OUTPUT_DIMS, cnt, wf, s, w0, (const uint32_t*)feat)
                    : launch_persistent_infer(infer_tcnn_kernel<3, 1>, 64 * kTcnnWaves, bpc[1], (cnt + 31) / 32, qc,
                                              out + c0 * NRC_OUTPUT_DIMS, cnt, wf, s, w0, (const uint32_t*)feat);
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}

hipError_t launch_wide_pack(const float* w_infer, const float* w_train, const WideImages& im, hipStream_t s) {
    ModelBuffers mb{};
    mb.params = const_cast<float*>(w_train);
    mb.infer = const_cast<float*>(w_infer);
    hipLaunchKernelGGL(wide_adam_pack_kernel, dim3(kWideRowUnits * 32 / 256), dim3(256), 0, s, (int)kPackOnly,
                       (const float*)nullptr, 0, (const float*)nullptr, 0, (float*)nullptr, (float*)nullptr, mb,
                       OptimArgs{}, 0.0f, 1.0f, im);
    return hipGetLastError();
}

hipError_t launch_infer_wide(int prec, int enc, const float* queries, float* out, int64_t n, const void* img,
                             const uint32_t* scales, const float* thr, float* rgba, int64_t n_acc, int mode, float w,
                             hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int variant = prec >> 4;  // debug: kernel variant (nrc_debug_infer_precision)
    prec &= 15;
    if ((prec != 0 && prec != 1) || (enc != 0 && enc != 2) || (mode != -1 && mode != 0 && mode != 2) || variant > 2)
        return hipErrorInvalidValue;
    const int64_t ntiles = (n + 31) / 32;
    if (variant == 2) {
#if NRC_DEBUG_KERNELS  // FP8 with round 5's med3 clamp (relu_fp8x4_med3): A/B only, debug library
        if (enc != 0 || mode != -1 || prec != 1) return hipErrorInvalidValue;
        static int bv2 = 0;
        const InferEpilogue e{};
        return launch_persistent_infer(infer_wide_kernel<0, 1, -1, 512, true, true>, 512, bv2, ntiles, queries, out, n,
                                       reinterpret_cast<const _Float16*>(img), s, e, scales);
#else
        return hipErrorNotSupported;
#endif
    }
    if (variant == 1) {
#if NRC_DEBUG_KERNELS  // 1024-thread blocks (4 waves per SIMD): A/B only, debug library
        if (enc != 0 || mode != -1) return hipErrorInvalidValue;
        static int bv[2] = {};
        const InferEpilogue e{};
        if (prec == 0)
            return launch_persistent_infer(infer_wide_kernel<0, 0, -1, 1024>, 1024, bv[0], ntiles, queries, out, n,
                                           reinterpret_cast<const _Float16*>(img), s, e, scales);
        return launch_persistent_infer(infer_wide_kernel<0, 1, -1, 1024>, 1024, bv[1], ntiles, queries, out, n,
                                       reinterpret_cast<const _Float16*>(img), s, e, scales);
#else
        return hipErrorNotSupported;
#endif
    }
    static int bpc[2][2][3] = {};
    const InferEpilogue epi{thr, reinterpret_cast<float4*>(rgba), n_acc, w};
    const _Float16* im = reinterpret_cast<const _Float16*>(img);
    // per-block LDS work queue (round 2; the round-1 fixed-tiles-per-wave shape measured 1,010.9 vs 981.8 us f16 and
    // 714.7 vs 669.2 us FP8 per 2^23 queries, profiles/r02_infer/ab_wide_queue_vs_round1.json, and was removed)
    int& b = bpc[prec][enc >> 1][mode + 1 == 0 ? 0 : mode == 0 ? 1 : 2];
#define NRC_WIDE_LAUNCH(E, P, M)                                                                                  \
    return launch_persistent_infer(infer_wide_kernel<E, P, M, 512, true>, 512, b, ntiles, queries, out, n, im, s, epi, \
                                   scales)
#define NRC_WIDE_MODES(E, P)                  \
    switch (mode) {                           \
        case -1: NRC_WIDE_LAUNCH(E, P, -1);   \
        case 0: NRC_WIDE_LAUNCH(E, P, 0);     \
        default: NRC_WIDE_LAUNCH(E, P, 2);    \
    }
    if (enc == 0) {
        if (prec == 0) { NRC_WIDE_MODES(0, 0) } else { NRC_WIDE_MODES(0, 1) }
    } else {
        if (prec == 0) { NRC_WIDE_MODES(2, 0) } else { NRC_WIDE_MODES(2, 1) }
    }
#undef NRC_WIDE_MODES
#undef NRC_WIDE_LAUNCH
}

int64_t wide_bpad(int64_t b) { return (b + 31) / 32 * 32; }
// Workspace row stride: 32 samples (64 B) past bpad. With a power-of-two stride (bpad = 16,384 -> 32 KiB) the 32 rows
// of one MFMA operand load all map to the same L2 channel; the pad spreads them (wide_dw_kernel 36.1 -> 28.8 us per
// 16,384-sample step; pads of 8 / 16 / 48 / 64 / 128 / 160 samples measured 87.8 / 85.0 / 87.1 / 92.7 / 95 / 85 us
// per step against 84.9 for 32 and 92.0 unpadded; later, with the other changes in: pads of 256 / 1,024 / 2,048
// samples 70.9 us, 2,080 / 3,104 / 4,128 samples 63.4-64.4, 32 samples 63.1 -- the channel interleave is finer than
// 512 B).
int64_t wide_ld(int64_t b) { return wide_bpad(b) + 32; }
int wide_chunks(int64_t b) { return (int)((wide_bpad(b) + kWideChunk - 1) / kWideChunk); }

hipError_t launch_wide_train_fwd_bwd(int enc, const float* queries, const float* targets, int64_t b, float n_total,
                                     float loss_scale, const _Float16* fwd16, const _Float16* bwd16, _Float16* ws_in,
                                     _Float16* ws_d, float* slabs, float* loss_partials, hipStream_t s) {
    if (b <= 0) return hipSuccess;
    const int64_t bpad = wide_bpad(b), ld = wide_ld(b);
    const int tiles = (int)(bpad / 32);
    const int blocks = (tiles + 1) / 2;
    if (enc == 2)
        hipLaunchKernelGGL(wide_fwd_bwd_lds_kernel<2>, dim3(blocks), dim3(128), 0, s, queries, targets, b, bpad, ld,
                           n_total, loss_scale, (const h8*)fwd16, (const h8*)bwd16, ws_in, ws_d, loss_partials);
    else
        hipLaunchKernelGGL(wide_fwd_bwd_lds_kernel<0>, dim3(blocks), dim3(128), 0, s, queries, targets, b, bpad, ld,
                           n_total, loss_scale, (const h8*)fwd16, (const h8*)bwd16, ws_in, ws_d, loss_partials);
    const int nch = wide_chunks(b);
    hipLaunchKernelGGL(wide_dw_kernel, dim3(6 * nch), dim3(256), 0, s, ws_in, ws_d, bpad, ld, nch, slabs);
    return hipGetLastError();
}

hipError_t launch_wide_adam(int mode, const float* slabs, int nchunks, const float* loss_partials, int nlp,
                            float* grad_io, float* loss_out, const ModelBuffers& mb, const OptimArgs& oa,
                            const WideImages& im, hipStream_t s) {
    const float step = (float)(oa.step ? oa.step : 1);
    const float lr_t = oa.lr * sqrtf(1.0f - powf(oa.beta2, step)) / (1.0f - powf(oa.beta1, step));
    const float ema_debias = 1.0f - powf(oa.ema_decay, step);
    hipLaunchKernelGGL(wide_adam_pack_kernel, dim3(kWideRowUnits * 32 / 256), dim3(256), 0, s, mode, slabs, nchunks,
                       loss_partials, nlp, grad_io, loss_out, mb, oa, lr_t, ema_debias, im);
    return hipGetLastError();
}


hipError_t launch_fp8_convert(const float* x, uint8_t* y, int64_t n, int relu, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(fp8_convert_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, y, n, relu);
    return hipGetLastError();
}

hipError_t launch_encode_sh(const float* queries, float* enc, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(encode_sh_kernel, dim3((unsigned)((2 * n + 255) / 256)), dim3(256), 0, s, queries, enc, n);
    return hipGetLastError();
}

hipError_t launch_encode_hash(const float* queries, const _Float16* grid, float* enc, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(encode_hash_kernel, dim3((unsigned)((2 * n + 255) / 256)), dim3(256), 0, s, queries,
                       reinterpret_cast<const uint32_t*>(grid), enc, n);
    return hipGetLastError();
}

hipError_t launch_infer_accumulate(const float* queries, float* out, int64_t n, const _Float16* wf, const float* thr,
                                   float* rgba, int64_t n_acc, int mode, float w, hipStream_t s, bool padq) {
    if (n <= 0) return hipSuccess;
    const int64_t ntiles = (n + 31) / 32;
    static int bpc[4] = {};
    const InferEpilogue epi{thr, reinterpret_cast<float4*>(rgba), n_acc, w};
    // one 1024-thread block per CU drawing tiles from an LDS work queue (round 2: 82.6 vs 86.7 us per 1080p frame for
    // the round-1 512-thread shape, bit-identical, profiles/r02_frame/; the round-1 shape was removed in round 3)
    constexpr int X = 2048 | 65536, XP = X | kAblPadQ;
    switch (mode + (padq ? 1 : 0)) {
        case 0: return launch_persistent_infer(infer_accumulate_kernel<0, 1024, X>, 1024, bpc[0], ntiles, queries, out, n, wf, s, epi);
        case 2: return launch_persistent_infer(infer_accumulate_kernel<2, 1024, X>, 1024, bpc[1], ntiles, queries, out, n, wf, s, epi);
        case 1: return launch_persistent_infer(infer_accumulate_kernel<0, 1024, XP>, 1024, bpc[2], ntiles, queries, out, n, wf, s, epi);
        case 3: return launch_persistent_infer(infer_accumulate_kernel<2, 1024, XP>, 1024, bpc[3], ntiles, queries, out, n, wf, s, epi);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_encode(const float* queries, float* enc, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t threads = 2 * n;
    const int grid = (int)((threads + 255) / 256);
    hipLaunchKernelGGL(encode_kernel, dim3(grid), dim3(256), 0, s, queries, enc, n);
    return hipGetLastError();
}

int train_blocks(int64_t b) { return (int)((b + kTrainSamplesPerBlock - 1) / kTrainSamplesPerBlock); }

hipError_t launch_train_fwd_bwd(const float* queries, const float* targets, int64_t b, float n_total,
                                float loss_scale, const _Float16* wf, const _Float16* wb, float* slabs,
                                float* loss_partials, hipStream_t s, int enc) {
    if (b <= 0) return hipSuccess;
    if (enc == 2)
        hipLaunchKernelGGL((train_kernel<false, 2>), dim3(train_blocks(b)), dim3(256), 0, s, queries, targets, b,
                           n_total, loss_scale, (const h8*)wf, (const h8*)wb, slabs, loss_partials, nullptr, nullptr,
                           nullptr);
    else
        hipLaunchKernelGGL(train_kernel<false>, dim3(train_blocks(b)), dim3(256), 0, s, queries, targets, b, n_total,
                           loss_scale, (const h8*)wf, (const h8*)wb, slabs, loss_partials, nullptr, nullptr, nullptr);
    return hipGetLastError();
}

#if NRC_DEBUG_KERNELS
hipError_t launch_train_stamped(const float* queries, const float* targets, int64_t b, float n_total, float loss_scale,
                                const _Float16* wf, const _Float16* wb, float* slabs, float* loss_partials,
                                uint64_t* stamps, hipStream_t s) {
    if (b <= 0) return hipSuccess;
    hipLaunchKernelGGL(train_kernel<true>, dim3(train_blocks(b)), dim3(256), 0, s, queries, targets, b, n_total,
                       loss_scale, (const h8*)wf, (const h8*)wb, slabs, loss_partials, stamps);
    return hipGetLastError();
}

#else
hipError_t launch_train_stamped(const float*, const float*, int64_t, float, float, const _Float16*, const _Float16*, float*,
                                float*, uint64_t*, hipStream_t) {
    return hipErrorNotSupported;
}
#endif

// Sparse Adam + EMA + f16 table packs for the HashGrid parameters (tcnn non-matrix params, SURVEY §8(f) row 3;
// oracle/nrc_hash_oracle.c orc_hash_adam_ema): an entry whose gradient is exactly zero keeps its moments, weight
// and step counter; bias correction uses the entry's own step. The fused mode reads the f16 gradient the training
// kernel accumulated and zeroes it for the next step; kApplyOnly reads a caller's (all-reduced) f32 gradient
// without writing it.
// An exact fixed-point sum (value x 2^24, grid_scatter_kernel) rounded once to f16, nearest-even; overflow -> inf.
__device__ __forceinline__ _Float16 fixed_to_f16(int64_t v) {
    const uint32_t sign = v < 0 ? 0x8000u : 0u;
    const uint64_t a = v < 0 ? (uint64_t)(-v) : (uint64_t)v;
    if (a < 1024u) return __builtin_bit_cast(_Float16, (uint16_t)(sign | (uint32_t)a));  // subnormal / zero: exact
    const int msb = 63 - __builtin_clzll(a), shift = msb - 10;  // keep 11 significant bits
    uint64_t mant = shift > 0 ? a >> shift : a;
    if (shift > 0) {
        const uint64_t rem = a & ((1ull << shift) - 1), half = 1ull << (shift - 1);
        if (rem > half || (rem == half && (mant & 1u))) ++mant;
    }
    int be = shift + 1;  // biased exponent: value = mant / 1024 * 2^(shift - 14)
    if (mant == 2048u) {
        mant = 1024u;
        ++be;
    }
    if (be >= 31) return __builtin_bit_cast(_Float16, (uint16_t)(sign | 0x7C00u));
    return __builtin_bit_cast(_Float16, (uint16_t)(sign | ((uint32_t)be << 10) | (uint32_t)(mant - 1024u)));
}

// the value of a non-finite code (GridNonFinite)
__device__ __forceinline__ float nonfinite_value(uint32_t code) {
    return code == 1u ? __builtin_inff() : code == 2u ? -__builtin_inff() : __builtin_nanf("");
}

// parameter i's non-finite code of the step tagged nf.tag (0 if none), cleared for the next step
__device__ __forceinline__ uint32_t take_nonfinite(const GridNonFinite& nf, int i) {
    if (!nf.codes || __hip_atomic_load(nf.tag_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != nf.tag) return 0u;
    const uint32_t c = nf.codes[i];
    if (c) nf.codes[i] = 0;
    return c;
}

// the f16 gradient of an exact sum and its non-finite code
__device__ __forceinline__ float fixed_gradient(int64_t v, uint32_t code) {
    return code ? nonfinite_value(code) : (float)fixed_to_f16(v);
}

constexpr int64_t kFixedSat = 1ll << 41, kFixedOff = 1ll << 47;
__device__ __forceinline__ int64_t fixed_encode(int64_t v, uint32_t code) {
    v = v < -kFixedSat ? -kFixedSat : (v > kFixedSat ? kFixedSat : v);
    return v + ((code & 1u) ? (1ll << 48) : 0ll) + ((code & 2u) ? (1ll << 55) : 0ll);
}
__device__ __forceinline__ float fixed_decode_gradient(int64_t e) {
    const uint64_t u = (uint64_t)(e + kFixedOff);
    const uint32_t code = (((u >> 48) & 127u) ? 1u : 0u) | (((u >> 55) & 127u) ? 2u : 0u);
    return fixed_gradient((int64_t)(u & ((1ull << 48) - 1)) - kFixedOff, code);
}

// tcnn's grid Adam for parameter i with this step's gradient (already divided by the loss scale): an exactly-zero
// gradient keeps moments, weight and the entry's own step counter (no l2); the EMA over every entry, and the two f16
// tables repacked. The state is loaded first and unconditionally (grid_adam_load: the moments of an untouched entry too),
// so that every load of a parameter is in flight before its gradient is known and before any store (the conditional
// loads after the gradient made grid_adam_kernel a chain of memory round trips per parameter; measured neutral, 56.2 vs
// 56.5 us per Hash step; in the merged hash_adam_kernel the conditional loads read 1.6 MB less and took 13.7 vs 13.4 us).
struct GridAdamIn {
    float w, m, v, e;
    uint32_t st;
};
__device__ __forceinline__ GridAdamIn grid_adam_load(int i, const GridBuffers& gb) {
    return GridAdamIn{gb.params[i], gb.m[i], gb.v[i], gb.ema[i], gb.steps[i]};
}
__device__ __forceinline__ void grid_adam_step(int i, float gradient, const GridAdamIn& a, const GridBuffers& gb,
                                               const OptimArgs& oa, float ema_debias) {
#pragma clang fp contract(off)
    float w = a.w;
    if (gradient != 0.0f) {
        const float am = a.m, av = a.v;
        const uint32_t st = a.st + 1u;
        gb.steps[i] = st;
        // two powf per parameter made this kernel VALU-bound (~12 us per step): table lookup instead
        float s2, d1;
        if (st <= gb.bias_len) {
            const float2 bc = gb.bias[st];
            s2 = bc.x;
            d1 = bc.y;
        } else {
            s2 = sqrtf(1.0f - powf(oa.beta2, (float)st));
            d1 = 1.0f - powf(oa.beta1, (float)st);
        }
        const float lr_i = oa.lr * s2 / d1;
        const float gsq = gradient * gradient;
        const float m1 = oa.beta1 * am + (1.0f - oa.beta1) * gradient;
        const float v1 = oa.beta2 * av + (1.0f - oa.beta2) * gsq;
        gb.m[i] = m1;
        gb.v[i] = v1;
        const float eff = lr_i / (sqrtf(v1) + oa.eps);
        w = w - eff * m1;
        gb.params[i] = w;
    }
    const float e = a.e * oa.ema_decay + w * (1.0f - oa.ema_decay);
    gb.ema[i] = e;
    const float inf = e / ema_debias;
    gb.infer[i] = inf;
    gb.table_train[i] = (_Float16)w;
    gb.table_infer[i] = (_Float16)inf;
}

__device__ __forceinline__ void grid_adam_body(const int blk, int mode, const GridBuffers& gb, const OptimArgs& oa,
                                               float ema_debias) {
#pragma clang fp contract(off)
    const int i = blk * 256 + threadIdx.x;
    if (i >= gb.n) return;
    if (mode == kPackOnly) {
        gb.table_train[i] = (_Float16)gb.params[i];
        gb.table_infer[i] = (_Float16)gb.infer[i];
    } else {
        const GridAdamIn a = grid_adam_load(i, gb);
        float gradient;
        if (mode == kApplyOnly) {
            gradient = gb.grad32[i] / oa.loss_scale;
        } else if (mode == kApplyFixed) {
            gradient = fixed_decode_gradient(gb.fixed[i]) / oa.loss_scale;
            if (gb.fixed == gb.grad64) gb.grad64[i] = 0;
        } else {
            // the step's exact sum: the level's per-slice partials (grid_scatter_kernel's plain-store levels, round 5)
            // added in slice order, else the atomic accumulator (zeroed for the next step); exact int64 either way
            // level and table part are block-uniform (256 parameters per block, 8,192 / 16,384 per part)
            const int l = __builtin_amdgcn_readfirstlane(i < 8192 ? 0 : 1 + ((i - 8192) >> 16));
            int64_t sum = 0;
            if (gb.part.base && gb.part.nslice[l]) {
                const int j = i - (l == 0 ? 0 : 8192 + ((l - 1) << 16)), stride = l == 0 ? 8192 : 65536;
                const int nparts = l == 0 ? 1 : NRC_HASH_T / 8192;
                const int part = __builtin_amdgcn_readfirstlane(j / (2 * 8192));
                const int ns = gb.part.nslice[l];
                // every slice's form flag (scalar loads), then every slice's partial, branch-free: an int32 element is
                // read as the aligned 8-byte pair holding it (the lanes of a wave still read each line once)
                uint32_t wide = 0;
#pragma unroll
                for (int sl = 0; sl < kMaxPartialSlices; ++sl)
                    wide |= (sl < ns ? gb.part.flags[gb.part.foff[l] + min(sl, ns - 1) * nparts + part] : 0u) << sl;
                const int64_t* src = gb.part.base + gb.part.off[l] + j;
                const int64_t* src32 = reinterpret_cast<const int64_t*>(gb.part.base32 + gb.part.off[l] + (j & ~1));
                int64_t v[kMaxPartialSlices];
#pragma unroll
                for (int sl = 0; sl < kMaxPartialSlices; ++sl) {
                    const int sc = min(sl, ns - 1);
                    const bool w = (wide >> sc) & 1u;
                    const int64_t raw = *(w ? src + (int64_t)sc * stride : src32 + (int64_t)sc * (stride / 2));
                    v[sl] = w ? raw : (int64_t)(int32_t)(uint32_t)(raw >> (32 * (j & 1)));
                }
#pragma unroll
                for (int sl = 0; sl < kMaxPartialSlices; ++sl) sum += sl < ns ? v[sl] : 0;
            } else {
                sum = gb.grad64[i];
                gb.grad64[i] = 0;
            }
            gradient = fixed_gradient(sum, take_nonfinite(gb.nf, i)) / oa.loss_scale;
        }
        grid_adam_step(i, gradient, a, gb, oa, ema_debias);
    }
}

__global__ __launch_bounds__(256) void grid_adam_kernel(int mode, GridBuffers gb, OptimArgs oa, float ema_debias) {
    grid_adam_body(blockIdx.x, mode, gb, oa, ema_debias);
}

hipError_t launch_grid_adam(int mode, const GridBuffers& gb, const OptimArgs& oa, hipStream_t s) {
    const float step = (float)(oa.step ? oa.step : 1);
    const float ema_debias = 1.0f - powf(oa.ema_decay, step);
    hipLaunchKernelGGL(grid_adam_kernel, dim3((unsigned)((gb.n + 255) / 256)), dim3(256), 0, s, mode, gb, oa,
                       ema_debias);
    return hipGetLastError();
}

// Data-parallel export of the grid gradient: the f16-rounded exact sum as f32 into the exchange buffer, the fixed-point
// accumulator zeroed for the next step.
__global__ __launch_bounds__(256) void grid_grad_export_kernel(int64_t* __restrict__ g64, float* __restrict__ g32,
                                                               int n, GridNonFinite nf) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    g32[i] = fixed_gradient(g64[i], take_nonfinite(nf, i));
    g64[i] = 0;
}

hipError_t launch_grid_grad_export(int64_t* g64, float* g32, int n, const GridNonFinite& nf, hipStream_t s) {
    hipLaunchKernelGGL(grid_grad_export_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g64, g32, n, nf);
    return hipGetLastError();
}

// the exact sums in the exchange encoding (kFixedMaxRanks); in place when out == g64
__global__ __launch_bounds__(256) void grid_grad_export_fixed_kernel(int64_t* g64, int64_t* out, int n,
                                                                     GridNonFinite nf) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int64_t v = g64[i];
    out[i] = fixed_encode(v, take_nonfinite(nf, i));
    if (out != g64) g64[i] = 0;
}

hipError_t launch_grid_grad_export_fixed(int64_t* g64, int64_t* out, int n, const GridNonFinite& nf, hipStream_t s) {
    hipLaunchKernelGGL(grid_grad_export_fixed_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g64, out, n,
                       nf);
    return hipGetLastError();
}

// Trilinear grid-gradient scatter (tcnn kernel_grid_backward), deterministic. Block = (level, quarter of the level's
// table, slice of the step's samples): it recomputes each sample's 8 corners at its level and adds w_corner * dy (each
// product rounded to f16, as tcnn's half2 atomicAdd sees it) to an LDS copy of its quarter table as an exact
// fixed-point integer (f16 value x 2^24: every f16 is an integer multiple of 2^-24, |value| < 2^16, so a step's sum
// fits 64 bits), then flushes the touched entries with one 64-bit global integer atomic each, in entry order.
// Integer addition is associative: the sums are exact and the same in every run whatever the order of the adds
// (round 1 accumulated in f16 with packed-half atomics, which made Hash training order-dependent). grid_adam_kernel
// rounds each exact sum to f16 once (fixed_to_f16) -- the oracle's f64 sum rounded to f16
// (oracle/nrc_hash_oracle.c) -- and zeroes it.
// On MI355X device-scope atomics execute at the memory side and 64 lanes adding to 64 random rows run ~17x below the
// contiguous rate (MI355X_MICROARCH.md § Global float atomics): the random adds stay in the CU and the global ones
// walk the table in order. The slice length is per level: the coarse levels cover the scene with a handful of cells
// (position * 0.005 spans ~1.6 * 2^l cells per axis), so their LDS adds collide on a few addresses and serialise --
// a block's time grows with (slice samples / touched entries) -- while a fine level's block costs mostly its
// table flush. So the slice doubles per level from `min` to `max`.
// Round 5: from level kScatterPartFirst (knob scatter_part) a block stores its part of its slice densely as per-slice
// partial sums instead of the atomic flush (ScatterPartials, int32 where every sum fits), summed by grid_adam_kernel.
constexpr int kScatterThreads = 1024, kScatterPart = 8192, kScatterPer = 2;
struct ScatterPlan {
    int first_block[NRC_HASH_LEVELS + 1];  // level l owns blocks [first_block[l], first_block[l + 1])
    int slice[NRC_HASH_LEVELS];            // samples per block at level l
    int compact_first;                     // levels from here queue their in-part corners (below: direct adds)
};
constexpr int scatter_parts(int level) { return level == 0 ? 1 : NRC_HASH_T / kScatterPart; }

// finite f16 value (bits) x 2^24 as an exact integer (inf / NaN are routed to GridNonFinite by the caller)
__device__ __forceinline__ int64_t f16_to_fixed(uint32_t h) {
    const uint32_t e = (h >> 10) & 31u, m = h & 1023u;
    const int64_t mag = e == 0 ? (int64_t)m : (int64_t)(m | 1024u) << (e - 1);
    return (h & 0x8000u) ? -mag : mag;
}
// the same integer in 4 VALU for |value| < 128 (the scatter's usual case): the f16 is exact in f32, x 2^24 is exact,
// and the result, an integer below 2^31, converts exactly to int32; larger values take the bit-field path above
__device__ __forceinline__ int64_t f16_to_fixed_fast(uint32_t h) {
    if ((h & 0x7FFFu) >= 0x5800u) return f16_to_fixed(h);  // |value| >= 128 (f16 exponent field >= 22)
    const float f = (float)__builtin_bit_cast(_Float16, (uint16_t)h) * 16777216.0f;
    return (int64_t)(int32_t)f;
}

// Round 5: the corners are compacted before their fixed-point adds. A block owns one table part (a quarter of a fine
// level), so each lane's 8 corners land in it with probability 1/4 at the fine levels -- but the f16 -> fixed-point
// conversion and the 64-bit LDS add of a corner ran for the whole wave whenever one lane needed them (exec-masked
// branches), and the kernel was VALU-bound (PMC: VALU busy ~70 % of its 19.6 us). Now each wave appends the in-part
// corners' (entry, contribution pair) words to its own LDS queue (ballot + mbcnt offsets) and drains the queue with
// all 64 lanes busy when it holds more than kScatterQueue - 64 words, and at the end. The sums are the same exact
// integers (integer adds in any order). Only the fine levels (knob scatter_compact, default kScatterCompactFirst):
// at the coarse ones a block's part holds all 8 corners of most samples, on a few entries, and the queued adds of a
// drain then collide on them at once.
constexpr int kScatterQueue = 192;  // words per wave: 16 waves x 192 x 8 B = 24 KiB beside the 128-KiB table

// bcap: the workspace's row stride (its capacity; the plan's slices may end before it); b: the step's samples -- the
// training kernel writes positions and dy for the samples of its blocks only (64-sample blocks may end before the
// plan's last slice), so the ones past b are not read
__global__ __launch_bounds__(kScatterThreads) void grid_scatter_kernel(const float4* __restrict__ pos,
                                                                       const uint32_t* __restrict__ dy, int64_t bcap,
                                                                       int64_t b, ScatterPlan plan,
                                                                       unsigned long long* __restrict__ grad,
                                                                       GridNonFinite nf, ScatterPartials pt) {
    __shared__ unsigned long long acc[kScatterPart][2];  // 128 KiB: one block per CU
    __shared__ uint64_t queue[kScatterThreads / 64][kScatterQueue];
    int level = 0;
#pragma unroll
    for (int l = 1; l < NRC_HASH_LEVELS; ++l) level += (int)blockIdx.x >= plan.first_block[l];
    const int local = (int)blockIdx.x - plan.first_block[level];
    const int nparts = level == 0 ? 1 : NRC_HASH_T / kScatterPart;
    const int part = local % nparts;
    const int64_t slice = plan.slice[level], s0 = (int64_t)(local / nparts) * slice;
    const uint32_t lbase = NRC_HASH_LEVEL_ENTRY_OFFSET(level), lsize = level == 0 ? 4096u : (uint32_t)NRC_HASH_T;
    const uint32_t e0 = (uint32_t)part * kScatterPart;
    const uint32_t ne = min((uint32_t)kScatterPart, lsize - e0);
    const uint32_t* dyl = dy + (int64_t)level * bcap;
    const int64_t s1 = min(min(bcap, b), s0 + slice);
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t* const q = queue[threadIdx.x >> 6];
    uint32_t qn = 0;  // words in this wave's queue (wave-uniform)
    // the first batch's loads are issued before the table is zeroed (their latency hides behind it)
    uint32_t dv[kScatterPer];
    float4 p[kScatterPer];
    int64_t s = s0 + threadIdx.x;
    auto load = [&]() {
#pragma unroll
        for (int j = 0; j < kScatterPer; ++j) {
            const int64_t sj = s + (int64_t)j * kScatterThreads;
            dv[j] = sj < s1 ? dyl[sj] : 0u;
            p[j] = sj < s1 ? pos[sj] : float4{0.0f, 0.0f, 0.0f, 0.0f};
        }
    };
    // every queued word: (entry - e0) << 32 | the f16 contribution pair; the wave's own LDS writes are read back by
    // other lanes of the same wave (LDS executes a wave's instructions in order; the fence keeps the compiler's order)
    // the fixed-point adds of one corner's contribution pair cb at table entry e0 + e
    auto add = [&](const uint32_t e, const uint32_t cb) {
#pragma unroll
        for (int f = 0; f < 2; ++f) {
            const uint32_t hb = (cb >> (16 * f)) & 0xFFFFu;
            if ((hb & 0x7C00u) == 0x7C00u) {
                // inf / NaN: no fixed-point value; recorded for the kernels that round the sums
                const uint32_t gi = 2u * (lbase + e0 + e) + (uint32_t)f;
                const uint32_t code = (hb & 0x3FFu) ? 3u : ((hb & 0x8000u) ? 2u : 1u);
                atomicOr(reinterpret_cast<uint32_t*>(nf.codes) + (gi >> 2), code << (8u * (gi & 3u)));
                __hip_atomic_store(nf.tag_dev, nf.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (hb & 0x7FFFu) {
                atomicAdd(&acc[e][f], (unsigned long long)f16_to_fixed_fast(hb));
            }
        }
    };
    const bool compact = level >= plan.compact_first;
    auto drain = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t t = lane; t < qn; t += 64) {
            const uint64_t w = q[t];
            add((uint32_t)(w >> 32), (uint32_t)w);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        qn = 0;
    };
    load();
    for (uint32_t i = threadIdx.x; i < ne; i += kScatterThreads) acc[i][0] = acc[i][1] = 0ull;
    __syncthreads();
    for (;;) {
#pragma unroll
        for (int j = 0; j < kScatterPer; ++j) {
            const h2v d = __builtin_bit_cast(h2v, dv[j]);
            const float dy0 = (float)d[0], dy1 = (float)d[1];
            const bool active = (dv[j] & 0x7FFF7FFFu) != 0u;  // not both dy zero (also the samples past the slice)
            HashCorners C;
            if (level <= 1) hash_corners<true>(p[j].x, p[j].y, p[j].z, level, C);
            else hash_corners<false>(p[j].x, p[j].y, p[j].z, level, C);
#pragma unroll
            for (int cc = 0; cc < 8; ++cc) {
                const uint32_t e = C.entry[cc] - lbase - e0;
                // w * dy rounded to f32, then to f16 (tcnn's half2 product): the empty asm keeps the compiler from
                // fusing the two roundings into one v_fma_mixlo_f16 (another number in double-rounding cases)
                float w0 = C.w[cc] * dy0, w1 = C.w[cc] * dy1;
                asm volatile("" : "+v"(w0), "+v"(w1));
                const h2v c = {(_Float16)w0, (_Float16)w1};
                const uint32_t cb = __builtin_bit_cast(uint32_t, c);
                const bool in = active && e < ne && (cb & 0x7FFF7FFFu) != 0u;  // zero contributions add nothing
                if (compact) {  // block-uniform
                    const uint64_t m = __ballot(in);
                    if (m) {  // wave-uniform
                        const uint32_t off =
                            __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        if (in) q[qn + off] = ((uint64_t)e << 32) | cb;
                        qn += (uint32_t)__popcll(m);
                        if (qn > (uint32_t)(kScatterQueue - 64)) drain();
                    }
                } else if (in) {
                    add(e, cb);
                }
            }
        }
        s += (int64_t)kScatterPer * kScatterThreads;
        if (s0 + (s - s0 - threadIdx.x) >= s1) break;  // block-uniform
        load();
    }
    if (qn) drain();
    __syncthreads();
    if (pt.base && pt.nslice[level]) {
        // round 5, the fine levels (most entries touched): this block's part of its slice stored densely, zeros
        // included, with plain 16-byte stores instead of memory-side atomics; grid_adam_kernel sums the slices. As
        // int32 when every sum of the part fits (half the bytes), else as int64 (flagged)
        const int sl = local / nparts;
        bool wide = false;
        for (uint32_t i = threadIdx.x; i < ne; i += kScatterThreads) {
            const int64_t v0 = (int64_t)acc[i][0], v1 = (int64_t)acc[i][1];
            wide = wide || v0 != (int64_t)(int32_t)v0 || v1 != (int64_t)(int32_t)v1;
        }
        const bool any_wide = __syncthreads_or(wide) != 0;
        const int64_t el = pt.off[level] + (int64_t)sl * 2 * lsize + 2 * e0;
        if (any_wide) {
            typedef long long i2v __attribute__((ext_vector_type(2)));
            i2v* const dst = reinterpret_cast<i2v*>(pt.base + el);
            for (uint32_t i = threadIdx.x; i < ne; i += kScatterThreads)
                dst[i] = i2v{(long long)acc[i][0], (long long)acc[i][1]};
        } else {
            typedef int i4v __attribute__((ext_vector_type(4)));
            i4v* const dst = reinterpret_cast<i4v*>(pt.base32 + el);  // two entries per 16-byte store
            for (uint32_t i = threadIdx.x; 2 * i < ne; i += kScatterThreads)
                dst[i] = i4v{(int)acc[2 * i][0], (int)acc[2 * i][1], (int)acc[2 * i + 1][0], (int)acc[2 * i + 1][1]};
        }
        if (threadIdx.x == 0) pt.flags[pt.foff[level] + sl * nparts + part] = any_wide ? 1u : 0u;
        return;
    }
    for (uint32_t i = threadIdx.x; i < 2 * ne; i += kScatterThreads) {
        const unsigned long long v = acc[i >> 1][i & 1];
        if (v) __hip_atomic_fetch_add(grad + 2 * (uint64_t)(lbase + e0) + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// the plan of launch_train_hash (slice per level: min(smax, smin << l)) and the partial-sum layout it implies
static ScatterPlan scatter_plan(int64_t bcap, int& nb) {
    const int kmin = knob(kKnobScatterMin), kmax = knob(kKnobScatterMax);
    const int smin = kmin > 0 ? kmin : 2048, smax = kmax > 0 ? kmax : 4096;
    ScatterPlan plan;
    nb = 0;
    for (int l = 0; l < NRC_HASH_LEVELS; ++l) {
        const int sl = (int)std::min<int64_t>((int64_t)smax, (int64_t)smin << l);
        plan.first_block[l] = nb;
        plan.slice[l] = sl;
        nb += scatter_parts(l) * (int)((bcap + sl - 1) / sl);
    }
    plan.first_block[NRC_HASH_LEVELS] = nb;
    const int kc = knob(kKnobScatterCompact);
    plan.compact_first = kc >= 0 ? kc : kScatterCompactFirst;
    return plan;
}

ScatterPartials scatter_partials_layout(int64_t b, int first_level) {
    const int64_t bcap = (int64_t)train_blocks(b) * kTrainSamplesPerBlock;
    int nb = 0;
    const ScatterPlan plan = scatter_plan(bcap, nb);
    ScatterPartials p;
    for (int l = first_level; l < NRC_HASH_LEVELS; ++l) {
        const int ns = (int)((bcap + plan.slice[l] - 1) / plan.slice[l]);
        if (ns > kMaxPartialSlices) continue;  // a large batch: the atomic flush (partials would grow with the batch)
        p.off[l] = p.total;
        p.foff[l] = p.nflags;
        p.nslice[l] = ns;
        p.total += (int64_t)ns * 2 * (l == 0 ? 4096 : NRC_HASH_T);
        p.nflags += ns * scatter_parts(l);
    }
    return p;
}

hipError_t launch_train_hash(const float* queries, const float* targets, int64_t b, float n_total, float loss_scale,
                             const _Float16* wf, const _Float16* wb, const _Float16* grid, int64_t* grid_grad,
                             float* slabs, float* loss_partials, hipStream_t s, const HashScatter* sc, bool padq,
                             bool t16, uint32_t* feat, int groups) {
    if (b <= 0) return hipSuccess;
    const int blocks = train_blocks(b);
    // bcap: the samples the scatter plan covers (128-sample blocks); the workspace's row stride is its capacity
    // sc->bcap (>= bcap), the same for every writer and reader (nrc_debug_hash_scatter_inputs too)
    const int64_t bcap = (int64_t)blocks * kTrainSamplesPerBlock, stride = sc ? sc->bcap : 0;
    if (!sc || !sc->pos || !sc->dy || stride < bcap || !sc->nf.codes || !sc->nf.tag_dev || !sc->nf.tag)
        return hipErrorInvalidValue;
    if (t16) {  // round 5: the t16 role-split kernel (nrc_train16.hip), f16 slabs in the t16 layout
        const uint32_t* g = reinterpret_cast<const uint32_t*>(grid);
        // the batch's level features first, one level table per block in LDS (hash_feature_kernel, as for inference):
        // the training kernel's 128 blocks would otherwise gather 2 M table entries at their CUs' L1 line rate.
        // feat null: the 128-sample gathering encoder (ENC 1, groups 2). A batch larger than the feature workspace
        // (kHashFeatStride samples) runs in chunks of that many: per chunk the feature pass, then the
        // training kernel over the chunk's samples with its slabs, loss partials and scatter rows offset -- block i of
        // chunk c is block c0 / (64 groups) + i of the whole batch, the same slabs as one launch would write.
        // P = 8 query ranges per level (the minimum of the kernel's block map): 16,384-sample step 63.7 us vs 63.9 (16)
        // and 67.8 (32), profiles/r05_hash/
        if (!feat && (groups != 2 || padq)) return hipErrorNotSupported;  // no padded / 64-sample gathering instance
        const int64_t chunk = feat ? kHashFeatStride : b;
        static_assert(kHashFeatStride % 128 == 0, "chunks start on a block boundary of either block size");
        const int qd = padq ? NRC_INPUT_DIMS_PADDED : NRC_INPUT_DIMS;
        for (int64_t c0 = 0; c0 < b; c0 += chunk) {
            const int64_t cnt = std::min<int64_t>(chunk, b - c0);
            const float* qc = queries + c0 * qd;
            if (feat) {
                // the gather pass by default: fused step 54.3 vs 55.8 us with the LDS pass, parameters bitwise equal
                // (profiles/r05_hash/ab_train_feature_gather.json)
                if (knob(kKnobHashTrainFeat) != 0) launch_hash_feature_gather(qc, cnt, g, feat, padq, s);
                else launch_hash_feature_pass(qc, cnt, g, feat, padq, s, 8);
            }
            const int64_t blk0 = c0 / (64 * groups);
            const hipError_t e = launch_train16_hash(
                qc, targets + c0 * 3, cnt, n_total, loss_scale, wf, wb,
                reinterpret_cast<_Float16*>(slabs) + blk0 * slab_floats(0), loss_partials + blk0,
                HashTrainOut{g, feat, sc->pos + c0, sc->dy + c0, stride}, s, padq, groups);
            if (e != hipSuccess) return e;
        }
    } else if (padq)
        hipLaunchKernelGGL((train_kernel<false, 1, true>), dim3(blocks), dim3(256), 0, s, queries, targets, b, n_total,
                           loss_scale, (const h8*)wf, (const h8*)wb, slabs, loss_partials, nullptr,
                           reinterpret_cast<const uint32_t*>(grid), nullptr, sc->pos, sc->dy, stride);
    else
        hipLaunchKernelGGL((train_kernel<false, 1>), dim3(blocks), dim3(256), 0, s, queries, targets, b, n_total,
                           loss_scale, (const h8*)wf, (const h8*)wb, slabs, loss_partials, nullptr,
                           reinterpret_cast<const uint32_t*>(grid), nullptr, sc->pos, sc->dy,
                           stride);
    // tuning overrides (A/B knobs scatter_min / scatter_max); defaults from the sweep of the exact 64-bit scatter,
    // profiles/r03_hash/scatter_plan_sweep.txt (round 1's f16 scatter: profiles/r01_hash/README.md)
    int nb = 0;
    const ScatterPlan plan = scatter_plan(bcap, nb);
    if (sc->part.base) {  // the partial layout must be this plan's (levels without slices flush with atomics)
        int first = 0;
        while (first < NRC_HASH_LEVELS && !sc->part.nslice[first]) ++first;
        const ScatterPartials want = scatter_partials_layout(b, first);
        for (int l = 0; l < NRC_HASH_LEVELS; ++l)
            if (want.off[l] != sc->part.off[l] || want.nslice[l] != sc->part.nslice[l]) return hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(grid_scatter_kernel, dim3(nb), dim3(kScatterThreads), 0, s, sc->pos, sc->dy, stride, b, plan,
                       reinterpret_cast<unsigned long long*>(grid_grad), sc->nf, sc->part);
    return hipGetLastError();
}

void adam_host_factors(const OptimArgs& oa, float& lr_t, float& ema_debias) {
    // Bias corrections in host f32 (glibc powf/sqrtf), identical to the oracle's.
    const float step = (float)(oa.step ? oa.step : 1);
    lr_t = oa.lr * sqrtf(1.0f - powf(oa.beta2, step)) / (1.0f - powf(oa.beta1, step));
    ema_debias = 1.0f - powf(oa.ema_decay, step);
}

// Round 5: the fused Hash step's two optimizer updates in one launch: blocks [0, nred) reduce the MLP's f16 slabs and
// apply its Adam/EMA (reduce_adam_body, the latency-bound part), the rest apply the grid Adam (grid_adam_body, the
// memory-bound part), so that the MLP update runs beside the grid's instead of after it, behind one kernel boundary
// instead of two. Both bodies are inlined (a first version with noinline halves took 75 us per step) and the same
// float operations as their own launches: the state is bitwise that of launch_reduce_adam + launch_grid_adam (leaving
// the grid's f32 inference copy to a refresh before reads measured no faster: 50.59 vs 50.63 us per step).
__global__ __launch_bounds__(kRedThreads) void hash_adam_kernel(int nred, const float* __restrict__ slabs, int nslabs,
                                                                const float* __restrict__ loss_partials,
                                                                float* __restrict__ loss_out, ModelBuffers mb,
                                                                OptimArgs oa, float lr_t, float ema_debias,
                                                                GridBuffers gb, float grid_ema_debias) {
    static_assert(kRedThreads == 256, "the grid Adam's blocks are 256 threads");
    if ((int)blockIdx.x < nred)
        reduce_adam_body<true>(blockIdx.x, kReduceFused, slabs, nslabs, loss_partials, nullptr, loss_out, mb, oa, lr_t,
                               ema_debias);
    else
        grid_adam_body((int)blockIdx.x - nred, kReduceFused, gb, oa, grid_ema_debias);
}

hipError_t launch_hash_adam(const float* slabs, int nslabs, const float* loss_partials, float* loss_out,
                            const ModelBuffers& mb, const GridBuffers& gb, const OptimArgs& oa, hipStream_t s) {
    if (!mb.slab_f16) return hipErrorInvalidValue;  // the t16 training kernel's f16 slabs
    float lr_t, ema_debias;
    adam_host_factors(oa, lr_t, ema_debias);
    const float grid_ema_debias = 1.0f - powf(oa.ema_decay, (float)(oa.step ? oa.step : 1));
    const int nred = mb.n_slab / (kRedParams * kRedVec), ngrid = (gb.n + 255) / 256;
    hipLaunchKernelGGL(hash_adam_kernel, dim3((unsigned)(nred + ngrid)), dim3(kRedThreads), 0, s, nred, slabs, nslabs,
                       loss_partials, loss_out, mb, oa, lr_t, ema_debias, gb, grid_ema_debias);
    return hipGetLastError();
}

hipError_t launch_reduce_adam(int mode, const float* slabs, int nslabs, const float* loss_partials, float* grad_io,
                              float* loss_out, const ModelBuffers& mb, const OptimArgs& oa, hipStream_t s) {
    float lr_t, ema_debias;
    adam_host_factors(oa, lr_t, ema_debias);
    // reduce modes walk the slab positions, apply / pack modes the parameters
    const int grid = (mode == kReduceFused || mode == kReduceOnly ? mb.n_slab : mb.n_mlp) / (kRedParams * kRedVec);
#if NRC_DEBUG_KERNELS
    if (mode == kReduceFused) g_last_clock_waves = std::min<int64_t>(grid, kInferClockWavesMax);
#endif
    if (mb.slab_f16)
        hipLaunchKernelGGL(reduce_adam_kernel<true>, dim3(grid), dim3(kRedThreads), 0, s, mode, slabs, nslabs, loss_partials,
                           grad_io, loss_out, mb, oa, lr_t, ema_debias);
    else
        hipLaunchKernelGGL(reduce_adam_kernel<false>, dim3(grid), dim3(kRedThreads), 0, s, mode, slabs, nslabs,
                           loss_partials, grad_io, loss_out, mb, oa, lr_t, ema_debias);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// One-shot peer gradient exchange of nrc_train_dp (round 4). Each rank owns a receive buffer
// (uncached device memory, exported by IPC handle): data [2 parities][world][stride] f32, then one flag per (parity,
// source rank), 64 B apart. A step with sequence number seq (parity seq & 1):
//   peer_push_kernel   block r copies this rank's gradient (NRC_GRAD_FLOATS incl. the loss slot) into slot [par][rank]
//                      of rank r's buffer (xGMI peer stores; r == rank: its own buffer), fences at system scope and
//                      releases flag [par][rank] = seq there;
//   peer_apply_kernel  waits (acquire, system scope) until every flag [par][*] of its own buffer reads seq, sums the
//                      world gradients in rank order (the same float operations on every rank: bitwise-identical
//                      replicas) and runs adam_pack_one (kApplyOnly) per parameter; block 0 sums the loss likewise.
// Two parities suffice: a rank writes parity p of a peer only after that peer's flag for the previous step of the
// other parity was seen by its own apply, which the peer issued after its apply of the step before (stream order).
// The wait is bounded (about 10 s, then error word 2 and NRC_ERR_INTERNAL): a missing peer ends the kernel.
// ------------------------------------------------------------------------------------------------
constexpr int kPeerFlagStride = 16;  // u32 per flag (64 B)
constexpr int kPeerSplit = 4;        // push blocks (and flags) per destination: each copies a quarter of the gradient
int peer_stride(int nfl) { return (nfl + 63) / 64 * 64; }

__global__ __launch_bounds__(1024) void peer_push_kernel(const float* __restrict__ grad, int nfl, PeerPtrs dst, int rank,
                                                         int world, int stride, uint32_t seq) {
    const int r = blockIdx.x / kPeerSplit, part = blockIdx.x % kPeerSplit, par = (int)(seq & 1u);
    const int n4 = nfl / 4, b4 = part * n4 / kPeerSplit, e4 = (part + 1) * n4 / kPeerSplit;
    const float4* s4 = reinterpret_cast<const float4*>(grad);
    float4* d4 = reinterpret_cast<float4*>(dst.p[r] + ((int64_t)par * world + rank) * stride);
    constexpr int kPer = 2;  // float4 per thread: a quarter of NRC_GRAD_FLOATS (1,409) over 1,024 threads
    float4 v[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) v[k] = s4[min(b4 + (int)threadIdx.x + 1024 * k, e4 - 1)];  // branch-free: both in flight
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = b4 + (int)threadIdx.x + 1024 * k;
        if (i < e4) d4[i] = v[k];
    }
    // The destination is uncached device memory: the stores bypass the L2, and their acknowledgements (vmcnt) mean
    // they have reached memory. Waiting for them, then the barrier, orders every thread's data before the flag -- with
    // no system-scope release fence, whose L2 write-back (all of this XCD's dirty lines: the training slabs) cost 4-8 us
    // per launch in the first version (profiles/r04_dp/).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t* const flags = reinterpret_cast<uint32_t*>(dst.p[r] + (int64_t)2 * world * stride);
        __hip_atomic_store(flags + ((par * world + rank) * kPeerSplit + part) * kPeerFlagStride, seq, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <int WMAX>  // the world's bucket (2, 4, 8, 16): the rank-order sum is unrolled over WMAX ranks
__global__ __launch_bounds__(256) void peer_apply_kernel(const float* __restrict__ xbuf, int world, int stride, uint32_t seq,
                                                         int polls, uint32_t* err, float* __restrict__ loss_out,
                                                         ModelBuffers mb, OptimArgs oa, float lr_t, float ema_debias) {
    const int par = (int)(seq & 1u);
    const int nflags = world * kPeerSplit;
    __shared__ uint32_t timed_out;
    if (threadIdx.x < 64) {
        // wave 0 polls every (source rank, part) flag, one per lane (lanes past them re-read flag 0): the loop is
        // wave-uniform (ballot) and holds no store (tests/test_asm_hazards.py rule 3). Relaxed system-scope polls of
        // uncached memory (no L2 invalidate per poll); the data loads below are issued after the flags have returned
        // (the barrier follows the loop) and read memory, not a cache. Fast polls first (~0.1 ms), then ~4 us apart:
        // about 10 s in all (polls = 2^21; the px_polls knob shortens it for tests).
        const int lane = threadIdx.x;
        const uint32_t* f = reinterpret_cast<const uint32_t*>(xbuf + (int64_t)2 * world * stride) +
                            (par * nflags + (lane < nflags ? lane : 0)) * kPeerFlagStride;
        int i = 0;
        for (; i < polls; ++i) {
            const bool ready = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == seq;
            if (__builtin_amdgcn_readfirstlane(__ballot(!ready) == 0ull)) break;
            if (i < 4096) __builtin_amdgcn_s_sleep(1);
            else __builtin_amdgcn_s_sleep(127);
        }
        if (lane == 0) timed_out = i == polls ? 1u : 0u;
    }
    __syncthreads();
    if (timed_out && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const float* const base = xbuf + (int64_t)par * world * stride;
    // peer-written uncached memory, read at system scope; the world sum in rank order, branch-free (a rank past the
    // world re-reads rank 0 and is not added)
    auto ld = [&](int r, int p) {
        return __hip_atomic_load(base + (int64_t)r * stride + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    };
    auto world_sum = [&](int p) {
        float v[WMAX];
#pragma unroll
        for (int r = 0; r < WMAX; ++r) v[r] = ld(r < world ? r : 0, p);
        float g = v[0];
#pragma unroll
        for (int r = 1; r < WMAX; ++r) g = r < world ? g + v[r] : g;
        return g;
    };
    if (blockIdx.x == 0 && threadIdx.x == 0 && loss_out) loss_out[0] = world_sum(mb.n_total);
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= mb.n_mlp) return;
    adam_pack_one(kApplyOnly, p, world_sum(p), mb, oa, lr_t, ema_debias);
}

// ------------------------------------------------------------------------------------------------
// The exchange fused into the reduction (round 4): one launch after the gradient pass replaces reduce (kReduceOnly) +
// peer_push_kernel + peer_apply_kernel. Block i of every rank reduces the same 64 slab positions (the slab map is the
// same on every rank), so the exchange runs per block: wave 0 of block i stores its 64 reduced partials -- slab order,
// one contiguous 512-B store per destination -- into slot [par][rank] of every rank's buffer, then polls its own
// buffer's slots [par][0..world) at its positions and sums the world's partials in rank order before the same
// Adam/EMA as kReduceFused. Every element is a tagged 8-byte word (f32 value | step sequence number << 32), written
// with one 64-bit store and read with one 64-bit load (single-copy atomic; RCCL's LL protocol rests on the same
// property of xGMI): a reader that sees the tag sees the value, so there is no flag, no store acknowledgement to wait
// for before a flag and no second load after it -- one memory round trip where the flag protocol took three (the
// first fused version: 10.8 us per world-1 step, profiles/r04_fused/). A block waits only for the blocks of the same
// index on the other ranks, which store before they wait: no cycle, whatever the residency (ranks sharing a device
// take the split form below). The Adam state is loaded with the slab loads, before the wait. Buffer layout after the
// push/apply region's (peer_buffer_bytes): [2][world][xstride] tagged words (slab order, the loss at n_slab). Two
// parities suffice as for the push/apply pair: a rank's step k kernel starts after all its blocks of step k - 1 saw
// every peer's step k - 1 words, which those peers stored after their step k - 2 kernels (and reads) had ended.
// ------------------------------------------------------------------------------------------------
__host__ __device__ constexpr int px_stride(int n_slab) { return (n_slab + 1 + 63) / 64 * 64; }
size_t px_region_offset(int world, int nfl) {
    return sizeof(float) * ((size_t)2 * world * peer_stride(nfl)) + sizeof(uint32_t) * 2 * world * kPeerSplit * kPeerFlagStride;
}
size_t peer_buffer_bytes(int world, int nfl, int n_slab) {
    return px_region_offset(world, nfl) + sizeof(uint64_t) * (size_t)2 * world * px_stride(n_slab);
}
__device__ __forceinline__ uint64_t px_word(float v, uint32_t seq) {
    return ((uint64_t)seq << 32) | (uint64_t)__builtin_bit_cast(uint32_t, v);
}

// Wave-level second half of the exchange for chunk blk (64 slab positions, one per lane; this wave's lane = position
// blk * 64 + lane): wait until every rank's word at the lane's position (and, for chunk 0, the loss) carries this step's
// tag, sum the world's partials in rank order, Adam/EMA. ain: the position's Adam state, loaded before the wait.
// Shared by the fused kernel and the split path's apply kernel. OWNREG (fused): this rank's own partial and loss are
// the registers mine / mine_l (never stored to nor read back from memory), so only the other ranks' words are awaited.
template <int WMAX, bool OWNREG>
__device__ __forceinline__ void exchange_wait_apply(const char* own, int lane, int blk, int par, int rank, int world,
                                                    int xstride, int pp, uint32_t seq, int polls, uint32_t* err,
                                                    float* loss_out,
                                                    float mine, float mine_l, const AdamIn& ain, const ModelBuffers& mb,
                                                    const OptimArgs& oa, float lr_t, float ema_debias) {
#pragma clang fp contract(off)
    const int mypos = blk * kRedParams * kRedVec + lane;
    // lane 0 of chunk 0 also waits for the loss words (position n_slab), every other lane re-reads its own position
    const bool has_loss = blk == 0 && lane == 0 && loss_out;
    const uint64_t* const xb = reinterpret_cast<const uint64_t*>(own) + (int64_t)par * world * xstride;
    uint64_t w[WMAX], wl[WMAX];
    int i = 0;
    // OWNREG at world 1: nothing to wait for (the loop would only re-read a row that is never awaited)
    for (; i < polls && !(OWNREG && world == 1); ++i) {
        bool ready = true;
#pragma unroll
        for (int r = 0; r < WMAX; ++r) {
            // a rank past the world (and, OWNREG, this rank) re-reads a row that is never awaited: the other rank's, so
            // that the loads stay branch-free
            const bool skip = r >= world || (OWNREG && r == rank);
            const int64_t row = (int64_t)(r < world ? r : 0) * xstride;
            w[r] = __hip_atomic_load(xb + row + mypos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            wl[r] = __hip_atomic_load(xb + row + (has_loss ? mb.n_slab : mypos), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_SYSTEM);
            ready = ready && (skip || ((uint32_t)(w[r] >> 32) == seq && (uint32_t)(wl[r] >> 32) == seq));
        }
        if (__builtin_amdgcn_readfirstlane(__ballot(!ready) == 0ull)) break;  // wave-uniform, no store in the loop
        if (i < 4096) __builtin_amdgcn_s_sleep(1);
        else __builtin_amdgcn_s_sleep(127);
    }
    if (i == polls && lane == 0) __hip_atomic_store(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if constexpr (OWNREG) {
#pragma unroll
        for (int r = 0; r < WMAX; ++r)
            if (r == rank) {
                w[r] = px_word(mine, seq);
                wl[r] = px_word(mine_l, seq);
            }
    }
    // the world sum in rank order (branch-free: a rank past the world is not added)
    auto world_sum = [&](const uint64_t (&v)[WMAX]) {
        float g = __builtin_bit_cast(float, (uint32_t)v[0]);
#pragma unroll
        for (int r = 1; r < WMAX; ++r) g = r < world ? g + __builtin_bit_cast(float, (uint32_t)v[r]) : g;
        return g;
    };
    const float gsum = world_sum(w);
    if (has_loss) loss_out[0] = world_sum(wl);
    if (pp < 0) return;  // padding position (dummy layer-0 K slots)
    adam_pack_pre(pp, gsum, ain, mb, oa, lr_t, ema_debias);
}

template <bool H, int WMAX, bool WAIT>
__global__ __launch_bounds__(kRedThreads) void reduce_exchange_kernel(const float* __restrict__ slabs, int nslabs,
                                                                      const float* __restrict__ loss_partials,
                                                                      PeerPtrs dst, size_t region, int rank, int world,
                                                                      uint32_t seq, int polls, uint32_t* err,
                                                                      float* loss_out, ModelBuffers mb, OptimArgs oa,
                                                                      float lr_t, float ema_debias) {
#pragma clang fp contract(off)
    typedef float f4 __attribute__((ext_vector_type(4)));
    __shared__ f4 part[kRedGroups][kRedParams];
    const int pl = threadIdx.x & (kRedParams - 1), grp = threadIdx.x / kRedParams;
    const int p0 = (blockIdx.x * kRedParams + pl) * kRedVec;
    const int par = (int)(seq & 1u), blk = blockIdx.x, nblk = gridDim.x;
    const int xstride = px_stride(mb.n_slab);
    float L = 0.0f;  // this rank's loss (block 0, wave 0)
    if (blockIdx.x == 0 && threadIdx.x < 64) {
        L = lane_partial_sum(loss_partials, nslabs, threadIdx.x);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) L += __shfl_xor(L, off, 64);
    }
    // slab sums as reduce_adam_kernel's reduce modes (same loads, same float sums, Adam state prefetched)
    const int mypos = blockIdx.x * kRedParams * kRedVec + (threadIdx.x & (kRedParams * kRedVec - 1));
    int pp_raw;
    if constexpr (H) pp_raw = t16_slab_param(mypos);
    else pp_raw = mb.slab_param[mypos];
    f4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
    auto ld = [&](int slab) -> f4 {
        if constexpr (H) {
            const h4 v = *(const h4*)((const _Float16*)slabs + (int64_t)slab * mb.n_slab + p0);
            return f4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
        } else {
            return *(const f4*)&slabs[(int64_t)slab * mb.n_slab + p0];
        }
    };
    const int nmine = grp < nslabs ? (nslabs - grp + kRedGroups - 1) / kRedGroups : 0;
    auto ldc = [&](int k) -> f4 { return ld(min(grp + k * kRedGroups, nslabs - 1)); };
    const int pp = threadIdx.x < kRedParams * kRedVec ? pp_raw : -1;
    AdamIn ain{};
    if (WAIT && pp >= 0) ain = adam_load(pp, mb);
    f4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ldc(u);
    asm volatile("" : "+v"(ain.fp), "+v"(ain.ft), "+v"(ain.bp));
    for (int base = 0;;) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const bool in = base + u < nmine;
            if (u & 1) a1 += in ? v[u] : f4{0.f, 0.f, 0.f, 0.f};
            else a0 += in ? v[u] : f4{0.f, 0.f, 0.f, 0.f};
        }
        base += 8;
        if (base >= nmine) break;
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = ldc(base + u);
    }
    part[grp][pl] = a0 + a1;
    __syncthreads();
    if (threadIdx.x >= kRedParams * kRedVec) return;
    // wave 0 from here: one slab position per lane
    const int lane = threadIdx.x, lp = lane / kRedVec, comp = lane % kRedVec;
    float t8[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t8[u] = part[2 * u][lp][comp] + part[2 * u + 1][lp][comp];
    const float g1 = ((t8[0] + t8[1]) + (t8[2] + t8[3])) + ((t8[4] + t8[5]) + (t8[6] + t8[7]));
    // push: slot [par][rank] of every rank as tagged words, then the loss (block 0); no wait, no flag (px_word). The
    // fused form keeps its own partials in registers (no own slot written or read); the split form's apply kernel
    // reads them back. dst.p is indexed by a wave-uniform rank: a per-lane index into the kernel-argument array would
    // go through scratch.
    const uint64_t word = px_word(g1, seq), lword = px_word(L, seq);
    for (int r = 0; r < world; ++r) {
        if (WAIT && r == rank) continue;
        uint64_t* const d = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(dst.p[r]) + region) +
                            ((int64_t)par * world + rank) * xstride;
        __hip_atomic_store(d + mypos, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (blk == 0 && lane == 0) __hip_atomic_store(d + mb.n_slab, lword, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if constexpr (WAIT)
        exchange_wait_apply<WMAX, true>(reinterpret_cast<const char*>(dst.p[rank]) + region, lane, blk, par, rank, world,
                                        xstride, pp, seq, polls, err, loss_out, g1, L, ain, mb, oa, lr_t, ema_debias);
    (void)nblk;
}

// The split path's second kernel: 4 waves per block, wave w of block b takes chunk 4b + w (the fused kernel's second
// half): 92 blocks of 256 threads for the Frequency slab, the footprint of round 4's first apply kernel.
template <bool H, int WMAX>
__global__ __launch_bounds__(256) void exchange_apply_kernel(const char* __restrict__ own, int nblk, int world,
                                                             uint32_t seq, int polls, uint32_t* err,
                                                             float* loss_out, ModelBuffers mb, OptimArgs oa,
                                                             float lr_t, float ema_debias) {
    const int lane = threadIdx.x & 63;
    const int blk = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    if (blk >= nblk) return;  // wave-uniform
    const int mypos = blk * kRedParams * kRedVec + lane;
    int pp;
    if constexpr (H) pp = t16_slab_param(mypos);
    else pp = mb.slab_param[mypos];
    AdamIn ain{};
    if (pp >= 0) ain = adam_load(pp, mb);
    exchange_wait_apply<WMAX, false>(own, lane, blk, (int)(seq & 1u), 0, world, px_stride(mb.n_slab), pp, seq, polls,
                                     err, loss_out, 0.0f, 0.0f, ain, mb, oa, lr_t, ema_debias);
}

hipError_t launch_reduce_exchange(const float* slabs, int nslabs, const float* loss_partials, const PeerPtrs& dst,
                                  int rank, int world, int nfl, uint32_t seq, uint32_t* err, float* loss_out,
                                  const ModelBuffers& mb, const OptimArgs& oa, hipStream_t s, int form, int polls) {
    if (world < 1 || world > kPeerMaxRanks || rank < 0 || rank >= world || !err || nslabs < 1 || polls < 1 ||
        form < kPxFused || form > kPxApplyOnly)
        return hipErrorInvalidValue;
    for (int r = 0; r < world; ++r)
        if (!dst.p[r]) return hipErrorInvalidValue;
    float lr_t, ema_debias;
    adam_host_factors(oa, lr_t, ema_debias);
    const int nblk = mb.n_slab / (kRedParams * kRedVec);
    const size_t region = px_region_offset(world, nfl);
    const char* own = reinterpret_cast<const char*>(dst.p[rank]) + region;
    const bool push = form != kPxApplyOnly, apply = form == kPxSplit || form == kPxApplyOnly;
#define NRC_RX(HH, W)                                                                                                   \
    do {                                                                                                                \
        if (form == kPxFused) {                                                                                         \
            hipLaunchKernelGGL((reduce_exchange_kernel<HH, W, true>), dim3(nblk), dim3(kRedThreads), 0, s, slabs,       \
                               nslabs, loss_partials, dst, region, rank, world, seq, polls, err, loss_out, mb, oa,      \
                               lr_t, ema_debias);                                                                       \
            break;                                                                                                      \
        }                                                                                                               \
        if (push)                                                                                                       \
            hipLaunchKernelGGL((reduce_exchange_kernel<HH, W, false>), dim3(nblk), dim3(kRedThreads), 0, s, slabs,      \
                               nslabs, loss_partials, dst, region, rank, world, seq, polls, err, loss_out, mb, oa,      \
                               lr_t, ema_debias);                                                                       \
        if (apply)                                                                                                      \
            hipLaunchKernelGGL((exchange_apply_kernel<HH, W>), dim3((nblk + 3) / 4), dim3(256), 0, s, own, nblk, world, \
                               seq, polls, err, loss_out, mb, oa, lr_t, ema_debias);                                    \
    } while (0)
#define NRC_RXW(HH)                     \
    if (world <= 2) NRC_RX(HH, 2);      \
    else if (world <= 4) NRC_RX(HH, 4); \
    else if (world <= 8) NRC_RX(HH, 8); \
    else NRC_RX(HH, 16)
    if (mb.slab_f16) {
        NRC_RXW(true);
    } else {
        NRC_RXW(false);
    }
#undef NRC_RXW
#undef NRC_RX
    return hipGetLastError();
}

hipError_t launch_peer_push(const float* grad, int nfl, const PeerPtrs& dst, int rank, int world, uint32_t seq,
                            hipStream_t s) {
    if (world < 2 || world > kPeerMaxRanks || rank < 0 || rank >= world || (nfl & 3)) return hipErrorInvalidValue;
    for (int r = 0; r < world; ++r)
        if (!dst.p[r]) return hipErrorInvalidValue;
    if ((nfl / 4 + kPeerSplit - 1) / kPeerSplit > 2 * 1024) return hipErrorInvalidValue;  // kPer float4 per thread
    hipLaunchKernelGGL(peer_push_kernel, dim3(world * kPeerSplit), dim3(1024), 0, s, grad, nfl, dst, rank, world,
                       peer_stride(nfl), seq);
    return hipGetLastError();
}

hipError_t launch_peer_apply(const float* xbuf, int world, int nfl, uint32_t seq, uint32_t* err, float* loss_out,
                             const ModelBuffers& mb, const OptimArgs& oa, hipStream_t s, int polls) {
    if (world < 2 || world > kPeerMaxRanks || !xbuf || !err || polls < 1) return hipErrorInvalidValue;
    float lr_t, ema_debias;
    adam_host_factors(oa, lr_t, ema_debias);
    const dim3 grid((mb.n_mlp + 255) / 256);
    const int st = peer_stride(nfl);
    if (world <= 2)
        hipLaunchKernelGGL(peer_apply_kernel<2>, grid, dim3(256), 0, s, xbuf, world, st, seq, polls, err, loss_out, mb, oa, lr_t, ema_debias);
    else if (world <= 4)
        hipLaunchKernelGGL(peer_apply_kernel<4>, grid, dim3(256), 0, s, xbuf, world, st, seq, polls, err, loss_out, mb, oa, lr_t, ema_debias);
    else if (world <= 8)
        hipLaunchKernelGGL(peer_apply_kernel<8>, grid, dim3(256), 0, s, xbuf, world, st, seq, polls, err, loss_out, mb, oa, lr_t, ema_debias);
    else
        hipLaunchKernelGGL(peer_apply_kernel<16>, grid, dim3(256), 0, s, xbuf, world, st, seq, polls, err, loss_out, mb, oa, lr_t, ema_debias);
    return hipGetLastError();
}

}  // namespace nrc_amd

