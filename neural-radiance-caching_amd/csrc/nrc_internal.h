// nrc_internal.h — host-side declarations shared by the C-ABI (nrc_capi.cpp) and the gfx950 kernels
// (nrc_kernels.hip). Not part of the public interface (that is include/nrc/nrc_c.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nrc/layout.h"

// 1 in libnrc_amd_debug.so: diagnostic builds (phase stamps, in-kernel clocks) and the A/B kernels that lost their
// comparisons; 0 in the product library libnrc_amd.so
#ifndef NRC_DEBUG_KERNELS
#define NRC_DEBUG_KERNELS 0
#endif

namespace nrc_amd {

// ---- MFMA fragment images (f16). One fragment = one v_mfma_f32_32x32x16_f16 A operand for a whole
// wave: 64 lanes x 8 halves = 1 KiB, stored lane-linear so a wave loads it with one ds_read_b128.
constexpr int kFragHalves = 512;
// forward image: L0 2 M-blocks x 5 k-steps, L1..L4 2 x 4 each, L5 1 x 4          = 46 fragments
constexpr int kFwdFrags = 2 * 5 + 4 * 2 * 4 + 4;
// backward image (W_l^T for l = 5..1): L5^T 2 M-blocks x 1 k-step, L4^T..L1^T 2 x 4 = 34 fragments
constexpr int kBwdFrags = 2 + 4 * 2 * 4;
constexpr int kFwdHalves = kFwdFrags * kFragHalves;  // 23552 halves = 46 KiB
constexpr int kBwdHalves = kBwdFrags * kFragHalves;  // 17408 halves = 34 KiB

// ---- Training layout "t16" (round 2, Frequency encoding): v_mfma_f32_16x16x32_f16 with 16 samples per wave, 8
// waves = 128 samples per block (nrc_train16.hip). Lane l = (g = l >> 4, c = l & 15). A fragment (1 KiB) is the A
// operand of one 16x16x32 MFMA for a wave: lane (g, m) holds A[row m][k = 8g + j], j = 0..7.
// Forward image: L0 4 M-blocks x 3 k-steps (the 96-slot encoder layout below), L1..L4 4 x 2, L5 1 x 2 = 46 frags.
// Backward image (W_l^T): L5^T 4 M-blocks of a 16x16x16 operand (K = the 16 output rows; 512 B used of each 1-KiB
// slot, lane (g, m) holds 4 halves k = 4g + j), L4^T..L1^T 4 x 2 = 36 frags.
__host__ __device__ constexpr int t16_fwd_frag(int layer, int mb, int s) {
    return layer == 0 ? mb * 3 + s : layer <= 4 ? 12 + (layer - 1) * 8 + mb * 2 + s : 44 + s;
}
__host__ __device__ constexpr int t16_bwd_frag(int layer, int mb, int s) {
    return layer == 5 ? mb : 4 + (layer - 1) * 8 + mb * 2 + s;
}
constexpr int kT16FwdFrags = 46, kT16BwdFrags = 36;
// Row of a 64-row activation / delta held in B-operand k-step s, lane group g, element j: accumulator-as-operand of
// the 16x16 C layout (M-blocks 2s and 2s + 1, rows 4g .. 4g + 3 of each).
__host__ __device__ constexpr int t16_row(int s, int g, int j) { return 32 * s + 16 * (j >> 2) + 4 * g + (j & 3); }
// Layer-0 input: 96 K slots, 24 per lane group g (its 16 samples' features), slot n = 0..23 of group g is
// K = 32 (n / 8) + 8 g + n % 8. Every lane computes the same kinds in the same slots: n 0..8 TriangleWave (dims
// n / 3, octaves 3g + n % 3), 9, 10 Identity (dims 2g, 2g + 1), 12..15 / 16..19 OneBlob (dims 2g / 2g + 1),
// 11 and 20..23 padding 1.0 (pad id 5g + 0..4). Group 3's Identity / OneBlob slots and the pad ids >= 14 are dummies
// with zero weights. Returns the canonical feature (0..79) of slot K, or -1.
__host__ __device__ constexpr int t16_slot_feature(int K) {
    return [](int g, int n) {
        if (n <= 8) return 12 * (n / 3) + 3 * g + n % 3;
        if (n == 9 || n == 10) return g < 3 ? 60 + 2 * g + (n - 9) : -1;
        if (n >= 12 && n <= 19) return g < 3 ? 36 + 4 * (2 * g + (n >= 16)) + (n & 3) : -1;
        const int pid = 5 * g + (n == 11 ? 0 : n - 19);
        return pid < 14 ? 66 + pid : -1;
    }((K % 32) / 8, 8 * (K / 32) + K % 8);
}
// InputEncoding::Hash in the t16 layout (round 5): the same 96 K slots with lane group g's 9 TriangleWave slots replaced
// by its 4 grid levels 4g .. 4g + 3 (n 0..7: canonical feature 8g + n, so K = canonical feature for the 32 grid
// features) and a pad slot (n 8); OneBlob / Identity slots as for Frequency (canonical 32.. / 56..); the two
// constant-one features 62, 63 in group 0's slots n 8 and 11; every other slot a dummy with zero weights.
__host__ __device__ constexpr int t16_hash_slot_feature(int K) {
    return [](int g, int n) {
        if (n <= 7) return 8 * g + n;
        if (n == 8 || n == 11) return g == 0 ? (n == 8 ? 62 : 63) : -1;
        if (n == 9 || n == 10) return g < 3 ? 56 + 2 * g + (n - 9) : -1;
        if (n >= 12 && n <= 19) return g < 3 ? 32 + 4 * (2 * g + (n >= 16)) + (n & 3) : -1;
        return -1;
    }((K % 32) / 8, 8 * (K / 32) + K % 8);
}
static_assert(t16_hash_slot_feature(13) == 13 && t16_hash_slot_feature(32 + 1) == 56 && t16_hash_slot_feature(32 + 4) == 32,
              "t16 Hash slot map");
// Hash backward image in the t16 layout: the 36 fragments of W_l^T, then W0^T restricted to the 32 grid features as
// 16x16x32 A operands: fragment 36 + 2 mb + s holds rows (grid slots) 16 mb .. 16 mb + 15, k-step s of delta_0's rows
constexpr int kT16BwdFragsHash = kT16BwdFrags + 4;
// Weight-gradient slab of one block in the t16 layout (f16 elements): per layer, 16x16 dW tiles (tm, tn) row-major
// (L0 4 x 6 tiles, L1..L4 4 x 4, L5 1 x 4: 23,552 elements, as the 32x32 slab), stored as column pairs: tiles
// (tm, 2p) and (tm, 2p + 1) are one 1-KiB record [lane 0..63][8], elements 0..3 = accumulator registers 0..3 of the
// even tile, 4..7 of the odd one, so a wave holding both writes them with one 16-byte store per lane. Register i of
// lane l holds dW[16 tm + 4 (l >> 4) + i][16 tn + (l & 15)] (layer 0: column = K slot).
__host__ __device__ constexpr int t16_ntn(int L) { return L == 0 ? 6 : 4; }
__host__ __device__ constexpr int t16_slab_base(int L, int tm, int tn) {
    return (L == 0 ? 0 : L <= 4 ? 6144 + (L - 1) * 4096 : 22528) + (tm * t16_ntn(L) + tn) * 256;
}
__host__ __device__ constexpr int t16_slab_pos(int L, int tm, int tn, int lane, int i) {
    return t16_slab_base(L, tm, tn & ~1) + lane * 8 + 4 * (tn & 1) + i;
}
static_assert(t16_slab_base(5, 0, 4) == 23552, "t16 slab size");
// Inverse of t16_slab_pos (Frequency layer offsets of layout.h): the canonical parameter of slab position pos, -1 for the
// dummy layer-0 K slots. Closed form so the reduction needs no map load before the parameter's Adam state
// (checked against build_t16_slab_map at nrc_init).
__host__ __device__ constexpr int t16_slab_param(int pos) {
    const int L = pos < 6144 ? 0 : pos < 22528 ? 1 + (pos - 6144) / 4096 : 5;
    const int off = pos - (L == 0 ? 0 : L <= 4 ? 6144 + (L - 1) * 4096 : 22528);
    const int ntn = t16_ntn(L), rec = off >> 9, q = off & 511, lane = q >> 3, e = q & 7;
    const int tm = rec / (ntn >> 1), tn = 2 * (rec % (ntn >> 1)) + (e >> 2);
    const int row = 16 * tm + 4 * (lane >> 4) + (e & 3), col = 16 * tn + (lane & 15);
    const int f = L == 0 ? t16_slot_feature(col) : col;
    const int in_dim = L == 0 ? NRC_ENC_WIDTH : 64;
    const int loff = L == 0 ? NRC_W0_OFFSET : L <= 4 ? NRC_W1_OFFSET + (L - 1) * 4096 : NRC_W5_OFFSET;
    return f < 0 ? -1 : loff + row * in_dim + f;
}
static_assert(t16_slab_param(t16_slab_pos(3, 2, 1, 37, 2)) == NRC_W1_OFFSET + 2 * 4096 + (32 + 4 * 2 + 2) * 64 + 16 + 5,
              "t16 slab inverse");
// The same inverse for InputEncoding::Hash's t16 slabs (round 5): t16_hash_slot_feature, in_dim 64, the Hash layer
// offsets (checked against build_t16_slab_map at nrc_init).
__host__ __device__ constexpr int t16_hash_slab_param(int pos) {
    const int L = pos < 6144 ? 0 : pos < 22528 ? 1 + (pos - 6144) / 4096 : 5;
    const int off = pos - (L == 0 ? 0 : L <= 4 ? 6144 + (L - 1) * 4096 : 22528);
    const int ntn = t16_ntn(L), rec = off >> 9, q = off & 511, lane = q >> 3, e = q & 7;
    const int tm = rec / (ntn >> 1), tn = 2 * (rec % (ntn >> 1)) + (e >> 2);
    const int row = 16 * tm + 4 * (lane >> 4) + (e & 3), col = 16 * tn + (lane & 15);
    const int f = L == 0 ? t16_hash_slot_feature(col) : col;
    const int in_dim = L == 0 ? NRC_HASH_ENC_WIDTH : 64;
    const int loff = L == 0 ? NRC_HASH_W0_OFFSET : L <= 4 ? NRC_HASH_W1_OFFSET + (L - 1) * 4096 : NRC_HASH_W5_OFFSET;
    return f < 0 ? -1 : loff + row * in_dim + f;
}

// Gradient exchange buffer: loss-scaled dL/dW (NRC_NUM_PARAMS f32) followed by the minibatch loss.

constexpr int kTrainSamplesPerBlock = 128;  // 4 waves x 32 samples

// Fragment index helpers (see DESIGN.md "MFMA operand images").
__host__ __device__ constexpr int fwd_frag(int layer, int mb, int kk) {
    return layer == 0 ? mb * 5 + kk : (layer <= 4 ? 10 + (layer - 1) * 8 + mb * 4 + kk : 42 + kk);
}
__host__ __device__ constexpr int bwd_frag(int layer, int mb, int kk) {
    return layer == 5 ? mb : 2 + (layer - 1) * 8 + mb * 4 + kk;
}
// Row index of element j of a B fragment for k-step kk taken from a 32x32 accumulator pair
// (accumulator-as-operand, cdna_hip_programming.md §3): lane half h.
__host__ __device__ constexpr int acc_row(int kk, int h, int j) {
    return 32 * (kk >> 1) + 16 * (kk & 1) + 8 * (j >> 2) + 4 * h + (j & 3);
}
// Layer-0 K slot -> canonical encoded feature. Each lane half computes 40 slots (n = 8*kk + j):
// 18 TriangleWave (3 dims x 6 of the 12 octaves), 12 OneBlob (3 dims x 4 bins), 3 Identity, 7 pad.
__host__ __device__ constexpr int slot_feature(int n, int h) {
    return n < 18   ? (n / 6) * 12 + (n % 6) + 6 * h
           : n < 30 ? 36 + (3 * h + (n - 18) / 4) * 4 + (n - 18) % 4
           : n < 33 ? 60 + 3 * h + (n - 30)
                    : 66 + (n - 33) + 7 * h;
}
// Hash config (64-wide input): 32 slots per lane half: 16 HashGrid features (levels 8h..8h+7), 12 OneBlob
// (dims 3+3h..5+3h), 3 Identity, 1 pad.
__host__ __device__ constexpr int hash_slot_feature(int n, int h) {
    return n < 16   ? 16 * h + n
           : n < 28 ? 32 + (3 * h + (n - 16) / 4) * 4 + (n - 16) % 4
           : n < 31 ? 56 + 3 * h + (n - 28)
                    : 62 + h;
}
__host__ __device__ constexpr int hash_k0_feature(int K) {
    return hash_slot_feature(8 * (K >> 4) + (K & 7), (K >> 3) & 1);
}
// Backward image of the Hash config: 4 extra fragments (kBwdFrags .. +3) hold W0^T for the 32 grid features,
// M rows permuted so that accumulator register r of lane half h is grid feature 16h + r:
// row m <-> feature 16*((m>>2)&1) + 4*(m>>3) + (m&3).
constexpr int kBwdFragsHash = kBwdFrags + 4;
constexpr int kBwdHalvesHash = kBwdFragsHash * kFragHalves;
__host__ __device__ constexpr int hash_dx_row(int feature) {
    return (feature & 3) + 4 * (feature >> 4) + 8 * ((feature >> 2) & 3);
}

// K index (column of the layer-0 MFMA, 0..79) -> canonical feature.
__host__ __device__ constexpr int k0_feature(int K) {
    return slot_feature(8 * (K >> 4) + (K & 7), (K >> 3) & 1);
}
// FrequencySH extension (80-wide): per lane half 18 TriangleWave, 8 SH coefficients (8h..8h+7), OneBlob of dims
// 5+2h, 6+2h (8 slots), 3 Identity, 3 pad.
__host__ __device__ constexpr int sh_slot_feature(int n, int h) {
    return n < 18   ? (n / 6) * 12 + (n % 6) + 6 * h
           : n < 26 ? 36 + 8 * h + (n - 18)
           : n < 34 ? 52 + (2 * h + (n - 26) / 4) * 4 + (n - 26) % 4
           : n < 37 ? 68 + 3 * h + (n - 34)
                    : 74 + 3 * h + (n - 37);
}
__host__ __device__ constexpr int sh_k0_feature(int K) {
    return sh_slot_feature(8 * (K >> 4) + (K & 7), (K >> 3) & 1);
}
// layer-0 K index -> canonical feature, per encoding (0 Frequency, 1 Hash, 2 FrequencySH)
__host__ __device__ constexpr int enc_k0_feature(int enc, int K) {
    return enc == 1 ? hash_k0_feature(K) : enc == 2 ? sh_k0_feature(K) : k0_feature(K);
}

// ---- width-128 network (BASELINE configs[4]). f16 image: 156 fragments of 1 KiB in the layout of
// the 64-wide forward image (L0 4 M-blocks x 5 k-steps, L1..L4 4 x 8, L5 1 x 8). FP8 image: the 20 f16 layer-0
// fragments, then 34 fp8 fragments of layers 1..5 (L1..L4 4 M-blocks x 2 k-steps of 64, L5 1 x 2), each 2 KiB =
// two 1-KiB planes (bytes 0-15 / 16-31 of every lane's 32-byte MX-MFMA operand, lane-linear 16 B so that each plane
// is one conflict-free ds_read_b128), plus per-row E8M0 scales [5 layers][32 lanes] (byte mb = row 32 mb + lane).
constexpr int kWideF16Frags = 4 * 5 + 4 * 4 * 8 + 8;  // 156
constexpr int kWide8Frags = 4 * 4 * 2 + 2;            // 34
constexpr int kWideF16Bytes = kWideF16Frags * 1024;                   // 159744
constexpr int kWide8Bytes = 20 * 1024 + kWide8Frags * 2048;           // 90112
__host__ __device__ constexpr int wide_frag(int layer, int mb, int kk) {
    return layer == 0 ? mb * 5 + kk : layer <= 4 ? 20 + (layer - 1) * 32 + mb * 8 + kk : 148 + kk;
}
__host__ __device__ constexpr int wide8_frag(int layer, int mb, int s) {
    return layer <= 4 ? (layer - 1) * 8 + mb * 2 + s : 32 + s;
}
// Byte j (0..31) of lane half h of an fp8 B operand for k-step s, built from the accumulators of M-blocks 2s and
// 2s + 1 (register j & 15 of block 2s + (j >> 4)): the previous layer's output row it carries.
__host__ __device__ constexpr int f8_row(int s, int h, int j) {
    return 64 * s + 32 * (j >> 4) + (j & 3) + 8 * ((j & 15) >> 2) + 4 * h;
}
// the width-128 weight images a step rewrites: f16 inference (img16; img8 = FP8 image whose first 20 KiB are the f16
// layer-0 fragments, scales = per-row E8M0 words) and the training forward / backward images; enc 0 Frequency, 2 SH
struct WideImages {
    _Float16* img16;
    uint8_t* img8;
    uint32_t* scales;
    _Float16 *fwd16, *bwd16;
    int enc;
};
// every width-128 image: inference f16 + FP8 (+ row scales) from w_infer, training fwd/bwd from w_train
hipError_t launch_wide_pack(const float* w_infer, const float* w_train, const WideImages& im, hipStream_t s);
// prec 0 = f16, 1 = fp8; enc 0 = Frequency, 2 = FrequencySH; mode -1 plain, 0 / 2 fused accumulation
hipError_t launch_infer_wide(int prec, int enc, const float* queries, float* out, int64_t n, const void* img,
                             const uint32_t* scales, const float* thr, float* rgba, int64_t n_acc, int mode, float w,
                             hipStream_t s);
// width-128 training (nrc_kernels.hip): backward image W_l^T (L5^T 4 M-blocks x 1 k-step, L4^T..L1^T 4 x 8)
constexpr int kWideBwdFrags = 4 + 4 * 4 * 8;  // 132
constexpr int kWideBwdBytes = kWideBwdFrags * 1024;
// workspace rows ([feature][bpad] f16): inputs x (80) + a_0..a_4 (5 x 128) = 720; deltas 5 x 128 + 16 = 656
constexpr int kWideInRows = 80 + 5 * 128, kWideDRows = 5 * 128 + 16;
int64_t wide_bpad(int64_t b);
int64_t wide_ld(int64_t b);  // row stride (f16 elements) of the width-128 training workspace
int wide_chunks(int64_t b);
hipError_t launch_wide_train_fwd_bwd(int enc, const float* queries, const float* targets, int64_t b, float n_total,
                                     float loss_scale, const _Float16* fwd16, const _Float16* bwd16, _Float16* ws_in,
                                     _Float16* ws_d, float* slabs, float* loss_partials, hipStream_t s);
// the optimizer step and (modes other than kReduceOnly) every image of im, in one launch
hipError_t launch_wide_adam(int mode, const float* slabs, int nchunks, const float* loss_partials, int nlp,
                            float* grad_io, float* loss_out, const struct ModelBuffers& mb, const struct OptimArgs& oa,
                            const WideImages& im, hipStream_t s);
// diagnostic: e4m3 conversion exactly as the FP8 kernels do it (clamp to [lo, 448], v_cvt_pk_fp8_f32)
hipError_t launch_fp8_convert(const float* x, uint8_t* y, int64_t n, int relu, hipStream_t s);

// ---- kernel launchers (nrc_kernels.hip). All are stream-ordered and capture-safe.
// pools / parity: the handle's work-pool counters (kInferPoolBytes, zeroed at allocation) and its launch parity, which
// the pooled variants flip (see ABL & 16384 in nrc_kernels.hip); variants that do not pool ignore both
// [0, 8 KiB): the pooled variant's two sets of 32 counters; then the steal variant's two sets of kStealMaxBlocks
// per-block range counters, 64 B apart (ABL & 32768 in nrc_kernels.hip)
constexpr int kStealMaxBlocks = 1024, kStealStride = 16, kStealSetWords = kStealMaxBlocks * kStealStride;
constexpr int kInferPoolBytes = 2 * 32 * 32 * 4 + 2 * kStealSetWords * 4;
hipError_t launch_infer(const float* queries, float* out, int64_t n, const _Float16* wf, hipStream_t s,
                        uint32_t* pools = nullptr, int* parity = nullptr, bool padq = false);
// the product kernel is variant 47; the debug library (NRC_DEBUG_KERNELS) also has the A/B variants 0, 23, 30, 39 (round
// 2's product: 47 with the 32x32x16 output layer), 40 (39 + in-kernel clock) and 48 (47 + in-kernel clock)
constexpr int kProductInferVariant = 47;
hipError_t launch_infer_variant(int variant, const float* queries, float* out, int64_t n, const _Float16* wf,
                                hipStream_t s, uint32_t* pools = nullptr, int* parity = nullptr);
constexpr int kNumInferVariants = 65;  // 50: launch_infer16 (the t16 image)
// Frequency inference on v_mfma_f32_16x16x32_f16 (nrc_infer16.hip) from the t16-layout inference image
hipError_t launch_infer16(const float* queries, float* out, int64_t n, const _Float16* wf16, hipStream_t s);
// per-wave (cycles, 100 MHz ticks) of the last clocked variant launch (31, 32)
hipError_t read_infer_clock(uint64_t* host, int64_t cap_waves, int64_t* waves);
// inference with accumulate_render_radiance fused for queries [0, n_acc) (mode 0 Full / 2 CacheOnly)
hipError_t launch_infer_accumulate(const float* queries, float* out, int64_t n, const _Float16* wf, const float* thr,
                                   float* rgba, int64_t n_acc, int mode, float w, hipStream_t s, bool padq = false);
// InputEncoding::Hash inference (mode -1: plain; 0 / 2: fused accumulation for queries [0, n_acc))
// feat: the handle's [NRC_HASH_LEVELS][kHashFeatStride] level-feature workspace (hash_feature_kernel, round 3), or
// nullptr for the round-2 gather kernel (also knob "hash_infer" = 1)
constexpr int64_t kHashFeatStride = (int64_t)1 << 21;  // queries per feature pass (128 MiB of features)
hipError_t launch_infer_hash(const float* queries, float* out, int64_t n, const _Float16* wf, const _Float16* grid,
                             const float* thr, float* rgba, int64_t n_acc, int mode, float w, hipStream_t s,
                             uint32_t* feat = nullptr, bool padq = false);
hipError_t launch_encode_hash(const float* queries, const _Float16* grid, float* enc, int64_t n, hipStream_t s);
// FrequencySH extension
hipError_t launch_infer_sh(const float* queries, float* out, int64_t n, const _Float16* wf, const float* thr,
                           float* rgba, int64_t n_acc, int mode, float w, hipStream_t s);
hipError_t launch_encode_sh(const float* queries, float* enc, int64_t n, hipStream_t s);
// tcnn-numerics inference (NRC_PRECISION_F16_ACC16, Frequency, width 64): f16 accumulation per 16-wide K chunk;
// w0 = the f32 inference weights (canonical blob; layer 0 is rebuilt from it in canonical K order)
hipError_t launch_infer_tcnn(const float* queries, float* out, int64_t n, const _Float16* wf, const float* w0,
                             hipStream_t s);
// the same numerics for InputEncoding::Hash (round 5): feature pass into feat, then the f16-accumulate MLP pass;
// w0 = the f32 inference MLP blob (Hash W0 [64][64] first)
hipError_t launch_infer_hash_tcnn(const float* queries, float* out, int64_t n, const _Float16* wf, const float* w0,
                                  const _Float16* grid, uint32_t* feat, hipStream_t s);
hipError_t launch_encode(const float* queries, float* enc, int64_t n, hipStream_t s);
hipError_t launch_encode_fast(const float* queries, float* enc, int64_t n, hipStream_t s, int variant = 0);
// fwd+loss+bwd+per-block dW partials. n_total = 3 * global batch.
hipError_t launch_train_fwd_bwd(const float* queries, const float* targets, int64_t b, float n_total,
                                float loss_scale, const _Float16* wf, const _Float16* wb, float* slabs,
                                float* loss_partials, hipStream_t s, int enc = 0);
int train_blocks(int64_t b);
// diagnostic: same kernel with s_memtime stamps (16 per block) — never used by the product path
hipError_t launch_train_stamped(const float* queries, const float* targets, int64_t b, float n_total, float loss_scale,
                                const _Float16* wf, const _Float16* wb, float* slabs, float* loss_partials,
                                uint64_t* stamps, hipStream_t s);

// kApplyFixed (grid_adam_kernel only): the gradient is an all-reduced exchange-encoded fixed-point array (GridBuffers::fixed)
enum ReduceMode { kReduceFused = 0, kReduceOnly = 1, kApplyOnly = 2, kPackOnly = 3, kApplyFixed = 4 };

// One-shot peer gradient exchange of nrc_train_dp (nrc_kernels.hip, round 4): receive buffers of peer_buffer_bytes, one
// per rank, IPC-mapped into every other rank; dst.p[r] = rank r's buffer as seen from this process.
constexpr int kPeerMaxRanks = 16;
struct PeerPtrs {
    float* p[kPeerMaxRanks];
};
int peer_stride(int nfl);
// the receive buffer: the push/apply region (nfl floats per slot) and the fused exchange's region (slab order, n_slab)
size_t peer_buffer_bytes(int world, int nfl, int n_slab);
struct OptimArgs {
    float lr, beta1, beta2, eps, l2_reg, ema_decay, loss_scale;
    uint32_t step;
};
// Per-block weight-gradient slab, fragment-major: the 32x32 dW blocks one after another (layer 0 blocks (mb, nb)
// with nb over 3 column blocks (80-wide input incl. the x_hi block) or 2 (Hash), layers 1..4 blocks (mb, nb), layer 5
// the two 16x32 halves), each block as [j = 0..3][lane 0..63][4 floats]: register 4j + e of lane `lane` of the
// MFMA accumulator. The training kernel then writes every block with lane-contiguous 16-byte stores; the reduce
// maps positions to parameters through ModelBuffers::slab_param (-1 for the x_hi block's padding lanes).
__host__ __device__ constexpr int slab_l0_nb(int enc) { return enc == 1 ? 2 : 3; }
__host__ __device__ constexpr int slab_block_base(int enc, int L, int mb, int nb) {
    return L == 0 ? (mb * slab_l0_nb(enc) + nb) * 1024
           : L <= 4 ? 2 * slab_l0_nb(enc) * 1024 + (L - 1) * 4096 + (mb * 2 + nb) * 1024
                    : 2 * slab_l0_nb(enc) * 1024 + 4 * 4096 + nb * 512;
}
__host__ __device__ constexpr int slab_floats(int enc) { return slab_block_base(enc, 5, 0, 2); }
static_assert(slab_floats(0) == 23552 && slab_floats(1) == NRC_HASH_MLP_PARAMS, "slab sizes");

struct ModelBuffers {
    float *params, *m, *v, *ema, *infer;  // f32 master / Adam / EMA / debiased EMA (inference)
    _Float16 *wf_train, *wb_train, *wf_infer;
    _Float16* wf_infer16;  // t16 nets: the inference image in the t16 layout (at fwdt_pos), else null
    const int *fwd_pos, *bwd_pos;
    const int* fwdt_pos;  // position in wf_train (the t16 layout for Frequency; fwd_pos otherwise)
    bool slab_f16;        // slabs hold f16 partials (t16)
    int n_mlp;  // MLP (matrix) parameter count = slab stride: 22528 Frequency, 21504 Hash
    int n_total;  // all parameters (MLP + grid): index of the loss in a data-parallel gradient buffer
    const int* slab_param;  // [n_slab] parameter of each slab position, -1 = padding
    int n_slab;             // slab stride (floats per training block)
    int slab_closed;        // f16 slabs of the t16 layout: the reduction maps positions in closed form instead of
                            // loading slab_param -- 1 Frequency (t16_slab_param), 2 Hash (t16_hash_slab_param); 0 map
};

// slabs: f16 (nrc_train16.hip slab_pair), reduced by launch_reduce_adam (ModelBuffers::slab_f16)
hipError_t launch_train16(const float* queries, const float* targets, int64_t b, float n_total, float loss_scale,
                          const _Float16* wf, const _Float16* wb, _Float16* slabs, float* loss_partials, uint64_t* stamps,
                          hipStream_t s, bool split = false, int groups = 2, bool padq = false);
// Round 6: one launch for the whole width-64 Frequency step of the role-split kernel (128-sample blocks): trainer
// blocks + reducer blocks that wait for them on the counters at sync (2 x 256 B, zero at allocation) and then run
// kReduceFused's sums and Adam/EMA from agent-scope loads of the slabs -- state bitwise the same as
// launch_train16 + launch_reduce_adam. hipErrorNotSupported when trainers + reducers exceed max_blocks (the CU count).
// err: the handle's protocol word (3 = the reducers' bounded wait gave up).
hipError_t launch_train16_fused(const float* queries, const float* targets, int64_t b, float n_total, float loss_scale,
                                const _Float16* wf, const _Float16* wb, _Float16* slabs, float* loss_partials,
                                uint32_t* sync, uint32_t* err, int polls, float* loss_out, const ModelBuffers& mb,
                                const OptimArgs& oa, hipStream_t s, bool padq, int max_blocks, int mode,
                                uint32_t gen, uint32_t* flags, int max_flags);
// InputEncoding::Hash on the t16 role-split kernel (round 5): the encoder reads levels 4g .. 4g + 3 from the feature
// pass's workspace (or gathers them from the f16 training table); the chain waves also write each sample's position and its 16 levels' (dy0, dy1) = W0^T delta_0 of the
// grid features (f16 pairs, [level][sample], zeros past b) for grid_scatter_kernel. wb: kT16BwdFragsHash fragments.
struct HashTrainOut {
    const uint32_t* table;  // f16 training table as half2 entries
    const uint32_t* feat;   // the samples' level features ([level][kHashFeatStride], hash_feature_kernel over the batch
                            // with the training table), or null: the kernel gathers from the table itself
    float4* pos;            // [bcap]
    uint32_t* dy;           // [NRC_HASH_LEVELS][bcap]
    int64_t bcap;
};
hipError_t launch_train16_hash(const float* queries, const float* targets, int64_t b, float n_total, float loss_scale,
                               const _Float16* wf, const _Float16* wb, _Float16* slabs, float* loss_partials,
                               const HashTrainOut& ho, hipStream_t s, bool padq = false, int groups = 2);
// samples per block of the role-split t16 kernel: 64 x groups (knob "t16_groups"; 128 by default)
int t16_groups();  // split: the role-split kernel (NRC_T16_SPLIT at init)
// Decoupled-chain Frequency training kernel (nrc_train_dc.hip, round 3): shape 0..5 (dc_samples_per_block), same f16
// slab format as launch_train16; one slab per block of dc_samples_per_block(shape) samples.
int dc_samples_per_block(int shape);
// stamps (diagnostic, may be null): 16 uint64 per wave [block][wave][16], dc_waves_per_block(shape) waves per block;
// err (required): set to 1 by a wave whose bounded LDS-protocol wait ran out (the step's slabs are then invalid)
hipError_t launch_train_dc(int shape, const float* queries, const float* targets, int64_t b, float n_total,
                           float loss_scale, const _Float16* wf, const _Float16* wb, _Float16* slabs,
                           float* loss_partials, uint32_t* err, hipStream_t s, uint64_t* stamps = nullptr, bool padq = false);
int dc_waves_per_block(int shape);
// the production shape for a batch of b samples
int dc_auto_shape(int64_t b);

// ---- process-wide A/B knobs (nrc_debug_set_knob; never read from the environment). -1 = the production choice.
enum Knob : int {
    kKnobTrainKernel = 0,  // Frequency training: -1 / 0 decoupled chain (dc), 1 round-2 t16 role split, 2 round-2 t16
                           // 4-wave, 32 round-1 32x32x16 (read at nrc_init)
    kKnobTrainShape = 1,   // dc shape (0..5), -1 = dc_auto_shape(b)
    kKnobScatterMin = 2,   // Hash grid scatter slice plan (samples per block at level 0 / cap), -1 = 2048 / 4096
    kKnobScatterMax = 3,
    kKnobDcDw0Delay = 4,  // debug library: s_sleep(127) rounds dW wave 0 of the dc kernel spends after its step 5
    kKnobHashInfer = 5,   // Hash inference: -1 / 0 LDS-table feature pass + MLP kernel (round 3), 1 the gather kernel
    kKnobHashFeatAbl = 6,  // debug library: hash_feature_kernel ablation (1 no gathers, 2 no position loads, 4 no stores)
    kKnobT16Groups = 7,    // role-split t16 training kernel: 16-sample groups per chain wave (1: 64-sample blocks; -1 = 2)
    kKnobHashFeatP = 8,    // Hash feature pass: query ranges per level (multiple of 8; -1 = 32 above 2^19 queries, else 8)
    kKnobPeerPath = 9,     // nrc_train_dp over the peer exchange: -1 automatic (fused, or split when a peer shares this
                           // rank's device), 0 the reduce + push + apply launches (round 4's first version), 1 fused,
                           // 2 split (reduce + push, then wait + sum + Adam); tests: 3 the split form's gradient pass +
                           // push alone (no optimizer step), 4 its wait + sum + Adam alone (the step the last 3 pushed)
    kKnobPxPolls = 10,     // bound of the peer exchange's wait loops (-1 = kPeerPolls, about 10 s; 1..2^21)
    kKnobScatterPart = 11, // Hash training: first grid level whose scatter stores per-slice partials (-1 default, 0..16)
    kKnobScatterCompact = 12, // Hash training: first grid level whose scatter queues its in-part corners (-1 default, 0..16)
    kKnobHashTrainFeat = 13,  // Hash training: the batch's level features by 0 the LDS pass, 1 gathers (-1 = 1)
    kKnobHashAdam = 14,       // Hash training: 0 = the MLP and grid optimizer updates as two launches (-1: one)
    kKnobTrainFused = 15,     // width-64 Frequency step on the role-split kernel: 1 = one launch (launch_train16_fused,
                              // A/B: 14.4-14.8 vs 12.0 us per step); -1 / 0 the training and
                              // optimizer kernels as two launches (read at nrc_init)
    kKnobFuseMode = 16,       // fused step A/B: 0 (-1) per-block flags, 1 / 2 an arrival counter per block / per wave;
                              // timing ablations (wrong results) 3 no reducers, 4 reducers that only wait
    kKnobTcnnReentry = 17,    // tcnn-numerics inference: the f16 accumulator back into f32 by 0 two 32x32x16 identity
                              // MFMAs per block and chunk (round 6, first form), 1 (-1) four 4x4x4 identity MFMAs
    kKnobTrainPrio = 18,      // debug library, A/B: role-split training kernel with 1 the dW waves / 2 the chain waves
                              // at s_setprio 1 (-1 / 0: no priority)
    kKnobCount = 19
};
int knob(Knob k);

// host-f32 Adam step-size and EMA debias of optimizer step oa.step (tcnn adam.h; identical to the oracle's)
void adam_host_factors(const OptimArgs& oa, float& lr_t, float& ema_debias);
// Non-finite grid-gradient contributions: an f16 product w * dy that is inf or NaN cannot enter the fixed-point sum, so
// grid_scatter_kernel ORs a code into codes[param] (1 = +inf, 2 = -inf, 3 = NaN; +inf and -inf together make NaN, as
// in tcnn's f16 atomics) and stores the scatter's tag into *tag_dev. The kernels that round the step's sums read codes
// only when *tag_dev equals their tag (a per-handle sequence number, never 0), and clear the codes they read.
struct GridNonFinite {
    uint8_t* codes = nullptr;   // [n] one byte per grid parameter, zero between steps
    uint32_t* tag_dev = nullptr;
    uint32_t tag = 0;
};
// HashGrid parameters (the grid part of the model arrays) and their optimizer state
// Per-slice partial sums of the grid scatter (round 5): level l's nslice[l] sample slices x its entries x 2 features,
// int64 fixed point, at base + off[l]; every scatter block of such a level stores its part of one slice densely (plain
// stores, no global atomics), and grid_adam_kernel sums the slices in slice order. Levels with nslice 0 (the coarse
// ones: few entries touched, so dense stores would be mostly zeros) and every level when base is null add into grad64
// with global atomics instead (the data-parallel exports read grad64).
// A block's part of a slice is stored as int32 when every one of its sums fits (the usual case: |sum| < 128 in f16
// units), else as int64; flags[foff[l] + slice * parts(l) + part] says which (1 = int64), so the partial bytes the
// grid Adam reads are halved without giving up exactness.
struct ScatterPartials {
    int64_t* base = nullptr;   // int64 form, element e of (level l, slice s) at base + off[l] + s * 2 * entries(l) + e
    int32_t* base32 = nullptr; // int32 form, the same element indexing
    uint32_t* flags = nullptr; // per (level, slice, part): 1 = that block stored the int64 form
    int64_t off[NRC_HASH_LEVELS] = {};
    int foff[NRC_HASH_LEVELS] = {};
    int nslice[NRC_HASH_LEVELS] = {};
    int64_t total = 0;  // elements of the layout (each form)
    int nflags = 0;
};
// the layout of a b-sample step under the current scatter plan (knobs scatter_min / scatter_max), partial sums for
// levels first_level.. (nslice 0 below: those levels flush into grad64 with atomics; total 0 when first_level = 16)
ScatterPartials scatter_partials_layout(int64_t b, int first_level);
// default first level (knob scatter_part): fused step 63.0 us all-atomic, 58.3 / 57.6 / 57.4 / 56.5 / 57.2 from level
// 0 / 2 / 4 / 6 / 8 (profiles/r05_hash/ab_scatter_part.json, parameters bitwise equal)
constexpr int kScatterPartFirst = 6;
// at most this many slices per level use partials (bigger batches flush with atomics: the partial bytes, and the grid
// Adam's reads of them, grow with the batch; 8 slices = 32,768 samples at the default plan, 40 MiB)
constexpr int kMaxPartialSlices = 8;
// default first level of the corner queue (knob scatter_compact): step 57.3 us without, 56.0 from level 4, 55.8 from
// level 10 (profiles/r05_hash/ab_scatter_compact_repeat.json, 12 interleaved rounds x 2)
constexpr int kScatterCompactFirst = 10;
struct GridBuffers {
    float *params, *m, *v, *ema, *infer;
    ScatterPartials part;  // kReduceFused: the step's partial sums when part.base is set (else grad64)
    int64_t* grad64;      // [n] exact fixed-point sums (value x 2^24) of the f16 contributions, accumulated by
                          // grid_scatter_kernel, rounded to f16 and zeroed by grid_adam_kernel
    const float* grad32;  // kApplyOnly: the all-reduced data-parallel gradient (f32 [n], read-only)
    const int64_t* fixed; // kApplyFixed: the all-reduced exchange-encoded sums [n] (may be grad64 itself)
    uint32_t* steps;  // per-entry Adam step counters
    GridNonFinite nf;     // non-finite contributions of the step being consumed (kReduceFused)
    _Float16 *table_train, *table_infer;
    // Adam bias corrections per step count st = 1..bias_len: bias[st] = (sqrtf(1 - beta2^st), 1 - beta1^st), host
    // glibc powf as in the oracle (the kernel falls back to device powf past bias_len)
    const float2* bias;
    uint32_t bias_len;
    int n;
};
// steps covered by the bias table (past it the kernel calls powf; for the default betas 0.9 / 0.999 both
// corrections are exactly 1.0f there)
constexpr uint32_t kGridBiasLen = 1u << 16;
hipError_t launch_grid_adam(int mode, const GridBuffers& gb, const OptimArgs& oa, hipStream_t s);
// Hash training workspace: per sample its position and the 16 levels' (dy0, dy1) f16 pairs ([level][sample]),
// written by the training kernel and consumed by grid_scatter_kernel.
struct HashScatter {
    float4* pos;   // [bcap]
    uint32_t* dy;  // [NRC_HASH_LEVELS][bcap]
    int64_t bcap;
    GridNonFinite nf;
    ScatterPartials part;  // base set: flush into per-slice partials (plain stores) instead of grad64 (atomics)
};
// Data-parallel exports of the grid accumulator (both zero it for the next step and consume the non-finite codes):
// f32 -- each sum rounded to f16 (nrc_train_grad); fixed -- the exact sum in the exchange encoding below, for an int64
// sum over ranks (nrc_train_grad_fixed, nrc_train_dp; out may be g64 itself, which is then not zeroed).
hipError_t launch_grid_grad_export(int64_t* g64, float* g32, int n, const GridNonFinite& nf, hipStream_t s);
hipError_t launch_grid_grad_export_fixed(int64_t* g64, int64_t* out, int n, const GridNonFinite& nf, hipStream_t s);
// Exchange encoding of a rank's exact sum v (value x 2^24) and its non-finite code c, such that the int64 SUM over up to
// kFixedMaxRanks ranks decodes to the global sum and code: clamp(v, +-2^41) + 2^48 [c has +inf] + 2^55 [c has -inf].
// |sum| >= 65520 x 2^24 rounds to f16 inf, so the clamp changes no result unless partial sums beyond 131072 cancel across
// ranks (tcnn's f16 running sum is already inf there). The 7-bit marker counts bound the world size.
constexpr int kFixedMaxRanks = 63;
hipError_t launch_infer_stamped(const float* queries, float* out, int64_t n, const _Float16* wf, uint64_t* stamps,
                                int64_t* waves, hipStream_t s);
// feat (t16 only, may be null): the handle's level-feature workspace; the batch's features are computed into it first
hipError_t launch_train_hash(const float* queries, const float* targets, int64_t b, float n_total, float loss_scale,
                             const _Float16* wf, const _Float16* wb, const _Float16* grid, int64_t* grid_grad,
                             float* slabs, float* loss_partials, hipStream_t s, const HashScatter* sc = nullptr, bool padq = false,
                             bool t16 = false, uint32_t* feat = nullptr, int groups = 2);
// the fused Hash step's MLP reduce + Adam and grid Adam (kReduceFused both) in one launch (t16 f16 slabs only)
hipError_t launch_hash_adam(const float* slabs, int nslabs, const float* loss_partials, float* loss_out,
                            const ModelBuffers& mb, const GridBuffers& gb, const OptimArgs& oa, hipStream_t s);
hipError_t launch_reduce_adam(int mode, const float* slabs, int nslabs, const float* loss_partials,
                              float* grad_io, float* loss_out, const ModelBuffers& mb, const OptimArgs& oa,
                              hipStream_t s);
hipError_t launch_peer_push(const float* grad, int nfl, const PeerPtrs& dst, int rank, int world, uint32_t seq,
                            hipStream_t s);
// polls: bound of every wait loop (kPeerPolls in production, about 10 s; knob "px_polls" for tests)
constexpr int kPeerPolls = 1 << 21;
hipError_t launch_peer_apply(const float* xbuf, int world, int nfl, uint32_t seq, uint32_t* err, float* loss_out,
                             const ModelBuffers& mb, const OptimArgs& oa, hipStream_t s, int polls = kPeerPolls);
// Forms of the exchange inside the reduction: kPxFused -- reduce + push + wait + rank-order sum + Adam/EMA in one launch
// after the gradient pass (world 1..16, ranks on separate devices); kPxSplit -- the same as two launches (reduce + push,
// then wait + sum + Adam in a small grid) for ranks that share a device; kPxPushOnly / kPxApplyOnly -- the split form's
// first / second launch on its own (sequenced single-process tests, knob peer_path 3 / 4)
enum PxForm { kPxFused = 0, kPxSplit = 1, kPxPushOnly = 2, kPxApplyOnly = 3 };
hipError_t launch_reduce_exchange(const float* slabs, int nslabs, const float* loss_partials, const PeerPtrs& dst,
                                  int rank, int world, int nfl, uint32_t seq, uint32_t* err, float* loss_out,
                                  const ModelBuffers& mb, const OptimArgs& oa, hipStream_t s, int form,
                                  int polls = kPeerPolls);

// ---- per-handle scratch used by the frame driver (nrc_capi.cpp): NRC_NUM_BATCHES loss slots on the device and a
// pinned host mirror
struct nrc_loss_slots {  // four minibatch-loss slots in host-mapped coherent pinned memory
    float* dev;   // device view (what the kernels write)
    float* host;  // host view (valid after a stream sync)
};
}  // namespace nrc_amd
struct nrc_net;
namespace nrc_amd {
nrc_loss_slots net_loss_slots(nrc_net* net);
// the attached communicator (nrc_set_comm): false if none; rank / world of it
bool net_comm(nrc_net* net, int* rank, int* world);
// per-handle device scratch of the frame driver (grown on demand, freed with the handle; stream-ordered use only)
void* net_frame_scratch(nrc_net* net, size_t bytes);
// the handle's RadianceQuery records are padded (nrc_config.query_layout = NRC_QUERY_PADDED)
bool net_padq(nrc_net* net);
// inference can take the fused accumulation epilogue (not with NRC_PRECISION_F16_ACC16)
bool net_infer_fusable(nrc_net* net);
// throws NRC_ERR_INTERNAL if a training kernel or a peer-exchange wait reported a timeout (after a stream sync)
void net_check_protocol(nrc_net* net);
// nrc_train_dp with the loss left in a device slot (frame driver)
void net_train_dp_async(nrc_net* net, const float* in, const float* tgt, uint32_t b_local, uint32_t global_b,
                        float* loss_d);

// ---- per-frame kernels around the network (nrc_frame.hip, include/nrc/frame.h)
// queries / end_queries + train_queries (RadianceQuery arrays, NULL = off): USE_REFLECTANCE_FACTORING 1
hipError_t launch_accumulate(const float* rad, const float* thr, float* rgba, uint32_t n, int mode, float w,
                             hipStream_t s, const float* queries = nullptr, bool padq = false);
hipError_t launch_propagate(const void* ends, const float* end_rad, uint32_t tiles, const void* records,
                            float* targets, uint32_t nrec, hipStream_t s, const float* end_queries = nullptr,
                            const float* train_queries = nullptr, bool padq = false);
hipError_t launch_permutation(uint64_t seed, uint32_t frame, int* perm, uint32_t n, hipStream_t s);
// the reference's shuffle contract (NRCUtil.cu:19-35): stable LSD radix sort of (keys[i], i) over 32 key bits; vals_out
// receives the sorted indices, keys_out (may be null) the sorted keys; temp: sort_pairs_temp_bytes(n) bytes
size_t sort_pairs_temp_bytes(uint32_t n);
hipError_t launch_sort_pairs(const uint32_t* keys, uint32_t* keys_out, int* vals_out, uint32_t n, void* temp,
                             hipStream_t s);
hipError_t launch_permute(const float* qs, const float* ts, const int* perm, uint64_t seed, uint32_t frame,
                          uint32_t nrec, float* qd, float* td, uint32_t n_out, hipStream_t s, bool padq = false);

}  // namespace nrc_amd
