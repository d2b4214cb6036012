/*
 * nrc_oracle.h — CPU restatement of the reference's NRC query/train arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker (or the timed CPU baseline). The product path
 * (neural-radiance-caching_amd/) never links or calls it.
 *
 * PARITY UNPINNED: the reference's arithmetic lives in tiny-cuda-nn (submodule
 * github.com/Depersonalizc/tiny-cuda-nn, /root/reference/.gitmodules:1-3), which is empty in the
 * reference snapshot, has no recoverable pinned commit and is not importable here. The reference
 * holds no tests, golden vectors or fixtures for this path. This oracle restates
 * tcnn's published algorithm as the reference configures it (NRCNetworkConfigs.h:11-83) and is
 * cross-checked against an independent float64 numpy restatement and torch autograd
 * (tests/test_oracle.py). Spec choices are tagged [H]/[M]/[L] as in SURVEY.md Appendix A.
 */
#ifndef NRC_ORACLE_H
#define NRC_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Numerics modes.
 *  ORC_FP32  : exact f32 weights/activations, f64 dot products rounded to f32 per layer.
 *  ORC_MIXED : the GPU build's numerics model: f16 encoded inputs, f16 weights, f32 accumulate,
 *              f16 activations between layers, f16 output; f16 loss/backprop gradients; f32 dW.
 *  ORC_TCNN  : tcnn FullyFusedMLP emulation [M]: as MIXED, but every matmul accumulates in f16
 *              (one f16 rounding per 16-wide k chunk, WMMA 16x16x16), and the parameter gradient
 *              is stored as f16 (tcnn keeps PARAMS_T gradients). */
enum { ORC_FP32 = 0, ORC_MIXED = 1, ORC_TCNN = 2, ORC_FP8 = 3 /* width-128 inference only */ };

float orc_f16_round(float x);

/* Composite encoding of n queries (15 f32 each, AoS) into n x 80 f32 in canonical tcnn feature
 * order: [0,36) TriangleWave, [36,60) OneBlob, [60,66) Identity, [66,80) padding = 1.0. */
void orc_encode(const float* queries, int64_t n, float* enc);

/* Forward pass with the given parameter blob (22528 f32, canonical order, layout.h).
 * out: n x 3 f32. nthreads >= 1. */
void orc_forward(const float* params, const float* queries, int64_t n, int mode, float* out,
                 int nthreads);

/* One training minibatch: loss-scaled parameter gradient of
 *   L = sum_{s<b, c<3} (y_sc - t_sc)^2 / (lum(y_s)^2 + 0.01) / n_total
 * (RelativeL2Luminance, denominator not differentiated). Writes grad[22528] = loss_scale * dL/dW
 * and returns L (the reference's Trainer::loss()). n_total = 3 * global batch. */
double orc_grad(const float* params, const float* queries, const float* targets, int64_t b,
                double n_total, float loss_scale, int mode, float* grad, int nthreads);

/* Extension encoding NRC_ENCODING_FREQUENCY_SH (see nrc_oracle.c): 80-wide, same MLP shape as Frequency. */
void orc_encode_sh(const float* queries, int64_t n, float* enc);
/* Non-compact RadianceQuery (16 f32, USE_COMPACT_RADIANCE_QUERY 0) into n x 80 in the reference's padded order:
 * [0,36) TriangleWave, 36 pad_, [37,61) OneBlob, [61,67) Identity, [67,80) 1.0. */
void orc_encode_padded(const float* queries, int64_t n, float* enc);
/* kind flag: the queries are non-compact 16-float records (orc_encode_padded; Frequency only here, Hash: the
 * orc_hash_*_layout functions) */
#define ORC_KIND_PADDED 16
/* orc_forward / orc_grad for an encoding kind (NRC_ENCODING_FREQUENCY or NRC_ENCODING_FREQUENCY_SH, | ORC_KIND_PADDED) */
void orc_forward_enc(int kind, const float* params, const float* queries, int64_t n, int mode, float* out,
                     int nthreads);
double orc_grad_enc(int kind, const float* params, const float* queries, const float* targets, int64_t b,
                    double n_total, float loss_scale, int mode, float* grad, int nthreads);

/* tcnn Adam step followed by the EMA(decay) wrapper [M]. Updates params/m/v/ema in place and
 * writes the debiased EMA weights (the inference weights) to infer_params. step is 1-based. */
void orc_adam_ema(float* params, float* m, float* v, float* ema, float* infer_params,
                  uint32_t step, const float* grad, float loss_scale, float lr, float beta1,
                  float beta2, float eps, float l2_reg, float ema_decay, int64_t n);

/* tcnn-style xavier-uniform initialisation (per matrix, fan_in+fan_out of the padded shapes) from
 * a pcg32 stream; init parity with tcnn is not attainable [M], parity tests inject weights. */
void orc_init_params(float* params, uint64_t seed);


/* ---- width-128 network (nrc_wide_oracle.c; BASELINE configs[4]) ----
 * params: NRC_WIDE_NUM_PARAMS f32 canonical blob. kind: NRC_ENCODING_FREQUENCY or NRC_ENCODING_FREQUENCY_SH.
 * mode: ORC_FP32, ORC_MIXED or ORC_FP8 (spec in nrc_wide_oracle.c). */
void orc_wide_forward(int kind, const float* params, const float* queries, int64_t n, int mode, float* out,
                      int nthreads);
/* RNE onto OCP e4m3fn, |x| <= 448 */
float orc_e4m3(float x);
int orc_fp8_row_exponent(float amax);
/* FP8 inference weights (values incl. their row scale) and the row exponents exps[5][128] of W1..W5 */
void orc_wide_quantize(const float* params, float* q, int32_t* exps);
/* loss-scaled gradient + loss of one minibatch (ORC_FP32 / ORC_MIXED), as orc_grad_enc at width 128; the optimizer
 * step is orc_adam_ema with n = NRC_WIDE_NUM_PARAMS. */
double orc_wide_grad(int kind, const float* params, const float* queries, const float* targets, int64_t b,
                     double n_total, float loss_scale, int mode, float* grad, int nthreads);

/* ---- per-frame kernels around the network (nrc_frame_oracle.c) ---- */
void orc_accumulate(const float* radiance, const float* throughput, float* rgba, int64_t n, int mode,
                    uint32_t iteration_index);
void orc_propagate(const void* end_vertices, const float* end_radiance, int64_t num_tiles, const void* records,
                   float* targets, int64_t num_records);
/* USE_REFLECTANCE_FACTORING 1 forms (queries: compact RadianceQuery arrays, 15 floats per record) */
void orc_accumulate_factored(const float* radiance, const float* throughput, const float* queries, float* rgba,
                             int64_t n, int mode, uint32_t iteration_index);
void orc_propagate_factored(const void* end_vertices, const float* end_radiance, const float* end_queries,
                            int64_t num_tiles, const void* records, float* targets, const float* train_queries,
                            int64_t num_records);
void orc_feistel_keys(uint64_t seed, uint32_t frame, uint32_t keys[4]);
void orc_permutation(uint64_t seed, uint32_t frame, int32_t* perm, uint32_t n);
void orc_sort_pairs(const uint32_t* keys, uint32_t* sorted_keys, int32_t* perm, uint32_t n);
void orc_permute(const float* q_src, const float* t_src, const int32_t* perm, uint64_t seed, uint32_t frame,
                 int32_t num_records, float* q_dst, float* t_dst, uint32_t n_out);

/* ---- InputEncoding::Hash model (nrc_hash_oracle.c; NRCNetworkConfigs.h:84-128) ----
 * params: NRC_HASH_NUM_PARAMS f32 = MLP (W0[64][64] ...) then the grid table [entry][2]. */
void orc_hash_encode(const float* params, const float* queries, int64_t n, int mode, float* enc /* n x 64 */);
void orc_hash_forward(const float* params, const float* queries, int64_t n, int mode, float* out, int nthreads);
double orc_hash_grad(const float* params, const float* queries, const float* targets, int64_t b, double n_total,
                     float loss_scale, int mode, float* grad, int nthreads);
/* the same for a query layout (NRC_QUERY_COMPACT / NRC_QUERY_PADDED: the padded encoding is HashGrid 0..31 | pad_ 32 |
 * OneBlob 33..56 | Identity 57..62 | 1.0) */
void orc_hash_forward_layout(int layout, const float* params, const float* queries, int64_t n, int mode, float* out,
                             int nthreads);
double orc_hash_grad_layout(int layout, const float* params, const float* queries, const float* targets, int64_t b,
                            double n_total, float loss_scale, int mode, float* grad, int nthreads);
void orc_hash_adam_ema(float* params, float* m, float* v, float* ema, float* infer_params, uint32_t* grid_steps,
                       uint32_t step, const float* grad, float loss_scale, float lr, float beta1, float beta2,
                       float eps, float l2_reg, float ema_decay);
void orc_hash_init_params(float* params, uint64_t seed);
void orc_hash_corners(const float* q, int level, uint32_t* entries, float* weights);
/* round a double straight to the nearest f16 (RNE), as a half-precision FMA does */
float orc_f16_round_double(double x);

#ifdef __cplusplus
}
#endif

#endif
