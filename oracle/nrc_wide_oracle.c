/*
 * nrc_wide_oracle.c — CPU restatement of the width-128 network of BASELINE.json configs[4] (SURVEY.md §8 C5:
 * "128-wide MLP, CDNA4 fp8 MFMA"): forward (csrc/nrc_kernels.hip infer_wide_kernel) and training gradient
 * (wide_fwd_bwd_kernel + wide_dw_kernel).
 *
 * TEST INFRASTRUCTURE ONLY (see nrc_oracle.h): only tests/, smoke() and bench.py's cpu_baseline leg load it.
 *
 * PARITY UNPINNED, and beyond the reference: the reference only configures "n_neurons": 64
 * (/root/reference/nrc/inc/NRCNetworkConfigs.h:26-33); C5 is BASELINE's stretch config. The model is that
 * FullyFusedMLP with n_neurons = 128 — W0[128][80], W1..W4[128][128], W5[16][128], no biases, ReLU hidden and
 * output, same Composite encodings (orc_encode / orc_encode_sh) — in the canonical blob order of
 * include/nrc/layout.h (NRC_WIDE_*). Numerics modes:
 *   ORC_FP32  : f32 weights and activations, f64 dot products rounded to f32 per layer.
 *   ORC_MIXED : the 64-wide build's model at width 128: f16 inputs/weights/activations, f32 accumulation, f16 output.
 *   ORC_FP8   : the FP8 inference path (spec choice of this build):
 *               layer 0 as MIXED (f16 encoding x f16 W0, f32 accumulation);
 *               every layer's ReLU output is clamped to [0, 448] and rounded to nearest even onto OCP e4m3fn
 *               (= med3(y, 0, 448) + v_cvt_pk_fp8_f32, checked bit-exact on gfx950 by tools/microbench/fp8_probe);
 *               W1..W5 are e4m3fn with one power-of-two scale 2^e per output row, e the smallest integer with
 *               max_k |W[row][k]| <= 448 * 2^e (E8M0 scale of the MX-scaled MFMA), elements RNE(W / 2^e);
 *               dot products in f64 rounded to f32 (the hardware's 64-element fp8 block sum is not f32-exact:
 *               error <= ~2.2e-5 of sum|a*b|, fp8_probe), final ReLU output rounded to f16 as the f16 path does.
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "../include/nrc/layout.h"
#include "nrc_oracle.h"

static const int kWIn[NRC_NUM_LAYERS] = {NRC_ENC_WIDTH, NRC_WIDE_WIDTH, NRC_WIDE_WIDTH, NRC_WIDE_WIDTH,
                                         NRC_WIDE_WIDTH, NRC_WIDE_WIDTH};
static const int kWOut[NRC_NUM_LAYERS] = {NRC_WIDE_WIDTH, NRC_WIDE_WIDTH, NRC_WIDE_WIDTH,
                                          NRC_WIDE_WIDTH, NRC_WIDE_WIDTH, NRC_OUT_PADDED};
static const int kWOff[NRC_NUM_LAYERS] = {NRC_WIDE_W0_OFFSET, NRC_WIDE_W1_OFFSET, NRC_WIDE_W1_OFFSET + 16384,
                                          NRC_WIDE_W1_OFFSET + 32768, NRC_WIDE_W1_OFFSET + 49152, NRC_WIDE_W5_OFFSET};

/* RNE onto OCP e4m3fn (bias 7, 3 mantissa bits, subnormals 2^-9 * m), |x| <= 448 assumed. */
float orc_e4m3(float x) {
    const double a = fabs((double)x);
    if (a == 0.0) return x;
    int e = 0;
    frexp(a, &e);
    int eq = e - 1; /* floor(log2 a) */
    if (eq < -6) eq = -6;
    const double quantum = ldexp(1.0, eq - 3);
    const double v = nearbyint(a / quantum) * quantum; /* exact scaling; nearbyint rounds half to even */
    return (float)(x < 0.0f ? -v : v);
}

/* smallest e with amax <= 448 * 2^e (448 = 0.875 * 2^9), clamped to the E8M0 range; 0 for an all-zero row */
int orc_fp8_row_exponent(float amax) {
    if (!(amax > 0.0f)) return 0;
    int E = 0;
    const float M = frexpf(amax, &E); /* amax = M * 2^E, M in [0.5, 1) */
    int e = M <= 0.875f ? E - 9 : E - 8;
    if (e < -127) e = -127;
    if (e > 127) e = 127;
    return e;
}

/* FP8 inference weights: q[p] = RNE_e4m3(W / 2^e_row) * 2^e_row for W1..W5 (exact in f32); W0 = f16(W).
 * exps[(l - 1) * 128 + row] = e_row for l = 1..5 (rows 16..127 of W5: 0). */
void orc_wide_quantize(const float* params, float* q, int32_t* exps) {
    for (int i = 0; i < NRC_WIDE_W1_OFFSET; ++i) q[i] = orc_f16_round(params[i]);
    for (int l = 1; l < NRC_NUM_LAYERS; ++l) {
        for (int row = 0; row < NRC_WIDE_WIDTH; ++row) {
            if (row >= kWOut[l]) {
                exps[(l - 1) * NRC_WIDE_WIDTH + row] = 0;
                continue;
            }
            const float* w = params + kWOff[l] + row * kWIn[l];
            float amax = 0.0f;
            for (int k = 0; k < kWIn[l]; ++k) amax = fmaxf(amax, fabsf(w[k]));
            const int e = orc_fp8_row_exponent(amax);
            exps[(l - 1) * NRC_WIDE_WIDTH + row] = e;
            for (int k = 0; k < kWIn[l]; ++k)
                q[kWOff[l] + row * kWIn[l] + k] = ldexpf(orc_e4m3(ldexpf(w[k], -e)), e);
        }
    }
}

static float act_fp8(float y) {
    const float c = y < 0.0f ? 0.0f : (y > 448.0f ? 448.0f : y);
    return orc_e4m3(c);
}

static void wide_forward_one(const float* w, const float* q, int mode, int kind, float* out3) {
    float buf[2][NRC_WIDE_WIDTH];
    float enc[NRC_ENC_WIDTH];
    if (kind == NRC_ENCODING_FREQUENCY_SH) orc_encode_sh(q, 1, enc);
    else orc_encode(q, 1, enc);
    if (mode != ORC_FP32)
        for (int f = 0; f < NRC_ENC_WIDTH; ++f) enc[f] = orc_f16_round(enc[f]);
    const float* in = enc;
    for (int l = 0; l < NRC_NUM_LAYERS; ++l) {
        float* o = buf[l & 1];
        for (int r = 0; r < kWOut[l]; ++r) {
            const float* wr = w + kWOff[l] + r * kWIn[l];
            double acc = 0.0;
            for (int k = 0; k < kWIn[l]; ++k) acc += (double)wr[k] * (double)in[k];
            const float y = (float)acc;
            const float a = y > 0.0f ? y : 0.0f;
            if (l == NRC_NUM_LAYERS - 1 || mode == ORC_MIXED) o[r] = mode == ORC_FP32 ? a : orc_f16_round(a);
            else if (mode == ORC_FP8) o[r] = act_fp8(y);
            else o[r] = a;
        }
        in = o;
    }
    for (int c = 0; c < NRC_OUTPUT_DIMS; ++c) out3[c] = in[c];
}

typedef struct {
    const float* w;
    const float* queries;
    int64_t begin, end;
    int mode, kind;
    float* out;
} wide_job;

static void* wide_job_run(void* arg) {
    wide_job* J = (wide_job*)arg;
    for (int64_t s = J->begin; s < J->end; ++s)
        wide_forward_one(J->w, J->queries + s * NRC_INPUT_DIMS, J->mode, J->kind, J->out + s * NRC_OUTPUT_DIMS);
    return NULL;
}

void orc_wide_forward(int kind, const float* params, const float* queries, int64_t n, int mode, float* out,
                      int nthreads) {
    if (n <= 0) return;
    float* w = (float*)malloc(sizeof(float) * NRC_WIDE_NUM_PARAMS);
    if (mode == ORC_FP8) {
        int32_t* exps = (int32_t*)malloc(sizeof(int32_t) * 5 * NRC_WIDE_WIDTH);
        orc_wide_quantize(params, w, exps);
        free(exps);
    } else {
        for (int i = 0; i < NRC_WIDE_NUM_PARAMS; ++i) w[i] = mode == ORC_FP32 ? params[i] : orc_f16_round(params[i]);
    }
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((int64_t)nthreads > n) nthreads = (int)n;
    pthread_t th[256];
    wide_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].w = w;
        jobs[t].queries = queries;
        jobs[t].begin = n * t / nthreads;
        jobs[t].end = n * (t + 1) / nthreads;
        jobs[t].mode = mode;
        jobs[t].kind = kind;
        jobs[t].out = out;
        if (nthreads > 1) pthread_create(&th[t], NULL, wide_job_run, &jobs[t]);
        else wide_job_run(&jobs[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(w);
}

/* ---- training (ORC_FP32 / ORC_MIXED): the 64-wide grad_job of nrc_oracle.c at width 128 ----
 * forward as orc_wide_forward; RelativeL2Luminance gradient (loss-scaled, f16 in MIXED), ReLU output gate;
 * delta chain delta_{l-1} = relu'(a_{l-1}) (W_l^T delta_l), f16-rounded in MIXED; dW_l = sum_s delta_l in_l^T in f64. */
typedef struct {
    const float* w;
    const float* queries;
    const float* targets;
    int64_t begin, end;
    int mode, kind;
    float n_total, loss_scale;
    double* grad;
    double loss;
} wide_grad_job;

static void* wide_grad_run(void* arg) {
    wide_grad_job* J = (wide_grad_job*)arg;
    const int mode = J->mode;
    float enc[NRC_ENC_WIDTH], act[5][NRC_WIDE_WIDTH], y[NRC_OUT_PADDED];
    float d[2][NRC_WIDE_WIDTH];
    for (int64_t s = J->begin; s < J->end; ++s) {
        const float* q = J->queries + s * NRC_INPUT_DIMS;
        if (J->kind == NRC_ENCODING_FREQUENCY_SH) orc_encode_sh(q, 1, enc);
        else orc_encode(q, 1, enc);
        if (mode != ORC_FP32)
            for (int f = 0; f < NRC_ENC_WIDTH; ++f) enc[f] = orc_f16_round(enc[f]);
        const float* in = enc;
        for (int l = 0; l < NRC_NUM_LAYERS; ++l) {
            float* o = l < 5 ? act[l] : y;
            for (int r = 0; r < kWOut[l]; ++r) {
                const float* wr = J->w + kWOff[l] + r * kWIn[l];
                double acc = 0.0;
                for (int k = 0; k < kWIn[l]; ++k) acc += (double)wr[k] * (double)in[k];
                const float a = (float)acc > 0.0f ? (float)acc : 0.0f;
                o[r] = mode == ORC_FP32 ? a : orc_f16_round(a);
            }
            in = o;
        }
        const float* t = J->targets + s * NRC_OUTPUT_DIMS;
        const float lum = 0.299f * y[0] + 0.587f * y[1] + 0.114f * y[2];
        const float denom = lum * lum + NRC_LUM_EPS;
        float* delta = d[1];
        for (int c = 0; c < NRC_OUT_PADDED; ++c) delta[c] = 0.0f;
        for (int c = 0; c < NRC_OUTPUT_DIMS; ++c) {
            const float diff = y[c] - t[c];
            J->loss += (double)(diff * diff / denom / J->n_total);
            float g = J->loss_scale * 2.0f * diff / denom / J->n_total;
            if (mode != ORC_FP32) g = orc_f16_round(g);
            delta[c] = y[c] > 0.0f ? g : 0.0f;
        }
        int dout = NRC_OUT_PADDED;
        for (int l = NRC_NUM_LAYERS - 1; l >= 0; --l) {
            const float* inl = l == 0 ? enc : act[l - 1];
            const int in_dim = kWIn[l];
            double* gW = J->grad + kWOff[l];
            for (int o = 0; o < dout; ++o) {
                const double dd = (double)delta[o];
                if (dd == 0.0) continue;
                for (int k = 0; k < in_dim; ++k) gW[o * in_dim + k] += dd * (double)inl[k];
            }
            if (l == 0) break;
            float* nd = delta == d[0] ? d[1] : d[0];
            for (int k = 0; k < in_dim; ++k) {
                double acc = 0.0;
                for (int o = 0; o < dout; ++o) acc += (double)J->w[kWOff[l] + o * in_dim + k] * (double)delta[o];
                const float v = inl[k] > 0.0f ? (float)acc : 0.0f;
                nd[k] = mode == ORC_FP32 ? v : orc_f16_round(v);
            }
            delta = nd;
            dout = in_dim;
        }
    }
    return NULL;
}

double orc_wide_grad(int kind, const float* params, const float* queries, const float* targets, int64_t b,
                     double n_total, float loss_scale, int mode, float* grad, int nthreads) {
    for (int i = 0; i < NRC_WIDE_NUM_PARAMS; ++i) grad[i] = 0.0f;
    if (b <= 0) return 0.0;
    float* w = (float*)malloc(sizeof(float) * NRC_WIDE_NUM_PARAMS);
    for (int i = 0; i < NRC_WIDE_NUM_PARAMS; ++i) w[i] = mode == ORC_FP32 ? params[i] : orc_f16_round(params[i]);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((int64_t)nthreads > b) nthreads = (int)b;
    wide_grad_job* jobs = (wide_grad_job*)calloc((size_t)nthreads, sizeof(wide_grad_job));
    pthread_t th[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].w = w;
        jobs[t].queries = queries;
        jobs[t].targets = targets;
        jobs[t].begin = b * t / nthreads;
        jobs[t].end = b * (t + 1) / nthreads;
        jobs[t].mode = mode;
        jobs[t].kind = kind;
        jobs[t].n_total = (float)n_total;
        jobs[t].loss_scale = loss_scale;
        jobs[t].grad = (double*)calloc(NRC_WIDE_NUM_PARAMS, sizeof(double));
        if (nthreads > 1) pthread_create(&th[t], NULL, wide_grad_run, &jobs[t]);
        else wide_grad_run(&jobs[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    double loss = 0.0;
    for (int i = 0; i < NRC_WIDE_NUM_PARAMS; ++i) {
        double acc = 0.0;
        for (int t = 0; t < nthreads; ++t) acc += jobs[t].grad[i];
        grad[i] = (float)acc;
    }
    for (int t = 0; t < nthreads; ++t) {
        loss += jobs[t].loss;
        free(jobs[t].grad);
    }
    free(jobs);
    free(w);
    return loss;
}
