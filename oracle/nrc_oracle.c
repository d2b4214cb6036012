/*
 * nrc_oracle.c — CPU restatement of the NRC query/train arithmetic (tiny-cuda-nn as configured by
 * /root/reference/nrc/inc/NRCNetworkConfigs.h:11-83 and driven by /root/reference/nrc/src/NRCNetwork.cu).
 *
 * TEST INFRASTRUCTURE ONLY — see nrc_oracle.h. PARITY UNPINNED (tcnn source absent, no reference
 * fixtures); cross-checked against tests/oracle_np.py (float64) and torch autograd.
 *
 * Scalar C, no SIMD intrinsics, no BLAS. pthreads split samples across threads; every reduction
 * over samples is done in f64 per thread and summed in thread order.
 */
#include "nrc_oracle.h"
#include "../include/nrc/layout.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* binary16 round-to-nearest-even (tcnn __float2half)                                          */
/* ------------------------------------------------------------------------------------------ */
static uint16_t f32_to_f16_bits(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t exp = (x >> 23) & 0xffu;
    uint32_t mant = x & 0x7fffffu;
    if (exp == 0xffu) return (uint16_t)(sign | 0x7c00u | (mant ? (0x200u | (mant >> 13)) : 0u));
    int e = (int)exp - 127 + 15;
    if (e >= 31) return (uint16_t)(sign | 0x7c00u);
    if (e <= 0) {
        if (e < -10) return (uint16_t)sign;
        mant |= 0x800000u;
        int shift = 14 - e;
        uint32_t hm = mant >> shift;
        uint32_t rem = mant & ((1u << shift) - 1u);
        uint32_t halfway = 1u << (shift - 1);
        if (rem > halfway || (rem == halfway && (hm & 1u))) hm++;
        return (uint16_t)(sign | hm);
    }
    uint32_t hm = mant >> 13;
    uint32_t rem = mant & 0x1fffu;
    uint32_t h = sign | ((uint32_t)e << 10) | hm;
    if (rem > 0x1000u || (rem == 0x1000u && (hm & 1u))) h++;
    return (uint16_t)h;
}

static float f16_bits_to_f32(uint16_t h) {
    uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
    uint32_t exp = ((uint32_t)h >> 10) & 0x1fu;
    uint32_t mant = (uint32_t)h & 0x3ffu;
    uint32_t x;
    if (exp == 0) {
        if (mant == 0) {
            x = sign;
        } else {
            int e = -1;
            do { mant <<= 1; e++; } while (!(mant & 0x400u));
            mant &= 0x3ffu;
            x = sign | ((uint32_t)(127 - 15 - e) << 23) | (mant << 13);
        }
    } else if (exp == 31) {
        x = sign | 0x7f800000u | (mant << 13);
    } else {
        x = sign | ((exp - 15 + 127) << 23) | (mant << 13);
    }
    float f;
    memcpy(&f, &x, 4);
    return f;
}

float orc_f16_round(float x) { return f16_bits_to_f32(f32_to_f16_bits(x)); }

/* ------------------------------------------------------------------------------------------ */
/* Encoding                                                                                    */
/* ------------------------------------------------------------------------------------------ */

/* TriangleWave (tcnn encodings/triangle_wave.h) [M/L]: feature index d*n_frequencies + k holds
 * tri(2^k * x_d) (dimension-major, NRCNetworkConfigs.h:58-63). Spec choice [L]: period-1 wave in
 * [0,1], tri(u) = |2*(u - floor(u)) - 1|. 2^k scaling is exact (scalbnf). */
static float tri_wave(float x, int k) {
    float u = ldexpf(x, k);
    float fr = u - floorf(u);
    return fabsf(2.0f * fr - 1.0f);
}

/* OneBlob quartic-kernel CDF (tcnn encodings/oneblob.h) [M]: inv_radius = n_bins. */
static float quartic_cdf(float x, float inv_radius) {
    float u = x * inv_radius;
    float u2 = u * u;
    float u4 = u2 * u2;
    float v = (1.0f / 16.0f) * u * (15.0f - 10.0f * u2 + 3.0f * u4) + 0.5f;
    return fminf(fmaxf(v, 0.0f), 1.0f);
}

/* OneBlob, n_bins = 4 (NRCNetworkConfigs.h:72-76) [M]: bin b of dimension x holds
 *   right_cdf(b) - left_cdf(b),  left_cdf(b) = K(b/4 - x) + K(b/4 - x - 1) + K(b/4 - x + 1)
 *   right_cdf(b) = left_cdf(b+1) for b < 3, left_cdf(0) + 1 for b = 3 (period-1 wrap).
 * Inputs are the raw angles / roughness written by hit.cu:599-607; out-of-[0,1] inputs are NOT
 * normalised (the reference does not), and saturate as the formula dictates. */
static void one_blob(float x, float out[4]) {
    float left[4];
    for (int b = 0; b < 4; ++b) {
        float lb = ldexpf((float)b, -2);
        left[b] = quartic_cdf(lb - x, 4.0f) + quartic_cdf(lb - x - 1.0f, 4.0f) +
                  quartic_cdf(lb - x + 1.0f, 4.0f);
    }
    for (int b = 0; b < 4; ++b) {
        float right = (b < 3) ? left[b + 1] : left[0] + 1.0f;
        out[b] = right - left[b];
    }
}

void orc_encode(const float* queries, int64_t n, float* enc) {
    for (int64_t s = 0; s < n; ++s) {
        const float* q = queries + s * NRC_INPUT_DIMS;
        float* e = enc + s * NRC_ENC_WIDTH;
        for (int d = 0; d < NRC_TRI_DIMS; ++d)
            for (int k = 0; k < NRC_TRI_FREQS; ++k) e[d * NRC_TRI_FREQS + k] = tri_wave(q[d], k);
        for (int d = 0; d < NRC_BLOB_DIMS; ++d) one_blob(q[3 + d], e + 36 + d * NRC_BLOB_BINS);
        for (int d = 0; d < NRC_IDENT_DIMS; ++d) e[60 + d] = q[9 + d];
        /* Composite padding to the FullyFusedMLP input width with 1.0 [M] (survey A.4). */
        for (int f = NRC_ENC_REAL; f < NRC_ENC_WIDTH; ++f) e[f] = 1.0f;
    }
}

/* Non-compact RadianceQuery (USE_COMPACT_RADIANCE_QUERY 0; neural_radiance_caching.h:38-40, :107-111): 16 floats,
 * pad_ after the position; the Composite gains an Identity(1) of pad_ after the TriangleWave (NRCNetworkConfigs.h:61-67):
 * [0,36) TriangleWave | 36 pad_ | [37,61) OneBlob | [61,67) Identity | [67,80) padding 1.0 (tcnn's Composite pads the
 * 67 features to the FullyFusedMLP's input width 80 [M]). */
void orc_encode_padded(const float* queries, int64_t n, float* enc) {
    for (int64_t s = 0; s < n; ++s) {
        const float* q = queries + s * NRC_INPUT_DIMS_PADDED;
        float* e = enc + s * NRC_ENC_WIDTH;
        for (int d = 0; d < NRC_TRI_DIMS; ++d)
            for (int k = 0; k < NRC_TRI_FREQS; ++k) e[d * NRC_TRI_FREQS + k] = tri_wave(q[d], k);
        e[36] = q[3];
        for (int d = 0; d < NRC_BLOB_DIMS; ++d) one_blob(q[4 + d], e + 37 + d * NRC_BLOB_BINS);
        for (int d = 0; d < NRC_IDENT_DIMS; ++d) e[61 + d] = q[10 + d];
        for (int f = 67; f < NRC_ENC_WIDTH; ++f) e[f] = 1.0f;
    }
}

/* Extension encoding NRC_ENCODING_FREQUENCY_SH (not in the reference; BASELINE.json north_star "frequency +
 * one-blob + spherical-harmonics"): TriangleWave(pos) 36 | SphericalHarmonics degree 4 of the direction 16 |
 * OneBlob(normal theta/phi, roughness x/y) 16 | Identity(albedos) 6 | pad 1.0 x 6 = 80. The direction is the unit
 * vector of (theta, phi) under cartesianToSphericalUnitVector's convention (shader_common.h:320-333):
 * d = (sin t cos p, sin t sin p, cos t). SH basis and constants: the real SH of tcnn's SphericalHarmonics
 * encoding (degree 4 = 16 coefficients), evaluated on d directly. */
static void sh16(float x, float y, float z, float* o) {
    const float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
    o[0] = 0.28209479177387814f;
    o[1] = -0.48860251190291987f * y;
    o[2] = 0.48860251190291987f * z;
    o[3] = -0.48860251190291987f * x;
    o[4] = 1.0925484305920792f * xy;
    o[5] = -1.0925484305920792f * yz;
    o[6] = 0.94617469575755997f * z2 - 0.31539156525251999f;
    o[7] = -1.0925484305920792f * xz;
    o[8] = 0.54627421529603959f * x2 - 0.54627421529603959f * y2;
    o[9] = 0.59004358992664352f * y * (-3.0f * x2 + y2);
    o[10] = 2.8906114426405538f * xy * z;
    o[11] = 0.45704579946446572f * y * (1.0f - 5.0f * z2);
    o[12] = 0.3731763325901154f * z * (5.0f * z2 - 3.0f);
    o[13] = 0.45704579946446572f * x * (1.0f - 5.0f * z2);
    o[14] = 1.4453057213202769f * z * (x2 - y2);
    o[15] = 0.59004358992664352f * x * (-x2 + 3.0f * y2);
}

void orc_encode_sh(const float* queries, int64_t n, float* enc) {
    for (int64_t s = 0; s < n; ++s) {
        const float* q = queries + s * NRC_INPUT_DIMS;
        float* e = enc + s * NRC_ENC_WIDTH;
        for (int d = 0; d < NRC_TRI_DIMS; ++d)
            for (int k = 0; k < NRC_TRI_FREQS; ++k) e[d * NRC_TRI_FREQS + k] = tri_wave(q[d], k);
        const float st = sinf(q[3]), ct = cosf(q[3]), sp = sinf(q[4]), cp = cosf(q[4]);
        sh16(st * cp, st * sp, ct, e + 36);
        for (int d = 0; d < 4; ++d) one_blob(q[5 + d], e + 52 + d * NRC_BLOB_BINS);
        for (int d = 0; d < NRC_IDENT_DIMS; ++d) e[68 + d] = q[9 + d];
        for (int f = 74; f < NRC_ENC_WIDTH; ++f) e[f] = 1.0f;
    }
}

static void encode_kind(int kind, const float* q, float* enc) {
    if (kind & ORC_KIND_PADDED) orc_encode_padded(q, 1, enc);
    else if (kind == NRC_ENCODING_FREQUENCY_SH) orc_encode_sh(q, 1, enc);
    else orc_encode(q, 1, enc);
}
/* floats per RadianceQuery record of an encoding kind */
static int64_t kind_qdims(int kind) { return (kind & ORC_KIND_PADDED) ? NRC_INPUT_DIMS_PADDED : NRC_INPUT_DIMS; }

/* ------------------------------------------------------------------------------------------ */
/* Network                                                                                     */
/* ------------------------------------------------------------------------------------------ */
static const int kLayerIn[NRC_NUM_LAYERS] = {NRC_ENC_WIDTH, 64, 64, 64, 64, 64};
static const int kLayerOut[NRC_NUM_LAYERS] = {64, 64, 64, 64, 64, NRC_OUT_PADDED};
static const int kLayerOff[NRC_NUM_LAYERS] = {NRC_W0_OFFSET, NRC_W1_OFFSET, NRC_W2_OFFSET,
                                              NRC_W3_OFFSET, NRC_W4_OFFSET, NRC_W5_OFFSET};

static inline float relu(float x) { return x > 0.0f ? x : 0.0f; }

/* y[o] = sum_k W[o][k] x[k] (W row-major [out][in]) with the mode's accumulation numerics. */
static void matvec(const float* W, const float* x, int out_dim, int in_dim, int mode, float* y) {
    for (int o = 0; o < out_dim; ++o) {
        const float* w = W + (int64_t)o * in_dim;
        if (mode == ORC_TCNN) {
            float acc = 0.0f;
            for (int c = 0; c < in_dim; c += 16) {
                double part = 0.0;
                for (int k = c; k < c + 16 && k < in_dim; ++k) part += (double)w[k] * (double)x[k];
                acc = orc_f16_round((float)((double)acc + part));
            }
            y[o] = acc;
        } else {
            double acc = 0.0;
            for (int k = 0; k < in_dim; ++k) acc += (double)w[k] * (double)x[k];
            y[o] = (float)acc;
        }
    }
}

/* x[k] = sum_o W[o][k] d[o] (transposed product) */
static void matvec_t(const float* W, const float* d, int out_dim, int in_dim, int mode, float* x) {
    for (int k = 0; k < in_dim; ++k) {
        if (mode == ORC_TCNN) {
            float acc = 0.0f;
            for (int c = 0; c < out_dim; c += 16) {
                double part = 0.0;
                for (int o = c; o < c + 16 && o < out_dim; ++o)
                    part += (double)W[(int64_t)o * in_dim + k] * (double)d[o];
                acc = orc_f16_round((float)((double)acc + part));
            }
            x[k] = acc;
        } else {
            double acc = 0.0;
            for (int o = 0; o < out_dim; ++o) acc += (double)W[(int64_t)o * in_dim + k] * (double)d[o];
            x[k] = (float)acc;
        }
    }
}

/* Weights as the forward sees them: f16 copy of the f32 master in MIXED/TCNN (tcnn PARAMS_T). */
static float* mode_weights(const float* params, int mode) {
    float* w = (float*)malloc(sizeof(float) * NRC_NUM_PARAMS);
    for (int i = 0; i < NRC_NUM_PARAMS; ++i) w[i] = (mode == ORC_FP32) ? params[i] : orc_f16_round(params[i]);
    return w;
}

/* Per-sample forward. acts (optional): enc[80], a1..a5[64 each], y[16] — stored as the mode's
 * values (f16-rounded in MIXED/TCNN). */
typedef struct {
    float enc[NRC_ENC_WIDTH];
    float a[5][NRC_WIDTH];
    float y[NRC_OUT_PADDED];
} sample_acts;

static void forward_one(const float* w, const float* q, int mode, int kind, sample_acts* A) {
    encode_kind(kind, q, A->enc);
    if (mode != ORC_FP32)
        for (int f = 0; f < NRC_ENC_WIDTH; ++f) A->enc[f] = orc_f16_round(A->enc[f]);
    const float* in = A->enc;
    for (int l = 0; l < 5; ++l) {
        float z[NRC_WIDTH];
        matvec(w + kLayerOff[l], in, kLayerOut[l], kLayerIn[l], mode, z);
        for (int o = 0; o < NRC_WIDTH; ++o) {
            float v = relu(z[o]);
            A->a[l][o] = (mode == ORC_FP32) ? v : orc_f16_round(v);
        }
        in = A->a[l];
    }
    float z[NRC_OUT_PADDED];
    matvec(w + kLayerOff[5], in, NRC_OUT_PADDED, NRC_WIDTH, mode, z);
    for (int o = 0; o < NRC_OUT_PADDED; ++o) {
        float v = relu(z[o]); /* output_activation ReLU, NRCNetworkConfigs.h:29 */
        A->y[o] = (mode == ORC_FP32) ? v : orc_f16_round(v);
    }
}

typedef struct {
    const float* w;
    const float* queries;
    const float* targets;
    int64_t begin, end;
    int mode, kind;
    float* out;
    /* grad job */
    double n_total;
    float loss_scale;
    double* grad;
    double loss;
} job_t;

static void* forward_job(void* arg) {
    job_t* J = (job_t*)arg;
    sample_acts A;
    for (int64_t s = J->begin; s < J->end; ++s) {
        forward_one(J->w, J->queries + s * kind_qdims(J->kind), J->mode, J->kind, &A);
        for (int c = 0; c < NRC_OUTPUT_DIMS; ++c) J->out[s * NRC_OUTPUT_DIMS + c] = A.y[c];
    }
    return NULL;
}

static int clamp_threads(int nthreads, int64_t n) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((int64_t)nthreads > n) nthreads = (int)(n > 0 ? n : 1);
    return nthreads;
}

void orc_forward(const float* params, const float* queries, int64_t n, int mode, float* out,
                 int nthreads) {
    orc_forward_enc(NRC_ENCODING_FREQUENCY, params, queries, n, mode, out, nthreads);
}

void orc_forward_enc(int kind, const float* params, const float* queries, int64_t n, int mode, float* out,
                     int nthreads) {
    if (n <= 0) return;
    float* w = mode_weights(params, mode);
    nthreads = clamp_threads(nthreads, n);
    job_t jobs[256];
    pthread_t th[256];
    for (int t = 0; t < nthreads; ++t) {
        memset(&jobs[t], 0, sizeof(job_t));
        jobs[t].w = w;
        jobs[t].queries = queries;
        jobs[t].begin = n * t / nthreads;
        jobs[t].end = n * (t + 1) / nthreads;
        jobs[t].mode = mode;
        jobs[t].kind = kind;
        jobs[t].out = out;
        if (nthreads > 1) pthread_create(&th[t], NULL, forward_job, &jobs[t]);
        else forward_job(&jobs[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(w);
}

/* RelativeL2Luminance (tcnn losses/relative_l2_luminance.h) [M]: per channel c < 3,
 *   lum = 0.299 r + 0.587 g + 0.114 b of the prediction; denom = lum^2 + 0.01
 *   value = diff^2 / denom / n_total ; grad = loss_scale * 2 diff / denom / n_total
 * Padded output rows 3..15 get zero value and gradient. */
static void* grad_job(void* arg) {
    job_t* J = (job_t*)arg;
    const int mode = J->mode;
    const float* w = J->w;
    sample_acts A;
    const float n_total = (float)J->n_total;
    for (int64_t s = J->begin; s < J->end; ++s) {
        forward_one(w, J->queries + s * kind_qdims(J->kind), mode, J->kind, &A);
        const float* t = J->targets + s * NRC_OUTPUT_DIMS;
        const float lum = 0.299f * A.y[0] + 0.587f * A.y[1] + 0.114f * A.y[2];
        const float denom = lum * lum + NRC_LUM_EPS;
        float d5[NRC_OUT_PADDED];
        for (int c = 0; c < NRC_OUT_PADDED; ++c) d5[c] = 0.0f;
        for (int c = 0; c < NRC_OUTPUT_DIMS; ++c) {
            const float diff = A.y[c] - t[c];
            J->loss += (double)(diff * diff / denom / n_total);
            float g = J->loss_scale * 2.0f * diff / denom / n_total;
            if (mode != ORC_FP32) g = orc_f16_round(g);
            /* ReLU output activation backward: pass where the forward output is > 0 */
            d5[c] = (A.y[c] > 0.0f) ? g : 0.0f;
        }
        /* dW5 += d5 a5^T ; delta chain down to layer 0 */
        const float* delta = d5;
        int dout = NRC_OUT_PADDED;
        float dbuf[2][NRC_WIDTH];
        for (int l = 5; l >= 0; --l) {
            const float* in = (l == 0) ? A.enc : A.a[l - 1];
            const int in_dim = kLayerIn[l];
            double* gW = J->grad + kLayerOff[l];
            for (int o = 0; o < dout; ++o) {
                const double d = (double)delta[o];
                if (d == 0.0) continue;
                for (int k = 0; k < in_dim; ++k) gW[(int64_t)o * in_dim + k] += d * (double)in[k];
            }
            if (l == 0) break;
            float* nd = dbuf[l & 1];
            matvec_t(w + kLayerOff[l], delta, dout, in_dim, mode, nd);
            for (int k = 0; k < in_dim; ++k) {
                float v = (in[k] > 0.0f) ? nd[k] : 0.0f; /* ReLU backward on a_l */
                nd[k] = (mode == ORC_FP32) ? v : orc_f16_round(v);
            }
            delta = nd;
            dout = in_dim;
        }
    }
    return NULL;
}

double orc_grad(const float* params, const float* queries, const float* targets, int64_t b,
                double n_total, float loss_scale, int mode, float* grad, int nthreads) {
    return orc_grad_enc(NRC_ENCODING_FREQUENCY, params, queries, targets, b, n_total, loss_scale, mode, grad, nthreads);
}

double orc_grad_enc(int kind, const float* params, const float* queries, const float* targets, int64_t b,
                    double n_total, float loss_scale, int mode, float* grad, int nthreads) {
    for (int i = 0; i < NRC_NUM_PARAMS; ++i) grad[i] = 0.0f;
    if (b <= 0) return 0.0;
    float* w = mode_weights(params, mode);
    nthreads = clamp_threads(nthreads, b);
    job_t* jobs = (job_t*)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t th[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].w = w;
        jobs[t].queries = queries;
        jobs[t].targets = targets;
        jobs[t].begin = b * t / nthreads;
        jobs[t].end = b * (t + 1) / nthreads;
        jobs[t].mode = mode;
        jobs[t].kind = kind;
        jobs[t].n_total = n_total;
        jobs[t].loss_scale = loss_scale;
        jobs[t].grad = (double*)calloc(NRC_NUM_PARAMS, sizeof(double));
        if (nthreads > 1) pthread_create(&th[t], NULL, grad_job, &jobs[t]);
        else grad_job(&jobs[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    double loss = 0.0;
    for (int i = 0; i < NRC_NUM_PARAMS; ++i) {
        double acc = 0.0;
        for (int t = 0; t < nthreads; ++t) acc += jobs[t].grad[i];
        grad[i] = (mode == ORC_TCNN) ? orc_f16_round((float)acc) : (float)acc;
    }
    for (int t = 0; t < nthreads; ++t) {
        loss += jobs[t].loss;
        free(jobs[t].grad);
    }
    free(jobs);
    free(w);
    return loss;
}

/* ------------------------------------------------------------------------------------------ */
/* Optimizer: tcnn optimizers/adam.h adam_step [M] + optimizers/exponential_moving_average.h [M/L] */
/* ------------------------------------------------------------------------------------------ */
void orc_adam_ema(float* params, float* m, float* v, float* ema, float* infer_params,
                  uint32_t step, const float* grad, float loss_scale, float lr, float beta1,
                  float beta2, float eps, float l2_reg, float ema_decay, int64_t n) {
    /* Debiasing with the (1-based) step count; all parameters are matrix weights, so every
     * parameter steps every call and the per-parameter step counters of tcnn coincide. */
    const float lr_t = lr * sqrtf(1.0f - powf(beta2, (float)step)) / (1.0f - powf(beta1, (float)step));
    const float ema_debias = 1.0f - powf(ema_decay, (float)step);
    for (int64_t i = 0; i < n; ++i) {
        float gradient = grad[i] / loss_scale;
        const float w = params[i];
        gradient += l2_reg * w; /* l2_reg applies to matrix params (NRCNetworkConfigs.h:50) */
        const float gsq = gradient * gradient;
        const float m1 = m[i] = beta1 * m[i] + (1.0f - beta1) * gradient;
        const float v1 = v[i] = beta2 * v[i] + (1.0f - beta2) * gsq;
        const float eff = lr_t / (sqrtf(v1) + eps);
        const float nw = w - eff * m1;
        params[i] = nw;
        /* EMA(decay 0.99), NRCNetworkConfigs.h:19-23: filtered from the f32 master weights;
         * [L] debiased by 1 - decay^step for the inference copy. */
        const float e = ema[i] = ema[i] * ema_decay + nw * (1.0f - ema_decay);
        infer_params[i] = e / ema_debias;
    }
}

/* pcg32 (O'Neill), as tcnn's common/random.h. */
typedef struct { uint64_t state, inc; } pcg32;
static uint32_t pcg32_next(pcg32* r) {
    uint64_t old = r->state;
    r->state = old * 6364136223846793005ULL + r->inc;
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((~rot + 1u) & 31));
}
static void pcg32_seed(pcg32* r, uint64_t initstate, uint64_t initseq) {
    r->state = 0u;
    r->inc = (initseq << 1u) | 1u;
    pcg32_next(r);
    r->state += initstate;
    pcg32_next(r);
}
static float pcg32_float(pcg32* r) {
    union { uint32_t u; float f; } x;
    x.u = (pcg32_next(r) >> 9) | 0x3f800000u;
    return x.f - 1.0f;
}

void orc_init_params(float* params, uint64_t seed) {
    pcg32 rng;
    pcg32_seed(&rng, seed, 0xda3e39cb94b95bdbULL);
    for (int l = 0; l < NRC_NUM_LAYERS; ++l) {
        const float scale = sqrtf(6.0f / (float)(kLayerIn[l] + kLayerOut[l]));
        const int cnt = kLayerIn[l] * kLayerOut[l];
        for (int i = 0; i < cnt; ++i) params[kLayerOff[l] + i] = (pcg32_float(&rng) * 2.0f - 1.0f) * scale;
    }
}
