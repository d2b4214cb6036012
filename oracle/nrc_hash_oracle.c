/*
 * nrc_hash_oracle.c — CPU restatement of the reference's InputEncoding::Hash model
 * (/root/reference/nrc/inc/NRCNetworkConfigs.h:84-128): Composite{HashGrid(pos), OneBlob, Identity} ->
 * FullyFusedMLP 64x5 ReLU/ReLU -> RelativeL2Luminance -> EMA(Adam(lr 1e-2, l2 1e-6, eps 1e-15)).
 *
 * TEST INFRASTRUCTURE ONLY (see nrc_oracle.h). PARITY UNPINNED, as for the Frequency model: the HashGrid
 * arithmetic lives in tiny-cuda-nn (encodings/grid.h), absent from the reference snapshot. Restated from the
 * published algorithm (Mueller et al. 2022, "Instant Neural Graphics Primitives", and tcnn's documented
 * GridEncoding) with spec choices tagged [H]/[M]/[L]:
 *  [H] level l: scale = 2^(l log2 b) * N_min - 1 = 16*2^l - 1, resolution = ceil(scale) + 1 = 16*2^l;
 *      entries = min(resolution^3, 2^15), rounded up to a multiple of 8 (levels 0, 1 dense; 2..15 hashed).
 *  [H] pos = fmaf(scale, x, 0.5); cell = (uint32)(int)floorf(pos); frac = pos - floor; trilinear weights
 *      weight = prod_d (corner_d ? frac_d : 1 - frac_d), f32, dims in order 0, 1, 2.
 *  [H] dense index x + y*res + z*res^2 (uint32 wrap-around), hashed index x ^ y*2654435761 ^ z*805459861;
 *      both taken modulo the level's entry count. Inputs outside [0, 1] (the reference feeds position*0.005,
 *      i.e. [-0.05, 0.05]) wrap through the uint32 cell index exactly as the formula does.
 *  [M] grid parameters initialised uniform in [-1e-4, 1e-4]; stored as f16 for the forward (PARAMS_T);
 *      interpolation as tcnn's kernel_grid: result = fma((half)weight, value, result) in half precision,
 *      corners in order 0..7 (MIXED and TCNN modes; the GPU's v_pk_fma_f16). FP32 mode: exact f64 sum.
 *  [M] grid gradient: sum over samples and corners of weight * dL/dfeature; tcnn accumulates it with half2
 *      atomics [L], as the GPU build does. Here (MIXED / TCNN) every contribution weight * dy is rounded to f16,
 *      the contributions are summed in f64 and the sum is rounded to f16; the atomics' per-add f16 rounding in
 *      arbitrary order is not reproducible, so the tests compare the grid update with sign / support tolerances.
 *  [M] tcnn Adam treats the grid as non-matrix parameters: no l2 regularisation, an entry whose gradient is
 *      exactly zero is skipped (moments, weight and its step counter untouched), and bias correction uses
 *      the entry's own step counter. The EMA wrapper filters every parameter every step [L].
 */
#include "nrc_oracle.h"
#include "../include/nrc/layout.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define HL NRC_HASH_LEVELS
#define ENC NRC_HASH_ENC_WIDTH

static const int kIn[NRC_NUM_LAYERS] = {ENC, 64, 64, 64, 64, 64};
static const int kOut[NRC_NUM_LAYERS] = {64, 64, 64, 64, 64, NRC_OUT_PADDED};
static int layer_off(int l) { return l == 0 ? 0 : (l <= 4 ? NRC_HASH_W1_OFFSET + (l - 1) * 4096 : NRC_HASH_W5_OFFSET); }

static uint32_t level_entries(int l) { return l == 0 ? 4096u : (uint32_t)NRC_HASH_T; }

/* corner indices (level-local entries) and trilinear weights of one level */
static void level_corners(int l, const float x[3], uint32_t idx[8], float w[8]) {
    const float scale = ldexpf(16.0f, l) - 1.0f;
    const uint32_t res = 16u << l;
    float fr[3];
    uint32_t cell[3];
    for (int d = 0; d < 3; ++d) {
        const float pos = fmaf(scale, x[d], 0.5f);
        const float fl = floorf(pos);
        cell[d] = (uint32_t)(int32_t)fl;
        fr[d] = pos - fl;
    }
    const uint32_t mask = level_entries(l) - 1u;
    for (int c = 0; c < 8; ++c) {
        float wt = 1.0f;
        uint32_t g[3];
        for (int d = 0; d < 3; ++d) {
            const int bit = (c >> d) & 1;
            wt *= bit ? fr[d] : 1.0f - fr[d];
            g[d] = cell[d] + (uint32_t)bit;
        }
        uint32_t i;
        if (l <= 1) i = g[0] + g[1] * res + g[2] * res * res; /* dense levels: res^3 <= 2^15 */
        else i = g[0] ^ (g[1] * NRC_HASH_PRIME1) ^ (g[2] * NRC_HASH_PRIME2);
        idx[c] = i & mask;
        w[c] = wt;
    }
}

/* Round-to-nearest-even of a double straight to the nearest f16 value (no intermediate f32 rounding, which
 * could double-round): scale to the f16 ulp of |x|, nearbyint (RNE in the default mode), scale back. */
float orc_f16_round_double(double x) {
    if (x != x || x == 0.0) return (float)x;
    const double ax = fabs(x);
    int e;
    frexp(ax, &e);                      /* ax = m * 2^e, m in [0.5, 1) */
    int ulp_exp = (e - 1) - 10;         /* f16 has 10 fraction bits */
    if (ulp_exp < -24) ulp_exp = -24;   /* subnormal f16 spacing */
    const double r = ldexp(nearbyint(ldexp(x, -ulp_exp)), ulp_exp);
    if (fabs(r) > 65504.0) return x > 0 ? INFINITY : -INFINITY;
    return (float)r;
}

/* Grid table as the forward sees it (f16-rounded in MIXED / TCNN). */
static float* grid_view(const float* grid, int mode) {
    float* t = (float*)malloc(sizeof(float) * NRC_HASH_GRID_PARAMS);
    for (int i = 0; i < NRC_HASH_GRID_PARAMS; ++i) t[i] = mode == ORC_FP32 ? grid[i] : orc_f16_round(grid[i]);
    return t;
}

/* enc[64] of one query (padq: a non-compact 16-float record); table = grid_view() */
static void encode_one(const float* table, const float* q, int mode, float* enc, int padq) {
    for (int l = 0; l < HL; ++l) {
        uint32_t idx[8];
        float w[8];
        level_corners(l, q, idx, w);
        const float* T = table + 2 * (size_t)NRC_HASH_LEVEL_ENTRY_OFFSET(l);
        for (int f = 0; f < 2; ++f) {
            if (mode == ORC_FP32) {
                double acc = 0.0;
                for (int c = 0; c < 8; ++c) acc += (double)w[c] * (double)T[2 * idx[c] + f];
                enc[2 * l + f] = (float)acc;
            } else { /* half fma: the product of two halves and a half addend are exact in f64, one rounding */
                float acc = 0.0f;
                for (int c = 0; c < 8; ++c)
                    acc = orc_f16_round_double((double)orc_f16_round(w[c]) * (double)T[2 * idx[c] + f] + (double)acc);
                enc[2 * l + f] = acc;
            }
        }
    }
    /* OneBlob(dims 3-8) and Identity(dims 9-14): the Frequency composite's features 36..65 (padded records: pad_,
     * then the padded composite's 37..66, NRCNetworkConfigs.h:106-111) */
    float full[NRC_ENC_WIDTH];
    if (padq) {
        orc_encode_padded(q, 1, full);
        for (int k = 0; k < 31; ++k) enc[32 + k] = (mode == ORC_FP32) ? full[36 + k] : orc_f16_round(full[36 + k]);
        enc[63] = 1.0f;
        return;
    }
    orc_encode(q, 1, full);
    for (int k = 0; k < 30; ++k) enc[32 + k] = (mode == ORC_FP32) ? full[36 + k] : orc_f16_round(full[36 + k]);
    enc[62] = enc[63] = 1.0f; /* Composite padding to the FullyFusedMLP width [M] */
}

void orc_hash_encode(const float* params, const float* queries, int64_t n, int mode, float* enc) {
    float* table = grid_view(params + NRC_HASH_GRID_OFFSET, mode);
    for (int64_t s = 0; s < n; ++s) encode_one(table, queries + s * NRC_INPUT_DIMS, mode, enc + s * ENC, 0);
    free(table);
}

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

static void matvec_t(const float* W, const float* d, int out_dim, int in_dim, int mode, float* x) {
    for (int k = 0; k < in_dim; ++k) {
        double acc = 0.0;
        if (mode == ORC_TCNN) {
            float a = 0.0f;
            for (int c = 0; c < out_dim; c += 16) {
                double part = 0.0;
                for (int o = c; o < c + 16 && o < out_dim; ++o) part += (double)W[(int64_t)o * in_dim + k] * (double)d[o];
                a = orc_f16_round((float)((double)a + part));
            }
            x[k] = a;
            continue;
        }
        for (int o = 0; o < out_dim; ++o) acc += (double)W[(int64_t)o * in_dim + k] * (double)d[o];
        x[k] = (float)acc;
    }
}

typedef struct {
    float enc[ENC];
    float a[5][64];
    float y[NRC_OUT_PADDED];
} acts_t;

static float rnd(float v, int mode) { return mode == ORC_FP32 ? v : orc_f16_round(v); }

static void forward_one(const float* w, const float* table, const float* q, int mode, acts_t* A, int padq) {
    encode_one(table, q, mode, A->enc, padq);
    const float* in = A->enc;
    for (int l = 0; l < 5; ++l) {
        float z[64];
        matvec(w + layer_off(l), in, 64, kIn[l], mode, z);
        for (int o = 0; o < 64; ++o) A->a[l][o] = rnd(z[o] > 0.0f ? z[o] : 0.0f, mode);
        in = A->a[l];
    }
    float z[NRC_OUT_PADDED];
    matvec(w + layer_off(5), in, NRC_OUT_PADDED, 64, mode, z);
    for (int o = 0; o < NRC_OUT_PADDED; ++o) A->y[o] = rnd(z[o] > 0.0f ? z[o] : 0.0f, mode);
}

typedef struct {
    const float *w, *table, *queries, *targets;
    int64_t begin, end;
    int mode;
    int padq; /* non-compact 16-float records */
    float* out;
    double n_total;
    float loss_scale;
    double *grad, loss;
} job_t;

static void* fwd_job(void* arg) {
    job_t* J = (job_t*)arg;
    acts_t A;
    for (int64_t s = J->begin; s < J->end; ++s) {
        forward_one(J->w, J->table, J->queries + s * (J->padq ? NRC_INPUT_DIMS_PADDED : NRC_INPUT_DIMS), J->mode, &A,
                    J->padq);
        for (int c = 0; c < 3; ++c) J->out[s * 3 + c] = A.y[c];
    }
    return NULL;
}

static float* mlp_view(const float* params, int mode) {
    float* w = (float*)malloc(sizeof(float) * NRC_HASH_MLP_PARAMS);
    for (int i = 0; i < NRC_HASH_MLP_PARAMS; ++i) w[i] = rnd(params[i], mode);
    return w;
}

static int nthr(int t, int64_t n) {
    if (t < 1) t = 1;
    if (t > 256) t = 256;
    if ((int64_t)t > n) t = (int)(n > 0 ? n : 1);
    return t;
}

void orc_hash_forward(const float* params, const float* queries, int64_t n, int mode, float* out, int nthreads) {
    orc_hash_forward_layout(NRC_QUERY_COMPACT, params, queries, n, mode, out, nthreads);
}

void orc_hash_forward_layout(int layout, const float* params, const float* queries, int64_t n, int mode, float* out,
                             int nthreads) {
    if (n <= 0) return;
    float* w = mlp_view(params, mode);
    float* table = grid_view(params + NRC_HASH_GRID_OFFSET, mode);
    nthreads = nthr(nthreads, n);
    job_t jobs[256];
    pthread_t th[256];
    for (int t = 0; t < nthreads; ++t) {
        memset(&jobs[t], 0, sizeof(job_t));
        jobs[t].w = w;
        jobs[t].table = table;
        jobs[t].queries = queries;
        jobs[t].begin = n * t / nthreads;
        jobs[t].end = n * (t + 1) / nthreads;
        jobs[t].mode = mode;
        jobs[t].padq = layout == NRC_QUERY_PADDED;
        jobs[t].out = out;
        if (nthreads > 1) pthread_create(&th[t], NULL, fwd_job, &jobs[t]);
        else fwd_job(&jobs[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(w);
    free(table);
}

/* RelativeL2Luminance + backward through the MLP and into the grid (see nrc_oracle.c grad_job) */
static void* grad_job(void* arg) {
    job_t* J = (job_t*)arg;
    const int mode = J->mode;
    acts_t A;
    const float n_total = (float)J->n_total;
    for (int64_t s = J->begin; s < J->end; ++s) {
        const float* q = J->queries + s * (J->padq ? NRC_INPUT_DIMS_PADDED : NRC_INPUT_DIMS);
        forward_one(J->w, J->table, q, mode, &A, J->padq);
        const float* t = J->targets + s * 3;
        const float lum = 0.299f * A.y[0] + 0.587f * A.y[1] + 0.114f * A.y[2];
        const float denom = lum * lum + NRC_LUM_EPS;
        float d5[NRC_OUT_PADDED] = {0};
        for (int c = 0; c < 3; ++c) {
            const float diff = A.y[c] - t[c];
            J->loss += (double)(diff * diff / denom / n_total);
            const float g = rnd(J->loss_scale * 2.0f * diff / denom / n_total, mode);
            d5[c] = A.y[c] > 0.0f ? g : 0.0f;
        }
        const float* delta = d5;
        int dout = NRC_OUT_PADDED;
        float dbuf[2][64];
        for (int l = 5; l >= 0; --l) {
            const float* in = l == 0 ? A.enc : A.a[l - 1];
            double* gW = J->grad + layer_off(l);
            for (int o = 0; o < dout; ++o) {
                const double d = (double)delta[o];
                if (d == 0.0) continue;
                for (int k = 0; k < kIn[l]; ++k) gW[(int64_t)o * kIn[l] + k] += d * (double)in[k];
            }
            float* nd = dbuf[l & 1];
            matvec_t(J->w + layer_off(l), delta, dout, kIn[l], mode, nd);
            if (l == 0) {
                /* dL/d(grid feature), f16 in MIXED / TCNN, scattered with the trilinear weights */
                for (int lv = 0; lv < HL; ++lv) {
                    uint32_t idx[8];
                    float w[8];
                    level_corners(lv, q, idx, w);
                    double* G = J->grad + NRC_HASH_GRID_OFFSET + 2 * (size_t)NRC_HASH_LEVEL_ENTRY_OFFSET(lv);
                    for (int f = 0; f < 2; ++f) {
                        const float dy = rnd(nd[2 * lv + f], mode);
                        if (dy == 0.0f) continue;
                        for (int c = 0; c < 8; ++c)
                            G[2 * idx[c] + f] += mode == ORC_FP32 ? (double)w[c] * (double)dy
                                                                  : (double)orc_f16_round(w[c] * dy);
                    }
                }
                break;
            }
            for (int k = 0; k < kIn[l]; ++k) nd[k] = rnd(in[k] > 0.0f ? nd[k] : 0.0f, mode);
            delta = nd;
            dout = kIn[l];
        }
    }
    return NULL;
}

double orc_hash_grad(const float* params, const float* queries, const float* targets, int64_t b, double n_total,
                     float loss_scale, int mode, float* grad, int nthreads) {
    return orc_hash_grad_layout(NRC_QUERY_COMPACT, params, queries, targets, b, n_total, loss_scale, mode, grad,
                                nthreads);
}

double orc_hash_grad_layout(int layout, const float* params, const float* queries, const float* targets, int64_t b,
                            double n_total, float loss_scale, int mode, float* grad, int nthreads) {
    for (int i = 0; i < NRC_HASH_NUM_PARAMS; ++i) grad[i] = 0.0f;
    if (b <= 0) return 0.0;
    float* w = mlp_view(params, mode);
    float* table = grid_view(params + NRC_HASH_GRID_OFFSET, mode);
    nthreads = nthr(nthreads, b);
    job_t* jobs = (job_t*)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t th[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].w = w;
        jobs[t].table = table;
        jobs[t].queries = queries;
        jobs[t].targets = targets;
        jobs[t].begin = b * t / nthreads;
        jobs[t].end = b * (t + 1) / nthreads;
        jobs[t].mode = mode;
        jobs[t].padq = layout == NRC_QUERY_PADDED;
        jobs[t].n_total = n_total;
        jobs[t].loss_scale = loss_scale;
        jobs[t].grad = (double*)calloc(NRC_HASH_NUM_PARAMS, sizeof(double));
        if (nthreads > 1) pthread_create(&th[t], NULL, grad_job, &jobs[t]);
        else grad_job(&jobs[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    double loss = 0.0;
    for (int i = 0; i < NRC_HASH_NUM_PARAMS; ++i) {
        double acc = 0.0;
        for (int t = 0; t < nthreads; ++t) acc += jobs[t].grad[i];
        /* the grid gradient is an f16 buffer (half2 atomics) except in FP32 mode */
        grad[i] = (i >= NRC_HASH_GRID_OFFSET && mode != ORC_FP32) ? orc_f16_round_double(acc) : (float)acc;
    }
    for (int t = 0; t < nthreads; ++t) {
        loss += jobs[t].loss;
        free(jobs[t].grad);
    }
    free(jobs);
    free(w);
    free(table);
    return loss;
}

void orc_hash_adam_ema(float* params, float* m, float* v, float* ema, float* infer_params, uint32_t* grid_steps,
                       uint32_t step, const float* grad, float loss_scale, float lr, float beta1, float beta2,
                       float eps, float l2_reg, float ema_decay) {
    const float lr_t = lr * sqrtf(1.0f - powf(beta2, (float)step)) / (1.0f - powf(beta1, (float)step));
    const float ema_debias = 1.0f - powf(ema_decay, (float)step);
    for (int64_t i = 0; i < NRC_HASH_NUM_PARAMS; ++i) {
        float w = params[i];
        float gradient = grad[i] / loss_scale;
        const int is_matrix = i < NRC_HASH_MLP_PARAMS;
        int update = 1;
        float lr_i = lr_t;
        if (is_matrix) {
            gradient += l2_reg * w;
        } else if (gradient == 0.0f) {
            update = 0; /* sparse: untouched entries keep moments, weight and step */
        } else {
            uint32_t* st = &grid_steps[i - NRC_HASH_MLP_PARAMS];
            *st += 1;
            lr_i = lr * sqrtf(1.0f - powf(beta2, (float)*st)) / (1.0f - powf(beta1, (float)*st));
        }
        if (update) {
            const float gsq = gradient * gradient;
            const float m1 = m[i] = beta1 * m[i] + (1.0f - beta1) * gradient;
            const float v1 = v[i] = beta2 * v[i] + (1.0f - beta2) * gsq;
            const float eff = lr_i / (sqrtf(v1) + eps);
            w = w - eff * m1;
            params[i] = w;
        }
        const float e = ema[i] = ema[i] * ema_decay + w * (1.0f - ema_decay);
        infer_params[i] = e / ema_debias;
    }
}

typedef struct { uint64_t state, inc; } pcg_t;
static uint32_t pcg_next(pcg_t* r) {
    uint64_t old = r->state;
    r->state = old * 6364136223846793005ULL + r->inc;
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((~rot + 1u) & 31));
}
static float pcg_float(pcg_t* r) {
    union { uint32_t u; float f; } x;
    x.u = (pcg_next(r) >> 9) | 0x3f800000u;
    return x.f - 1.0f;
}

/* MLP: xavier-uniform per matrix from pcg32(seed, 0xda3e39cb94b95bdb) (as orc_init_params); grid: uniform
 * [-1e-4, 1e-4] from pcg32(seed, 0x9e3779b97f4a7c15) [M]. */
void orc_hash_init_params(float* params, uint64_t seed) {
    pcg_t r = {0u, (0xda3e39cb94b95bdbULL << 1u) | 1u};
    pcg_next(&r);
    r.state += seed;
    pcg_next(&r);
    for (int l = 0; l < NRC_NUM_LAYERS; ++l) {
        const float scale = sqrtf(6.0f / (float)(kIn[l] + kOut[l]));
        for (int i = 0; i < kIn[l] * kOut[l]; ++i) params[layer_off(l) + i] = (pcg_float(&r) * 2.0f - 1.0f) * scale;
    }
    pcg_t g = {0u, (0x9e3779b97f4a7c15ULL << 1u) | 1u};
    pcg_next(&g);
    g.state += seed;
    pcg_next(&g);
    for (int i = 0; i < NRC_HASH_GRID_PARAMS; ++i)
        params[NRC_HASH_GRID_OFFSET + i] = (pcg_float(&g) * 2.0f - 1.0f) * 1e-4f;
}

/* Corner indices (global table entries) and weights of query q, level l — for tests. */
void orc_hash_corners(const float* q, int level, uint32_t* entries, float* weights) {
    uint32_t idx[8];
    level_corners(level, q, idx, weights);
    for (int c = 0; c < 8; ++c) entries[c] = (uint32_t)NRC_HASH_LEVEL_ENTRY_OFFSET(level) + idx[c];
}
