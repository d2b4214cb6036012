/*
 * nrc_frame_oracle.c — CPU restatement of the reference's per-frame NRC kernels around the network
 * (SURVEY.md §8(f) rows 2 and 4), scalar loops in the reference's own order.
 *
 * TEST INFRASTRUCTURE ONLY (see nrc_oracle.h): loaded by tests/ as the checker, never by the product.
 *
 * Parity pin: these kernels live in the reference itself (nrc/shaders/nrc_helpers.cu), not in the absent
 * tiny-cuda-nn, but they need CUDA + the renderer's SystemData and cannot be built here; the reference
 * holds no fixtures for them. The restatement follows the source line by line; floating-point contraction
 * follows nvcc's --use_fast_math build of the module (CMakeLists.txt:256-257, which implies --fmad=true):
 * every `a += b * c` on float3 is a per-component fmaf. The accumulation weight 1/(it+1) is the correctly
 * rounded quotient here and in the GPU build (nvcc's fast-math reciprocal may differ by 1 ulp). Denormal
 * flushing (fast-math ftz) is not emulated: fixtures stay in the normal range.
 */
#include "nrc_oracle.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float x, y, z; } f3;
typedef struct {
    int32_t prop_to;
    f3 lt;
    int32_t pixel, tile, len;
} train_record; /* neural_radiance_caching.h:57-75 */
typedef struct {
    int32_t start;
    float mask;
    int32_t pixel, tile;
} end_vertex; /* neural_radiance_caching.h:78-94 */

_Static_assert(sizeof(train_record) == 28, "TrainingRecord is 28 B");
_Static_assert(sizeof(end_vertex) == 16, "TrainingSuffixEndVertex is 16 B");

/* accumulate_render_radiance, nrc_helpers.cu:77-129 (USE_REFLECTANCE_FACTORING 0). */
void orc_accumulate(const float* radiance, const float* throughput, float* rgba, int64_t n, int mode,
                    uint32_t iteration_index) {
    const float w = 1.0f / (float)(iteration_index + 1); /* :98 */
    for (int64_t i = 0; i < n; i++) {
        const float* L = radiance + 3 * i;
        const float* T = throughput + 3 * i;
        float* o = rgba + 4 * i;
        switch (mode) {
        case 0: /* Full, :93-103 */
            for (int c = 0; c < 3; c++) {
                float r = T[c] * L[c];
                o[c] = fmaf(r, w, o[c]);
            }
            o[3] = 1.0f;
            break;
        case 2: /* CacheOnly, :108-115 */
            for (int c = 0; c < 3; c++) o[c] = L[c] * T[c];
            o[3] = 1.0f;
            break;
        case 4: /* DebugCacheNoThroughputModulation, :116-123 */
            for (int c = 0; c < 3; c++) o[c] = L[c];
            o[3] = 1.0f;
            break;
        case 5: /* DebugThroughputOnly, :124-127 */
            for (int c = 0; c < 3; c++) o[c] = T[c];
            o[3] = 1.0f;
            break;
        default: /* NoCache, CacheFirstVertex: return, :104-107 */
            break;
        }
    }
}

/* propagate_train_radiance, nrc_helpers.cu:131-224 (USE_REFLECTANCE_FACTORING 0), tile-serial.
 * Hardening matches the GPU build: index >= num_records ends a chain, at most num_records steps. */
void orc_propagate(const void* end_vertices, const float* end_radiance, int64_t num_tiles, const void* records,
                   float* targets, int64_t num_records) {
    const end_vertex* ev = (const end_vertex*)end_vertices;
    const train_record* rec = (const train_record*)records;
    for (int64_t t = 0; t < num_tiles; t++) {
        f3 last;
        last.x = end_radiance[3 * t + 0] * ev[t].mask; /* :154 */
        last.y = end_radiance[3 * t + 1] * ev[t].mask;
        last.z = end_radiance[3 * t + 2] * ev[t].mask;
        int32_t i = ev[t].start; /* :162 */
        for (int64_t steps = 0; i >= 0 && i < num_records && steps < num_records; steps++) { /* :179 */
            float* tg = targets + 3 * (int64_t)i;
            tg[0] = fmaf(rec[i].lt.x, last.x, tg[0]); /* :199, :205 */
            tg[1] = fmaf(rec[i].lt.y, last.y, tg[1]);
            tg[2] = fmaf(rec[i].lt.z, last.z, tg[2]);
            last.x = tg[0]; /* :213 */
            last.y = tg[1];
            last.z = tg[2];
            i = rec[i].prop_to; /* :214 */
        }
    }
}

/* ---- USE_REFLECTANCE_FACTORING 1 (config.h:118): reflectance() = diffuse + specular of a compact RadianceQuery
 * (neural_radiance_caching.h:118; floats 9..11 and 12..14). */
static f3 reflectance(const float* q) {
    f3 r;
    r.x = q[9] + q[12];
    r.y = q[10] + q[13];
    r.z = q[11] + q[14];
    return r;
}

/* accumulate_render_radiance with factoring: nrc_helpers.cu:93-97 (Full: radiance = T * L; radiance *= refl;
 * dst += radiance * w), :109-113 (CacheOnly: L * T, then * refl), :116-120 (Debug...NoThroughputModulation: L * refl,
 * also copy_radiance_to_output_buffer :65-68), :124-127 (DebugThroughputOnly: T). queries: the render queries. */
void orc_accumulate_factored(const float* radiance, const float* throughput, const float* queries, float* rgba,
                             int64_t n, int mode, uint32_t iteration_index) {
    const float w = 1.0f / (float)(iteration_index + 1);
    for (int64_t i = 0; i < n; i++) {
        const float* L = radiance + 3 * i;
        const float* T = throughput + 3 * i;
        float* o = rgba + 4 * i;
        float R[3] = {1.0f, 1.0f, 1.0f};
        if (mode == 0 || mode == 2 || mode == 4) {
            const f3 r = reflectance(queries + 15 * i);
            R[0] = r.x;
            R[1] = r.y;
            R[2] = r.z;
        }
        switch (mode) {
        case 0:
            for (int c = 0; c < 3; c++) {
                float r = T[c] * L[c];
                r = r * R[c];
                o[c] = fmaf(r, w, o[c]);
            }
            o[3] = 1.0f;
            break;
        case 2:
            for (int c = 0; c < 3; c++) {
                float r = L[c] * T[c];
                o[c] = r * R[c];
            }
            o[3] = 1.0f;
            break;
        case 4:
            for (int c = 0; c < 3; c++) o[c] = L[c] * R[c];
            o[3] = 1.0f;
            break;
        case 5:
            for (int c = 0; c < 3; c++) o[c] = T[c];
            o[3] = 1.0f;
            break;
        default:
            break;
        }
    }
}

/* propagate_train_radiance with factoring, nrc_helpers.cu:154-160 (lastRadiance = endRadiance * mask, then
 * *= endQuery.reflectance()), :189-214 (radianceTo = target * refl; radianceTo += lt * last; target = safeDiv(
 * radianceTo, refl) with safeDiv :28-35 = b != 0 ? a / b : 0 per component; last = radianceTo). */
void orc_propagate_factored(const void* end_vertices, const float* end_radiance, const float* end_queries,
                            int64_t num_tiles, const void* records, float* targets, const float* train_queries,
                            int64_t num_records) {
    const end_vertex* ev = (const end_vertex*)end_vertices;
    const train_record* rec = (const train_record*)records;
    for (int64_t t = 0; t < num_tiles; t++) {
        f3 last;
        last.x = end_radiance[3 * t + 0] * ev[t].mask;
        last.y = end_radiance[3 * t + 1] * ev[t].mask;
        last.z = end_radiance[3 * t + 2] * ev[t].mask;
        const f3 re = reflectance(end_queries + 15 * t);
        last.x *= re.x;
        last.y *= re.y;
        last.z *= re.z;
        int32_t i = ev[t].start;
        for (int64_t steps = 0; i >= 0 && i < num_records && steps < num_records; steps++) {
            float* tg = targets + 3 * (int64_t)i;
            const f3 R = reflectance(train_queries + 15 * (int64_t)i);
            f3 v;
            v.x = tg[0] * R.x;
            v.y = tg[1] * R.y;
            v.z = tg[2] * R.z;
            v.x = fmaf(rec[i].lt.x, last.x, v.x);
            v.y = fmaf(rec[i].lt.y, last.y, v.y);
            v.z = fmaf(rec[i].lt.z, last.z, v.z);
            tg[0] = R.x != 0.0f ? v.x / R.x : 0.0f;
            tg[1] = R.y != 0.0f ? v.y / R.y : 0.0f;
            tg[2] = R.z != 0.0f ? v.z / R.z : 0.0f;
            last = v;
            i = rec[i].prop_to;
        }
    }
}

/* ---- the shuffle permutation (keyed Feistel bijection, replaces curand keys + cub sort,
 * NRCUtil.cu:19-35). Stated independently of the HIP build from the written spec. */
static uint32_t mix32(uint32_t x) { /* "lowbias32" integer hash */
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

void orc_feistel_keys(uint64_t seed, uint32_t frame, uint32_t keys[4]) {
    for (uint32_t r = 0; r < 4; r++)
        keys[r] = mix32((uint32_t)seed ^ mix32((uint32_t)(seed >> 32) ^ mix32(frame + 0x9e3779b9U * (r + 1))));
}

static int half_bits(uint32_t n) {
    int b = 2;
    while (b < 32 && (1ULL << b) < (uint64_t)n) b++;
    if (b & 1) b++;
    return b / 2;
}

static uint32_t feistel(uint32_t x, int h, const uint32_t k[4]) {
    const uint32_t mask = (1U << h) - 1U;
    uint32_t L = x >> h, R = x & mask;
    for (int r = 0; r < 4; r++) {
        uint32_t nl = R;
        R = L ^ (mix32(R ^ k[r]) & mask);
        L = nl;
    }
    return (L << h) | R;
}

void orc_permutation(uint64_t seed, uint32_t frame, int32_t* perm, uint32_t n) {
    uint32_t k[4];
    orc_feistel_keys(seed, frame, k);
    const int h = half_bits(n);
    for (uint32_t d = 0; d < n; d++) {
        uint32_t x = feistel(d, h, k);
        while (x >= n) x = feistel(x, h, k);
        perm[d] = (int32_t)x;
    }
}

/* The reference's shuffle contract itself, NRCUtil.cu:19-35: cub::DeviceRadixSort::SortPairs(keys, values = the
 * indices 0..n-1 (Device.cpp:1187-1192), n, begin_bit 0, end_bit 32). cub (absent from the snapshot; CUDA toolkit
 * library) documents SortPairs as a stable least-significant-digit radix sort: ascending keys, pairs with equal keys in
 * their input order. Restated as cub's algorithm: LSD passes over 8-bit digits, each a stable counting sort.
 * sorted_keys may be NULL. */
void orc_sort_pairs(const uint32_t* keys, uint32_t* sorted_keys, int32_t* perm, uint32_t n) {
    if (n == 0) return;
    uint32_t* ka = (uint32_t*)malloc(sizeof(uint32_t) * n);
    uint32_t* kb = (uint32_t*)malloc(sizeof(uint32_t) * n);
    int32_t* va = (int32_t*)malloc(sizeof(int32_t) * n);
    int32_t* vb = (int32_t*)malloc(sizeof(int32_t) * n);
    for (uint32_t i = 0; i < n; i++) {
        ka[i] = keys[i];
        va[i] = (int32_t)i;
    }
    for (int shift = 0; shift < 32; shift += 8) {
        uint32_t count[257] = {0};
        for (uint32_t i = 0; i < n; i++) count[((ka[i] >> shift) & 255U) + 1]++;
        for (int d = 0; d < 256; d++) count[d + 1] += count[d];
        for (uint32_t i = 0; i < n; i++) { /* in input order: stable */
            const uint32_t pos = count[(ka[i] >> shift) & 255U]++;
            kb[pos] = ka[i];
            vb[pos] = va[i];
        }
        uint32_t* tk = ka; ka = kb; kb = tk;
        int32_t* tv = va; va = vb; vb = tv;
    }
    memcpy(perm, va, sizeof(int32_t) * n);
    if (sorted_keys) memcpy(sorted_keys, ka, sizeof(uint32_t) * n);
    free(ka); free(kb); free(va); free(vb);
}

/* permute_train_data, nrc_helpers.cu:226-249. perm == NULL: the Feistel permutation of (seed, frame)
 * over [0, n_out). */
void orc_permute(const float* q_src, const float* t_src, const int32_t* perm, uint64_t seed, uint32_t frame,
                 int32_t num_records, float* q_dst, float* t_dst, uint32_t n_out) {
    const int32_t nr = num_records < (int32_t)n_out ? num_records : (int32_t)n_out; /* :236 */
    if (nr <= 0) return;                                                        /* :237 */
    uint32_t k[4];
    orc_feistel_keys(seed, frame, k);
    const int h = half_bits(n_out);
    for (uint32_t d = 0; d < n_out; d++) {
        uint32_t p;
        if (perm) {
            p = (uint32_t)perm[d];
        } else {
            p = feistel(d, h, k);
            while (p >= n_out) p = feistel(p, h, k);
        }
        const uint32_t s = p % (uint32_t)nr; /* :245; a negative caller entry is read as unsigned (never OOB) */
        memcpy(q_dst + 15 * (int64_t)d, q_src + 15 * (int64_t)s, 60);
        memcpy(t_dst + 3 * (int64_t)d, t_src + 3 * (int64_t)s, 12);
    }
}
