/*
 * nrc/layout.h — per-sample buffer layouts and model constants of the NRC query/train path.
 *
 * Plain C (C99 / C++ / HIP). No GPU or torch types. Every constant cites the reference line it mirrors.
 *
 *   RadianceQuery  <- /root/reference/nrc/shaders/neural_radiance_caching.h:100-118 with
 *                     USE_COMPACT_RADIANCE_QUERY = 1 (/root/reference/nrc/shaders/config.h:113)
 *   constants      <- neural_radiance_caching.h:29-54
 *   model config   <- /root/reference/nrc/inc/NRCNetworkConfigs.h:11-83 (Frequency encoding)
 */
#ifndef NRC_LAYOUT_H
#define NRC_LAYOUT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- batch constants: neural_radiance_caching.h:29-31 ---- */
#define NRC_NUM_BATCHES                    4
#define NRC_NUM_TRAINING_RECORDS_PER_FRAME 65536
#define NRC_BATCH_SIZE                     (NRC_NUM_TRAINING_RECORDS_PER_FRAME / NRC_NUM_BATCHES) /* 16384 */
/* tcnn::BATCH_SIZE_GRANULARITY, used by NRCNetwork.cu:48-49, :72 */
#define NRC_BATCH_SIZE_GRANULARITY         256

/* ---- network I/O dims: neural_radiance_caching.h:33-41 (compact query) ---- */
#define NRC_INPUT_DIMS  15 /* pos(3) dir(2) normal(2) roughness(2) diffuse(3) specular(3) */
#define NRC_OUTPUT_DIMS 3  /* RGB radiance */

/* ---- InputEncoding: neural_radiance_caching.h:24-27 ---- */
#define NRC_ENCODING_FREQUENCY 0
#define NRC_ENCODING_HASH      1
/* extension (not in the reference): Frequency with the direction encoded by degree-4 spherical harmonics
 * (BASELINE.json north_star "frequency + one-blob + spherical-harmonics"); same 80-wide MLP shape */
#define NRC_ENCODING_FREQUENCY_SH 2

/* ---- default learning rates TRAIN_LR(): neural_radiance_caching.h:47-54 ---- */
#define NRC_TRAIN_LR_FREQUENCY 1e-3f
#define NRC_TRAIN_LR_HASH      1e-2f

/* RadianceQuery, compact layout: 15 packed f32 = 60 bytes, 4-byte aligned, array-of-structs.
 * Value semantics (hit.cu:589-617): position = world position * 0.005 (Cornell);
 * direction/normal = (theta, phi) from cartesianToSphericalUnitVector (shader_common.h:320-333);
 * roughness = (1,1) for diffuse events (hit.cu:481-483); diffuse/specular albedo. */
typedef struct nrc_radiance_query {
    float position[3];
    float direction1, direction2;
    float normal1, normal2;
    float roughness1, roughness2;
    float diffuse[3];
    float specular[3];
} nrc_radiance_query;

/* RadianceQuery, non-compact layout (USE_COMPACT_RADIANCE_QUERY 0: neural_radiance_caching.h:38-40, :107-111):
 * 16 f32 = 64 bytes, a pad_ float after the position (hit.cu:608 writes 0.0f), float2 direction / normal /
 * roughness. Selected per handle by nrc_config.query_layout = NRC_QUERY_PADDED; the encodings then carry the
 * reference's extra Identity(1) of pad_ right after the position encoding (NRCNetworkConfigs.h:61-67, :106-111):
 *   Frequency: TriangleWave 0..35 | pad_ 36 | OneBlob 37..60 | Identity 61..66 | 1.0 x 13 (67..79)
 *   Hash:      HashGrid 0..31     | pad_ 32 | OneBlob 33..56 | Identity 57..62 | 1.0 (63)
 * i.e. the same widths (80 / 64) with one constant-one column fewer; W0's columns follow that order. */
#define NRC_INPUT_DIMS_PADDED 16
#define NRC_QUERY_COMPACT 0 /* USE_COMPACT_RADIANCE_QUERY 1 (config.h:113): 15 floats */
#define NRC_QUERY_PADDED  1 /* USE_COMPACT_RADIANCE_QUERY 0: 16 floats */
typedef struct nrc_radiance_query_padded {
    float position[3];
    float pad_;
    float direction[2];
    float normal[2];
    float roughness[2];
    float diffuse[3];
    float specular[3];
} nrc_radiance_query_padded;

/* Radiance outputs and training targets: packed float3, 12 bytes (neural_radiance_caching.h:144, :175). */
typedef struct nrc_float3 { float x, y, z; } nrc_float3;

/* ---- Frequency-config model shape (NRCNetworkConfigs.h:26-33, :51-81) ----
 * Composite encoding: TriangleWave(dims 0-2, 12 freqs) -> 36, OneBlob(dims 3-8, 4 bins) -> 24,
 * Identity(dims 9-14) -> 6; 66 features, padded with constant 1.0 to 80 (FullyFusedMLP input
 * granularity 16). FullyFusedMLP: 64 neurons, 5 hidden layers, ReLU hidden + ReLU output, no bias,
 * output padded to 16 rows (only 3 used). */
#define NRC_TRI_DIMS       3
#define NRC_TRI_FREQS      12
#define NRC_BLOB_DIMS      6
#define NRC_BLOB_BINS      4
#define NRC_IDENT_DIMS     6
#define NRC_ENC_REAL       (NRC_TRI_DIMS * NRC_TRI_FREQS + NRC_BLOB_DIMS * NRC_BLOB_BINS + NRC_IDENT_DIMS) /* 66 */
#define NRC_ENC_WIDTH      80  /* padded encoding width = FullyFusedMLP input width */
#define NRC_WIDTH          64
#define NRC_HIDDEN_LAYERS  5   /* => 1 input matmul + 4 hidden matmuls + 1 output matmul */
#define NRC_NUM_LAYERS     6
#define NRC_OUT_PADDED     16

/* Canonical parameter blob (f32): W0[64][80], W1..W4[64][64], W5[16][64], each row-major [out][in].
 * This is the order of nrc_get_params/nrc_set_params and of the golden fixtures. */
#define NRC_W0_OFFSET   0
#define NRC_W1_OFFSET   (NRC_W0_OFFSET + NRC_WIDTH * NRC_ENC_WIDTH)   /* 5120  */
#define NRC_W2_OFFSET   (NRC_W1_OFFSET + NRC_WIDTH * NRC_WIDTH)       /* 9216  */
#define NRC_W3_OFFSET   (NRC_W2_OFFSET + NRC_WIDTH * NRC_WIDTH)       /* 13312 */
#define NRC_W4_OFFSET   (NRC_W3_OFFSET + NRC_WIDTH * NRC_WIDTH)       /* 17408 */
#define NRC_W5_OFFSET   (NRC_W4_OFFSET + NRC_WIDTH * NRC_WIDTH)       /* 21504 */
#define NRC_NUM_PARAMS  (NRC_W5_OFFSET + NRC_OUT_PADDED * NRC_WIDTH)  /* 22528 */

/* ---- Hash-config model shape (NRCNetworkConfigs.h:84-128) ----
 * Composite encoding: HashGrid(dims 0-2: 16 levels x 2 features, log2 hashmap 15, base resolution 16,
 * per-level scale 2) -> 32, OneBlob(dims 3-8, 4 bins) -> 24, Identity(dims 9-14) -> 6; 62 features padded
 * with 1.0 to 64. Level l: scale = 16 * 2^l - 1, resolution = 16 * 2^l; entries = min(resolution^3, 2^15)
 * (levels 0, 1 dense: 4096 and 32768 entries; levels 2..15 hashed: 32768 each). */
#define NRC_HASH_LEVELS        16
#define NRC_HASH_FEATURES      2
#define NRC_HASH_LOG2_T        15
#define NRC_HASH_T             (1 << NRC_HASH_LOG2_T)
#define NRC_HASH_BASE_RES      16
#define NRC_HASH_ENC_REAL      (NRC_HASH_LEVELS * NRC_HASH_FEATURES + NRC_BLOB_DIMS * NRC_BLOB_BINS + NRC_IDENT_DIMS) /* 62 */
#define NRC_HASH_ENC_WIDTH     64
#define NRC_HASH_ENTRIES       (4096 + (NRC_HASH_LEVELS - 1) * NRC_HASH_T)          /* 495616 */
#define NRC_HASH_GRID_PARAMS   (NRC_HASH_ENTRIES * NRC_HASH_FEATURES)               /* 991232 */
/* parameter blob of the Hash config: MLP W0[64][64], W1..W4[64][64], W5[16][64] (matrix params, Adam with
 * l2), then the grid table [entry][feature] (non-matrix params: sparse Adam, no l2) */
#define NRC_HASH_W0_OFFSET     0
#define NRC_HASH_W1_OFFSET     (NRC_HASH_W0_OFFSET + NRC_WIDTH * NRC_HASH_ENC_WIDTH)  /* 4096  */
#define NRC_HASH_W5_OFFSET     (NRC_HASH_W1_OFFSET + 4 * NRC_WIDTH * NRC_WIDTH)       /* 20480 */
#define NRC_HASH_MLP_PARAMS    (NRC_HASH_W5_OFFSET + NRC_OUT_PADDED * NRC_WIDTH)      /* 21504 */
#define NRC_HASH_GRID_OFFSET   NRC_HASH_MLP_PARAMS
#define NRC_HASH_NUM_PARAMS    (NRC_HASH_MLP_PARAMS + NRC_HASH_GRID_PARAMS)           /* 1012736 */
/* first table entry of level l */
#define NRC_HASH_LEVEL_ENTRY_OFFSET(l) ((l) == 0 ? 0 : 4096 + ((l) - 1) * NRC_HASH_T)
#define NRC_HASH_PRIME1 2654435761u /* tcnn coherent prime hash: x * 1 ^ y * 2654435761 ^ z * 805459861 */
#define NRC_HASH_PRIME2 805459861u

/* ---- width-128 network (BASELINE.json configs[4]; beyond the reference's n_neurons = 64) ----
 * The same FullyFusedMLP with 128 neurons: W0[128][80], W1..W4[128][128], W5[16][128], canonical blob order as
 * above. Frequency and FrequencySH encodings (80-wide input). Inference in f16 or FP8 (nrc_config.infer_precision). */
#define NRC_WIDE_WIDTH         128
#define NRC_WIDE_W0_OFFSET     0
#define NRC_WIDE_W1_OFFSET     (NRC_WIDE_W0_OFFSET + NRC_WIDE_WIDTH * NRC_ENC_WIDTH)       /* 10240 */
#define NRC_WIDE_W5_OFFSET     (NRC_WIDE_W1_OFFSET + 4 * NRC_WIDE_WIDTH * NRC_WIDE_WIDTH)  /* 75776 */
#define NRC_WIDE_NUM_PARAMS    (NRC_WIDE_W5_OFFSET + NRC_OUT_PADDED * NRC_WIDE_WIDTH)      /* 77824 */

/* tcnn defaults used by the Frequency config (survey Appendix A.7-A.8). */
#define NRC_LOSS_SCALE     128.0f
#define NRC_ADAM_BETA1     0.9f
#define NRC_ADAM_BETA2     0.999f
#define NRC_ADAM_EPS_FREQ  1e-8f
#define NRC_ADAM_EPS_HASH  1e-15f
#define NRC_ADAM_L2_REG    1e-6f
#define NRC_EMA_DECAY      0.99f
#define NRC_LUM_EPS        0.01f

#ifdef __cplusplus
}
#endif

#endif /* NRC_LAYOUT_H */
