/*
 * nrc/frame.h — C-ABI of the per-frame GPU steps either side of the NRC module (SURVEY.md §8(f) rows 2
 * and 4): the renderer-side kernels the reference launches around nrc::Network::infer/train after the
 * OptiX trace (Device::render, /root/reference/nrc/src/Device.cpp:2493-2515), and one call that runs
 * that whole post-trace sequence for a frame.
 *
 *   infer (render + train-suffix-end queries)      Device.cpp:1272-1301  -> nrc_infer
 *   accumulate_render_radiance                     nrc_helpers.cu:77-129 -> nrc_accumulate_render_radiance
 *   (CacheFirstVertex: infer + copy_radiance_to_output_buffer, nrc_helpers.cu:54-73, Device.cpp:1339-1370)
 *   propagate_train_radiance                       nrc_helpers.cu:131-224 -> nrc_propagate_train_radiance
 *   generateRandomPermutationForTrain              NRCUtil.cu:19-35       -> nrc_generate_train_permutation
 *   permute_train_data                             nrc_helpers.cu:226-249 -> nrc_permute_train_data
 *   NUM_BATCHES x train                            Device.cpp:1473-1512   -> nrc_train
 *
 * Same conventions as nrc_c.h: plain device pointers, int status, stream-ordered, never throws.
 * Records are the reference's structs byte for byte (neural_radiance_caching.h:56-99); the reference
 * is built with USE_REFLECTANCE_FACTORING 0 (config.h:118), the only variant restated here.
 */
#ifndef NRC_FRAME_H
#define NRC_FRAME_H

#include "nrc_c.h"

#ifdef __cplusplus
extern "C" {
#endif

#define NRC_TRAIN_RECORD_INDEX_NONE        (-1) /* neural_radiance_caching.h:43 */
#define NRC_TRAIN_RECORD_INDEX_BUFFER_FULL (-2) /* neural_radiance_caching.h:44 */

/* TrainingRecord (neural_radiance_caching.h:57-75): one non-Dirac vertex of a training path. 28 B. */
typedef struct nrc_training_record {
    int32_t prop_to;             /* next record towards the camera, or TRAIN_RECORD_INDEX_NONE */
    nrc_float3 local_throughput; /* modulates the radiance propagated from the previous record */
    int32_t pixel_index, tile_index, prop_length; /* debug fields, carried but unused */
} nrc_training_record;

/* TrainingSuffixEndVertex (neural_radiance_caching.h:78-94): terminal vertex of a tile's train suffix. 16 B. */
typedef struct nrc_train_suffix_end_vertex {
    int32_t start_train_record; /* first record of the propagation chain (< 0: none) */
    float radiance_mask;        /* 1: self-training (use the inferred radiance), 0: unbiased */
    int32_t pixel_index, tile_index;
} nrc_train_suffix_end_vertex;

/* nrc::RenderMode (neural_radiance_caching.h:14-22) */
typedef enum nrc_render_mode {
    NRC_RENDER_FULL = 0,
    NRC_RENDER_NO_CACHE = 1,
    NRC_RENDER_CACHE_ONLY = 2,
    NRC_RENDER_CACHE_FIRST_VERTEX = 3,
    NRC_RENDER_DEBUG_CACHE_NO_THROUGHPUT_MODULATION = 4,
    NRC_RENDER_DEBUG_THROUGHPUT_ONLY = 5
} nrc_render_mode;

/* accumulate_render_radiance (nrc_helpers.cu:77-129) over n pixels (the reference's 2-D launch over the
 * resolution visits pixel y*W+x, i.e. exactly [0, n)). output_rgba is the float4 frame buffer
 * (USE_FP32_OUTPUT, config.h:77). Full: out.rgb += (throughput*radiance) * 1/(iteration_index+1);
 * CacheOnly: out = throughput*radiance; DebugCacheNoThroughputModulation: out = radiance;
 * DebugThroughputOnly: out = throughput; NoCache / CacheFirstVertex: no-op. w = 1 wherever written. */
nrc_status nrc_accumulate_render_radiance(const nrc_float3* end_render_radiance_d,
                                          const nrc_float3* end_render_throughput_d, float* output_rgba_d,
                                          uint32_t num_pixels, int mode, uint32_t iteration_index,
                                          hipStream_t stream);

/* infer() with accumulate_render_radiance fused into the inference epilogue:
 * queries [0, num_pixels) are the render queries — their radiance goes straight into output_rgba exactly as
 * nrc_accumulate_render_radiance would put it (bit-identical) and is NOT written to results_d; queries
 * [num_pixels, n) (the train-suffix ends) are written to results_d as infer() does. mode: Full or CacheOnly
 * (other modes: NRC_ERR_INVALID_ARGUMENT — use nrc_infer + nrc_accumulate_render_radiance). Saves the 24 B/pixel
 * radiance round trip through HBM and one launch. Uses the inference (EMA) weights, the handle's stream. */
nrc_status nrc_infer_accumulate(nrc_net* net, const float* queries_d, float* results_d, uint32_t n,
                                const nrc_float3* end_render_throughput_d, float* output_rgba_d, uint32_t num_pixels,
                                int mode, uint32_t iteration_index);

/* copy_radiance_to_output_buffer (nrc_helpers.cu:54-73): out = (radiance, 1) for n pixels. */
nrc_status nrc_copy_radiance_to_output(const nrc_float3* radiance_d, float* output_rgba_d, uint32_t num_pixels,
                                       hipStream_t stream);

/* propagate_train_radiance (nrc_helpers.cu:131-224): for every tile t, walk the record chain from
 * end_vertices[t].start_train_record along prop_to, doing
 *     last = end_train_radiance[t] * radiance_mask;  target[i] += local_throughput[i] * last;  last = target[i]
 * Chains of different tiles are disjoint (each train path owns its records), as in the reference.
 * Hardening (documented deviation): an index >= num_records ends the chain and a chain is cut after
 * num_records steps, so corrupt links can neither fault nor hang the GPU. */
nrc_status nrc_propagate_train_radiance(const nrc_train_suffix_end_vertex* end_vertices_d,
                                        const nrc_float3* end_train_radiance_d, uint32_t num_tiles,
                                        const nrc_training_record* records_d, nrc_float3* train_targets_d,
                                        uint32_t num_records, hipStream_t stream);

/* USE_REFLECTANCE_FACTORING 1 (config.h:118; the reference's compile-time variant, off in its shipped build): the
 * cache then learns radiance / reflectance, reflectance() = diffuse + specular of the RadianceQuery
 * (neural_radiance_caching.h:118). Accumulation multiplies by the render query's reflectance after the throughput
 * product (nrc_helpers.cu:95-97, 111-113, 118-120; copy_radiance_to_output_buffer :66-68); propagation multiplies the
 * end radiance by the end query's reflectance and each record's target by its own before the update, stores
 * safeDiv(radiance, reflectance) (a zero component gives 0, :28-35, :191-204) and carries the radiance itself.
 * end_render_queries / end_train_queries are the inference queries of those pixels / tiles; train_queries the records'
 * queries as traced (train_queries_d[0]). Divisions are IEEE (the reference's fast-math build divides approximately). */
nrc_status nrc_accumulate_render_radiance_factored(const nrc_float3* end_render_radiance_d,
                                                   const float* end_render_queries_d,
                                                   const nrc_float3* end_render_throughput_d, float* output_rgba_d,
                                                   uint32_t num_pixels, int mode, uint32_t iteration_index,
                                                   hipStream_t stream);
nrc_status nrc_copy_radiance_to_output_factored(const nrc_float3* radiance_d, const float* queries_d,
                                                float* output_rgba_d, uint32_t num_pixels, hipStream_t stream);
nrc_status nrc_propagate_train_radiance_factored(const nrc_train_suffix_end_vertex* end_vertices_d,
                                                 const nrc_float3* end_train_radiance_d,
                                                 const float* end_train_queries_d, uint32_t num_tiles,
                                                 const nrc_training_record* records_d, nrc_float3* train_targets_d,
                                                 const float* train_queries_d, uint32_t num_records,
                                                 hipStream_t stream);

/* The training shuffle's permutation (NRCUtil.cu:19-35 contract: a fresh pseudo-random permutation of
 * [0, n) per frame). The reference sorts curand keys with cub radix sort; here the permutation is a keyed
 * 4-round Feistel bijection with cycle walking, a pure function of (seed, frame_index, d) — no sort, no
 * temp storage, reproducible. 1 <= n <= 2^30. */
nrc_status nrc_generate_train_permutation(uint64_t seed, uint32_t frame_index, int32_t* permutation_d, uint32_t n,
                                          hipStream_t stream);

/* The reference's shuffle itself (NRCUtil.cu:19-35): cub::DeviceRadixSort::SortPairs(keys, [0, n)) over key bits
 * [0, 32) -- the permutation a STABLE sort of the caller's 32-bit keys makes of the indices (ascending keys, equal keys in
 * index order), e.g. of the renderer's 65,536 curand keys or a recorded key section (nrc/stream.h). permutation_d[n]
 * receives the sorted indices, sorted_keys_d (may be NULL) the sorted keys; no buffer may overlap another. temp_d: device
 * memory of at least nrc_sort_train_permutation_temp_bytes(n) bytes (4-byte aligned). 1 <= n <= 2^24; n = 0 is a
 * no-op. An LSD radix sort of 8-bit digits, two launches per digit. */
size_t nrc_sort_train_permutation_temp_bytes(uint32_t n);
nrc_status nrc_sort_train_permutation(const uint32_t* keys_d, uint32_t* sorted_keys_d, int32_t* permutation_d,
                                      uint32_t n, void* temp_d, size_t temp_bytes, hipStream_t stream);

/* permute_train_data (nrc_helpers.cu:226-249): for d in [0, n_out):
 *     s = perm(d) % min(num_records, n_out);  queries_dst[d] = queries_src[s];  targets_dst[d] = targets_src[s]
 * perm(d) = permutation_d[d] if permutation_d != NULL (any caller-made permutation, e.g. the reference's
 * curand+cub one: results are then byte-identical), else the Feistel permutation of (seed, frame_index)
 * computed in-kernel. num_records <= 0: no-op (nrc_helpers.cu:237). Records are copied as raw bytes. */
nrc_status nrc_permute_train_data(const float* queries_src_d, const nrc_float3* targets_src_d,
                                  const int32_t* permutation_d, uint64_t seed, uint32_t frame_index,
                                  int32_t num_records, float* queries_dst_d, nrc_float3* targets_dst_d,
                                  uint32_t n_out, hipStream_t stream);

/* The entry points above that read RadianceQuery records, for padded 16-float records (USE_COMPACT_RADIANCE_QUERY 0,
 * layout.h; the reference's same kernels compiled with the other struct). nrc_process_frame follows the handle's
 * nrc_config.query_layout by itself. */
nrc_status nrc_accumulate_render_radiance_factored_padded(const nrc_float3* end_render_radiance_d,
                                                          const float* end_render_queries_d,
                                                          const nrc_float3* end_render_throughput_d,
                                                          float* output_rgba_d, uint32_t num_pixels, int mode,
                                                          uint32_t iteration_index, hipStream_t stream);
nrc_status nrc_copy_radiance_to_output_factored_padded(const nrc_float3* radiance_d, const float* queries_d,
                                                       float* output_rgba_d, uint32_t num_pixels, hipStream_t stream);
nrc_status nrc_propagate_train_radiance_factored_padded(const nrc_train_suffix_end_vertex* end_vertices_d,
                                                        const nrc_float3* end_train_radiance_d,
                                                        const float* end_train_queries_d, uint32_t num_tiles,
                                                        const nrc_training_record* records_d,
                                                        nrc_float3* train_targets_d, const float* train_queries_d,
                                                        uint32_t num_records, hipStream_t stream);
nrc_status nrc_permute_train_data_padded(const float* queries_src_d, const nrc_float3* targets_src_d,
                                         const int32_t* permutation_d, uint64_t seed, uint32_t frame_index,
                                         int32_t num_records, float* queries_dst_d, nrc_float3* targets_dst_d,
                                         uint32_t n_out, hipStream_t stream);

/* ---- one frame of Device::render's post-trace NRC sequence (Device.cpp:2493-2515) ---- */
typedef struct nrc_frame_buffers {
    /* [screen + tiles] queries / results: render queries first, then one per train-suffix end (tile) */
    const float* queries_inference_d;
    nrc_float3* results_inference_d;
    const nrc_float3* last_render_throughput_d;  /* [screen] */
    float* output_rgba_d;                         /* [screen] float4 */
    const float* queries_cache_vis_d;             /* [screen], CacheFirstVertex only (may be NULL otherwise) */
    nrc_float3* results_cache_vis_d;              /* [screen], CacheFirstVertex only */
    const nrc_train_suffix_end_vertex* end_vertices_d; /* [tiles] */
    const nrc_training_record* train_records_d;   /* [65536] */
    float* train_queries_d[2];                    /* DoubleBuffer<RadianceQuery>: [0] as traced, [1] shuffled */
    nrc_float3* train_targets_d[2];               /* DoubleBuffer<float3>: [0] emission so far (+= propagation) */
    const int32_t* permutation_d;                 /* NULL: the key sort below, or the Feistel permutation of
                                                     (shuffle_seed, frame_index) */
    const uint32_t* shuffle_keys_d;               /* [65536] keys whose stable sort gives the permutation
                                                     (nrc_sort_train_permutation; the reference's curand keys); used
                                                     when permutation_d is NULL; NULL: Feistel */
} nrc_frame_buffers;

typedef struct nrc_frame_params {
    uint32_t screen_size;         /* #pixels */
    uint32_t num_tiles;
    int32_t num_training_records; /* the trace's atomic counter (may exceed 65536; clamped as Device.cpp:2493) */
    int32_t render_mode;          /* nrc_render_mode */
    uint32_t iteration_index;     /* sysData.pf.iterationIndex (accumulation weight) */
    uint32_t frame_index;         /* shuffle key */
    uint64_t shuffle_seed;
    int32_t train;                /* 0: inference/accumulation only */
    int32_t keep_render_results;  /* 1: also write the render queries' radiance to results_inference (unfused
                                     infer + accumulate, e.g. for the reference's debug dump); 0: fused */
    int32_t reflectance_factoring; /* 1: USE_REFLECTANCE_FACTORING 1 (the *_factored kernels above; unfused) */
} nrc_frame_params;

/* Runs, on the handle's stream: infer -> accumulate (fused into infer for Full / CacheOnly unless
 * keep_render_results; cache-vis for CacheFirstVertex) -> [if records] propagate -> shuffle -> NUM_BATCHES x train.
 * loss_h (optional) receives the mean of the NUM_BATCHES minibatch losses (Device.cpp:1503-1511) and makes the call
 * block once at the end (the reference blocks after every minibatch); 0 if the frame did not train. */
nrc_status nrc_process_frame(nrc_net* net, const nrc_frame_buffers* buffers, const nrc_frame_params* params,
                             float* loss_h);
/* Data-parallel form: this replica renders the pixels [pixel_begin, pixel_end) — it infers and
 * accumulates only those render queries, writing only that range of results / output_rgba — and infers ALL the
 * train-suffix ends, so propagation and the shuffle are identical on every replica. With a communicator attached
 * (nrc_set_comm) each of the NUM_BATCHES minibatches is trained as nrc_train_dp over the global 16,384 samples, this
 * rank taking its contiguous 1/world slice (BASELINE configs[3]: 2,048 per rank at 8 GPUs). Without one it equals
 * nrc_process_frame restricted to the pixel range. */
nrc_status nrc_process_frame_shard(nrc_net* net, const nrc_frame_buffers* buffers, const nrc_frame_params* params,
                                   uint32_t pixel_begin, uint32_t pixel_end, float* loss_h);

#ifdef __cplusplus
}
#endif

#endif /* NRC_FRAME_H */
