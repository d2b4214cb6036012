// nrc_frame_capi.cpp — C-ABI of the per-frame steps around the network (include/nrc/frame.h) and the
// frame driver nrc_process_frame, which replays Device::render's post-trace NRC sequence
// (/root/reference/nrc/src/Device.cpp:2493-2515) on the handle's stream.
#include <algorithm>
#include <cstdint>

#include "nrc/frame.h"
#include "nrc_guard.h"
#include "nrc_internal.h"

using namespace nrc_amd;

namespace {

void require(bool ok, const char* msg) {
    if (!ok) throw ApiError(NRC_ERR_INVALID_ARGUMENT, msg);
}

void check(nrc_status st) {
    if (st != NRC_OK) throw ApiError(st, nrc_last_error());
}

bool aligned(const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; }

float accumulation_weight(uint32_t iteration_index) {
    return 1.0f / (float)(iteration_index + 1u);  // nrc_helpers.cu:98
}

bool valid_mode(int mode) { return mode >= NRC_RENDER_FULL && mode <= NRC_RENDER_DEBUG_THROUGHPUT_ONLY; }

constexpr uint32_t kMaxPermute = 1u << 26;  // 18 dwords per record stay inside a 32-bit grid index

}  // namespace

extern "C" {

nrc_status nrc_accumulate_render_radiance(const nrc_float3* rad, const nrc_float3* thr, float* rgba, uint32_t n,
                                          int mode, uint32_t iteration_index, hipStream_t stream) {
    return guarded([&] {
        require(valid_mode(mode), "unknown render mode");
        if (n == 0 || mode == NRC_RENDER_NO_CACHE || mode == NRC_RENDER_CACHE_FIRST_VERTEX) return;
        require(rgba && aligned(rgba, 16), "output_rgba must be a 16-byte aligned float4 buffer");
        require(mode == NRC_RENDER_DEBUG_THROUGHPUT_ONLY || rad, "radiance buffer is NULL");
        require(mode == NRC_RENDER_DEBUG_CACHE_NO_THROUGHPUT_MODULATION || thr, "throughput buffer is NULL");
        require(aligned(rad, 4) && aligned(thr, 4), "float3 buffers must be 4-byte aligned");
        HIP_CHECK(launch_accumulate(reinterpret_cast<const float*>(rad), reinterpret_cast<const float*>(thr), rgba, n,
                                    mode, accumulation_weight(iteration_index), stream));
    });
}

namespace {
nrc_status accumulate_factored(const nrc_float3* rad, const float* queries, const nrc_float3* thr, float* rgba,
                               uint32_t n, int mode, uint32_t iteration_index, hipStream_t stream, bool padq) {
    return guarded([&] {
        require(valid_mode(mode), "unknown render mode");
        if (n == 0 || mode == NRC_RENDER_NO_CACHE || mode == NRC_RENDER_CACHE_FIRST_VERTEX) return;
        require(rgba && aligned(rgba, 16), "output_rgba must be a 16-byte aligned float4 buffer");
        require(mode == NRC_RENDER_DEBUG_THROUGHPUT_ONLY || (rad && queries), "radiance / query buffer is NULL");
        require(mode == NRC_RENDER_DEBUG_CACHE_NO_THROUGHPUT_MODULATION || thr, "throughput buffer is NULL");
        require(aligned(rad, 4) && aligned(thr, 4) && aligned(queries, 4), "buffers must be 4-byte aligned");
        // DebugThroughputOnly does not read the queries (nrc_helpers.cu:124-127): any non-NULL pointer selects RF
        static const float kNoQueries = 0.0f;
        HIP_CHECK(launch_accumulate(reinterpret_cast<const float*>(rad), reinterpret_cast<const float*>(thr), rgba, n,
                                    mode, accumulation_weight(iteration_index), stream, queries ? queries : &kNoQueries,
                                    padq));
    });
}
}  // namespace

nrc_status nrc_accumulate_render_radiance_factored(const nrc_float3* rad, const float* queries, const nrc_float3* thr,
                                                   float* rgba, uint32_t n, int mode, uint32_t iteration_index,
                                                   hipStream_t stream) {
    return accumulate_factored(rad, queries, thr, rgba, n, mode, iteration_index, stream, false);
}

nrc_status nrc_accumulate_render_radiance_factored_padded(const nrc_float3* rad, const float* queries,
                                                          const nrc_float3* thr, float* rgba, uint32_t n, int mode,
                                                          uint32_t iteration_index, hipStream_t stream) {
    return accumulate_factored(rad, queries, thr, rgba, n, mode, iteration_index, stream, true);
}

nrc_status nrc_copy_radiance_to_output_factored(const nrc_float3* rad, const float* queries, float* rgba, uint32_t n,
                                                hipStream_t stream) {
    return accumulate_factored(rad, queries, nullptr, rgba, n, NRC_RENDER_DEBUG_CACHE_NO_THROUGHPUT_MODULATION, 0,
                               stream, false);
}

nrc_status nrc_copy_radiance_to_output_factored_padded(const nrc_float3* rad, const float* queries, float* rgba,
                                                       uint32_t n, hipStream_t stream) {
    return accumulate_factored(rad, queries, nullptr, rgba, n, NRC_RENDER_DEBUG_CACHE_NO_THROUGHPUT_MODULATION, 0,
                               stream, true);
}

nrc_status nrc_copy_radiance_to_output(const nrc_float3* rad, float* rgba, uint32_t n, hipStream_t stream) {
    return nrc_accumulate_render_radiance(rad, nullptr, rgba, n, NRC_RENDER_DEBUG_CACHE_NO_THROUGHPUT_MODULATION, 0,
                                          stream);
}

nrc_status nrc_propagate_train_radiance(const nrc_train_suffix_end_vertex* ends, const nrc_float3* end_rad,
                                        uint32_t tiles, const nrc_training_record* records, nrc_float3* targets,
                                        uint32_t nrec, hipStream_t stream) {
    return guarded([&] {
        if (tiles == 0 || nrec == 0) return;
        require(ends && end_rad && records && targets, "NULL buffer");
        require(aligned(ends, 4) && aligned(end_rad, 4) && aligned(records, 4) && aligned(targets, 4),
                "buffers must be 4-byte aligned");
        require(nrec <= (uint32_t)INT32_MAX, "num_records too large");
        HIP_CHECK(launch_propagate(ends, reinterpret_cast<const float*>(end_rad), tiles, records,
                                   reinterpret_cast<float*>(targets), nrec, stream));
    });
}

namespace {
nrc_status propagate_factored(const nrc_train_suffix_end_vertex* ends, const nrc_float3* end_rad,
                              const float* end_queries, uint32_t tiles, const nrc_training_record* records,
                              nrc_float3* targets, const float* train_queries, uint32_t nrec, hipStream_t stream,
                              bool padq) {
    return guarded([&] {
        if (tiles == 0 || nrec == 0) return;
        require(ends && end_rad && records && targets && end_queries && train_queries, "NULL buffer");
        require(aligned(ends, 4) && aligned(end_rad, 4) && aligned(records, 4) && aligned(targets, 4) &&
                    aligned(end_queries, 4) && aligned(train_queries, 4),
                "buffers must be 4-byte aligned");
        require(nrec <= (uint32_t)INT32_MAX, "num_records too large");
        HIP_CHECK(launch_propagate(ends, reinterpret_cast<const float*>(end_rad), tiles, records,
                                   reinterpret_cast<float*>(targets), nrec, stream, end_queries, train_queries, padq));
    });
}
}  // namespace

nrc_status nrc_propagate_train_radiance_factored(const nrc_train_suffix_end_vertex* ends, const nrc_float3* end_rad,
                                                 const float* end_queries, uint32_t tiles,
                                                 const nrc_training_record* records, nrc_float3* targets,
                                                 const float* train_queries, uint32_t nrec, hipStream_t stream) {
    return propagate_factored(ends, end_rad, end_queries, tiles, records, targets, train_queries, nrec, stream, false);
}

nrc_status nrc_propagate_train_radiance_factored_padded(const nrc_train_suffix_end_vertex* ends,
                                                        const nrc_float3* end_rad, const float* end_queries,
                                                        uint32_t tiles, const nrc_training_record* records,
                                                        nrc_float3* targets, const float* train_queries, uint32_t nrec,
                                                        hipStream_t stream) {
    return propagate_factored(ends, end_rad, end_queries, tiles, records, targets, train_queries, nrec, stream, true);
}

nrc_status nrc_generate_train_permutation(uint64_t seed, uint32_t frame, int32_t* perm, uint32_t n,
                                          hipStream_t stream) {
    return guarded([&] {
        if (n == 0) return;
        require(perm != nullptr && aligned(perm, 4), "permutation buffer must be non-NULL and 4-byte aligned");
        require(n <= (1u << 30), "n must be <= 2^30");
        HIP_CHECK(launch_permutation(seed, frame, perm, n, stream));
    });
}

size_t nrc_sort_train_permutation_temp_bytes(uint32_t n) { return sort_pairs_temp_bytes(n); }

nrc_status nrc_sort_train_permutation(const uint32_t* keys, uint32_t* sorted_keys, int32_t* perm, uint32_t n,
                                      void* temp, size_t temp_bytes, hipStream_t stream) {
    return guarded([&] {
        if (n == 0) return;
        require(n <= (1u << 24), "n must be <= 2^24");
        require(keys && aligned(keys, 4), "keys must be non-NULL and 4-byte aligned");
        require(perm && aligned(perm, 4), "permutation buffer must be non-NULL and 4-byte aligned");
        require(!sorted_keys || aligned(sorted_keys, 4), "sorted_keys must be 4-byte aligned");
        require(temp && aligned(temp, 4) && temp_bytes >= sort_pairs_temp_bytes(n),
                "temp must be 4-byte aligned and hold nrc_sort_train_permutation_temp_bytes(n) bytes");
        HIP_CHECK(launch_sort_pairs(keys, sorted_keys, perm, n, temp, stream));
    });
}

namespace {
nrc_status permute_train(const float* qs, const nrc_float3* ts, const int32_t* perm, uint64_t seed, uint32_t frame,
                         int32_t num_records, float* qd, nrc_float3* td, uint32_t n_out, hipStream_t stream, bool padq) {
    return guarded([&] {
        const uint32_t nrec = (uint32_t)std::min<int64_t>(num_records, (int64_t)n_out);  // nrc_helpers.cu:236
        if (num_records <= 0 || n_out == 0) return;                                      // :237
        require(n_out <= kMaxPermute, "n_out must be <= 2^26");
        require(qs && ts && qd && td, "NULL buffer");
        require(aligned(qs, 4) && aligned(ts, 4) && aligned(qd, 4) && aligned(td, 4) && aligned(perm, 4),
                "buffers must be 4-byte aligned");
        HIP_CHECK(launch_permute(qs, reinterpret_cast<const float*>(ts), perm, seed, frame, nrec, qd,
                                 reinterpret_cast<float*>(td), n_out, stream, padq));
    });
}
}  // namespace

nrc_status nrc_permute_train_data(const float* qs, const nrc_float3* ts, const int32_t* perm, uint64_t seed,
                                  uint32_t frame, int32_t num_records, float* qd, nrc_float3* td, uint32_t n_out,
                                  hipStream_t stream) {
    return permute_train(qs, ts, perm, seed, frame, num_records, qd, td, n_out, stream, false);
}

nrc_status nrc_permute_train_data_padded(const float* qs, const nrc_float3* ts, const int32_t* perm, uint64_t seed,
                                         uint32_t frame, int32_t num_records, float* qd, nrc_float3* td,
                                         uint32_t n_out, hipStream_t stream) {
    return permute_train(qs, ts, perm, seed, frame, num_records, qd, td, n_out, stream, true);
}

namespace {
// Device::render's post-trace sequence for the pixels [p0, p1) of the frame (all of it: [0, screen)). A data-parallel
// replica (communicator attached, nrc_set_comm) renders a pixel shard and trains on its 1/world slice of every
// minibatch; the train-suffix ends (tiles) are inferred in full on every rank, so propagation and the shuffle are
// identical everywhere and the sliced minibatches together are exactly the single-GPU minibatches.
void process_frame(nrc_net* net, const nrc_frame_buffers* fb, const nrc_frame_params* p, uint32_t p0, uint32_t p1,
                   float* loss_h) {
    require(net && fb && p, "NULL argument");
    require(valid_mode(p->render_mode), "unknown render mode");
    require(p0 <= p1 && p1 <= p->screen_size, "bad pixel range");
    hipStream_t s = nullptr;
    check(nrc_get_stream(net, &s));
    if (loss_h) *loss_h = 0.0f;
    const uint32_t screen = p->screen_size, tiles = p->num_tiles;
    const int mode = p->render_mode;
    const bool whole = p0 == 0 && p1 == screen;
    const uint32_t npix = p1 - p0;

    // Device::nrcInferRadiance (Device.cpp:1272-1301): render queries are skipped for NoCache / CacheFirstVertex
    const bool skip_render = mode == NRC_RENDER_NO_CACHE || mode == NRC_RENDER_CACHE_FIRST_VERTEX;
    require((uint64_t)screen + tiles <= UINT32_MAX, "screen_size + num_tiles overflows");
    const float* qi = fb->queries_inference_d;
    nrc_float3* ri = fb->results_inference_d;
    const bool padq = net_padq(net);  // RadianceQuery records of the handle's layout (nrc_config.query_layout)
    const size_t QD = padq ? NRC_INPUT_DIMS_PADDED : NRC_INPUT_DIMS;
    // Full / CacheOnly: accumulate_render_radiance runs in the inference epilogue (row 4 fusion); with reflectance
    // factoring the separate (factored) accumulation kernel runs instead
    const bool rf = p->reflectance_factoring != 0;
    // (a handle inferring with tcnn's f16 accumulation has no fused form: it takes infer + accumulate)
    const bool fuse = !skip_render && !p->keep_render_results && !rf && net_infer_fusable(net) &&
                      (mode == NRC_RENDER_FULL || mode == NRC_RENDER_CACHE_ONLY);
    if ((uint64_t)screen + tiles > 0) require(qi && ri, "inference buffers are NULL");
    auto infer_range = [&](uint32_t first, uint32_t count, uint32_t acc_pixels) {
        // queries [first, first + count); the first acc_pixels of them are render queries of pixels first..
        if (count == 0) return;
        const float* q = qi + (size_t)first * QD;
        float* r = reinterpret_cast<float*>(ri + first);
        if (fuse && acc_pixels > 0)
            check(nrc_infer_accumulate(net, q, r, count, fb->last_render_throughput_d + first,
                                       fb->output_rgba_d + (size_t)first * 4, acc_pixels, mode, p->iteration_index));
        else
            check(nrc_infer_stream(net, q, r, count, s));
    };
    if (whole && !skip_render) {
        infer_range(0, screen + tiles, screen);  // one launch over the contiguous render + tile queries
    } else {
        if (!skip_render) infer_range(p0, npix, npix);
        infer_range(screen, tiles, 0);
    }
    // Device::nrcAccumulateRadiance (Device.cpp:1310-1337)
    if (!skip_render && !fuse && npix > 0) {
        if (rf)
            check(accumulate_factored(fb->results_inference_d + p0, qi + (size_t)p0 * QD, fb->last_render_throughput_d + p0,
                                      fb->output_rgba_d + (size_t)p0 * 4, npix, mode, p->iteration_index, s, padq));
        else
            check(nrc_accumulate_render_radiance(fb->results_inference_d + p0, fb->last_render_throughput_d + p0,
                                                 fb->output_rgba_d + (size_t)p0 * 4, npix, mode, p->iteration_index, s));
    }
    // Device::nrcVisualizeFirstRadiance (Device.cpp:1339-1370)
    if (mode == NRC_RENDER_CACHE_FIRST_VERTEX && npix > 0) {
        require(fb->queries_cache_vis_d && fb->results_cache_vis_d, "cache-vis buffers are NULL");
        check(nrc_infer_stream(net, fb->queries_cache_vis_d + (size_t)p0 * QD,
                               reinterpret_cast<float*>(fb->results_cache_vis_d + p0), npix, s));
        if (rf)
            check(accumulate_factored(fb->results_cache_vis_d + p0, fb->queries_cache_vis_d + (size_t)p0 * QD, nullptr,
                                      fb->output_rgba_d + (size_t)p0 * 4, npix,
                                      NRC_RENDER_DEBUG_CACHE_NO_THROUGHPUT_MODULATION, 0, s, padq));
        else
            check(nrc_copy_radiance_to_output(fb->results_cache_vis_d + p0, fb->output_rgba_d + (size_t)p0 * 4, npix,
                                              s));
    }

    // Training (Device.cpp:2505-2512): only when the trace produced records
    const int32_t nrec = std::min(p->num_training_records, (int32_t)NRC_NUM_TRAINING_RECORDS_PER_FRAME);
    if (!p->train || nrec <= 0) return;
    require(fb->train_queries_d[0] && fb->train_queries_d[1] && fb->train_targets_d[0] && fb->train_targets_d[1],
            "training double buffers are NULL");
    // Device::nrcPropagateRadiance (Device.cpp:1382-1419): end radiance = results after the render part
    if (rf)  // the end queries are the inference queries after the render part; the records' are as traced
        check(propagate_factored(fb->end_vertices_d, fb->results_inference_d + screen, qi + (size_t)screen * QD, tiles,
                                 fb->train_records_d, fb->train_targets_d[0], fb->train_queries_d[0], (uint32_t)nrec, s,
                                 padq));
    else
        check(nrc_propagate_train_radiance(fb->end_vertices_d, fb->results_inference_d + screen, tiles,
                                           fb->train_records_d, fb->train_targets_d[0], (uint32_t)nrec, s));
    // Device::nrcShuffleTrainingData (Device.cpp:1427-1469). The permutation: the caller's, else the stable sort of the
    // caller's keys (the reference's curand keys + cub radix sort, NRCUtil.cu:19-35), else the Feistel permutation
    const int32_t* perm = fb->permutation_d;
    if (!perm && fb->shuffle_keys_d) {
        const uint32_t N = NRC_NUM_TRAINING_RECORDS_PER_FRAME;
        char* scratch = static_cast<char*>(net_frame_scratch(net, sizeof(int32_t) * N + sort_pairs_temp_bytes(N)));
        int32_t* sorted = reinterpret_cast<int32_t*>(scratch);
        HIP_CHECK(launch_sort_pairs(fb->shuffle_keys_d, nullptr, sorted, N, scratch + sizeof(int32_t) * N, s));
        perm = sorted;
    }
    check(permute_train(fb->train_queries_d[0], fb->train_targets_d[0], perm, p->shuffle_seed,
                        p->frame_index, nrec, fb->train_queries_d[1], fb->train_targets_d[1],
                        NRC_NUM_TRAINING_RECORDS_PER_FRAME, s, padq));
    // Device::nrcTrainRadiance (Device.cpp:1473-1512): NUM_BATCHES steps, mean loss. The minibatch losses
    // land in host-mapped slots and are read after one sync at the end (the reference syncs after
    // every minibatch, Device.cpp:1504); summed in the same order, so the mean is the same float.
    const nrc_loss_slots slots = net_loss_slots(net);
    int rank = 0, world = 1;
    const bool dp = net_comm(net, &rank, &world);
    // this rank's slice of every minibatch (dp::shard_range): sizes differ by at most one sample
    const uint32_t base = NRC_BATCH_SIZE / world, rem = NRC_BATCH_SIZE % world;
    const uint32_t s0 = rank * base + std::min<uint32_t>(rank, rem), sn = base + (rank < (int)rem ? 1 : 0);
    for (int b = 0; b < NRC_NUM_BATCHES; ++b) {
        const size_t first = (size_t)b * NRC_BATCH_SIZE + (dp ? s0 : 0);
        const float* bq = fb->train_queries_d[1] + first * QD;
        const float* bt = reinterpret_cast<const float*>(fb->train_targets_d[1] + first);
        if (dp)
            net_train_dp_async(net, bq, bt, sn, NRC_BATCH_SIZE, slots.dev + b);
        else
            check(nrc_train_async(net, bq, bt, NRC_BATCH_SIZE, slots.dev + b));
    }
    if (loss_h) {
        HIP_CHECK(hipStreamSynchronize(s));  // the slots are host-mapped: the kernels wrote them directly
        net_check_protocol(net);  // a timed-out exchange wait or LDS protocol wait invalidates the losses
        float total = 0.0f;
        for (int b = 0; b < NRC_NUM_BATCHES; ++b) total += slots.host[b];
        *loss_h = total * (1.0f / NRC_NUM_BATCHES);
    }
}
}  // namespace

nrc_status nrc_process_frame(nrc_net* net, const nrc_frame_buffers* fb, const nrc_frame_params* p, float* loss_h) {
    return guarded([&] { process_frame(net, fb, p, 0, p ? p->screen_size : 0, loss_h); });
}

nrc_status nrc_process_frame_shard(nrc_net* net, const nrc_frame_buffers* fb, const nrc_frame_params* p,
                                   uint32_t pixel_begin, uint32_t pixel_end, float* loss_h) {
    return guarded([&] { process_frame(net, fb, p, pixel_begin, pixel_end, loss_h); });
}

}  // extern "C"
