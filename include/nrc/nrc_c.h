/*
 * nrc/nrc_c.h — C-ABI of the MI355X-native neural radiance cache (drop-in for the reference's
 * nrc::Network query/train module, /root/reference/nrc/inc/NRCNetwork.h:20-75).
 *
 * Plain C: opaque handle, plain device pointers and sizes, int status codes; no C++ or torch types
 * cross this boundary. Exceptions never cross it: every entry point returns an nrc_status and the
 * message of the last failure on the calling thread is available from nrc_last_error().
 *
 * Buffers are the reference's, byte for byte (include/nrc/layout.h): queries are packed 60-byte
 * RadianceQuery records (15 f32, 4-byte aligned; 64-byte records of 16 f32 with nrc_config.query_layout =
 * NRC_QUERY_PADDED, the reference's USE_COMPACT_RADIANCE_QUERY 0), outputs and targets packed 12-byte float3.
 * All work is enqueued on a HIP stream and is asynchronous unless a host loss pointer is given
 * (that call blocks, as NRCNetwork.cu:54-55 does). A handle is not thread-safe.
 */
#ifndef NRC_C_H
#define NRC_C_H

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime_api.h>

#include "layout.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef enum nrc_status {
    NRC_OK = 0,
    NRC_ERR_INVALID_ARGUMENT = 1, /* std::invalid_argument in the reference (NRCNetworkConfigs.h:129-131) */
    NRC_ERR_DESTROYED = 2,        /* call after destroy(): a silent no-op in the reference (NRCNetwork.cu:43, :66) */
    NRC_ERR_NOT_INITIALIZED = 3,
    NRC_ERR_HIP = 4,              /* HIP runtime failure (CU_CHECK -> std::runtime_error in the reference) */
    NRC_ERR_UNSUPPORTED = 5,
    NRC_ERR_OUT_OF_MEMORY = 6,
    NRC_ERR_INTERNAL = 7          /* includes a training kernel's LDS-protocol timeout (sticky until nrc_init) */
} nrc_status;

typedef struct nrc_net nrc_net;

/* Optional hyper-parameter overrides; nrc_default_config() returns the reference's values for an
 * encoding (NRCNetworkConfigs.h:11-83, neural_radiance_caching.h:47-54). */
typedef struct nrc_config {
    float learning_rate; /* Adam learning rate, TRAIN_LR(encoding) */
    float beta1, beta2, epsilon, l2_reg;
    float ema_decay;     /* EMA optimizer wrapper decay (0.99) */
    float loss_scale;    /* f16 loss scale (128) */
    uint64_t seed;       /* weight initialisation seed */
    /* Extensions (BASELINE.json configs[4]; not in the reference, whose FullyFusedMLP has 64 neurons): */
    uint32_t width;           /* MLP neurons: 64 (reference) or 128 (NRC_WIDE_*; Frequency / FrequencySH only) */
    uint32_t infer_precision; /* nrc_precision of infer(): F16 (default), F16_ACC16 (tcnn's f16 accumulation, width 64
                               * Frequency or Hash) or FP8 (width 128 only) */
    /* RadianceQuery layout of every query buffer of the handle (the reference's compile-time
     * USE_COMPACT_RADIANCE_QUERY, config.h:113): NRC_QUERY_COMPACT (default, 15 f32) or NRC_QUERY_PADDED (16 f32 with
     * pad_ and its Identity(1) feature, layout.h). Padded: width 64, Frequency or Hash, infer_precision F16; the
     * parameter blob of nrc_get_state / nrc_set_state is in that encoding's column order (layout.h), while the
     * data-parallel gradient buffer (nrc_train_grad / nrc_train_apply) is in the handle's internal order. */
    uint32_t query_layout;
} nrc_config;

/* Arithmetic of infer() (nrc_config.infer_precision). F16: f16 operands, f32 accumulation per layer (the fast path).
 * F16_ACC16: tiny-cuda-nn's FullyFusedMLP numerics, an f16 accumulator rounded after every 16-wide K chunk in K order
 * (NRCNetworkConfigs.h:26-33; oracle mode ORC_TCNN), about 3-4x slower; infer / infer_stream only.
 * FP8: e4m3 weights (one power-of-two scale per output row) and e4m3 activations on the MX-scaled fp8 MFMA for layers
 * 1..5, layer 0 in f16. */
typedef enum nrc_precision {
    NRC_PRECISION_F16 = 0,
    NRC_PRECISION_FP8 = 1,
    NRC_PRECISION_F16_ACC16 = 2
} nrc_precision;

/* HyperParams (NRCNetwork.h:10-13) */
typedef struct nrc_hyper_params {
    float learning_rate;
} nrc_hyper_params;

/* Optimizer / model state slots for nrc_get_state / nrc_set_state (checkpoint, parity fixtures). */
typedef enum nrc_state_slot {
    NRC_STATE_PARAMS = 0, /* f32 master weights used by training (canonical blob, layout.h) */
    NRC_STATE_INFER = 1,  /* weights used by infer(): debiased EMA after the first step */
    NRC_STATE_EMA = 2,    /* raw (biased) EMA accumulator */
    NRC_STATE_ADAM_M = 3,
    NRC_STATE_ADAM_V = 4
} nrc_state_slot;

const char* nrc_version(void);
/* Message of the last failing call on this thread ("" if none). */
const char* nrc_last_error(void);
nrc_config nrc_default_config(int encoding);

/* Network() / ~Network() (NRCNetwork.h:22-24): allocate / free an empty handle. nrc_free on a handle
 * that was never destroyed prints the reference's warning (NRCNetwork.cu:29-33) and releases it. */
nrc_status nrc_create(nrc_net** out);
nrc_status nrc_free(nrc_net* net);

/* init<Verbose>(stream, encoding) (NRCNetwork.h:26-31, NRCNetwork.cu:106-112): set the stream,
 * select the encoding's config and (re)build the model with freshly initialised weights and
 * optimizer state. cfg may be NULL (reference defaults). verbose prints the config JSON
 * (printConfig_, NRCNetwork.cu:122-127). Re-init after destroy revives the handle. */
nrc_status nrc_init(nrc_net* net, hipStream_t stream, int encoding, const nrc_config* cfg, int verbose);

/* destroy() (NRCNetwork.h:41): release all device state; later calls return NRC_ERR_DESTROYED.
 * Idempotent. */
nrc_status nrc_destroy(nrc_net* net);

/* train(in, tgt, loss_h) / train(in, tgt, stream, loss_h) (NRCNetwork.h:44-46): one optimizer step on
 * exactly NRC_BATCH_SIZE (16384) samples. loss_h may be NULL; if not, the call blocks and writes the
 * minibatch loss (Trainer::loss()). */
nrc_status nrc_train(nrc_net* net, const float* inputs_d, const float* targets_d, float* loss_h);
nrc_status nrc_train_stream(nrc_net* net, const float* inputs_d, const float* targets_d, hipStream_t stream,
                            float* loss_h);
/* Extension: a step on any batch size b >= 1 (the reference fixes b = 16384). */
nrc_status nrc_train_batch(nrc_net* net, const float* inputs_d, const float* targets_d, uint32_t b, float* loss_h);
/* Extension (the asynchronous loss read-back SURVEY.md §8(b) allows): one step on b samples on the handle's
 * stream whose minibatch loss is written to device memory loss_d (may be NULL); never blocks. */
nrc_status nrc_train_async(nrc_net* net, const float* inputs_d, const float* targets_d, uint32_t b, float* loss_d);

/* infer(in, out, n) / infer(in, out, n, stream) (NRCNetwork.h:49-51). Processes exactly n queries
 * (the reference rounds n up to 256 and reads/writes past n, NRCNetwork.cu:72; this one never
 * touches the tail). n = 0 is a no-op. Uses the inference (EMA) weights. InputEncoding::Hash keeps one
 * level-feature workspace per handle: an inference on another stream than the previous one first waits for it (an
 * event), so calls on two streams serialise on the GPU rather than overlap. One handle is not for concurrent calls
 * from several host threads. */
nrc_status nrc_infer(nrc_net* net, const float* inputs_d, float* outputs_d, uint32_t n);
nrc_status nrc_infer_stream(nrc_net* net, const float* inputs_d, float* outputs_d, uint32_t n, hipStream_t stream);

nrc_status nrc_set_stream(nrc_net* net, hipStream_t stream);           /* setStream (NRCNetwork.h:53) */
nrc_status nrc_get_stream(const nrc_net* net, hipStream_t* stream);
nrc_status nrc_set_hyper_params(nrc_net* net, const nrc_hyper_params* hp); /* setHyperParams (:55) */
/* setConfig (:57, NRCNetwork.cu:96-99): like the reference it only replaces the config; on a live handle the
 * model (encoding, weights, optimizer state, learning rate) is untouched and nrc_get_config_json reports the new
 * encoding's default config. nrc_init always uses its own encoding argument. */
nrc_status nrc_set_config(nrc_net* net, int encoding);
nrc_status nrc_get_learning_rate(const nrc_net* net, float* lr);       /* getLearningRate (:61) */
/* printConfig_ equivalent: the model config as JSON (tcnn's schema). Writes at most cap bytes incl. NUL;
 * *needed (optional) receives the full length + 1. */
nrc_status nrc_get_config_json(const nrc_net* net, char* buf, size_t cap, size_t* needed);

/* ---- data-parallel split of train() (new capability: the reference has no collectives) ----
 * nrc_train_grad writes the loss-scaled gradient of this rank's b samples, normalised by the GLOBAL
 * batch (3 * global_b), into grad_d[nrc_get_grad_floats()] (f32, device): the gradient of every parameter
 * in nrc_get_state order (grad_d[0 .. num_params)), then the local loss at grad_d[num_params]. Sum grad_d
 * over ranks (e.g. an RCCL all-reduce), then nrc_train_apply performs the identical Adam + EMA step on every
 * rank. loss_h: as in nrc_train.
 * Frequency / FrequencySH: NRC_GRAD_FLOATS (88 KiB). Hash: NRC_HASH_GRAD_FLOATS (3.9 MiB: the MLP gradient,
 * then the grid-table gradient [entry][2]; the sparse grid Adam steps exactly the entries whose SUMMED gradient
 * is non-zero, as the single-GPU step over the global batch does). */
#define NRC_GRAD_FLOATS      (NRC_NUM_PARAMS + 4)
#define NRC_HASH_GRAD_FLOATS (NRC_HASH_NUM_PARAMS + 4)
nrc_status nrc_get_grad_floats(const nrc_net* net, uint64_t* n);
nrc_status nrc_train_grad(nrc_net* net, const float* inputs_d, const float* targets_d, uint32_t b,
                          uint32_t global_b, float* grad_d);
nrc_status nrc_train_apply(nrc_net* net, const float* grad_d, float* loss_h);
/* Hash only: the exact grid exchange (new capability). The grid-table gradient is an exact fixed-point sum per step
 * (value x 2^24 of tcnn's f16 contributions); nrc_train_grad rounds each rank's sum to f16 before the exchange, so a
 * world-N step differs from one GPU stepping the whole global minibatch. nrc_train_grad_fixed writes the MLP gradient
 * and the loss into grad_d as nrc_train_grad does (its grid part is not written) and this rank's exact grid sums into
 * grid_fixed_d[NRC_HASH_GRID_PARAMS] (int64, device) in an exchange encoding whose integer SUM over at most
 * NRC_FIXED_MAX_RANKS ranks is the global sum (non-finite contributions included: +inf, -inf, NaN as tcnn's f16 atomics
 * combine them). Sum grad_d (f32: [0, NRC_HASH_MLP_PARAMS) and the loss at [NRC_HASH_NUM_PARAMS]) and grid_fixed_d
 * (int64) over ranks, then nrc_train_apply_fixed rounds each global grid sum to f16 once: every rank applies bitwise the
 * grid gradient a single GPU forms over the global minibatch with the same weights. nrc_train_dp uses this exchange
 * for Hash networks. */
#define NRC_FIXED_MAX_RANKS 63
nrc_status nrc_train_grad_fixed(nrc_net* net, const float* inputs_d, const float* targets_d, uint32_t b,
                                uint32_t global_b, float* grad_d, int64_t* grid_fixed_d);
nrc_status nrc_train_apply_fixed(nrc_net* net, const float* grad_d, const int64_t* grid_fixed_d, float* loss_h);

/* ---- data parallelism inside the library: RCCL over xGMI (new capability) ----
 * The reference's callers are C++ (Device::nrcTrainRadiance, Device.cpp:1503-1509): one process (or thread) per GPU
 * creates an RCCL communicator, attaches it to its handle, and calls nrc_train_dp where it called train(); the
 * gradient exchange then happens inside the library on the handle's stream:
 *     local fwd/bwd of b_local samples, normalised by 3 * global_b (nrc_train_grad)
 *  -> ncclAllReduce(sum) of the NRC_GRAD_FLOATS buffer incl. the loss (Hash: the f32 MLP gradient and loss plus
 *     the int64 exact grid sums of nrc_train_grad_fixed, one RCCL group)
 *  -> the identical Adam + EMA step on every rank (nrc_train_apply), so the replicas stay bit-identical.
 * With world = 1 the step is bitwise the fused nrc_train step. C callers without rccl.h can create the
 * communicator through the nrc_comm_* helpers (one unique id made on rank 0 and shared by any means). */
#define NRC_COMM_UNIQUE_ID_BYTES 128 /* NCCL_UNIQUE_ID_BYTES */
nrc_status nrc_comm_get_unique_id(void* id_out /* NRC_COMM_UNIQUE_ID_BYTES */);
/* ncclCommInitRank on the calling thread's current HIP device; *comm_out receives the ncclComm_t. */
nrc_status nrc_comm_init_rank(void** comm_out, const void* unique_id, int world, int rank);
nrc_status nrc_comm_destroy(void* comm);
/* Attach an ncclComm_t (owned by the caller; NULL detaches). Rank and world size are read from it. */
nrc_status nrc_set_comm(nrc_net* net, void* nccl_comm);
nrc_status nrc_get_comm_rank(const nrc_net* net, int* rank, int* world);
/* One data-parallel optimizer step over a global minibatch of global_b samples of which this rank holds b_local
 * (b_local may be 0). loss_h: the global minibatch loss (blocking, as nrc_train). Requires an attached comm. */
nrc_status nrc_train_dp(nrc_net* net, const float* inputs_d, const float* targets_d, uint32_t b_local,
                        uint32_t global_b, float* loss_h);
/* nrc_train_dp whose global minibatch loss goes to device memory loss_d (may be NULL); never blocks. The form for one
 * host thread driving several in-process ranks round-robin (nrc_peer_exchange_open_local): a blocking loss read on
 * rank 0 would wait for a step that needs its peers' words, which the same thread has not issued yet. */
nrc_status nrc_train_dp_async(nrc_net* net, const float* inputs_d, const float* targets_d, uint32_t b_local,
                              uint32_t global_b, float* loss_d);

/* One-shot peer exchange (round 4; width-64 Frequency / FrequencySH): instead of an RCCL all-reduce, each rank stores
 * its gradient straight into a receive buffer of every peer over xGMI (IPC-mapped uncached device memory) and releases
 * a flag; the Adam step waits for all flags and sums the world gradients in rank order (bitwise-identical replicas;
 * at world 2 bitwise the RCCL sum). Set up once, collectively:
 *   nrc_peer_exchange_handle(net, world, h)   allocate this rank's buffer, return its IPC handle (64 B);
 *   exchange the handles by any means (torch.distributed, MPI, RCCL all-gather);
 *   nrc_peer_exchange_open(net, rank, world, all_handles)   (world x 64 B in rank order) map the peers' buffers.
 * While open, nrc_train_dp (and nrc_process_frame_shard) use it and need no communicator. Every rank must call
 * nrc_train_dp the same number of times; a peer missing for ~10 s ends the wait with NRC_ERR_INTERNAL. Close on
 * every rank after a barrier. */
#define NRC_PEER_HANDLE_BYTES 64
nrc_status nrc_peer_exchange_handle(nrc_net* net, int world, void* handle_out);
nrc_status nrc_peer_exchange_open(nrc_net* net, int rank, int world, const void* handles);
nrc_status nrc_peer_exchange_close(nrc_net* net);
/* In-process setup (round 5): one process driving several handles -- one per device, as the reference's multi-device
 * renderer keeps one Device per GPU in one process, or several on one device. nets[r] becomes rank r; each
 * handle's receive buffer is allocated on its own device and the others store into it through plain device pointers
 * (peer access enabled between the devices; no IPC). Replaces any exchange the handles had open. The handles share
 * each other's buffers, so they form one group: nrc_peer_exchange_close or nrc_destroy on any member, or a new open
 * that takes a member, waits for every member's stream and closes the exchange of all of them. Handles on one device
 * take the split form of the exchange (nrc_train_dp of each must then run on its own stream, since a rank's wait
 * completes only after its peers have pushed); on separate devices the fused form. A single host thread that issues the
 * ranks' steps round-robin must not block on a loss inside the round (nrc_train_dp's loss_h, nrc_process_frame_shard's
 * loss): rank 0's step completes only once every peer's step has been issued. Use nrc_train_dp_async and read the
 * losses after the round, or one host thread per rank. */
nrc_status nrc_peer_exchange_open_local(nrc_net* const* nets, int world);

/* ---- state access (host buffers of nrc_get_num_params() f32; synchronous) ----
 * Frequency: NRC_NUM_PARAMS (layout.h canonical blob). Hash: NRC_HASH_NUM_PARAMS = MLP blob then the grid table
 * [entry][2] (the grid's per-entry Adam step counters are internal). */
nrc_status nrc_get_num_params(const nrc_net* net, uint64_t* n);
nrc_status nrc_get_state(nrc_net* net, int slot, float* host_dst);
nrc_status nrc_set_state(nrc_net* net, int slot, const float* host_src);
nrc_status nrc_get_step(const nrc_net* net, uint32_t* step);
nrc_status nrc_set_step(nrc_net* net, uint32_t step);

/* ---- test / tuning entries ---- */
/* Process-wide A/B knobs (the library reads no environment variables): "train_kernel" (training kernel at nrc_init:
 * Frequency -1/0 decoupled chain, 1 / 2 round-2 t16 role-split / 4-wave; 32 the round-1 32x32x16 kernel, for Frequency
 * and Hash), "train_shape" (decoupled chain block shape 0..7, -1 = by batch size), "scatter_min" / "scatter_max" (Hash
 * grid-scatter slice plan), "hash_infer" (Hash: 1 = gather the table entries per query -- the round-2 inference kernel
 * and, in training, the t16 kernel's gathering encoder -- instead of the LDS-table feature pass), "t16_groups" (1 = 64-sample blocks
 * of the role-split kernel, debug library), "peer_path" (nrc_train_dp over a peer exchange: 0 reduce / push / apply
 * launches, 1 fused, 2 split; tests: 3 the split form's gradient pass + push alone, 4 its wait + sum + Adam alone),
 * "px_polls" (bound of the exchange's wait loops, -1 = 2^21 polls, about 10 s), "scatter_part" (Hash training: first
 * grid level whose scatter stores per-slice partial sums instead of adding with atomics, 16 = none), "scatter_compact"
 * (Hash training: first grid level whose scatter queues its in-part corners before the adds, 16 = none),
 * "hash_train_feat" (Hash training: the batch's level features by 0 the LDS-table pass, 1 gathers), "hash_adam" (Hash
 * training: 0 = the MLP and grid optimizer updates as two launches instead of one), "hash_feat_p"
 * (Hash inference: query ranges per level of the feature pass); debug library only: "dc_dw0_delay", "hash_feat_abl".
 * -1 restores the production choice. A value outside a knob's range (train_kernel -1/0/1/2/32,
 * train_shape -1..7, scatter_min / scatter_max -1 or 16..2^20, hash_infer -1..1, t16_groups -1/1/2, dc_dw0_delay -1..2^20, hash_feat_abl
 * -1..36, hash_feat_p -1 or a multiple of 8 in 8..256, peer_path -1..4, px_polls -1 or 1..2^21, scatter_part / scatter_compact -1..16, hash_train_feat -1..1, hash_adam -1..0) is
 * NRC_ERR_INVALID_ARGUMENT and leaves the knob unchanged. */
nrc_status nrc_debug_set_knob(const char* name, int value);
nrc_status nrc_debug_get_knob(const char* name, int* value);
/* Test entry: set the peer exchange's sequence number (the tag of the last step; the next step uses seq + 1, and
 * 0xFFFFFFFF is followed by 2 so that the buffer parity keeps alternating). Between steps, the same value on every rank. */
nrc_status nrc_debug_set_peer_seq(nrc_net* net, uint32_t seq);
/* Inference through a specific kernel variant for in-process A/B timing; results are identical in meaning to
 * nrc_infer_stream. The product library has variant 47 (the production kernel) only; the debug library
 * (libnrc_amd_debug.so) also has 0, 23, 30, 39 (47 with the 32x32x16 output layer), 40 / 48 (39 / 47 + in-kernel
 * clock) and 50 / 51 (the 16x16x32 kernel). */
nrc_status nrc_debug_infer_variant(nrc_net* net, int variant, const float* inputs_d, float* outputs_d, uint32_t n,
                                   hipStream_t stream);
/* Diagnostic (debug library): after a launch of a clocked inference variant (40, 48), per wave 6 uint64: s_memtime cycles
 * of its persistent loop, s_memrealtime (100 MHz) at loop start, at loop end and at wave start, HW_ID, XCC_ID:
 * 6 * *waves values into host_dst (at most cap_waves waves). */
nrc_status nrc_debug_read_infer_clock(uint64_t* host_dst, uint32_t cap_waves, uint32_t* waves);
/* Diagnostic (debug library): the training fwd/bwd kernel with s_memtime phase stamps written to stamps_d: 16 uint64
 * per wave, [block][wave][16]: the decoupled-chain kernel for b <= 4096 (nrc_train_dc.hip, dc_waves_per_block waves
 * per block), else the 4-wave t16 kernel [block][4][16]; performs no optimizer step. */
nrc_status nrc_debug_train_stamps(nrc_net* net, const float* inputs_d, const float* targets_d, uint32_t b,
                                  uint64_t* stamps_d);
/* Diagnostic (InputEncoding::Hash): the inputs of the last training call's grid-gradient scatter, copied on the
 * handle's stream into device buffers: pos_d [b][4] floats (position, 0), dy_d [16 levels][b] packed f16 pairs
 * (dL/d feature 0, 1 of that level, loss-scaled). b <= the last call's sample count. */
nrc_status nrc_debug_hash_scatter_inputs(nrc_net* net, float* pos_d, uint32_t* dy_d, uint32_t b);
/* Diagnostic (debug library): the round-1 inference kernel with s_memtime phase stamps; per wave of its grid, 8 uint64
 * cycle sums (encode + prefetch, layers 0..4, output layer, epilogue) go to stamps_d, which must hold
 * 8 * NRC_INFER_STAMP_WAVES_MAX entries; *waves_h receives the number of waves written. */
#define NRC_INFER_STAMP_WAVES_MAX 8192
nrc_status nrc_debug_infer_stamps(nrc_net* net, const float* inputs_d, float* outputs_d, uint32_t n,
                                  uint64_t* stamps_d, uint64_t* waves_h);
/* Width-128 networks: inference with either precision's weight image (both are packed from the inference
 * weights), regardless of the configured infer_precision (A/B timing and parity tests). Bits 4+ of precision pick a
 * kernel variant of the debug library (Frequency only): 1 = 1024-thread blocks, 2 = FP8 with the ReLU on the
 * converted bytes. */
nrc_status nrc_debug_infer_precision(nrc_net* net, int precision, const float* inputs_d, float* outputs_d, uint32_t n,
                                     hipStream_t stream);
/* e4m3 conversion exactly as the FP8 kernels do it: clamp to [relu ? 0 : -448, 448], round to nearest even. */
nrc_status nrc_debug_fp8_convert(const float* x_d, uint8_t* y_d, uint32_t n, int relu, hipStream_t stream);
/* the Composite encoding alone, f32 [n][80] canonical tcnn feature order ---- */
nrc_status nrc_encode(const float* inputs_d, float* encoded_d, uint32_t n, hipStream_t stream);
/* the encoder the MLP kernels actually run (closed-form OneBlob, f16-rounded), same output format */
nrc_status nrc_debug_encode_fast(const float* inputs_d, float* encoded_d, uint32_t n, hipStream_t stream);
/* The production encoder of the handle's configured encoding, f32 canonical order: Frequency / FrequencySH [n][80],
 * Hash [n][64] (with the inference (EMA) grid table). */
nrc_status nrc_debug_encode_net(nrc_net* net, const float* inputs_d, float* encoded_d, uint32_t n, hipStream_t stream);
/* encoder variants: 0 = encode_fast, 1 = omod doubling-chain triangle wave, 2 = encoder v3 (tent-map triangle
 * wave, clamped OneBlob wrap) */
nrc_status nrc_debug_encode_fast_variant(int variant, const float* inputs_d, float* encoded_d, uint32_t n,
                                         hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* NRC_C_H */
