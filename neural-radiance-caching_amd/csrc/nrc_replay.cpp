// nrc_replay — replays a recorded NRC sample stream (include/nrc/stream.h) through the MI355X NRC module,
// frame by frame, exactly as the reference renderer drives it after the OptiX trace (Device::render,
// /root/reference/nrc/src/Device.cpp:2493-2515): infer -> accumulate -> propagate -> shuffle -> 4 x train.
// It is the C++ stand-in for the renderer: plain C-ABI calls on hipMalloc'ed buffers, no torch.
//
//   nrc_replay <stream.nrcs> [--frames N] [--no-train] [--dump-output out.f32] [--dump-results out.f32]
//              [--ranks N | --rank r --world N --id-file F]
//
// Prints one JSON line per frame (loss, GPU ms of the frame's NRC work) and a summary line.
//
// Data parallel: with --ranks N the process forks N ranks (before any HIP call; rank r uses HIP
// device r % device_count), or an external launcher starts each rank with --rank/--world/--id-file. Rank 0 writes
// the RCCL unique id to the id file, every rank attaches a communicator to its handle (nrc_set_comm) and replays
// its shard of every frame through nrc_process_frame_shard: the pixels shard_range(screen, r, N), every
// train-suffix end, and its 1/N slice of each 16,384-sample minibatch, the gradient all-reduced inside the
// library. Dumps get a ".rank<r>" suffix for N > 1 (only the rank's pixel range of the output is written).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <thread>

#include "nrc/stream.h"

namespace {

void die(const char* what, nrc_status st) {
    std::fprintf(stderr, "nrc_replay: %s failed (%d): %s\n", what, (int)st, nrc_last_error());
    std::exit(2);
}
#define NRC(call)                                   \
    do {                                            \
        nrc_status st_ = (call);                    \
        if (st_ != NRC_OK) die(#call, st_);         \
    } while (0)
#define HIP(call)                                                                        \
    do {                                                                                 \
        hipError_t e_ = (call);                                                          \
        if (e_ != hipSuccess) {                                                          \
            std::fprintf(stderr, "nrc_replay: %s: %s\n", #call, hipGetErrorString(e_));  \
            std::exit(2);                                                                \
        }                                                                                \
    } while (0)

template <class T>
T* dalloc(size_t count) {
    void* p = nullptr;
    HIP(hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T)));
    HIP(hipMemset(p, 0, std::max<size_t>(count, 1) * sizeof(T)));
    return static_cast<T*>(p);
}

void dump(const char* path, const void* dev, size_t bytes) {
    std::vector<char> h(bytes);
    HIP(hipMemcpy(h.data(), dev, bytes, hipMemcpyDeviceToHost));
    FILE* f = std::fopen(path, "wb");
    if (!f || std::fwrite(h.data(), 1, bytes, f) != bytes) {
        std::fprintf(stderr, "nrc_replay: cannot write %s\n", path);
        std::exit(2);
    }
    std::fclose(f);
}

void shard_range(uint32_t n, int rank, int world, uint32_t* begin, uint32_t* end) {
    const uint32_t base = n / world, rem = n % world;
    *begin = rank * base + std::min<uint32_t>(rank, rem);
    *end = *begin + base + (rank < (int)rem ? 1 : 0);
}

// rank 0 publishes the RCCL unique id (write + rename, so readers never see a partial file); the others wait for it
void exchange_id(const std::string& file, int rank, unsigned char* id) {
    if (rank == 0) {
        NRC(nrc_comm_get_unique_id(id));
        const std::string tmp = file + ".tmp";
        FILE* f = std::fopen(tmp.c_str(), "wb");
        if (!f || std::fwrite(id, 1, NRC_COMM_UNIQUE_ID_BYTES, f) != NRC_COMM_UNIQUE_ID_BYTES) {
            std::fprintf(stderr, "nrc_replay: cannot write %s\n", tmp.c_str());
            std::exit(2);
        }
        std::fclose(f);
        if (std::rename(tmp.c_str(), file.c_str()) != 0) std::exit(2);
        return;
    }
    for (int i = 0; i < 6000; ++i) {  // 60 s
        FILE* f = std::fopen(file.c_str(), "rb");
        if (f) {
            const size_t got = std::fread(id, 1, NRC_COMM_UNIQUE_ID_BYTES, f);
            std::fclose(f);
            if (got == NRC_COMM_UNIQUE_ID_BYTES) return;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    std::fprintf(stderr, "nrc_replay: rank %d timed out waiting for %s\n", rank, file.c_str());
    std::exit(2);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <stream> [--frames N] [--no-train] [--dump-output F] [--dump-results F]\n",
                     argv[0]);
        return 2;
    }
    const char* path = argv[1];
    long max_frames = -1;
    bool train = true;
    const char *dump_out = nullptr, *dump_res = nullptr;
    int ranks = 0, rank = 0, world = 1;
    std::string id_file;
    for (int i = 2; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--frames") && i + 1 < argc) max_frames = std::atol(argv[++i]);
        else if (!std::strcmp(argv[i], "--no-train")) train = false;
        else if (!std::strcmp(argv[i], "--dump-output") && i + 1 < argc) dump_out = argv[++i];
        else if (!std::strcmp(argv[i], "--dump-results") && i + 1 < argc) dump_res = argv[++i];
        else if (!std::strcmp(argv[i], "--ranks") && i + 1 < argc) ranks = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--rank") && i + 1 < argc) rank = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--world") && i + 1 < argc) world = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--id-file") && i + 1 < argc) id_file = argv[++i];
        else {
            std::fprintf(stderr, "nrc_replay: unknown argument %s\n", argv[i]);
            return 2;
        }
    }
    if (ranks > 0) {
        // fork the ranks before anything touches HIP; the parent only waits
        world = ranks;
        char tmpl[] = "/tmp/nrc_replay_id_XXXXXX";
        const int fd = mkstemp(tmpl);
        if (fd < 0) return 2;
        close(fd);
        std::remove(tmpl);
        id_file = tmpl;
        std::vector<pid_t> kids;
        for (int r = 0; r < ranks; ++r) {
            const pid_t pid = fork();
            if (pid < 0) return 2;
            if (pid == 0) {
                rank = r;
                kids.clear();
                break;
            }
            kids.push_back(pid);
        }
        if (!kids.empty()) {
            int rc = 0;
            for (pid_t k : kids) {
                int st = 0;
                waitpid(k, &st, 0);
                if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = 1;
            }
            std::remove(id_file.c_str());
            return rc;
        }
    }
    const bool dp = world > 1 || ranks > 0 || !id_file.empty();
    if (dp && (world < 1 || rank < 0 || rank >= world || id_file.empty())) {
        std::fprintf(stderr, "nrc_replay: --rank/--world/--id-file (or --ranks) required for data parallelism\n");
        return 2;
    }
    std::string rank_suffix = world > 1 ? ".rank" + std::to_string(rank) : "";

    // pass 1: headers only, to size the buffers (the reference sizes them from the resolution, Device.cpp:1246-1257)
    nrc_stream* s = nullptr;
    NRC(nrc_stream_open(path, &s, nullptr, nullptr));
    nrc_stream_frame_header h{};
    int eos = 0;
    uint32_t max_screen = 0, max_tiles = 0;
    uint32_t query_layout = NRC_QUERY_COMPACT;  // the stream's RadianceQuery records: the handle is made to match
    NRC(nrc_stream_query_layout(s, &query_layout));
    long frames = 0;
    for (;;) {
        NRC(nrc_stream_next_frame(s, &h, &eos));
        if (eos || (max_frames >= 0 && frames >= max_frames)) break;
        max_screen = std::max(max_screen, h.screen_size);
        max_tiles = std::max(max_tiles, h.num_tiles);
        ++frames;
    }
    NRC(nrc_stream_close(s));

    if (dp) {
        int ndev = 0;
        HIP(hipGetDeviceCount(&ndev));
        HIP(hipSetDevice(rank % std::max(ndev, 1)));
    }
    hipStream_t stream;
    HIP(hipStreamCreate(&stream));
    const size_t cap = NRC_NUM_TRAINING_RECORDS_PER_FRAME;
    const size_t nq = (size_t)max_screen + max_tiles;
    const size_t QD = query_layout == NRC_QUERY_PADDED ? NRC_INPUT_DIMS_PADDED : NRC_INPUT_DIMS;
    nrc_frame_buffers fb{};
    float* queries_inference = dalloc<float>(nq * QD);
    nrc_float3* results_inference = dalloc<nrc_float3>(nq);
    nrc_float3* throughput = dalloc<nrc_float3>(max_screen);
    float* output = dalloc<float>((size_t)max_screen * 4);
    float* queries_vis = dalloc<float>((size_t)max_screen * QD);
    nrc_float3* results_vis = dalloc<nrc_float3>(max_screen);
    nrc_train_suffix_end_vertex* ends = dalloc<nrc_train_suffix_end_vertex>(max_tiles);
    nrc_training_record* records = dalloc<nrc_training_record>(cap);
    float* tq[2] = {dalloc<float>(cap * QD), dalloc<float>(cap * QD)};
    nrc_float3* tt[2] = {dalloc<nrc_float3>(cap), dalloc<nrc_float3>(cap)};
    int32_t* perm = dalloc<int32_t>(cap);
    uint32_t* keys = dalloc<uint32_t>(cap);
    fb.queries_inference_d = queries_inference;
    fb.results_inference_d = results_inference;
    fb.last_render_throughput_d = throughput;
    fb.output_rgba_d = output;
    fb.queries_cache_vis_d = queries_vis;
    fb.results_cache_vis_d = results_vis;
    fb.end_vertices_d = ends;
    fb.train_records_d = records;
    fb.train_queries_d[0] = tq[0];
    fb.train_queries_d[1] = tq[1];
    fb.train_targets_d[0] = tt[0];
    fb.train_targets_d[1] = tt[1];
    void* const dst[NRC_SEC_COUNT] = {queries_inference, throughput, queries_vis, ends, records, tq[0], tt[0], perm,
                                      nullptr, nullptr, nullptr, keys};

    nrc_net* net = nullptr;
    NRC(nrc_create(&net));
    nrc_config cfg = nrc_default_config(NRC_ENCODING_FREQUENCY);
    cfg.query_layout = query_layout;
    NRC(nrc_init(net, stream, NRC_ENCODING_FREQUENCY, &cfg, 0));
    void* comm = nullptr;
    if (dp) {
        unsigned char id[NRC_COMM_UNIQUE_ID_BYTES];
        exchange_id(id_file, rank, id);
        NRC(nrc_comm_init_rank(&comm, id, world, rank));
        NRC(nrc_set_comm(net, comm));
    }

    hipEvent_t e0, e1;
    HIP(hipEventCreate(&e0));
    HIP(hipEventCreate(&e1));
    NRC(nrc_stream_open(path, &s, nullptr, nullptr));
    double total_ms = 0.0, total_loss = 0.0;
    uint32_t last_screen = 0, last_tiles = 0;
    for (long f = 0; f < frames; ++f) {
        NRC(nrc_stream_next_frame(s, &h, &eos));
        // Device::render zeroes the training targets before the trace (Device.cpp:2471-2476)
        HIP(hipMemsetAsync(tt[0], 0, cap * sizeof(nrc_float3), stream));
        for (int sec = 0; sec < NRC_SEC_COUNT; ++sec)
            if (dst[sec] && (h.sections & (1u << sec))) NRC(nrc_stream_read_section(s, sec, dst[sec], stream));
        fb.permutation_d = (h.sections & (1u << NRC_SEC_PERMUTATION)) ? perm : nullptr;
        fb.shuffle_keys_d = (h.sections & (1u << NRC_SEC_SHUFFLE_KEYS)) ? keys : nullptr;
        nrc_frame_params p{};
        p.screen_size = h.screen_size;
        p.num_tiles = h.num_tiles;
        p.num_training_records = h.num_training_records;
        p.render_mode = h.render_mode;
        p.iteration_index = h.iteration_index;
        p.frame_index = h.frame_index;
        p.shuffle_seed = h.shuffle_seed;
        p.train = train ? 1 : 0;
        float loss = 0.0f;
        HIP(hipEventRecord(e0, stream));
        if (dp) {
            uint32_t p0 = 0, p1 = 0;
            shard_range(h.screen_size, rank, world, &p0, &p1);
            NRC(nrc_process_frame_shard(net, &fb, &p, p0, p1, &loss));
        } else {
            NRC(nrc_process_frame(net, &fb, &p, &loss));
        }
        HIP(hipEventRecord(e1, stream));
        HIP(hipEventSynchronize(e1));
        float ms = 0.0f;
        HIP(hipEventElapsedTime(&ms, e0, e1));
        total_ms += ms;
        total_loss += loss;
        last_screen = h.screen_size;
        last_tiles = h.num_tiles;
        std::printf("{\"frame\": %u, \"loss\": %.9g, \"gpu_ms\": %.4f, \"records\": %d, \"tiles\": %u}\n",
                    h.frame_index, (double)loss, (double)ms, h.num_training_records, h.num_tiles);
    }
    NRC(nrc_stream_close(s));
    HIP(hipStreamSynchronize(stream));
    if (dump_out) dump((dump_out + rank_suffix).c_str(), output, (size_t)last_screen * 4 * sizeof(float));
    if (dump_res)
        dump((dump_res + rank_suffix).c_str(), results_inference, ((size_t)last_screen + last_tiles) * sizeof(nrc_float3));
    uint32_t step = 0;
    NRC(nrc_get_step(net, &step));
    std::printf("{\"frames\": %ld, \"mean_loss\": %.9g, \"mean_gpu_ms\": %.4f, \"train_steps\": %u, \"rank\": %d, "
                "\"world\": %d}\n", frames, frames ? total_loss / frames : 0.0, frames ? total_ms / frames : 0.0, step, rank,
                world);
    NRC(nrc_destroy(net));
    NRC(nrc_free(net));
    if (comm) NRC(nrc_comm_destroy(comm));
    return 0;
}
