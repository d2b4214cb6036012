// nrc_stream.cpp — recorded NRC sample streams (include/nrc/stream.h): writer used at the renderer's dump
// points (Device.cpp:1289-1300, :1479-1496) and reader used by the replayers. Host code; device buffers are
// staged through a pinned chunk so a 1080p frame (~200 MB) never needs a second full-size host copy.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "nrc/stream.h"
#include "nrc_guard.h"

using namespace nrc_amd;

namespace {

constexpr char kMagic[8] = {'N', 'R', 'C', 'S', 'T', 'R', 'M', '\0'};
constexpr char kFrameTag[4] = {'F', 'R', 'M', 'E'};
constexpr uint32_t kHeaderBytes = 64;
constexpr uint32_t kFrameHeaderBytes = 64;
constexpr size_t kChunk = size_t(16) << 20;

struct FileHeader {
    char magic[8];
    uint32_t version, header_bytes, query_bytes, record_bytes, end_vertex_bytes, float3_bytes;
    uint32_t width, height, capacity, reserved;
    uint64_t reserved2[2];
};
static_assert(sizeof(FileHeader) == kHeaderBytes, "file header is 64 B");
static_assert(sizeof(nrc_stream_frame_header) == 48, "frame header is 48 B");

void require(bool ok, const std::string& msg) {
    if (!ok) throw ApiError(NRC_ERR_INVALID_ARGUMENT, msg);
}

bool is_device(const void* p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // plain host memory (or no GPU at all): not an error here
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

}  // namespace

struct nrc_stream {
    FILE* f = nullptr;
    bool writing = false;
    uint32_t width = 0, height = 0;
    uint32_t query_layout = NRC_QUERY_COMPACT;  // of the query sections (file header query_bytes 60 / 64)
    bool have_frame = false;
    nrc_stream_frame_header cur{};
    int64_t payload_start = 0;
    void* staging = nullptr;  // pinned, kChunk bytes, allocated on first device transfer

    void* stage() {
        if (!staging) HIP_CHECK(hipHostMalloc(&staging, kChunk, hipHostMallocDefault));
        return staging;
    }
    ~nrc_stream() {
        if (f) fclose(f);
        if (staging) (void)hipHostFree(staging);
    }
};

namespace {

void write_bytes(nrc_stream* s, const void* p, uint64_t n, hipStream_t stream) {
    if (n == 0) return;
    if (!is_device(p)) {
        require(fwrite(p, 1, n, s->f) == n, "short write");
        return;
    }
    const char* src = static_cast<const char*>(p);
    for (uint64_t off = 0; off < n; off += kChunk) {
        const size_t c = (size_t)std::min<uint64_t>(kChunk, n - off);
        HIP_CHECK(hipMemcpyAsync(s->stage(), src + off, c, hipMemcpyDeviceToHost, stream));
        HIP_CHECK(hipStreamSynchronize(stream));
        require(fwrite(s->staging, 1, c, s->f) == c, "short write");
    }
}

void read_bytes(nrc_stream* s, void* p, uint64_t n, hipStream_t stream) {
    if (n == 0) return;
    if (!is_device(p)) {
        require(fread(p, 1, n, s->f) == n, "truncated stream");
        return;
    }
    char* dst = static_cast<char*>(p);
    for (uint64_t off = 0; off < n; off += kChunk) {
        const size_t c = (size_t)std::min<uint64_t>(kChunk, n - off);
        require(fread(s->stage(), 1, c, s->f) == c, "truncated stream");
        HIP_CHECK(hipMemcpyAsync(dst + off, s->staging, c, hipMemcpyHostToDevice, stream));
        HIP_CHECK(hipStreamSynchronize(stream));  // the staging chunk is reused
    }
}

uint64_t section_offset(const nrc_stream_frame_header& h, int section) {
    uint64_t off = 0;
    for (int i = 0; i < section; ++i)
        if (h.sections & (1u << i)) off += nrc_stream_section_bytes(&h, i);
    return off;
}

}  // namespace

extern "C" {

uint64_t nrc_stream_section_bytes(const nrc_stream_frame_header* h, int section) {
    if (!h) return 0;
    const uint64_t screen = h->screen_size, tiles = h->num_tiles;
    const uint64_t nrec =
        (uint64_t)std::clamp<int64_t>(h->num_training_records, 0, NRC_NUM_TRAINING_RECORDS_PER_FRAME);
    const uint64_t q = sizeof(float) * (h->query_layout == NRC_QUERY_PADDED ? NRC_INPUT_DIMS_PADDED : NRC_INPUT_DIMS);
    const uint64_t f3 = sizeof(nrc_float3);
    switch (section) {
    case NRC_SEC_QUERIES_INFERENCE: return (screen + tiles) * q;
    case NRC_SEC_LAST_RENDER_THROUGHPUT: return screen * f3;
    case NRC_SEC_QUERIES_CACHE_VIS: return screen * q;
    case NRC_SEC_END_VERTICES: return tiles * sizeof(nrc_train_suffix_end_vertex);
    case NRC_SEC_TRAIN_RECORDS: return nrec * sizeof(nrc_training_record);
    case NRC_SEC_TRAIN_QUERIES: return nrec * q;
    case NRC_SEC_TRAIN_TARGETS: return nrec * f3;
    case NRC_SEC_PERMUTATION: return (uint64_t)NRC_NUM_TRAINING_RECORDS_PER_FRAME * sizeof(int32_t);
    case NRC_SEC_RESULTS_INFERENCE: return (screen + tiles) * f3;
    case NRC_SEC_OUTPUT_RGBA: return screen * 4 * sizeof(float);
    case NRC_SEC_LOSSES: return NRC_NUM_BATCHES * sizeof(float);
    case NRC_SEC_SHUFFLE_KEYS: return (uint64_t)NRC_NUM_TRAINING_RECORDS_PER_FRAME * sizeof(uint32_t);
    default: return 0;
    }
}

nrc_status nrc_stream_create(const char* path, uint32_t width, uint32_t height, nrc_stream** out) {
    return nrc_stream_create_layout(path, width, height, NRC_QUERY_COMPACT, out);
}

nrc_status nrc_stream_create_layout(const char* path, uint32_t width, uint32_t height, uint32_t query_layout,
                                    nrc_stream** out) {
    return guarded([&] {
        require(path && out, "NULL argument");
        require(query_layout == NRC_QUERY_COMPACT || query_layout == NRC_QUERY_PADDED, "unknown query_layout");
        *out = nullptr;
        auto s = std::make_unique<nrc_stream>();
        s->f = fopen(path, "wb");
        require(s->f != nullptr, std::string("cannot create ") + path);
        s->writing = true;
        s->width = width;
        s->height = height;
        s->query_layout = query_layout;
        FileHeader fh{};
        std::memcpy(fh.magic, kMagic, 8);
        fh.version = NRC_STREAM_VERSION;
        fh.header_bytes = kHeaderBytes;
        fh.query_bytes = sizeof(float) * (query_layout == NRC_QUERY_PADDED ? NRC_INPUT_DIMS_PADDED : NRC_INPUT_DIMS);
        fh.record_bytes = sizeof(nrc_training_record);
        fh.end_vertex_bytes = sizeof(nrc_train_suffix_end_vertex);
        fh.float3_bytes = sizeof(nrc_float3);
        fh.width = width;
        fh.height = height;
        fh.capacity = NRC_NUM_TRAINING_RECORDS_PER_FRAME;
        require(fwrite(&fh, 1, sizeof fh, s->f) == sizeof fh, "short write");
        *out = s.release();
    });
}

nrc_status nrc_stream_open(const char* path, nrc_stream** out, uint32_t* width, uint32_t* height) {
    return guarded([&] {
        require(path && out, "NULL argument");
        *out = nullptr;
        auto s = std::make_unique<nrc_stream>();
        s->f = fopen(path, "rb");
        require(s->f != nullptr, std::string("cannot open ") + path);
        FileHeader fh{};
        require(fread(&fh, 1, sizeof fh, s->f) == sizeof fh, "not an NRC stream (short header)");
        require(std::memcmp(fh.magic, kMagic, 8) == 0, "not an NRC stream (bad magic)");
        require(fh.version == NRC_STREAM_VERSION, "unsupported stream version " + std::to_string(fh.version));
        require(fh.header_bytes == kHeaderBytes && (fh.query_bytes == 60 || fh.query_bytes == 64) &&
                    fh.record_bytes == 28 && fh.end_vertex_bytes == 16 && fh.float3_bytes == 12,
                "stream record sizes do not match this build");
        require(fh.capacity == NRC_NUM_TRAINING_RECORDS_PER_FRAME, "stream capacity does not match this build");
        s->query_layout = fh.query_bytes == 64 ? NRC_QUERY_PADDED : NRC_QUERY_COMPACT;
        s->width = fh.width;
        s->height = fh.height;
        if (width) *width = fh.width;
        if (height) *height = fh.height;
        *out = s.release();
    });
}

nrc_status nrc_stream_close(nrc_stream* s) {
    return guarded([&] {
        if (!s) return;
        const bool ok = !s->writing || fflush(s->f) == 0;
        delete s;
        require(ok, "flush failed");
    });
}

nrc_status nrc_stream_write_frame(nrc_stream* s, const nrc_stream_frame_header* hdr, const void* const* sections,
                                  hipStream_t stream) {
    return guarded([&] {
        require(s && hdr, "NULL argument");
        require(s->writing, "stream is open for reading");
        nrc_stream_frame_header h = *hdr;
        h.sections = 0;
        h.payload_bytes = 0;
        h.query_layout = s->query_layout;
        for (int i = 0; i < NRC_SEC_COUNT; ++i)
            if (sections && sections[i]) {
                h.sections |= 1u << i;
                h.payload_bytes += nrc_stream_section_bytes(&h, i);
            }
        char pad[kFrameHeaderBytes - 4 - sizeof h] = {};
        require(fwrite(kFrameTag, 1, 4, s->f) == 4 && fwrite(&h, 1, sizeof h, s->f) == sizeof h &&
                    fwrite(pad, 1, sizeof pad, s->f) == sizeof pad,
                "short write");
        for (int i = 0; i < NRC_SEC_COUNT; ++i)
            if (h.sections & (1u << i)) write_bytes(s, sections[i], nrc_stream_section_bytes(&h, i), stream);
    });
}

nrc_status nrc_stream_next_frame(nrc_stream* s, nrc_stream_frame_header* hdr, int* end_of_stream) {
    return guarded([&] {
        require(s && hdr && end_of_stream, "NULL argument");
        require(!s->writing, "stream is open for writing");
        *end_of_stream = 0;
        if (s->have_frame)
            require(fseeko(s->f, (off_t)(s->payload_start + (int64_t)s->cur.payload_bytes), SEEK_SET) == 0,
                    "seek failed");
        s->have_frame = false;
        char tag[4];
        const size_t got = fread(tag, 1, 4, s->f);
        if (got == 0 && feof(s->f)) {
            *end_of_stream = 1;
            return;
        }
        require(got == 4 && std::memcmp(tag, kFrameTag, 4) == 0, "corrupt stream (bad frame tag)");
        nrc_stream_frame_header h{};
        char pad[kFrameHeaderBytes - 4 - sizeof h];
        require(fread(&h, 1, sizeof h, s->f) == sizeof h && fread(pad, 1, sizeof pad, s->f) == sizeof pad,
                "truncated stream (frame header)");
        h.query_layout = s->query_layout;  // the file header's record size decides
        uint64_t need = 0;
        for (int i = 0; i < NRC_SEC_COUNT; ++i)
            if (h.sections & (1u << i)) need += nrc_stream_section_bytes(&h, i);
        require(h.payload_bytes >= need, "corrupt stream (payload shorter than its sections)");
        s->payload_start = (int64_t)ftello(s->f);
        s->cur = h;
        s->have_frame = true;
        *hdr = h;
    });
}

nrc_status nrc_stream_read_section(nrc_stream* s, int section, void* dst, hipStream_t stream) {
    return guarded([&] {
        require(s && dst, "NULL argument");
        require(s->have_frame, "no current frame (call nrc_stream_next_frame)");
        require(section >= 0 && section < NRC_SEC_COUNT && (s->cur.sections & (1u << section)),
                "section not present in this frame");
        const uint64_t off = section_offset(s->cur, section);
        require(fseeko(s->f, (off_t)(s->payload_start + (int64_t)off), SEEK_SET) == 0, "seek failed");
        read_bytes(s, dst, nrc_stream_section_bytes(&s->cur, section), stream);
    });
}

nrc_status nrc_stream_query_layout(const nrc_stream* s, uint32_t* query_layout) {
    return guarded([&] {
        require(s && query_layout, "NULL argument");
        *query_layout = s->query_layout;
    });
}

}  // extern "C"
