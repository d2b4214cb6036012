/*
 * nrc/stream.h — recorded NRC sample streams: a file format holding, per frame,
 * exactly the buffers the renderer hands to the NRC module and its surrounding kernels, so that a frame
 * sequence can be recorded once (from the reference renderer or a synthetic generator) and replayed
 * bit-identically through nrc_process_frame (include/nrc/frame.h) without OptiX.
 *
 * The sections are the buffers the reference's own debug dump points copy out
 * (/root/reference/nrc/src/Device.cpp:1289-1300 queries/results at infer, :1479-1496 shuffled training
 * samples) plus the trace outputs the post-trace kernels read (Device.cpp:1382-1469).
 *
 * Layout (little-endian, no padding, sizes in bytes):
 *   file header   64: "NRCSTRM\0", u32 version (1), u32 header_bytes (64), u32 query_bytes (60, or 64 for a stream
 *                     of padded RadianceQuery records: nrc_stream_create_layout),
 *                     u32 record_bytes (28), u32 end_vertex_bytes (16), u32 float3_bytes (12),
 *                     u32 width, u32 height, u32 capacity (65536), u32 reserved, u64 reserved[2]
 *   per frame:    "FRME" + nrc_stream_frame_header (48) + 12 reserved bytes = 64, then every present
 *                 section in ascending section order, each exactly nrc_stream_section_bytes() long.
 * A reader skips unknown trailing bytes of a frame via payload_bytes, so sections can be added later.
 */
#ifndef NRC_STREAM_H
#define NRC_STREAM_H

#include "frame.h"

#ifdef __cplusplus
extern "C" {
#endif

#define NRC_STREAM_VERSION 1

typedef enum nrc_stream_section {
    NRC_SEC_QUERIES_INFERENCE = 0,      /* (screen + tiles) x RadianceQuery (60 B) */
    NRC_SEC_LAST_RENDER_THROUGHPUT = 1, /* screen x float3 */
    NRC_SEC_QUERIES_CACHE_VIS = 2,      /* screen x RadianceQuery (CacheFirstVertex frames) */
    NRC_SEC_END_VERTICES = 3,           /* tiles x TrainingSuffixEndVertex (16 B) */
    NRC_SEC_TRAIN_RECORDS = 4,          /* nrec x TrainingRecord (28 B), nrec = min(num_training_records, capacity) */
    NRC_SEC_TRAIN_QUERIES = 5,          /* nrec x RadianceQuery */
    NRC_SEC_TRAIN_TARGETS = 6,          /* nrec x float3: radiance gathered during the trace (emission, env) */
    NRC_SEC_PERMUTATION = 7,            /* capacity x int32: a caller-made shuffle (absent: Feistel of shuffle_seed) */
    NRC_SEC_RESULTS_INFERENCE = 8,      /* (screen + tiles) x float3: recorded infer() outputs (for comparison) */
    NRC_SEC_OUTPUT_RGBA = 9,            /* screen x float4: recorded frame buffer after accumulation */
    NRC_SEC_LOSSES = 10,                /* NUM_BATCHES x f32: recorded minibatch losses */
    NRC_SEC_SHUFFLE_KEYS = 11,          /* capacity x u32: the frame's shuffle keys (the reference's curand keys,
                                           NRCUtil.cu:25); the permutation is their stable sort (frame.h) */
    NRC_SEC_COUNT = 12
} nrc_stream_section;

typedef struct nrc_stream_frame_header {
    uint32_t frame_index;
    uint32_t iteration_index;
    int32_t render_mode;          /* nrc_render_mode */
    uint32_t screen_size;
    uint32_t num_tiles;
    int32_t num_training_records; /* raw trace counter (may exceed capacity) */
    uint32_t sections;            /* bit i set <=> section i present */
    uint32_t query_layout;        /* the stream's RadianceQuery layout (NRC_QUERY_COMPACT / NRC_QUERY_PADDED): set by
                                   * the writer and the reader from the file header; sizes the query sections */
    uint64_t shuffle_seed;
    uint64_t payload_bytes;       /* bytes of all sections that follow; filled in by the writer */
} nrc_stream_frame_header;

typedef struct nrc_stream nrc_stream;

/* Bytes of a section for a frame (0 for an unknown section). capacity = NRC_NUM_TRAINING_RECORDS_PER_FRAME. */
uint64_t nrc_stream_section_bytes(const nrc_stream_frame_header* hdr, int section);

/* Create a stream file for writing (truncates). width/height are informational (0 = unknown). */
nrc_status nrc_stream_create(const char* path, uint32_t width, uint32_t height, nrc_stream** out);
/* The same for a RadianceQuery layout (nrc_config.query_layout: NRC_QUERY_COMPACT 60-byte or NRC_QUERY_PADDED 64-byte
 * records in the query sections); nrc_stream_create is the compact layout. */
nrc_status nrc_stream_create_layout(const char* path, uint32_t width, uint32_t height, uint32_t query_layout,
                                    nrc_stream** out);
/* The query layout of an open stream. */
nrc_status nrc_stream_query_layout(const nrc_stream* s, uint32_t* query_layout);
/* Open a stream file for reading; width/height may be NULL. */
nrc_status nrc_stream_open(const char* path, nrc_stream** out, uint32_t* width, uint32_t* height);
nrc_status nrc_stream_close(nrc_stream* s);

/* Append one frame. sections[i] (NRC_SEC_COUNT entries; the array itself may be NULL = none) points at
 * section i's bytes in host or device memory — device buffers (the renderer's, at the reference's dump
 * points) are staged through the host on `stream`; NULL = absent. hdr->sections and hdr->payload_bytes
 * are derived from which pointers are non-NULL. */
nrc_status nrc_stream_write_frame(nrc_stream* s, const nrc_stream_frame_header* hdr, const void* const* sections,
                                  hipStream_t stream);

/* Advance to the next frame and read its header. *end_of_stream = 1 (and NRC_OK) after the last frame. */
nrc_status nrc_stream_next_frame(nrc_stream* s, nrc_stream_frame_header* hdr, int* end_of_stream);

/* Copy a present section of the current frame into dst (host or device memory, at least
 * nrc_stream_section_bytes() long). Sections may be read in any order, any number of times. */
nrc_status nrc_stream_read_section(nrc_stream* s, int section, void* dst, hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* NRC_STREAM_H */
