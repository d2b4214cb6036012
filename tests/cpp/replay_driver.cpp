// C++ caller of the drop-in: the reference renderer's per-frame call pattern (Device.cpp:1272-1302,
// :1473-1513) through nrc::Network (include/nrc/network.hpp), on hipMalloc'ed buffers.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "nrc/network.hpp"

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main() {
    const uint32_t numQueries = 1920 * 1080 / 8;
    std::vector<float> q(numQueries * nrc::NN_INPUT_DIMS), tq(nrc::NUM_TRAINING_RECORDS_PER_FRAME * 15),
        tt(nrc::NUM_TRAINING_RECORDS_PER_FRAME * 3);
    uint32_t s = 12345u;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (s >> 8) * (1.0f / 16777216.0f); };
    for (auto& v : q) v = rnd();
    for (auto& v : tq) v = rnd();
    for (auto& v : tt) v = 0.5f * rnd();
    float *q_d, *out_d, *tq_d, *tt_d;
    CHECK(hipMalloc(&q_d, q.size() * 4));
    CHECK(hipMalloc(&out_d, numQueries * 12));
    CHECK(hipMalloc(&tq_d, tq.size() * 4));
    CHECK(hipMalloc(&tt_d, tt.size() * 4));
    CHECK(hipMemcpy(q_d, q.data(), q.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(tq_d, tq.data(), tq.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(tt_d, tt.data(), tt.size() * 4, hipMemcpyHostToDevice));
    hipStream_t stream;
    CHECK(hipStreamCreate(&stream));
    float firstLoss = 0.f, lastLoss = 0.f;
    {
        nrc::Network net;
        net.init<true>(stream, nrc::InputEncoding::Frequency);
        for (int frame = 0; frame < 5; ++frame) {
            net.infer(q_d, out_d, numQueries);
            float batchLoss = 0.f, totalLoss = 0.f;
            for (int b = 0; b < nrc::NUM_BATCHES; b++) {
                net.train(tq_d + b * nrc::BATCH_SIZE * 15, tt_d + b * nrc::BATCH_SIZE * 3, &batchLoss);
                totalLoss += batchLoss;
            }
            if (frame == 0) firstLoss = totalLoss / nrc::NUM_BATCHES;
            lastLoss = totalLoss / nrc::NUM_BATCHES;
        }
        net.infer(q_d, out_d, numQueries, stream);
        CHECK(hipStreamSynchronize(stream));
        net.destroy();
        net.destroy();
        net.infer(q_d, out_d, numQueries);  // silent no-op after destroy
    }
    std::vector<float> out(numQueries * 3);
    CHECK(hipMemcpy(out.data(), out_d, out.size() * 4, hipMemcpyDeviceToHost));
    for (float v : out)
        if (!std::isfinite(v) || v < 0.f) {
            std::printf("bad output %f\n", v);
            return 2;
        }
    std::printf("loss first %g last %g\n", firstLoss, lastLoss);
    if (!(lastLoss < firstLoss)) return 3;
    std::printf("replay ok\n");
    return 0;
}
