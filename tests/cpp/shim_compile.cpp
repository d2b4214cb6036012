// Compile check of the header-only C++ mirror (tests/test_abi.py): the reference's call pattern.
#include "nrc/network.hpp"

void frame(nrc::Network& net, hipStream_t stream, float* queries, float* results, uint32_t n, float* trainIn,
           float* trainTgt) {
    net.init<true>(stream, nrc::InputEncoding::Frequency);       // Device.cpp:420
    net.setHyperParams({nrc::TRAIN_LR(nrc::InputEncoding::Frequency)});  // Device.cpp:2411
    net.infer(queries, results, n);                               // Device.cpp:1287
    float batchLoss = 0.0f, totalLoss = 0.0f;
    for (int b = 0; b < nrc::NUM_BATCHES; b++) {                  // Device.cpp:1503-1509
        net.train(trainIn + b * nrc::BATCH_SIZE * nrc::NN_INPUT_DIMS, trainTgt + b * nrc::BATCH_SIZE * 3, &batchLoss);
        totalLoss += batchLoss;
    }
    (void)net.getLearningRate();
    net.destroy();                                                // Device.cpp:429
}

// include/nrc/frame.h: the reference's record layouts byte for byte (neural_radiance_caching.h:57-94) and the
// struct sizes the ctypes mirror in neural-radiance-caching_amd/frame.py assumes.
#include "nrc/frame.h"
static_assert(sizeof(nrc_training_record) == 28, "TrainingRecord");
static_assert(sizeof(nrc_train_suffix_end_vertex) == 16, "TrainingSuffixEndVertex");
static_assert(sizeof(nrc_frame_buffers) == 13 * sizeof(void*), "nrc_frame_buffers");
static_assert(sizeof(nrc_frame_params) == 40, "nrc_frame_params");
