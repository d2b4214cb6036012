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
