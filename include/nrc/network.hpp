// nrc/network.hpp — header-only C++ mirror of the reference's nrc::Network
// (/root/reference/nrc/inc/NRCNetwork.h:20-75) over the C-ABI in nrc_c.h.
//
// Drop-in for the renderer's call sites (Device.cpp:419-420, :1287, :1349, :1504, :2411, :2419, :429):
// the same method names, overloads and semantics, with hipStream_t in place of CUstream. Like the
// reference, train()/infer() after destroy() are silent no-ops; every other failure throws
// std::runtime_error (std::invalid_argument for an unsupported encoding), as tcnn / CU_CHECK do.
#pragma once

#include <cstdint>
#include <cstdio>
#include <limits>
#include <stdexcept>
#include <string>

#include "nrc_c.h"

namespace nrc {

enum class InputEncoding : int { Frequency = NRC_ENCODING_FREQUENCY, Hash = NRC_ENCODING_HASH };

constexpr int NUM_BATCHES = NRC_NUM_BATCHES;
constexpr int NUM_TRAINING_RECORDS_PER_FRAME = NRC_NUM_TRAINING_RECORDS_PER_FRAME;
constexpr int BATCH_SIZE = NRC_BATCH_SIZE;
constexpr int NN_INPUT_DIMS = NRC_INPUT_DIMS;
constexpr int NN_OUTPUT_DIMS = NRC_OUTPUT_DIMS;

constexpr float TRAIN_LR(InputEncoding encoding) {
    return encoding == InputEncoding::Frequency ? NRC_TRAIN_LR_FREQUENCY
           : encoding == InputEncoding::Hash    ? NRC_TRAIN_LR_HASH
                                                : 1e-4f;
}

struct HyperParams {
    float learningRate;
};

struct TrainingStat {
    float loss{std::numeric_limits<float>::quiet_NaN()};
    int numTrainRecords{0};
};

class Network {
public:
    Network() { check(nrc_create(&m_net)); }
    ~Network() { nrc_free(m_net); }  // warns like NRCNetwork.cu:29-33 if destroy() was skipped
    Network(const Network&) = delete;
    Network& operator=(const Network&) = delete;

    template <bool Verbose = false>
    void init(hipStream_t stream, InputEncoding encoding) {
        const nrc_status s = nrc_init(m_net, stream, static_cast<int>(encoding), nullptr, Verbose ? 1 : 0);
        if (s == NRC_ERR_INVALID_ARGUMENT) throw std::invalid_argument(nrc_last_error());
        check(s);
    }

    void destroy() { check(nrc_destroy(m_net)); }

    // Perform a single training step on BATCH_SIZE samples
    void train(float* batchInputs_d, float* batchTargets_d, float* loss_h = nullptr) {
        quiet(nrc_train(m_net, batchInputs_d, batchTargets_d, loss_h));
    }
    void train(float* batchInputs_d, float* batchTargets_d, hipStream_t stream, float* loss_h = nullptr) {
        quiet(nrc_train_stream(m_net, batchInputs_d, batchTargets_d, stream, loss_h));
    }

    // Perform inference on the input
    void infer(float* inputs_d, float* outputs_d, uint32_t numInputs) {
        quiet(nrc_infer(m_net, inputs_d, outputs_d, numInputs));
    }
    void infer(float* inputs_d, float* outputs_d, uint32_t numInputs, hipStream_t stream) {
        quiet(nrc_infer_stream(m_net, inputs_d, outputs_d, numInputs, stream));
    }

    void setStream(hipStream_t stream) { check(nrc_set_stream(m_net, stream)); }

    void setHyperParams(const HyperParams& hp) {
        const nrc_hyper_params p{hp.learningRate};
        check(nrc_set_hyper_params(m_net, &p));
    }

    void setConfig(InputEncoding encoding) {
        const nrc_status s = nrc_set_config(m_net, static_cast<int>(encoding));
        if (s == NRC_ERR_INVALID_ARGUMENT) throw std::invalid_argument(nrc_last_error());
        check(s);
    }

    float getLearningRate() const {
        float lr = 0.0f;
        check(nrc_get_learning_rate(m_net, &lr));
        return lr;
    }

    std::string configJson() const {
        size_t need = 0;
        check(nrc_get_config_json(m_net, nullptr, 0, &need));
        std::string s(need, '\0');
        check(nrc_get_config_json(m_net, &s[0], need, nullptr));
        s.resize(need ? need - 1 : 0);
        return s;
    }

    nrc_net* handle() const { return m_net; }

private:
    static void check(nrc_status s) {
        if (s != NRC_OK) throw std::runtime_error(std::string("nrc: ") + nrc_last_error());
    }
    static void quiet(nrc_status s) {
        if (s == NRC_ERR_DESTROYED) return;  // NRCNetwork.cu:43, :66
        check(s);
    }

    nrc_net* m_net = nullptr;
};

}  // namespace nrc
