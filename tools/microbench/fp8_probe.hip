// fp8_probe.hip — checks the three hardware facts the width-128 FP8 inference path relies on:
//  1. v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 A and B) pairs byte j of lane (r, h) of A with byte j of lane (n, h)
//     of B (whatever k that is), so D[m][n] = sum_{h,j} A(m,h,j) B(n,h,j): weights can be permuted to match the
//     accumulator-as-operand byte order without knowing the k map. The sum is NOT f32-exact: measured error up to
//     2.2e-5 of sum|a*b| (results land on a grid ~13 bits below the largest product), so the check is 1e-4 of it;
//  2. the scale-A operand's op_sel picks byte `opsel` of the lane's 32-bit scale register, one E8M0 scale per row
//     (lanes r and r + 32 given the same value);
//  3. v_cvt_pk_fp8_f32 rounds to nearest even onto OCP e4m3fn (checked against a CPU RNE at every e4m3 boundary),
//     with the default MODE and with the inference kernels' MODE (IEEE off, f32 output denormals flushed).
// Build: hipcc --offload-arch=gfx950 -O2 fp8_probe.hip -o fp8_probe ; prints PASS/FAIL lines, exit 0 iff all pass.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 2;                                                              \
        }                                                                          \
    } while (0)

template <int OPSEL>
__global__ void mfma_probe(const v8i* a, const v8i* b, const uint32_t* sa, float* d) {
    const int l = threadIdx.x;
    v16f c = {};
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[l], b[l], c, 0, 0, OPSEL, sa[l], 0, 127);
    for (int i = 0; i < 16; ++i) d[l * 16 + i] = c[i];
}

__global__ void cvt_probe(const float* x, uint8_t* y, int n, int flush_mode) {
    if (flush_mode) {
        __builtin_amdgcn_s_setreg((1 << 11) | (4 << 6) | 1, 1u);
        __builtin_amdgcn_s_setreg((0 << 11) | (9 << 6) | 1, 0u);
    }
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (2 * i + 1 >= n + 1) return;
    const float a = x[2 * i], bb = (2 * i + 1 < n) ? x[2 * i + 1] : 0.0f;
    const uint32_t r = __builtin_amdgcn_cvt_pk_fp8_f32(a, bb, 0, false);
    y[2 * i] = (uint8_t)(r & 0xff);
    if (2 * i + 1 < n) y[2 * i + 1] = (uint8_t)((r >> 8) & 0xff);
}

static float e4m3_value(uint8_t c) {
    const int s = c >> 7, e = (c >> 3) & 15, m = c & 7;
    float v = e == 0 ? std::ldexp((float)m, -9) : std::ldexp(1.0f + m / 8.0f, e - 7);
    return s ? -v : v;
}
// RNE onto e4m3fn for |x| <= 448
static uint8_t e4m3_rne(float x) {
    const uint8_t s = std::signbit(x) ? 0x80 : 0;
    const double a = std::fabs((double)x);
    int e = 0;
    std::frexp(a, &e);  // a = f * 2^e, f in [0.5, 1)
    int eq = e - 1;      // floor(log2 a)
    if (a == 0.0 || eq < -6) eq = -6;
    const double quantum = std::ldexp(1.0, eq - 3);
    const double q = std::nearbyint(a / quantum);  // RNE (default rounding mode)
    const double v = q * quantum;
    // encode v
    if (v == 0.0) return s;
    int ev = 0;
    std::frexp(v, &ev);
    int E = ev - 1;
    if (E < -6) return s | (uint8_t)std::lround(v / std::ldexp(1.0, -9));  // subnormal
    const int m = (int)std::lround((v / std::ldexp(1.0, E) - 1.0) * 8.0);
    return s | (uint8_t)(((E + 7) << 3) | m);
}

static uint32_t rng_state = 12345u;
static uint32_t rnd() {
    rng_state = rng_state * 1664525u + 1013904223u;
    return rng_state >> 8;
}

// Dump mode (fp8_probe dump <file>): T trials of random A, B (bytes), C (f32) and the hardware D, for offline
// modelling of the block sum: per trial 64x32 A bytes, 64x32 B bytes, 64x16 C floats, 64x16 D floats.
__global__ void mfma_dump(const v8i* a, const v8i* b, const float* cin, float* d, int trials) {
    const int l = threadIdx.x;
    for (int t = 0; t < trials; ++t) {
        v16f c;
        for (int i = 0; i < 16; ++i) c[i] = cin[(t * 64 + l) * 16 + i];
        c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[t * 64 + l], b[t * 64 + l], c, 0, 0, 0, 127, 0, 127);
        for (int i = 0; i < 16; ++i) d[(t * 64 + l) * 16 + i] = c[i];
    }
}

static int dump(const char* path) {
    const int T = 256;
    std::vector<uint8_t> A(T * 64 * 32), B(T * 64 * 32);
    std::vector<float> C(T * 64 * 16), D(T * 64 * 16);
    for (int t = 0; t < T; ++t) {
        const int span = 1 + t % 14;  // exponent spread of the operands
        for (int i = 0; i < 64 * 32; ++i) {
            for (int which = 0; which < 2; ++which) {
                uint8_t c;
                do {
                    const int e = 7 - span / 2 + (int)(rnd() % (span + 1));
                    c = (uint8_t)(((rnd() & 1) << 7) | ((e & 15) << 3) | (rnd() & 7));
                } while ((c & 0x7f) == 0x7f || ((c >> 3) & 15) == 0);
                if (t % 4 == 3 && (rnd() % 4) == 0) c &= 0x80;  // some zeros
                (which ? B : A)[t * 64 * 32 + i] = c;
            }
        }
        for (int i = 0; i < 64 * 16; ++i) {
            const float u = (float)(rnd() & 0xffff) / 65536.0f - 0.5f;
            C[t * 64 * 16 + i] = (t % 2) ? std::ldexp(u, (int)(rnd() % 16) - 8) : 0.0f;
        }
    }
    v8i *dA, *dB;
    float *dC, *dD;
    CK(hipMalloc(&dA, A.size()));
    CK(hipMalloc(&dB, B.size()));
    CK(hipMalloc(&dC, C.size() * 4));
    CK(hipMalloc(&dD, D.size() * 4));
    CK(hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(mfma_dump, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD, T);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost));
    FILE* f = std::fopen(path, "wb");
    if (!f) return 3;
    std::fwrite(&T, 4, 1, f);
    std::fwrite(A.data(), 1, A.size(), f);
    std::fwrite(B.data(), 1, B.size(), f);
    std::fwrite(C.data(), 4, C.size(), f);
    std::fwrite(D.data(), 4, D.size(), f);
    std::fclose(f);
    std::printf("dumped %d trials to %s\n", T, path);
    return 0;
}

int main(int argc, char** argv) {
    if (argc == 3 && std::strcmp(argv[1], "dump") == 0) return dump(argv[2]);
    int fails = 0;
    // ---- 1 + 2: MFMA pairing and scale byte select
    std::vector<uint8_t> A(64 * 32), B(64 * 32);
    for (auto& v : A) {
        uint8_t c;
        do c = (uint8_t)(rnd() & 0xff); while ((c & 0x7f) == 0x7f || ((c >> 3) & 15) > 9 || ((c >> 3) & 15) < 4);
        v = c;
    }
    for (auto& v : B) {
        uint8_t c;
        do c = (uint8_t)(rnd() & 0xff); while ((c & 0x7f) == 0x7f || ((c >> 3) & 15) > 9 || ((c >> 3) & 15) < 4);
        v = c;
    }
    std::vector<uint32_t> SA(64);
    for (int l = 0; l < 64; ++l) {
        const int r = l & 31;
        uint32_t w = 0;
        for (int byte = 0; byte < 4; ++byte) w |= (uint32_t)(127 - 2 + ((r + byte) % 5)) << (8 * byte);
        SA[l] = w;
    }
    v8i *dA, *dB;
    uint32_t* dS;
    float* dD;
    CK(hipMalloc(&dA, 64 * 32));
    CK(hipMalloc(&dB, 64 * 32));
    CK(hipMalloc(&dS, 64 * 4));
    CK(hipMalloc(&dD, 64 * 16 * 4));
    CK(hipMemcpy(dA, A.data(), 64 * 32, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), 64 * 32, hipMemcpyHostToDevice));
    CK(hipMemcpy(dS, SA.data(), 64 * 4, hipMemcpyHostToDevice));
    for (int opsel = 0; opsel < 4; ++opsel) {
        switch (opsel) {
            case 0: hipLaunchKernelGGL(mfma_probe<0>, dim3(1), dim3(64), 0, 0, dA, dB, dS, dD); break;
            case 1: hipLaunchKernelGGL(mfma_probe<1>, dim3(1), dim3(64), 0, 0, dA, dB, dS, dD); break;
            case 2: hipLaunchKernelGGL(mfma_probe<2>, dim3(1), dim3(64), 0, 0, dA, dB, dS, dD); break;
            case 3: hipLaunchKernelGGL(mfma_probe<3>, dim3(1), dim3(64), 0, 0, dA, dB, dS, dD); break;
        }
        CK(hipDeviceSynchronize());
        std::vector<float> D(64 * 16);
        CK(hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost));
        double maxrel = 0.0;
        int bad = 0;
        for (int l = 0; l < 64; ++l)
            for (int i = 0; i < 16; ++i) {
                const int n = l & 31, m = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5);
                double ref = 0.0, mag = 0.0;
                for (int h = 0; h < 2; ++h)
                    for (int j = 0; j < 32; ++j) {
                        const double p = (double)e4m3_value(A[(m + 32 * h) * 32 + j]) * (double)e4m3_value(B[(n + 32 * h) * 32 + j]);
                        ref += p;
                        mag += std::fabs(p);
                    }
                const int sbyte = (SA[m] >> (8 * opsel)) & 0xff;
                ref *= std::ldexp(1.0, sbyte - 127);
                mag *= std::ldexp(1.0, sbyte - 127);
                const double rel = std::fabs(D[l * 16 + i] - ref) / mag;
                if (rel > 1e-4 && bad < 4 && opsel == 0)
                    std::printf("  m=%d n=%d gpu=%.9g ref=%.9g sum|ab|=%.6g ratio=%.6g\n", m, n, D[l * 16 + i], ref, mag,
                                D[l * 16 + i] / ref);
                maxrel = std::max(maxrel, rel);
                if (rel > 1e-4) ++bad;
            }
        std::printf("%s mfma_scale 32x32x64 e4m3: symmetric A/B byte pairing + scale-A byte %d per row: max err/sum|ab| %.3g, "
                    "%d/1024 bad\n",
                    bad ? "FAIL" : "PASS", opsel, maxrel, bad);
        fails += bad != 0;
    }
    // ---- 3: conversion
    std::vector<float> X;
    for (int c = 0; c < 0x7f; ++c) {
        const float lo = e4m3_value((uint8_t)c), hi = e4m3_value((uint8_t)(c + 1));
        const float mid = 0.5f * (lo + hi);
        X.push_back(lo);
        X.push_back(mid);
        X.push_back(std::nextafter(mid, 0.0f));
        X.push_back(std::nextafter(mid, 1e9f));
        X.push_back(std::nextafter(lo, 1e9f));
        if (c + 1 == 0x7e) X.push_back(hi);
    }
    X.push_back(448.0f);
    for (int i = 0; i < 200000; ++i) {
        const float u = (float)(rnd() & 0xffffff) / 16777216.0f;
        X.push_back(std::ldexp(1.0f + u, (int)(rnd() % 20) - 12));
    }
    X.push_back(1e-40f);  // f32 denormal
    X.push_back(0.0f);
    const int nx = (int)X.size();
    for (int i = 0; i < nx; ++i)
        if (X[i] > 448.0f) X[i] = 448.0f;
    const int nneg = nx;
    for (int i = 0; i < nneg; ++i) X.push_back(-X[i]);
    const int n = (int)X.size();
    float* dX;
    uint8_t* dY;
    CK(hipMalloc(&dX, n * 4));
    CK(hipMalloc(&dY, n + 1));
    CK(hipMemcpy(dX, X.data(), n * 4, hipMemcpyHostToDevice));
    for (int mode = 0; mode < 2; ++mode) {
        hipLaunchKernelGGL(cvt_probe, dim3((n / 2 + 256) / 256), dim3(256), 0, 0, dX, dY, n, mode);
        CK(hipDeviceSynchronize());
        std::vector<uint8_t> Y(n);
        CK(hipMemcpy(Y.data(), dY, n, hipMemcpyDeviceToHost));
        int bad = 0;
        for (int i = 0; i < n; ++i) {
            const uint8_t ref = e4m3_rne(X[i]);
            if (Y[i] != ref && !(X[i] == 0.0f && ((Y[i] & 0x7f) == 0) && ((ref & 0x7f) == 0))) {
                if (bad < 8) std::printf("  cvt mismatch x=%.9g gpu=0x%02x cpu=0x%02x\n", X[i], Y[i], ref);
                ++bad;
            }
        }
        std::printf("%s v_cvt_pk_fp8_f32 = RNE e4m3fn (%s MODE): %d/%d mismatches\n", bad ? "FAIL" : "PASS",
                    mode ? "IEEE off + f32 output-denorm flush" : "default", bad, n);
        fails += bad != 0;
    }
    std::printf(fails ? "FP8 PROBE FAIL\n" : "FP8 PROBE PASS\n");
    return fails ? 1 : 0;
}
