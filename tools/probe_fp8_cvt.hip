// Probe: what v_cvt_pk_fp8_f32 (and the gfx950 scaled form) return for out-of-range, negative and non-finite inputs
// on this hardware (the FP8 inference path clamps with med3 before converting; whether the convert saturates by itself
// decides if that clamp can go). One wave, results printed from the host; OVFL = 1 runs the converts with
// MODE.FP16_OVFL (bit 23) set, to see whether that mode bit saturates the FP8 converts as it does f16 results.
//   hipcc --offload-arch=gfx950 -O2 tools/probe_fp8_cvt.hip -o tools/probe_fp8_cvt && ./tools/probe_fp8_cvt
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>

template <int OVFL>
__global__ void probe(const float* in, uint32_t* out, int n) {
    if (OVFL) __builtin_amdgcn_s_setreg((0 << 11) | (23 << 6) | 1 /* hwreg(HW_REG_MODE, 23, 1) */, 1u);
    const int i = threadIdx.x;
    if (i >= n) return;
    const float x = in[i];
    out[3 * i + 0] = __builtin_amdgcn_cvt_pk_fp8_f32(x, 0.0f, 0u, false);
    typedef short s2 __attribute__((ext_vector_type(2)));
    const s2 z = {0, 0};
    out[3 * i + 1] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(z, x, 0.0f, 1.0f, false));
    out[3 * i + 2] = __builtin_amdgcn_cvt_pk_bf8_f32(x, 0.0f, 0u, false);
}

int main() {
    const float v[] = {0.0f, -0.0f, 1.0f, -1.0f, 0.3f, 240.0f, 448.0f, 460.0f, 464.0f, 480.0f, 500.0f, 1000.0f,
                       -1000.0f, 1e30f, -1e30f, INFINITY, -INFINITY, NAN, 1e-9f, -1e-9f};
    const int n = sizeof(v) / sizeof(v[0]);
    float* din;
    uint32_t* dout;
    if (hipMalloc(&din, sizeof(v)) != hipSuccess || hipMalloc(&dout, 3 * n * 4) != hipSuccess) return 1;
    if (hipMemcpy(din, v, sizeof(v), hipMemcpyHostToDevice) != hipSuccess) return 1;
    for (int ovfl = 0; ovfl < 2; ++ovfl) {
        if (ovfl) probe<1><<<1, 64>>>(din, dout, n);
        else probe<0><<<1, 64>>>(din, dout, n);
        uint32_t r[3 * 64];
        if (hipMemcpy(r, dout, 3 * n * 4, hipMemcpyDeviceToHost) != hipSuccess) return 2;
        printf("MODE.FP16_OVFL = %d\n%14s  %6s  %6s  %6s\n", ovfl, "x", "fp8", "sc_fp8", "bf8");
        for (int i = 0; i < n; ++i)
            printf("%14g  0x%02x    0x%02x    0x%02x\n", v[i], r[3 * i] & 0xff, r[3 * i + 1] & 0xff, r[3 * i + 2] & 0xff);
    }
    return hipFree(din) != hipSuccess || hipFree(dout) != hipSuccess;
}
