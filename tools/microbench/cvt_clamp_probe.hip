// What the VOP3 clamp bit does on v_cvt_pk_f16_f32 (gfx950): does it clamp to [0, 1] or only saturate at the f16
// range? (If it dropped negatives alone it would be a one-instruction ReLU + pack.)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

__global__ void probe(const float* x, unsigned* y, int n) {
    const int i = threadIdx.x;
    if (i >= n) return;
    unsigned a, b, c;
    asm volatile("v_cvt_pk_f16_f32 %0, %1, %2 clamp" : "=v"(a) : "v"(x[i]), "v"(x[i]));
    asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(b) : "v"(x[i]), "v"(x[i]));
    asm volatile("v_pk_max_f16 %0, %1, 0 clamp" : "=v"(c) : "v"(b));
    y[3 * i] = a;
    y[3 * i + 1] = b;
    y[3 * i + 2] = c;
}

static float h2f(unsigned short h) {
    const unsigned s = (h >> 15) & 1, e = (h >> 10) & 31, m = h & 1023;
    float v = e == 0 ? std::ldexp((float)m, -24) : e == 31 ? (m ? NAN : INFINITY) : std::ldexp((float)(m | 1024), (int)e - 25);
    return s ? -v : v;
}

int main() {
    const float h[] = {-70000.f, -2.f, -0.5f, -1e-6f, 0.f, 1e-6f, 0.25f, 0.999f, 1.f, 1.5f, 100.f, 70000.f, NAN};
    const int n = sizeof(h) / sizeof(h[0]);
    float* x;
    unsigned* y;
    (void)hipMalloc(&x, sizeof(h));
    (void)hipMalloc(&y, 12 * n);
    (void)hipMemcpy(x, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, x, y, n);
    unsigned r[3 * 16];
    (void)hipMemcpy(r, y, 12 * n, hipMemcpyDeviceToHost);
    printf("{\"rows\": [\n");
    for (int i = 0; i < n; ++i)
        printf("%s{\"x\": %g, \"cvt_clamp\": %g, \"cvt\": %g, \"pk_max0_clamp\": %g}\n", i ? "," : "", h[i],
               h2f(r[3 * i] & 0xffff), h2f(r[3 * i + 1] & 0xffff), h2f(r[3 * i + 2] & 0xffff));
    printf("]}\n");
    return 0;
}
