// dp_lat.hip -- dependent-latency probes on one wave: v_fma_f64 chain, v_add_f64 chain,
// and a 4-op node step (fma, fma, fma, add) as in the up chain; cycles per op / per step.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define N 4096
__global__ void k_fma(double* out, long long* cyc, double a, double b) {
    double x = threadIdx.x;
    long long t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < N; ++i) x = __builtin_fma(a, x, b);
    long long t1 = clock64();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_step(double* out, long long* cyc, double a, double b, double c, double d) {
    double x = threadIdx.x, p = threadIdx.x * 0.5, q = threadIdx.x * 0.25;
    long long t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < N; ++i) {
        double acc = __builtin_fma(a, x, b);
        acc = __builtin_fma(c, p, acc);
        acc = __builtin_fma(d, q, acc);
        x = acc + 0.125;
    }
    long long t1 = clock64();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_f32(float* out, long long* cyc, float a, float b) {
    float x = threadIdx.x;
    long long t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < N; ++i) x = __builtin_fmaf(a, x, b);
    long long t1 = clock64();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
    double* o; float* of; long long* c; long long h;
    (void)hipMalloc(&o, 64 * 8); (void)hipMalloc(&of, 64 * 4); (void)hipMalloc(&c, 8);
    for (int it = 0; it < 2; ++it) {
        hipLaunchKernelGGL(k_fma, dim3(1), dim3(64), 0, 0, o, c, 0.999, 0.5);
        (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        if (it) printf("dependent v_fma_f64: %.2f cycles/op\n", (double)h / N);
        hipLaunchKernelGGL(k_step, dim3(1), dim3(64), 0, 0, o, c, 0.999, 0.5, 0.25, 0.125);
        (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        if (it) printf("node step fma,fma,fma,add: %.2f cycles/step\n", (double)h / N);
        hipLaunchKernelGGL(k_f32, dim3(1), dim3(64), 0, 0, of, c, 0.999f, 0.5f);
        (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        if (it) printf("dependent v_fma_f32: %.2f cycles/op\n", (double)h / N);
    }
    return 0;
}
