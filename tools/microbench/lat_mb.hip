// lat_mb.hip -- dependent-latency probes on gfx950 (one wave): fp64 fma/add/mul, fp32 fma, LDS read
#include <hip/hip_runtime.h>
#include <stdio.h>

#define N 64
template <int OP>
__global__ void k(double* out, long long* cyc) {
    double x = out[threadIdx.x], s = out[threadIdx.x + 64];
    float xf = (float)x, sf = (float)s;
    long long t0 = clock64();
    for (int it = 0; it < 64; ++it) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            if (OP == 0) x = __builtin_fma(s, x, 1.0);
            if (OP == 1) x = x + s;
            if (OP == 2) x = x * s;
            if (OP == 3) xf = __builtin_fmaf(sf, xf, 1.0f);
        }
    }
    long long t1 = clock64();
    out[threadIdx.x] = x + xf;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    double* o;
    long long* c;
    (void)hipMalloc(&o, 128 * 8);
    (void)hipMemset(o, 0, 128 * 8);
    (void)hipMalloc(&c, 8);
    const char* names[] = {"v_fma_f64", "v_add_f64", "v_mul_f64", "v_fma_f32"};
    for (int op = 0; op < 4; ++op) {
        for (int it = 0; it < 2; ++it) {
            if (op == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, o, c);
            if (op == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, o, c);
            if (op == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, o, c);
            if (op == 3) hipLaunchKernelGGL(k<3>, dim3(1), dim3(64), 0, 0, o, c);
        }
        (void)hipDeviceSynchronize();
        long long h;
        (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        printf("dependent %-10s %6.1f cycles\n", names[op], (double)h / (64.0 * N));
    }
    return 0;
}
