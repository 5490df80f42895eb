// issue_mb.hip -- single-wave cost of the chain group body ingredients (cycles per node, G=8):
//   1 row reads only   2 + broadcast S reads   3 + fma chain   4 + row writes
//   5 + readfirstlane S   6 = 4 with S read per lane (no broadcast)   7 = 4 + global store per node
#include <hip/hip_runtime.h>
#include <stdio.h>

#define G 8
#define NG 2048

template <int V>
__global__ __launch_bounds__(64) void k(double* out, long long* cyc) {
    __shared__ double rows[G][128];
    __shared__ double Sl[G][64];
    __shared__ double S[G];
    const int lane = threadIdx.x;
    for (int i = lane; i < G * 128; i += 64) (&rows[0][0])[i] = 1.0 + i * 1e-7;
    for (int i = lane; i < G * 64; i += 64) (&Sl[0][0])[i] = 0.5;
    if (lane < G) S[lane] = 0.5;
    __syncthreads();
    double x0 = 0, x1 = 0;
    const long long t0 = clock64();
    for (int g = 0; g < NG; ++g) {
        double t[G][2], s[G];
#pragma unroll
        for (int kk = 0; kk < G; ++kk) {
            t[kk][0] = rows[kk][lane * 2];
            t[kk][1] = rows[kk][lane * 2 + 1];
            if (V >= 2 && V != 6) s[kk] = S[kk];
            if (V == 6) s[kk] = Sl[kk][lane];
            if (V < 2) s[kk] = 0.5;
        }
#pragma unroll
        for (int kk = 0; kk < G; ++kk) {
            double sv = s[kk];
            if (V == 5) sv = __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(sv)),
                                               __builtin_amdgcn_readfirstlane(__double2loint(sv)));
            if (V >= 3) {
                x0 = __builtin_fma(sv, x0, t[kk][0]);
                x1 = __builtin_fma(sv, x1, t[kk][1]);
            } else {
                x0 += t[kk][0];
                x1 += t[kk][1] * sv;
            }
            if (V >= 4 && V != 7) {
                rows[kk][lane * 2] = x0;
                rows[kk][lane * 2 + 1] = x1;
            }
            if (V == 7) *reinterpret_cast<double2*>(out + 128 + ((g * G + kk) & 4095) * 128 + lane * 2) = make_double2(x0, x1);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
    const long long t1 = clock64();
    out[lane] = x0 + x1;
    if (lane == 0) cyc[0] = t1 - t0;
}

static double* o;
static long long* c;
template <int V>
void run(const char* name) {
    for (int it = 0; it < 2; ++it) hipLaunchKernelGGL(k<V>, dim3(1), dim3(64), 0, 0, o, c);
    (void)hipDeviceSynchronize();
    long long h;
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("%-34s %7.1f cycles/node\n", name, (double)h / (NG * G));
}

int main() {
    (void)hipMalloc(&o, (128 + 4096 * 128) * 8);
    (void)hipMemset(o, 0, 128 * 8);
    (void)hipMalloc(&c, 16);
    run<1>("1 row reads");
    run<2>("2 + broadcast S reads");
    run<3>("3 + fma chain");
    run<4>("4 + row writes");
    run<5>("5 + readfirstlane S");
    run<6>("6 = 4 with per-lane S reads");
    run<7>("7 = 3 + global row store");
    return 0;
}
