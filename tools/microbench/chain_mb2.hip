// chain_mb2.hip -- decomposition of the chain wave's per-node cost (see chain_mb.hip):
// variants of one 64-thread chain wave over an LDS ring (states pre-set, no helpers).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R 90
#define NODES 16384

struct Hdr {
    int state;
    int pad[3];
    double S;
};
struct Ring {
    double x[R][128];
    Hdr h[R];
};

__device__ __forceinline__ int lds_state(int* p) {
    const int v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    return v;
}

// WRITE: write the result row back; DEP: x = fma(S, x, t) (else x += t*S independent per node)
template <int G, int WRITE, int DEP, int POLL>
__global__ __launch_bounds__(64) void k_v(double* out, long long* cyc) {
    __shared__ Ring ring;
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < R * 128; i += blockDim.x) (&ring.x[0][0])[i] = 1.0 + i * 1e-6;
    for (int i = threadIdx.x; i < R; i += blockDim.x) {
        ring.h[i].state = 1;
        ring.h[i].S = 0.5;
    }
    __syncthreads();
    double x0 = 0, x1 = 0, y0 = 0, y1 = 0;
    const long long t0 = clock64();
    int e0 = 0;
    for (int j0 = 0; j0 < NODES; j0 += G) {
        int eg[G];
#pragma unroll
        for (int g = 0; g < G; ++g) eg[g] = e0 + g < R ? e0 + g : e0 + g - R;
        double t[G][2], S[G];
        bool ok;
        do {
            int st[G];
#pragma unroll
            for (int g = 0; g < G; ++g) st[g] = POLL ? lds_state(&ring.h[eg[g]].state) : 1;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                S[g] = ring.h[eg[g]].S;
                t[g][0] = ring.x[eg[g]][lane * 2];
                t[g][1] = ring.x[eg[g]][lane * 2 + 1];
            }
            ok = true;
#pragma unroll
            for (int g = 0; g < G; ++g) ok &= st[g] == 1;
        } while (!ok);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            if (DEP) {
                x0 = __builtin_fma(S[g], x0, t[g][0]);
                x1 = __builtin_fma(S[g], x1, t[g][1]);
            } else {
                y0 = t[g][0] * S[g];
                y1 = t[g][1] * S[g];
                x0 += y0;
                x1 += y1;
            }
            if (WRITE) {
                ring.x[eg[g]][lane * 2] = DEP ? x0 : y0;
                ring.x[eg[g]][lane * 2 + 1] = DEP ? x1 : y1;
            }
        }
        e0 = e0 + G < R ? e0 + G : e0 + G - R;
    }
    const long long t1 = clock64();
    out[lane] = x0 + x1;
    if (lane == 0) cyc[0] = t1 - t0;
}

// latency probes: dependent LDS reads; dependent fp64 fma
__global__ void k_lat(double* out, long long* cyc, int n) {
    __shared__ int nxt[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) nxt[i] = (i * 17 + 5) & 1023;
    __syncthreads();
    int p = threadIdx.x & 3;
    long long t0 = clock64();
    for (int i = 0; i < n; ++i) p = nxt[p];
    long long t1 = clock64();
    double x = out[threadIdx.x], s = out[threadIdx.x + 64];
    for (int i = 0; i < n; ++i) x = __builtin_fma(s, x, 1.0);
    long long t2 = clock64();
    out[threadIdx.x] = x + p;
    if (threadIdx.x == 0) {
        cyc[0] = t1 - t0;
        cyc[1] = t2 - t1;
    }
}

static double* o;
static long long* c;

template <int G, int W, int D, int P>
void run(const char* name) {
    for (int it = 0; it < 2; ++it) hipLaunchKernelGGL((k_v<G, W, D, P>), dim3(1), dim3(64), 0, 0, o, c);
    (void)hipDeviceSynchronize();
    long long h;
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("%-40s %8.1f cycles/node\n", name, (double)h / NODES);
}

int main() {
    (void)hipMalloc(&o, 128 * 8);
    (void)hipMemset(o, 0, 128 * 8);
    (void)hipMalloc(&c, 16);
    run<8, 1, 1, 1>("G8 write dep poll (baseline)");
    run<8, 0, 1, 1>("G8 nowrite dep poll");
    run<8, 1, 0, 1>("G8 write indep poll");
    run<8, 0, 0, 1>("G8 nowrite indep poll");
    run<8, 1, 1, 0>("G8 write dep nopoll");
    run<16, 1, 1, 1>("G16 write dep poll");
    run<4, 1, 1, 1>("G4 write dep poll");
    hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, o, c, 4096);
    (void)hipDeviceSynchronize();
    long long h[2];
    (void)hipMemcpy(h, c, 16, hipMemcpyDeviceToHost);
    printf("dependent ds_read latency   %8.1f cycles\n", (double)h[0] / 4096);
    printf("dependent v_fma_f64 latency %8.1f cycles\n", (double)h[1] / 4096);
    return 0;
}
