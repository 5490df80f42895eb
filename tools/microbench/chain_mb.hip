// chain_mb.hip -- microbenchmark of the long-path chain wave's inner loop (sm_chain.hip):
// cycles per node of  poll state -> read row -> x = fma(S, x, t) -> write row -> publish
// out of an LDS ring, with optional helper-wave load on the same workgroup.
//   mode 0: chain wave alone, states pre-set (pure chain latency)
//   mode 1 (k_mb1): + 15 waves spinning on LDS with s_sleep (as helpers waiting for the chain)
//   mode 2: + 15 helper waves refilling entries the chain has finished (full protocol)
// Build: hipcc --offload-arch=gfx950 -O3 -o chain_mb chain_mb.hip ; run: ./chain_mb
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define R 90
#define G 8
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
__device__ __forceinline__ void lds_store(int* p, int v) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

template <int MODE, int PRIO>
__global__ __launch_bounds__(1024) void k_mb(double* out, long long* cyc) {
    __shared__ Ring ring;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int i = threadIdx.x; i < R * 128; i += blockDim.x) (&ring.x[0][0])[i] = 1.0 + i * 1e-6;
    for (int i = threadIdx.x; i < R; i += blockDim.x) {
        ring.h[i].state = MODE == 2 ? (i < R ? 2 * i + 1 : 0) : 1;
        ring.h[i].S = 0.5;
    }
    __syncthreads();
    if (wave == 0) {
        if (PRIO) __builtin_amdgcn_s_setprio(3);
        double x0 = 0, x1 = 0;
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
                for (int g = 0; g < G; ++g) st[g] = lds_state(&ring.h[eg[g]].state);
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    S[g] = ring.h[eg[g]].S;
                    t[g][0] = ring.x[eg[g]][lane * 2];
                    t[g][1] = ring.x[eg[g]][lane * 2 + 1];
                }
                ok = true;
#pragma unroll
                for (int g = 0; g < G; ++g) ok &= MODE == 2 ? st[g] == 2 * (j0 + g) + 1 : st[g] == 1;
            } while (!ok);
#pragma unroll
            for (int g = 0; g < G; ++g) {
                x0 = __builtin_fma(S[g], x0, t[g][0]);
                x1 = __builtin_fma(S[g], x1, t[g][1]);
                ring.x[eg[g]][lane * 2] = MODE == 2 ? x0 : t[g][0];
                ring.x[eg[g]][lane * 2 + 1] = MODE == 2 ? x1 : t[g][1];
            }
            if (MODE == 2) {
#pragma unroll
                for (int g = 0; g < G; ++g) lds_store(&ring.h[eg[g]].state, 2 * (j0 + g) + 2);
            }
            e0 = e0 + G < R ? e0 + G : e0 + G - R;
        }
        const long long t1 = clock64();
        out[blockIdx.x * 64 + lane] = x0 + x1;
        if (lane == 0) cyc[blockIdx.x] = t1 - t0;
    } else if (MODE == 2) {
        // helper hh owns entries [hh*6, hh*6+6): refill node j+R after the chain finished node j
        const int hh = wave - 1;
        for (int base = hh * 6 + R; base < NODES + R; base += R) {
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const int e = hh * 6 + k;
                const int jp = base - R + k;
                if (jp >= NODES) break;
                while (lds_state(&ring.h[e].state) != 2 * jp + 2) __builtin_amdgcn_s_sleep(1);
                const double v0 = ring.x[e][lane * 2], v1 = ring.x[e][lane * 2 + 1];
                ring.x[e][lane * 2] = v0 * 0.5 + 1.0;
                ring.x[e][lane * 2 + 1] = v1 * 0.5 + 1.0;
                if (base + k < NODES) {
                    __builtin_amdgcn_s_waitcnt(0xC07F);
                    lds_store(&ring.h[e].state, 2 * (base + k) + 1);
                }
            }
        }
    }
}

// mode 1 needs the done flag from the chain wave too
template <int PRIO>
__global__ __launch_bounds__(1024) void k_mb1(double* out, long long* cyc) {
    __shared__ Ring ring;
    __shared__ int done;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int i = threadIdx.x; i < R * 128; i += blockDim.x) (&ring.x[0][0])[i] = 1.0 + i * 1e-6;
    for (int i = threadIdx.x; i < R; i += blockDim.x) {
        ring.h[i].state = 1;
        ring.h[i].S = 0.5;
    }
    if (threadIdx.x == 0) done = 0;
    __syncthreads();
    if (wave == 0) {
        if (PRIO) __builtin_amdgcn_s_setprio(3);
        double x0 = 0, x1 = 0;
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
                for (int g = 0; g < G; ++g) st[g] = lds_state(&ring.h[eg[g]].state);
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
                x0 = __builtin_fma(S[g], x0, t[g][0]);
                x1 = __builtin_fma(S[g], x1, t[g][1]);
                ring.x[eg[g]][lane * 2] = t[g][0];
                ring.x[eg[g]][lane * 2 + 1] = t[g][1];
            }
            e0 = e0 + G < R ? e0 + G : e0 + G - R;
        }
        const long long t1 = clock64();
        out[blockIdx.x * 64 + lane] = x0 + x1;
        if (lane == 0) cyc[blockIdx.x] = t1 - t0;
        lds_store(&done, 1);
    } else {
        while (lds_state(&done) == 0) __builtin_amdgcn_s_sleep(1);
    }
}

int main() {
    double* out;
    long long* cyc;
    (void)hipMalloc(&out, 64 * 8 * 8);
    (void)hipMalloc(&cyc, 8 * 8);
    long long h[8];
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    auto run = [&](const char* name, void (*launch)()) {
        for (int it = 0; it < 2; ++it) {
            (void)hipEventRecord(a);
            launch();
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
        }
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        (void)hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-34s %8.1f cycles/node  %7.1f ns/node (wall)\n", name, (double)h[0] / NODES, ms * 1e6 / NODES);
    };
    static double* o;
    static long long* c;
    o = out;
    c = cyc;
    run("mode0 chain alone (64 thr)", [] { hipLaunchKernelGGL((k_mb<0, 1>), dim3(1), dim3(64), 0, 0, o, c); });
    run("mode0 chain alone, 16 idle waves", [] { hipLaunchKernelGGL((k_mb1<1>), dim3(1), dim3(1024), 0, 0, o, c); });
    run("mode0 no prio, 16 idle waves", [] { hipLaunchKernelGGL((k_mb1<0>), dim3(1), dim3(1024), 0, 0, o, c); });
    run("mode2 full protocol prio", [] { hipLaunchKernelGGL((k_mb<2, 1>), dim3(1), dim3(1024), 0, 0, o, c); });
    run("mode2 full protocol no prio", [] { hipLaunchKernelGGL((k_mb<2, 0>), dim3(1), dim3(1024), 0, 0, o, c); });
    return 0;
}
