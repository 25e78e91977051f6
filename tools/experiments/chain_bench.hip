// Microbenchmark: cycles per dependent float add of a sequential fold (the update's PCL-order sums).
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o _var/chain_bench tools/experiments/chain_bench.hip
// One workgroup of 64 threads; lanes 0..6 each fold 4096 floats (a) from registers only (pure
// dependent-add latency), (b) from LDS in groups of 32 read one group ahead (fold_seq's scheme),
// (c) from LDS with two groups in flight.  Prints cycles per add (s_memtime delta / adds).
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 4096;

__device__ __forceinline__ void grp_load(float4 (&g)[8], const float* f) {
#pragma unroll
    for (int u = 0; u < 8; ++u) g[u] = *reinterpret_cast<const float4*>(f + 4 * u);
}
__device__ __forceinline__ float grp_add(float acc, const float4 (&g)[8]) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        acc = acc + g[u].x;
        acc = acc + g[u].y;
        acc = acc + g[u].z;
        acc = acc + g[u].w;
    }
    return acc;
}

__device__ __forceinline__ void g4_load(float4 (&g)[4], const float* f) {
#pragma unroll
    for (int u = 0; u < 4; ++u) g[u] = *reinterpret_cast<const float4*>(f + 4 * u);
}
__device__ __forceinline__ float g4_add(float acc, const float4 (&g)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        acc = acc + g[u].x;
        acc = acc + g[u].y;
        acc = acc + g[u].z;
        acc = acc + g[u].w;
    }
    return acc;
}

__global__ __launch_bounds__(64) void chain_kernel(const float* in, float* out, long long* cyc, int mode) {
    __shared__ float buf[7][N + 4];
    const int lane = threadIdx.x;
    for (int r = 0; r < 7; ++r)
        for (int i = lane; i < N; i += 64) buf[r][i] = in[r * N + i];
    __syncthreads();
    float acc = -0.0f;
    long long t0 = 0, t1 = 0;
    if (lane < 7) {
        const float* f = buf[lane];
        t0 = __builtin_amdgcn_s_memtime();
        if (mode == 0) {
            float a = f[0], b = f[1], c = f[2], d = f[3];
            for (int k = 0; k < N; k += 4) {
                acc = acc + a;
                acc = acc + b;
                acc = acc + c;
                acc = acc + d;
                __builtin_amdgcn_sched_barrier(0);
            }
        } else if (mode == 1) {
            float4 a[8], b[8];
            grp_load(a, f);
            for (int k = 0; k < N; k += 64) {
                grp_load(b, f + k + 32);
                __builtin_amdgcn_sched_barrier(0);
                acc = grp_add(acc, a);
                grp_load(a, f + ((k + 64) % N));
                __builtin_amdgcn_sched_barrier(0);
                acc = grp_add(acc, b);
            }
        } else if (mode == 3) {
            float4 a[8], b[8];
            grp_load(a, f);
            grp_load(b, f + 32);
            for (int k = 0; k < N; k += 256) {
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    acc = grp_add(acc, a);
                    acc = grp_add(acc, b);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        } else if (mode == 4) {
            float4 a[4], b[4], c[4];
            g4_load(a, f);
            g4_load(b, f + 16);
            for (int k = 0; k < N; k += 48) {
                g4_load(c, f + ((k + 32) % N));
                __builtin_amdgcn_sched_barrier(0);
                acc = g4_add(acc, a);
                g4_load(a, f + ((k + 48) % N));
                __builtin_amdgcn_sched_barrier(0);
                acc = g4_add(acc, b);
                g4_load(b, f + ((k + 64) % N));
                __builtin_amdgcn_sched_barrier(0);
                acc = g4_add(acc, c);
            }
        } else if (mode == 2) {
            float4 a[8], b[8], c[8];
            grp_load(a, f);
            grp_load(b, f + 32);
            for (int k = 0; k < N; k += 96) {
                grp_load(c, f + ((k + 64) % N));
                __builtin_amdgcn_sched_barrier(0);
                acc = grp_add(acc, a);
                grp_load(a, f + ((k + 96) % N));
                __builtin_amdgcn_sched_barrier(0);
                acc = grp_add(acc, b);
                grp_load(b, f + ((k + 128) % N));
                __builtin_amdgcn_sched_barrier(0);
                acc = grp_add(acc, c);
            }
        }
        t1 = __builtin_amdgcn_s_memtime();
        out[lane] = acc;
        if (lane == 0) cyc[mode] = t1 - t0;
    }
}

int main() {
    float *in, *out;
    long long* cyc;
    hipMalloc(&in, 7 * N * sizeof(float));
    hipMalloc(&out, 64 * sizeof(float));
    hipMalloc(&cyc, 8 * sizeof(long long));
    hipMemset(in, 0, 7 * N * sizeof(float));
    const char* names[5] = {"registers", "lds_1ahead", "lds_2ahead", "registers_unrolled256", "lds16_2ahead"};
    for (int rep = 0; rep < 3; ++rep)
        for (int mode = 0; mode < 5; ++mode) {
            chain_kernel<<<1, 64>>>(in, out, cyc, mode);
            hipDeviceSynchronize();
            long long c = 0;
            hipMemcpy(&c, cyc + mode, sizeof(c), hipMemcpyDeviceToHost);
            const int adds = mode == 2 ? (N / 96 + (N % 96 ? 1 : 0)) * 96 : mode == 4 ? (N / 48 + (N % 48 ? 1 : 0)) * 48 : N;
            if (rep == 2) printf("{\"mode\": \"%s\", \"cycles\": %lld, \"cycles_per_add\": %.2f}\n", names[mode], c, (double)c / adds);
        }
    return 0;
}
