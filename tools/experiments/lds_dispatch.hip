// Microbenchmark: what a dependent kernel launch costs by its shape (round 6, the single-pair search's
// ~5 us outside its workgroups).  A chain alternates an "update"-like kernel (1 workgroup of 1024
// threads, 130 KB of LDS) with a "search"-like kernel of G workgroups x T threads and L bytes of LDS;
// each kernel writes a little, touches its LDS and spins ~2 us.  Prints the chain's time per pair of
// kernels for each search shape (HIP events around 200 pairs).
//   hipcc -O3 --offload-arch=gfx950 -o _var/lds_dispatch tools/experiments/lds_dispatch.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int T, int L>
__global__ __launch_bounds__(T) void body_kernel(int* v, int spin) {
    extern __shared__ int lds[];
    __shared__ int fixed[L / 4];
    fixed[threadIdx.x % (L / 4)] = threadIdx.x;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin) {
    }
    if (threadIdx.x == 0) v[blockIdx.x] = fixed[(blockIdx.x + 1) % (L / 4)] + v[blockIdx.x];
}

struct Big {  // a kernel argument block the size of icp4r's PairArgs + WorkArgs
    long long f[96];
};
template <int T, int L>
__global__ __launch_bounds__(T) void big_kernel(Big b, int* v, int spin) {
    __shared__ int fixed[L / 4];
    fixed[threadIdx.x % (L / 4)] = threadIdx.x;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin) {
    }
    if (threadIdx.x == 0) v[blockIdx.x] = fixed[(blockIdx.x + 1) % (L / 4)] + v[blockIdx.x] + (int)b.f[blockIdx.x % 96];
}

int main() {
    int* v;
    hipMalloc(&v, 1 << 20);
    hipMemset(v, 0, 1 << 20);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int K = 200, spin = 200;  // 2 us of 100 MHz ticks
    auto run = [&](const char* name, auto launch_b) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a, s);
            for (int k = 0; k < K; ++k) {
                hipLaunchKernelGGL((body_kernel<1024, 130 * 1024>), dim3(1), dim3(1024), 0, s, v, spin);
                launch_b();
            }
            hipEventRecord(b, s);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (rep) printf("%-44s %.2f us per pair (update-like + search-like, 2 x 2 us of body)\n", name, ms * 1e3 / K);
        }
    };
    run("search 16 x 1024 thr, 155 KB LDS", [&] {
        hipLaunchKernelGGL((body_kernel<1024, 155 * 1024>), dim3(16), dim3(1024), 0, s, v, spin);
    });
    run("search 16 x 1024 thr, 40 KB LDS", [&] {
        hipLaunchKernelGGL((body_kernel<1024, 40 * 1024>), dim3(16), dim3(1024), 0, s, v, spin);
    });
    run("search 1 x 1024 thr, 155 KB LDS", [&] {
        hipLaunchKernelGGL((body_kernel<1024, 155 * 1024>), dim3(1), dim3(1024), 0, s, v, spin);
    });
    run("search 16 x 256 thr, 40 KB LDS", [&] {
        hipLaunchKernelGGL((body_kernel<256, 40 * 1024>), dim3(16), dim3(256), 0, s, v, spin);
    });
    run("search 64 x 256 thr, 40 KB LDS", [&] {
        hipLaunchKernelGGL((body_kernel<256, 40 * 1024>), dim3(64), dim3(256), 0, s, v, spin);
    });
    run("no search (update-like only)", [&] {});
    Big big = {};
    for (int k = 0; k < 96; ++k) big.f[k] = k;
    run("search 16 x 1024 thr, 155 KB LDS, 768-B args", [&] {
        hipLaunchKernelGGL((big_kernel<1024, 155 * 1024>), dim3(16), dim3(1024), 0, s, big, v, spin);
    });
    run("search 1 x 64 thr, 4 KB LDS, 768-B args", [&] {
        hipLaunchKernelGGL((big_kernel<64, 4 * 1024>), dim3(1), dim3(64), 0, s, big, v, spin);
    });
    return 0;
}
