// Microbenchmark: the gap between dependent kernels on one stream, plain launches vs a hipGraph.
//   hipcc -O3 --offload-arch=gfx950 -o _var/launch_gap tools/experiments/launch_gap.hip
// K kernels in a chain (each reads the previous one's value): tiny (1 workgroup) and "dirty" (each
// also streams 32 MB of stores, so the L2 holds dirty lines at every kernel boundary).  Prints the
// time per kernel for plain stream launches and for the same chain captured once and replayed.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void step_kernel(int* v, float* big, long long nbig) {
    if (blockIdx.x == 0 && threadIdx.x == 0) v[0] = v[0] + 1;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nbig; i += (long long)gridDim.x * blockDim.x)
        big[i] = (float)i;
}

int main() {
    const int K = 200;
    int* v;
    float* big;
    const long long nbig = 8ll << 20;  // 32 MB
    hipMalloc(&v, 4);
    hipMalloc(&big, nbig * 4);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int dirty = 0; dirty < 2; ++dirty) {
        const int grid = dirty ? 1024 : 1;
        const long long nb = dirty ? nbig : 0;
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a, s);
            for (int k = 0; k < K; ++k) step_kernel<<<grid, 256, 0, s>>>(v, big, nb);
            hipEventRecord(b, s);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (rep) printf("{\"mode\": \"stream\", \"dirty\": %d, \"us_per_kernel\": %.2f}\n", dirty, ms * 1e3 / K);
        }
        hipGraph_t g;
        hipGraphExec_t ge;
        hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
        for (int k = 0; k < K; ++k) step_kernel<<<grid, 256, 0, s>>>(v, big, nb);
        hipStreamEndCapture(s, &g);
        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a, s);
            hipGraphLaunch(ge, s);
            hipEventRecord(b, s);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (rep) printf("{\"mode\": \"graph\", \"dirty\": %d, \"us_per_kernel\": %.2f}\n", dirty, ms * 1e3 / K);
        }
        hipGraphExecDestroy(ge);
        hipGraphDestroy(g);
    }
    // the stores alone (one kernel writing 32 MB K times in one launch is not the same; report the
    // single dirty kernel's duration for reference)
    hipEventRecord(a, s);
    step_kernel<<<1024, 256, 0, s>>>(v, big, nbig);
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("{\"mode\": \"single_dirty_kernel\", \"us\": %.2f}\n", ms * 1e3);
    return 0;
}
