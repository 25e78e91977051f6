// Which physical CUs (XCC, SE, SH, CU from HW_REG_HW_ID / HW_REG_XCC_ID) run the workgroups of a
// stream created with hipExtStreamCreateWithCUMask, for a few mask shapes — to choose the CU
// partition of run_pairs' pair groups.  Prints one JSON line per mask.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <map>
#include <set>
#include <vector>

__global__ void probe(uint32_t* out, int spin) {
    if (threadIdx.x == 0) {
        out[blockIdx.x * 2] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
        out[blockIdx.x * 2 + 1] = __builtin_amdgcn_s_getreg(20 | (31 << 11));
    }
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)spin) __builtin_amdgcn_s_sleep(2);
}

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

int main() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int nw = (ncu + 31) / 32;
    const int nblk = 4096;
    uint32_t* d = nullptr;
    CK(hipMalloc(&d, nblk * 2 * sizeof(uint32_t)));
    std::vector<uint32_t> h(nblk * 2);
    const char* names[] = {"all", "low_half", "high_half", "even", "odd", "first32", "mod16_lo8"};
    for (int mi = 0; mi < 7; ++mi) {
        std::vector<uint32_t> mask(nw, 0);
        for (int b = 0; b < ncu; ++b) {
            bool on = false;
            switch (mi) {
                case 0: on = true; break;
                case 1: on = b < ncu / 2; break;
                case 2: on = b >= ncu / 2; break;
                case 3: on = (b & 1) == 0; break;
                case 4: on = (b & 1) == 1; break;
                case 5: on = b < 32; break;
                case 6: on = (b % 16) < 8; break;
            }
            if (on) mask[b / 32] |= 1u << (b % 32);
        }
        hipStream_t s;
        CK(hipExtStreamCreateWithCUMask(&s, nw, mask.data()));
        CK(hipMemsetAsync(d, 0xFF, nblk * 2 * sizeof(uint32_t), s));
        probe<<<nblk, 64, 0, s>>>(d, 2000);  // 2000 ticks of the 100 MHz clock: 20 us per workgroup
        CK(hipGetLastError());
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h.data(), d, nblk * 2 * sizeof(uint32_t), hipMemcpyDeviceToHost));
        CK(hipStreamDestroy(s));
        std::set<uint32_t> cus;
        std::map<int, std::set<int>> xcc_of_mod8;
        std::map<int, int> per_xcc;
        for (int b = 0; b < nblk; ++b) {
            const uint32_t hw = h[b * 2], xcc = h[b * 2 + 1] & 0xF;
            const uint32_t cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
            cus.insert((xcc << 16) | (se << 8) | (sh << 4) | cu);
            xcc_of_mod8[b % 8].insert((int)xcc);
            per_xcc[(int)xcc]++;
        }
        printf("{\"mask\": \"%s\", \"distinct_cus\": %zu, \"wg_per_xcc\": {", names[mi], cus.size());
        bool first = true;
        for (auto& kv : per_xcc) {
            printf("%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second);
            first = false;
        }
        printf("}, \"xccs_of_block_mod8\": [");
        for (int r = 0; r < 8; ++r) {
            printf("%s[", r ? ", " : "");
            bool f2 = true;
            for (int x : xcc_of_mod8[r]) {
                printf("%s%d", f2 ? "" : ", ", x);
                f2 = false;
            }
            printf("]");
        }
        printf("], \"cus\": [");
        first = true;
        for (uint32_t c : cus) {
            printf("%s\"%u.%u.%u.%u\"", first ? "" : ", ", c >> 16, (c >> 8) & 7, (c >> 4) & 1, c & 15);
            first = false;
        }
        printf("]}\n");
        fflush(stdout);
    }
    CK(hipFree(d));
    return 0;
}
