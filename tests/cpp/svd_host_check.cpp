// CPU check of the DEVICE float Umeyama rotation (icp4r_math.hpp, compiled for the host) against the
// oracle's float restatement: the PCL-numerics path must be a bit-exact restatement, so the two
// sources must agree bit for bit on every input (tests/test_abi.py runs this; no GPU needed).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <random>
#include <cstring>
#include "icp4r_math.hpp"
extern "C" void oracle_rot_f32(const float* sigma, float* R);
int main() {
  std::mt19937 g(0); std::normal_distribution<float> nd(0, 100);
  int bad = 0;
  for (int t = 0; t < 2000; ++t) {
    float S[9]; for (auto& v : S) v = nd(g);
    if (t % 4 == 1) { S[6] = S[3] * 0.5f; S[7] = S[4] * 0.5f; S[8] = S[5] * 0.5f; }  // rank-deficient
    if (t % 4 == 2) for (int k = 0; k < 9; ++k) S[k] = (k % 4 == 0 ? 500.0f : 0.0f) + 0.01f * S[k];  // near identity
    if (t % 16 == 3) for (int k = 0; k < 9; ++k) S[k] = (k < 3) ? S[k] : (k < 6 ? 2.0f * S[k - 3] : -S[k - 6]);  // rank 1
    if (t % 16 == 7) for (int k = 0; k < 9; ++k) S[k] = 0.0f;  // rank 0
    icp4r::SvdWorkF w; icp4r::umeyama_rotation_f32(S, w);
    float R[9]; oracle_rot_f32(S, R);
    if (memcmp(R, w.R, 36)) { if (bad < 2) { for (int k=0;k<9;++k) printf("%.9g/%.9g ", w.R[k], R[k]); printf("\n"); } bad++; }
    // the register-resident variant the update's solve runs (static indices, same operations)
    float Rr[9]; icp4r::umeyama_rotation_f32_reg(S, Rr);
    if (memcmp(R, Rr, 36)) { if (bad < 4) { for (int k=0;k<9;++k) printf("%.9g/%.9g ", Rr[k], R[k]); printf(" (reg)\n"); } bad++; }
  }
  printf("host-compiled device SVD (LDS-struct and register variants) vs oracle: %d mismatches of 4000\n", bad);
  return bad != 0;
}
