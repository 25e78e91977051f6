// CPU check of the DEVICE float Umeyama rotation (icp4r_math.hpp: Eigen 3.3's JacobiSVD<Matrix3f> +
// umeyama, compiled for the host) against the oracle's float restatement (oracle/icp_oracle.c rot_f32):
// the PCL-numerics path must be a bit-exact restatement, so the two sources must agree bit for bit on
// every input (tests/test_abi.py runs this; no GPU needed).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <random>
#include <cstring>
#include "icp4r_math.hpp"
extern "C" void oracle_rot_f32(const float* sigma, float* R);
int main() {
  std::mt19937 g(0); std::normal_distribution<float> nd(0, 100);
  std::uniform_real_distribution<float> ang(-0.2f, 0.2f), ex(-20.0f, 20.0f);
  int bad = 0, n = 0;
  for (int t = 0; t < 4000; ++t) {
    float S[9]; for (auto& v : S) v = nd(g);
    if (t % 4 == 1) { S[6] = S[3] * 0.5f; S[7] = S[4] * 0.5f; S[8] = S[5] * 0.5f; }  // rank-deficient
    if (t % 4 == 2) for (int k = 0; k < 9; ++k) S[k] = (k % 4 == 0 ? 500.0f : 0.0f) + 0.01f * S[k];  // near identity
    if (t % 16 == 3) for (int k = 0; k < 9; ++k) S[k] = (k < 3) ? S[k] : (k < 6 ? 2.0f * S[k - 3] : -S[k - 6]);  // rank 1
    if (t % 16 == 7) for (int k = 0; k < 9; ++k) S[k] = 0.0f;  // rank 0
    if (t % 16 == 11) {  // ICP-like: a small rotation times a flat (radar) spread, wide dynamic range
      const float a = ang(g), c = cosf(a), s = sinf(a), sx = 400.0f, sy = 90.0f, sz = 0.5f * (1 + t % 3);
      const float M[9] = {c * sx, -s * sy, 0.01f * sz, s * sx, c * sy, -0.02f * sz, 0.001f * sx, 0.003f * sy, sz};
      for (int k = 0; k < 9; ++k) S[k] = M[k];
    }
    if (t % 16 == 15) for (int k = 0; k < 9; ++k) S[k] = S[k] * ldexpf(1.0f, (int)ex(g));  // scaled
    if (t % 32 == 5) { S[1] = S[3]; S[2] = S[6]; S[5] = S[7]; }  // symmetric
    if (t % 32 == 21) { for (int k = 0; k < 9; ++k) S[k] = 0.0f; S[0] = 3.0f; S[4] = -2.0f; S[8] = 1.0f; }  // diagonal, signs
    float R[9]; oracle_rot_f32(S, R);
    float Rr[9]; icp4r::umeyama_rotation_f32_reg(S, Rr);
    ++n;
    if (memcmp(R, Rr, 36)) { if (bad < 4) { for (int k=0;k<9;++k) printf("%.9g/%.9g ", Rr[k], R[k]); printf("\n"); } bad++; }
  }
  printf("host-compiled device SVD (Eigen JacobiSVD restatement) vs oracle: %d mismatches of %d\n", bad, n);
  return bad != 0;
}
