// mfma_order.hip — probe: is v_mfma_f32_16x16x4_f32 bit-identical to an
// ascending-k fmaf chain (lane group q = l/16 holding k = q)?  Also re-checks
// v_mfma_f32_32x32x2_f32 (lane half h = k).  Prints mismatch counts for the
// candidate orders.  Build: hipcc --offload-arch=gfx950 -O2 mfma_order.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// T trials of a 16x16x(4*S) product, one wave per trial
__global__ void k16(const float* A, const float* B, const float* C0, float* D, int S) {
  const int t = blockIdx.x, l = threadIdx.x;
  const float* a = A + t * 16 * 4 * S;  // A[m][k], k = 4s+q
  const float* b = B + t * 4 * S * 16;  // B[k][n]
  floatx4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = C0[t * 256 + (4 * (l / 16) + r) * 16 + l % 16];
  for (int s = 0; s < S; ++s) {
    const int k = 4 * s + l / 16;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[(l % 16) * 4 * S + k], b[k * 16 + l % 16], acc, 0,
                                               0, 0);
  }
  for (int r = 0; r < 4; ++r) D[t * 256 + (4 * (l / 16) + r) * 16 + l % 16] = acc[r];
}
__global__ void k32(const float* A, const float* B, const float* C0, float* D, int S) {
  const int t = blockIdx.x, l = threadIdx.x;
  const float* a = A + t * 32 * 2 * S;
  const float* b = B + t * 2 * S * 32;
  floatx16 acc;
  for (int e = 0; e < 16; ++e)
    acc[e] = C0[t * 1024 + (8 * (e >> 2) + 4 * (l / 32) + (e & 3)) * 32 + l % 32];
  for (int s = 0; s < S; ++s) {
    const int k = 2 * s + l / 32;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[(l % 32) * 2 * S + k], b[k * 32 + l % 32], acc, 0,
                                               0, 0);
  }
  for (int e = 0; e < 16; ++e)
    D[t * 1024 + (8 * (e >> 2) + 4 * (l / 32) + (e & 3)) * 32 + l % 32] = acc[e];
}

static float rnd(unsigned& s) {
  s = s * 1664525u + 1013904223u;
  float u = ((s >> 8) & 0xffff) / 65536.0f * 2.0f - 1.0f;
  int e = (int)((s >> 24) % 24) - 12;  // wide dynamic range exposes order
  return std::ldexp(u, e);
}

int main() {
  const int T = 64, S = 8;
  for (int shape = 0; shape < 2; ++shape) {
    const int MN = shape == 0 ? 16 : 32, KS = shape == 0 ? 4 : 2, K = KS * S;
    std::vector<float> A(T * MN * K), B(T * K * MN), C0(T * MN * MN), D(T * MN * MN);
    unsigned sd = 12345 + shape;
    for (auto& v : A) v = rnd(sd);
    for (auto& v : B) v = rnd(sd);
    for (auto& v : C0) v = rnd(sd);
    float *dA, *dB, *dC, *dD;
    hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4);
    hipMalloc(&dC, C0.size() * 4); hipMalloc(&dD, D.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dC, C0.data(), C0.size() * 4, hipMemcpyHostToDevice);
    if (shape == 0) hipLaunchKernelGGL(k16, dim3(T), dim3(64), 0, 0, dA, dB, dC, dD, S);
    else hipLaunchKernelGGL(k32, dim3(T), dim3(64), 0, 0, dA, dB, dC, dD, S);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    // candidate orders: 0 ascending fma chain; 1 descending within the
    // instruction; 2 pairwise tree within the instruction, fma into C
    long bad[3] = {0, 0, 0};
    double maxrel = 0;
    for (int t = 0; t < T; ++t)
      for (int i = 0; i < MN; ++i)
        for (int j = 0; j < MN; ++j) {
          const float* a = &A[t * MN * K + i * K];
          float c[3];
          for (int o = 0; o < 3; ++o) c[o] = C0[t * MN * MN + i * MN + j];
          double exact = c[0];
          for (int s = 0; s < S; ++s) {
            for (int q = 0; q < KS; ++q) {
              const int k = KS * s + q;
              c[0] = std::fmaf(a[k], B[t * K * MN + k * MN + j], c[0]);
              exact += (double)a[k] * B[t * K * MN + k * MN + j];
            }
            for (int q = KS - 1; q >= 0; --q) {
              const int k = KS * s + q;
              c[1] = std::fmaf(a[k], B[t * K * MN + k * MN + j], c[1]);
            }
            float p = 0;
            for (int q = 0; q < KS; ++q) p += a[KS * s + q] * B[t * K * MN + (KS * s + q) * MN + j];
            c[2] = c[2] + p;
          }
          const float got = D[t * MN * MN + i * MN + j];
          for (int o = 0; o < 3; ++o) bad[o] += std::memcmp(&got, &c[o], 4) != 0;
          maxrel = std::fmax(maxrel, std::fabs(got - exact) / (std::fabs(exact) + 1e-30));
        }
    printf("%s: mismatches asc=%ld desc=%ld tree=%ld of %d, max rel vs fp64 %.3g\n",
           shape == 0 ? "16x16x4f32" : "32x32x2f32", bad[0], bad[1], bad[2], T * MN * MN, maxrel);
  }
  return 0;
}
