// chain_probe.hip — cycles per dependent v_add_f32 in one wave (the batch-norm
// reductions' lane chains: each of the reference's 8 AVX lanes is a strictly
// sequential add chain).  Timing only; results discarded.
//
//   hipcc --offload-arch=gfx950 -O3 scripts/chain_probe.hip -o scripts/chain_probe
//
// one 64-thread block; L active lanes run a chain of STEPS dependent adds
// (C chains interleaved per lane); cycles by s_memtime around the loop.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int STEPS = 1 << 16;

template <int C>
__global__ void chain(float* out, unsigned long long* cyc, int lanes, float x) {
  const int l = threadIdx.x;
  float acc[C];
  for (int c = 0; c < C; ++c) acc[c] = 0.f;
  float v0 = x * l, v1 = x + l, v2 = x - l, v3 = x * 0.5f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (l < lanes) {
    for (int s = 0; s < STEPS; s += 4) {
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = acc[c] + v0;
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = acc[c] + v1;
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = acc[c] + v2;
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = acc[c] + v3;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float r = 0;
  for (int c = 0; c < C; ++c) r += acc[c];
  out[l] = r;
  if (l == 0) cyc[0] = t1 - t0;
}

int main() {
  float* out;
  unsigned long long* cyc;
  if (hipMalloc(&out, 64 * sizeof(float)) != hipSuccess) return 1;
  if (hipMalloc(&cyc, sizeof(unsigned long long)) != hipSuccess) return 1;
  auto run = [&](const char* name, auto kern, int lanes, int chains) {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, out, cyc, lanes, 1e-3f);
    unsigned long long c = 0;
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("{\"kernel\": \"%s\", \"lanes\": %d, \"chains_per_lane\": %d, \"cycles_per_dependent_add\": %.2f}\n",
           name, lanes, chains, (double)c / STEPS);
  };
  run("chain1", chain<1>, 8, 1);
  run("chain1", chain<1>, 16, 1);
  run("chain1", chain<1>, 64, 1);
  run("chain2", chain<2>, 8, 2);
  run("chain4", chain<4>, 8, 4);
  (void)hipFree(out);
  (void)hipFree(cyc);
  return 0;
}
