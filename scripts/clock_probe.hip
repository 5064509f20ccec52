// clock_probe.hip — sustained clock and MFMA rate of the bare wave loops of
// mfma_probe.hip under a long load (timing only; results are discarded).
//
//   hipcc --offload-arch=gfx950 -O3 scripts/clock_probe.hip -o scripts/clock_probe
//   ./scripts/clock_probe [ms per loop shape, default 400]
//
// Each shape runs back-to-back launches (256 blocks of 512 threads, 2 waves
// per SIMD) for the given time; thread 0 of block 0 stamps s_memtime (shader
// clock) and s_memrealtime (100 MHz) at the start and end of every launch, and
// the last quarter of the launches gives the held clock and TFLOP/s.  Shows
// whether the 16x16x4 loop (conv tiles) and the 32x32x2 loop (SGEMM) hold
// different clocks at the same MFMA occupancy.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int STEPS = 4096;

__device__ __forceinline__ void stamp(unsigned long long* st, int slot) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st[2 * slot] = __builtin_amdgcn_s_memtime();
    st[2 * slot + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

__global__ __launch_bounds__(512, 1) void m16_lds4(float* out, float x, unsigned long long* st) {
  stamp(st, 0);
  __shared__ float lds[32 * 192 + 32 * 144];
  for (int i = threadIdx.x; i < 32 * 336; i += 512) lds[i] = x * i;
  __syncthreads();
  const int lane = threadIdx.x & 63, r16 = lane & 15, q = lane >> 4, wm = threadIdx.x >> 6;
  floatx4 acc[11];
  for (int j = 0; j < 11; ++j) acc[j] = floatx4{0, 0, 0, 0};
  auto frag = [&](int s, float4& a, float4 (&b)[11]) {
    const int kq = (s & 1) * 4 + q;
    a = *reinterpret_cast<const float4*>(lds + kq * 576 + 4 * ((wm * 16 + r16) ^ (s & 1)));
    const float* bp = lds + 32 * 144 + kq * 768 + 4 * r16;
#pragma unroll
    for (int j = 0; j < 11; ++j) b[j] = *reinterpret_cast<const float4*>(bp + 64 * j);
  };
  float4 a0, b0[11], a1, b1[11];
  frag(0, a0, b0);
  auto mm = [&](const float4& a, const float4 (&b)[11]) {
#pragma unroll
    for (int j = 0; j < 11; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b[j].x, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 11; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b[j].y, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 11; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b[j].z, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 11; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b[j].w, acc[j], 0, 0, 0);
  };
  for (int s = 0; s < STEPS / 4; s += 2) {
    frag(s + 1, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    mm(a0, b0);
    frag(s + 2, a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    mm(a1, b1);
  }
  float r = 0;
  for (int j = 0; j < 11; ++j) r += acc[j][0] + acc[j][3];
  out[blockIdx.x * 512 + threadIdx.x] = r;
  stamp(st, 1);
}

__global__ __launch_bounds__(512, 1) void m16_regs(float* out, float x, unsigned long long* st) {
  stamp(st, 0);
  floatx4 acc[11];
  for (int j = 0; j < 11; ++j) acc[j] = floatx4{0, 0, 0, 0};
  float a = x * threadIdx.x, b = x + threadIdx.x;
  for (int s = 0; s < STEPS; ++s) {
#pragma unroll
    for (int j = 0; j < 11; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
  }
  float r = 0;
  for (int j = 0; j < 11; ++j) r += acc[j][0] + acc[j][3];
  out[blockIdx.x * 512 + threadIdx.x] = r;
  stamp(st, 1);
}

__global__ __launch_bounds__(512, 1) void m32_regs(float* out, float x, unsigned long long* st) {
  stamp(st, 0);
  floatx16 acc[8];
  for (int j = 0; j < 8; ++j)
    for (int e = 0; e < 16; ++e) acc[j][e] = 0;
  float a = x * threadIdx.x, b = x + threadIdx.x;
  for (int s = 0; s < STEPS / 2; ++s) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j], 0, 0, 0);
  }
  float r = 0;
  for (int j = 0; j < 8; ++j) r += acc[j][0] + acc[j][15];
  out[blockIdx.x * 512 + threadIdx.x] = r;
  stamp(st, 1);
}

__global__ __launch_bounds__(512, 1) void m32_lds4(float* out, float x, unsigned long long* st) {
  stamp(st, 0);
  __shared__ float lds[32 * 256 * 2];
  for (int i = threadIdx.x; i < 32 * 512; i += 512) lds[i] = x * i;
  __syncthreads();
  const int lane = threadIdx.x & 63, lc = lane & 31, h = lane >> 5, wid = threadIdx.x >> 6;
  const int g = wid >> 2, wq = wid & 3;
  floatx16 acc[8];
  for (int j = 0; j < 8; ++j)
    for (int e = 0; e < 16; ++e) acc[j][e] = 0;
  auto frag = [&](int s, float4 (&a)[4], float4 (&b)[2]) {
    const int gg = s & 3;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a[i] = *reinterpret_cast<const float4*>(lds + ((gg * 2 + h) * 256 + g * 128 + 32 * i + lc) * 4);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      b[j] = *reinterpret_cast<const float4*>(lds + 8192 + ((gg * 2 + h) * 256 + wq * 64 + 32 * j + lc) * 4);
  };
  auto mm = [&](const float4 (&a)[4], const float4 (&b)[2]) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[2 * i + j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][c], b[j][c], acc[2 * i + j], 0, 0, 0);
  };
  float4 a0[4], b0[2], a1[4], b1[2];
  frag(0, a0, b0);
  for (int s = 0; s < STEPS / 8; s += 2) {
    frag(s + 1, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    mm(a0, b0);
    frag(s + 2, a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    mm(a1, b1);
  }
  float r = 0;
  for (int j = 0; j < 8; ++j) r += acc[j][0] + acc[j][15];
  out[blockIdx.x * 512 + threadIdx.x] = r;
  stamp(st, 1);
}

template <class F>
void run(const char* name, F kernel, double flop_per_wave, float* out, unsigned long long* st,
         double run_ms) {
  // time one launch, then size the run
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(kernel, dim3(256), dim3(512), 0, 0, out, 1e-3f, st);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(kernel, dim3(256), dim3(512), 0, 0, out, 1e-3f, st);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float one = 0;
  (void)hipEventElapsedTime(&one, e0, e1);
  const int reps = (int)(run_ms / (one > 0.01f ? one : 0.01f)) + 4, tail = reps / 4;
  for (int r = 0; r < reps - tail; ++r)
    hipLaunchKernelGGL(kernel, dim3(256), dim3(512), 0, 0, out, 1e-3f, st + 4 * r % 4096);
  (void)hipEventRecord(e0, 0);
  for (int r = 0; r < tail; ++r)
    hipLaunchKernelGGL(kernel, dim3(256), dim3(512), 0, 0, out, 1e-3f, st + 4 * (r % 1024));
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const int n = tail < 1024 ? tail : 1024;
  std::vector<unsigned long long> h(4 * n);
  (void)hipMemcpy(h.data(), st, 4 * n * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  double cyc = 0, rt = 0;
  for (int i = 0; i < n; ++i) {
    cyc += (double)(h[4 * i + 2] - h[4 * i]);
    rt += (double)(h[4 * i + 3] - h[4 * i + 1]);
  }
  const double ghz = cyc / (rt * 10.0);  // s_memrealtime: 100 MHz
  const double tf = flop_per_wave * 256 * 8 * tail / (ms * 1e-3) / 1e12;
  printf("{\"kernel\": \"%s\", \"reps\": %d, \"ms_per_launch\": %.4f, \"tflops\": %.1f, \"frac\": %.3f, "
         "\"clock_ghz\": %.3f, \"tflops_per_ghz_frac\": %.3f}\n",
         name, reps, ms / tail, tf, tf / 157.3, ghz, tf / (157.3 * ghz / 2.4));
  fflush(stdout);
}

int main(int argc, char** argv) {
  const double run_ms = argc > 1 ? atof(argv[1]) : 400.0;
  float* out;
  unsigned long long* st;
  if (hipMalloc(&out, 256 * 512 * sizeof(float)) != hipSuccess) return 1;
  if (hipMalloc(&st, 4096 * sizeof(unsigned long long)) != hipSuccess) return 1;
  const double f16 = 2.0 * 16 * 16 * 4 * 11 * STEPS;       // per wave
  const double f32 = 2.0 * 32 * 32 * 2 * 8 * (STEPS / 2);  // per wave
  run("m32_regs", m32_regs, f32, out, st, run_ms);
  run("m16_regs", m16_regs, f16, out, st, run_ms);
  run("m32_lds4", m32_lds4, f32, out, st, run_ms);
  run("m16_lds4", m16_lds4, f16, out, st, run_ms);
  run("m32_regs", m32_regs, f32, out, st, run_ms);
  (void)hipFree(out);
  (void)hipFree(st);
  return 0;
}
