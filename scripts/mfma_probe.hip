// mfma_probe.hip — sustained fp32 MFMA rate of the loop shapes the conv and
// dW kernels use (timing only; results are discarded).
//
//   hipcc --offload-arch=gfx950 -O3 scripts/mfma_probe.hip -o scripts/mfma_probe
//   ./scripts/mfma_probe
//
// Every kernel runs 2 waves per SIMD (512-thread blocks, one per CU, 256
// blocks) and reports TFLOP/s against the 157.3 TF fp32 MFMA peak:
//   m16_regs    11 independent v_mfma_f32_16x16x4_f32 per step, operands in
//               registers (no LDS)
//   m16_lds     the same with each step's 12 operands read from LDS by
//               ds_read_b32 one step ahead (conv_tile's 128x176 wave loop)
//   m32_regs    8 independent v_mfma_f32_32x32x2_f32 per step, registers
//   m32_lds     the same with one ds_read_b128 + two ds_read_b32 per step
//               (the 256x256 SGEMM wave loop)
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int STEPS = 4096;

__global__ __launch_bounds__(512, 1) void m16_regs(float* out, float x) {
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
}

__global__ __launch_bounds__(512, 1) void m16_lds(float* out, float x) {
  __shared__ float lds[32 * 192 + 32 * 144];
  for (int i = threadIdx.x; i < 32 * 336; i += 512) lds[i] = x * i;
  __syncthreads();
  const int lane = threadIdx.x & 63, r16 = lane & 15, q = lane >> 4, wm = threadIdx.x >> 6;
  floatx4 acc[11];
  for (int j = 0; j < 11; ++j) acc[j] = floatx4{0, 0, 0, 0};
  auto frag = [&](int s, float& a, float (&b)[11]) {
    const int k = 4 * (s & 7) + q;
    a = lds[k * 144 + ((wm * 16 + r16) ^ ((s & 7) << 2))];
    const float* bp = lds + 32 * 144 + k * 192 + r16;
#pragma unroll
    for (int j = 0; j < 11; ++j) b[j] = bp[16 * j];
  };
  float a0, b0[11], a1, b1[11];
  frag(0, a0, b0);
  for (int s = 0; s < STEPS; s += 2) {
    frag(s + 1, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 11; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0[j], acc[j], 0, 0, 0);
    frag(s + 2, a0, b0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 11; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1[j], acc[j], 0, 0, 0);
  }
  float r = 0;
  for (int j = 0; j < 11; ++j) r += acc[j][0] + acc[j][3];
  out[blockIdx.x * 512 + threadIdx.x] = r;
}

__global__ __launch_bounds__(512, 1) void m32_regs(float* out, float x) {
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
}

__global__ __launch_bounds__(512, 1) void m32_lds(float* out, float x) {
  __shared__ float lds[32 * 256 * 2];
  for (int i = threadIdx.x; i < 32 * 512; i += 512) lds[i] = x * i;
  __syncthreads();
  const int lane = threadIdx.x & 63, lc = lane & 31, h = lane >> 5, wid = threadIdx.x >> 6;
  const int g = wid >> 2, wq = wid & 3;
  floatx16 acc[8];
  for (int j = 0; j < 8; ++j)
    for (int e = 0; e < 16; ++e) acc[j][e] = 0;
  auto frag = [&](int s, float (&a)[4], float (&b)[2]) {
    const int k = 2 * (s & 15) + h;
    const float4 v = *reinterpret_cast<const float4*>(lds + k * 256 + ((g * 128 + 4 * lc) ^ (((k >> 2) & 3) << 3)));
    a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
    const float* bp = lds + 32 * 256 + k * 256 + wq * 64 + lc;
    b[0] = bp[0];
    b[1] = bp[32];
  };
  float a0[4], b0[2], a1[4], b1[2];
  frag(0, a0, b0);
  for (int s = 0; s < STEPS / 2; s += 2) {
    frag(s + 1, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[2 * i + j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[i], b0[j], acc[2 * i + j], 0, 0, 0);
    frag(s + 2, a0, b0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[2 * i + j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[i], b1[j], acc[2 * i + j], 0, 0, 0);
  }
  float r = 0;
  for (int j = 0; j < 8; ++j) r += acc[j][0] + acc[j][15];
  out[blockIdx.x * 512 + threadIdx.x] = r;
}


// m16_lds4: conv_tile's wave loop with k-permuted LDS images: one
// ds_read_b128 per operand fragment feeds 4 MFMA steps (12 reads per 44 MFMAs)
__global__ __launch_bounds__(512, 1) void m16_lds4(float* out, float x) {
  __shared__ float lds[32 * 192 + 32 * 144];
  for (int i = threadIdx.x; i < 32 * 336; i += 512) lds[i] = x * i;
  __syncthreads();
  const int lane = threadIdx.x & 63, r16 = lane & 15, q = lane >> 4, wm = threadIdx.x >> 6;
  floatx4 acc[11];
  for (int j = 0; j < 11; ++j) acc[j] = floatx4{0, 0, 0, 0};
  auto frag = [&](int s, float4& a, float4 (&b)[11]) {
    const int kq = (s & 1) * 4 + q;  // k-quad row
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
}


// m32_lds4: the 256x256 SGEMM wave loop (wave tile 128 x 64 = 4 x 2 32x32x2
// accumulators) with k-permuted slots: per 4 MFMA steps one ds_read_b128 per
// A fragment (4) and per B fragment (2), 6 reads per 32 MFMAs (vs 12)
__global__ __launch_bounds__(512, 1) void m32_lds4(float* out, float x) {
  __shared__ float lds[32 * 256 * 2];
  for (int i = threadIdx.x; i < 32 * 512; i += 512) lds[i] = x * i;
  __syncthreads();
  const int lane = threadIdx.x & 63, lc = lane & 31, h = lane >> 5, wid = threadIdx.x >> 6;
  const int g = wid >> 2, wq = wid & 3;
  floatx16 acc[8];
  for (int j = 0; j < 8; ++j)
    for (int e = 0; e < 16; ++e) acc[j][e] = 0;
  // slot images [group][h][row] of 16 bytes: A 256 rows, B 256 columns
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
}

template <class F>
void run(const char* name, F kernel, double flop_per_wave, float* out) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kernel, dim3(256), dim3(512), 0, 0, out, 1e-3f);
  (void)hipEventRecord(e0, 0);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kernel, dim3(256), dim3(512), 0, 0, out, 1e-3f);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double tf = flop_per_wave * 256 * 8 * reps / (ms * 1e-3) / 1e12;
  printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"tflops\": %.1f, \"frac\": %.3f}\n", name, ms / reps, tf,
         tf / 157.3);
}

int main() {
  float* out;
  if (hipMalloc(&out, 256 * 512 * sizeof(float)) != hipSuccess) return 1;
  const double f16 = 2.0 * 16 * 16 * 4 * 11 * STEPS;          // per wave
  const double f32 = 2.0 * 32 * 32 * 2 * 8 * (STEPS / 2);     // per wave
  run("m16_regs", m16_regs, f16, out);
  run("m16_lds", m16_lds, f16, out);
  run("m16_lds4", m16_lds4, f16, out);
  run("m32_regs", m32_regs, f32, out);
  run("m32_lds", m32_lds, f32, out);
  run("m32_lds4", m32_lds4, f32, out);
  (void)hipFree(out);
  return 0;
}
