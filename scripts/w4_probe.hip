// w4_probe.hip — the wave loop of sgemm_nn_w4.hip in isolation (timing only;
// results discarded): one wave per SIMD (256-thread blocks, one per CU, 256
// blocks), wave tile 128 x 128 = 4 x 4 v_mfma_f32_32x32x2_f32 accumulators,
// operands from the kernel's own LDS images (A: 256 rows x 32 k, 16-byte
// k-chunks XOR-swizzled by (row >> 1) & 7; B: 32 k-rows x 256 columns with
// interleaved columns, rotated by 32 floats on odd k).
//
//   w4_b32   A by 4 ds_read_b32 per step (the product kernel's reads)
//   w4_b128  A by one ds_read_b128 per tile and step PAIR: the lane's 16-byte
//            chunk holds k = 4j .. 4j+3 of its row; step 2j takes component
//            h, step 2j+1 component 2+h (the other two are the partner
//            half's) — 2 A reads per step instead of 4, conflict-free
//   w4_read2 A by one ds_read2_b32 per tile and step pair (offsets 0 and 2
//            from the lane's k = 4j + h): half the A read instructions
//   w4_regs  operands in registers (the MFMA ceiling of the shape)
//
//   hipcc --offload-arch=gfx950 -O3 scripts/w4_probe.hip -o scripts/w4_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int STEPS = 4096;  // MFMA steps (k pairs) per wave
constexpr int BK = 32;

template <int MODE>
__global__ __launch_bounds__(256, 1) void w4_loop(float* out, float x) {
  __shared__ __attribute__((aligned(16))) float lds[256 * 32 + 32 * 256];
  for (int i = threadIdx.x; i < 256 * 32 + 32 * 256; i += 256) lds[i] = x * (i & 1023);
  __syncthreads();
  const int lane = threadIdx.x & 63, lc = lane & 31, h = lane >> 5, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  floatx16 acc[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) asm volatile("" : "+a"(acc[i][j]));
  const int swz = (lc >> 1) & 7;
  const int a_lane = (wm * 128 + lc) * BK + h;
  const int a_row = (wm * 128 + lc) * BK;
  const int b_col = 256 * 32 + h * 256 + ((wn * 128 + 4 * lc - 32 * h) & 255);
  auto mma = [&](const float (&a)[4], const float (&b)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
  };
  auto bfr = [&](int s, float (&b)[4]) {
    const floatx4 v = *reinterpret_cast<const floatx4*>(lds + b_col + 2 * (s & 15) * 256);
    b[0] = v[0]; b[1] = v[1]; b[2] = v[2]; b[3] = v[3];
  };
  if constexpr (MODE == 2) {
    float a[4] = {x, x + 1, x + 2, x + 3}, b[4] = {x, x * 2, x * 3, x * 4};
    for (int s = 0; s < STEPS; ++s) mma(a, b);
  } else if constexpr (MODE == 0) {
    auto frag = [&](int s, float (&a)[4], float (&b)[4]) {
      const int ss = s & 15;
      const int ka = 4 * ((ss >> 1) ^ swz) + 2 * (ss & 1);
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = lds[a_lane + 32 * BK * i + ka];
      bfr(s, b);
    };
    float a0[4], b0[4], a1[4], b1[4];
    frag(0, a0, b0);
    for (int s = 0; s < STEPS; s += 2) {
      frag(s + 1, a1, b1);
      __builtin_amdgcn_sched_barrier(0);
      mma(a0, b0);
      frag(s + 2, a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      mma(a1, b1);
    }
  } else if constexpr (MODE == 3) {
    // step pair j = s/2: one ds_read2_b32 per tile (the lane's k = 4j + h
    // and 4j + 2 + h: offsets 0 and 2 dwords from its own base)
    auto fragA = [&](int s, float (&ae)[4], float (&ao)[4]) {
      const int j = (s >> 1) & 7;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float* p = lds + a_row + 32 * BK * i + 4 * (j ^ swz) + h;
        ae[i] = p[0];
        ao[i] = p[2];
      }
    };
    float E0[4], O0[4], E1[4], O1[4];
    float b0[4], b1[4], b2[4], b3[4];
    fragA(0, E0, O0);
    bfr(0, b0);
    bfr(1, b1);
    for (int s = 0; s < STEPS; s += 4) {
      fragA(s + 2, E1, O1);
      bfr(s + 2, b2);
      __builtin_amdgcn_sched_barrier(0);
      mma(E0, b0);
      bfr(s + 3, b3);
      __builtin_amdgcn_sched_barrier(0);
      mma(O0, b1);
      fragA(s + 4, E0, O0);
      bfr(s + 4, b0);
      __builtin_amdgcn_sched_barrier(0);
      mma(E1, b2);
      bfr(s + 5, b1);
      __builtin_amdgcn_sched_barrier(0);
      mma(O1, b3);
    }
  } else {
    // step pair j = s/2: one b128 per tile
    auto fragA = [&](int s, floatx4 (&a)[4]) {
      const int j = (s >> 1) & 7;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i] = *reinterpret_cast<const floatx4*>(lds + a_row + 32 * BK * i + 4 * (j ^ swz));
    };
    floatx4 A0[4], A1[4];
    float b0[4], b1[4], b2[4], b3[4];
    fragA(0, A0);
    bfr(0, b0);
    bfr(1, b1);
    for (int s = 0; s < STEPS; s += 4) {
      fragA(s + 2, A1);
      bfr(s + 2, b2);
      __builtin_amdgcn_sched_barrier(0);
      {
        float a[4], c[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) { a[i] = h ? A0[i][1] : A0[i][0]; c[i] = h ? A0[i][3] : A0[i][2]; }
        mma(a, b0);
        bfr(s + 3, b3);
        __builtin_amdgcn_sched_barrier(0);
        mma(c, b1);
      }
      fragA(s + 4, A0);
      bfr(s + 4, b0);
      __builtin_amdgcn_sched_barrier(0);
      {
        float a[4], c[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) { a[i] = h ? A1[i][1] : A1[i][0]; c[i] = h ? A1[i][3] : A1[i][2]; }
        mma(a, b2);
        bfr(s + 5, b1);
        __builtin_amdgcn_sched_barrier(0);
        mma(c, b3);
      }
    }
  }
  float r = 0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) r += acc[i][j][0] + acc[i][j][15];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <class F>
void run(const char* name, F kernel, float* out) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int w = 0; w < 5; ++w) hipLaunchKernelGGL(kernel, dim3(256), dim3(256), 0, 0, out, 1e-3f);
  (void)hipEventRecord(e0, 0);
  const int reps = 20;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kernel, dim3(256), dim3(256), 0, 0, out, 1e-3f);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flop = 2.0 * 128 * 128 * 2 * STEPS * 4 * 256;  // per launch
  const double tf = flop * reps / (ms * 1e-3) / 1e12;
  printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"tflops\": %.1f, \"frac\": %.3f}\n", name, ms / reps, tf,
         tf / 157.3);
}

int main() {
  float* out;
  if (hipMalloc(&out, 256 * 256 * sizeof(float)) != hipSuccess) return 1;
  for (int rep = 0; rep < 2; ++rep) {
    run("w4_regs", w4_loop<2>, out);
    run("w4_b32", w4_loop<0>, out);
    run("w4_b128", w4_loop<1>, out);
    run("w4_read2", w4_loop<3>, out);
  }
  (void)hipFree(out);
  return 0;
}
