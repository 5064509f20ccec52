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

// ring: the same chain fed from LDS the way block_chains_ws feeds it (rows
// of 768 terms, groups of 16 read by four ds_read_b128 three groups ahead,
// s_waitcnt lgkmcnt(8) before each group), no other wave on the CU
constexpr int RLDT = 840, RTERMS = 768, RREPS = 64;
__global__ void ring(float* out, unsigned long long* cyc, int lanes, float x) {
  __shared__ __attribute__((aligned(16))) float U[8 * RLDT];
  const int l = threadIdx.x;
  for (int i = l; i < 8 * RLDT; i += 64) U[i] = x * (float)(i & 7);
  __syncthreads();
  typedef float f4 __attribute__((ext_vector_type(4)));
  float acc = 0.f;
  const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const float*)(U + (l & 7) * RLDT);
  auto rd = [&](int q, f4 (&v)[4]) {
    const unsigned a = base + 4u * (unsigned)q;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v[0]) : "v"(a));
    asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(v[1]) : "v"(a));
    asm volatile("ds_read_b128 %0, %1 offset:32" : "=v"(v[2]) : "v"(a));
    asm volatile("ds_read_b128 %0, %1 offset:48" : "=v"(v[3]) : "v"(a));
  };
  auto wait8 = [&](f4 (&v)[4]) {
    asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
  };
  auto add16 = [&](const f4 (&v)[4]) {
#pragma unroll
    for (int z = 0; z < 16; ++z) acc = acc + v[z >> 2][z & 3];
  };
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (l < lanes) {
    for (int r = 0; r < RREPS; ++r) {
      f4 va[4], vb[4], vc[4];
      rd(0, va);
      rd(16, vb);
      rd(32, vc);
      for (int q = 0; q < RTERMS; q += 48) {
        wait8(va);
        add16(va);
        rd((q + 48) % RTERMS, va);
        wait8(vb);
        add16(vb);
        rd((q + 64) % RTERMS, vb);
        wait8(vc);
        add16(vc);
        rd((q + 80) % RTERMS, vc);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(va[0]), "+v"(va[1]), "+v"(va[2]), "+v"(va[3]),
                   "+v"(vb[0]), "+v"(vb[1]), "+v"(vb[2]), "+v"(vb[3]), "+v"(vc[0]), "+v"(vc[1]),
                   "+v"(vc[2]), "+v"(vc[3]));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = acc;
  if (l == 0) cyc[0] = t1 - t0;
}

// ring16: lanes 8..15 read the chain lanes' next four terms of every group
// (one ds_read_b128 carries 8 terms of each chain), handed over by a DPP
// row_ror:8 move off the chain: twice the terms in flight per LDS
// instruction for four extra (independent) VALU moves per 8 adds
__global__ void ring16(float* out, unsigned long long* cyc, int lanes, float x) {
  __shared__ __attribute__((aligned(16))) float U[8 * RLDT];
  const int l = threadIdx.x;
  for (int i = l; i < 8 * RLDT; i += 64) U[i] = x * (float)(i & 7);
  __syncthreads();
  typedef float f4 __attribute__((ext_vector_type(4)));
  float acc = 0.f;
  const int half = (l >> 3) & 1;
  const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const float*)(U + (l & 7) * RLDT) + 16u * half;
  // group of 16 terms: lane l reads q..q+3 and q+8..q+11, lane l+8 reads
  // q+4..q+7 and q+12..q+15
  auto rd = [&](int q, f4 (&v)[2]) {
    const unsigned a = base + 4u * (unsigned)q;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v[0]) : "v"(a));
    asm volatile("ds_read_b128 %0, %1 offset:32" : "=v"(v[1]) : "v"(a));
  };
  auto wait = [&](f4 (&v)[2]) {
    asm volatile("s_waitcnt lgkmcnt(10)" : "+v"(v[0]), "+v"(v[1]));
  };
  auto add16 = [&](const f4 (&v)[2]) {
    float o[8];
#pragma unroll
    for (int z = 0; z < 8; ++z)
      o[z] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                 0, __builtin_bit_cast(int, (float)v[z >> 2][z & 3]), 0x128, 0xf, 0xf, false));
    // (the moves stay moves: folded into the adds as DPP operands they would
    // sit on the chain)
    asm volatile("" : "+v"(o[0]), "+v"(o[1]), "+v"(o[2]), "+v"(o[3]), "+v"(o[4]), "+v"(o[5]),
                 "+v"(o[6]), "+v"(o[7]));
#pragma unroll
    for (int z = 0; z < 4; ++z) acc = acc + v[0][z];
#pragma unroll
    for (int z = 0; z < 4; ++z) acc = acc + o[z];
#pragma unroll
    for (int z = 0; z < 4; ++z) acc = acc + v[1][z];
#pragma unroll
    for (int z = 0; z < 4; ++z) acc = acc + o[4 + z];
  };
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (l < 16) {
    for (int r = 0; r < RREPS; ++r) {
      f4 g[6][2];
#pragma unroll
      for (int i = 0; i < 6; ++i) rd(16 * i, g[i]);
      for (int q = 0; q < RTERMS; q += 96) {
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          wait(g[i]);
          add16(g[i]);
          rd((q + 96 + 16 * i) % RTERMS, g[i]);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = acc;
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
  {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(ring, dim3(1), dim3(64), 0, 0, out, cyc, 8, 1e-3f);
    unsigned long long c = 0;
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("{\"kernel\": \"ring (ws feed)\", \"lanes\": 8, \"cycles_per_dependent_add\": %.2f}\n",
           (double)c / (RREPS * RTERMS));
  }
  {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(ring16, dim3(1), dim3(64), 0, 0, out, cyc, 16, 1e-3f);
    unsigned long long c = 0;
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("{\"kernel\": \"ring16 (reader lanes + DPP)\", \"lanes\": 16, \"cycles_per_dependent_add\": %.2f}\n",
           (double)c / (RREPS * RTERMS));
  }
  (void)hipFree(out);
  (void)hipFree(cyc);
  return 0;
}
