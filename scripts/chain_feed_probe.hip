// chain_feed_probe.hip — what feeds a dependent v_add_f32 chain at the bare
// rate (the batch-norm reductions' AVX-lane chains, batchnorm.hip).  Timing
// only; results discarded.  One 64-thread block per mode, nothing else on
// the CU; cycles by s_memtime around the loop, per dependent add.
//
//   hipcc --offload-arch=gfx950 -O3 scripts/chain_feed_probe.hip -o scripts/chain_feed_probe
//
//   lds8     8 chain lanes, 16-term groups by four ds_read_b128 three groups
//            ahead (block_chains_ws's feed)
//   lds64    the same with all 64 lanes chains (8 planes a wave)
//   vmem8    8 chain lanes, terms by global_load_dwordx4 from an L2-hot
//            lane-major buffer, 8 groups ahead (vmcnt counted)
//   vmem64   the same, 64 lanes
//   lds_inter  one ds_read_b128 after every four adds, 12 quads ahead
//   lds_indep  the lds8 feed, the adds into 4 independent accumulators
//   bare     the chain on register operands
//   vmem8d   8 chain lanes, dword loads at the raw layout's stride (lane l
//            reads a[8t + l]), 48 ahead
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int RLDT = 840, RTERMS = 768, RREPS = 64;

__global__ void lds_ring(float* out, unsigned long long* cyc, int lanes, float x) {
  __shared__ __attribute__((aligned(16))) float U[8 * RLDT];
  const int l = threadIdx.x;
  for (int i = l; i < 8 * RLDT; i += 64) U[i] = x * (float)(i & 7);
  __syncthreads();
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

// lane-major buffer: lane l's terms at buf[l * RTERMS + i] (RTERMS per lane,
// 64 lanes), re-walked RREPS times (L2 / L1 resident)
constexpr int VG = 8;  // groups of 4 terms in flight
__global__ void vmem_ring(const float* __restrict__ buf, float* out, unsigned long long* cyc,
                          int lanes) {
  const int l = threadIdx.x;
  float acc = 0.f;
  const float* row = buf + (size_t)l * RTERMS;
  auto ld = [&](int q, f4& v) {
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(row + q));
  };
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (l < lanes) {
    for (int r = 0; r < RREPS; ++r) {
      f4 v[VG];
#pragma unroll
      for (int g = 0; g < VG; ++g) ld(4 * g, v[g]);
      for (int q = 0; q < RTERMS; q += 4 * VG) {
#pragma unroll
        for (int g = 0; g < VG; ++g) {
          asm volatile("s_waitcnt vmcnt(%1)" : "+v"(v[g]) : "n"(VG - 1));
#pragma unroll
          for (int z = 0; z < 4; ++z) acc = acc + v[g][z];
          ld((q + 4 * VG + 4 * g) % RTERMS, v[g]);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = acc;
  if (l == 0) cyc[0] = t1 - t0;
}

// raw layout: lane l's term t at a[8t + l] (dword loads, 48 ahead)
constexpr int DG = 48;
__global__ void vmem_dword(const float* __restrict__ buf, float* out, unsigned long long* cyc,
                           int lanes) {
  const int l = threadIdx.x;
  float acc = 0.f;
  const float* row = buf + l;
  auto ld = [&](int t, float& v) {
    asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(row + 8 * t));
  };
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (l < lanes) {
    for (int r = 0; r < RREPS; ++r) {
      float v[DG];
#pragma unroll
      for (int g = 0; g < DG; ++g) ld(g, v[g]);
      for (int q = 0; q < RTERMS; q += DG) {
#pragma unroll
        for (int g = 0; g < DG; ++g) {
          asm volatile("s_waitcnt vmcnt(%1)" : "+v"(v[g]) : "n"(DG - 1));
          acc = acc + v[g];
          ld((q + DG + g) % RTERMS, v[g]);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = acc;
  if (l == 0) cyc[0] = t1 - t0;
}


// lds_inter: the same ring, one ds_read_b128 after every four adds (reads
// spread through the group, the wait per four adds)
__global__ void lds_inter(float* out, unsigned long long* cyc, int lanes, float x) {
  __shared__ __attribute__((aligned(16))) float U[8 * RLDT];
  const int l = threadIdx.x;
  for (int i = l; i < 8 * RLDT; i += 64) U[i] = x * (float)(i & 7);
  __syncthreads();
  float acc = 0.f;
  const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const float*)(U + (l & 7) * RLDT);
  auto rd1 = [&](int q, f4& v) {
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(base + 4u * (unsigned)q));
  };
  constexpr int NQ = 12;  // quads in flight
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (l < lanes) {
    for (int r = 0; r < RREPS; ++r) {
      f4 v[NQ];
#pragma unroll
      for (int g = 0; g < NQ; ++g) rd1(4 * g, v[g]);
      for (int q = 0; q < RTERMS; q += 4 * NQ) {
#pragma unroll
        for (int g = 0; g < NQ; ++g) {
          asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v[g]) : "n"(NQ - 1));
#pragma unroll
          for (int z = 0; z < 4; ++z) acc = acc + v[g][z];
          rd1((q + 4 * NQ + 4 * g) % RTERMS, v[g]);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = acc;
  if (l == 0) cyc[0] = t1 - t0;
}

// lds_indep: block_chains_ws's reads, the 16 adds of a group into 4
// independent accumulators (the feed's own cost, chain latency hidden)
__global__ void lds_indep(float* out, unsigned long long* cyc, int lanes, float x) {
  __shared__ __attribute__((aligned(16))) float U[8 * RLDT];
  const int l = threadIdx.x;
  for (int i = l; i < 8 * RLDT; i += 64) U[i] = x * (float)(i & 7);
  __syncthreads();
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
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
    for (int z = 0; z < 16; ++z) acc[z & 3] = acc[z & 3] + v[z >> 2][z & 3];
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
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  if (l == 0) cyc[0] = t1 - t0;
}

// bare: the dependent chain over register operands (no feed)
__global__ void bare(float* out, unsigned long long* cyc, int lanes, float x) {
  const int l = threadIdx.x;
  float acc = 0.f;
  f4 v = {x, x * 2, x * 3, x * 4};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (l < lanes) {
    for (int r = 0; r < RREPS * RTERMS; r += 16) {
#pragma unroll
      for (int z = 0; z < 16; ++z) acc = acc + v[z & 3];
      asm volatile("" : "+v"(v));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = acc;
  if (l == 0) cyc[0] = t1 - t0;
}

int main() {
  float *out, *buf;
  unsigned long long* cyc;
  if (hipMalloc(&out, 64 * sizeof(float)) != hipSuccess) return 1;
  if (hipMalloc(&cyc, sizeof(unsigned long long)) != hipSuccess) return 1;
  if (hipMalloc(&buf, 64 * RTERMS * 8 * sizeof(float)) != hipSuccess) return 1;
  (void)hipMemset(buf, 0, 64 * RTERMS * 8 * sizeof(float));
  auto report = [&](const char* name, int lanes) {
    unsigned long long c = 0;
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("{\"feed\": \"%s\", \"lanes\": %d, \"cycles_per_dependent_add\": %.2f}\n", name, lanes,
           (double)c / (RREPS * RTERMS));
  };
  for (int rep = 0; rep < 2; ++rep) {
    for (int lanes : {8, 64}) {
      for (int w = 0; w < 3; ++w)
        hipLaunchKernelGGL(lds_ring, dim3(1), dim3(64), 0, 0, out, cyc, lanes, 1e-3f);
      report("lds_b128", lanes);
      for (int w = 0; w < 3; ++w)
        hipLaunchKernelGGL(lds_inter, dim3(1), dim3(64), 0, 0, out, cyc, lanes, 1e-3f);
      report("lds_b128_interleaved_12ahead", lanes);
      for (int w = 0; w < 3; ++w)
        hipLaunchKernelGGL(lds_indep, dim3(1), dim3(64), 0, 0, out, cyc, lanes, 1e-3f);
      report("lds_b128_4_independent_accs", lanes);
      for (int w = 0; w < 3; ++w)
        hipLaunchKernelGGL(bare, dim3(1), dim3(64), 0, 0, out, cyc, lanes, 1e-3f);
      report("bare_registers", lanes);
      for (int w = 0; w < 3; ++w)
        hipLaunchKernelGGL(vmem_ring, dim3(1), dim3(64), 0, 0, buf, out, cyc, lanes);
      report("vmem_dwordx4_lane_major", lanes);
      for (int w = 0; w < 3; ++w)
        hipLaunchKernelGGL(vmem_dword, dim3(1), dim3(64), 0, 0, buf, out, cyc, lanes);
      report("vmem_dword_raw_stride8", lanes);
    }
  }
  (void)hipFree(out);
  (void)hipFree(cyc);
  (void)hipFree(buf);
  return 0;
}
