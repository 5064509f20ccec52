// sgemm_sdot.hip — gemm(NoTrans, Trans) in the reference's sdot order.
//
// Replaces sgemm_nt / s_nt (ntensors.pas:1957-2005) over sdot_avx2
// (1233-1306): C[i,j] := C[i,j] + ALPHA * sdot(K, A[i,:], B[j,:]) after the
// cblas_sgemm beta pre-scale (2231-2286).  sdot_avx2 keeps 8 FMA lanes, lane l
// an ascending fma chain over k = l (mod 8) started at +0 (the masked tail is
// the same chain's last element, or fma(0, 0, x) = x), then sums
// s_l = lane_l + lane_{l+4} and returns (s0 + s1) + (s2 + s3).
//
// Here each residue class is an ascending f32-MFMA chain (v_mfma_f32_32x32x2
// is a bit-exact k-ordered fmaf chain, profiles/r01_mfma_order_probe.txt):
// a block owns a 32 x 32*TN output tile and its 8 waves are the 8 residue
// classes; MFMA step s of wave r consumes k = r + 16s + 8h (lane half h).
// Both operands are k-contiguous rows, staged global -> registers -> LDS
// ([row][k], odd row stride) in k-tiles of 64, double-buffered with one
// barrier per tile.  Zero-filled k >= K adds fma(0, 0, x) = x (a chain that
// starts at +0 never holds -0).  The epilogue meets the 8 partial tiles in LDS
// (classes r and r + 4 first, in four tiles of space) and applies the
// reference's pairwise sum, alpha product and C add, each rounded separately
// (built with -ffp-contract=off).
#include <algorithm>

#include "tns_internal.hpp"

namespace tns {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int SD_NT = 512;       // 8 waves = 8 residue classes
// k per tile: BK/8 per residue class = BK/16 MFMA steps.  64 by default;
// 256 for few output tiles over long k (conv dW: k = oH*oW up to 173056),
// where the chains are short per tile and the exposed global-load latency of
// every tile dominated (one block per image at 2.3 TF on YOLOv3 layer 0).

__device__ __attribute__((aligned(16))) static float4 g_sd_zero;

template <int TN, int VEC, int SD_BK, bool O32 = false>
__global__ __launch_bounds__(SD_NT) __attribute__((amdgpu_waves_per_eu(O32 ? 6 : 1)))
void sgemm_nt_sdot_kernel(GemmArgs p) {
  constexpr int SD_KP = SD_BK + 1;  // LDS row stride
  constexpr int BM = 32, BN = 32 * TN, ROWS = BM + BN;
  constexpr int KV = SD_BK / VEC;               // staging units per row
  constexpr int U = ROWS * KV / SD_NT;          // staging units per thread
  static_assert(ROWS * KV % SD_NT == 0, "staging split");
  constexpr int STAGE = ROWS * SD_KP;
  // float4 and O32 staging: the epilogue meets the partials in two halves (4
  // tiles of LDS: one more block per CU at 32 x 64, YOLOv3 52^2 / 26^2 dW
  // 0.163 -> 0.156 ms; with O32's 80 VGPRs, 13^2 dW 0.280 -> 0.226 ms); the
  // 64-bit-addressed scalar form is held to 2 blocks by its 94 VGPRs and keeps
  // all 8 tiles and one barrier
  constexpr bool HALVES = VEC == 4 || O32;
  constexpr int PART = (HALVES ? 4 : 8) * BM * BN;
  constexpr int LDS = 2 * STAGE > PART ? 2 * STAGE : PART;
  __shared__ float lds[LDS];

  const int tid = threadIdx.x, r = tid >> 6, lane = tid & 63;
  const int l31 = lane & 31, h = lane >> 5;
  const int tiles_m = (int)((p.M + BM - 1) / BM);
  const int64_t m0 = (int64_t)(blockIdx.x % tiles_m) * BM;
  const int64_t n0 = (int64_t)(blockIdx.x / tiles_m) * BN;
  const int64_t bz = blockIdx.y;
  const float* __restrict__ A = p.A + bz * p.strideA;
  const float* __restrict__ B = p.B + bz * p.strideB;
  float* __restrict__ C = p.C + bz * p.strideC;
  const int64_t M = p.M, N = p.N, K = p.K;

  float st[U * VEC];
  // O32 (scalar staging, each image's operands addressable in 32 bits): a
  // thread's k column tid % KV is the same for every staging unit and unit u
  // is an A row iff u < UA, so a load is the uniform base plus a 32-bit row
  // offset and one clamped k per tile.  Rows past M / N read the last row
  // (their outputs are never stored); k >= K reads zero.
  constexpr int UA = BM * KV / SD_NT;
  static_assert(!O32 || (VEC == 1 && SD_NT % KV == 0 && BM % (SD_NT / KV) == 0), "O32 form");
  const int kcol = tid % KV;
  int roff[O32 ? U : 1];
  if constexpr (O32) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = tid / KV + u * (SD_NT / KV);
      roff[u] = u < UA ? (int)(std::min<int64_t>(m0 + row, M - 1) * p.lda)
                       : (int)(std::min<int64_t>(n0 + row - BM, N - 1) * p.ldb);
    }
  }
  auto load_into = [&](float (&st)[U * VEC], int64_t k0) {
    if constexpr (O32) {
      const int kk = (int)k0 + kcol;
      const bool kin = kk < K;
      const int kc = kin ? kk : 0;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float v = (u < UA ? A : B)[roff[u] + kc];
        st[u] = kin ? v : 0.0f;
      }
      return;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = tid + SD_NT * u;
      const int row = idx / KV;
      const int64_t k = k0 + VEC * (idx % KV);
      const bool isa = row < BM;
      const int64_t g = isa ? m0 + row : n0 + row - BM;
      // VEC = 4 only when K % 4 == 0: a float4 is wholly inside or outside
      const bool ok = (g < (isa ? M : N)) & (k < K);
      const float* src = ok ? (isa ? A + g * p.lda : B + g * p.ldb) + k
                            : reinterpret_cast<const float*>(&g_sd_zero);
      if constexpr (VEC == 4) {
        const float4 v = *reinterpret_cast<const float4*>(src);
        st[4 * u + 0] = v.x;
        st[4 * u + 1] = v.y;
        st[4 * u + 2] = v.z;
        st[4 * u + 3] = v.w;
      } else {
        st[u] = *src;
      }
    }
  };
  auto load = [&](int64_t k0) { load_into(st, k0); };
  auto store_from = [&](const float (&st)[U * VEC], float* buf) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = tid + SD_NT * u;
      const int row = idx / KV, k = VEC * (idx % KV);
#pragma unroll
      for (int c = 0; c < VEC; ++c) buf[row * SD_KP + k + c] = st[VEC * u + c];
    }
  };
  auto store = [&](float* buf) { store_from(st, buf); };

  floatx16 acc[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.0f;

  const int nt = (int)((K + SD_BK - 1) / SD_BK);
  auto mma_tile = [&](const float* cur) {
#pragma unroll
    for (int s = 0; s < SD_BK / 16; ++s) {
      const int kk = r + 16 * s + 8 * h;  // residue class r, ascending
      const float a = cur[l31 * SD_KP + kk];
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, cur[(BM + 32 * j + l31) * SD_KP + kk],
                                                      acc[j], 0, 0, 0);
    }
  };
  if constexpr (SD_BK == 256) {
    // long-k form: global loads run TWO tiles ahead (two register sets), so
    // a tile's load latency is covered by two tiles of MFMA chains
    float st2[U * VEC];
    auto body = [&](float (&ld)[U * VEC], const float (&sv)[U * VEC], int t) {
      if (t + 2 < nt) load_into(ld, (int64_t)(t + 2) * SD_BK);
      mma_tile(lds + (t & 1) * STAGE);
      if (t + 1 < nt) store_from(sv, lds + ((t + 1) & 1) * STAGE);
      __syncthreads();
    };
    if (nt > 0) {
      load_into(st, 0);
      store_from(st, lds);
      if (nt > 1) load_into(st, SD_BK);
      __syncthreads();
      for (int t = 0; t < nt; t += 2) {
        body(st2, st, t);              // tile t+1 from st, tile t+2 into st2
        if (t + 1 < nt) body(st, st2, t + 1);  // tile t+2 from st2, t+3 into st
      }
    }
  } else if (nt > 0) {
    load(0);
    store(lds);
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
      if (t + 1 < nt) load((int64_t)(t + 1) * SD_BK);
      mma_tile(lds + (t & 1) * STAGE);
      if (t + 1 < nt) store(lds + ((t + 1) & 1) * STAGE);
      __syncthreads();
    }
  }

  // partial tiles of the residue classes (every wave has passed the last
  // barrier, so the operand buffers are free).  HALVES: classes 4..7 ->
  // lds[r - 4][row][col]; class r < 4 then forms s_r = lane_r + lane_{r+4} in
  // its registers and leaves it in lds[r].  Else class r -> lds[r].
  auto part_at = [&](int j, int e) {
    const int row = (e & 3) + 8 * (e >> 2) + 4 * h;
    return ((HALVES ? (r & 3) : r) * BM + row) * BN + 32 * j + l31;
  };
  if (!HALVES || r >= 4) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) lds[part_at(j, e)] = acc[j][e];
  }
  __syncthreads();
  if constexpr (HALVES) {
    if (r < 4) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int i = part_at(j, e);
          lds[i] = acc[j][e] + lds[i];
        }
    }
    __syncthreads();
  }
  const float alpha = p.alpha, beta = p.beta;
  for (int o = tid; o < BM * BN; o += SD_NT) {
    const int64_t m = m0 + o / BN, n = n0 + o % BN;
    if (m >= M || n >= N) continue;
    constexpr int T = BM * BN;
    float s0, s1, s2, s3;
    if constexpr (HALVES) {
      s0 = lds[o], s1 = lds[T + o], s2 = lds[2 * T + o], s3 = lds[3 * T + o];
    } else {
      s0 = lds[o] + lds[4 * T + o], s1 = lds[T + o] + lds[5 * T + o];
      s2 = lds[2 * T + o] + lds[6 * T + o], s3 = lds[3 * T + o] + lds[7 * T + o];
    }
    const float dot = (s0 + s1) + (s2 + s3);
    const float sum = alpha * dot;  // sum := ALPHA * sdot(...)
    float* cp = C + m * p.ldc + n;
    if (p.beta_mode == BETA_STORE) {
      *cp = sum;
      continue;
    }
    float c0;
    if (p.beta_mode == BETA_ZERO)
      c0 = 0.0f;
    else if (p.beta_mode == BETA_SCALE)
      c0 = beta * *cp;  // cblas_sgemm's mulvs pre-scale
    else
      c0 = *cp;
    *cp = c0 + sum;  // C[i,j] := C[i,j] + sum
  }
}

template <int TN, int VEC, int BK = 64, bool O32 = false>
hipError_t launch_tn(const GemmArgs& a, hipStream_t s) {
  const int64_t tiles = ((a.M + 31) / 32) * ((a.N + 32 * TN - 1) / (32 * TN));
  if (tiles > 0x7fffffff) return hipErrorInvalidValue;
  for (int64_t b0 = 0; b0 < a.batch; b0 += 65535) {
    GemmArgs sub = a;
    const int64_t nb = a.batch - b0 < 65535 ? a.batch - b0 : 65535;
    sub.A = a.A + b0 * a.strideA;
    sub.B = a.B + b0 * a.strideB;
    sub.C = a.C + b0 * a.strideC;
    sub.batch = nb;
    hipLaunchKernelGGL((sgemm_nt_sdot_kernel<TN, VEC, BK, O32>), dim3((unsigned)tiles, (unsigned)nb),
                       dim3(SD_NT), 0, s, sub);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

bool k_vec4(const float* p, int64_t ld, int64_t stride, int64_t batch, int64_t K) {
  if ((reinterpret_cast<uintptr_t>(p) & 15) != 0) return false;
  if (ld % 4 != 0 || K % 4 != 0) return false;
  return batch <= 1 || stride % 4 == 0;
}

}  // namespace

static int g_sdot_form = -1;
void set_sdot_form(int form) { g_sdot_form = form < 0 ? -1 : form; }

// MFMA: 32x64 tiles when they still give >= 4 blocks per CU, else 32x32;
// few outputs over a long k go to the VALU chain kernel
hipError_t launch_sgemm_nt_sdot(const GemmArgs& a, hipStream_t s) {
  if (a.M <= 0 || a.N <= 0 || a.batch <= 0) return hipSuccess;
  if (g_sdot_form >= SDOT_FORM_RC) return launch_sdot_rc(g_sdot_form - SDOT_FORM_RC, a, s);
  if (g_sdot_form > 0) return launch_sdot_chains(a, g_sdot_form - 1, s);
  // few outputs over a long k (conv dW of the 416/208/104-pixel YOLOv3
  // layers): the VALU chain kernel, tile by output count (scripts/
  // sdot_forms.py, profiles/r02_sdot_forms.json: YOLOv3 layer 0 dW at batch
  // 8 1.44 -> 0.28 ms, layer 2 0.35 -> 0.10 ms, layer 5 0.089 -> 0.056 ms;
  // the 104^2 1x1 layers' 65536 outputs on four residues a lane, 0.130 ->
  // 0.115 ms a call, profiles/r04_bwd_dw_sweep.json)
  const int64_t t32 = ((a.M + 31) / 32) * ((a.N + 31) / 32) * a.batch;
  if (g_sdot_form < 0 && a.K >= 4096 && t32 <= 64) {
    const int64_t outs = a.M * a.N * a.batch;
    return launch_sdot_chains(a, outs <= 8192 ? 1 : (outs <= 32768 ? 2 : 6), s);
  }
  // many 64x64 tiles over a short k (conv dW of the 26^2 / 13^2 layers, k =
  // pixels per image): two waves per 32x32 tile, four residue chains each
  // (sgemm_sdot_rc.hip; profiles/r03_dw_forms.json: 4-7 % on those layers,
  // behind this kernel on the 52^2 ones)
  const int64_t t64 = ((a.M + 63) / 64) * ((a.N + 63) / 64) * a.batch;
  if (g_sdot_form < 0 && a.K <= 1024 && t64 >= 512 && sdot_rc_applies(a))
    return launch_sdot_rc(1, a, s);
  const bool v = k_vec4(a.A, a.lda, a.strideA, a.batch, a.K) &&
                 k_vec4(a.B, a.ldb, a.strideB, a.batch, a.K);
  const int64_t b64 = ((a.M + 31) / 32) * ((a.N + 63) / 64) * a.batch;
  // scalar staging with 32-bit row offsets when each image's A and B fit them
  const bool o32 = (a.M - 1) * a.lda + a.K <= 0x7fffffffLL && (a.N - 1) * a.ldb + a.K <= 0x7fffffffLL;
  if (b64 >= 1024)
    return v ? launch_tn<2, 4>(a, s) : (o32 ? launch_tn<2, 1, 64, true>(a, s) : launch_tn<2, 1>(a, s));
  // few 32x32 tiles over a long k: 256-deep k-tiles (the 64-row LDS stages
  // take 2 x 65.8 KB of gfx950's 160 KB)
  if (a.K >= 16384 && ((a.M + 31) / 32) * ((a.N + 31) / 32) * a.batch < 512)
    return v ? launch_tn<1, 4, 256>(a, s) : launch_tn<1, 1, 256>(a, s);
  return v ? launch_tn<1, 4>(a, s) : launch_tn<1, 1>(a, s);
}

}  // namespace tns
