// sgemm.hip — SGEMM dispatch: tile-shape choice per problem and the variant
// table used by the tuning entry point (tns_hip_gemm_variant).  The kernel
// itself (MFMA main loop, numerics notes) is in sgemm_kernel.hpp.
#include <cmath>

#include "sgemm_kernel.hpp"

namespace tns {
namespace {

struct VariantInfo {
  const char* name;
  int bm, bn;
  ShapeLauncher fn;
};

#define TNS_ROW(ID, NAME, BMv, BNv, KIND) {NAME, BMv, BNv, &launch_shape_##ID},
const VariantInfo kVariants[] = {TNS_SHAPES(TNS_ROW)};
#undef TNS_ROW
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

unsigned* g_stamps = nullptr;  // block timeline buffer (diagnostic builds only)

enum {
  V_128x128 = 0, V_128x64 = 1, V_64x128 = 2, V_64x256 = 3, V_32x256 = 4, V_256x256w8 = 5,
  V_64x64 = 6, V_64x64m16 = 12, V_32x32m16 = 13, V_64x32m16 = 14, V_32x64m16 = 15,
  V_128x128m16 = 16, V_256x256w8m16 = 17, V_128x64w8 = 18, V_64x128w8 = 19, V_128x128w8 = 20,
  V_64x64d1 = 21, V_64x64w8m16 = 22
};

// float4 staging needs 16-B aligned rows and a contiguous extent that is a
// multiple of 4 (so every float4 is wholly inside or outside the operand).
bool vec4_ok(const float* p, int64_t ld, int64_t stride, int64_t batch, int64_t extent) {
  if ((reinterpret_cast<uintptr_t>(p) & 15) != 0) return false;
  if (ld % 4 != 0 || extent % 4 != 0) return false;
  if (batch > 1 && stride % 4 != 0) return false;
  return true;
}

// Shape heuristic: skinny-M conv GEMMs (filters 32/64) get short, wide tiles;
// otherwise the largest tile that still gives every CU work.
// TN with k <= 1024 (the conv backward's col = W^T . delta, K = filters)
// unless 256x256 tiles cover M x N exactly: 64x64 tiles on 16x16 MFMAs, on
// 32x32 MFMAs at k = 1024, 32x32 tiles below ~2 blocks per CU (scripts/
// sgemm_sweep.py --tn, YOLOv3 dX shapes at batch 8: 52^2 3x3 70 -> 88 TF,
// 26^2 83 -> 92, 13^2 68 -> 72, 1x1 layers 38-52 -> 47-60; 4096^2 x 1024
// stays on 256x256, 121 TF against 106 on 64x64).
//
// NN with float4 operands (the conv GEMMs of Conv2D and forwardGPU's
// gemmStridedBatched, strideA = 0; FC dX) by block count, as the implicit
// conv picks (b64 = blocks a 64x64 tile gives, batch included): skinny M on
// 32x64 / 64x128 tiles, >= 1200 blocks of a deep K on 128x64, >= 600 on
// 8-wave 64x64 16x16-MFMA tiles, fewer on 64x32 / 32x32 16x16-MFMA tiles
// (profiles/r03_sgemm_sweep_yolo.json: every YOLOv3 batch-8 shape within
// 10 % of the best swept tile; the old N >= 1024 rule was up to 2.4x off).
int pick_variant(const GemmArgs& a, bool av, bool bv, bool ta, bool tb) {
  const int64_t M = a.M, N = a.N, batch = a.batch;
  auto blocks = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn) * batch; };
  const bool big_exact = M % 256 == 0 && N % 256 == 0 && blocks(256, 256) >= 240 && av && bv;
  if (ta && !tb && a.K <= 1024 && M > 64 && !big_exact)
    return blocks(64, 64) < 512 ? V_32x32m16 : (a.K >= 1024 ? V_64x64 : V_64x64m16);
  if (!ta && !tb && !big_exact) {
    // the 8-wave and 64x32 / 32x64 shapes are float4-NN only: their
    // nearest general shape otherwise (N = 169 etc. is not a multiple of 4)
    const bool v4 = av && bv;
    const int64_t b64 = blocks(64, 64);
    if (M <= 32) {
      if (a.K < 32) return V_32x256;
      return blocks(32, 64) >= 1024 && v4 ? V_32x64m16 : V_32x32m16;
    }
    if (M <= 64) return b64 >= 600 ? (v4 ? V_64x128w8 : V_64x128) : V_32x32m16;
    if (b64 >= 1200 && M % 128 == 0 && a.K >= 1024) return V_128x64;
    if (b64 >= 600) return v4 ? V_64x64w8m16 : V_64x64;
    if (b64 >= 256 && a.K < 2048 && v4) return V_64x32m16;
    return V_32x32m16;
  }
  if (M <= 32) return V_32x256;
  if (M <= 64) return V_64x256;
  if (M >= 256 && blocks(256, 256) >= 240 && av && bv) return V_256x256w8;
  if (N >= 1024) return V_64x128;
  return V_128x64;
}

// Implicit-GEMM conv tile choice.  No split-K (bit-exactness), so the
// parallelism is the output tiles alone.  From the YOLOv3 sweep (scripts/
// conv_sweep.py; b64 = blocks a 64x64 tile would give):
//   b64 >= 1200, filters % 128 == 0  128x64, 8 waves of 32x32
//   b64 >= 600 (or 64 filters)       64x64, 8 waves of 32x16 (16x16 MFMA)
//   fewer blocks: 16x16-MFMA tiles, whose four times as many accumulator
//   chains per output area keep 256 CUs busy — 64x32 for deep K (the
//   1024-filter 3x3 layers), 32x32 for the fewest blocks, else 32x64.
int pick_conv_variant(const GemmArgs& a) {
  const int64_t M = a.M, N = a.N, K = a.K;
  if (M <= 32) return V_32x32m16;
  const int64_t b64 = ((M + 63) / 64) * ((N + 63) / 64);
  if (b64 >= 1200 && M % 128 == 0) return V_128x64w8;
  if (b64 >= 600) return V_64x64w8m16;
  if (K >= 2048) return V_64x32m16;
  if (b64 <= 200) return V_32x32m16;
  return V_32x64m16;
}

}  // namespace

hipError_t launch_sgemm_conv_variant(int variant, const GemmArgs& a_in, hipStream_t s) {
  GemmArgs a = a_in;
  a.stamps = g_stamps;
  if (a.M <= 0 || a.N <= 0 || a.batch <= 0) return hipSuccess;
  if (!a.conv || !a.ktab) return hipErrorInvalidValue;
  const bool av = vec4_ok(a.A, a.lda, a.strideA, a.batch, a.K);
  const int v = variant < 0 ? pick_conv_variant(a) : variant;
  switch (v) {
    case V_128x64: return launch_conv_128x64(a, av, s);
    case V_64x128: return launch_conv_64x128(a, av, s);
    case V_32x256: return launch_conv_32x256(a, av, s);
    case V_64x64: return launch_conv_64x64(a, av, s);
    case V_64x64m16: return launch_conv_64x64m16(a, av, s);
    case V_32x32m16: return launch_conv_32x32m16(a, av, s);
    case V_64x32m16: return launch_conv_64x32m16(a, av, s);
    case V_32x64m16: return launch_conv_32x64m16(a, av, s);
    case V_128x64w8: return launch_conv_128x64w8(a, av, s);
    case V_64x128w8: return launch_conv_64x128w8(a, av, s);
    case V_128x128w8: return launch_conv_128x128w8(a, av, s);
    case V_64x64d1: return launch_conv_64x64d1(a, av, s);
    case V_64x64w8m16: return launch_conv_64x64w8m16(a, av, s);
    default: return hipErrorInvalidValue;  // no implicit-conv instantiation
  }
}

hipError_t launch_sgemm_conv(const GemmArgs& a, hipStream_t s) {
  return launch_sgemm_conv_variant(-1, a, s);
}

// the last variant indices are the dedicated large-NN kernels (sgemm_nn_big.hip)
int sgemm_variant_count() { return kNumVariants + sgemm_nn_big_count(); }
const char* sgemm_variant_name(int v) {
  if (v >= kNumVariants) return sgemm_nn_big_name(v - kNumVariants);
  return (v >= 0 && v < kNumVariants) ? kVariants[v].name : "";
}

hipError_t launch_sgemm_variant(int variant, const GemmArgs& a_in, bool transA, bool transB,
                                hipStream_t s) {
  GemmArgs a = a_in;
  a.stamps = g_stamps;
  if (a.M <= 0 || a.N <= 0 || a.batch <= 0) return hipSuccess;
  // A is k-contiguous unless transposed; B is n-contiguous unless transposed
  const bool av = vec4_ok(a.A, a.lda, a.strideA, a.batch, transA ? a.M : a.K);
  const bool bv = vec4_ok(a.B, a.ldb, a.strideB, a.batch, transB ? a.K : a.N);
  if (variant >= kNumVariants) {
    if (transA || transB) return hipErrorInvalidValue;
    return launch_sgemm_nn_big(variant - kNumVariants, a, s);
  }
  if (variant < 0 && !transA && !transB) {
    const int nb = sgemm_nn_big_pick(a);
    if (nb >= 0) return launch_sgemm_nn_big(nb, a, s);
  }
  const int v = variant < 0 ? pick_variant(a, av, bv, transA, transB) : variant;
  if (v >= kNumVariants) return hipErrorInvalidValue;
  return kVariants[v].fn(a, transA, transB, av, bv, s);
}

hipError_t launch_sgemm(const GemmArgs& a, bool transA, bool transB, hipStream_t s) {
  return launch_sgemm_variant(-1, a, transA, transB, s);
}

#ifdef TNS_GEMM_STAMPS
// diagnostic build only (not in include/tns.h): every following launch
// records {start, end, HW_ID, XCC_ID} per block into dev_buf (8 words per
// block), or nothing when dev_buf is NULL
extern "C" int tns_debug_gemm_stamps(unsigned* dev_buf) {
  g_stamps = dev_buf;
  return 0;
}
#endif

}  // namespace tns
