// tns_api.cpp — the C ABI of libtensorium_hip.so (declared in include/tns.h).
//
// Host-side logic of the reference's hot path, restated for HIP:
//   * boundary A: op-table drop-ins with host pointers (cblas_sgemm & co,
//     ntensors.pas:345-385) staging through device scratch owned here;
//   * boundary B: the TNNCuda<T>-shaped device API (nncuda.pas:35-157);
//   * layer drivers: TTensor.Conv2D (ntensors.pas:8252-8349) and
//     TConvolutionalLayer.forward/forwardGPU (nConvolutionLayer.pas:457-569,
//     1022-1153).
// Nothing here falls back to the CPU: every compute entry point launches a
// gfx950 kernel or fails with a status.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <map>
#include <mutex>
#include <thread>
#include <vector>
#include <string>
#include <tuple>

#include "tns_internal.hpp"

namespace tns {

static thread_local std::string g_err;
static tns_error_hook_t g_hook = nullptr;
static int64_t g_strict_beta0 = 1;
static int64_t g_nt_sdot = 1;
static int64_t g_dx_fused = 1;
// conv backward col = W^T . delta: -1 conv_tile4's k-major-A forms where
// they apply, -2 the TN GEMM, v >= 0 form v (TNS_OPT_DX_TILE)
static int64_t g_dx_tile = -1;
static int64_t g_dx_conv = -1;
static int64_t g_dw_res = -1;
// state.delta of the 1x1 / stride-1 layers on conv1x1.hip (W^T over the delta
// planes, the col2im add in the epilogue) where conv1x1_pick takes the shape;
// TNS_DX_C1=0 (A/B): the TN product / conv_dx forms
static bool g_dx_c1 = !(getenv("TNS_DX_C1") && getenv("TNS_DX_C1")[0] == '0');
// the BN conv backward as one chain pass + normalizeDelta (launch_bn_backward_fused);
// TNS_BN_FUSED=0 (A/B): the three-pass form
static bool g_bn_fused = !(getenv("TNS_BN_FUSED") && getenv("TNS_BN_FUSED")[0] == '0');
// conv backward dW with the im2col matrix generated in the staging
// (dw_tile.hip): -1 by measured shape, -2 never, v >= 0 form v (TNS_OPT_DW_TILE)
static int64_t g_dw_tile = -1;
// conv backward: dW and state.delta concurrently on two streams (TNS_OPT_BWD_OVERLAP)
static int64_t g_bwd_overlap = 1;
static int64_t g_derive_sums = 0;
// TNS_OPT_SCRATCH_CAP: largest context scratch buffer in floats (0 = none);
// a larger request fails as an allocation failure would (tests reach the
// fallback paths with it)
static int64_t g_scratch_cap = 0;
static int64_t g_tt_exact = 1;
static int64_t g_srss_quirk = 0;
static int64_t g_conv_variant = -1;
static int64_t g_conv_pad = -1;

int set_error(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  if (g_hook) g_hook(code, buf);
  return code;
}

const char* hip_err_str(hipError_t e) { return hipGetErrorString(e); }

}  // namespace tns

using namespace tns;

struct tns_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  // device scratch, one buffer per SLOT_* below (im2col workspace, host-API
  // staging, dW partial sums, batch-norm block results, ...)
  static constexpr int kSlots = 12;
  float* scratch[kSlots] = {};
  size_t scratch_elems[kSlots] = {};
  // telemetry (TTensorMetrics-style, nopmetrics.pas:25-44)
  bool telemetry = false;
  double op_ms[TNS_OP_COUNT] = {0};
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::mutex mu;  // serialises host-API use of one context
  // host-pointer pipeline: copy stream and per-chunk events
  hipStream_t copy_stream = nullptr;
  std::vector<hipEvent_t> pipe_ev;
  // conv backward: state.delta's chain (TN + col2im) runs on this side
  // stream while the dW product runs on `stream` (fork / join events)
  hipStream_t aux_stream = nullptr;
  // the joined overlap's side stream (TNS_OPT_BWD_OVERLAP = 1: state.delta's
  // chain beside the call's dW, joined before the call returns) at the
  // context stream's priority; aux_stream, the pipelined dW products' stream,
  // sits at the lowest
  hipStream_t ovl_stream = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // TNS_OPT_BWD_OVERLAP = 2: dW products left running on aux_stream past the
  // call's return; the next call of any other entry point joins them first
  bool side_pending = false;
  hipStream_t home_stream = nullptr;  // the context's stream while `stream` is aux
  // the pending dW products' operand ranges: read (delta, input) and written
  // (weight_updates; the caller's workspace when the dW's im2col fills it).
  // A later call whose work on `stream` writes a read range, or touches a
  // written one, joins the side stream first; so does a call that takes a
  // scratch slot the side stream uses (side_slots)
  struct PendingDw {
    uintptr_t lo[2], hi[2];    // read by the dW
    uintptr_t wlo[2], whi[2];  // written by the dW
  };
  std::vector<PendingDw> pending;
  uint32_t side_slots = 0;
  // implicit-GEMM conv k-tables, one per (C, H, W, kH, kW, dY, dX)
  std::map<std::tuple<int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t>, int*> ktabs;
};

namespace {

enum { SLOT_COL = 0, SLOT_STAGE1 = 1, SLOT_STAGE2 = 2, SLOT_STAGE3 = 3, SLOT_DW = 4, SLOT_BN = 5,
       SLOT_MLP = 6, SLOT_WT = 7, SLOT_COL_DX = 8, SLOT_WPERM = 9, SLOT_RES_A = 10,
       SLOT_RES_B = 11, SLOT_COUNT = 12 };
static_assert(SLOT_COUNT == tns_ctx::kSlots, "one scratch buffer per slot");

int join_side(tns_ctx* c);

// scratch buffer `slot` of at least `elems` floats.  side: the caller is the
// pipelined conv backward taking a slot for the dW it queues behind the
// pending ones on the side stream (no join); any other caller of a slot the
// side stream still uses joins it first
int ensure_scratch(tns_ctx* c, int slot, int64_t elems, float** out, bool side = false) {
  if (elems < 1) elems = 1;
  if (!side && c->side_pending && (c->side_slots >> slot & 1u) && c->stream != c->aux_stream)
    if (int r = join_side(c)) return r;
  if (g_scratch_cap > 0 && elems > g_scratch_cap)
    return set_error(TNS_ERR_NOMEM, "scratch slot %d: %lld floats exceed the cap of %lld", slot,
                     (long long)elems, (long long)g_scratch_cap);
  if ((size_t)elems > c->scratch_elems[slot]) {
    if (c->scratch[slot]) {
      hipStreamSynchronize(c->stream);
      if (c->aux_stream) hipStreamSynchronize(c->aux_stream);
      if (c->ovl_stream) hipStreamSynchronize(c->ovl_stream);
      if (c->home_stream) hipStreamSynchronize(c->home_stream);
      hipFree(c->scratch[slot]);
      c->scratch[slot] = nullptr;
      c->scratch_elems[slot] = 0;
    }
    hipError_t e = hipMalloc(&c->scratch[slot], (size_t)elems * sizeof(float));
    if (e != hipSuccess) {
      c->scratch[slot] = nullptr;
      // (clear HIP's sticky last error: the launch helpers report
      // hipGetLastError(), and a caller that falls back after this failure
      // must not see it on its first launch)
      hipGetLastError();
      return set_error(TNS_ERR_NOMEM, "hipMalloc(%lld floats) failed: %s", (long long)elems,
                       hipGetErrorString(e));
    }
    c->scratch_elems[slot] = (size_t)elems;
  }
  *out = c->scratch[slot];
  return TNS_OK;
}

// give a scratch buffer back (every stream that may still use it drained)
void release_scratch(tns_ctx* c, int slot) {
  if (!c->scratch[slot]) return;
  hipStreamSynchronize(c->stream);
  if (c->aux_stream) hipStreamSynchronize(c->aux_stream);
  if (c->ovl_stream) hipStreamSynchronize(c->ovl_stream);
  if (c->home_stream) hipStreamSynchronize(c->home_stream);
  hipFree(c->scratch[slot]);
  c->scratch[slot] = nullptr;
  c->scratch_elems[slot] = 0;
}

// the conv backward's side stream and its fork / join events, created
// together on the context's device; false (nothing kept) if any of them
// cannot be created, and the caller runs its sequential schedule
bool ensure_side_stream(tns_ctx* c) {
  if (c->aux_stream && c->ovl_stream && c->ev_fork && c->ev_join) return true;
  int prev = -1;
  hipGetDevice(&prev);
  // the pipelined dW products' stream (off the critical path) at the lowest
  // queue priority and the context's stream at the highest: the context's
  // work is dispatched first where both wait for CU room (YOLOv3 training
  // backward 17.96 -> 17.81 ms with the chain waves' issue priority,
  // batchnorm.hip; TNS_STREAM_PRIO=0 turns it off).  The joined overlap
  // waits for both halves of a call, so its stream keeps the default
  // priority (at the lowest, the joined conv backward lost 0.25 ms)
  int least = 0, greatest = 0;
  const char* sp = getenv("TNS_STREAM_PRIO");
  const bool prio = !(sp && sp[0] == '0') &&
                    hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess;
  bool ok = hipSetDevice(c->device) == hipSuccess &&
            (prio ? hipStreamCreateWithPriority(&c->aux_stream, hipStreamNonBlocking, least)
                  : hipStreamCreateWithFlags(&c->aux_stream, hipStreamNonBlocking)) == hipSuccess &&
            hipStreamCreateWithFlags(&c->ovl_stream, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    if (c->aux_stream) hipStreamDestroy(c->aux_stream);
    if (c->ovl_stream) hipStreamDestroy(c->ovl_stream);
    if (c->ev_fork) hipEventDestroy(c->ev_fork);
    if (c->ev_join) hipEventDestroy(c->ev_join);
    c->aux_stream = c->ovl_stream = nullptr;
    c->ev_fork = c->ev_join = nullptr;
    hipGetLastError();
  }
  if (prev >= 0) hipSetDevice(prev);
  return ok;
}

struct OpTimer {
  tns_ctx* c;
  int op;
  explicit OpTimer(tns_ctx* c_, int op_) : c(c_), op(op_) {
    if (c->telemetry) hipEventRecord(c->ev0, c->stream);
  }
  ~OpTimer() {
    if (c->telemetry) {
      hipEventRecord(c->ev1, c->stream);
      hipEventSynchronize(c->ev1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, c->ev0, c->ev1);
      c->op_ms[op] += ms;
    }
  }
};

// the dW products a pipelined conv backward (TNS_OPT_BWD_OVERLAP = 2) left
// on the side stream: the context's stream waits for them from here on
int join_side(tns_ctx* c) {
  if (!c->side_pending) return TNS_OK;
  c->side_pending = false;
  c->pending.clear();
  c->side_slots = 0;
  hipError_t e = hipEventRecord(c->ev_join, c->aux_stream);
  if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, c->ev_join, 0);
  if (e != hipSuccess) return set_error(TNS_ERR_HIP, "backward join: %s", hipGetErrorString(e));
  return TNS_OK;
}

// every entry point: the context exists, and earlier calls' side-stream work
// is ordered before whatever this call enqueues
int check_ctx(tns_ctx* c, bool join = true) {
  if (!c) return set_error(TNS_ERR_ARG, "null tns_ctx");
  return join ? join_side(c) : TNS_OK;
}

// an operand's extent: n elements every |inc| from p (empty when p is null
// or n <= 0)
struct Span {
  uintptr_t lo = 0, hi = 0;
};
Span span(const float* p, int64_t n, int64_t inc = 1) {
  Span s;
  if (!p || n <= 0) return s;
  const int64_t a = inc < 0 ? -inc : (inc == 0 ? 1 : inc);
  s.lo = (uintptr_t)p;
  s.hi = (uintptr_t)(p + (n - 1) * a + 1);
  return s;
}
// a matrix operand of a (strided-batched) GEMM: rows x cols with leading
// dimension ld, batch copies every stride
Span span_mat(const float* p, int64_t rows, int64_t cols, int64_t ld, int64_t stride,
              int64_t batch) {
  if (rows <= 0 || cols <= 0 || batch <= 0) return Span{};
  return span(p, (batch - 1) * (stride > 0 ? stride : 0) + (rows - 1) * ld + cols);
}

// every non-conv entry point: the context exists, and — during a pipelined
// conv backward (TNS_OPT_BWD_OVERLAP = 2) — the side stream is joined only
// when this call's operands meet a pending dW's: it writes that dW's delta
// or input, or reads or writes its weight_updates / col workspace.  Calls
// that touch none of them (the shortcut's addvv between two conv layers, a
// route's copies, an upsample) leave the dW products running
int check_ops(tns_ctx* c, std::initializer_list<Span> writes, std::initializer_list<Span> reads) {
  if (!c) return set_error(TNS_ERR_ARG, "null tns_ctx");
  if (!c->side_pending) return TNS_OK;
  auto meet = [](const Span& a, uintptr_t lo, uintptr_t hi) {
    return a.lo < a.hi && lo < hi && a.lo < hi && lo < a.hi;
  };
  for (const tns_ctx::PendingDw& d : c->pending)
    for (int y = 0; y < 2; ++y) {
      for (const Span& w : writes)
        if (meet(w, d.lo[y], d.hi[y]) || meet(w, d.wlo[y], d.whi[y])) return join_side(c);
      for (const Span& r : reads)
        if (meet(r, d.wlo[y], d.whi[y])) return join_side(c);
    }
  return TNS_OK;
}

int hip_status(hipError_t e, const char* what) {
  if (e != hipSuccess) return set_error(TNS_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
  return TNS_OK;
}

int beta_mode_for(float beta) {
  if (beta == 1.0f) return BETA_ONE;
  if (beta == 0.0f && !g_strict_beta0) return BETA_ZERO;
  return BETA_SCALE;
}

int do_gemm(tns_ctx* c, bool ta, bool tb, int64_t M, int64_t N, int64_t K, float alpha,
            const float* A, int64_t lda, int64_t sA, const float* B, int64_t ldb, int64_t sB,
            float beta, float* C, int64_t ldc, int64_t sC, int64_t batch, int epi,
            const float* bias, int act, bool c_write_only = false, int variant = -1) {
  if (M < 0 || N < 0 || K < 0 || batch < 0)
    return set_error(TNS_ERR_ARG, "gemm: negative dimension");
  if (M == 0 || N == 0 || batch == 0) return TNS_OK;
  // leading dimensions, row-major (cblas_sgemm conventions)
  const int64_t minlda = ta ? M : K, minldb = tb ? K : N;
  if ((K > 0 && (lda < (minlda > 1 ? minlda : 1) || ldb < (minldb > 1 ? minldb : 1))) ||
      ldc < N)
    return set_error(TNS_ERR_ARG, "gemm: leading dimension too small (lda=%lld ldb=%lld ldc=%lld)",
                     (long long)lda, (long long)ldb, (long long)ldc);
  if (!C || (K > 0 && (!A || !B))) return set_error(TNS_ERR_ARG, "gemm: null operand");
  if (epi == EPI_BIAS_ACT && (!bias || !act_supported(act)))
    return set_error(TNS_ERR_ARG, "gemm: bad fused epilogue");
  GemmArgs a{};
  a.M = M; a.N = N; a.K = K;
  a.alpha = alpha; a.beta = beta;
  a.beta_mode = (c_write_only && beta == 0.0f) ? BETA_ZERO : beta_mode_for(beta);
  a.A = A; a.lda = lda; a.strideA = sA;
  a.B = B; a.ldb = ldb; a.strideB = sB;
  a.C = C; a.ldc = ldc; a.strideC = sC;
  a.batch = batch; a.epi = epi; a.bias = bias; a.act = act;
  OpTimer t(c, TNS_OP_GEMM);
  if (!ta && tb && g_nt_sdot && variant < 0 && epi == EPI_NONE)
    return hip_status(launch_sgemm_nt_sdot(a, c->stream), "sgemm_nt launch");
  if (ta && tb && g_tt_exact && variant < 0 && epi == EPI_NONE)
    return hip_status(launch_sgemm_tt(a, c->stream), "sgemm_tt launch");
  hipError_t e = launch_sgemm_variant(variant, a, ta, tb, c->stream);
  if (e == hipErrorInvalidValue && variant >= 0)
    return set_error(TNS_ERR_UNSUPPORTED, "gemm variant %d (%s) does not support this problem",
                     variant, sgemm_variant_name(variant));
  return hip_status(e, "sgemm launch");
}

ConvGeom geom(int64_t C, int64_t H, int64_t W, int64_t kH, int64_t kW, int64_t pH, int64_t pW,
              int64_t sY, int64_t sX, int64_t dY, int64_t dX) {
  ConvGeom g;
  g.C = C; g.H = H; g.W = W; g.kH = kH; g.kW = kW; g.padH = pH; g.padW = pW;
  g.sY = sY; g.sX = sX; g.dY = dY; g.dX = dX;
  g.oh = out_dim(H, pH, kH, dY, sY);
  g.ow = out_dim(W, pW, kW, dX, sX);
  return g;
}

int check_geom(const ConvGeom& g) {
  if (g.C < 0 || g.H < 0 || g.W < 0 || g.kH <= 0 || g.kW <= 0 || g.sY <= 0 || g.sX <= 0 ||
      g.dY <= 0 || g.dX <= 0 || g.padH < 0 || g.padW < 0)
    return set_error(TNS_ERR_ARG, "im2col: invalid geometry");
  // kernel indexing is 32-bit inside one plane (image plane, col row) and
  // over the col rows; offsets of planes and rows are 64-bit
  if (g.C * g.kH * g.kW > 0x7fffffffLL || (g.oh > 0 ? g.oh : 1) * (g.ow > 0 ? g.ow : 1) >
      0x7fffffffLL || g.H * g.W > 0x7fffffffLL)
    return set_error(TNS_ERR_ARG, "im2col: image too large for 32-bit indexing");
  return TNS_OK;
}

// k-table of an implicit-GEMM convolution over Hp x Wp padded images, built
// once per geometry on the context's stream (stream order makes it visible to
// the GEMM that follows)
int get_ktab(tns_ctx* c, int64_t C, int64_t Hp, int64_t Wp, int64_t kH, int64_t kW, int64_t dY,
             int64_t dX, const int** out) {
  auto key = std::make_tuple(C, Hp, Wp, kH, kW, dY, dX);
  auto it = c->ktabs.find(key);
  if (it != c->ktabs.end()) {
    *out = it->second;
    return TNS_OK;
  }
  const int64_t K = C * kH * kW;
  int* t = nullptr;
  hipError_t e = hipMalloc(&t, (size_t)(K + KTAB_PAD) * 2 * sizeof(int));
  if (e != hipSuccess)
    return set_error(TNS_ERR_NOMEM, "hipMalloc(k-table) failed: %s", hipGetErrorString(e));
  e = launch_build_ktab(t, (int)C, (int)Hp, (int)Wp, (int)kH, (int)kW, (int)dY, (int)dX,
                        c->stream);
  if (e != hipSuccess) {
    hipFree(t);
    return set_error(TNS_ERR_HIP, "k-table launch failed: %s", hipGetErrorString(e));
  }
  c->ktabs.emplace(key, t);
  *out = t;
  return TNS_OK;
}

// ---- default context for the host-pointer API (boundary A) ---------------
std::once_flag g_default_once;
tns_ctx* g_default = nullptr;
int g_default_status = TNS_OK;

tns_ctx* default_ctx() {
  std::call_once(g_default_once, [] {
    int dev = 0;
    hipGetDevice(&dev);
    g_default_status = tns_hip_create(dev, &g_default);
  });
  return g_default_status == TNS_OK ? g_default : nullptr;
}


// ---- boundary A: the host-pointer GEMM pipeline ----------------------------
// Operands arrive in host memory.  On the MI355X box PCIe moves ~56 GB/s in
// either direction and no more with both at once (pageable and pinned alike;
// scripts/pcie_probe.py, profiles/r02_pcie.json), so the copies bound the call
// and the GEMM is hidden under them: the call is cut into chunks — rows of C
// for a single GEMM (B, which every row needs, goes first), whole GEMMs for a
// batch — and chunk j computes on the context's stream while chunk j+1
// uploads and chunk j-1 downloads on the copy stream.  Device operands keep
// the host layout (same element offsets) in context scratch; C is copied
// back row by row (2-D copies) so host gaps between rows / GEMMs are never
// overwritten.
struct HostGemm {
  bool ta, tb;
  int64_t M, N, K;
  float alpha, beta;
  const float* A;
  int64_t lda, sA;
  const float* B;
  int64_t ldb, sB;
  float* C;
  int64_t ldc, sC;
  int64_t batch;
};

int64_t span_of(int64_t rows, int64_t ld, int64_t cols) {
  return rows > 0 && cols > 0 ? (rows - 1) * ld + cols : 0;
}

// rows x cols sub-matrix with row pitch ld, same element offsets on both sides
hipError_t copy_rows(float* dst, const float* src, int64_t rows, int64_t cols, int64_t ld,
                     hipMemcpyKind kind, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  if (cols == ld || rows == 1)
    return hipMemcpyAsync(dst, src, (size_t)span_of(rows, ld, cols) * 4, kind, s);
  return hipMemcpy2DAsync(dst, (size_t)ld * 4, src, (size_t)ld * 4, (size_t)cols * 4,
                          (size_t)rows, kind, s);
}

// GEMMs [b0, b1) of a strided operand (rows x cols, pitch ld, stride st)
hipError_t copy_batch(float* dst, const float* src, int64_t b0, int64_t b1, int64_t rows,
                      int64_t cols, int64_t ld, int64_t st, hipMemcpyKind kind, hipStream_t s) {
  const int64_t one = span_of(rows, ld, cols);
  if (b1 <= b0 || one == 0) return hipSuccess;
  const bool dense = (cols == ld || rows == 1) && (st == one || b1 - b0 == 1);
  if (dense)
    return hipMemcpyAsync(dst + b0 * st, src + b0 * st, (size_t)((b1 - b0 - 1) * st + one) * 4,
                          kind, s);
  for (int64_t b = b0; b < b1; ++b)
    if (hipError_t e = copy_rows(dst + b * st, src + b * st, rows, cols, ld, kind, s)) return e;
  return hipSuccess;
}

int ensure_copy_stream(tns_ctx* c, int nev) {
  if (!c->copy_stream)
    TNS_HIP_TRY(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
  while ((int)c->pipe_ev.size() < nev) {
    hipEvent_t e;
    TNS_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->pipe_ev.push_back(e);
  }
  return TNS_OK;
}

int host_gemm_pipeline(tns_ctx* c, const HostGemm& g, int64_t R, float* dA, float* dB, float* dC,
                       const float* dA_pre, const float* dB_pre, int64_t oneA, int64_t oneB,
                       hipStream_t cs, hipStream_t ks);

// dA_pre / dB_pre: device copies of a shared (stride 0) operand already on this
// context's device (multi-device broadcast), or nullptr
int host_gemm(tns_ctx* c, const HostGemm& g, const float* dA_pre, const float* dB_pre) {
  std::lock_guard<std::mutex> lk(c->mu);
  TNS_HIP_TRY(hipSetDevice(c->device));
  const int64_t a_rows = g.ta ? g.K : g.M, a_cols = g.ta ? g.M : g.K;
  const int64_t b_rows = g.tb ? g.N : g.K, b_cols = g.tb ? g.K : g.N;
  const int64_t oneA = span_of(a_rows, g.lda, a_cols), oneB = span_of(b_rows, g.ldb, b_cols);
  const int64_t oneC = span_of(g.M, g.ldc, g.N);
  // one block of A / B serving every chunk: B of a single GEMM (chunked by
  // rows of C, which need all of B) and stride-0 operands of a batch
  const bool sharedA = g.sA == 0 || g.batch == 1, sharedB = g.sB == 0 || g.batch == 1;
  const int64_t nA = sharedA ? oneA : (g.batch - 1) * g.sA + oneA;
  const int64_t nB = sharedB ? oneB : (g.batch - 1) * g.sB + oneB;
  const int64_t nC = (g.batch - 1) * g.sC + oneC;
  float *dA = nullptr, *dB = nullptr, *dC = nullptr;
  if (!dA_pre && oneA)
    if (int r = ensure_scratch(c, SLOT_STAGE1, nA, &dA)) return r;
  if (!dB_pre && oneB)
    if (int r = ensure_scratch(c, SLOT_STAGE2, nB, &dB)) return r;
  if (int r = ensure_scratch(c, SLOT_STAGE3, nC, &dC)) return r;
  // chunks: rows of C for one GEMM (>= 512 rows each, at most 4), GEMMs for
  // a batch (at most 16)
  const bool by_rows = g.batch == 1;
  int64_t R = by_rows ? std::min<int64_t>(4, std::max<int64_t>(1, g.M / 512))
                      : std::min<int64_t>(16, g.batch);
  if (int r = ensure_copy_stream(c, (int)(2 * R))) return r;
  hipStream_t cs = c->copy_stream, ks = c->stream;
  // every path out after the first copy is enqueued drains both streams: an
  // error must not leave an upload reading (or a download writing) the
  // caller's host buffers after the call has returned
  const int r = host_gemm_pipeline(c, g, R, dA, dB, dC, dA_pre, dB_pre, oneA, oneB, cs, ks);
  if (r != TNS_OK) {
    (void)hipStreamSynchronize(cs);
    (void)hipStreamSynchronize(ks);
  }
  return r;
}

int host_gemm_pipeline(tns_ctx* c, const HostGemm& g, int64_t R, float* dA, float* dB, float* dC,
                       const float* dA_pre, const float* dB_pre, int64_t oneA, int64_t oneB,
                       hipStream_t cs, hipStream_t ks) {
  const float* uA = dA_pre ? dA_pre : dA;
  const float* uB = dB_pre ? dB_pre : dB;
  const int64_t a_rows = g.ta ? g.K : g.M, a_cols = g.ta ? g.M : g.K;
  const int64_t b_rows = g.tb ? g.N : g.K, b_cols = g.tb ? g.K : g.N;
  const bool sharedA = g.sA == 0 || g.batch == 1, sharedB = g.sB == 0 || g.batch == 1;
  const bool upfrontA = g.sA == 0 && g.batch > 1;
  const bool by_rows = g.batch == 1;
  const int64_t units = by_rows ? g.M : g.batch;
  const bool needC = beta_mode_for(g.beta) != BETA_ZERO;
  const hipMemcpyKind H2D = hipMemcpyHostToDevice, D2H = hipMemcpyDeviceToHost;
  // shared operands first
  if (!dA_pre && upfrontA && oneA)
    TNS_HIP_TRY(copy_rows(dA, g.A, a_rows, a_cols, g.lda, H2D, cs));
  if (!dB_pre && sharedB && oneB)
    TNS_HIP_TRY(copy_rows(dB, g.B, b_rows, b_cols, g.ldb, H2D, cs));
  auto lo = [&](int64_t j) { return units * j / R; };
  auto download = [&](int64_t j) -> hipError_t {
    const int64_t u0 = lo(j), u1 = lo(j + 1);
    if (by_rows)
      return copy_rows(g.C + u0 * g.ldc, dC + u0 * g.ldc, u1 - u0, g.N, g.ldc, D2H, cs);
    return copy_batch(g.C, dC, u0, u1, g.M, g.N, g.ldc, g.sC, D2H, cs);
  };
  for (int64_t j = 0; j < R; ++j) {
    const int64_t u0 = lo(j), u1 = lo(j + 1);
    hipEvent_t up = c->pipe_ev[2 * j], done = c->pipe_ev[2 * j + 1];
    if (by_rows) {  // rows u0..u1 of C: rows of A (NoTrans) or its columns (Trans)
      if (!dA_pre && oneA) {
        if (g.ta)
          TNS_HIP_TRY(copy_rows(dA + u0, g.A + u0, g.K, u1 - u0, g.lda, H2D, cs));
        else
          TNS_HIP_TRY(copy_rows(dA + u0 * g.lda, g.A + u0 * g.lda, u1 - u0, g.K, g.lda, H2D, cs));
      }
      if (needC)
        TNS_HIP_TRY(copy_rows(dC + u0 * g.ldc, g.C + u0 * g.ldc, u1 - u0, g.N, g.ldc, H2D, cs));
    } else {
      if (!sharedA) TNS_HIP_TRY(copy_batch(dA, g.A, u0, u1, a_rows, a_cols, g.lda, g.sA, H2D, cs));
      if (!sharedB) TNS_HIP_TRY(copy_batch(dB, g.B, u0, u1, b_rows, b_cols, g.ldb, g.sB, H2D, cs));
      if (needC) TNS_HIP_TRY(copy_batch(dC, g.C, u0, u1, g.M, g.N, g.ldc, g.sC, H2D, cs));
    }
    TNS_HIP_TRY(hipEventRecord(up, cs));
    TNS_HIP_TRY(hipStreamWaitEvent(ks, up, 0));
    int r;
    if (by_rows)
      r = do_gemm(c, g.ta, g.tb, u1 - u0, g.N, g.K, g.alpha,
                  uA ? uA + (g.ta ? u0 : u0 * g.lda) : nullptr, g.lda, 0, uB, g.ldb, 0, g.beta,
                  dC + u0 * g.ldc, g.ldc, 0, 1, EPI_NONE, nullptr, 0);
    else
      r = do_gemm(c, g.ta, g.tb, g.M, g.N, g.K, g.alpha, uA ? uA + (sharedA ? 0 : u0 * g.sA) : nullptr,
                  g.lda, sharedA ? 0 : g.sA, uB ? uB + (sharedB ? 0 : u0 * g.sB) : nullptr, g.ldb,
                  sharedB ? 0 : g.sB, g.beta, dC + u0 * g.sC, g.ldc, g.sC, u1 - u0, EPI_NONE,
                  nullptr, 0);
    if (r) return r;
    TNS_HIP_TRY(hipEventRecord(done, ks));
    if (j > 0) {
      TNS_HIP_TRY(hipStreamWaitEvent(cs, c->pipe_ev[2 * j - 1], 0));
      TNS_HIP_TRY(download(j - 1));
    }
  }
  TNS_HIP_TRY(hipStreamWaitEvent(cs, c->pipe_ev[2 * R - 1], 0));
  TNS_HIP_TRY(download(R - 1));
  TNS_HIP_TRY(hipStreamSynchronize(cs));
  return TNS_OK;
}

// ---- several GPUs from one process (sgemm_strided_batched_multi)
// Slot i of a call owns a context on devices[i] (two slots may share a
// device); the batch is split into contiguous shards, the first batch % n
// slots one GEMM longer (tensorium_amd/shard.py, the reference's MP.&For
// blocks).  A shared operand (stride 0: the conv weights of
// nConvolutionLayer.pas:773) crosses PCIe once, to slot 0, and reaches the
// other devices by peer copies over xGMI.  Each slot runs the host pipeline
// above on its own host thread.
std::mutex g_pool_mu;
std::vector<tns_ctx*> g_pool;
std::mutex g_op_devices_mu;
std::vector<int32_t> g_op_devices;

int pool_ctx(int slot, int device, tns_ctx** out) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  if ((int)g_pool.size() <= slot) g_pool.resize(slot + 1, nullptr);
  if (g_pool[slot] && g_pool[slot]->device != device) {
    tns_hip_destroy(g_pool[slot]);
    g_pool[slot] = nullptr;
  }
  if (!g_pool[slot])
    if (int r = tns_hip_create(device, &g_pool[slot])) return r;
  *out = g_pool[slot];
  return TNS_OK;
}

int multi_host_gemm(const int32_t* devices, int n, const HostGemm& g) {
  std::vector<tns_ctx*> ctx(n);
  for (int i = 0; i < n; ++i)
    if (int r = pool_ctx(i, devices[i], &ctx[i])) return r;
  const int64_t a_rows = g.ta ? g.K : g.M, a_cols = g.ta ? g.M : g.K;
  const int64_t b_rows = g.tb ? g.N : g.K, b_cols = g.tb ? g.K : g.N;
  const int64_t oneA = span_of(a_rows, g.lda, a_cols), oneB = span_of(b_rows, g.ldb, b_cols);
  // shared operands: host -> slot 0 once, slot 0 -> every other slot by peer
  // copy; only the slots that get GEMMs (the first min(n, batch)) need them,
  // and with one such slot (a single GEMM: the op-table's plain gemm) there is
  // nothing to broadcast: slot 0 runs the ordinary pipeline, row-chunked
  // uploads included
  const int nwork = (int)std::min<int64_t>(n, g.batch);
  std::vector<const float*> preA(n, nullptr), preB(n, nullptr);
  auto broadcast = [&](const float* host, int64_t rows, int64_t cols, int64_t ld, int64_t elems,
                       int slot, std::vector<const float*>& pre) -> int {
    float* root;
    {
      std::lock_guard<std::mutex> lk(ctx[0]->mu);
      TNS_HIP_TRY(hipSetDevice(ctx[0]->device));
      if (int r = ensure_scratch(ctx[0], slot, elems, &root)) return r;
      TNS_HIP_TRY(copy_rows(root, host, rows, cols, ld, hipMemcpyHostToDevice, ctx[0]->stream));
      TNS_HIP_TRY(hipStreamSynchronize(ctx[0]->stream));
    }
    pre[0] = root;
    for (int i = 1; i < nwork; ++i) {
      std::lock_guard<std::mutex> lk(ctx[i]->mu);
      TNS_HIP_TRY(hipSetDevice(ctx[i]->device));
      float* d;
      if (int r = ensure_scratch(ctx[i], slot, elems, &d)) return r;
      if (ctx[i]->device == ctx[0]->device)
        TNS_HIP_TRY(hipMemcpyAsync(d, root, (size_t)elems * 4, hipMemcpyDeviceToDevice,
                                   ctx[i]->stream));
      else
        TNS_HIP_TRY(hipMemcpyPeerAsync(d, ctx[i]->device, root, ctx[0]->device,
                                       (size_t)elems * 4, ctx[i]->stream));
      TNS_HIP_TRY(hipStreamSynchronize(ctx[i]->stream));
      pre[i] = d;
    }
    return TNS_OK;
  };
  if (g.sA == 0 && oneA && nwork > 1)
    if (int r = broadcast(g.A, a_rows, a_cols, g.lda, oneA, SLOT_STAGE1, preA)) return r;
  if (g.sB == 0 && oneB && nwork > 1)
    if (int r = broadcast(g.B, b_rows, b_cols, g.ldb, oneB, SLOT_STAGE2, preB)) return r;
  std::vector<int> status(n, TNS_OK);
  std::vector<std::string> errs(n);
  std::vector<std::thread> th;
  const int64_t base = g.batch / n, extra = g.batch % n;
  for (int i = 0; i < n; ++i) {
    const int64_t s0 = i * base + std::min<int64_t>(i, extra);
    const int64_t cnt = base + (i < extra ? 1 : 0);
    if (cnt == 0) continue;
    HostGemm gi = g;
    gi.A = g.sA ? g.A + s0 * g.sA : g.A;
    gi.B = g.sB ? g.B + s0 * g.sB : g.B;
    gi.C = g.C + s0 * g.sC;
    gi.batch = cnt;
    th.emplace_back([&, i, gi] {
      status[i] = host_gemm(ctx[i], gi, preA[i], preB[i]);
      if (status[i]) errs[i] = g_err;  // the error string is thread-local
    });
  }
  for (auto& t : th) t.join();
  for (int i = 0; i < n; ++i)
    if (status[i]) return set_error(status[i], "slot %d (device %d): %s", i, devices[i],
                                    errs[i].c_str());
  return TNS_OK;
}

}  // namespace

extern "C" {

int tns_abi_version(void) { return TNS_ABI_VERSION; }
const char* tns_last_error(void) { return g_err.c_str(); }
void tns_clear_error(void) { g_err.clear(); }
void tns_set_error_hook(tns_error_hook_t hook) { g_hook = hook; }

int tns_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int tns_set_option(int32_t opt, int64_t value) {
  switch (opt) {
    case TNS_OPT_STRICT_BETA0:
      g_strict_beta0 = value ? 1 : 0;
      return TNS_OK;
    case TNS_OPT_CONV_VARIANT:
      g_conv_variant = value < 0 ? -1 : value;
      return TNS_OK;
    case TNS_OPT_CONV_PAD:
      g_conv_pad = value < 0 ? -1 : (value ? 1 : 0);
      return TNS_OK;
    case TNS_OPT_NT_SDOT:
      g_nt_sdot = value ? 1 : 0;
      return TNS_OK;
    case TNS_OPT_SRSS_QUIRK:
      g_srss_quirk = value ? 1 : 0;
      return TNS_OK;
    case TNS_OPT_TT_EXACT:
      g_tt_exact = value ? 1 : 0;
      return TNS_OK;
    case TNS_OPT_SDOT_FORM:
      if (value > sdot_chains_variant_count() &&
          (value < SDOT_FORM_RC || value >= SDOT_FORM_RC + sdot_rc_variant_count()))
        return set_error(TNS_ERR_ARG, "sdot form %lld out of range", (long long)value);
      set_sdot_form((int)value);
      return TNS_OK;
    case TNS_OPT_DX_FUSED:
      g_dx_fused = value < 0 ? 1 : (value > 2 ? 2 : value);
      return TNS_OK;
    case TNS_OPT_BWD_OVERLAP:
      g_bwd_overlap = value <= 0 ? 0 : (value >= 2 ? 2 : 1);
      return TNS_OK;
    case TNS_OPT_DW_TILE:
      if (value >= dw_tile_count()) return set_error(TNS_ERR_ARG, "no dW tile %lld", (long long)value);
      g_dw_tile = value < -1 ? -2 : value;
      return TNS_OK;
    case TNS_OPT_DX_TILE:
      if (value >= conv_tile4_ta_count()) return set_error(TNS_ERR_ARG, "no dX tile %lld", (long long)value);
      g_dx_tile = value < -1 ? -2 : value;
      return TNS_OK;
    case TNS_OPT_DW_RES:
      if (value >= dw_res_count()) return set_error(TNS_ERR_ARG, "no dW res form %lld", (long long)value);
      g_dw_res = value < -1 ? -2 : value;
      return TNS_OK;
    case TNS_OPT_DERIVE_SUMS:
      g_derive_sums = value ? 1 : 0;
      return TNS_OK;
    case TNS_OPT_SCRATCH_CAP:
      g_scratch_cap = value > 0 ? value : 0;
      return TNS_OK;
    case TNS_OPT_DX_CONV:
      if (value >= conv_tile4_dx3_count())
        return set_error(TNS_ERR_ARG, "no dX conv form %lld", (long long)value);
      g_dx_conv = value < -1 ? -2 : value;
      return TNS_OK;
    default:
      return set_error(TNS_ERR_ARG, "unknown option %d", opt);
  }
}

// ---- context ---------------------------------------------------------------
int tns_hip_create(int32_t deviceIndex, tns_ctx** out) {
  if (!out) return set_error(TNS_ERR_ARG, "tns_hip_create: null out");
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0)
    return set_error(TNS_ERR_HIP, "no HIP device available (%s)", hipGetErrorString(e));
  if (deviceIndex < 0 || deviceIndex >= n)
    return set_error(TNS_ERR_ARG, "device index %d out of range [0,%d)", deviceIndex, n);
  TNS_HIP_TRY(hipSetDevice(deviceIndex));
  tns_ctx* c = new tns_ctx();
  c->device = deviceIndex;
  {
    int least = 0, greatest = 0;
    const char* sp = getenv("TNS_STREAM_PRIO");  // (see ensure_side_stream)
    if (!(sp && sp[0] == '0') &&
        hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
      e = hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, greatest);
    else
      e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  }
  if (e != hipSuccess) {
    delete c;
    return set_error(TNS_ERR_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
  }
  c->own_stream = true;
  hipEventCreate(&c->ev0);
  hipEventCreate(&c->ev1);
  *out = c;
  return TNS_OK;
}

int tns_hip_destroy(tns_ctx* c) {
  if (!c) return TNS_OK;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->aux_stream) hipStreamSynchronize(c->aux_stream);
  if (c->ovl_stream) hipStreamSynchronize(c->ovl_stream);
  for (int i = 0; i < tns_ctx::kSlots; ++i)
    if (c->scratch[i]) hipFree(c->scratch[i]);
  for (auto& kv : c->ktabs) hipFree(kv.second);
  if (c->ev0) hipEventDestroy(c->ev0);
  if (c->ev1) hipEventDestroy(c->ev1);
  if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
  if (c->copy_stream) hipStreamDestroy(c->copy_stream);
  if (c->aux_stream) hipStreamDestroy(c->aux_stream);
  if (c->ovl_stream) hipStreamDestroy(c->ovl_stream);
  if (c->ev_fork) hipEventDestroy(c->ev_fork);
  if (c->ev_join) hipEventDestroy(c->ev_join);
  for (hipEvent_t e : c->pipe_ev) hipEventDestroy(e);
  delete c;
  return TNS_OK;
}

int tns_hip_set_stream(tns_ctx* c, void* s) {
  if (int r = check_ctx(c)) return r;
  if (c->own_stream && c->stream) {
    hipStreamSynchronize(c->stream);
    hipStreamDestroy(c->stream);
  }
  c->stream = (hipStream_t)s;
  c->own_stream = false;
  return TNS_OK;
}

void* tns_hip_get_stream(tns_ctx* c) {
  // (pipelined backward: work the caller enqueues on the stream must see
  // the pending dW products' weight_updates — join them first)
  if (!c || join_side(c)) return nullptr;
  return (void*)c->stream;
}

int tns_hip_pending_dw(tns_ctx* c) {
  if (!c) return -1;
  return c->side_pending ? (int)c->pending.size() : 0;
}

int tns_hip_finish(tns_ctx* c) {
  if (int r = check_ctx(c)) return r;
  return hip_status(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
}

int tns_hip_malloc(tns_ctx* c, int64_t n, float** out) {
  if (int r = check_ctx(c)) return r;
  if (!out || n < 0) return set_error(TNS_ERR_ARG, "tns_hip_malloc: bad args");
  hipError_t e = hipMalloc((void**)out, (size_t)(n > 0 ? n : 1) * sizeof(float));
  if (e != hipSuccess) return set_error(TNS_ERR_NOMEM, "hipMalloc: %s", hipGetErrorString(e));
  return TNS_OK;
}

int tns_hip_free(tns_ctx* c, float* p) {
  if (int r = check_ctx(c)) return r;
  return hip_status(hipFree(p), "hipFree");
}

int tns_hip_write_buffer(tns_ctx* c, float* dev, int64_t bytes, const void* host) {
  if (int r = check_ctx(c)) return r;
  if (bytes <= 0) return TNS_OK;
  TNS_HIP_TRY(hipMemcpyAsync(dev, host, (size_t)bytes, hipMemcpyHostToDevice, c->stream));
  return hip_status(hipStreamSynchronize(c->stream), "writeBuffer sync");
}

int tns_hip_read_buffer(tns_ctx* c, const float* dev, int64_t bytes, void* host) {
  if (int r = check_ctx(c)) return r;
  if (bytes <= 0) return TNS_OK;
  TNS_HIP_TRY(hipMemcpyAsync(host, dev, (size_t)bytes, hipMemcpyDeviceToHost, c->stream));
  return hip_status(hipStreamSynchronize(c->stream), "readBuffer sync");
}

// ---- boundary B: device API ---------------------------------------------------
int tns_hip_gemm(tns_ctx* c, uint8_t transA, uint8_t transB, int64_t M, int64_t N, int64_t K,
                 float ALPHA, const float* A, int64_t aOffset, int64_t lda, const float* B,
                 int64_t bOffset, int64_t ldb, float BETA, float* C, int64_t cOffset,
                 int64_t ldc) {
  if (int r = check_ops(c, {span_mat(C ? C + cOffset : nullptr, M, N, ldc, 0, 1)},
                        {transA ? span_mat(A ? A + aOffset : nullptr, K, M, lda, 0, 1)
                                : span_mat(A ? A + aOffset : nullptr, M, K, lda, 0, 1),
                         transB ? span_mat(B ? B + bOffset : nullptr, N, K, ldb, 0, 1)
                                : span_mat(B ? B + bOffset : nullptr, K, N, ldb, 0, 1)}))
    return r;
  return do_gemm(c, transA != 0, transB != 0, M, N, K, ALPHA, A ? A + aOffset : nullptr, lda, 0,
                 B ? B + bOffset : nullptr, ldb, 0, BETA, C ? C + cOffset : nullptr, ldc, 0, 1,
                 EPI_NONE, nullptr, 0);
}

int tns_hip_gemm_strided_batched(tns_ctx* c, uint8_t transA, uint8_t transB, int64_t M,
                                 int64_t N, int64_t K, float ALPHA, const float* A,
                                 int64_t aOffset, int64_t lda, int64_t strideA, const float* B,
                                 int64_t bOffset, int64_t ldb, int64_t strideB, float BETA,
                                 float* C, int64_t cOffset, int64_t ldc, int64_t strideC,
                                 int64_t batchCount) {
  if (int r = check_ops(
          c, {span_mat(C ? C + cOffset : nullptr, M, N, ldc, strideC, batchCount)},
          {transA ? span_mat(A ? A + aOffset : nullptr, K, M, lda, strideA, batchCount)
                  : span_mat(A ? A + aOffset : nullptr, M, K, lda, strideA, batchCount),
           transB ? span_mat(B ? B + bOffset : nullptr, N, K, ldb, strideB, batchCount)
                  : span_mat(B ? B + bOffset : nullptr, K, N, ldb, strideB, batchCount)}))
    return r;
  return do_gemm(c, transA != 0, transB != 0, M, N, K, ALPHA, A ? A + aOffset : nullptr, lda,
                 strideA, B ? B + bOffset : nullptr, ldb, strideB, BETA,
                 C ? C + cOffset : nullptr, ldc, strideC, batchCount, EPI_NONE, nullptr, 0);
}

int tns_hip_gemm_batched(tns_ctx* c, uint8_t transA, uint8_t transB, int64_t M, int64_t N,
                         int64_t K, float ALPHA, const float* const* A, int64_t aOffset,
                         int64_t lda, const float* const* B, int64_t bOffset, int64_t ldb,
                         float BETA, float* const* C, int64_t cOffset, int64_t ldc,
                         int64_t batchCount) {
  if (int r = check_ctx(c)) return r;
  if (batchCount < 0) return set_error(TNS_ERR_ARG, "gemmBatched: batchCount < 0");
  if (batchCount == 0) return TNS_OK;
  if (!A || !B || !C) return set_error(TNS_ERR_ARG, "gemmBatched: null pointer array");
  // The pointer arrays are read where they live (hipMemcpyDefault: device
  // arrays written by writeBuffer as nConvolutionLayer.pas:1083-1085 builds
  // them, or host arrays), in stream order after the work that wrote them.
  const size_t bytes = (size_t)batchCount * sizeof(void*);
  std::vector<const float*> pa(batchCount), pb(batchCount);
  std::vector<float*> pc(batchCount);
  TNS_HIP_TRY(hipSetDevice(c->device));
  TNS_HIP_TRY(hipMemcpyAsync(pa.data(), A, bytes, hipMemcpyDefault, c->stream));
  TNS_HIP_TRY(hipMemcpyAsync(pb.data(), B, bytes, hipMemcpyDefault, c->stream));
  TNS_HIP_TRY(hipMemcpyAsync(pc.data(), C, bytes, hipMemcpyDefault, c->stream));
  TNS_HIP_TRY(hipStreamSynchronize(c->stream));
  for (int64_t i = 0; i < batchCount; ++i)
    if (!pa[i] || !pb[i] || !pc[i])
      return set_error(TNS_ERR_ARG, "gemmBatched: null matrix pointer at entry %lld", (long long)i);
  // equally spaced entries (the common case: slices of one buffer) run as one
  // strided-batched launch; anything else GEMM by GEMM in array order
  auto stride_of = [&](auto& v, int64_t* st) {
    const intptr_t d = batchCount > 1 ? (const char*)v[1] - (const char*)v[0] : 0;
    if (d < 0 || d % (intptr_t)sizeof(float)) return false;
    for (int64_t i = 2; i < batchCount; ++i)
      if ((const char*)v[i] - (const char*)v[i - 1] != d) return false;
    *st = (int64_t)(d / (intptr_t)sizeof(float));
    return true;
  };
  // — only when the batch's GEMMs are independent: the C entries do not
  // overlap one another and no C entry overlaps an A or B entry (the launch
  // runs them concurrently; the loop below keeps the array order)
  const int64_t extA = transA ? (K - 1) * lda + M : (M - 1) * lda + K;
  const int64_t extB = transB ? (N - 1) * ldb + K : (K - 1) * ldb + N;
  const int64_t extC = (M - 1) * ldc + N;
  auto disjoint = [](const float* p, int64_t n, const float* q, int64_t m) {
    return p + n <= q || q + m <= p;
  };
  int64_t sA, sB, sC;
  if (stride_of(pa, &sA) && stride_of(pb, &sB) && stride_of(pc, &sC) &&
      (batchCount == 1 || sC >= extC) &&
      disjoint(pc[0] + cOffset, sC * (batchCount - 1) + extC, pa[0] + aOffset,
               sA * (batchCount - 1) + extA) &&
      disjoint(pc[0] + cOffset, sC * (batchCount - 1) + extC, pb[0] + bOffset,
               sB * (batchCount - 1) + extB))
    return do_gemm(c, transA != 0, transB != 0, M, N, K, ALPHA, pa[0] + aOffset, lda, sA,
                   pb[0] + bOffset, ldb, sB, BETA, pc[0] + cOffset, ldc, sC, batchCount, EPI_NONE,
                   nullptr, 0);
  for (int64_t i = 0; i < batchCount; ++i)
    if (int r = do_gemm(c, transA != 0, transB != 0, M, N, K, ALPHA, pa[i] + aOffset, lda, 0,
                        pb[i] + bOffset, ldb, 0, BETA, pc[i] + cOffset, ldc, 0, 1, EPI_NONE,
                        nullptr, 0))
      return r;
  return TNS_OK;
}

int tns_hip_im2col_strided_batched(tns_ctx* c, int64_t aChannels, int64_t aHeight,
                                   int64_t aWidth, int64_t kernelHeight, int64_t kernelWidth,
                                   int64_t padHeight, int64_t padWidth, int64_t strideY,
                                   int64_t strideX, int64_t dilationY, int64_t dilationX,
                                   const float* im, int64_t imStride, int64_t imOffset,
                                   float* col, int64_t colStride, int64_t colOffset,
                                   int64_t batchCount) {
  if (!c) return check_ctx(c);
  ConvGeom g = geom(aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight, padWidth,
                    strideY, strideX, dilationY, dilationX);
  if (int r = check_geom(g)) return r;
  if (!im || !col) return set_error(TNS_ERR_ARG, "im2col: null pointer");
  {
    const int64_t nb = batchCount > 0 ? batchCount : 0, colN = g.C * g.kH * g.kW * g.oh * g.ow;
    if (int r = check_ops(c, {span_mat(col + colOffset, 1, colN, colN, colStride, nb)},
                          {span_mat(im + imOffset, 1, g.C * g.H * g.W, 0, imStride, nb)}))
      return r;
  }
  OpTimer t(c, TNS_OP_IM2COL);
  return hip_status(launch_im2col(g, im + imOffset, imStride, col + colOffset, colStride,
                                  batchCount, c->stream),
                    "im2col launch");
}

int tns_hip_im2col(tns_ctx* c, int64_t aChannels, int64_t aHeight, int64_t aWidth,
                   int64_t kernelHeight, int64_t kernelWidth, int64_t padHeight, int64_t padWidth,
                   int64_t strideY, int64_t strideX, int64_t dilationY, int64_t dilationX,
                   const float* im, int64_t imOffset, float* col, int64_t colOffset) {
  return tns_hip_im2col_strided_batched(c, aChannels, aHeight, aWidth, kernelHeight, kernelWidth,
                                        padHeight, padWidth, strideY, strideX, dilationY,
                                        dilationX, im, 0, imOffset, col, 0, colOffset, 1);
}

int tns_hip_col2im_strided_batched(tns_ctx* c, int64_t aChannels, int64_t aHeight,
                                   int64_t aWidth, int64_t kernelHeight, int64_t kernelWidth,
                                   int64_t padHeight, int64_t padWidth, int64_t strideY,
                                   int64_t strideX, int64_t dilationY, int64_t dilationX,
                                   const float* col, int64_t colStride, int64_t colOffset,
                                   float* im, int64_t imStride, int64_t imOffset,
                                   int64_t batchCount) {
  if (!c) return check_ctx(c);
  ConvGeom g = geom(aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight, padWidth,
                    strideY, strideX, dilationY, dilationX);
  if (int r = check_geom(g)) return r;
  if (!im || !col) return set_error(TNS_ERR_ARG, "col2im: null pointer");
  {
    const int64_t nb = batchCount > 0 ? batchCount : 0, colN = g.C * g.kH * g.kW * g.oh * g.ow;
    if (int r = check_ops(c, {span_mat(im + imOffset, 1, g.C * g.H * g.W, 0, imStride, nb)},
                          {span_mat(col + colOffset, 1, colN, colN, colStride, nb)}))
      return r;
  }
  if (batchCount > 1 && imStride < aChannels * aHeight * aWidth)
    return set_error(TNS_ERR_ARG, "col2im: overlapping image strides");
  OpTimer t(c, TNS_OP_COL2IM);
  return hip_status(launch_col2im(g, col + colOffset, colStride, im + imOffset, imStride,
                                  batchCount, c->stream),
                    "col2im launch");
}

int tns_hip_col2im(tns_ctx* c, int64_t aChannels, int64_t aHeight, int64_t aWidth,
                   int64_t kernelHeight, int64_t kernelWidth, int64_t padHeight, int64_t padWidth,
                   int64_t strideY, int64_t strideX, int64_t dilationY, int64_t dilationX,
                   const float* col, int64_t colOffset, float* im, int64_t imOffset) {
  return tns_hip_col2im_strided_batched(c, aChannels, aHeight, aWidth, kernelHeight, kernelWidth,
                                        padHeight, padWidth, strideY, strideX, dilationY,
                                        dilationX, col, 0, colOffset, im, 0, imOffset, 1);
}

int tns_hip_forward_bias(tns_ctx* c, int64_t dstSize, float* dst, int64_t offset, int64_t srcSize,
                         const float* src, int64_t incb, int64_t batch) {
  if (int r = check_ops(c, {span(dst ? dst + offset : nullptr, dstSize)}, {span(src, srcSize, incb)}))
    return r;
  if (dstSize == 0) return TNS_OK;
  if (!dst || !src || srcSize <= 0 || batch <= 0 || dstSize % (srcSize * batch) != 0)
    return set_error(TNS_ERR_ARG, "forwardBias: sizes do not align");
  const int64_t bs = dstSize / (srcSize * batch);
  OpTimer t(c, TNS_OP_BIAS);
  return hip_status(launch_forward_bias(dst + offset, srcSize, bs, src, incb, batch, c->stream),
                    "forwardBias launch");
}

int tns_hip_backward_bias(tns_ctx* c, int64_t dstSize, float* dst, int64_t srcSize,
                          const float* src, int64_t srcOffset, int64_t incb, int64_t batch) {
  if (int r = check_ops(c, {span(dst, dstSize)}, {span(src ? src + srcOffset : nullptr, srcSize)}))
    return r;
  if (!dst || !src || dstSize <= 0 || batch <= 0 || srcSize % (dstSize * batch) != 0)
    return set_error(TNS_ERR_ARG, "backwardBias: sizes do not align");
  const int64_t bs = srcSize / (dstSize * batch);
  OpTimer t(c, TNS_OP_BIAS);
  if (bs == 1 && incb == 1)  // FC layers: the reference's sequential strided sum
    return hip_status(launch_add_sums(dst, src + srcOffset, batch, dstSize, 1, nullptr, c->stream),
                      "backwardBias launch");
  if (incb == 1 && bs >= 64) {  // conv blocks: lane chains per block
    float* part;
    if (int r = ensure_scratch(c, SLOT_BN, batch * dstSize, &part)) return r;
    return hip_status(launch_add_sums(dst, src + srcOffset, batch, dstSize, bs, part, c->stream),
                      "backwardBias launch");
  }
  return hip_status(launch_backward_bias(dst, dstSize, src + srcOffset, bs, batch, incb, c->stream),
                    "backwardBias launch");
}

int tns_hip_activate_array(tns_ctx* c, int64_t N, float* x, int64_t offset, int32_t activation) {
  if (int r = check_ops(c, {span(x ? x + offset : nullptr, N)}, {})) return r;
  if (!act_supported(activation))
    return set_error(TNS_ERR_UNSUPPORTED, "activation %d not implemented", activation);
  if (N <= 0) return TNS_OK;
  if (!x) return set_error(TNS_ERR_ARG, "activate: null pointer");
  OpTimer t(c, TNS_OP_ACTIVATE);
  return hip_status(launch_activate(x + offset, N, activation, c->stream), "activate launch");
}

int tns_hip_derive_array(tns_ctx* c, int64_t N, const float* x, int64_t offset,
                         int32_t activation, float* delta) {
  if (int r = check_ops(c, {span(delta, N)}, {span(x ? x + offset : nullptr, N)})) return r;
  if (!act_supported(activation))
    return set_error(TNS_ERR_UNSUPPORTED, "derivative %d not implemented", activation);
  if (N <= 0) return TNS_OK;
  if (!x || !delta) return set_error(TNS_ERR_ARG, "derive: null pointer");
  OpTimer t(c, TNS_OP_ACTIVATE);
  return hip_status(launch_derive(x + offset, N, activation, delta, c->stream), "derive launch");
}

int tns_hip_axpy(tns_ctx* c, int64_t N, float a, const float* x, int64_t xOffset, int64_t incx,
                 float* y, int64_t yOffset, int64_t incy) {
  if (int r = check_ops(c, {span(y ? y + yOffset : nullptr, N, incy)},
                        {span(x ? x + xOffset : nullptr, N, incx)}))
    return r;
  return hip_status(launch_axpy(N, a, x + xOffset, incx, y + yOffset, incy, c->stream), "axpy");
}

int tns_hip_sgd_update(tns_ctx* c, int64_t nWeights, float* weights, float* weight_updates,
                       int64_t n, float* biases, float* bias_updates, float* scales,
                       float* scale_updates, float lrOverBatch, float negDecayTimesBatch,
                       float momentum) {
  if (int r = check_ops(c, {span(weights, nWeights), span(weight_updates, nWeights), span(biases, n),
                            span(bias_updates, n), span(scales, n), span(scale_updates, n)},
                        {}))
    return r;
  if (nWeights < 0 || n < 0 || (nWeights > 0 && (!weights || !weight_updates)) ||
      (n > 0 && (!biases || !bias_updates)) || (!scales != !scale_updates))
    return set_error(TNS_ERR_ARG, "sgd_update: bad arguments");
  return hip_status(launch_sgd_update(nWeights, weights, weight_updates, n, biases, bias_updates,
                                      n > 0 ? scales : nullptr, scale_updates, lrOverBatch,
                                      negDecayTimesBatch, momentum, c->stream),
                    "sgd_update");
}

int tns_hip_scale(tns_ctx* c, int64_t N, float a, float* x, int64_t stride) {
  if (int r = check_ops(c, {span(x, N, stride)}, {})) return r;
  return hip_status(launch_scale(N, a, x, stride, c->stream), "scale");
}

int tns_hip_fill(tns_ctx* c, int64_t N, float* x, int64_t offset, float val, int64_t stride) {
  if (int r = check_ops(c, {span(x ? x + offset : nullptr, N, stride)}, {})) return r;
  return hip_status(launch_fill(N, x + offset, val, stride, c->stream), "fill");
}

int tns_hip_copy(tns_ctx* c, int64_t N, const float* src, int64_t srcOffset, int64_t inca,
                 float* dst, int64_t dstOffset, int64_t incb) {
  if (int r = check_ops(c, {span(dst ? dst + dstOffset : nullptr, N, incb)},
                        {span(src ? src + srcOffset : nullptr, N, inca)}))
    return r;
  return hip_status(launch_copy(N, src + srcOffset, inca, dst + dstOffset, incb, c->stream),
                    "copy");
}

int tns_hip_shortcut(tns_ctx* c, int64_t N, const float* a, int64_t aOffset, const float* b,
                     int64_t bOffset, float* out, int64_t outOffset, int32_t activation) {
  if (int r = check_ops(c, {span(out ? out + outOffset : nullptr, N)},
                        {span(a ? a + aOffset : nullptr, N), span(b ? b + bOffset : nullptr, N)}))
    return r;
  if (N < 0 || (N > 0 && (!a || !b || !out))) return set_error(TNS_ERR_ARG, "shortcut: bad args");
  if (!act_supported(activation))
    return set_error(TNS_ERR_UNSUPPORTED, "activation %d not implemented", activation);
  return hip_status(launch_shortcut(N, a + aOffset, b + bOffset, out + outOffset, activation,
                                    c->stream),
                    "shortcut");
}

int tns_hip_upsample(tns_ctx* c, int64_t aBatch, int64_t aChannels, int64_t outHeight,
                     int64_t outWidth, float* in, int64_t stride, int32_t isForward, float scale,
                     float* out, int32_t zeroIn) {
  {
    const int64_t small = aBatch * aChannels * outHeight * outWidth, big = small * stride * stride;
    const Span si = span(in, small), so = span(out, big);
    if (int r = isForward ? check_ops(c, {so}, {si}) : check_ops(c, {si}, {so})) return r;
  }
  const int64_t planes = aBatch * aChannels, H = outHeight, W = outWidth;
  if (aBatch < 0 || aChannels < 0 || H < 0 || W < 0 || stride < 1 ||
      H * stride > 0x7fffffff || W * stride > 0x7fffffff ||
      (planes * H * W > 0 && (!in || !out)))
    return set_error(TNS_ERR_ARG, "upsample: bad args");
  if (isForward)
    return hip_status(launch_upsample(planes, (int)H, (int)W, (int)stride, scale, in, out,
                                      c->stream),
                      "upsample");
  return hip_status(launch_upsample_backward(planes, (int)H, (int)W, (int)stride, scale, in, out,
                                             zeroIn, c->stream),
                    "upsample backward");
}

// TNNCuda.addvv / subvv / mulvv / fmavv / fmavss / inverseSqrt (nncuda.pas:120-151)
namespace {
int vv(tns_ctx* c, int op, int64_t N, const float* a, int64_t aOff, int64_t inca, const float* b,
       int64_t bOff, int64_t incb, const float* cc, int64_t cOff, int64_t incc, float* d,
       int64_t dOff, int64_t incd, const char* what) {
  if (int r = check_ops(c, {span(d ? d + dOff : nullptr, N, incd)},
                        {span(a ? a + aOff : nullptr, N, inca), span(b ? b + bOff : nullptr, N, incb),
                         span(cc ? cc + cOff : nullptr, N, incc)}))
    return r;
  if (N < 0 || (N > 0 && (!a || !b || !d || (op == 3 && !cc))))
    return set_error(TNS_ERR_ARG, "%s: bad args", what);
  return hip_status(launch_vv(op, N, a + aOff, inca, b + bOff, incb, cc ? cc + cOff : nullptr,
                              incc, d + dOff, incd, c->stream),
                    what);
}
}  // namespace

int tns_hip_addvv(tns_ctx* c, int64_t N, const float* src1, int64_t src1Offset, int64_t inca,
                  const float* src2, int64_t src2Offset, int64_t incb, float* dst,
                  int64_t dstOffset, int64_t incc) {
  return vv(c, 0, N, src1, src1Offset, inca, src2, src2Offset, incb, nullptr, 0, 0, dst,
            dstOffset, incc, "addvv");
}

int tns_hip_subvv(tns_ctx* c, int64_t N, const float* src1, int64_t src1Offset, int64_t inca,
                  const float* src2, int64_t src2Offset, int64_t incb, float* dst,
                  int64_t dstOffset, int64_t incc) {
  return vv(c, 1, N, src1, src1Offset, inca, src2, src2Offset, incb, nullptr, 0, 0, dst,
            dstOffset, incc, "subvv");
}

int tns_hip_mulvv(tns_ctx* c, int64_t N, const float* src1, int64_t src1Offset, int64_t inca,
                  const float* src2, int64_t src2Offset, int64_t incb, float* dst,
                  int64_t dstOffset, int64_t incc) {
  return vv(c, 2, N, src1, src1Offset, inca, src2, src2Offset, incb, nullptr, 0, 0, dst,
            dstOffset, incc, "mulvv");
}

int tns_hip_fmavv(tns_ctx* c, int64_t N, const float* src1, int64_t src1Offset, int64_t inca,
                  const float* src2, int64_t src2Offset, int64_t incb, const float* src3,
                  int64_t src3Offset, int64_t incc, float* dst, int64_t dstOffset,
                  int64_t incd) {
  return vv(c, 3, N, src1, src1Offset, inca, src2, src2Offset, incb, src3, src3Offset, incc, dst,
            dstOffset, incd, "fmavv");
}

int tns_hip_fmavss(tns_ctx* c, int64_t N, const float* src, int64_t offset, float scalar,
                   float bias, float* dst) {
  if (int r = check_ops(c, {span(dst ? dst + offset : nullptr, N)},
                        {span(src ? src + offset : nullptr, N)}))
    return r;
  if (N < 0 || (N > 0 && (!src || !dst))) return set_error(TNS_ERR_ARG, "fmavss: bad args");
  return hip_status(launch_fmavss(N, src + offset, scalar, bias, dst + offset, c->stream),
                    "fmavss");
}

int tns_hip_inverse_sqrt(tns_ctx* c, int64_t N, float alpha, const float* src, float* dst,
                         int64_t stride, int64_t offset) {
  (void)alpha;  // unused by the reference kernel too
  if (int r = check_ops(c, {span(dst ? dst + offset : nullptr, N, stride)},
                        {span(src ? src + offset : nullptr, N, stride)}))
    return r;
  if (N < 0 || stride < 1 || (N > 0 && (!src || !dst)))
    return set_error(TNS_ERR_ARG, "inverseSqrt: bad args");
  return hip_status(launch_inverse_sqrt(N, src + offset, dst + offset, stride, c->stream),
                    "inverseSqrt");
}

int tns_hip_sgemm_strided_batched_multi(const int32_t* devices, int32_t n, uint8_t transA,
                                        uint8_t transB, int64_t M, int64_t N, int64_t K,
                                        float alpha, const float* A, int64_t lda,
                                        int64_t strideA, const float* B, int64_t ldb,
                                        int64_t strideB, float beta, float* C, int64_t ldc,
                                        int64_t strideC, int64_t batchCount) {
  if (!devices || n <= 0) return set_error(TNS_ERR_ARG, "sgemm_multi: no devices");
  const int nd = tns_device_count();
  for (int i = 0; i < n; ++i)
    if (devices[i] < 0 || devices[i] >= nd)
      return set_error(TNS_ERR_ARG, "sgemm_multi: device %d out of range [0,%d)", devices[i], nd);
  if (M < 0 || N < 0 || K < 0 || batchCount < 0)
    return set_error(TNS_ERR_ARG, "sgemm_multi: negative dimension");
  if (M == 0 || N == 0 || batchCount == 0) return TNS_OK;
  if (!C || (K > 0 && (!A || !B))) return set_error(TNS_ERR_ARG, "sgemm_multi: null operand");
  HostGemm g{transA != 0, transB != 0, M, N, K, alpha, beta, A, lda, strideA, B, ldb, strideB,
             C, ldc, strideC, batchCount};
  return multi_host_gemm(devices, n, g);
}

int tns_set_op_devices(const int32_t* devices, int32_t n) {
  const int nd = tns_device_count();
  for (int i = 0; i < n; ++i)
    if (!devices || devices[i] < 0 || devices[i] >= nd)
      return set_error(TNS_ERR_ARG, "set_op_devices: bad device list");
  std::lock_guard<std::mutex> lk(g_op_devices_mu);
  g_op_devices.assign(devices, devices + (n > 0 ? n : 0));
  return TNS_OK;
}

int tns_hip_yolo_forward(tns_ctx* c, int64_t batch, int64_t anchors, int64_t classes, int64_t hw,
                         const float* in, float* out) {
  {
    const int64_t n = batch * anchors * (classes + 5) * hw;
    if (int r = check_ops(c, {span(out, n)}, {span(in, n)})) return r;
  }
  if (batch < 0 || anchors < 0 || classes < 0 || hw < 0 ||
      (batch * anchors * hw > 0 && (!in || !out)))
    return set_error(TNS_ERR_ARG, "yolo: bad args");
  return hip_status(launch_yolo(batch, (int)anchors, (int)classes, hw, in, out, c->stream), "yolo");
}

int tns_hip_clamp(tns_ctx* c, int64_t N, float alpha, const float* src, float* dst,
                  int64_t stride, int64_t offset) {
  if (int r = check_ops(c, {span(dst ? dst + offset : nullptr, N, stride)},
                        {span(src ? src + offset : nullptr, N, stride)}))
    return r;
  return hip_status(launch_clamp(N, alpha, src + offset, dst + offset, stride, c->stream),
                    "clamp");
}

// ---- batch norm / softmax ------------------------------------------------------
namespace {
int blocks_of(int64_t total, int64_t channels, int64_t groups, int64_t* bs, const char* what) {
  if (channels <= 0 || groups <= 0 || total < 0 || total % (channels * groups) != 0)
    return set_error(TNS_ERR_ARG, "%s: sizes do not align (total=%lld channels=%lld groups=%lld)",
                     what, (long long)total, (long long)channels, (long long)groups);
  *bs = total / (channels * groups);
  return TNS_OK;
}
}  // namespace

int tns_hip_means_and_vars(tns_ctx* c, int64_t srcSize, int64_t dstSize, int64_t groups,
                           const float* src, int64_t offset, float* means, float* vars) {
  if (int r = check_ops(c, {span(means, dstSize), span(vars, dstSize)},
                        {span(src ? src + offset : nullptr, srcSize)}))
    return r;
  int64_t bs;
  if (int r = blocks_of(srcSize, dstSize, groups, &bs, "meansAndVars")) return r;
  if (!src || !means || !vars) return set_error(TNS_ERR_ARG, "meansAndVars: null pointer");
  float* part;
  if (int r = ensure_scratch(c, SLOT_BN, 2 * groups * dstSize, &part)) return r;
  return hip_status(launch_means_vars(src + offset, groups, dstSize, bs, means, vars,
                                      (int)g_srss_quirk, part, c->stream),
                    "meansAndVars");
}

int tns_hip_means(tns_ctx* c, int64_t srcSize, int64_t dstSize, int64_t groups,
                  const float* src, int64_t offset, float* means) {
  if (int r = check_ops(c, {span(means, dstSize)}, {span(src ? src + offset : nullptr, srcSize)}))
    return r;
  int64_t bs;
  if (int r = blocks_of(srcSize, dstSize, groups, &bs, "means")) return r;
  if (!src || !means) return set_error(TNS_ERR_ARG, "means: null pointer");
  float* part;
  if (int r = ensure_scratch(c, SLOT_BN, 2 * groups * dstSize, &part)) return r;
  return hip_status(launch_means_vars(src + offset, groups, dstSize, bs, means, nullptr,
                                      (int)g_srss_quirk, part, c->stream, 1),
                    "means");
}

int tns_hip_variances(tns_ctx* c, int64_t srcSize, int64_t dstSize, int64_t groups,
                      const float* src, int64_t offset, const float* means, float* vars) {
  if (int r = check_ops(c, {span(vars, dstSize)},
                        {span(src ? src + offset : nullptr, srcSize), span(means, dstSize)}))
    return r;
  int64_t bs;
  if (int r = blocks_of(srcSize, dstSize, groups, &bs, "variances")) return r;
  if (!src || !means || !vars) return set_error(TNS_ERR_ARG, "variances: null pointer");
  float* part;
  if (int r = ensure_scratch(c, SLOT_BN, 2 * groups * dstSize, &part)) return r;
  return hip_status(launch_means_vars(src + offset, groups, dstSize, bs,
                                      const_cast<float*>(means), vars, (int)g_srss_quirk, part,
                                      c->stream, 2),
                    "variances");
}

int tns_hip_normalize(tns_ctx* c, int64_t srcSize, int64_t dstSize, int64_t groups,
                      const float* means, int64_t meansStride, const float* vars,
                      int64_t varsStride, float* dst, int64_t dstOffset) {
  if (int r = check_ops(c, {span(dst ? dst + dstOffset : nullptr, dstSize)},
                        {span(means, srcSize, meansStride), span(vars, srcSize, varsStride)}))
    return r;
  int64_t bs;
  if (int r = blocks_of(dstSize, srcSize, groups, &bs, "normalize")) return r;
  if (!dst || !means || !vars) return set_error(TNS_ERR_ARG, "normalize: null pointer");
  return hip_status(launch_normalize(dst + dstOffset, groups, srcSize, bs, means, meansStride,
                                     vars, varsStride, c->stream),
                    "normalize");
}

int tns_hip_forward_scale(tns_ctx* c, int64_t dstSize, float* dst, int64_t offset,
                          int64_t scaleSize, const float* scale, int64_t incb, int64_t batch) {
  return tns_hip_forward_scale_add(c, dstSize, dst, offset, scaleSize, scale, nullptr, incb,
                                   batch);
}

int tns_hip_forward_scale_add(tns_ctx* c, int64_t dstSize, float* dst, int64_t offset,
                              int64_t scaleSize, const float* scales, const float* biases,
                              int64_t incb, int64_t batch) {
  if (int r = check_ops(c, {span(dst ? dst + offset : nullptr, dstSize)},
                        {span(scales, scaleSize, incb), span(biases, scaleSize, incb)}))
    return r;
  int64_t bs;
  if (int r = blocks_of(dstSize, scaleSize, batch, &bs, "forwardScale")) return r;
  if (!dst || !scales) return set_error(TNS_ERR_ARG, "forwardScale: null pointer");
  return hip_status(launch_scale_add(dst + offset, batch, scaleSize, bs, scales, biases, incb,
                                     c->stream),
                    "forwardScale");
}

int tns_hip_means_and_vars_delta(tns_ctx* c, int64_t srcSize, int64_t dstSize, int64_t groups,
                                 const float* delta, const float* x, int64_t offset,
                                 const float* mean, const float* variance, float* mean_delta,
                                 float* variance_delta) {
  if (int r = check_ops(c, {span(mean_delta, dstSize), span(variance_delta, dstSize)},
                        {span(delta ? delta + offset : nullptr, srcSize),
                         span(x ? x + offset : nullptr, srcSize), span(mean, dstSize),
                         span(variance, dstSize)}))
    return r;
  int64_t bs;
  if (int r = blocks_of(srcSize, dstSize, groups, &bs, "meansAndVarsDelta")) return r;
  if (!delta || !x || !mean || !variance || !mean_delta || !variance_delta)
    return set_error(TNS_ERR_ARG, "meansAndVarsDelta: null pointer");
  float* part;
  if (int r = ensure_scratch(c, SLOT_BN, 2 * groups * dstSize, &part)) return r;
  return hip_status(launch_mean_var_delta(delta + offset, x + offset, mean, variance, groups,
                                          dstSize, bs, mean_delta, variance_delta,
                                          (int)g_srss_quirk, part, c->stream),
                    "meansAndVarsDelta");
}

int tns_hip_normalize_delta(tns_ctx* c, int64_t deltaSize, int64_t meanSize, int64_t groups,
                            float* delta, const float* x, int64_t offset, const float* mean,
                            const float* variance, const float* mean_delta,
                            const float* variance_delta) {
  if (int r = check_ops(c, {span(delta ? delta + offset : nullptr, deltaSize)},
                        {span(x ? x + offset : nullptr, deltaSize), span(mean, meanSize),
                         span(variance, meanSize), span(mean_delta, meanSize),
                         span(variance_delta, meanSize)}))
    return r;
  int64_t bs;
  if (int r = blocks_of(deltaSize, meanSize, groups, &bs, "normalizeDelta")) return r;
  if (!delta || !x || !mean || !variance || !mean_delta || !variance_delta)
    return set_error(TNS_ERR_ARG, "normalizeDelta: null pointer");
  return hip_status(launch_normalize_delta(x + offset, mean, variance, mean_delta,
                                           variance_delta, delta + offset, groups, meanSize, bs,
                                           c->stream),
                    "normalizeDelta");
}

int tns_hip_add_dots(tns_ctx* c, int64_t N, int64_t dstSize, int64_t groups, const float* src1,
                     const float* src2, int64_t srcOffset, float* dst) {
  if (int r = check_ops(c, {span(dst, dstSize)},
                        {span(src1 ? src1 + srcOffset : nullptr, N),
                         span(src2 ? src2 + srcOffset : nullptr, N)}))
    return r;
  int64_t bs;
  if (int r = blocks_of(N, dstSize, groups, &bs, "addDots")) return r;
  if (!dst || !src1 || !src2) return set_error(TNS_ERR_ARG, "addDots: null pointer");
  float* part;
  if (int r = ensure_scratch(c, SLOT_BN, 2 * groups * dstSize, &part)) return r;
  return hip_status(launch_add_dots(dst, src1 + srcOffset, src2 + srcOffset, groups, dstSize, bs,
                                    part, c->stream),
                    "addDots");
}

int tns_hip_softmax_batch(tns_ctx* c, int64_t N, const float* input, int64_t iOffset,
                          int64_t batch, int64_t batch_size, int64_t groups, int64_t group_size,
                          int64_t stride, float temp, float* output, int64_t oOffset) {
  if (int r = check_ops(c, {span(output ? output + oOffset : nullptr, N)},
                        {span(input ? input + iOffset : nullptr, N)}))
    return r;
  if (!input || !output || N < 0) return set_error(TNS_ERR_ARG, "softmaxBatch: bad args");
  return hip_status(launch_softmax_batch(N, input + iOffset, batch, batch_size, groups,
                                         group_size, stride, temp, output + oOffset, c->stream),
                    "softmaxBatch");
}

int tns_hip_cross_entropy_softmax(tns_ctx* c, int64_t N, const float* pred, const float* truth,
                                  float* delta, float* error) {
  if (int r = check_ops(c, {span(delta, N), span(error, N)}, {span(pred, N), span(truth, N)}))
    return r;
  if (!pred || !truth || !delta || !error) return set_error(TNS_ERR_ARG, "xent: null pointer");
  return hip_status(launch_xent_softmax(N, pred, truth, delta, error, c->stream), "xent");
}

int tns_hip_sum(tns_ctx* c, int64_t N, const float* src, int64_t offset, float* out) {
  if (int r = check_ops(c, {span(out, 1)}, {span(src ? src + offset : nullptr, N)})) return r;
  if (!src || !out || N < 0) return set_error(TNS_ERR_ARG, "sum: bad args");
  return hip_status(launch_vssum(N, src + offset, out, c->stream), "sum");
}

int64_t tns_mlp_buffer_floats(int32_t nlayers, const int64_t* widths, int32_t bn, int64_t batch) {
  if (nlayers <= 0 || nlayers > 32 || !widths) return -1;
  return mlp_buffer_floats(nlayers, widths, bn, batch);
}

int tns_hip_mlp_train_step(tns_ctx* c, int32_t nlayers, const int64_t* widths,
                           const int32_t* acts, int32_t bn, int64_t batch, const float* X,
                           const float* truth, float learningRate, float momentum, float decay,
                           float* buf, float* cost) {
  if (int r = check_ctx(c)) return r;
  if (nlayers <= 0 || nlayers > MLP_MAX_LAYERS || !widths || !acts || !X || !truth || !buf ||
      !cost)
    return set_error(TNS_ERR_ARG, "mlp_train_step: bad arguments");
  if (batch < 2) return set_error(TNS_ERR_ARG, "mlp_train_step: batch must be >= 2 (BN)");
  MlpArgs a;
  a.nlayers = nlayers;
  int64_t omax = 0;
  for (int l = 0; l <= nlayers; ++l) {
    if (widths[l] <= 0) return set_error(TNS_ERR_ARG, "mlp_train_step: width %d <= 0", l);
    a.widths[l] = widths[l];
    if (l > 0 && widths[l] > omax) omax = widths[l];
  }
  if (9 * batch * omax > 40960)
    return set_error(TNS_ERR_ARG, "mlp_train_step: 9*batch*max(width) exceeds LDS staging");
  // (the kernels index a layer's weights and activations with 32-bit ints)
  for (int l = 0; l < nlayers; ++l)
    if (widths[l] * widths[l + 1] > 0x7fffffffLL)
      return set_error(TNS_ERR_ARG, "mlp_train_step: layer %d has %lld weights (32-bit indexing)",
                       l, (long long)(widths[l] * widths[l + 1]));
  if (batch * widths[0] > 0x7fffffffLL)
    return set_error(TNS_ERR_ARG, "mlp_train_step: batch x input width exceeds 32-bit indexing");
  for (int l = 0; l < nlayers; ++l) {
    if (!act_supported(acts[l]))
      return set_error(TNS_ERR_UNSUPPORTED, "mlp_train_step: activation %d", acts[l]);
    a.acts[l] = acts[l];
  }
  a.bn = bn != 0;
  a.batch = batch;
  a.X = X;
  a.truth = truth;
  a.lr = learningRate;
  a.momentum = momentum;
  a.decay = decay;
  a.buf = buf;
  a.cost = cost;
  // layer 0's residue partials (8 x batch x widths[1]), handed from the
  // layer-0 forward launch to the fused one
  if (int r = ensure_scratch(c, SLOT_MLP, 8 * batch * widths[1], &a.l0part)) return r;
  return hip_status(launch_mlp_train_step(a, c->stream), "mlp_train_step");
}

// ---- layer drivers ------------------------------------------------------------
int tns_hip_conv2d(tns_ctx* c, int64_t batch, int64_t C, int64_t H, int64_t W,
                   const float* input, const float* weights, int64_t filters, int64_t kH,
                   int64_t kW, int64_t wPadding, int64_t hPadding, int64_t xStride,
                   int64_t yStride, int64_t xDilation, int64_t yDilation, float* workspace,
                   float* out) {
  if (int r = check_ctx(c)) return r;
  // ntensors.pas:8266-8269: negative padding => "same"-style default
  if (wPadding < 0) wPadding = xDilation + kW / 2 - 1;
  if (hPadding < 0) hPadding = yDilation + kH / 2 - 1;
  // Conv2D hands (xDilation, yDilation) to im2col's (dilationY, dilationX)
  // slots (ntensors.pas:8303); keep the swap so non-square dilation matches.
  ConvGeom g = geom(C, H, W, kH, kW, hPadding, wPadding, yStride, xStride, xDilation, yDilation);
  if (int r = check_geom(g)) return r;
  // output size as the layer computes it (nConvolutionLayer.pas:92-100)
  const int64_t oh = out_dim(H, hPadding, kH, yDilation, yStride);
  const int64_t ow = out_dim(W, wPadding, kW, xDilation, xStride);
  const int64_t outImg = oh * ow, kSize = kH * kW, k = C * kSize;
  if (oh <= 0 || ow <= 0 || batch <= 0) return TNS_OK;
  const float* Bp;
  int64_t strideB;
  if (kSize != 1 || xDilation * yDilation != 1 || xStride * yStride != 1) {
    strideB = k * outImg;
    float* ws = workspace;
    if (!ws)
      if (int r = ensure_scratch(c, 0, batch * strideB, &ws)) return r;
    {
      OpTimer t(c, TNS_OP_IM2COL);
      if (int r = hip_status(launch_im2col(g, input, C * H * W, ws, strideB, batch, c->stream),
                             "im2col launch"))
        return r;
    }
    Bp = ws;
  } else {
    strideB = C * H * W;
    Bp = input;
  }
  // one strided-batched launch with the weights shared (strideA = 0) — the
  // GPU path of nConvolutionLayer.pas:1078; beta = 0 as in Conv2D (8328)
  // The layer output is write-only here: beta = 0 does not read it (for any
  // finite previous contents this equals the reference's 0*C up to the sign
  // of an all-zero chain).
  return do_gemm(c, false, false, filters, outImg, k, 1.0f, weights, k, 0, Bp, outImg, strideB,
                 0.0f, out, outImg, outImg * filters, batch, EPI_NONE, nullptr, 0, true);
}

namespace {
// TConvolutionalLayer.forward's Conv2D, with forwardBias + activate fused into
// the GEMM epilogue (bias_act) or the bare convolution (the batch-norm path,
// whose statistics need the raw output)
int conv_forward_impl(tns_ctx* c, int64_t batch, int64_t C, int64_t H, int64_t W,
                      const float* input, const float* weights, const float* biases,
                      int64_t filters, int64_t kSize, int64_t stride, int64_t padding,
                      int64_t dilation, int32_t activation, float* workspace, float* out,
                      int32_t fused, bool bias_act) {
  const int64_t oh = out_dim(H, padding, kSize, dilation, stride);
  const int64_t ow = out_dim(W, padding, kSize, dilation, stride);
  if (!fused) {
    if (int r = tns_hip_conv2d(c, batch, C, H, W, input, weights, filters, kSize, kSize, padding,
                               padding, stride, stride, dilation, dilation, workspace, out))
      return r;
    if (!bias_act) return TNS_OK;
    OpTimer t(c, TNS_OP_BIAS);
    return hip_status(launch_bias_activate(out, filters, oh * ow, biases, batch, activation,
                                           c->stream),
                      "bias+activate launch");
  }
  if (fused < TNS_CONV_UNFUSED || fused > TNS_CONV_IMPLICIT)
    return set_error(TNS_ERR_ARG, "conv_forward: unknown schedule %d", fused);
  ConvGeom g = geom(C, H, W, kSize, kSize, padding, padding, stride, stride, dilation, dilation);
  if (int r = check_geom(g)) return r;
  const int64_t outImg = oh * ow, ks = kSize * kSize, k = C * ks;
  if (oh <= 0 || ow <= 0 || batch <= 0) return TNS_OK;
  const bool needs_col = ks != 1 || dilation != 1 || stride != 1;
  // TNS_CONV_FUSED: implicit GEMM (batch folded into N: one launch with the
  // tile shapes of pick_conv_variant, measured at or ahead of the per-image
  // GEMM on every YOLOv3 layer, 1x1 ones included)
  // (a padded 1x1/s1 convolution is left to the reference's direct path,
  // which ignores the padding — ntensors.pas:8286)
  const bool direct_ok = needs_col || padding == 0;
  // implicit-GEMM limits (32-bit buffer offsets within one image, k-table
  // entries, 16-bit window offsets); the library choice falls back to the
  // im2col schedule past them
  const int64_t img_max = C * (H + 2 * padding) * (W + 2 * padding);
  const bool fits = !(k > 0x0fffffffLL - KTAB_PAD || img_max * 4 > 0x7fffffffLL ||
                      (kSize - 1) * dilation >= 0x8000);
  const bool implicit =
      direct_ok && (fused == TNS_CONV_IMPLICIT || (fused == TNS_CONV_FUSED && fits));
  if (implicit) {
    // implicit GEMM: batch folded into N, B gathered from zero-padded images
    if (!input || !weights || !out || (bias_act && !biases))
      return set_error(TNS_ERR_ARG, "conv_forward: null operand");
    // short-k first layers (3-channel 3x3): the direct kernel, one HBM pass
    // (TNS_OPT_CONV_VARIANT >= 0 forces a GEMM tile instead)
    if (g_conv_variant < 0 && conv_direct_applies(C, kSize, filters)) {
      OpTimer t(c, TNS_OP_GEMM);
      return hip_status(launch_conv_direct(input, weights, bias_act ? biases : nullptr, out, batch,
                                           C, H, W, filters, kSize, stride, padding, dilation, oh,
                                           ow, activation, c->stream),
                        "direct conv launch");
    }
    // 1x1 / stride-1 layers straight from the input planes (conv1x1.hip)
    // where picked, or forced by TNS_OPT_CONV_VARIANT = 600 + v
    if (kSize == 1 && stride == 1 && padding == 0 && dilation == 1) {
      int cv = -1;
      if (g_conv_variant >= 600)
        cv = (int)(g_conv_variant - 600);
      else if (g_conv_variant < 0)
        cv = conv1x1_pick(filters, batch * outImg, k, outImg);
      if (cv >= 0) {
        {
          OpTimer t(c, TNS_OP_GEMM);
          const hipError_t e = launch_conv1x1(cv, weights, input, bias_act ? biases : nullptr, out,
                                              batch, filters, k, outImg,
                                              act_transcendental(activation) ? 4 : activation,
                                              c->stream);
          if (e == hipErrorInvalidValue)
            return set_error(TNS_ERR_UNSUPPORTED, "conv1x1 form %d does not fit this layer", cv);
          if (int r = hip_status(e, "conv1x1 launch")) return r;
        }
        if (bias_act && act_transcendental(activation)) {
          OpTimer t(c, TNS_OP_ACTIVATE);
          return hip_status(launch_activate(out, batch * filters * outImg, activation, c->stream),
                            "activate launch");
        }
        return TNS_OK;
      }
    } else if (g_conv_variant >= 600) {
      return set_error(TNS_ERR_UNSUPPORTED, "conv1x1 forms need a 1x1 stride-1 unpadded layer");
    }
    // the two-pass slab form (conv_slab.hip) where picked, or forced by
    // TNS_OPT_CONV_VARIANT = 500 + v
    {
      const int64_t N = batch * outImg;
      int sv = -1;
      if (g_conv_variant >= 500 && g_conv_variant < 600)
        sv = (int)(g_conv_variant - 500);
      else if (g_conv_variant < 0 && dilation == 1)
        sv = conv_slab_pick(filters, N, k, kSize);
      if (sv >= 0) {
        const int64_t need = conv_slab_floats(sv, N, k);
        if (need < 0) return set_error(TNS_ERR_ARG, "no conv slab form %d", sv);
        float* slab = nullptr;
        if (int r = ensure_scratch(c, SLOT_COL, need, &slab)) return r;
        ConvSlabArgs sa{};
        sa.input = input; sa.weights = weights; sa.bias = bias_act ? biases : nullptr; sa.out = out;
        sa.batch = batch; sa.C = C; sa.H = H; sa.W = W; sa.M = filters; sa.K = k; sa.ks = kSize;
        sa.stride = stride; sa.pad = padding; sa.dil = dilation; sa.ow = ow; sa.ohw = outImg;
        sa.act = act_transcendental(activation) ? 4 : activation;
        {
          OpTimer t(c, TNS_OP_GEMM);
          const hipError_t e = launch_conv_slab(sv, sa, slab, c->stream);
          if (e == hipErrorInvalidValue)
            return set_error(TNS_ERR_UNSUPPORTED, "conv slab form %d does not fit this layer", sv);
          if (int r = hip_status(e, "conv slab launch")) return r;
        }
        if (bias_act && act_transcendental(activation)) {
          OpTimer t(c, TNS_OP_ACTIVATE);
          return hip_status(launch_activate(out, batch * filters * outImg, activation, c->stream),
                            "activate launch");
        }
        return TNS_OK;
      }
    }
    // tiles with a bounds-checked gather from the unpadded images where they
    // apply: the LDS-DMA ring (conv_dma.hip), the ping-pong schedule
    // (conv_pp.hip) or the plane-sized lock-step tiles (conv_tile.hip);
    // TNS_OPT_CONV_VARIANT 400 + v forces conv_patch tile v (3x3 stride-1
    // pad-1 layers), 300 + v conv_dma tile v, 200 + v conv_pp
    // tile v, 100 + v conv_tile tile v, 0..99 the sgemm_kernel.hpp shapes
    {
      int tv = -1, pv = -1, dv = -1, ev = -1;
      const int64_t img0 = C * H * W;
      if ((kSize == 1 || kSize == 3) && k % 32 == 0 && img0 * 4 <= 0x7fffffffLL &&
          (g_conv_variant < 0 || g_conv_variant >= 100)) {
        GemmArgs probe{};
        probe.M = filters; probe.N = batch * outImg; probe.K = k;
        probe.conv_sY = (int)stride;
        probe.A = weights; probe.lda = k;
        const bool patch_ok = kSize == 3 && stride == 1 && padding == 1 && dilation == 1;
        if (g_conv_variant >= 400)
          ev = patch_ok ? (int)(g_conv_variant - 400) : -1;
        else if (g_conv_variant >= 300)
          dv = (int)(g_conv_variant - 300);
        else if (g_conv_variant >= 200)
          pv = (int)(g_conv_variant - 200);
        else if (g_conv_variant >= 100)
          tv = (int)(g_conv_variant - 100);
        else if ((dv = conv_dma_pick(probe, (int)kSize)) < 0)
          tv = conv_tile_pick(probe, (int)kSize);
      }
      if (pv >= 0) tv = 1000 + pv;
      if (dv >= 0) tv = 2000 + dv;
      if (ev >= 0) tv = 3000 + ev;
      if (g_conv_variant >= 400 && ev < 0)
        return set_error(TNS_ERR_UNSUPPORTED, "conv_patch needs a 3x3 stride-1 pad-1 layer");
      if (tv >= 0) {
        // forms reading A from the slot-ordered weights: permute them first
        const float* wA = weights;
        if (tv < 1000 && conv_tile_is_ap(tv)) {
          float* wp = nullptr;
          if (int r = ensure_scratch(c, SLOT_WPERM, filters * k, &wp)) return r;
          OpTimer t(c, TNS_OP_GEMM);
          if (int r = hip_status(conv_tile4_permute(weights, wp, filters, k, c->stream),
                                 "weight permute launch"))
            return r;
          wA = wp;
        }
        const int64_t chunk = std::max<int64_t>(
            1, std::min<int64_t>(0x7fffffffLL / (4 * img0),
                                 0x7fffffffLL / std::max<int64_t>(outImg, 1)));
        for (int64_t b0 = 0; b0 < batch; b0 += chunk) {
          const int64_t nb = std::min(chunk, batch - b0);
          GemmArgs a{};
          a.M = filters; a.N = nb * outImg; a.K = k;
          a.alpha = 1.0f; a.beta = 0.0f; a.beta_mode = BETA_ZERO;
          a.A = wA; a.lda = k; a.strideA = 0;
          a.B = input + b0 * img0; a.ldb = outImg; a.strideB = img0;
          a.C = out + b0 * outImg * filters; a.ldc = outImg; a.strideC = outImg * filters;
          a.batch = 1; a.epi = bias_act ? EPI_BIAS_ACT : EPI_NONE; a.bias = biases;
          a.act = act_transcendental(activation) ? 4 : activation;
          a.conv = 2;
          a.conv_H = (int)H; a.conv_W = (int)W; a.conv_ow = (int)ow; a.conv_ohw = (int)outImg;
          a.conv_sY = (int)stride; a.conv_sX = (int)stride;
          a.conv_pH = (int)padding; a.conv_pW = (int)padding;
          a.conv_bytes = (int)(4 * nb * img0);
          OpTimer t(c, TNS_OP_GEMM);
          hipError_t e =
              tv >= 3000 ? launch_conv_patch(tv - 3000, a, c->stream)
              : tv >= 2000 ? launch_conv_dma(tv - 2000, a, (int)kSize, (int)dilation, c->stream)
              : tv >= 1000 ? launch_conv_pp(tv - 1000, a, (int)kSize, (int)dilation, c->stream)
                           : launch_conv_tile(tv, a, (int)kSize, (int)dilation, c->stream);
          if (e == hipErrorInvalidValue)
            return set_error(TNS_ERR_UNSUPPORTED, "conv tile %d does not fit this layer", tv);
          if (int r = hip_status(e, "conv tile launch")) return r;
        }
        if (bias_act && act_transcendental(activation)) {
          OpTimer t(c, TNS_OP_ACTIVATE);
          return hip_status(launch_activate(out, batch * filters * outImg, activation, c->stream),
                            "activate launch");
        }
        return TNS_OK;
      }
    }
    // Materialise the zero border (padded images, no bounds checks in the
    // GEMM) when that copy costs under ~5% of the GEMM: copy time
    // ~bytes/4 TB/s vs GEMM ~flops/80 TF/s.
    const double flops = 2.0 * (double)filters * (double)(batch * outImg) * (double)k;
    const int64_t Hpad = H + 2 * padding, Wpad = W + 2 * padding;
    const bool padded = padding == 0 ||
                        (g_conv_pad < 0 ? 8.0 * (double)(batch * C * Hpad * Wpad) * 400.0 < flops
                                        : g_conv_pad == 1);
    const int64_t Hs = padded ? Hpad : H, Ws = padded ? Wpad : W, img = C * Hs * Ws;
    // (k-table: 8-byte entries in one buffer resource, window offsets packed
    // in 16 bits)
    if (k > 0x0fffffffLL - KTAB_PAD || img * 4 > 0x7fffffffLL || (kSize - 1) * dilation >= 0x8000)
      return set_error(TNS_ERR_ARG, "conv_forward: image too large for the implicit GEMM");
    const int* kt = nullptr;
    if (int r = get_ktab(c, C, Hs, Ws, kSize, kSize, dilation, dilation, &kt)) return r;
    const float* src = input;
    if (padded && padding > 0) {
      float* pbuf = nullptr;
      if (int r = ensure_scratch(c, 1, batch * img, &pbuf)) return r;
      OpTimer t(c, TNS_OP_IM2COL);
      if (int r = hip_status(launch_pad_images(input, batch, C, H, W, padding, padding, pbuf,
                                               c->stream), "pad launch"))
        return r;
      src = pbuf;
    }
    // buffer offsets are 32-bit: images per launch such that the B extent
    // stays below 2^31 bytes (and N below 2^31)
    const int64_t chunk = std::max<int64_t>(
        1, std::min<int64_t>(0x7fffffffLL / (4 * img), 0x7fffffffLL / std::max<int64_t>(outImg, 1)));
    for (int64_t b0 = 0; b0 < batch; b0 += chunk) {
      const int64_t nb = std::min(chunk, batch - b0);
      GemmArgs a{};
      a.M = filters; a.N = nb * outImg; a.K = k;
      a.alpha = 1.0f; a.beta = 0.0f; a.beta_mode = BETA_ZERO;
      a.A = weights; a.lda = k; a.strideA = 0;
      a.B = src + b0 * img; a.ldb = outImg; a.strideB = img;
      a.C = out + b0 * outImg * filters; a.ldc = outImg; a.strideC = outImg * filters;
      a.batch = 1; a.epi = bias_act ? EPI_BIAS_ACT : EPI_NONE; a.bias = biases;
      a.act = act_transcendental(activation) ? 4 : activation;
      a.conv = padded ? 1 : 2; a.ktab = kt; a.ktab_n = (int)(k + KTAB_PAD);
      a.conv_H = (int)Hs; a.conv_W = (int)Ws; a.conv_ow = (int)ow; a.conv_ohw = (int)outImg;
      a.conv_sY = (int)stride; a.conv_sX = (int)stride;
      a.conv_pH = padded ? 0 : (int)padding; a.conv_pW = a.conv_pH;
      a.conv_bytes = (int)(4 * nb * img);
      OpTimer t(c, TNS_OP_GEMM);
      // (99: the sgemm_kernel.hpp shape heuristic, bypassing conv_tile)
      hipError_t e = launch_sgemm_conv_variant(g_conv_variant == 99 ? -1 : (int)g_conv_variant,
                                               a, c->stream);
      if (e == hipErrorInvalidValue)
        return set_error(TNS_ERR_UNSUPPORTED, "conv variant %lld unsupported",
                         (long long)g_conv_variant);
      if (int r = hip_status(e, "implicit conv launch")) return r;
    }
    if (bias_act && act_transcendental(activation)) {
      OpTimer t(c, TNS_OP_ACTIVATE);
      return hip_status(launch_activate(out, batch * filters * outImg, activation, c->stream),
                        "activate launch");
    }
    return TNS_OK;
  }
  const float* Bp;
  int64_t strideB;
  if (needs_col) {
    strideB = k * outImg;
    float* ws = workspace;
    if (!ws)
      if (int r = ensure_scratch(c, 0, batch * strideB, &ws)) return r;
    {
      OpTimer t(c, TNS_OP_IM2COL);
      if (int r = hip_status(launch_im2col(g, input, C * H * W, ws, strideB, batch, c->stream),
                             "im2col launch"))
        return r;
    }
    Bp = ws;
  } else {
    strideB = C * H * W;
    Bp = input;
  }
  // conv GEMM with forwardBias + activate fused into the epilogue
  // (logistic / tanh: bias in the epilogue, activation in its own pass)
  const bool transc = act_transcendental(activation);
  if (int r = do_gemm(c, false, false, filters, outImg, k, 1.0f, weights, k, 0, Bp, outImg,
                      strideB, 0.0f, out, outImg, outImg * filters, batch,
                      bias_act ? EPI_BIAS_ACT : EPI_NONE, biases, transc ? 4 : activation, true))
    return r;
  if (!transc || !bias_act) return TNS_OK;
  OpTimer t(c, TNS_OP_ACTIVATE);
  return hip_status(launch_activate(out, batch * filters * outImg, activation, c->stream),
                    "activate launch");
}
}  // namespace

int tns_hip_conv_forward(tns_ctx* c, int64_t batch, int64_t C, int64_t H, int64_t W,
                         const float* input, const float* weights, const float* biases,
                         int64_t filters, int64_t kSize, int64_t stride, int64_t padding,
                         int64_t dilation, int32_t activation, float* workspace, float* out,
                         int32_t fused) {
  if (int r = check_ctx(c)) return r;
  if (!act_supported(activation))
    return set_error(TNS_ERR_UNSUPPORTED, "activation %d not implemented", activation);
  return conv_forward_impl(c, batch, C, H, W, input, weights, biases, filters, kSize, stride,
                           padding, dilation, activation, workspace, out, fused, true);
}

int tns_hip_conv_forward_train(tns_ctx* c, int64_t batch, int64_t C, int64_t H, int64_t W,
                               const float* input, const float* weights, int64_t filters,
                               int64_t kSize, int64_t stride, int64_t padding, int64_t dilation,
                               int32_t activation, const float* scales, const float* biases,
                               float* rolling_mean, float* rolling_variance, float bnMomentum,
                               int32_t training, float* mean, float* variance, float* x,
                               float* x_norm, float* workspace, float* out) {
  if (int r = check_ctx(c)) return r;
  if (!act_supported(activation))
    return set_error(TNS_ERR_UNSUPPORTED, "activation %d not implemented", activation);
  if (!scales || !biases || !rolling_mean || !rolling_variance || !out ||
      (training && (!mean || !variance || !x || !x_norm)))
    return set_error(TNS_ERR_ARG, "conv_forward_train: null operand");
  const int64_t oh = out_dim(H, padding, kSize, dilation, stride);
  const int64_t ow = out_dim(W, padding, kSize, dilation, stride);
  if (oh <= 0 || ow <= 0 || batch <= 0 || filters <= 0) return TNS_OK;
  const int64_t bs = oh * ow;
  // state.input.Conv2D(weights, output, ...) (nConvolutionLayer.pas:508)
  if (int r = conv_forward_impl(c, batch, C, H, W, input, weights, nullptr, filters, kSize,
                                stride, padding, dilation, activation, workspace, out,
                                TNS_CONV_FUSED, false))
    return r;
  OpTimer t(c, TNS_OP_BIAS);
  if (!training)  // blockNormalize with the rolling statistics, scale, bias, activate
    return hip_status(launch_bn_apply(out, nullptr, nullptr, out, batch, filters, bs,
                                      rolling_mean, rolling_variance, scales, biases, activation,
                                      c->stream),
                      "batchNorm launch");
  float* part;
  if (int r = ensure_scratch(c, SLOT_BN, 2 * batch * filters, &part)) return r;
  if (int r = hip_status(launch_means_vars(out, batch, filters, bs, mean, variance,
                                           (int)g_srss_quirk, part, c->stream),
                         "meansAndVars launch"))
    return r;
  if (int r = hip_status(launch_rolling_update(filters, rolling_mean, rolling_variance, mean,
                                               variance, bnMomentum, c->stream),
                         "rolling update launch"))
    return r;
  return hip_status(launch_bn_apply(out, x, x_norm, out, batch, filters, bs, mean, variance,
                                    scales, biases, activation, c->stream),
                    "batchNorm launch");
}

namespace {
struct ConvBN {  // batchNormBack operands (nbaselayer.pas:372-395); scales == nullptr: none
  const float *scales, *x, *x_norm, *mean, *variance;
  float *scale_updates, *mean_delta, *variance_delta;
};

int conv_backward_impl(tns_ctx* c, int64_t batch, int64_t C, int64_t H, int64_t W,
                       const float* input, const float* weights, int64_t filters, int64_t kSize,
                       int64_t stride, int64_t padding, int64_t dilation, int32_t activation,
                       const float* output, float* delta, float* bias_updates,
                       float* weight_updates, float* workspace, float* state_delta,
                       const ConvBN& bn) {
  // (pipelined mode: this call's dW queues behind the pending ones on the
  // side stream; its other work touches none of their operands)
  if (!c) return check_ctx(c);
  bool pipe = g_bwd_overlap == 2 && !c->telemetry && ensure_side_stream(c);
  if (int r = check_ctx(c, !pipe)) return r;
  if (!act_supported(activation))
    return set_error(TNS_ERR_UNSUPPORTED, "activation %d not implemented", activation);
  // delta / output are [batch][filters][outH*outW] with the layer's outH =
  // (h + 2p - k) div s + 1 (nConvolutionLayer.pas:92-100); the backward
  // im2col / col2im pad with padding*dilation (640, 665), which yields those
  // columns for the "same" paddings at any dilation — other geometries make
  // the reference read past its workspace and are refused
  ConvGeom g = geom(C, H, W, kSize, kSize, padding * dilation, padding * dilation, stride, stride,
                    dilation, dilation);
  if (int r = check_geom(g)) return r;
  if (g.oh != (H + 2 * padding - kSize) / stride + 1 ||
      g.ow != (W + 2 * padding - kSize) / stride + 1)
    return set_error(TNS_ERR_UNSUPPORTED,
                     "conv_backward: dilation %lld with padding %lld gives %lldx%lld im2col "
                     "columns but the layer's output is %lldx%lld (nConvolutionLayer.pas:92-100, "
                     "640)",
                     (long long)dilation, (long long)padding, (long long)g.oh, (long long)g.ow,
                     (long long)((H + 2 * padding - kSize) / stride + 1),
                     (long long)((W + 2 * padding - kSize) / stride + 1));
  const int64_t i_m = filters, i_n = kSize * kSize * C, i_k = g.oh * g.ow;
  const int64_t colSize = i_n * i_k;
  if (batch <= 0 || i_k <= 0 || filters <= 0) return TNS_OK;
  if (!input || !weights || !output || !delta || !weight_updates || (!bn.scales && !bias_updates))
    return set_error(TNS_ERR_ARG, "conv_backward: null operand");
  if (bn.scales && (!bn.x || !bn.x_norm || !bn.mean || !bn.variance || !bn.scale_updates ||
                    !bn.mean_delta || !bn.variance_delta))
    return set_error(TNS_ERR_ARG, "conv_backward: null batch-norm operand");
  if (pipe) {
    // this call writes delta (in place) and state.delta on the context's
    // stream: if a pending dW reads either (an earlier call on the same
    // layers, e.g. the previous pass), the side stream is joined first (no
    // per-call event: the join is only paid where the ranges meet)
    // (the same test as every other entry point's, over this call's
    // context-stream operands; its own dW queues on the side stream)
    const int64_t nf = bn.scales ? filters : 0;
    if (int r = check_ops(c,
                          {span(delta, batch * filters * i_k), span(state_delta, batch * C * H * W),
                           span(bias_updates, bn.scales ? 0 : filters), span(bn.scale_updates, nf),
                           span(bn.mean_delta, nf), span(bn.variance_delta, nf)},
                          {span(output, batch * filters * i_k), span(weights, filters * i_n),
                           span(bn.x, nf ? batch * filters * i_k : 0),
                           span(bn.x_norm, nf ? batch * filters * i_k : 0),
                           span(bn.scales, nf), span(bn.mean, nf), span(bn.variance, nf)}))
      return r;
  }
  float* part;
  if (int r = ensure_scratch(c, SLOT_BN, 3 * batch * filters, &part)) return r;
  // batchNormBack's five passes as one chain pass over delta, output, x_norm
  // and x (the three reductions) + normalizeDelta deriving and scaling each
  // term as it loads it, where the chain kernels apply
  hipError_t fe = hipErrorNotSupported;
  if (bn.scales && g_bn_fused)
    fe = launch_bn_backward_fused(bn.scale_updates, bn.x_norm, delta, output, activation, bn.x,
                                  bn.mean, bn.variance, bn.scales, bn.mean_delta,
                                  bn.variance_delta, batch, filters, i_k, (int)g_srss_quirk, part,
                                  c->stream);
  if (fe != hipErrorNotSupported) {
    if (int r = hip_status(fe, "batchNormBack launch")) return r;
  } else if (bn.scales) {
    // Derivative(): delta *= f'(output), then batchNormBack:
    // scale_updates.addDots(x_norm, delta); delta.forwardScale(scales);
    // MeansAndVarsDelta; normalizeDelta — and no bias_updates term
    // (nConvolutionLayer.pas:601-604).  Three passes instead of five: the
    // derive rides addDots' loads (each derived term written back), and the
    // scale is applied to each delta term as MeansAndVarsDelta and
    // normalizeDelta load it (the same one rounding forwardScale would store)
    if (int r = hip_status(launch_add_dots_derive(bn.scale_updates, bn.x_norm, delta, output,
                                                  activation, batch, filters, i_k, part,
                                                  c->stream),
                           "derive + addDots launch"))
      return r;
    const float* fold = bn_folds_scale(i_k) ? bn.scales : nullptr;
    if (!fold)
      if (int r = hip_status(launch_scale_add(delta, batch, filters, i_k, bn.scales, nullptr, 1,
                                              c->stream), "forwardScale launch"))
        return r;
    if (int r = hip_status(launch_mean_var_delta(delta, bn.x, bn.mean, bn.variance, batch, filters,
                                                 i_k, bn.mean_delta, bn.variance_delta,
                                                 (int)g_srss_quirk, part, c->stream, fold),
                           "meansAndVarsDelta launch"))
      return r;
    if (int r = hip_status(launch_normalize_delta(bn.x, bn.mean, bn.variance, bn.mean_delta,
                                                  bn.variance_delta, delta, batch, filters, i_k,
                                                  c->stream, fold), "normalizeDelta launch"))
      return r;
  } else {
    // Derivative(): delta *= f'(output), then bias_updates.addSums(delta) —
    // one pass (each derived term written back as it enters the sums' chains)
    if (g_derive_sums) {
      if (int r = hip_status(launch_derive_add_sums(bias_updates, delta, output, activation, batch,
                                                    filters, i_k, part, c->stream),
                             "derive + addSums launch"))
        return r;
    } else {
      if (int r = hip_status(launch_derive(output, batch * filters * i_k, activation, delta,
                                           c->stream), "derive launch"))
        return r;
      if (int r = hip_status(launch_add_sums(bias_updates, delta, batch, filters, i_k, part,
                                             c->stream), "addSums launch"))
        return r;
    }
  }
  // state.input.im2Col(...) — a 1x1/s1/p0 col matrix is the input itself
  const bool needs_col = kSize != 1 || stride != 1 || padding != 0 || dilation != 1;
  // state.delta of stride-1 layers without the col matrix (conv_dx.hip)
  // state.delta of a 1x1 / stride-1 layer as a 1x1 convolution of the delta
  // planes with W^T on conv1x1.hip, the col2im add in its epilogue (the same
  // chains and the same add as the TN product with EPI_ADD)
  const int dx1 = state_delta && g_dx_c1 && g_dx_fused != 2 && kSize == 1 && stride == 1 &&
                          padding == 0 && dilation == 1
                      ? conv1x1_pick(C, batch * i_k, filters, i_k)
                      : -1;
  const bool fused_dx =
      dx1 < 0 && state_delta && dilation == 1 &&
      ((g_dx_fused == 1 && conv_dx_fused_applies(C, H, W, kSize, stride, filters, g.oh, g.ow)) ||
       (g_dx_fused == 2 && conv_dx_fused_fits(C, H, W, stride, filters, g.oh, g.ow)));
  // dW with the im2col matrix generated inside the sdot-order product
  // (dw_tile.hip): no col matrix, no im2col pass
  DwArgs da{};
  int dwv = -1;
  if (g_nt_sdot && g_dw_tile != -2 && (kSize == 1 || kSize == 3) &&
      C * H * W < (1LL << 27) && i_n <= 0x7fffffffLL && i_k <= 0x7fffffffLL && batch <= 65535) {
    da.delta = delta; da.x = input; da.part = nullptr;
    da.M = (int)i_m; da.N = (int)i_n; da.HW = (int)i_k;
    da.C = (int)C; da.H = (int)H; da.W = (int)W; da.oW = (int)g.ow;
    da.stride = (int)stride; da.pad = (int)(padding * dilation); da.dil = (int)dilation;
    da.va = i_k % 4 == 0 && (reinterpret_cast<uintptr_t>(delta) & 15) == 0;
    da.alpha = 1.0f;
    da.strideA = i_m * i_k; da.strideX = C * H * W; da.strideP = i_m * i_n; da.batch = batch;
    dwv = g_dw_tile >= 0 ? (int)g_dw_tile : dw_tile_pick(da, (int)kSize);
  }
  // dW as residue chains in sequence over residue-major copies of delta and
  // the im2col matrix (dw_res.hip): the 3x3 layers with large outputs
  int dwr = -1;
  if (g_nt_sdot && g_dw_res != -2 && g_dw_tile < 0 && batch <= 65535 && i_k >= 64) {
    if (g_dw_res >= 0)
      dwr = (int)g_dw_res;
    else if (kSize == 3)  // (1x1 layers: behind the sdot kernels, 0.048 -> 0.058 ms at 52^2)
      dwr = dw_res_pick(i_m, i_n, i_k, batch);
  }
  // its scratch (residue-major copies, group planes: in addition to the
  // caller's workspace), sized before any fork; when the form was picked by
  // shape and that memory cannot be had, the dW falls back to the paths
  // that need only the workspace (dw_tile, or im2col + the sdot kernels)
  DwResArgs dres{};
  if (dwr >= 0) {
    const int64_t rowlen = 8 * dw_res_k4(i_k);
    int r = ensure_scratch(c, SLOT_RES_A, batch * i_m * rowlen + 32, &dres.dA, pipe);
    if (!r)
      r = ensure_scratch(c, SLOT_RES_B, batch * dw_res_b_rows(dwr, i_n) * rowlen + 32, &dres.dB,
                         pipe);
    if (!r) r = ensure_scratch(c, SLOT_DW, batch * dw_res_groups(dwr) * i_m * i_n, &dres.part, pipe);
    if (r) {
      if (g_dw_res >= 0) return r;  // (forced: the error stands)
      tns_clear_error();
      release_scratch(c, SLOT_RES_A);
      release_scratch(c, SLOT_RES_B);
      dwr = -1;
    }
  }
  if (dwr >= 0) dwv = -1;
  // a 1x1/s1/p0 layer's col2im adds each col element to its own pixel once:
  // the dX product adds into state.delta in its epilogue instead (EPI_ADD,
  // the same add), no col matrix
  const bool dx_direct = state_delta && !needs_col && !fused_dx;
  // state.delta of a stride-1 3x3 layer as one implicit transposed
  // convolution (conv_tile4 DX forms: each tap's filter chain added to the
  // pixel in scol2im's order), no col matrix
  // (stride 2: four such convolutions, one per output pixel parity class,
  // each over the taps col2im adds to that class)
  int dxc = -1;
  const bool dxc_s2 = stride == 2;
  if (state_delta && !fused_dx && kSize == 3 && (stride == 1 || stride == 2) && dilation == 1 &&
      g_dx_conv != -2)
    dxc = g_dx_conv >= 0 ? (int)g_dx_conv
          : dxc_s2   ? conv_tile4_dx3s2_pick(batch, C, H, W, filters, kSize, padding)
                     : conv_tile4_dx3_pick(batch, C, H, W, filters, kSize, padding);
  // dW (im2col + sdot or dw_tile, accumulate) and state.delta (TN + col2im
  // or the fused kernel) read delta and write disjoint outputs: with a
  // state.delta they run concurrently, state.delta's chain on the context's
  // side stream (fork / join events), each with its own col buffer —
  // nothing changes in either result.  Telemetry times ops one by one, so it
  // keeps them in sequence.
  bool overlap = !pipe && state_delta && g_bwd_overlap && !c->telemetry && ensure_side_stream(c);
  const bool dw_col = needs_col && dwv < 0 && dwr < 0;  // dW reads an im2col matrix
  // state.delta's own col buffer when both chains need one at once (the
  // overlap's extra memory, tns.h); if it cannot be had, the sequential
  // schedule shares the one col buffer instead
  float* dx_ws = nullptr;
  const bool dx_col = state_delta && !fused_dx && !dx_direct && dxc < 0;  // dX writes a col matrix
  if (overlap && dw_col && dx_col && ensure_scratch(c, SLOT_COL_DX, batch * colSize, &dx_ws)) {
    tns_clear_error();
    overlap = false;
  }
  // (pipelined: state.delta's chain always has its own col buffer — the
  // pending dW products may still read the shared one)
  // (if that buffer cannot be had: the pending dW joined, this call in
  // sequence within the caller's workspace)
  if (pipe && dx_col && ensure_scratch(c, SLOT_COL_DX, batch * colSize, &dx_ws)) {
    tns_clear_error();
    dx_ws = nullptr;
    pipe = false;
    if (int r = join_side(c)) return r;
  }
  float* ws = workspace;
  if (!ws && (dw_col || (dx_col && !dx_ws && !(overlap && dw_col))))
    if (int r = ensure_scratch(c, SLOT_COL, batch * colSize, &ws, pipe)) return r;
  if (!dx_ws) dx_ws = ws;  // col buffer of state.delta's chain
  // scratch of the fused state.delta kernel, sized before any fork (a growth
  // inside the side-stream chain would free a buffer the main stream may use)
  float* wt = nullptr;
  if (fused_dx || dxc >= 0 || dx1 >= 0)
    if (int r = ensure_scratch(c, SLOT_WT, filters * C * kSize * kSize, &wt)) return r;

  auto run_dw = [&]() -> int {
    const float* col = input;
    if (dwr >= 0) {
      DwResArgs d = dres;  // (scratch sized above)
      d.g = g;
      d.x = input; d.xStride = C * H * W;
      d.delta = delta; d.weight_updates = weight_updates;
      d.M = i_m; d.N = i_n; d.K = i_k; d.batch = batch;
      d.direct = !needs_col; d.alpha = 1.0f;
      OpTimer t(c, TNS_OP_GEMM);
      const hipError_t e = launch_dw_res(dwr, d, c->stream);
      if (e == hipErrorInvalidValue)
        return set_error(TNS_ERR_UNSUPPORTED, "dW res form %d does not fit this layer", dwr);
      return hip_status(e, "dW res launch");
    }
    if (dwv >= 0) {
      float* part = nullptr;
      if (int r = ensure_scratch(c, SLOT_DW, batch * i_m * i_n, &part, pipe)) return r;
      da.part = part;
      {
        OpTimer t(c, TNS_OP_GEMM);
        const hipError_t e = launch_dw_tile(dwv, da, (int)kSize, c->stream);
        if (e == hipErrorInvalidValue)
          return set_error(TNS_ERR_UNSUPPORTED, "dW tile %d does not fit this layer", dwv);
        if (int r = hip_status(e, "dW tile launch")) return r;
      }
      return hip_status(launch_add_in_order(weight_updates, part, i_m * i_n, batch, c->stream),
                        "dW accumulate launch");
    }
    if (needs_col) {
      OpTimer t(c, TNS_OP_IM2COL);
      if (int r = hip_status(launch_im2col(g, input, C * H * W, ws, colSize, batch, c->stream),
                             "im2col launch"))
        return r;
      col = ws;
    }
    // weight_updates += delta_b . col_b^T, one NT GEMM per image (beta = 1),
    // in image order as the reference loop (nConvolutionLayer.pas:636-640):
    // each image adds sum_b = 1*sdot(...) to C.  The sums of different images
    // are independent, so they are computed by ONE strided-batched sdot launch
    // (each stored as is, BETA_STORE), then added to C image by image in the
    // reference's order — the same roundings, batch-fold more parallelism for
    // the few-tile, long-k dW shapes.
    if (g_nt_sdot && batch > 1) {
      float* part = nullptr;
      if (int r = ensure_scratch(c, SLOT_DW, batch * i_m * i_n, &part, pipe)) return r;
      GemmArgs a{};
      a.M = i_m; a.N = i_n; a.K = i_k;
      a.alpha = 1.0f; a.beta = 0.0f; a.beta_mode = BETA_STORE;
      a.A = delta; a.lda = i_k; a.strideA = i_m * i_k;
      a.B = col; a.ldb = i_k; a.strideB = colSize;
      a.C = part; a.ldc = i_n; a.strideC = i_m * i_n;
      a.batch = batch; a.epi = EPI_NONE;
      {
        OpTimer t(c, TNS_OP_GEMM);
        if (int r = hip_status(launch_sgemm_nt_sdot(a, c->stream), "sgemm_nt launch")) return r;
      }
      return hip_status(launch_add_in_order(weight_updates, part, i_m * i_n, batch, c->stream),
                        "dW accumulate launch");
    }
    for (int64_t b = 0; b < batch; ++b)
      if (int r = do_gemm(c, false, true, i_m, i_n, i_k, 1.0f, delta + b * i_m * i_k, i_k, 0,
                          col + b * colSize, i_k, 0, 1.0f, weight_updates, i_n, 0, 1, EPI_NONE,
                          nullptr, 0))
        return r;
    return TNS_OK;
  };

  auto run_dx = [&]() -> int {
    if (fused_dx) {
      // per image pixel: each window tap's ascending-f chain, added to the
      // pixel in (kr, kc) order for the taps scol2im does not skip — the same
      // roundings as the two stages below (646-660)
      OpTimer t(c, TNS_OP_GEMM);
      return hip_status(launch_conv_dx_col2im(weights, wt, delta, state_delta, batch, C, H, W,
                                              filters, kSize, padding, dilation, g.oh, g.ow,
                                              c->stream),
                        "fused dX + col2im launch");
    }
    // col_b = W^T . delta_b (TN strided batched, weights shared, beta = 0 into
    // the workspace), then col2im accumulates into state.delta (646-660).  All
    // images in one launch on conv_tile4's k-major-A forms where they apply (a
    // 1x1 "convolution" over the delta planes, the same chains), else the TN
    // GEMM
    if (dxc >= 0) {
      OpTimer t(c, TNS_OP_GEMM);
      if (int r = hip_status(
              dxc_s2 ? launch_transpose_taps(weights, wt, filters, C, kSize * kSize, c->stream,
                                             conv_tile4_dx3s2_order(padding))
                     : launch_transpose_taps(weights, wt, filters, C, kSize * kSize, c->stream),
              "weights transpose launch"))
        return r;
      const hipError_t e =
          dxc_s2 ? launch_conv_tile4_dx3s2(dxc, wt, delta, state_delta, batch, C, H, W, filters,
                                           padding, g.oh, g.ow, c->stream)
                 : launch_conv_tile4_dx3(dxc, wt, delta, state_delta, batch, C, H, W, filters,
                                         kSize, padding, g.oh, g.ow, c->stream);
      if (e != hipErrorInvalidValue) return hip_status(e, "dX conv launch");
      return set_error(TNS_ERR_UNSUPPORTED, "dX conv form %d does not fit this layer", dxc);
    }
    bool done = false;
    float* col = dx_direct ? state_delta : dx_ws;
    if (dx1 >= 0) {  // (1x1 / stride 1: dx_direct)
      OpTimer t(c, TNS_OP_GEMM);
      if (int r = hip_status(launch_transpose(weights, wt, filters, C, c->stream),
                             "weights transpose launch"))
        return r;
      const hipError_t e = launch_conv1x1(dx1, wt, delta, nullptr, state_delta, batch, C, filters,
                                          i_k, 0, c->stream, true);
      if (e == hipSuccess) return TNS_OK;
      if (e != hipErrorInvalidValue) return hip_status(e, "dX 1x1 launch");
      // (operands off the 16-byte alignment the DMA needs: the TN product)
    }
    if (g_dx_tile != -2) {
      const int dv = g_dx_tile >= 0 ? (int)g_dx_tile : conv_tile4_dx_pick(i_n, batch * i_k, i_m, kSize);
      if (dv >= 0) {
        OpTimer t(c, TNS_OP_GEMM);
        const hipError_t e = launch_conv_tile4_dx(dv, weights, delta, col, batch, C, kSize,
                                                  filters, g.oh, g.ow, c->stream, dx_direct);
        if (e == hipSuccess)
          done = true;
        else if (e != hipErrorInvalidValue || g_dx_tile >= 0)
          return e == hipErrorInvalidValue
                     ? set_error(TNS_ERR_UNSUPPORTED, "dX tile %d does not fit this layer", dv)
                     : hip_status(e, "dX tile launch");
      }
    }
    if (!done)
      if (int r = do_gemm(c, true, false, i_n, i_k, i_m, 1.0f, weights, i_n, 0, delta, i_k,
                          i_m * i_k, 0.0f, col, i_k, colSize, batch,
                          dx_direct ? EPI_ADD : EPI_NONE, nullptr, 0, true))
        return r;
    if (dx_direct) return TNS_OK;
    OpTimer t(c, TNS_OP_COL2IM);
    return hip_status(launch_col2im(g, dx_ws, colSize, state_delta, C * H * W, batch, c->stream),
                      "col2im launch");
  };

  if (pipe) {
    // dW enqueued on the side stream behind the earlier calls' (fork: after
    // this call's derive / bias sums), state.delta's chain on the context's
    // stream; no join — the side stream's work is joined by the next call of
    // any other entry point (tns.h TNS_OPT_BWD_OVERLAP)
    TNS_HIP_TRY(hipEventRecord(c->ev_fork, c->stream));
    TNS_HIP_TRY(hipStreamWaitEvent(c->aux_stream, c->ev_fork, 0));
    hipStream_t main = c->stream;
    c->home_stream = main;
    c->stream = c->aux_stream;
    const int rw = run_dw();
    c->stream = main;
    c->home_stream = nullptr;
    c->side_pending = true;
    // the record of this dW's operands and of the scratch slots it uses
    // (kept after a failed launch too: whatever it enqueued stays ordered)
    tns_ctx::PendingDw d;
    const Span rd = span(delta, batch * filters * i_k), ri = span(input, batch * C * H * W);
    const Span wu = span(weight_updates, i_m * i_n);
    const Span wc = dw_col && ws == workspace ? span(ws, batch * colSize) : Span{};
    d.lo[0] = rd.lo; d.hi[0] = rd.hi;
    d.lo[1] = ri.lo; d.hi[1] = ri.hi;
    d.wlo[0] = wu.lo; d.whi[0] = wu.hi;
    d.wlo[1] = wc.lo; d.whi[1] = wc.hi;
    c->pending.push_back(d);
    c->side_slots |= 1u << SLOT_RES_A | 1u << SLOT_RES_B | 1u << SLOT_DW |
                     (dw_col && ws != workspace ? 1u << SLOT_COL : 0u);
    if (rw) return rw;
    return state_delta ? run_dx() : TNS_OK;
  }
  if (!overlap) {
    if (int r = run_dw()) return r;
    return state_delta ? run_dx() : TNS_OK;
  }
  TNS_HIP_TRY(hipEventRecord(c->ev_fork, c->stream));
  TNS_HIP_TRY(hipStreamWaitEvent(c->ovl_stream, c->ev_fork, 0));
  int rx;
  {
    // state.delta's chain enqueued on the overlap stream (every launch inside
    // run_dx goes to c->stream), the context's stream restored after
    hipStream_t main = c->stream;
    c->stream = c->ovl_stream;
    rx = run_dx();
    c->stream = main;
  }
  // joined even after an error, so later work on the stream stays ordered
  const hipError_t ej = hipEventRecord(c->ev_join, c->ovl_stream);
  const int rw = run_dw();
  const hipError_t ew = ej == hipSuccess ? hipStreamWaitEvent(c->stream, c->ev_join, 0) : ej;
  if (rx) return rx;
  if (rw) return rw;
  return hip_status(ew, "backward join");
}
}  // namespace

int tns_hip_conv_backward(tns_ctx* c, int64_t batch, int64_t C, int64_t H, int64_t W,
                          const float* input, const float* weights, int64_t filters,
                          int64_t kSize, int64_t stride, int64_t padding, int64_t dilation,
                          int32_t activation, const float* output, float* delta,
                          float* bias_updates, float* weight_updates, float* workspace,
                          float* state_delta) {
  return conv_backward_impl(c, batch, C, H, W, input, weights, filters, kSize, stride, padding,
                            dilation, activation, output, delta, bias_updates, weight_updates,
                            workspace, state_delta, ConvBN{});
}

int tns_hip_conv_backward_bn(tns_ctx* c, int64_t batch, int64_t C, int64_t H, int64_t W,
                             const float* input, const float* weights, int64_t filters,
                             int64_t kSize, int64_t stride, int64_t padding, int64_t dilation,
                             int32_t activation, const float* output, float* delta,
                             const float* scales, const float* x, const float* x_norm,
                             const float* mean, const float* variance, float* scale_updates,
                             float* mean_delta, float* variance_delta, float* weight_updates,
                             float* workspace, float* state_delta) {
  if (!scales) return set_error(TNS_ERR_ARG, "conv_backward_bn: null scales");
  ConvBN bn{scales, x, x_norm, mean, variance, scale_updates, mean_delta, variance_delta};
  return conv_backward_impl(c, batch, C, H, W, input, weights, filters, kSize, stride, padding,
                            dilation, activation, output, delta, nullptr, weight_updates,
                            workspace, state_delta, bn);
}

int tns_gemm_variant_count(void) { return sgemm_variant_count(); }
int tns_sdot_chains_variant_count(void) { return sdot_chains_variant_count(); }
int tns_conv_tile_variant_count(void) { return conv_tile_count(); }
int tns_conv_slab_count(void) { return conv_slab_count(); }
int tns_conv1x1_count(void) { return conv1x1_count(); }
const char* tns_conv1x1_name(int32_t v) { return conv1x1_name(v); }
const char* tns_conv_slab_name(int32_t v) { return conv_slab_name(v); }
int tns_conv_dx_tile_count(void) { return conv_tile4_ta_count(); }
int tns_conv_dx_conv_count(void) { return conv_tile4_dx3_count(); }
int tns_conv_dw_res_count(void) { return dw_res_count(); }
int tns_conv_dw_tile_count(void) { return dw_tile_count(); }
int tns_conv_pp_variant_count(void) { return conv_pp_count(); }
const char* tns_conv_pp_variant_name(int32_t v) { return conv_pp_name(v); }
int tns_conv_dma_variant_count(void) { return conv_dma_count(); }
const char* tns_conv_dma_variant_name(int32_t v) { return conv_dma_name(v); }
int tns_conv_patch_variant_count(void) { return conv_patch_count(); }
const char* tns_conv_patch_variant_name(int32_t v) { return conv_patch_name(v); }
const char* tns_conv_tile_variant_name(int32_t v) { return conv_tile_name(v); }
const char* tns_sdot_chains_variant_name(int32_t v) { return sdot_chains_variant_name(v); }
int tns_sdot_rc_variant_count(void) { return sdot_rc_variant_count(); }
const char* tns_sdot_rc_variant_name(int32_t v) { return sdot_rc_variant_name(v); }
const char* tns_gemm_variant_name(int32_t v) { return sgemm_variant_name(v); }

int tns_hip_gemm_variant(tns_ctx* c, int32_t variant, uint8_t transA, uint8_t transB, int64_t M,
                         int64_t N, int64_t K, float ALPHA, const float* A, int64_t aOffset,
                         int64_t lda, int64_t strideA, const float* B, int64_t bOffset,
                         int64_t ldb, int64_t strideB, float BETA, float* C, int64_t cOffset,
                         int64_t ldc, int64_t strideC, int64_t batchCount) {
  if (int r = check_ctx(c)) return r;
  if (variant >= sgemm_variant_count())
    return set_error(TNS_ERR_ARG, "gemm variant %d out of range", variant);
  return do_gemm(c, transA != 0, transB != 0, M, N, K, ALPHA, A ? A + aOffset : nullptr, lda,
                 strideA, B ? B + bOffset : nullptr, ldb, strideB, BETA,
                 C ? C + cOffset : nullptr, ldc, strideC, batchCount, EPI_NONE, nullptr, 0, false,
                 variant);
}

int tns_hip_set_telemetry(tns_ctx* c, int32_t enable) {
  if (int r = check_ctx(c)) return r;
  c->telemetry = enable != 0;
  if (c->telemetry)
    for (double& v : c->op_ms) v = 0.0;
  return TNS_OK;
}

double tns_hip_op_ms(tns_ctx* c, int32_t op) {
  if (!c || op < 0 || op >= TNS_OP_COUNT) return 0.0;
  return c->op_ms[op];
}

// ---- boundary A: host-pointer op-table drop-ins ------------------------------
// Each stages operands through the default context's scratch and returns when
// C (or col/im) holds the result.  No status channel exists in the Pascal
// pointer types, so failures go to tns_last_error() / the error hook.

void tns_cblas_sgemm_batch_strided(int32_t Layout, int32_t TransA, int32_t TransB, int64_t M,
                                   int64_t N, int64_t K, float alpha, const float* A, int64_t lda,
                                   int64_t strideA, const float* B, int64_t ldb, int64_t strideB,
                                   float beta, float* C, int64_t ldc, int64_t strideC,
                                   int64_t batch_size) {
  (void)Layout;  // ignored, as cblas_sgemm ignores Order (ntensors.pas:2231)
  if ((TransA != TNS_CblasNoTrans && TransA != TNS_CblasTrans) ||
      (TransB != TNS_CblasNoTrans && TransB != TNS_CblasTrans)) {
    set_error(TNS_ERR_ARG, "cblas_sgemm: bad transpose enum");
    return;
  }
  if (M <= 0 || N <= 0 || batch_size <= 0) return;
  HostGemm g{TransA == TNS_CblasTrans, TransB == TNS_CblasTrans, M, N, K, alpha, beta,
             A, lda, strideA, B, ldb, strideB, C, ldc, strideC, batch_size};
  {
    std::lock_guard<std::mutex> lk(g_op_devices_mu);
    if (g_op_devices.size() > 1) {  // tns_set_op_devices: spread over several GPUs
      multi_host_gemm(g_op_devices.data(), (int)g_op_devices.size(), g);
      return;
    }
  }
  tns_ctx* c = default_ctx();
  if (!c) return;
  host_gemm(c, g, nullptr, nullptr);
}

void tns_cblas_sgemm(int32_t Order, int32_t TransA, int32_t TransB, int64_t M, int64_t N,
                     int64_t K, float ALPHA, const float* A, int64_t lda, const float* B,
                     int64_t ldb, float BETA, float* C, int64_t ldc) {
  tns_cblas_sgemm_batch_strided(Order, TransA, TransB, M, N, K, ALPHA, A, lda, 0, B, ldb, 0,
                                BETA, C, ldc, 0, 1);
}

void tns_im2col_strided_batched(int64_t aChannels, int64_t aHeight, int64_t aWidth,
                                int64_t kernelHeight, int64_t kernelWidth, int64_t padHeight,
                                int64_t padWidth, int64_t strideY, int64_t strideX,
                                int64_t dilationY, int64_t dilationX, const float* im,
                                int64_t imStride, int64_t imOffset, float* col,
                                int64_t colStride, int64_t colOffset, int64_t batchCount) {
  tns_ctx* c = default_ctx();
  if (!c || batchCount <= 0) return;
  ConvGeom g = geom(aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight, padWidth,
                    strideY, strideX, dilationY, dilationX);
  if (check_geom(g) || g.oh <= 0 || g.ow <= 0) return;
  std::lock_guard<std::mutex> lk(c->mu);
  hipSetDevice(c->device);
  const int64_t imgElems = aChannels * aHeight * aWidth;
  const int64_t colElems = aChannels * kernelHeight * kernelWidth * g.oh * g.ow;
  // pack images/cols densely on the device; strides apply on the host side
  float *dIm = nullptr, *dCol = nullptr;
  if (ensure_scratch(c, 1, imgElems * batchCount, &dIm) ||
      ensure_scratch(c, 2, colElems * batchCount, &dCol))
    return;
  hipStream_t s = c->stream;
  for (int64_t b = 0; b < batchCount; ++b)
    if (hip_status(hipMemcpyAsync(dIm + b * imgElems, im + imOffset + b * imStride,
                                  imgElems * 4, hipMemcpyHostToDevice, s),
                   "H2D im"))
      return;
  {
    OpTimer t(c, TNS_OP_IM2COL);
    if (hip_status(launch_im2col(g, dIm, imgElems, dCol, colElems, batchCount, s), "im2col"))
      return;
  }
  for (int64_t b = 0; b < batchCount; ++b)
    if (hip_status(hipMemcpyAsync(col + colOffset + b * colStride, dCol + b * colElems,
                                  colElems * 4, hipMemcpyDeviceToHost, s),
                   "D2H col"))
      return;
  hip_status(hipStreamSynchronize(s), "sync");
}

void tns_im2col(int64_t aChannels, int64_t aHeight, int64_t aWidth, int64_t kernelHeight,
                int64_t kernelWidth, int64_t padHeight, int64_t padWidth, int64_t strideY,
                int64_t strideX, int64_t dilationY, int64_t dilationX, const float* inData,
                int64_t inOffset, float* outData, int64_t outOffset, uint8_t multiThread) {
  (void)multiThread;  // the device kernel is always parallel and race-free
  tns_im2col_strided_batched(aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight,
                             padWidth, strideY, strideX, dilationY, dilationX, inData, 0,
                             inOffset, outData, 0, outOffset, 1);
}

void tns_col2im_strided_batched(int64_t aChannels, int64_t aHeight, int64_t aWidth,
                                int64_t kernelHeight, int64_t kernelWidth, int64_t padHeight,
                                int64_t padWidth, int64_t strideY, int64_t strideX,
                                int64_t dilationY, int64_t dilationX, const float* inData,
                                int64_t inStride, int64_t inOffset, float* outData,
                                int64_t outStride, int64_t outOffset, int64_t batchCount) {
  tns_ctx* c = default_ctx();
  if (!c || batchCount <= 0) return;
  ConvGeom g = geom(aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight, padWidth,
                    strideY, strideX, dilationY, dilationX);
  if (check_geom(g) || g.oh <= 0 || g.ow <= 0) return;
  std::lock_guard<std::mutex> lk(c->mu);
  hipSetDevice(c->device);
  const int64_t imgElems = aChannels * aHeight * aWidth;
  const int64_t colElems = aChannels * kernelHeight * kernelWidth * g.oh * g.ow;
  float *dIm = nullptr, *dCol = nullptr;
  if (ensure_scratch(c, 1, imgElems * batchCount, &dIm) ||
      ensure_scratch(c, 2, colElems * batchCount, &dCol))
    return;
  hipStream_t s = c->stream;
  for (int64_t b = 0; b < batchCount; ++b) {
    if (hip_status(hipMemcpyAsync(dCol + b * colElems, inData + inOffset + b * inStride,
                                  colElems * 4, hipMemcpyHostToDevice, s),
                   "H2D col"))
      return;
    // col2im accumulates into the existing image (ntensors.pas:11703)
    if (hip_status(hipMemcpyAsync(dIm + b * imgElems, outData + outOffset + b * outStride,
                                  imgElems * 4, hipMemcpyHostToDevice, s),
                   "H2D im"))
      return;
  }
  {
    OpTimer t(c, TNS_OP_COL2IM);
    if (hip_status(launch_col2im(g, dCol, colElems, dIm, imgElems, batchCount, s), "col2im"))
      return;
  }
  for (int64_t b = 0; b < batchCount; ++b)
    if (hip_status(hipMemcpyAsync(outData + outOffset + b * outStride, dIm + b * imgElems,
                                  imgElems * 4, hipMemcpyDeviceToHost, s),
                   "D2H im"))
      return;
  hip_status(hipStreamSynchronize(s), "sync");
}

void tns_col2im(int64_t aChannels, int64_t aHeight, int64_t aWidth, int64_t kernelHeight,
                int64_t kernelWidth, int64_t padHeight, int64_t padWidth, int64_t strideY,
                int64_t strideX, int64_t dilationY, int64_t dilationX, const float* inData,
                int64_t inOffset, float* outData, int64_t outOffset, int64_t batch,
                uint8_t multiThread) {
  (void)batch;        // scol2im's `batch` argument is unused by the reference too
  (void)multiThread;  // race-free gather; matches the single-threaded order
  tns_col2im_strided_batched(aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight,
                             padWidth, strideY, strideX, dilationY, dilationX, inData, 0,
                             inOffset, outData, 0, outOffset, 1);
}

}  // extern "C"
