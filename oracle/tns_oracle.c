/*
 * tns_oracle.c — TEST INFRASTRUCTURE ONLY (see tns_oracle.h header).
 *
 * CPU restatement of the reference's configured CPU path
 * (USE_AVX2 + USE_MULTITHREADING, ntensors.pas / nactivation.pas /
 * nConvolutionLayer.pas).  Written fresh in C; each function cites the
 * Pascal it restates.  PARITY UNPINNED by reference artefacts (no tests,
 * fixtures or compilable sources in the reference) — pinned by hand-derived
 * known-answer vectors in tests/golden/ instead.
 *
 * Build: oracle/Makefile (gcc -O3 -mavx2 -mfma -ffp-contract=off).  Every
 * FMA the reference issues (vfmadd231ps/ss) is an explicit fmaf() here and
 * nothing else is contracted, so results are reproducible bit for bit.
 */
#include "tns_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* ------------------------------------------------------------------------ */
/* steroids TOPool restatement (steroids.pas:281-296, 606-641)               */
/* ------------------------------------------------------------------------ */
static int g_threads = 0;

static int default_threads(void) {
  /* GetSystemThreadCount = max(ProcessorCount, 4).  On a shared GPU box the
   * process's CPU share is given by TNS_ORACLE_THREADS / OMP_NUM_THREADS
   * (nproc there reports the whole machine). */
  const char* env = getenv("TNS_ORACLE_THREADS");
  if (!env || !*env) env = getenv("OMP_NUM_THREADS");
  long n = env && *env ? strtol(env, NULL, 10) : 0;
  if (n <= 0) n = sysconf(_SC_NPROCESSORS_ONLN);
  if (n < 4) n = 4;
  if (n > 256) n = 256;
  return (int)n;
}

void ora_set_threads(int n) { g_threads = n > 0 ? n : 0; }
int ora_get_threads(void) { return g_threads > 0 ? g_threads : default_threads(); }

typedef void (*range_fn)(int64_t from, int64_t to, void* p); /* inclusive */

typedef struct {
  range_fn fn;
  void* p;
  int64_t from, to;
} job_t;

static void* job_main(void* arg) {
  job_t* j = (job_t*)arg;
  j->fn(j->from, j->to, j->p);
  return NULL;
}

/* TOPool.&For(proc, _from, _to): contiguous groups of ceil((N+1)/P) items,
 * the first (N mod P)+1 groups one larger (steroids.pas:606-641).  Result
 * independence from the partition is what the tests rely on; the partition
 * itself only matters for timing. */
static void par_for(range_fn fn, int64_t from, int64_t to, void* p) {
  if (to < from) return;
  int P = ora_get_threads();
  int64_t n = to - from; /* N in the reference (= count-1) */
  if (P <= 1 || n < 1) {
    fn(from, to, p);
    return;
  }
  int64_t group_t = (n + 1 + P - 1) / P;
  int64_t group_m = n % P;
  pthread_t th[256];
  job_t jobs[256];
  if (P > 256) P = 256;
  int used = 0;
  int64_t ii = 0;
  for (int i = 0; i < P; i++) {
    int64_t start = ii;
    ii += group_t - (int64_t)(i > group_m);
    int64_t end = ii - 1;
    if (ii <= start) break;
    if (from + end > to) end = to - from;
    jobs[used].fn = fn;
    jobs[used].p = p;
    jobs[used].from = from + start;
    jobs[used].to = from + end;
    used++;
    if (from + end >= to) break;
  }
  for (int i = 1; i < used; i++) pthread_create(&th[i], NULL, job_main, &jobs[i]);
  job_main(&jobs[0]);
  for (int i = 1; i < used; i++) pthread_join(th[i], NULL);
}

/* ------------------------------------------------------------------------ */
/* BLAS-1                                                                    */
/* ------------------------------------------------------------------------ */
void ora_saxpy(int64_t N, float a, const float* restrict x, float* restrict y) {
  /* every element: vfmadd231ps/ss y <- a*x + y, single rounding */
  for (int64_t i = 0; i < N; i++) y[i] = fmaf(a, x[i], y[i]);
}

float ora_sdot(int64_t N, const float* A, const float* B) {
  /* sdot_avx2 SIMD_REGS=8 branch, ntensors.pas:1268-1303 */
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int64_t blocks = N >> 3;
  const float* a = A;
  const float* b = B;
  for (int64_t t = 0; t < blocks; t++) {
    for (int l = 0; l < 8; l++) acc[l] = fmaf(a[l], b[l], acc[l]);
    a += 8;
    b += 8;
  }
  int64_t rem = N & 7;
  if (rem) {
    /* vmaskmovps loads zeros into the masked lanes; the FMA still runs on
     * all 8 lanes (masked lanes add 0*0). */
    for (int l = 0; l < 8; l++) {
      float xa = l < rem ? a[l] : 0.0f;
      float xb = l < rem ? b[l] : 0.0f;
      acc[l] = fmaf(xa, xb, acc[l]);
    }
  }
  /* vextractf128 + vaddps: s_l = acc_l + acc_{l+4}; vhaddps twice */
  float s0 = acc[0] + acc[4], s1 = acc[1] + acc[5];
  float s2 = acc[2] + acc[6], s3 = acc[3] + acc[7];
  float h0 = s0 + s1, h1 = s2 + s3;
  return h0 + h1;
}

/* ------------------------------------------------------------------------ */
/* SGEMM                                                                     */
/* ------------------------------------------------------------------------ */
typedef struct {
  int64_t M, N, K, lda, ldb, ldc;
  float alpha;
  const float* A;
  const float* B;
  float* C;
} gemm_p;

/* s_nn (ntensors.pas:2061-2133): for each row, kk ascending,
 * saxpy(N, ALPHA*A[kk], B + kk*ldb, C). */
static void s_nn(int64_t f, int64_t t, void* vp) {
  gemm_p* p = (gemm_p*)vp;
  for (int64_t i = f; i <= t; i++) {
    const float* a = p->A + i * p->lda;
    float* c = p->C + i * p->ldc;
    for (int64_t kk = 0; kk < p->K; kk++) {
      float a_part = p->alpha * a[kk];
      ora_saxpy(p->N, a_part, p->B + kk * p->ldb, c);
    }
  }
}

/* s_nt (1957-1985): C[i,j] += ALPHA * sdot(K, A_i, B_j). */
static void s_nt(int64_t f, int64_t t, void* vp) {
  gemm_p* p = (gemm_p*)vp;
  for (int64_t i = f; i <= t; i++)
    for (int64_t j = 0; j < p->N; j++) {
      float sum = p->alpha * ora_sdot(p->K, p->A + i * p->lda, p->B + j * p->ldb);
      p->C[i * p->ldc + j] = p->C[i * p->ldc + j] + sum;
    }
}

/* s_tn (2007-2033): A_PART = ALPHA*A[kk*lda+i]; saxpy(N, A_PART, B_kk, C_i). */
static void s_tn(int64_t f, int64_t t, void* vp) {
  gemm_p* p = (gemm_p*)vp;
  for (int64_t i = f; i <= t; i++)
    for (int64_t kk = 0; kk < p->K; kk++) {
      float a_part = p->alpha * p->A[kk * p->lda + i];
      ora_saxpy(p->N, a_part, p->B + kk * p->ldb, p->C + i * p->ldc);
    }
}

/* s_tt (2159-2182): sum := sum + ALPHA*A[i+kk*lda]*B[kk+j*ldb] (no FMA
 * contraction in FPC: (ALPHA*A)*B rounded, then added); C += sum.  The
 * configured (USE_MULTITHREADING) sgemm_tt covers all M rows; the single-
 * threaded branch's M-2 bound (2204) is a reference bug not restated. */
static void s_tt(int64_t f, int64_t t, void* vp) {
  gemm_p* p = (gemm_p*)vp;
  for (int64_t i = f; i <= t; i++)
    for (int64_t j = 0; j < p->N; j++) {
      float sum = 0.0f;
      for (int64_t kk = 0; kk < p->K; kk++) {
        float t1 = p->alpha * p->A[i + kk * p->lda];
        float t2 = t1 * p->B[kk + j * p->ldb];
        sum = sum + t2;
      }
      p->C[i * p->ldc + j] = p->C[i * p->ldc + j] + sum;
    }
}

/* mulvs = cblas_sscal -> sscal AVX (ntensors.pas:1439-1464, 1566-1578):
 * vmulps, single rounding; beta = 0 gives 0*C (NaN/Inf propagate). */
static void beta_scale(int64_t r0, int64_t r1, int64_t N, float beta, float* C, int64_t ldc) {
  if (beta == 1.0f) return;
  for (int64_t i = r0; i < r1; i++) {
    float* c = C + i * ldc;
    for (int64_t j = 0; j < N; j++) c[j] = beta * c[j];
  }
}

static range_fn pick(int32_t ta, int32_t tb) {
  int a = ta == 112, b = tb == 112;
  if (!a && !b) return s_nn;
  if (!a && b) return s_nt;
  if (a && !b) return s_tn;
  return s_tt;
}

void ora_sgemm(int32_t order, int32_t transA, int32_t transB, int64_t M, int64_t N,
               int64_t K, float alpha, const float* A, int64_t lda, const float* B,
               int64_t ldb, float beta, float* C, int64_t ldc) {
  (void)order; /* Order is ignored by the reference (always row-major) */
  beta_scale(0, M, N, beta, C, ldc);
  gemm_p p = {M, N, K, lda, ldb, ldc, alpha, A, B, C};
  par_for(pick(transA, transB), 0, M - 1, &p);
}

void ora_sgemm_rows(int32_t transA, int32_t transB, int64_t row0, int64_t row1, int64_t M,
                    int64_t N, int64_t K, float alpha, const float* A, int64_t lda,
                    const float* B, int64_t ldb, float beta, float* C, int64_t ldc) {
  if (row1 > M) row1 = M;
  if (row0 >= row1) return;
  beta_scale(row0, row1, N, beta, C, ldc);
  gemm_p p = {M, N, K, lda, ldb, ldc, alpha, A, B, C};
  par_for(pick(transA, transB), row0, row1 - 1, &p);
}

void ora_sgemm_batch_strided(int32_t order, int32_t transA, int32_t transB, int64_t M,
                             int64_t N, int64_t K, float alpha, const float* A, int64_t lda,
                             int64_t strideA, const float* B, int64_t ldb, int64_t strideB,
                             float beta, float* C, int64_t ldc, int64_t strideC,
                             int64_t batch) {
  for (int64_t i = 0; i < batch; i++)
    ora_sgemm(order, transA, transB, M, N, K, alpha, A + i * strideA, lda, B + i * strideB,
              ldb, beta, C + i * strideC, ldc);
}

/* ------------------------------------------------------------------------ */
/* im2col / col2im                                                           */
/* ------------------------------------------------------------------------ */
static int64_t out_dim(int64_t in, int64_t pad, int64_t k, int64_t dil, int64_t stride) {
  /* Pascal `div` truncates toward zero, like C '/' */
  return (in + 2 * pad - (dil * (k - 1) + 1)) / stride + 1;
}

/* i2c_ext for one channel (ntensors.pas:11430-11466) */
static void i2c_channel(int64_t ch, int64_t H, int64_t W, int64_t kH, int64_t kW,
                        int64_t padH, int64_t padW, int64_t sY, int64_t sX, int64_t dY,
                        int64_t dX, int64_t oh, int64_t ow, const float* im, float* col) {
  const float* d_im = im + H * W * ch;
  float* d_col = col + kH * kW * oh * ow * ch;
  for (int64_t kr = 0; kr < kH; kr++)
    for (int64_t kc = 0; kc < kW; kc++) {
      int64_t input_row = -padH + kr * dY;
      for (int64_t orow = 0; orow < oh; orow++) {
        if ((uint64_t)input_row < (uint64_t)H) {
          int64_t input_col = -padW + kc * dX;
          for (int64_t ocol = 0; ocol < ow; ocol++) {
            d_col[ocol] = ((uint64_t)input_col < (uint64_t)W) ? d_im[input_row * W + input_col]
                                                               : 0.0f;
            input_col += sX;
          }
        } else {
          for (int64_t ocol = 0; ocol < ow; ocol++) d_col[ocol] = 0.0f;
        }
        d_col += ow;
        input_row += sY;
      }
    }
}

void ora_im2col(int64_t C, int64_t H, int64_t W, int64_t kH, int64_t kW, int64_t padH,
                int64_t padW, int64_t strideY, int64_t strideX, int64_t dilY, int64_t dilX,
                const float* im, int64_t imOffset, float* col, int64_t colOffset) {
  int64_t ow = out_dim(W, padW, kW, dilX, strideX);
  int64_t oh = out_dim(H, padH, kH, dilY, strideY);
  if (oh <= 0 || ow <= 0) return;
  for (int64_t ch = 0; ch < C; ch++)
    i2c_channel(ch, H, W, kH, kW, padH, padW, strideY, strideX, dilY, dilX, oh, ow,
                im + imOffset, col + colOffset);
}

typedef struct {
  int64_t C, H, W, kH, kW, padH, padW, sY, sX, dY, dX;
  const float* im;
  int64_t imStride, imOffset;
  float* col;
  int64_t colStride, colOffset;
} i2c_batch_p;

static void i2c_images(int64_t f, int64_t t, void* vp) {
  i2c_batch_p* p = (i2c_batch_p*)vp;
  for (int64_t b = f; b <= t; b++)
    ora_im2col(p->C, p->H, p->W, p->kH, p->kW, p->padH, p->padW, p->sY, p->sX, p->dY, p->dX,
               p->im + b * p->imStride, p->imOffset, p->col + b * p->colStride, p->colOffset);
}

void ora_im2col_strided_batched(int64_t C, int64_t H, int64_t W, int64_t kH, int64_t kW,
                                int64_t padH, int64_t padW, int64_t strideY, int64_t strideX,
                                int64_t dilY, int64_t dilX, const float* im, int64_t imStride,
                                int64_t imOffset, float* col, int64_t colStride,
                                int64_t colOffset, int64_t batch) {
  /* threads go over images (mp.&For, ntensors.pas:11520-11523); pure copies,
   * so the order cannot change a value */
  i2c_batch_p p = {C,    H,        W,        kH,  kW,        padH,     padW, strideY, strideX,
                   dilY, dilX,     im,       imStride, imOffset, col, colStride, colOffset};
  par_for(i2c_images, 0, batch - 1, &p);
}

/* c2i (ntensors.pas:11650-11715) for one (channel, kernel offset) index i. */
static void c2i_one(int64_t i, int64_t H, int64_t W, int64_t kH, int64_t kW, int64_t padH,
                    int64_t padW, int64_t sY, int64_t sX, int64_t dY, int64_t dX, int64_t oh,
                    int64_t ow, const float* col, float* im) {
  int64_t ksize = kH * kW;
  int64_t chan = i / ksize;
  const float* data_col = col + i * oh * ow;
  float* data_im = im + H * W * chan;
  int64_t index = i % ksize;
  int64_t kr = index / kW, kc = index % kW;
  /* NOTE the reference's col2im dilation formula: (k - pad) * dil
   * (11693, 11700), not im2col's -pad + k*dil.  Restated as is. */
  int64_t input_row = (kr - padH) * dY;
  for (int64_t orow = 0; orow < oh; orow++) {
    if ((uint64_t)input_row >= (uint64_t)H) {
      data_col += ow;
    } else {
      int64_t input_col = (kc - padW) * dX;
      for (int64_t ocol = 0; ocol < ow; ocol++) {
        if ((uint64_t)input_col < (uint64_t)W) {
          int64_t idx = input_row * W + input_col;
          data_im[idx] = data_im[idx] + data_col[0];
        }
        data_col++;
        input_col += sX;
      }
    }
    input_row += sY;
  }
}

void ora_col2im(int64_t C, int64_t H, int64_t W, int64_t kH, int64_t kW, int64_t padH,
                int64_t padW, int64_t strideY, int64_t strideX, int64_t dilY, int64_t dilX,
                const float* col, int64_t colOffset, float* im, int64_t imOffset) {
  /* scol2im (11717-11763): single-threaded order i = 0 .. C*k^2-1.  The
   * multithreaded batch=1 variant races (mp2.&for over i, 11752); parity is
   * defined against this deterministic order. */
  int64_t oh = out_dim(H, padH, kH, dilY, strideY);
  int64_t ow = out_dim(W, padW, kW, dilX, strideX);
  if (oh <= 0 || ow <= 0) return;
  for (int64_t i = 0; i < C * kH * kW; i++)
    c2i_one(i, H, W, kH, kW, padH, padW, strideY, strideX, dilY, dilX, oh, ow,
            col + colOffset, im + imOffset);
}

typedef struct {
  int64_t C, H, W, kH, kW, padH, padW, sY, sX, dY, dX;
  const float* col;
  int64_t colStride, colOffset;
  float* im;
  int64_t imStride, imOffset;
} c2i_batch_p;

static void c2i_images(int64_t f, int64_t t, void* vp) {
  c2i_batch_p* p = (c2i_batch_p*)vp;
  for (int64_t b = f; b <= t; b++)
    ora_col2im(p->C, p->H, p->W, p->kH, p->kW, p->padH, p->padW, p->sY, p->sX, p->dY, p->dX,
               p->col + b * p->colStride, p->colOffset, p->im + b * p->imStride, p->imOffset);
}

void ora_col2im_strided_batched(int64_t C, int64_t H, int64_t W, int64_t kH, int64_t kW,
                                int64_t padH, int64_t padW, int64_t strideY, int64_t strideX,
                                int64_t dilY, int64_t dilX, const float* col, int64_t colStride,
                                int64_t colOffset, float* im, int64_t imStride,
                                int64_t imOffset, int64_t batch) {
  c2i_batch_p p = {C,    H,    W,   kH,        kW,        padH, padW,     strideY, strideX,
                   dilY, dilX, col, colStride, colOffset, im,   imStride, imOffset};
  par_for(c2i_images, 0, batch - 1, &p);
}

/* ------------------------------------------------------------------------ */
/* bias / activation                                                         */
/* ------------------------------------------------------------------------ */
void ora_add_bias(int64_t N, float* a, int64_t blockSize, const float* b, int64_t incb,
                  int64_t batch) {
  /* vsAddB -> vssAddI_avx: c[j] := c[j] + bb, single rounding */
  for (int64_t k = 0; k < batch; k++)
    for (int64_t i = 0; i < N; i++) {
      float* c = a + (k * N + i) * blockSize;
      float bb = b[i * incb];
      for (int64_t j = 0; j < blockSize; j++) c[j] = c[j] + bb;
    }
}

void ora_backward_bias(int64_t nDst, float* dst, int64_t groups, int64_t blockSize,
                       const float* src) {
  /* addSums (7729-7781), generic (non-blockSize=1) branch order:
   * _sum := _sum + sumv(blockSize, block_j, 1) for j ascending; sumv =
   * vsSumI (3624-3635), which with stride 1 on an AVX2 x86-64 host is
   * vssum_avx2 (3592-3620): 8 lanes, fold, sequential tail. */
  for (int64_t i = 0; i < nDst; i++) {
    float sum = 0.0f;
    for (int64_t j = 0; j < groups; j++)
      sum = sum + ora_vssum(blockSize, src + (j * nDst + i) * blockSize);
    dst[i] = dst[i] + sum;
  }
}

static float logistic_f(float x) { return (float)(1.0 / (1.0 + exp(-(double)x))); }

int ora_activate(float* x, int64_t N, int32_t act) {
  switch (act) {
    case 0: /* acLOGISTIC: scalar logistic_activate (293-297); the AVX2
               logistic_array approximation is not a valid oracle */
      for (int64_t i = 0; i < N; i++) x[i] = logistic_f(x[i]);
      return 0;
    case 1: /* acRELU: x*(x>0) (305-310) */
      for (int64_t i = 0; i < N; i++) x[i] = x[i] * (float)(x[i] > 0.0f);
      return 0;
    case 4: /* acLINEAR: no-op */
      return 0;
    case 6: /* acTANH */
      /* tanh_activate (351-357): px := exp(x); nx := exp(-x) as singles,
       * then (px - nx)/(px + nx) in single (NaN once exp overflows) */
      for (int64_t i = 0; i < N; i++) {
        const float px = (float)exp((double)x[i]), nx = (float)exp(-(double)x[i]);
        x[i] = (px - nx) / (px + nx);
      }
      return 0;
    case 8:
    case 9: /* acREVLEAKY, acLEAKY: leaky_array (234-267): if 0 > x then x*0.1f */
      for (int64_t i = 0; i < N; i++)
        if (0.0f > x[i]) x[i] = 0.1f * x[i];
      return 0;
    case 13: /* acHARDTAN */
      for (int64_t i = 0; i < N; i++) x[i] = x[i] < -1.0f ? -1.0f : (x[i] > 1.0f ? 1.0f : x[i]);
      return 0;
    default:
      return -1;
  }
}

int ora_gradient(const float* x, int64_t N, int32_t act, float* delta) {
  switch (act) {
    case 0: /* logistic_gradient (423-426): (1-x)*x */
      for (int64_t i = 0; i < N; i++) delta[i] = delta[i] * ((1.0f - x[i]) * x[i]);
      return 0;
    case 1: /* ord(x>0) */
      for (int64_t i = 0; i < N; i++) delta[i] = delta[i] * (float)(x[i] > 0.0f);
      return 0;
    case 4:
      return 0;
    case 6: /* tanh_gradient: 1 - x*x */
      for (int64_t i = 0; i < N; i++) delta[i] = delta[i] * (1.0f - x[i] * x[i]);
      return 0;
    case 8:
    case 9: /* leaky_gradient (472-476): x>0 ? 1 : 0.1 */
      for (int64_t i = 0; i < N; i++) delta[i] = delta[i] * (x[i] > 0.0f ? 1.0f : 0.1f);
      return 0;
    case 13: /* hardtan_gradient: (x>-1 and x<1) */
      for (int64_t i = 0; i < N; i++)
        delta[i] = delta[i] * ((x[i] > -1.0f && x[i] < 1.0f) ? 1.0f : 0.0f);
      return 0;
    default:
      return -1;
  }
}

/* ------------------------------------------------------------------------ */
/* Conv2D / conv layer                                                       */
/* ------------------------------------------------------------------------ */
void ora_conv2d(int64_t batch, int64_t C, int64_t H, int64_t W, const float* input,
                const float* weights, int64_t filters, int64_t kH, int64_t kW, int64_t wPadding,
                int64_t hPadding, int64_t xStride, int64_t yStride, int64_t xDilation,
                int64_t yDilation, float* workspace, float* out) {
  /* output size as nConvolutionLayer.outWidth/outHeight (92-100) */
  int64_t oh = out_dim(H, hPadding, kH, yDilation, yStride);
  int64_t ow = out_dim(W, wPadding, kW, xDilation, xStride);
  int64_t kSize = kH * kW, outImg = oh * ow, k = C * kSize;
  int64_t strideB;
  const float* Bp;
  if (kSize != 1 || xDilation * yDilation != 1 || xStride * yStride != 1) {
    strideB = C * kSize * outImg;
    /* reference passes (xDilation, yDilation) into the (dilationY,
     * dilationX) slots (ntensors.pas:8303) */
    ora_im2col_strided_batched(C, H, W, kH, kW, hPadding, wPadding, yStride, xStride, xDilation,
                               yDilation, input, C * H * W, 0, workspace, strideB, 0, batch);
    Bp = workspace;
  } else {
    strideB = C * H * W;
    Bp = input;
  }
  for (int64_t b = 0; b < batch; b++)
    ora_sgemm(101, 111, 111, filters, outImg, k, 1.0f, weights, k, Bp + b * strideB, outImg,
              0.0f, out + b * outImg * filters, outImg);
}

void ora_conv_forward(int64_t batch, int64_t C, int64_t H, int64_t W, const float* input,
                      const float* weights, const float* biases, int64_t filters, int64_t kSize,
                      int64_t stride, int64_t padding, int64_t dilation, int32_t act,
                      float* workspace, float* out) {
  ora_conv2d(batch, C, H, W, input, weights, filters, kSize, kSize, padding, padding, stride,
             stride, dilation, dilation, workspace, out);
  int64_t oh = out_dim(H, padding, kSize, dilation, stride);
  int64_t ow = out_dim(W, padding, kSize, dilation, stride);
  ora_add_bias(filters, out, oh * ow, biases, 1, batch);
  ora_activate(out, batch * filters * oh * ow, act);
}

/* The backward's geometry (nConvolutionLayer.pas:571-671): delta and output
 * are [batch][filters][outH*outW] with the layer's outH = (h + 2p - k) div s
 * + 1 (92-100, no dilation), while the backward im2col / col2im pad with
 * padding*dilation (640, 665).  Their column count equals outH*outW for the
 * "same" paddings p = (k-1)/2 at any dilation; other combinations make the
 * reference read past its workspace and are refused (returns 0). */
int64_t ora_conv_backward_oh(int64_t H, int64_t kSize, int64_t stride, int64_t padding,
                             int64_t dilation) {
  int64_t layer = (H + 2 * padding - kSize) / stride + 1;
  int64_t col = out_dim(H, padding * dilation, kSize, dilation, stride);
  return layer == col ? layer : 0;
}

/* everything after the bias / batch-norm gradient: im2col, dW, dX + col2im */
int ora_conv_backward_core(int64_t batch, int64_t C, int64_t H, int64_t W, const float* input,
                           const float* weights, int64_t filters, int64_t kSize, int64_t stride,
                           int64_t padding, int64_t dilation, const float* delta,
                           float* weight_updates, float* workspace, float* state_delta) {
  int64_t oh = ora_conv_backward_oh(H, kSize, stride, padding, dilation);
  int64_t ow = ora_conv_backward_oh(W, kSize, stride, padding, dilation);
  if (!oh || !ow) return -1;
  int64_t i_m = filters, i_n = kSize * kSize * C, i_k = oh * ow, colSize = i_n * i_k;
  /* state.input.im2Col(k, k, p*d, p*d, stride_y, stride_x, d, d, workspace) */
  ora_im2col_strided_batched(C, H, W, kSize, kSize, padding * dilation, padding * dilation,
                             stride, stride, dilation, dilation, input, C * H * W, 0, workspace,
                             colSize, 0, batch);
  /* weight_updates += delta_b . col_b^T, one NT gemm per image, beta = 1 */
  for (int64_t b = 0; b < batch; b++)
    ora_sgemm(101, 111, 112, i_m, i_n, i_k, 1.0f, delta + b * i_m * i_k, i_k,
              workspace + b * colSize, i_k, 1.0f, weight_updates, i_n);
  if (state_delta) {
    /* col_b = W^T . delta_b (TN, strideA 0, beta 0), then col2im accumulate */
    ora_sgemm_batch_strided(101, 112, 111, i_n, i_k, i_m, 1.0f, weights, i_n, 0, delta, i_k,
                            i_m * i_k, 0.0f, workspace, i_k, colSize, batch);
    ora_col2im_strided_batched(C, H, W, kSize, kSize, padding * dilation, padding * dilation,
                               stride, stride, dilation, dilation, workspace, colSize, 0,
                               state_delta, C * H * W, 0, batch);
  }
  return 0;
}

int ora_conv_backward(int64_t batch, int64_t C, int64_t H, int64_t W, const float* input,
                      const float* weights, int64_t filters, int64_t kSize, int64_t stride,
                      int64_t padding, int64_t dilation, int32_t act, const float* output,
                      float* delta, float* bias_updates, float* weight_updates,
                      float* workspace, float* state_delta) {
  /* TConvolutionalLayer.backward, no batch-norm (nConvolutionLayer.pas:571-671) */
  int64_t oh = ora_conv_backward_oh(H, kSize, stride, padding, dilation);
  int64_t ow = ora_conv_backward_oh(W, kSize, stride, padding, dilation);
  if (!oh || !ow) return -1;
  int64_t i_k = oh * ow;
  /* Derivative(): delta *= f'(output) */
  if (ora_gradient(output, batch * filters * i_k, act, delta)) return -2;
  /* bias_updates.addSums(delta) */
  ora_add_sums(bias_updates, delta, batch, filters, i_k);
  return ora_conv_backward_core(batch, C, H, W, input, weights, filters, kSize, stride, padding,
                                dilation, delta, weight_updates, workspace, state_delta);
}

void ora_fuse_batchnorm(int64_t filters, int64_t filterSize, float* weights, float* biases,
                        const float* scales, const float* rollingMean,
                        const float* rollingVariance) {
  /* precomputed := scales/sqrt(max(var, sEPSILON)); b -= mean*precomputed;
   * W *= precomputed  (nConvolutionLayer.pas:102-126) */
  const float eps = 0.000001f;
  for (int64_t f = 0; f < filters; f++) {
    float v = rollingVariance[f] > eps ? rollingVariance[f] : eps;
    float pre = scales[f] / sqrtf(v);
    biases[f] = biases[f] - rollingMean[f] * pre;
    for (int64_t i = 0; i < filterSize; i++) weights[f * filterSize + i] *= pre;
  }
}

/* ------------------------------------------------------------------------ */
/* synthetic data                                                            */
/* ------------------------------------------------------------------------ */
static uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void ora_fill_uniform(float* x, int64_t n, uint64_t seed, uint64_t stream, float lo, float hi) {
  uint64_t key = splitmix64(seed * 0x100000001B3ull ^ (stream + 0x632BE59BD9B4E019ull));
  float range = hi - lo;
  for (int64_t i = 0; i < n; i++) {
    uint64_t r = splitmix64(key + (uint64_t)i);
    float u = (float)(r >> 40) * (1.0f / 16777216.0f); /* 24 bits, exact */
    x[i] = fmaf(range, u, lo);
  }
}

/* ---- non-convolutional YOLOv3 layers (forward) -------------------------- */

/* TAddLayer.forward (naddlayer.pas:667-720), one input of equal size:
 * TSingleTensor.addvv(input, from.output) -> output, then the activation. */
int ora_shortcut(int64_t n, const float* a, const float* b, float* out, int32_t act) {
  for (int64_t i = 0; i < n; i++) out[i] = a[i] + b[i];
  return ora_activate(out, n, act);
}

/* upsample(..., isForward = true, ...) (nupsamplelayer.pas:83-113) */
void ora_upsample(int64_t planes, int64_t h, int64_t w, int64_t stride, float scale,
                  const float* in, float* out) {
  for (int64_t c = 0; c < planes; c++)
    for (int64_t y = 0; y < h * stride; y++)
      for (int64_t x = 0; x < w * stride; x++) {
        const int64_t in_index = (c * h + y / stride) * w + x / stride;
        const int64_t out_index = (c * h * stride + y) * stride * w + x;
        out[out_index] = scale * in[in_index];
      }
}

/* TYoloLayer.forward, inference part (nyololayer.pas:786-825, newCoords
 * false, scaleXY 1): input copied, logistic over entries 0..1 and 4..4+classes
 * of every (image, anchor); data [batch][anchors][classes+5][hw]. */
void ora_yolo_forward(int64_t batch, int64_t anchors, int64_t classes, int64_t hw,
                      const float* in, float* out) {
  const int64_t entries = classes + 5;
  memcpy(out, in, (size_t)(batch * anchors * entries * hw) * sizeof(float));
  for (int64_t b = 0; b < batch; b++)
    for (int64_t a = 0; a < anchors; a++) {
      float* base = out + (b * anchors + a) * entries * hw;
      ora_activate(base, 2 * hw, 0);
      ora_activate(base + 4 * hw, (1 + classes) * hw, 0);
    }
}

