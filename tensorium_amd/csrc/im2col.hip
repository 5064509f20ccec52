// im2col.hip — im2col / col2im for gfx950.
//
// im2col restates sim2Col (ntensors.pas:11415-11491) and its batched form
// (11493-11532): col[((c*kH+kr)*kW+kc)*oh*ow + orow*ow + ocol] =
//   im[c][-padH + kr*dY + orow*sY][-padW + kc*dX + ocol*sX], 0 outside.
// Pure copies => bit-exact.  Main form (im2col_rows_kernel): a block stages
// the input rows of one (image, channel, kernel row, chunk of output rows) in
// LDS and writes the kW col rows of that chunk from there, 16-byte stores
// contiguous across the wave (nontemporal for col matrices far larger than
// the caches).  HBM-write bound.  The output-stationary gather kernel (each
// thread 4 consecutive col elements, scalar gathers through L2) remains for
// rows too wide for LDS.
//
// col2im restates c2i/scol2im (ntensors.pas:11650-11763) as a race-free
// GATHER: one thread per image pixel sums, in ascending kernel index order
// (the single-threaded reference order), every col element that the
// reference would scatter-add into it, starting from the pixel's current
// value (the reference accumulates and never zeroes im).  Same float adds in
// the same order => bit-exact.  The reference's col2im dilation formula,
// input_row := (kernel_row - pad) * dil  (11693, 11700), is kept.
#include <algorithm>

#include "tns_internal.hpp"

namespace tns {

int64_t out_dim(int64_t in, int64_t pad, int64_t k, int64_t dil, int64_t stride) {
  return (in + 2 * pad - (dil * (k - 1) + 1)) / stride + 1;
}

namespace {
// k-table of the implicit-GEMM convolution: the im2col row k = (c, kr, kc)
// reads padded image element [c][orow*sY + kr*dY][ocol*sX + kc*dX] — the same
// element sim2Col copies (ntensors.pas:11460), shifted by the padding.
__global__ void ktab_kernel(int* t, int K, int total, int Hs, int Ws, int kH, int kW, int dY,
                            int dX) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= total) return;
  if (k >= K) {  // sentinel: out of the buffer's range and of any window
    t[k] = (int)0x80000000u;
    t[total + k] = 0x4000 | (0x4000 << 16);
    return;
  }
  const int kc = k % kW, r = k / kW;
  const int kr = r % kH, c = r / kH;
  t[k] = 4 * (c * Hs * Ws + kr * dY * Ws + kc * dX);
  t[total + k] = (kr * dY) | ((kc * dX) << 16);
}

// planes whose padded size fits 32-bit indexing: grid x -> pixels of one
// padded plane, y -> plane (no per-element 64-bit division)
__global__ void pad_plane_kernel(const float* __restrict__ im, float* __restrict__ out, int H,
                                 int W, int pH, int pW) {
  const int Hp = H + 2 * pH, Wp = W + 2 * pW;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Hp * Wp) return;
  const int64_t pl = blockIdx.y;
  const int y = i / Wp, x = i - y * Wp;
  const int iy = y - pH, ix = x - pW;
  out[pl * Hp * Wp + i] = ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
                              ? im[pl * H * W + iy * W + ix]
                              : 0.0f;
}

__global__ void pad_kernel(const float* __restrict__ im, float* __restrict__ out, int64_t planes,
                           int H, int W, int pH, int pW) {
  const int Hp = H + 2 * pH, Wp = W + 2 * pW;
  const int64_t total = planes * Hp * Wp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(i % Wp);
    const int64_t t = i / Wp;
    const int y = (int)(t % Hp);
    const int64_t pl = t / Hp;
    const int iy = y - pH, ix = x - pW;
    out[i] = ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
                 ? im[(pl * H + iy) * W + ix]
                 : 0.0f;
  }
}
}  // namespace

hipError_t launch_build_ktab(int* ktab, int C, int Hp, int Wp, int kH, int kW, int dY, int dX,
                             hipStream_t s) {
  const int K = C * kH * kW;
  if (K < 0) return hipErrorInvalidValue;
  const int total = K + KTAB_PAD;
  hipLaunchKernelGGL(ktab_kernel, dim3((total + 255) / 256), dim3(256), 0, s, ktab, K, total, Hp,
                     Wp, kH, kW, dY, dX);
  return hipGetLastError();
}

hipError_t launch_pad_images(const float* im, int64_t batch, int64_t C, int64_t H, int64_t W,
                             int64_t pH, int64_t pW, float* out, hipStream_t s) {
  const int64_t total = batch * C * (H + 2 * pH) * (W + 2 * pW);
  if (total <= 0) return hipSuccess;
  const int64_t plane = (H + 2 * pH) * (W + 2 * pW);
  if (plane <= 0x7fffff00LL && H * W <= 0x7fffffffLL) {
    for (int64_t p0 = 0; p0 < batch * C; p0 += 65535) {
      const int64_t np = std::min<int64_t>(65535, batch * C - p0);
      hipLaunchKernelGGL(pad_plane_kernel, dim3((unsigned)((plane + 255) / 256), (unsigned)np),
                         dim3(256), 0, s, im + p0 * H * W, out + p0 * plane, (int)H, (int)W,
                         (int)pH, (int)pW);
      if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  int64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(pad_kernel, dim3((unsigned)blocks), dim3(256), 0, s, im, out, batch * C,
                     (int)H, (int)W, (int)pH, (int)pW);
  return hipGetLastError();
}

namespace {

struct I2CArgs {
  int C, H, W, kH, kW, padH, padW, sY, sX, dY, dX, oh, ow;
  const float* im;
  int64_t imStride;
  float* col;
  int64_t colStride;
  int rows;         // C*kH*kW
  int quads;        // ceil(oh*ow / VEC)
};

template <int VEC>
__global__ __launch_bounds__(256) void im2col_kernel(I2CArgs a) {
  // grid: x -> position quads of one col row, y -> (image, col row)
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= a.quads) return;
  const int row = blockIdx.y % a.rows;
  const int64_t img = blockIdx.y / a.rows;
  const int kc = row % a.kW;
  const int t = row / a.kW;
  const int kr = t % a.kH;
  const int c = t / a.kH;
  const int ohw = a.oh * a.ow;
  const float* __restrict__ im = a.im + img * a.imStride + (int64_t)c * a.H * a.W;
  float* __restrict__ col = a.col + img * a.colStride + (int64_t)row * ohw;

  const int p0 = q * VEC;
  int orow = p0 / a.ow;
  int ocol = p0 - orow * a.ow;
  float v[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    const int ir = -a.padH + kr * a.dY + orow * a.sY;
    const int ic = -a.padW + kc * a.dX + ocol * a.sX;
    float x = 0.0f;
    if ((unsigned)ir < (unsigned)a.H && (unsigned)ic < (unsigned)a.W && p0 + e < ohw)
      x = im[ir * a.W + ic];
    v[e] = x;
    if (++ocol == a.ow) {
      ocol = 0;
      ++orow;
    }
  }
  if constexpr (VEC == 4) {
    *reinterpret_cast<float4*>(col + p0) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    if (p0 < ohw) col[p0] = v[0];
  }
}

// Row-staged im2col: a block owns (image, channel c, kernel row kr) and a
// chunk of R output rows.  It copies the R input rows that chunk reads
// (ir = -padH + kr*dY + orow*sY), zero-padded to Wp = W + 2*padW columns,
// into LDS once with coalesced loads, then writes the kW col rows (c, kr, kc)
// of the chunk — each a contiguous run of R*ow elements — from LDS.  Every
// input element is fetched from memory once per kernel row instead of once
// per (kr, kc) by scattered scalar loads.  Same values as the plain kernel.
typedef float floatx4 __attribute__((ext_vector_type(4)));

struct I2CRowArgs {
  I2CArgs g;
  int R;       // output rows per block
  int chunks;  // ceil(oh / R)
  int Wp;      // staged row length (covers every window column)
};

template <int VEC, bool NT>
__global__ __launch_bounds__(256) void im2col_rows_kernel(I2CRowArgs ra) {
  extern __shared__ float rows[];
  const I2CArgs& a = ra.g;
  const int chunk = blockIdx.x % ra.chunks;
  const int64_t t = blockIdx.x / ra.chunks;  // (image, c, kr)
  const int kr = (int)(t % a.kH);
  const int64_t t2 = t / a.kH;
  const int c = (int)(t2 % a.C);
  const int64_t img = t2 / a.C;
  const int orow0 = chunk * ra.R;
  const int nr = min(ra.R, a.oh - orow0);
  const float* __restrict__ im = a.im + img * a.imStride + (int64_t)c * a.H * a.W;
  const int Wp = ra.Wp;
  for (int i = threadIdx.x; i < nr * Wp; i += 256) {
    const int r = i / Wp, x = i - r * Wp;
    const int ir = -a.padH + kr * a.dY + (orow0 + r) * a.sY, ic = x - a.padW;
    rows[i] = ((unsigned)ir < (unsigned)a.H && (unsigned)ic < (unsigned)a.W) ? im[ir * a.W + ic]
                                                                            : 0.0f;
  }
  __syncthreads();
  const int ohw = a.oh * a.ow, n = nr * a.ow;
  for (int kc = 0; kc < a.kW; ++kc) {
    const int row = (c * a.kH + kr) * a.kW + kc;
    float* __restrict__ col = a.col + img * a.colStride + (int64_t)row * ohw + orow0 * a.ow;
    const int cx = kc * a.dX;
    if constexpr (VEC == 4) {
      // quads 256 apart per thread (each store instruction of a wave writes
      // 1 KB contiguous), four per pass: all LDS reads, then four stores
      constexpr int IT = 4;
      const int nq = n >> 2;
      const int dr = 1024 / a.ow, dc = 1024 - dr * a.ow;  // advance by 256 quads
      for (int q0 = threadIdx.x; q0 < nq; q0 += 256 * IT) {
        int r = (4 * q0) / a.ow;
        int oc0 = 4 * q0 - r * a.ow;
        floatx4 v[IT];
#pragma unroll
        for (int it = 0; it < IT; ++it) {
          int rr = r, oc = oc0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[it][e] = (q0 + 256 * it < nq) ? rows[rr * Wp + cx + oc * a.sX] : 0.0f;
            if (++oc == a.ow) {
              oc = 0;
              ++rr;
            }
          }
          r += dr;
          oc0 += dc;
          if (oc0 >= a.ow) {
            oc0 -= a.ow;
            ++r;
          }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it)
          if (q0 + 256 * it < nq) {
            floatx4* dst = reinterpret_cast<floatx4*>(col + 4 * (q0 + 256 * it));
            if constexpr (NT)
              __builtin_nontemporal_store(v[it], dst);
            else
              *dst = v[it];
          }
      }
    } else {
      for (int p0 = threadIdx.x; p0 < n; p0 += 256) {
        const int r = p0 / a.ow, oc = p0 - r * a.ow;
        col[p0] = rows[r * Wp + cx + oc * a.sX];
      }
    }
  }
}

struct C2IArgs {
  int C, H, W, kH, kW, padH, padW, sY, sX, dY, dX, oh, ow;
  const float* col;
  int64_t colStride;
  float* im;
  int64_t imStride;
  int64_t pixels;  // C*H*W
};

__global__ __launch_bounds__(256) void col2im_kernel(C2IArgs a) {
  const int64_t pix = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (pix >= a.pixels) return;
  const int64_t img = blockIdx.y;
  // within an image row, lanes take the columns of one residue class
  // x = k (mod sX) together (k-major order): the same kernel columns hit
  // them all and their col reads are consecutive, instead of sX-1 of sX lanes
  // idling per tap.  Per pixel nothing changes.
  const int q = (int)(pix % a.W);
  int x = q;
  if (a.sX > 1) {
    int k = 0, base = 0;
    while (k < a.sX - 1) {
      const int wk = (a.W - k + a.sX - 1) / a.sX;
      if (q < base + wk) break;
      base += wk;
      ++k;
    }
    x = k + (q - base) * a.sX;
  }
  const int y = (int)((pix / a.W) % a.H);
  const int c = (int)(pix / ((int64_t)a.W * a.H));
  float* __restrict__ im = a.im + img * a.imStride;
  const float* __restrict__ col = a.col + img * a.colStride;
  const int64_t ohw = (int64_t)a.oh * a.ow;
  const int64_t at = pix - q + x;
  float acc = im[at];
  for (int kr = 0; kr < a.kH; ++kr) {
    // rows: y = (kr - padH)*dY + orow*sY
    const int ry = y - (kr - a.padH) * a.dY;
    if (ry < 0 || ry % a.sY != 0) continue;
    const int orow = ry / a.sY;
    if (orow >= a.oh) continue;
    for (int kc = 0; kc < a.kW; ++kc) {
      const int rx = x - (kc - a.padW) * a.dX;
      if (rx < 0 || rx % a.sX != 0) continue;
      const int ocol = rx / a.sX;
      if (ocol >= a.ow) continue;
      const int64_t i = ((int64_t)c * a.kH + kr) * a.kW + kc;
      acc = acc + col[i * ohw + (int64_t)orow * a.ow + ocol];
    }
  }
  im[at] = acc;
}

// col2im_kernel with 32-bit pixel indexing (C*H*W < 2^31) and the stride
// as a template constant (S = sY = sX = 1 or 2; 0 = runtime): the per-tap
// divisibility tests and quotients become masks and shifts instead of
// integer divisions, which bound the general kernel.  Same adds, same order.
template <int S>
__global__ __launch_bounds__(256) void col2im_fast_kernel(C2IArgs a) {
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= (int)a.pixels) return;
  const int64_t img = blockIdx.y;
  const int sY = S ? S : a.sY, sX = S ? S : a.sX;
  const int rowi = pix / a.W;  // c*H + y
  const int q = pix - rowi * a.W;
  int x = q;
  if (sX > 1) {  // residue-class order, as col2im_kernel
    int k = 0, base = 0;
    while (k < sX - 1) {
      const int wk = (a.W - k + sX - 1) / sX;
      if (q < base + wk) break;
      base += wk;
      ++k;
    }
    x = k + (q - base) * sX;
  }
  const int c = rowi / a.H, y = rowi - c * a.H;
  float* __restrict__ im = a.im + img * a.imStride;
  const float* __restrict__ col = a.col + img * a.colStride;
  const int ohw = a.oh * a.ow;
  const int at = pix - q + x;
  float acc = im[at];
  for (int kr = 0; kr < a.kH; ++kr) {
    const int ry = y - (kr - a.padH) * a.dY;
    if (ry < 0 || ry % sY != 0) continue;
    const int orow = ry / sY;
    if (orow >= a.oh) continue;
    const float* __restrict__ crow = col + ((int64_t)(c * a.kH + kr) * a.kW) * ohw + orow * a.ow;
    for (int kc = 0; kc < a.kW; ++kc) {
      const int rx = x - (kc - a.padW) * a.dX;
      if (rx < 0 || rx % sX != 0) continue;
      const int ocol = rx / sX;
      if (ocol >= a.ow) continue;
      acc = acc + crow[(int64_t)kc * ohw + ocol];
    }
  }
  im[at] = acc;
}

}  // namespace

hipError_t launch_im2col(const ConvGeom& g, const float* im, int64_t imStride, float* col,
                         int64_t colStride, int64_t batch, hipStream_t s) {
  if (g.oh <= 0 || g.ow <= 0 || batch <= 0 || g.C <= 0) return hipSuccess;
  I2CArgs a;
  a.C = (int)g.C; a.H = (int)g.H; a.W = (int)g.W; a.kH = (int)g.kH; a.kW = (int)g.kW;
  a.padH = (int)g.padH; a.padW = (int)g.padW; a.sY = (int)g.sY; a.sX = (int)g.sX;
  a.dY = (int)g.dY; a.dX = (int)g.dX; a.oh = (int)g.oh; a.ow = (int)g.ow;
  a.im = im; a.imStride = imStride; a.col = col; a.colStride = colStride;
  a.rows = (int)(g.C * g.kH * g.kW);
  const int64_t ohw = g.oh * g.ow;
  const bool vec = (ohw % 4 == 0) && ((reinterpret_cast<uintptr_t>(col) & 15) == 0) &&
                   (colStride % 4 == 0 || batch == 1);
  const int VEC = vec ? 4 : 1;
  a.quads = (int)((ohw + VEC - 1) / VEC);
  // row-staged form: ~4096 (float4 form) or ~2048 col elements per kernel
  // column per block, chunks
  // of a multiple of 4 rows (aligned float4 runs) or the whole plane
  {
    // staged row: every window column (kc*dX + ocol*sX, zero outside the
    // image) — W + 2*padW, or more when out_dim's truncation toward zero
    // admits a window that overhangs the padded row
    const int64_t Wp = std::max<int64_t>(g.W + 2 * g.padW,
                                         (g.kW - 1) * g.dX + (g.ow - 1) * g.sX + 1);
    int64_t R = std::max<int64_t>(1, (vec ? 4096 : 2048) / g.ow);
    if (R >= g.oh)
      R = g.oh;
    else if (vec)
      R = std::max<int64_t>(4, R & ~int64_t(3));
    const int64_t chunks = (g.oh + R - 1) / R;
    const int64_t blocks = batch * g.C * g.kH * chunks;
    // the staged rows must fit LDS
    if (R * Wp * 4 <= 64 * 1024 && blocks <= 0x7fffffffLL) {
      I2CRowArgs ra;
      ra.g = a;
      ra.R = (int)R;
      ra.chunks = (int)chunks;
      ra.Wp = (int)Wp;
      const size_t lds = (size_t)(R * Wp * 4);
      // col matrices far larger than the caches stream past them
      // (nontemporal stores: 4.7-5.3 TB/s against 3.6-4.9 TB/s on the
      // large YOLOv3 layers); smaller ones stay cacheable for the GEMM
      const bool nt = batch * (int64_t)a.rows * ohw * 4 >= (int64_t)128 << 20;
      if (vec && nt)
        hipLaunchKernelGGL((im2col_rows_kernel<4, true>), dim3((unsigned)blocks), dim3(256), lds, s, ra);
      else if (vec)
        hipLaunchKernelGGL((im2col_rows_kernel<4, false>), dim3((unsigned)blocks), dim3(256), lds, s, ra);
      else
        hipLaunchKernelGGL((im2col_rows_kernel<1, false>), dim3((unsigned)blocks), dim3(256), lds, s, ra);
      return hipGetLastError();
    }
  }
  const int64_t ylim = 65535;
  const int64_t rows_total = (int64_t)a.rows * batch;
  // y = image*rows + row; split the batch so y fits the grid limit
  const int64_t imgs_per_launch = rows_total <= ylim ? batch : ylim / a.rows;
  if (imgs_per_launch <= 0) return hipErrorInvalidValue;
  for (int64_t b0 = 0; b0 < batch; b0 += imgs_per_launch) {
    const int64_t nb = batch - b0 < imgs_per_launch ? batch - b0 : imgs_per_launch;
    I2CArgs sub = a;
    sub.im = im + b0 * imStride;
    sub.col = col + b0 * colStride;
    dim3 grid((unsigned)((a.quads + 255) / 256), (unsigned)(nb * a.rows));
    if (vec)
      hipLaunchKernelGGL(im2col_kernel<4>, grid, dim3(256), 0, s, sub);
    else
      hipLaunchKernelGGL(im2col_kernel<1>, grid, dim3(256), 0, s, sub);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

namespace {
// 3x3 window, stride S (1 or 2): the nine taps' col entries are loaded
// together (taps outside the plane or off the stride grid read entry 0 and
// are skipped below), then added to the pixel in (kr, kc) order — the
// per-pixel order of col2im_fast_kernel, whose tap loop with its early
// continues issued one dependent load at a time.  Stride 2 keeps that
// kernel's lane order (the lanes of an image row take one column residue
// class together, so a tap's valid lanes read consecutive col entries).
template <int S>
__global__ __launch_bounds__(256) void col2im_k3_kernel(C2IArgs a) {
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= (int)a.pixels) return;
  const int64_t img = blockIdx.y;
  const int rowi = pix / a.W, q = pix - rowi * a.W;
  int x = q;
  if constexpr (S == 2) {
    const int w0 = (a.W + 1) / 2;  // columns of residue 0
    x = q < w0 ? 2 * q : 1 + 2 * (q - w0);
  }
  const int c = rowi / a.H, y = rowi - c * a.H;
  const int at = pix - q + x;
  float* __restrict__ im = a.im + img * a.imStride;
  const float* __restrict__ col = a.col + img * a.colStride;
  const int64_t ohw = (int64_t)a.oh * a.ow;
  float v[9];
  bool ok[9];
#pragma unroll
  for (int kr = 0; kr < 3; ++kr) {
    const int ry = y - (kr - a.padH) * a.dY;  // the reference's dilation formula
    const bool okr = ry >= 0 && ry % S == 0 && ry / S < a.oh;
#pragma unroll
    for (int kc = 0; kc < 3; ++kc) {
      const int rx = x - (kc - a.padW) * a.dX;
      const int t = kr * 3 + kc;
      ok[t] = okr && rx >= 0 && rx % S == 0 && rx / S < a.ow;
      v[t] = col[ok[t] ? (int64_t)(c * 9 + t) * ohw + (ry / S) * a.ow + rx / S : 0];
    }
  }
  float acc = im[at];
#pragma unroll
  for (int t = 0; t < 9; ++t)
    if (ok[t]) acc = acc + v[t];
  im[at] = acc;
}
}  // namespace

hipError_t launch_col2im(const ConvGeom& g, const float* col, int64_t colStride, float* im,
                         int64_t imStride, int64_t batch, hipStream_t s) {
  if (g.oh <= 0 || g.ow <= 0 || batch <= 0 || g.C <= 0) return hipSuccess;
  C2IArgs a;
  a.C = (int)g.C; a.H = (int)g.H; a.W = (int)g.W; a.kH = (int)g.kH; a.kW = (int)g.kW;
  a.padH = (int)g.padH; a.padW = (int)g.padW; a.sY = (int)g.sY; a.sX = (int)g.sX;
  a.dY = (int)g.dY; a.dX = (int)g.dX; a.oh = (int)g.oh; a.ow = (int)g.ow;
  a.col = col; a.colStride = colStride; a.im = im; a.imStride = imStride;
  a.pixels = g.C * g.H * g.W;
  for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
    const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
    C2IArgs sub = a;
    sub.col = col + b0 * colStride;
    sub.im = im + b0 * imStride;
    dim3 grid((unsigned)((a.pixels + 255) / 256), (unsigned)nb);
    if (a.pixels <= 0x7fffff00LL) {
      if (g.sY == 1 && g.sX == 1 && g.kH == 3 && g.kW == 3)
        hipLaunchKernelGGL(col2im_k3_kernel<1>, grid, dim3(256), 0, s, sub);
      else if (g.sY == 2 && g.sX == 2 && g.kH == 3 && g.kW == 3)
        hipLaunchKernelGGL(col2im_k3_kernel<2>, grid, dim3(256), 0, s, sub);
      else if (g.sY == 1 && g.sX == 1)
        hipLaunchKernelGGL(col2im_fast_kernel<1>, grid, dim3(256), 0, s, sub);
      else if (g.sY == 2 && g.sX == 2)
        hipLaunchKernelGGL(col2im_fast_kernel<2>, grid, dim3(256), 0, s, sub);
      else
        hipLaunchKernelGGL(col2im_fast_kernel<0>, grid, dim3(256), 0, s, sub);
    } else {
      hipLaunchKernelGGL(col2im_kernel, grid, dim3(256), 0, s, sub);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace tns
