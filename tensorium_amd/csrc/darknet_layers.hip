// darknet_layers.hip — the non-convolutional layers of a YOLOv3 forward on
// the HIP backend: shortcut (TAddLayer.forward,
// naddlayer.pas:667-720: addvv then activate), upsample (upsample(),
// nupsamplelayer.pas:83-113, forward direction) and yolo (TYoloLayer.forward,
// nyololayer.pas:786-825: copy, then logistic over x, y and objectness +
// classes of every anchor).  Route (TConcatLayer) is a sequence of copies of
// whole tensors (TTensor.concat, ntensors.pas:12045-12061) done with
// tns_hip_copy.  All are HBM-bound streaming kernels, float4 where aligned.
#include "tns_act.hpp"
#include "tns_internal.hpp"

namespace tns {
namespace {

// out = act(a + b) — one rounding for the add (addvv), then the activation
__global__ void shortcut_kernel(int64_t n, const float* __restrict__ a,
                                const float* __restrict__ b, float* __restrict__ out, int act) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = act_apply(a[i] + b[i], act);
}
// float4 form (n % 4 == 0, 16-byte aligned operands): same add + activation
__global__ void shortcut4_kernel(int64_t n4, const float4* __restrict__ a,
                                 const float4* __restrict__ b, float4* __restrict__ out, int act) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float4 x = a[i], y = b[i];
    out[i] = make_float4(act_apply(x.x + y.x, act), act_apply(x.y + y.y, act),
                         act_apply(x.z + y.z, act), act_apply(x.w + y.w, act));
  }
}

// out[(p*H*s + y)*W*s + x] = scale * in[(p*H + y/s)*W + x/s]; one thread per
// output float4 when W*s is a multiple of 4
template <int V>
__global__ void upsample_kernel(int64_t planes, int H, int W, int s, float scale,
                                const float* __restrict__ in, float* __restrict__ out) {
  const int OW = W * s, OH = H * s;
  const int64_t total = planes * OH * (OW / V);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int xq = (int)(i % (OW / V));
    const int64_t r = i / (OW / V);  // output row (plane, y)
    const int y = (int)(r % OH);
    const int64_t p = r / OH;
    const float* src = in + (p * H + y / s) * W;
    float v[V];
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = scale * src[(V * xq + j) / s];
    if constexpr (V == 4)
      *reinterpret_cast<float4*>(out + r * OW + 4 * xq) = make_float4(v[0], v[1], v[2], v[3]);
    else
      out[r * OW + xq] = v[0];
  }
}

// per (image, anchor): entries 0,1 (x, y) and 4 .. 4+classes (objectness and
// class scores) through the logistic; w, h copied
__global__ void yolo_kernel(int64_t batch, int anchors, int classes, int64_t hw,
                            const float* __restrict__ in, float* __restrict__ out) {
  const int entries = classes + 5;
  const int64_t total = batch * anchors * entries * hw;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)((i / hw) % entries);
    const float x = in[i];
    out[i] = (e == 2 || e == 3) ? x : act_apply(x, 0);  // acLOGISTIC
  }
}

// backward direction (isForward = 0): in[(p*H + Y)*W + X] accumulates
// scale*out over its s x s output pixels in the CPU loop's order (output row
// outer, column inner; nupsamplelayer.pas:101-110), each product and sum
// rounded.  One thread per input pixel, so no races (the reference CUDA
// kernel has all s*s threads add into the same input pixel).  zeroIn starts
// from 0 instead of the current input (the reverse layer's output.fill(0)).
__global__ void upsample_back_kernel(int64_t planes, int H, int W, int s, float scale,
                                     float* __restrict__ in, const float* __restrict__ out,
                                     int zero) {
  const int64_t total = planes * H * W;
  const int OW = W * s;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int X = (int)(i % W);
    const int64_t r = i / W;  // (plane, Y)
    const int Y = (int)(r % H);
    const int64_t p = r / H;
    float v = zero ? 0.0f : in[i];
    const float* o = out + ((p * H + Y) * s) * (int64_t)OW + (int64_t)X * s;
    for (int dy = 0; dy < s; ++dy)
      for (int dx = 0; dx < s; ++dx) v = v + scale * o[(int64_t)dy * OW + dx];
    in[i] = v;
  }
}

int blocks_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 16384 ? 16384 : b));
}

}  // namespace

hipError_t launch_shortcut(int64_t n, const float* a, const float* b, float* out, int act,
                           hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const uintptr_t al = reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
                       reinterpret_cast<uintptr_t>(out);
  if (n % 4 == 0 && (al & 15) == 0) {
    hipLaunchKernelGGL(shortcut4_kernel, dim3(blocks_for(n / 4)), dim3(256), 0, s, n / 4,
                       reinterpret_cast<const float4*>(a), reinterpret_cast<const float4*>(b),
                       reinterpret_cast<float4*>(out), act);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(shortcut_kernel, dim3(blocks_for(n)), dim3(256), 0, s, n, a, b, out, act);
  return hipGetLastError();
}

hipError_t launch_upsample(int64_t planes, int H, int W, int stride, float scale, const float* in,
                           float* out, hipStream_t s) {
  const int64_t total = planes * H * stride * W * stride;
  if (total <= 0) return hipSuccess;
  const bool v4 = (W * stride) % 4 == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  if (v4)
    hipLaunchKernelGGL(upsample_kernel<4>, dim3(blocks_for(total / 4)), dim3(256), 0, s, planes, H,
                       W, stride, scale, in, out);
  else
    hipLaunchKernelGGL(upsample_kernel<1>, dim3(blocks_for(total)), dim3(256), 0, s, planes, H, W,
                       stride, scale, in, out);
  return hipGetLastError();
}

hipError_t launch_upsample_backward(int64_t planes, int H, int W, int stride, float scale,
                                   float* in, const float* out, int zero, hipStream_t s) {
  const int64_t total = planes * H * W;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(upsample_back_kernel, dim3(blocks_for(total)), dim3(256), 0, s, planes, H, W,
                     stride, scale, in, out, zero);
  return hipGetLastError();
}

hipError_t launch_yolo(int64_t batch, int anchors, int classes, int64_t hw, const float* in,
                       float* out, hipStream_t s) {
  const int64_t total = batch * anchors * (classes + 5) * hw;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(yolo_kernel, dim3(blocks_for(total)), dim3(256), 0, s, batch, anchors, classes,
                     hw, in, out);
  return hipGetLastError();
}

}  // namespace tns
