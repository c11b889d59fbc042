// Image pre-processing for the ImageNet ensemble example (SURVEY K14;
// reference examples/models/openvino_imagenet_ensemble/resources/transformer/
// ImageNetTransformer.py:20-63: cv2 decode -> centre crop (bilinear up-size of
// an axis shorter than the crop, cv2.INTER_LINEAR) -> HWC uint8 to CHW float).
//
// One fused pass: every output element (c, y, x) computes its source
// coordinate in the decoded HWC image (resize + crop folded into one affine
// map), samples bilinearly in uint8 and writes fp32 CHW -- the intermediate
// resized image never exists.  Threads are laid out along x so the fp32
// stores are coalesced; the uint8 HWC gathers hit L2 (a 224x224 crop of a
// multi-megapixel image is < 1 MiB).
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace sca::kern {
namespace {

// cv2 INTER_LINEAR source coordinate for destination index d along an axis
// resized from n_src to n_dst (pixel-centre aligned, clamped).
__device__ __forceinline__ void lin_src(int d, int n_src, int n_dst, int& i0, int& i1, float& w) {
  if (n_src == n_dst) {
    i0 = i1 = d;
    w = 0.f;
    return;
  }
  const float scale = float(n_src) / float(n_dst);
  float s = (float(d) + 0.5f) * scale - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = int(s);
  if (i0 > n_src - 1) i0 = n_src - 1;
  i1 = i0 + 1 < n_src ? i0 + 1 : n_src - 1;
  w = s - float(i0);
}

__global__ __launch_bounds__(256) void crop_resize_chw(const uint8_t* __restrict__ img, int H, int W, int C,
                                                       int rh, int rw, int crop, float* __restrict__ out) {
  const int x = blockIdx.x * 256 + threadIdx.x;
  const int y = blockIdx.y;
  if (x >= crop) return;
  // Resized image is rh x rw; crop window starts at its centre.
  const int sx = rw / 2 - crop / 2 + x, sy = rh / 2 - crop / 2 + y;
  int x0, x1, y0, y1;
  float wx, wy;
  lin_src(sx, W, rw, x0, x1, wx);
  lin_src(sy, H, rh, y0, y1, wy);
  for (int c = 0; c < C; ++c) {
    const float p00 = img[(size_t(y0) * W + x0) * C + c], p01 = img[(size_t(y0) * W + x1) * C + c];
    const float p10 = img[(size_t(y1) * W + x0) * C + c], p11 = img[(size_t(y1) * W + x1) * C + c];
    float v = (p00 * (1.f - wx) + p01 * wx) * (1.f - wy) + (p10 * (1.f - wx) + p11 * wx) * wy;
    if (rw != W || rh != H) v = rintf(v);  // cv2 resizes uint8 -> uint8 (rounded) before the float cast
    out[(size_t(c) * crop + y) * crop + x] = v;
  }
}

// Eval-mode BatchNorm + ReLU in one pass over a bf16 activation (DenseNet's
// pre-activation norm -> relu, which cannot fold into a neighbouring conv):
// out = max(0, x * scale[c] + shift[c]) in fp32, rounded to bf16.  Channels
// innermost (NHWC, `cl`): a thread takes 8 consecutive channels as one
// 16-byte load (C % 8 == 0); NCHW: 8 consecutive pixels of one channel
// (HW % 8 == 0).  Replaces two kernels and one round trip through HBM.
__device__ __forceinline__ float bf16_to_f32(unsigned short h) { return __uint_as_float(unsigned(h) << 16); }
__device__ __forceinline__ unsigned short f32_to_bf16(float f) {  // round to nearest even (no NaNs here)
  const unsigned u = __float_as_uint(f);
  return (unsigned short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

__global__ __launch_bounds__(256) void scale_shift_relu_bf16(const uint4* __restrict__ x, const float* __restrict__ scale,
                                                             const float* __restrict__ shift, int C, int HW, int cl,
                                                             size_t n8, uint4* __restrict__ out) {
  const size_t i = size_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n8) return;
  const uint4 v = x[i];
  const unsigned short* h = reinterpret_cast<const unsigned short*>(&v);
  uint4 r;
  unsigned short* o = reinterpret_cast<unsigned short*>(&r);
  if (cl) {
    const int c0 = int((i * 8) % size_t(C));
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = f32_to_bf16(fmaxf(0.f, bf16_to_f32(h[k]) * scale[c0 + k] + shift[c0 + k]));
  } else {
    const int c = int(((i * 8) / size_t(HW)) % size_t(C));
    const float a = scale[c], b = shift[c];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = f32_to_bf16(fmaxf(0.f, bf16_to_f32(h[k]) * a + b));
  }
  out[i] = r;
}

// ResNet's residual join, relu(a + b), on bf16 in one pass (8 elements per
// thread as 16-byte vectors): replaces PyTorch's add and its ReLU kernel.
__global__ __launch_bounds__(256) void add_relu_bf16(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                                     size_t n8, uint4* __restrict__ out) {
  const size_t i = size_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n8) return;
  const uint4 va = a[i], vb = b[i];
  const unsigned short* ha = reinterpret_cast<const unsigned short*>(&va);
  const unsigned short* hb = reinterpret_cast<const unsigned short*>(&vb);
  uint4 r;
  unsigned short* o = reinterpret_cast<unsigned short*>(&r);
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = f32_to_bf16(fmaxf(0.f, bf16_to_f32(ha[k]) + bf16_to_f32(hb[k])));
  out[i] = r;
}

}  // namespace

void add_relu_bf16(const void* a, const void* b, size_t n, void* out, hipStream_t s) {
  const size_t n8 = n / 8;
  if (n8 == 0) return;
  hipLaunchKernelGGL(add_relu_bf16, dim3(unsigned((n8 + 255) / 256)), dim3(256), 0, s, static_cast<const uint4*>(a),
                     static_cast<const uint4*>(b), n8, static_cast<uint4*>(out));
}

bool scale_shift_relu_bf16_ok(int C, int HW, int channels_last) {
  return channels_last ? C % 8 == 0 : HW % 8 == 0;
}

void scale_shift_relu_bf16(const void* x, const float* scale, const float* shift, int N, int C, int HW,
                           int channels_last, void* out, hipStream_t s) {
  const size_t n8 = size_t(N) * C * HW / 8;
  if (n8 == 0) return;
  hipLaunchKernelGGL(scale_shift_relu_bf16, dim3(unsigned((n8 + 255) / 256)), dim3(256), 0, s,
                     static_cast<const uint4*>(x), scale, shift, C, HW, channels_last, n8, static_cast<uint4*>(out));
}

void crop_resize_chw_u8(const uint8_t* img, int H, int W, int C, int crop, float* out, hipStream_t s) {
  const int rh = H < crop ? crop : H, rw = W < crop ? crop : W;
  hipLaunchKernelGGL(crop_resize_chw, dim3((crop + 255) / 256, crop), dim3(256), 0, s, img, H, W, C, rh, rw, crop,
                     out);
}

}  // namespace sca::kern
