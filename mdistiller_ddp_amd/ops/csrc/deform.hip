// Deformable convolution (DCN v1 / modulated v2) sampling kernels for the
// detection backbone's DeformBottleneckBlock (reference
// detection/model/backbone/resnet.py:223-336, Detectron2's deform_conv ops).
//
// The convolution is split into a bilinear GATHER (this file) and plain GEMMs
// on hipBLASLt:
//   forward   cols[n, c*K + k, l] = m(n,g,k,l) * bilinear(x[n, c], p(n,g,k,l))
//             out[n] = W_g cols_g[n]                               (GEMM)
//   backward  dW = sum_n dout_g[n] cols_g[n]^T,  dcols = W_g^T dout_g  (GEMMs)
//             then ONE scatter pass: dx (bilinear weights, fp32 atomics),
//             d offset (the bilinear's coordinate derivative) and d mask,
//             owned per sample location -- no atomics for those.
// p = (kh*dil - pad + oh*stride + dy, kw*dil - pad + ow*stride + dx) with the
// offset layout [N, dg*K*2, Ho, Wo] (channel 2k = dy, 2k+1 = dx), mask
// [N, dg*K, Ho, Wo]; a corner outside the image contributes zero.
// One thread per (n, deformable group, tap, output pixel): the bilinear
// weights and corner addresses are computed once and reused for the group's
// C/dg channels; consecutive threads walk output pixels, so the cols writes
// (and the dcols reads) are coalesced.
#include "common.h"

namespace {

struct DefArgs {
  int N, C, H, W, Ho, Wo, KH, KW, sh, sw, ph, pw, dh, dw, dg;
};

struct Corners {
  int o[4];     // element offsets within a channel plane, -1 = outside
  float w[4];   // bilinear weights
  float ly, lx; // fractional parts (coordinate derivatives)
};

__device__ __forceinline__ Corners corners(float py, float px, int H, int W) {
  Corners c;
  const float y0f = floorf(py), x0f = floorf(px);
  const int y0 = (int)y0f, x0 = (int)x0f;
  c.ly = py - y0f;
  c.lx = px - x0f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int yy = y0 + (q >> 1), xx = x0 + (q & 1);
    const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
    const float wy = (q >> 1) ? c.ly : 1.f - c.ly, wx = (q & 1) ? c.lx : 1.f - c.lx;
    c.o[q] = ok ? yy * W + xx : -1;
    c.w[q] = ok ? wy * wx : 0.f;
  }
  return c;
}

template <typename T>
__global__ void __launch_bounds__(256)
deform_im2col_kernel(const T* __restrict__ x, const T* __restrict__ off, const T* __restrict__ mask,
                     T* __restrict__ cols, DefArgs a) {
  const int K = a.KH * a.KW, L = a.Ho * a.Wo, Cg = a.C / a.dg;
  const int64_t total = (int64_t)a.N * a.dg * K * L;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(i % L);
    int64_t r = i / L;
    const int k = (int)(r % K);
    r /= K;
    const int g = (int)(r % a.dg);
    const int n = (int)(r / a.dg);
    const int oh = l / a.Wo, ow = l - (l / a.Wo) * a.Wo;
    const int kh = k / a.KW, kw = k - (k / a.KW) * a.KW;
    const int64_t ob = (((int64_t)n * a.dg + g) * K + k) * 2 * L + l;
    const float py = (float)(oh * a.sh - a.ph + kh * a.dh) + io<T>::ld(off, ob);
    const float px = (float)(ow * a.sw - a.pw + kw * a.dw) + io<T>::ld(off, ob + L);
    const float m = mask ? io<T>::ld(mask, (((int64_t)n * a.dg + g) * K + k) * L + l) : 1.f;
    const Corners c = corners(py, px, a.H, a.W);
    const int64_t plane = (int64_t)a.H * a.W;
    const T* xs = x + ((int64_t)n * a.C + (int64_t)g * Cg) * plane;
    T* cs = cols + (((int64_t)n * a.C + (int64_t)g * Cg) * K + k) * L + l;
    for (int ci = 0; ci < Cg; ++ci) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (c.o[q] >= 0) v += c.w[q] * io<T>::ld(xs, c.o[q]);
      io<T>::st(cs, 0, m * v);
      xs += plane;
      cs += (int64_t)K * L;
    }
  }
}

// dcols [N, C*K, L] -> dx (accumulated, fp32), doff, dmask (written)
template <typename T>
__global__ void __launch_bounds__(256)
deform_col2im_kernel(const T* __restrict__ dcols, const T* __restrict__ x, const T* __restrict__ off,
                     const T* __restrict__ mask, float* __restrict__ dx, T* __restrict__ doff,
                     T* __restrict__ dmask, DefArgs a) {
  const int K = a.KH * a.KW, L = a.Ho * a.Wo, Cg = a.C / a.dg;
  const int64_t total = (int64_t)a.N * a.dg * K * L;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(i % L);
    int64_t r = i / L;
    const int k = (int)(r % K);
    r /= K;
    const int g = (int)(r % a.dg);
    const int n = (int)(r / a.dg);
    const int oh = l / a.Wo, ow = l - (l / a.Wo) * a.Wo;
    const int kh = k / a.KW, kw = k - (k / a.KW) * a.KW;
    const int64_t ob = (((int64_t)n * a.dg + g) * K + k) * 2 * L + l;
    const float py = (float)(oh * a.sh - a.ph + kh * a.dh) + io<T>::ld(off, ob);
    const float px = (float)(ow * a.sw - a.pw + kw * a.dw) + io<T>::ld(off, ob + L);
    const int64_t mo = (((int64_t)n * a.dg + g) * K + k) * L + l;
    const float m = mask ? io<T>::ld(mask, mo) : 1.f;
    const Corners c = corners(py, px, a.H, a.W);
    const int64_t plane = (int64_t)a.H * a.W;
    const T* xs = x + ((int64_t)n * a.C + (int64_t)g * Cg) * plane;
    float* dxs = dx + ((int64_t)n * a.C + (int64_t)g * Cg) * plane;
    const T* ds = dcols + (((int64_t)n * a.C + (int64_t)g * Cg) * K + k) * L + l;
    float gy = 0.f, gx = 0.f, gm = 0.f;
    for (int ci = 0; ci < Cg; ++ci) {
      const float d = io<T>::ld(ds, 0);
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = c.o[q] >= 0 ? io<T>::ld(xs, c.o[q]) : 0.f;
      const float val = c.w[0] * v[0] + c.w[1] * v[1] + c.w[2] * v[2] + c.w[3] * v[3];
      gm += d * val;
      const float dm = d * m;
      // bilinear coordinate derivatives (corner validity is piecewise constant)
      gy += dm * ((1.f - c.lx) * (v[2] - v[0]) + c.lx * (v[3] - v[1]));
      gx += dm * ((1.f - c.ly) * (v[1] - v[0]) + c.ly * (v[3] - v[2]));
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (c.o[q] >= 0 && c.w[q] != 0.f) atomicAdd(dxs + c.o[q], dm * c.w[q]);
      xs += plane;
      dxs += plane;
      ds += (int64_t)K * L;
    }
    io<T>::st(doff, ob, gy);
    io<T>::st(doff, ob + L, gx);
    if (dmask) io<T>::st(dmask, mo, gm);
  }
}

inline int def_blocks(int64_t total) {
  const int64_t b = (total + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

}  // namespace

// dt: 0 = fp32, 1 = bf16 (x, offset, mask, cols share it).  geom: 15 ints
// {N, C, H, W, Ho, Wo, KH, KW, sh, sw, ph, pw, dh, dw, dg} in host memory.
MDA_API int mda_deform_im2col(int64_t dt, const void* x, const void* off, const void* mask, void* cols,
                              const int64_t* geom, hipStream_t st) {
  DefArgs a{(int)geom[0], (int)geom[1], (int)geom[2], (int)geom[3], (int)geom[4], (int)geom[5],
            (int)geom[6], (int)geom[7], (int)geom[8], (int)geom[9], (int)geom[10], (int)geom[11],
            (int)geom[12], (int)geom[13], (int)geom[14]};
  if (a.dg < 1 || a.C % a.dg) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)a.N * a.dg * a.KH * a.KW * a.Ho * a.Wo;
  if (total <= 0) return 0;
  if (dt == DT_F32)
    hipLaunchKernelGGL(deform_im2col_kernel<float>, dim3(def_blocks(total)), dim3(256), 0, st,
                       (const float*)x, (const float*)off, (const float*)mask, (float*)cols, a);
  else
    hipLaunchKernelGGL(deform_im2col_kernel<bf16_t>, dim3(def_blocks(total)), dim3(256), 0, st,
                       (const bf16_t*)x, (const bf16_t*)off, (const bf16_t*)mask, (bf16_t*)cols, a);
  MDA_CHECK_LAUNCH();
}

// dx: fp32 [N, C, H, W], must be zeroed by the caller (accumulated atomically).
MDA_API int mda_deform_col2im(int64_t dt, const void* dcols, const void* x, const void* off,
                              const void* mask, float* dx, void* doff, void* dmask,
                              const int64_t* geom, hipStream_t st) {
  DefArgs a{(int)geom[0], (int)geom[1], (int)geom[2], (int)geom[3], (int)geom[4], (int)geom[5],
            (int)geom[6], (int)geom[7], (int)geom[8], (int)geom[9], (int)geom[10], (int)geom[11],
            (int)geom[12], (int)geom[13], (int)geom[14]};
  if (a.dg < 1 || a.C % a.dg) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)a.N * a.dg * a.KH * a.KW * a.Ho * a.Wo;
  if (total <= 0) return 0;
  if (dt == DT_F32)
    hipLaunchKernelGGL(deform_col2im_kernel<float>, dim3(def_blocks(total)), dim3(256), 0, st,
                       (const float*)dcols, (const float*)x, (const float*)off, (const float*)mask,
                       dx, (float*)doff, (float*)dmask, a);
  else
    hipLaunchKernelGGL(deform_col2im_kernel<bf16_t>, dim3(def_blocks(total)), dim3(256), 0, st,
                       (const bf16_t*)dcols, (const bf16_t*)x, (const bf16_t*)off,
                       (const bf16_t*)mask, dx, (bf16_t*)doff, (bf16_t*)dmask, a);
  MDA_CHECK_LAUNCH();
}
