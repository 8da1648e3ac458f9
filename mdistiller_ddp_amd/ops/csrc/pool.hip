// Max pooling on NHWC bf16 activations (survey K4): the ImageNet ResNet stem
// pool (3x3 / s2 / p1 on the 112x112 stem output) and the CIFAR VGG 2x2
// pools.  Forward writes the pooled map and, per output element, the window
// offset of its maximum (uint8); backward is a GATHER over the <= ceil(k/s)^2
// windows that contain each input pixel, so it is deterministic and
// atomic-free.  8 channels (16 bytes) per thread; ties keep the first
// maximum in window order, as PyTorch does.
#include "common.h"

namespace {

struct PoolParams {
  int N, H, W, C, Ho, Wo, k, s, p;
};

__global__ void __launch_bounds__(256)
maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, uint8_t* __restrict__ idx,
                   PoolParams q) {
  const int C8 = q.C / 8;
  const int64_t total = (int64_t)q.N * q.Ho * q.Wo * C8;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(t % C8);
    const int64_t pix = t / C8;
    const int ow = (int)(pix % q.Wo);
    const int64_t r = pix / q.Wo;
    const int oh = (int)(r % q.Ho);
    const int n = (int)(r / q.Ho);
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; }
    const int h0 = oh * q.s - q.p, w0 = ow * q.s - q.p;
    for (int kh = 0; kh < q.k; ++kh) {
      const int ih = h0 + kh;
      if ((unsigned)ih >= (unsigned)q.H) continue;
      for (int kw = 0; kw < q.k; ++kw) {
        const int iw = w0 + kw;
        if ((unsigned)iw >= (unsigned)q.W) continue;
        const uint4 v = *(const uint4*)(x + (((int64_t)n * q.H + ih) * q.W + iw) * q.C + c8 * 8);
        const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a = __uint_as_float(u[e] << 16), b = __uint_as_float(u[e] & 0xffff0000u);
          // first maximum wins; NaN propagates (as torch)
          if (a > best[2 * e] || (a != a && best[2 * e] == best[2 * e])) { best[2 * e] = a; bi[2 * e] = (uint8_t)(kh * q.k + kw); }
          if (b > best[2 * e + 1] || (b != b && best[2 * e + 1] == best[2 * e + 1])) { best[2 * e + 1] = b; bi[2 * e + 1] = (uint8_t)(kh * q.k + kw); }
        }
      }
    }
    const int64_t o = pix * q.C + c8 * 8;
    *(uint4*)(y + o) = make_uint4(pack_bf16x2(best[0], best[1]), pack_bf16x2(best[2], best[3]),
                                  pack_bf16x2(best[4], best[5]), pack_bf16x2(best[6], best[7]));
    if (idx) {
      uint2 packed;
      packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
      packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
      *(uint2*)(idx + o) = packed;
    }
  }
}

__global__ void __launch_bounds__(256)
maxpool_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                   bf16_t* __restrict__ dx, PoolParams q) {
  const int C8 = q.C / 8;
  const int64_t total = (int64_t)q.N * q.H * q.W * C8;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(t % C8);
    const int64_t pix = t / C8;
    const int iw = (int)(pix % q.W);
    const int64_t r = pix / q.W;
    const int ih = (int)(r % q.H);
    const int n = (int)(r / q.H);
    // outputs whose window holds (ih, iw): oh*s - p <= ih <= oh*s - p + k - 1
    const int ohl = max(0, (ih + q.p - q.k + q.s) / q.s), ohh = min(q.Ho - 1, (ih + q.p) / q.s);
    const int owl = max(0, (iw + q.p - q.k + q.s) / q.s), owh = min(q.Wo - 1, (iw + q.p) / q.s);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int oh = ohl; oh <= ohh; ++oh) {
      const int kh = ih - (oh * q.s - q.p);
      if (kh < 0 || kh >= q.k) continue;
      for (int ow = owl; ow <= owh; ++ow) {
        const int kw = iw - (ow * q.s - q.p);
        if (kw < 0 || kw >= q.k) continue;
        const uint8_t off = (uint8_t)(kh * q.k + kw);
        const int64_t o = (((int64_t)n * q.Ho + oh) * q.Wo + ow) * q.C + c8 * 8;
        const uint2 iv = *(const uint2*)(idx + o);
        const uint4 g = *(const uint4*)(dy + o);
        const uint32_t gu[4] = {g.x, g.y, g.z, g.w};
        const uint32_t iu[2] = {iv.x, iv.y};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint8_t w = (uint8_t)(iu[e >> 2] >> (8 * (e & 3)));
          const float gv = (e & 1) ? __uint_as_float(gu[e >> 1] & 0xffff0000u)
                                   : __uint_as_float(gu[e >> 1] << 16);
          if (w == off) acc[e] += gv;
        }
      }
    }
    *(uint4*)(dx + pix * q.C + c8 * 8) =
        make_uint4(pack_bf16x2(acc[0], acc[1]), pack_bf16x2(acc[2], acc[3]),
                   pack_bf16x2(acc[4], acc[5]), pack_bf16x2(acc[6], acc[7]));
  }
}

inline int grid_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

}  // namespace

// x [N, H, W, C] bf16 (C % 8 == 0) -> y [N, Ho, Wo, C] bf16, idx [N, Ho, Wo, C] uint8 (or null).
MDA_API int mda_maxpool_fwd(const void* x, void* y, void* idx, int64_t N, int64_t H, int64_t W,
                            int64_t C, int64_t Ho, int64_t Wo, int64_t k, int64_t s, int64_t p,
                            hipStream_t st) {
  if (C % 8 || k < 1 || k > 15 || s < 1 || p < 0 || 2 * p > k) return (int)hipErrorInvalidValue;
  PoolParams q{(int)N, (int)H, (int)W, (int)C, (int)Ho, (int)Wo, (int)k, (int)s, (int)p};
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for(N * Ho * Wo * C / 8)), dim3(256), 0, st,
                     (const bf16_t*)x, (bf16_t*)y, (uint8_t*)idx, q);
  MDA_CHECK_LAUNCH();
}

MDA_API int mda_maxpool_bwd(const void* dy, const void* idx, void* dx, int64_t N, int64_t H,
                            int64_t W, int64_t C, int64_t Ho, int64_t Wo, int64_t k, int64_t s,
                            int64_t p, hipStream_t st) {
  if (C % 8 || k < 1 || k > 15 || s < 1 || p < 0) return (int)hipErrorInvalidValue;
  PoolParams q{(int)N, (int)H, (int)W, (int)C, (int)Ho, (int)Wo, (int)k, (int)s, (int)p};
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for(N * H * W * C / 8)), dim3(256), 0, st,
                     (const bf16_t*)dy, (const uint8_t*)idx, (bf16_t*)dx, q);
  MDA_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Channel shuffle on NHWC bf16 (ShuffleNet, reference models/cifar/
// ShuffleNetv1.py:7-15 / ShuffleNetv2.py:22-31): y[m, j*g + i] = x[m, i*cpg + j]
// with cpg = C / g.  One thread per 2-channel output pair (4-byte stores),
// gathering inside the pixel's row (an L1/L2-resident C*2-byte span).  Its own
// inverse with g' = cpg, which is the backward.
namespace {
__global__ void __launch_bounds__(256)
channel_shuffle_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int64_t M, int C, int g) {
  const int cpg = C / g;
  const int64_t total2 = M * C / 2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total2;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = (i * 2) / C;
    const int c = (int)(i * 2 - m * C);
    const bf16_t* row = x + m * C;
    const int c1 = c + 1;
    const bf16_t a = row[(c % g) * cpg + c / g];
    const bf16_t b = row[(c1 % g) * cpg + c1 / g];
    *(uint32_t*)(y + i * 2) = (uint32_t)a | ((uint32_t)b << 16);
  }
}
}  // namespace

MDA_API int mda_channel_shuffle(const void* x, void* y, int64_t M, int64_t C, int64_t g, hipStream_t st) {
  if (C % g || C % 2) return (int)hipErrorInvalidValue;
  int64_t blocks = (M * C / 2 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(channel_shuffle_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const bf16_t*)x,
                     (bf16_t*)y, M, (int)C, (int)g);
  MDA_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Channel gather on NHWC bf16: y[m, c] = map[c] >= 0 ? x[m, map[c]] : 0, with
// Cx input and Cy output channels.  ShuffleNetV1 with physically padded groups
// (models/cifar/shufflenet.py): the channel shuffle between conv1 (groups of
// mid/g1 channels, each padded to a multiple of 8) and the grouped conv3
// (groups of mid/g, padded) is one such map; its backward is the inverse map.
// One thread per 2 output channels (4-byte stores); the map lives in LDS.
namespace {
__global__ void __launch_bounds__(256)
channel_gather_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                      const int* __restrict__ map, int64_t M, int Cx, int Cy) {
  __shared__ int smap[2048];
  for (int c = threadIdx.x; c < Cy; c += blockDim.x) smap[c] = map[c];
  __syncthreads();
  const int64_t total2 = M * Cy / 2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total2;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = (i * 2) / Cy;
    const int c = (int)(i * 2 - m * Cy);
    const bf16_t* row = x + m * Cx;
    const int j0 = smap[c], j1 = smap[c + 1];
    const uint32_t a = j0 >= 0 ? (uint32_t)row[j0] : 0u;
    const uint32_t b = j1 >= 0 ? (uint32_t)row[j1] : 0u;
    *(uint32_t*)(y + i * 2) = a | (b << 16);
  }
}
}  // namespace

// Two-source, two-destination channel gather:
//   y_d[m, c] = map_d[c] < 0 ? 0 : src_{map_d[c] >> 16}[m, map_d[c] & 0xffff]
// (row strides ld0 / ld1, destinations dense with Cy0 / Cy1 channels; Cy1 may
// be 0) -- ShuffleNetV2's concat + channel shuffle + split into the next
// unit's two channel-padded halves in ONE launch, and its backward (the
// inverse maps: both source gradients from both output gradients, one launch).
namespace {
__global__ void __launch_bounds__(256)
gather2_kernel(const bf16_t* __restrict__ x0, const bf16_t* __restrict__ x1, bf16_t* __restrict__ y0,
               bf16_t* __restrict__ y1, const int* __restrict__ map0, const int* __restrict__ map1,
               int64_t M, int ld0, int ld1, int Cy0, int Cy1) {
  __shared__ int smap[4096];
  const int Cy = Cy0 + Cy1;
  for (int c = threadIdx.x; c < Cy; c += blockDim.x) smap[c] = c < Cy0 ? map0[c] : map1[c - Cy0];
  __syncthreads();
  const int64_t total2 = M * Cy / 2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total2;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = (i * 2) / Cy;
    const int c = (int)(i * 2 - m * Cy);
    uint32_t v[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = smap[c + h];
      v[h] = 0u;
      if (e >= 0) {
        const int src = e >> 16, ch = e & 0xffff;
        v[h] = src ? (uint32_t)x1[m * ld1 + ch] : (uint32_t)x0[m * ld0 + ch];
      }
    }
    bf16_t* dst = c < Cy0 ? y0 + m * Cy0 + c : y1 + m * Cy1 + (c - Cy0);
    *(uint32_t*)dst = v[0] | (v[1] << 16);
  }
}
}  // namespace

MDA_API int mda_gather2(const void* x0, const void* x1, void* y0, const int* map0, int64_t Cy0,
                        void* y1, const int* map1, int64_t Cy1, int64_t M, int64_t ld0, int64_t ld1,
                        hipStream_t st) {
  if (Cy0 % 2 || Cy1 % 2 || Cy0 < 2 || Cy0 + Cy1 > 4096 || M < 1 || (Cy1 > 0 && !y1))
    return (int)hipErrorInvalidValue;
  int64_t blocks = (M * (Cy0 + Cy1) / 2 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(gather2_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const bf16_t*)x0,
                     (const bf16_t*)x1, (bf16_t*)y0, (bf16_t*)y1, map0, map1, M, (int)ld0, (int)ld1,
                     (int)Cy0, (int)Cy1);
  MDA_CHECK_LAUNCH();
}

MDA_API int mda_channel_gather(const void* x, void* y, const int* map, int64_t M, int64_t Cx,
                               int64_t Cy, hipStream_t st) {
  if (Cy % 2 || Cy > 2048 || Cx <= 0 || M <= 0) return (int)hipErrorInvalidValue;
  int64_t blocks = (M * Cy / 2 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(channel_gather_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     (const bf16_t*)x, (bf16_t*)y, map, M, (int)Cx, (int)Cy);
  MDA_CHECK_LAUNCH();
}


// ---------------------------------------------------------------------------
// ShuffleNetV1 stride-2 unit tail (reference ShuffleNetv1.py:49,57):
//   pre = cat([y3, avg_pool3x3_s2_p1(x)], channels); out = relu(pre)
// in ONE pass (the torch path ran avg_pool2d, cat and clamp: 3 launches), and
// its backward in one more: dz = dout * (pre > 0) (+ dpre); dy3 = dz[:, :C3];
// dxp = avg_pool backward of dz[:, C3:] as a gather over the <= 4 output
// pixels whose window covers each input pixel (count_include_pad: / 9).
// 8 channels per thread, 16-byte I/O; C3, Cx % 8 == 0.
namespace {

__device__ __forceinline__ void unpack8(const uint4& v, float (&f)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[2 * k] = __uint_as_float(w[k] << 16);
    f[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]),
                    pack_bf16x2(f[6], f[7]));
}

__global__ void __launch_bounds__(256)
shuffle_tail_fwd_kernel(const bf16_t* __restrict__ y3, const bf16_t* __restrict__ x,
                        bf16_t* __restrict__ pre, bf16_t* __restrict__ out, int N, int H, int W,
                        int Ho, int Wo, int C3, int Cx) {
  const int C = C3 + Cx, C8 = C / 8;
  const int64_t total = (int64_t)N * Ho * Wo * C8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / C8;
    const int c = (int)(i - m * C8) * 8;
    float v[8];
    if (c < C3) {
      unpack8(*(const uint4*)(y3 + m * C3 + c), v);
    } else {
      const int cx = c - C3;
      const int n = (int)(m / ((int64_t)Ho * Wo));
      const int r = (int)(m - (int64_t)n * Ho * Wo);
      const int oh = r / Wo, ow = r - (r / Wo) * Wo;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int ih = 2 * oh - 1 + kh, iw = 2 * ow - 1 + kw;
          if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) {
            float t[8];
            unpack8(*(const uint4*)(x + ((int64_t)(n * H + ih) * W + iw) * Cx + cx), t);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += t[e];
          }
        }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= (1.f / 9.f);
    }
    const uint4 pv = pack8(v);
    *(uint4*)(pre + m * C + c) = pv;
    float o[8];
    unpack8(pv, o);  // relu of the stored (rounded) pre-activation
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = fmaxf(o[e], 0.f);
    *(uint4*)(out + m * C + c) = pack8(o);
  }
}

__global__ void __launch_bounds__(256)
shuffle_tail_bwd_kernel(const bf16_t* __restrict__ dout, const bf16_t* __restrict__ dpre,
                        const bf16_t* __restrict__ pre, bf16_t* __restrict__ dy3,
                        bf16_t* __restrict__ dx, int N, int H, int W, int Ho, int Wo, int C3,
                        int Cx) {
  const int C = C3 + Cx;
  const int64_t n3 = (int64_t)N * Ho * Wo * (C3 / 8);
  const int64_t nx = (int64_t)N * H * W * (Cx / 8);
  auto dz8 = [&](int64_t o, float (&d)[8]) {
    float g[8], p[8];
    unpack8(*(const uint4*)(dout + o), g);
    unpack8(*(const uint4*)(pre + o), p);
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] = p[e] > 0.f ? g[e] : 0.f;
    if (dpre) {
      float q[8];
      unpack8(*(const uint4*)(dpre + o), q);
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] += q[e];
    }
  };
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n3 + nx;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (i < n3) {
      const int64_t m = i / (C3 / 8);
      const int c = (int)(i - m * (C3 / 8)) * 8;
      float d[8];
      dz8(m * C + c, d);
      *(uint4*)(dy3 + m * C3 + c) = pack8(d);
    } else {
      const int64_t j = i - n3;
      const int64_t px = j / (Cx / 8);
      const int cx = (int)(j - px * (Cx / 8)) * 8;
      const int n = (int)(px / ((int64_t)H * W));
      const int r = (int)(px - (int64_t)n * H * W);
      const int ih = r / W, iw = r - (r / W) * W;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int th = ih + 1 - kh;  // = 2 * oh
        if (th < 0 || (th & 1) || (th >> 1) >= Ho) continue;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int tw = iw + 1 - kw;
          if (tw < 0 || (tw & 1) || (tw >> 1) >= Wo) continue;
          float d[8];
          dz8(((int64_t)(n * Ho + (th >> 1)) * Wo + (tw >> 1)) * C + C3 + cx, d);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += d[e];
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] *= (1.f / 9.f);
      *(uint4*)(dx + px * Cx + cx) = pack8(acc);
    }
  }
}

inline int tail_blocks(int64_t work) {
  int64_t b = (work + 255) / 256;
  return (int)(b < 4096 ? (b < 1 ? 1 : b) : 4096);
}

}  // namespace

MDA_API int mda_shuffle_tail_fwd(const void* y3, const void* x, void* pre, void* out, int64_t N,
                                 int64_t H, int64_t W, int64_t Ho, int64_t Wo, int64_t C3,
                                 int64_t Cx, hipStream_t st) {
  if (C3 % 8 || Cx % 8 || Ho != (H + 1) / 2 || Wo != (W + 1) / 2) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(shuffle_tail_fwd_kernel, dim3(tail_blocks(N * Ho * Wo * (C3 + Cx) / 8)), dim3(256),
                     0, st, (const bf16_t*)y3, (const bf16_t*)x, (bf16_t*)pre, (bf16_t*)out, (int)N,
                     (int)H, (int)W, (int)Ho, (int)Wo, (int)C3, (int)Cx);
  MDA_CHECK_LAUNCH();
}

MDA_API int mda_shuffle_tail_bwd(const void* dout, const void* dpre, const void* pre, void* dy3,
                                 void* dx, int64_t N, int64_t H, int64_t W, int64_t Ho, int64_t Wo,
                                 int64_t C3, int64_t Cx, hipStream_t st) {
  if (C3 % 8 || Cx % 8 || Ho != (H + 1) / 2 || Wo != (W + 1) / 2) return (int)hipErrorInvalidValue;
  const int64_t work = N * Ho * Wo * C3 / 8 + N * H * W * Cx / 8;
  hipLaunchKernelGGL(shuffle_tail_bwd_kernel, dim3(tail_blocks(work)), dim3(256), 0, st,
                     (const bf16_t*)dout, (const bf16_t*)dpre, (const bf16_t*)pre, (bf16_t*)dy3,
                     (bf16_t*)dx, (int)N, (int)H, (int)W, (int)Ho, (int)Wo, (int)C3, (int)Cx);
  MDA_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Activation backward of a BN-less native conv (ops/hip_train.py _ConvTrain,
// e.g. VID's 1x1 -> ReLU regressors): dz = act'(pre) * dout (+ dpre), bf16,
// 8 elements per thread -- one launch instead of compare + where + fill.
namespace {
__global__ void __launch_bounds__(256)
act_bwd_kernel(const bf16_t* __restrict__ dout, const bf16_t* __restrict__ pre,
               const bf16_t* __restrict__ dpre, bf16_t* __restrict__ dz, int64_t n8, int act) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * blockDim.x) {
    float g[8], p[8], q[8];
    unpack8(((const uint4*)dout)[i], g);
    unpack8(((const uint4*)pre)[i], p);
    if (dpre) unpack8(((const uint4*)dpre)[i], q);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool on = act == 2 ? (p[e] > 0.f && p[e] < 6.f) : (act == 1 ? p[e] > 0.f : true);
      g[e] = (on ? g[e] : 0.f) + (dpre ? q[e] : 0.f);
    }
    ((uint4*)dz)[i] = pack8(g);
  }
}
}  // namespace

MDA_API int mda_act_bwd(const void* dout, const void* pre, const void* dpre, void* dz, int64_t n,
                        int64_t act, hipStream_t st) {
  if (n % 8 || n <= 0) return (int)hipErrorInvalidValue;
  int64_t blocks = (n / 8 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(act_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const bf16_t*)dout,
                     (const bf16_t*)pre, (const bf16_t*)dpre, (bf16_t*)dz, n / 8, (int)act);
  MDA_CHECK_LAUNCH();
}
