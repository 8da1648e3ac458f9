// Attention-transfer loss, fused forward + backward (survey K8; reference
// distillers/AT.py:8-21, p = 2):
//
//   a[n, p]  = mean_c f[n, c, p]^2                (per pixel attention map)
//   â[n, :]  = a[n, :] / max(||a[n, :]||_2, 1e-12)
//   loss     = mean_{n, p} (â_s - â_t)^2
//   dL/df_s[n, c, p] = 2 f_s[n, c, p] / C * (g_p - â_p <g, â>) / ||a_s||,
//                      g = 2 (â_s - â_t) / (N * HW)
//
// One workgroup per sample; NHWC features so each pixel's channels are one
// contiguous run (16-byte loads).  The two maps live in LDS (HW <= 4096), the
// student feature is read twice (map, then gradient) and the teacher once;
// nothing of size C x HW is ever materialised.  Per-sample loss partials are
// summed by the last-arriving workgroup in a fixed order (deterministic).
#include "common.h"

namespace {

constexpr int MAXHW = 4096;

template <typename TS>
__device__ __forceinline__ float sumsq_pixel(const TS* __restrict__ f, int C) {
  float s = 0.f;
  for (int c = 0; c < C; ++c) {
    float v = io<TS>::ld(f, c);
    s += v * v;
  }
  return s;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  return t;
}

template <typename TS, typename TT>
__global__ void __launch_bounds__(256)
at_loss_kernel(const TS* __restrict__ fs, const TT* __restrict__ ft, TS* __restrict__ grad,
               float* __restrict__ loss, float* __restrict__ partial, unsigned* __restrict__ counter,
               int N, int C, int Ct, int HW) {
  __shared__ float as_[MAXHW];
  __shared__ float at_[MAXHW];
  __shared__ float red[8];
  const int n = blockIdx.x;
  const TS* fsn = fs + (int64_t)n * HW * C;
  const TT* ftn = ft + (int64_t)n * HW * Ct;
  float ss = 0.f, st = 0.f;
  for (int p = threadIdx.x; p < HW; p += blockDim.x) {
    float a = sumsq_pixel<TS>(fsn + (int64_t)p * C, C) / C;
    float b = sumsq_pixel<TT>(ftn + (int64_t)p * Ct, Ct) / Ct;
    as_[p] = a;
    at_[p] = b;
    ss += a * a;
    st += b * b;
  }
  const float ns = fmaxf(sqrtf(block_sum(ss, red)), 1e-12f);
  const float nt = fmaxf(sqrtf(block_sum(st, red)), 1e-12f);
  const float inv_ns = 1.f / ns, inv_nt = 1.f / nt;
  const float gscale = 2.f / ((float)N * HW);
  float l = 0.f, gdot = 0.f;
  for (int p = threadIdx.x; p < HW; p += blockDim.x) {
    float d = as_[p] * inv_ns - at_[p] * inv_nt;
    l += d * d;
    gdot += gscale * d * as_[p] * inv_ns;
  }
  l = block_sum(l, red);
  gdot = block_sum(gdot, red);
  for (int p = threadIdx.x; p < HW; p += blockDim.x) {
    float ah = as_[p] * inv_ns;
    float g = gscale * (ah - at_[p] * inv_nt);
    float dLda = (g - ah * gdot) * inv_ns * (2.f / C);
    const TS* src = fsn + (int64_t)p * C;
    TS* dst = grad + ((int64_t)n * HW + p) * C;
    for (int c = 0; c < C; ++c) io<TS>::st(dst, c, dLda * io<TS>::ld(src, c));
  }
  if (threadIdx.x == 0) partial[n] = l;
  if (mda_arrive(counter, gridDim.x)) {
    if (threadIdx.x < 64) {
      float t = 0.f;
      for (int i = threadIdx.x; i < (int)gridDim.x; i += 64) t += partial[i];
      t = wave_sum(t);
      if (threadIdx.x == 0) loss[0] = t / ((float)N * HW);
    }
  }
}

// OFD partial L2 (reference distillers/OFD.py:11-21) with its gradient in one
// pass.  s (student connector output) and t (teacher pre-ReLU feature) are
// [M, C] bf16 (NHWC, M = N*H*W), m the per-channel margin:
//   l = (s-m)^2 [s>m & t<=m] + (s-t)^2 [s>t & m<t<=0] + (s-t)^2 [t>0]
// loss = scale * sum l (scale = weight / N: the reference's mean over the
// batch then sum), grad = scale * dl/ds.  8 channels per thread-iteration,
// per-block partials summed in block order by the last-arriving block.
// margin == nullptr selects the plain squared error l = (s-t)^2 (FitNet's
// hint MSE, reference distillers/FitNet.py:41-43, scale = weight / numel).
__global__ void __launch_bounds__(256)
ofd_loss_kernel(const bf16_t* __restrict__ s, const bf16_t* __restrict__ t,
                const float* __restrict__ margin, bf16_t* __restrict__ grad, float* __restrict__ partial,
                unsigned* __restrict__ counter, float* __restrict__ loss, int64_t M, int C, float scale) {
  __shared__ float red[4];
  const int64_t total8 = M * C / 8;
  const int C8 = C / 8;
  float acc = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total8;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % C8) * 8;
    const uint4 us = *(const uint4*)(s + i * 8);
    const uint4 ut = *(const uint4*)(t + i * 8);
    const uint32_t ws[4] = {us.x, us.y, us.z, us.w}, wt[4] = {ut.x, ut.y, ut.z, ut.w};
    float g[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sv = __uint_as_float((e & 1) ? (ws[e >> 1] & 0xffff0000u) : (ws[e >> 1] << 16));
      const float tv = __uint_as_float((e & 1) ? (wt[e >> 1] & 0xffff0000u) : (wt[e >> 1] << 16));
      float l = 0.f, d = 0.f;
      if (margin == nullptr) {  // plain squared error (FitNet hint)
        const float q = sv - tv; l = q * q; d = 2.f * q;
      } else {
        const float mv = margin[c0 + e];
        if (sv > mv && tv <= mv) { const float q = sv - mv; l += q * q; d += 2.f * q; }
        if (sv > tv && tv > mv && tv <= 0.f) { const float q = sv - tv; l += q * q; d += 2.f * q; }
        if (tv > 0.f) { const float q = sv - tv; l += q * q; d += 2.f * q; }
      }
      acc += l;
      g[e] = scale * d;
    }
    *(uint4*)(grad + i * 8) = make_uint4(pack_bf16x2(g[0], g[1]), pack_bf16x2(g[2], g[3]),
                                         pack_bf16x2(g[4], g[5]), pack_bf16x2(g[6], g[7]));
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
  if (mda_arrive(counter, gridDim.x)) {
    if (threadIdx.x < 64) {
      float v = 0.f;
      for (int i = threadIdx.x; i < (int)gridDim.x; i += 64) v += partial[i];
      v = wave_sum(v);
      if (threadIdx.x == 0) loss[0] = v * scale;
    }
  }
}

}  // namespace

// s, t: [M, C] bf16 NHWC (C % 8 == 0); margin [C] fp32; grad like s; loss[1];
// partial >= 1024 floats; counter: one zeroed uint (reset by the kernel).
MDA_API int mda_ofd_loss(const void* s, const void* t, const float* margin, void* grad, float* loss,
                         float* partial, unsigned* counter, int64_t M, int64_t C, float scale,
                         hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
  int64_t blocks = (M * C / 8 + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(ofd_loss_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const bf16_t*)s,
                     (const bf16_t*)t, margin, (bf16_t*)grad, partial, counter, loss, M, (int)C, scale);
  MDA_CHECK_LAUNCH();
}

// fs [N, HW, C] (NHWC), ft [N, HW, Ct]; grad like fs; loss[1]; partial >= N floats.
MDA_API int mda_at_loss(int64_t dts, int64_t dtt, const void* fs, const void* ft, void* grad,
                        float* loss, float* partial, unsigned* counter, int64_t N, int64_t C,
                        int64_t Ct, int64_t HW, float p, hipStream_t st) {
  if (HW > MAXHW || p != 2.f) return (int)hipErrorInvalidValue;
#define AT_L(TS, TT)                                                                            \
  hipLaunchKernelGGL((at_loss_kernel<TS, TT>), dim3((int)N), dim3(256), 0, st, (const TS*)fs,   \
                     (const TT*)ft, (TS*)grad, loss, partial, counter, (int)N, (int)C, (int)Ct, \
                     (int)HW)
  if (dts == DT_F32 && dtt == DT_F32) AT_L(float, float);
  else if (dts == DT_BF16 && dtt == DT_BF16) AT_L(bf16_t, bf16_t);
  else if (dts == DT_BF16 && dtt == DT_F32) AT_L(bf16_t, float);
  else AT_L(float, bf16_t);
#undef AT_L
  MDA_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// VID Gaussian NLL (reference distillers/VID.py:16-30) on bf16 NHWC maps:
//   loss = mean_{m,c} 0.5 * ((pred - ft)^2 / var_c + log var_c),
//   var_c = softplus(log_scale_c) + eps.
// Everything the loss and both gradients need is S_c = sum_m (pred - ft)^2:
//   vid_sums     S_c by 8-channel row loops, block tree in LDS, fp64 atomics
//   vid_finalize the scalar loss (one block, fixed-order sums and tree)
//   vid_bwd      dpred = go * (pred - ft) / (var_c M C);  block 0:
//                dls_c = go * 0.5 (M / var_c - S_c / var_c^2) sigmoid(ls_c) / (M C)
namespace {
__device__ __forceinline__ float vid_var(float ls, float eps) {
  return (ls > 20.f ? ls : log1pf(expf(ls))) + eps;
}

__global__ void __launch_bounds__(256)
vid_sums_kernel(const bf16_t* __restrict__ pred, const bf16_t* __restrict__ ft, int M, int C,
                double* __restrict__ acc) {
  __shared__ float red[256 * 8];
  const int C8 = C / 8;
  const int rpi = 256 / C8;
  const int cg = threadIdx.x % C8, r0 = threadIdx.x / C8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (r0 < rpi) {
    for (int m = blockIdx.x * rpi + r0; m < M; m += gridDim.x * rpi) {
      const int64_t o = (int64_t)m * C + cg * 8;
      const uint4 a = *(const uint4*)(pred + o), b = *(const uint4*)(ft + o);
      const uint32_t aw[4] = {a.x, a.y, a.z, a.w}, bw[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float d0 = __uint_as_float(aw[k] << 16) - __uint_as_float(bw[k] << 16);
        const float d1 = __uint_as_float(aw[k] & 0xffff0000u) - __uint_as_float(bw[k] & 0xffff0000u);
        s[2 * k] += d0 * d0;
        s[2 * k + 1] += d1 * d1;
      }
    }
  }
  if (r0 < rpi) {
#pragma unroll
    for (int k = 0; k < 8; ++k) red[r0 * C + cg * 8 + k] = s[k];
  }
  __syncthreads();
  // this block's partial row (summed in block order by the finalize kernel:
  // deterministic, no float atomics)
  double* part = acc + (int64_t)C * (1 + blockIdx.x);
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float t = 0.f;
    for (int r = 0; r < rpi; ++r) t += red[r * C + c];
    part[c] = (double)t;
  }
}

__global__ void __launch_bounds__(256)
vid_finalize_kernel(double* __restrict__ acc, const float* __restrict__ ls, int M, int C,
                    float eps, float* __restrict__ loss, int nb) {
  __shared__ double red[256];
  double t = 0.0;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    // eight independent partial sums (rows b = k mod 8) keep eight loads in
    // flight: one accumulator chained all nb loads (74 us for nb = 512);
    // combined in a fixed order (deterministic)
    double sk[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    int b = 0;
    for (; b + 8 <= nb; b += 8) {
#pragma unroll
      for (int k = 0; k < 8; ++k) sk[k] += acc[(int64_t)C * (1 + b + k) + c];
    }
    for (int k = 0; b < nb; ++b, ++k) sk[k] += acc[(int64_t)C * (1 + b) + c];
    const double sc = ((sk[0] + sk[1]) + (sk[2] + sk[3])) + ((sk[4] + sk[5]) + (sk[6] + sk[7]));
    acc[c] = sc;  // S_c, read by the backward
    const double v = (double)vid_var(ls[c], eps);
    t += sc / v + (double)M * log(v);
  }
  red[threadIdx.x] = t;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = (float)(0.5 * red[0] / ((double)M * C));
}

__global__ void __launch_bounds__(256)
vid_bwd_kernel(const bf16_t* __restrict__ pred, const bf16_t* __restrict__ ft,
               const float* __restrict__ ls, const double* __restrict__ acc,
               const float* __restrict__ go, int M, int C, float eps, bf16_t* __restrict__ dpred,
               float* __restrict__ dls) {
  __shared__ float s_k[2048];
  const float g = go[0];
  const float inv_mc = 1.f / ((float)M * (float)C);
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float v = vid_var(ls[c], eps);
    s_k[c] = g * inv_mc / v;
    if (blockIdx.x == 0 && dls) {
      const float sg = 1.f / (1.f + expf(-ls[c]));
      dls[c] = g * 0.5f * inv_mc * ((float)M / v - (float)acc[c] / (v * v)) * sg;
    }
  }
  __syncthreads();
  const int c8 = C / 8;
  const int64_t total = (int64_t)M * c8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % c8) * 8;
    const uint4 a = *(const uint4*)(pred + i * 8), b = *(const uint4*)(ft + i * 8);
    const uint32_t aw[4] = {a.x, a.y, a.z, a.w}, bw[4] = {b.x, b.y, b.z, b.w};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float d0 = __uint_as_float(aw[k] << 16) - __uint_as_float(bw[k] << 16);
      const float d1 = __uint_as_float(aw[k] & 0xffff0000u) - __uint_as_float(bw[k] & 0xffff0000u);
      o[k] = pack_bf16x2(d0 * s_k[c0 + 2 * k], d1 * s_k[c0 + 2 * k + 1]);
    }
    *(uint4*)(dpred + i * 8) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}
}  // namespace

// acc: [C] fp64, zeroed by the caller; loss: [1] fp32.
// acc: (1 + VID_MAX_BLOCKS) * C doubles -- S_c, then the per-block partial rows
constexpr int VID_MAX_BLOCKS = 512;

MDA_API int mda_vid_loss(const void* pred, const void* ft, const float* log_scale, int64_t M,
                         int64_t C, float eps, double* acc, float* loss, hipStream_t st) {
  if (C % 8 || C > 2048 || M <= 0) return (int)hipErrorInvalidValue;
  const int C8 = (int)C / 8, rpi = 256 / C8;
  int nb = (int)std::min<int64_t>((M + 4 * rpi - 1) / (4 * rpi), VID_MAX_BLOCKS);
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL(vid_sums_kernel, dim3(nb), dim3(256), 0, st, (const bf16_t*)pred,
                     (const bf16_t*)ft, (int)M, (int)C, acc);
  { const int rc = (int)hipGetLastError(); if (rc) return rc; }
  hipLaunchKernelGGL(vid_finalize_kernel, dim3(1), dim3(256), 0, st, acc, log_scale,
                     (int)M, (int)C, eps, loss, nb);
  MDA_CHECK_LAUNCH();
}

// go: [1] fp32 upstream gradient (device); dls may be null.
MDA_API int mda_vid_bwd(const void* pred, const void* ft, const float* log_scale, const double* acc,
                        const float* go, int64_t M, int64_t C, float eps, void* dpred, float* dls,
                        hipStream_t st) {
  if (C % 8 || C > 2048 || M <= 0) return (int)hipErrorInvalidValue;
  const int64_t work = M * C / 8;
  const int nb = (int)std::min<int64_t>((work + 255) / 256, 2048);
  hipLaunchKernelGGL(vid_bwd_kernel, dim3(nb), dim3(256), 0, st, (const bf16_t*)pred,
                     (const bf16_t*)ft, log_scale, acc, go, (int)M, (int)C, eps, (bf16_t*)dpred,
                     dls);
  MDA_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// NST (reference distillers/NST.py:12-35) on the batched Gram of
// W = [F_s | F_t] (ops/feat_losses.py _NSTGram): g [N, 2C, 2C] fp32 = W^T W,
// r_i = sqrt(g_ii) (F.normalize's column norms), normalised Grams
// S = g_ss / (r r), X = g_st / (r r), T = g_tt / (r r).
//   nst_fwd  per-sample ||S||^2 + ||T||^2 - 2||X||^2 (one block per sample)
//   nst_bwd  PQ [N, 2C, C]: rows c < C:  P_cd = (k S_cd - [c==d] dot_c) / (r_c r_d)
//                           rows C + c:  Q_cd = -k g_{C+c,d} / (r_d^2 r_{C+c}^2)
//            dot_c = k (sum_d S_cd^2 - sum_d X_cd^2), k = 4 go / (N C^2);
//            dF_s = W PQ (one batched GEMM by the caller).
namespace {
constexpr int NST_CMAX = 1024;

__device__ __forceinline__ float nst_r(const float* g, int C2, int i) {
  return fmaxf(sqrtf(fmaxf(g[(int64_t)i * C2 + i], 0.f)), 1e-12f);
}

// grid (N, ceil(2C / NST_FROWS)): one wave per row (NST_FROWS / 4 rows per
// wave), 16-byte column loads when C % 4 == 0; rows c < C weigh the S columns
// +1 and the X columns -2, rows C + c only their T columns (+1).  One partial
// per block (part [N][gridDim.y], summed by the caller) -- spread over
// N * 2C / 32 blocks instead of one block per sample reading its whole
// 3C^2-entry Gram (141 us for C = 256 at N = 64, profiles/r4_prof_nst.md).
constexpr int NST_FROWS = 32;

template <bool VEC>
__global__ void __launch_bounds__(256)
nst_fwd_kernel(const float* __restrict__ g, int C, float* __restrict__ part) {
  __shared__ float rr[2 * NST_CMAX];
  __shared__ float red[4];
  const int C2 = 2 * C;
  const float* gn = g + (int64_t)blockIdx.x * C2 * C2;
  for (int i = threadIdx.x; i < C2; i += blockDim.x) rr[i] = 1.f / nst_r(gn, C2, i);
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float acc = 0.f;
  for (int q = 0; q < NST_FROWS / 4; ++q) {
    const int row = blockIdx.y * NST_FROWS + wave * (NST_FROWS / 4) + q;
    if (row >= C2) break;
    const float* gr = gn + (int64_t)row * C2;
    const float rrow = rr[row];
    const int c0 = row < C ? 0 : C;
    float a = 0.f;
    if (VEC) {
      for (int j = c0 + lane * 4; j < C2; j += 256) {
        const float4 v = *(const float4*)(gr + j);
        const float w = (row < C && j >= C) ? -2.f : 1.f;
        const float e0 = v.x * rr[j], e1 = v.y * rr[j + 1], e2 = v.z * rr[j + 2], e3 = v.w * rr[j + 3];
        a += w * ((e0 * e0 + e1 * e1) + (e2 * e2 + e3 * e3));
      }
    } else {
      for (int j = c0 + lane; j < C2; j += 64) {
        const float e = gr[j] * rr[j];
        a += ((row < C && j >= C) ? -2.f : 1.f) * e * e;
      }
    }
    acc += a * rrow * rrow;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) red[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0)
    part[(int64_t)blockIdx.x * gridDim.y + blockIdx.y] = (red[0] + red[1]) + (red[2] + red[3]);
}

// grid (N, 2C / 8): 8 rows of PQ per block, one wave per row pair
__global__ void __launch_bounds__(256)
nst_bwd_kernel(const float* __restrict__ g, int N, int C, const float* __restrict__ go,
               float* __restrict__ pq) {
  __shared__ float rr[2 * NST_CMAX];
  __shared__ float red[8][32];
  const int C2 = 2 * C;
  const int n = blockIdx.x;
  const float* gn = g + (int64_t)n * C2 * C2;
  for (int i = threadIdx.x; i < C2; i += blockDim.x) rr[i] = nst_r(gn, C2, i);
  __syncthreads();
  const float k = 4.f * go[0] / ((float)N * (float)C * (float)C);
  const int sub = threadIdx.x / 32, lane = threadIdx.x % 32;  // 8 rows x 32 threads
  const int row = blockIdx.y * 8 + sub;
  float dot = 0.f;
  if (row < C) {
    float a = 0.f;
    for (int d = lane; d < C; d += 32) {
      const float s = gn[(int64_t)row * C2 + d] / (rr[row] * rr[d]);
      const float x = gn[(int64_t)row * C2 + C + d] / (rr[row] * rr[C + d]);
      a += s * s - x * x;
    }
    red[sub][lane] = a;
  }
  __syncthreads();
  if (row < C) {
    float a = 0.f;
    for (int l = 0; l < 32; ++l) a += red[sub][l];
    dot = k * a;
  }
  if (row < C2) {
    float* out = pq + ((int64_t)n * C2 + row) * C;
    for (int d = lane; d < C; d += 32) {
      float v;
      if (row < C) {
        const float s = gn[(int64_t)row * C2 + d] / (rr[row] * rr[d]);
        v = (k * s - (row == d ? dot : 0.f)) / (rr[row] * rr[d]);
      } else {
        const float rd = rr[d], rc = rr[row];
        v = -k * gn[(int64_t)row * C2 + d] / (rd * rd * rc * rc);
      }
      out[d] = v;
    }
  }
}
}  // namespace

// part: [N][ceil(2C / 32)] fp32 partial sums (the loss numerator is their sum).
MDA_API int mda_nst_fwd(const float* g, int64_t N, int64_t C, float* part, hipStream_t st) {
  if (C <= 0 || C > NST_CMAX || N <= 0) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)N, (unsigned)((2 * C + NST_FROWS - 1) / NST_FROWS));
  if (C % 4 == 0)
    hipLaunchKernelGGL(nst_fwd_kernel<true>, grid, dim3(256), 0, st, g, (int)C, part);
  else
    hipLaunchKernelGGL(nst_fwd_kernel<false>, grid, dim3(256), 0, st, g, (int)C, part);
  MDA_CHECK_LAUNCH();
}

MDA_API int mda_nst_bwd(const float* g, int64_t N, int64_t C, const float* go, float* pq,
                        hipStream_t st) {
  if (C <= 0 || C > NST_CMAX || N <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(nst_bwd_kernel, dim3((unsigned)N, (unsigned)((2 * C + 7) / 8)), dim3(256), 0, st,
                     g, (int)N, (int)C, go, pq);
  MDA_CHECK_LAUNCH();
}
