// CRD's Embed head (reference distillers/CRD.py:101-113): out = l2norm(x W^T + b)
// on fp32 features [N, K] -> [N, D], forward in one launch, backward in two,
// instead of the linear + pow / sum / pow / div chain and its autograd.
//
// forward   block per row n: x row in LDS, thread j: y_j = b_j + sum_k W[j,k] x_k,
//           ||y|| by a block reduction, out = y / ||y||, norm[n] kept
// backward  (a) block per row: dy = (dout - out * <out, dout>) / ||y||, stored
//               for (b); dx_k = sum_j dy_j W[j,k] (threads over k: W rows
//               read coalesced)
//           (b) block per output j: dW[j,:] += sum_n dy[n,j] x[n,:],
//               db[j] += sum_n dy[n,j] -- straight into the flat gradient
// The sizes (N <= a few hundred, K <= 2048, D <= 1024) make this a latency
// problem, not an MFMA one: every launch is a single wave of blocks.
#include "common.h"

namespace {

constexpr int EMB_MAXK = 2048;
constexpr int EMB_MAXD = 1024;

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  const int nw = (blockDim.x + 63) >> 6;
  for (int w = 0; w < nw; ++w) t += red[w];
  return t;
}

__global__ void __launch_bounds__(256)
embed_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                 const float* __restrict__ b, float* __restrict__ out, float* __restrict__ norm,
                 int K, int D) {
  __shared__ float xs[EMB_MAXK];
  __shared__ float ys[EMB_MAXD];
  __shared__ float red[8];
  const int n = blockIdx.x;
  for (int k = threadIdx.x; k < K; k += blockDim.x) xs[k] = x[(int64_t)n * K + k];
  __syncthreads();
  float ss = 0.f;
  for (int j = threadIdx.x; j < D; j += blockDim.x) {
    const float* wr = w + (int64_t)j * K;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int k = 0;
    for (; k + 4 <= K; k += 4) {
      const float4 wv = *(const float4*)(wr + k);
      a0 += wv.x * xs[k]; a1 += wv.y * xs[k + 1]; a2 += wv.z * xs[k + 2]; a3 += wv.w * xs[k + 3];
    }
    for (; k < K; ++k) a0 += wr[k] * xs[k];
    const float y = (b ? b[j] : 0.f) + ((a0 + a1) + (a2 + a3));
    ys[j] = y;
    ss += y * y;
  }
  const float nrm = sqrtf(block_sum(ss, red));
  const float inv = 1.f / nrm;  // the reference divides by the norm unguarded
  for (int j = threadIdx.x; j < D; j += blockDim.x) out[(int64_t)n * D + j] = ys[j] * inv;
  if (threadIdx.x == 0) norm[n] = nrm;
}

__global__ void __launch_bounds__(256)
embed_bwd_rows_kernel(const float* __restrict__ dout, const float* __restrict__ out,
                      const float* __restrict__ norm, const float* __restrict__ w,
                      float* __restrict__ dy, float* __restrict__ dx, int K, int D) {
  __shared__ float ds[EMB_MAXD];
  __shared__ float red[8];
  const int n = blockIdx.x;
  float dot = 0.f;
  for (int j = threadIdx.x; j < D; j += blockDim.x)
    dot += out[(int64_t)n * D + j] * dout[(int64_t)n * D + j];
  dot = block_sum(dot, red);
  const float inv = 1.f / norm[n];
  for (int j = threadIdx.x; j < D; j += blockDim.x) {
    const float g = (dout[(int64_t)n * D + j] - out[(int64_t)n * D + j] * dot) * inv;
    ds[j] = g;
    dy[(int64_t)n * D + j] = g;
  }
  __syncthreads();
  if (dx == nullptr) return;
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    float a0 = 0.f, a1 = 0.f;
    int j = 0;
    for (; j + 2 <= D; j += 2) {
      a0 += ds[j] * w[(int64_t)j * K + k];
      a1 += ds[j + 1] * w[(int64_t)(j + 1) * K + k];
    }
    for (; j < D; ++j) a0 += ds[j] * w[(int64_t)j * K + k];
    dx[(int64_t)n * K + k] = a0 + a1;
  }
}

__global__ void __launch_bounds__(256)
embed_bwd_w_kernel(const float* __restrict__ dy, const float* __restrict__ x, float* __restrict__ dw,
                   float* __restrict__ db, int N, int K, int D) {
  const int j = blockIdx.x;
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    float a0 = 0.f, a1 = 0.f;
    int n = 0;
    for (; n + 2 <= N; n += 2) {
      a0 += dy[(int64_t)n * D + j] * x[(int64_t)n * K + k];
      a1 += dy[(int64_t)(n + 1) * D + j] * x[(int64_t)(n + 1) * K + k];
    }
    for (; n < N; ++n) a0 += dy[(int64_t)n * D + j] * x[(int64_t)n * K + k];
    dw[(int64_t)j * K + k] += a0 + a1;
  }
  if (db != nullptr && threadIdx.x == 0) {
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += dy[(int64_t)n * D + j];
    db[j] += s;
  }
}

}  // namespace

MDA_API int mda_embed_fwd(const float* x, const float* w, const float* b, float* out, float* norm,
                          int64_t N, int64_t K, int64_t D, hipStream_t st) {
  if (N < 1 || K < 1 || K > EMB_MAXK || D < 1 || D > EMB_MAXD || (K % 4)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3((unsigned)N), dim3(256), 0, st, x, w, b, out, norm,
                     (int)K, (int)D);
  MDA_CHECK_LAUNCH();
}

// dy: [N, D] scratch; dx (optional) [N, K]; dw [D, K] / db [D] accumulated.
MDA_API int mda_embed_bwd(const float* dout, const float* out, const float* norm, const float* x,
                          const float* w, float* dy, float* dx, float* dw, float* db, int64_t N,
                          int64_t K, int64_t D, hipStream_t st) {
  if (N < 1 || K < 1 || K > EMB_MAXK || D < 1 || D > EMB_MAXD) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(embed_bwd_rows_kernel, dim3((unsigned)N), dim3(256), 0, st, dout, out, norm, w,
                     dy, dx, (int)K, (int)D);
  { const int rc = (int)hipGetLastError(); if (rc) return rc; }
  if (dw == nullptr) return 0;
  hipLaunchKernelGGL(embed_bwd_w_kernel, dim3((unsigned)D), dim3(256), 0, st, dy, x, dw, db, (int)N,
                     (int)K, (int)D);
  MDA_CHECK_LAUNCH();
}
