// KDSVD loss after the SVDs (reference distillers/KDSVD.py:8-35, 62-71), one
// launch forward and one backward instead of ~450 PyTorch elementwise kernels.
//
// Per sample n and stage i (eigen-decompositions of the student / teacher
// Grams already done by csrc/eig.hip; vs, vt: [N, W, W] eigenvector COLUMNS,
// lt: [N, W] teacher eigenvalues, descending):
//   s_t[j]   = normalize(sqrt(max(lt[:k], 0)))              (F.normalize, eps 1e-12)
//   cos[a,j] = sum_w vs[w, a] vt[w, j]            a < k+3, j < k
//   mask[a,j]= sign(cos[a,j]) where |cos[a,j]| == max_a |cos[., j]|, else 0
//   us[p,j]  = s_t[j] sum_a vs[p, a] mask[a, j],   ut[p,j] = s_t[j] vt[p, j]
// and for consecutive stages (i-1, i):
//   loss += sum_{p,q,j} (exp(-(us_i[p,j]-us_{i-1}[q,j])^2/8)
//                        - exp(-(ut_i[p,j]-ut_{i-1}[q,j])^2/8))^2 / N
// (non-finite terms dropped).  The selection (mask) and the teacher side carry
// no gradient; the backward launch recomputes everything and writes
// dvs[p, a] = sum_j mask[a,j] s_t[j] dus[p,j] (zero for a >= k+3).
// One block per sample; every sum has a fixed thread order (deterministic).
#include "common.h"

namespace {

constexpr int KS_MAXS = 4;   // stages
constexpr int KS_MAXW = 63;  // Gram size (csrc/eig.hip limit)
constexpr int KS_MAXK = 8;   // k (teacher vectors); k + 3 student vectors

struct KsArgs {
  const float* vs[KS_MAXS];
  const float* vt[KS_MAXS];
  const float* lt[KS_MAXS];
  float* dvs[KS_MAXS];
  int W[KS_MAXS];
  int S, N, k;
  float* loss_part;  // [N] forward
  const float* go;   // backward: device scalar d loss
};

__global__ void __launch_bounds__(256) kdsvd_post_kernel(KsArgs a) {
  __shared__ float s_st[KS_MAXS][KS_MAXK];
  __shared__ float s_mask[KS_MAXS][KS_MAXK + 3][KS_MAXK];
  __shared__ float s_us[KS_MAXS][KS_MAXW * KS_MAXK];
  __shared__ float s_ut[KS_MAXS][KS_MAXW * KS_MAXK];
  __shared__ float s_dus[KS_MAXS][KS_MAXW * KS_MAXK];
  __shared__ float s_red[256];
  const int n = blockIdx.x, tid = threadIdx.x;
  const int k = a.k, ka = k + 3;
  const bool bwd = a.go != nullptr;

  // teacher scales
  if (tid < a.S) {
    const int i = tid, W = a.W[i];
    const float* lt = a.lt[i] + (int64_t)n * W;
    float s[KS_MAXK], ss = 0.f;
    for (int j = 0; j < k; ++j) {
      s[j] = sqrtf(fmaxf(lt[j], 0.f));
      ss += s[j] * s[j];
    }
    const float inv = 1.f / fmaxf(sqrtf(ss), 1e-12f);
    for (int j = 0; j < k; ++j) s_st[i][j] = s[j] * inv;
  }
  // alignment cosines -> s_mask (holds cos first)
  for (int i = 0; i < a.S; ++i) {
    const int W = a.W[i];
    const float* vs = a.vs[i] + (int64_t)n * W * W;
    const float* vt = a.vt[i] + (int64_t)n * W * W;
    for (int t = tid; t < ka * k; t += blockDim.x) {
      const int aa = t / k, j = t - aa * k;
      float c = 0.f;
      for (int w = 0; w < W; ++w) c += vs[w * W + aa] * vt[w * W + j];
      s_mask[i][aa][j] = c;
    }
  }
  __syncthreads();
  if (tid < a.S * k) {
    const int i = tid / k, j = tid - i * k;
    float mx = 0.f;
    for (int aa = 0; aa < ka; ++aa) mx = fmaxf(mx, fabsf(s_mask[i][aa][j]));
    for (int aa = 0; aa < ka; ++aa) {
      const float c = s_mask[i][aa][j];
      s_mask[i][aa][j] = fabsf(c) == mx ? (c > 0.f ? 1.f : (c < 0.f ? -1.f : 0.f)) : 0.f;
    }
  }
  __syncthreads();
  // scaled, aligned vectors
  for (int i = 0; i < a.S; ++i) {
    const int W = a.W[i];
    const float* vs = a.vs[i] + (int64_t)n * W * W;
    const float* vt = a.vt[i] + (int64_t)n * W * W;
    for (int t = tid; t < W * k; t += blockDim.x) {
      const int p = t / k, j = t - p * k;
      float u = 0.f;
      for (int aa = 0; aa < ka; ++aa) u += vs[p * W + aa] * s_mask[i][aa][j];
      s_us[i][t] = u * s_st[i][j];
      s_ut[i][t] = vt[p * W + j] * s_st[i][j];
      s_dus[i][t] = 0.f;
    }
  }
  __syncthreads();
  const float inv_n = 1.f / (float)a.N;
  float part = 0.f;
  for (int i = 1; i < a.S; ++i) {
    const int Wi = a.W[i], Wb = a.W[i - 1];
    const float* us = s_us[i];
    const float* ub = s_us[i - 1];
    const float* ut = s_ut[i];
    const float* tb = s_ut[i - 1];
    if (!bwd) {
      for (int t = tid; t < Wi * Wb * k; t += blockDim.x) {
        const int p = t / (Wb * k), r = t - p * (Wb * k), q = r / k, j = r - q * k;
        const float ds = us[p * k + j] - ub[q * k + j], dt = ut[p * k + j] - tb[q * k + j];
        const float e = expf(-ds * ds * 0.125f) - expf(-dt * dt * 0.125f);
        const float l = e * e;
        if (isfinite(l)) part += l;
      }
    } else {
      const float g0 = a.go[0] * inv_n;
      // d/d us_i[p, j]: sum over q (one thread per (p, j))
      for (int t = tid; t < Wi * k; t += blockDim.x) {
        const int p = t / k, j = t - p * k;
        float acc = 0.f;
        for (int q = 0; q < Wb; ++q) {
          const float ds = us[p * k + j] - ub[q * k + j], dt = ut[p * k + j] - tb[q * k + j];
          const float sr = expf(-ds * ds * 0.125f), e = sr - expf(-dt * dt * 0.125f);
          if (isfinite(e * e)) acc += 2.f * e * sr * (-0.25f * ds);
        }
        s_dus[i][t] += acc * g0;
      }
      __syncthreads();  // (the stage-(i-1) rows below may belong to other threads)
      // d/d us_{i-1}[q, j]: sum over p
      for (int t = tid; t < Wb * k; t += blockDim.x) {
        const int q = t / k, j = t - q * k;
        float acc = 0.f;
        for (int p = 0; p < Wi; ++p) {
          const float ds = us[p * k + j] - ub[q * k + j], dt = ut[p * k + j] - tb[q * k + j];
          const float sr = expf(-ds * ds * 0.125f), e = sr - expf(-dt * dt * 0.125f);
          if (isfinite(e * e)) acc += 2.f * e * sr * (0.25f * ds);
        }
        s_dus[i - 1][t] += acc * g0;
      }
      __syncthreads();
    }
  }
  if (!bwd) {
    s_red[tid] = part;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (tid < o) s_red[tid] += s_red[tid + o];
      __syncthreads();
    }
    if (tid == 0) a.loss_part[n] = s_red[0] * inv_n;
    return;
  }
  // dvs[p, aa] = sum_j mask[aa, j] s_t[j] dus[p, j]
  for (int i = 0; i < a.S; ++i) {
    const int W = a.W[i];
    float* dvs = a.dvs[i] + (int64_t)n * W * W;
    for (int t = tid; t < W * W; t += blockDim.x) {
      const int p = t / W, aa = t - p * W;
      float g = 0.f;
      if (aa < ka)
        for (int j = 0; j < k; ++j) g += s_mask[i][aa][j] * s_st[i][j] * s_dus[i][p * k + j];
      dvs[t] = g;
    }
  }
}

}  // namespace

// vs / vt / lt / dvs: arrays of S device pointers (host memory); W: S ints.
// go == null: forward (loss_part[N] = each sample's loss / N); else backward
// (dvs written in full).
MDA_API int mda_kdsvd_post(const int64_t* vs, const int64_t* vt, const int64_t* lt, const int64_t* dvs,
                           const int64_t* W, int64_t S, int64_t N, int64_t k, float* loss_part,
                           const float* go, hipStream_t st) {
  if (S < 2 || S > KS_MAXS || k < 1 || k > KS_MAXK || N < 1) return (int)hipErrorInvalidValue;
  KsArgs a{};
  for (int i = 0; i < S; ++i) {
    if (W[i] < k + 3 || W[i] > KS_MAXW) return (int)hipErrorInvalidValue;
    a.vs[i] = (const float*)vs[i];
    a.vt[i] = (const float*)vt[i];
    a.lt[i] = (const float*)lt[i];
    a.dvs[i] = go ? (float*)dvs[i] : nullptr;
    a.W[i] = (int)W[i];
  }
  if (go == nullptr && loss_part == nullptr) return (int)hipErrorInvalidValue;
  a.S = (int)S; a.N = (int)N; a.k = (int)k;
  a.loss_part = loss_part;
  a.go = go;
  hipLaunchKernelGGL(kdsvd_post_kernel, dim3((unsigned)N), dim3(256), 0, st, a);
  MDA_CHECK_LAUNCH();
}
