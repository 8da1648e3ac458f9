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
#include <algorithm>

#include "common.h"

namespace {

constexpr int KS_MAXS = 4;   // stages
constexpr int KS_MAXW = 63;  // Gram size (csrc/eig.hip limit)
constexpr int KS_MAXK = 8;   // k (teacher vectors); k + 3 student vectors
constexpr float KS_DEGEN = 1e-6f;  // relative eigenvalue gap treated as degenerate (_GramEig too)

struct KsArgs {
  const float* vs[KS_MAXS];
  const float* vt[KS_MAXS];
  const float* lt[KS_MAXS];
  float* dvs[KS_MAXS];
  const float* ls[KS_MAXS];  // student eigenvalues [N, W] (D mode)
  float* ds[KS_MAXS];        // D mode: symmetrised Gram gradient dG + dG^T [N, W, W]
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
  __shared__ float s_dv[KS_MAXW * (KS_MAXK + 3)];
  __shared__ float s_k[KS_MAXW * (KS_MAXK + 3)];
  __shared__ float s_u[KS_MAXW * (KS_MAXK + 3)];
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
  if (a.ds[0] == nullptr) {
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
    return;
  }
  // D mode: through the eigendecomposition's backward as well (the
  // _GramEig.backward algebra with dV nonzero in its first ka columns only):
  //   K[i, j] = (v_i . dv_j) / (lam_j - lam_i)  (i != j, lam_i != lam_j; j < ka)
  //   U = V K,  D = dG + dG^T = sum_j (U_j v_j^T + v_j U_j^T)
  // and the caller forms dX = X D.
  for (int i = 0; i < a.S; ++i) {
    const int W = a.W[i];
    const float* vs = a.vs[i] + (int64_t)n * W * W;
    const float* lam = a.ls[i] + (int64_t)n * W;
    for (int t = tid; t < W * ka; t += blockDim.x) {
      const int p = t / ka, aa = t - p * ka;
      float g = 0.f;
      for (int j = 0; j < k; ++j) g += s_mask[i][aa][j] * s_st[i][j] * s_dus[i][p * k + j];
      s_dv[t] = g;
    }
    __syncthreads();
    // eigenvalues closer than 1e-6 of the largest (below the fp32
    // eigensolver's resolution) are one degenerate subspace: no term
    const float thr = KS_DEGEN * fabsf(lam[0]);
    for (int t = tid; t < W * ka; t += blockDim.x) {
      const int ii = t / ka, aa = t - ii * ka;
      float m = 0.f;
      for (int p = 0; p < W; ++p) m += vs[p * W + ii] * s_dv[p * ka + aa];
      const float diff = lam[aa] - lam[ii];
      s_k[t] = (ii != aa && fabsf(diff) > thr) ? m / diff : 0.f;
    }
    __syncthreads();
    for (int t = tid; t < W * ka; t += blockDim.x) {
      const int p = t / ka, aa = t - p * ka;
      float u = 0.f;
      for (int ii = 0; ii < W; ++ii) u += vs[p * W + ii] * s_k[ii * ka + aa];
      s_u[t] = u;
    }
    __syncthreads();
    float* d = a.ds[i] + (int64_t)n * W * W;
    for (int t = tid; t < W * W; t += blockDim.x) {
      const int p = t / W, q = t - p * W;
      float g = 0.f;
      for (int aa = 0; aa < ka; ++aa)
        g += s_u[p * ka + aa] * vs[q * W + aa] + vs[p * W + aa] * s_u[q * ka + aa];
      d[t] = g;
    }
    __syncthreads();  // s_dv / s_k / s_u reused by the next stage
  }
}

// ---------------------------------------------------------------------------
// The stages' Grams straight from the NHWC feature maps (bf16 or fp32):
// G_n[w1, w2] = sum_{h, c} x[n, h, w1, c] x[n, h, w2, c] -- the reference's
// X = feat.view(N, C*H, W) Gram -- fp32 accumulation, each block over one
// sample and one of KSPLIT row ranges (partial Grams summed by the
// eigensolver's loader, csrc/eig.hip).  Table entries: one per (stage,
// student/teacher), all in one launch.
constexpr int KG_MAXE = 8;
constexpr int KG_CC = 64;  // channels per LDS chunk
struct KgEntry {
  const void* x; float* g;
  int64_t pstride;  // floats between the KSPLIT partial Grams
  int B, H, W, C, bf16;
};
struct KgTable { KgEntry e[KG_MAXE]; int ksplit; };

__device__ __forceinline__ float kg_load(const void* x, int64_t i, int bf16) {
  return bf16 ? bf2f(((const bf16_t*)x)[i]) : ((const float*)x)[i];
}

template <int R>
__global__ void __launch_bounds__(256) kdsvd_gram_kernel(KgTable tab) {
  __shared__ float sl[KS_MAXW][KG_CC + 1];
  const KgEntry& en = tab.e[blockIdx.y];
  const int n = blockIdx.x, ks = blockIdx.z, tid = threadIdx.x;
  if (n >= en.B) return;
  const int H = en.H, W = en.W, C = en.C;
  const int h0 = (int)((int64_t)H * ks / tab.ksplit), h1 = (int)((int64_t)H * (ks + 1) / tab.ksplit);
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.f;
  for (int h = h0; h < h1; ++h) {
    const int64_t base = ((int64_t)n * H + h) * W * C;
    for (int c0 = 0; c0 < C; c0 += KG_CC) {
      const int cc = min(KG_CC, C - c0);
      __syncthreads();
      for (int t = tid; t < W * KG_CC; t += 256) {
        const int w = t / KG_CC, c = t - w * KG_CC;
        sl[w][c] = c < cc ? kg_load(en.x, base + (int64_t)w * C + c0 + c, en.bf16) : 0.f;
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int o = tid + 256 * r;
        if (o < W * W) {
          const int w1 = o / W, w2 = o - w1 * W;
          float s = 0.f;
          for (int c = 0; c < cc; ++c) s += sl[w1][c] * sl[w2][c];
          acc[r] += s;
        }
      }
    }
  }
  float* g = en.g + ks * en.pstride + (int64_t)n * W * W;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int o = tid + 256 * r;
    if (o < W * W) g[o] = acc[r];
  }
}

// bf16 Grams on the matrix cores: G = X^T X is A * A^T with A = X^T, so
// one fragment serves as both operands.  Block = one sample of one entry,
// wave q = the q-th quarter of the rows h (partial Gram q of KG_WAVES).
//   W > 16: mfma_f32_32x32x16_bf16, lane (pixel r = l & 31, half hh = l >> 5)
//           holds channels c + 8hh .. +8 of pixel r (C % 16 == 0);
//   W <= 16: mfma_f32_16x16x32_bf16, lane (pixel l & 15, group l >> 4) holds
//           channels c + 8 (l >> 4) .. +8 (C % 32 == 0).
constexpr int KG_WAVES = 4;
typedef __attribute__((ext_vector_type(8))) __bf16 kg_bf16x8;
typedef __attribute__((ext_vector_type(16))) float kg_f32x16;
typedef __attribute__((ext_vector_type(4))) float kg_f32x4;

__device__ __forceinline__ kg_bf16x8 kg_frag(const bf16_t* p, bool ok) {
  const uint4 v = ok ? *(const uint4*)p : make_uint4(0, 0, 0, 0);
  return __builtin_bit_cast(kg_bf16x8, v);
}

__global__ void __launch_bounds__(256) kdsvd_gram_mfma_kernel(KgTable tab) {
  const KgEntry& en = tab.e[blockIdx.y];
  const int n = blockIdx.x;
  if (n >= en.B) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int H = en.H, W = en.W, C = en.C;
  const int h0 = H * wave / KG_WAVES, h1 = H * (wave + 1) / KG_WAVES;
  const bf16_t* x = (const bf16_t*)en.x + (int64_t)n * H * W * C;
  float* g = en.g + wave * en.pstride + (int64_t)n * W * W;
  if (W > 16) {
    const int r = lane & 31, hh = lane >> 5;
    const bool ok = r < W;
    kg_f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    for (int h = h0; h < h1; ++h) {
      const bf16_t* px = x + ((int64_t)h * W + (ok ? r : 0)) * C + 8 * hh;
      for (int c = 0; c < C; c += 64) {
        kg_bf16x8 f[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) f[u] = kg_frag(px + c + 16 * u, ok && c + 16 * u < C);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[u], f[u], acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = (i & 3) + 8 * (i >> 2) + 4 * hh;
      if (row < W && r < W) g[row * W + r] = acc[i];
    }
  } else {
    const int r = lane & 15, q = lane >> 4;
    const bool ok = r < W;
    kg_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int h = h0; h < h1; ++h) {
      const bf16_t* px = x + ((int64_t)h * W + (ok ? r : 0)) * C + 8 * q;
      for (int c = 0; c < C; c += 128) {
        kg_bf16x8 f[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) f[u] = kg_frag(px + c + 32 * u, ok && c + 32 * u < C);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[u], f[u], acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = q * 4 + i;
      if (row < W && r < W) g[row * W + r] = acc[i];
    }
  }
}

// dX = X D per (sample, row h) slab: dx[n, h, w, c] = sum_w' x[n, h, w', c] D_n[w', w]
// (D symmetric), output in x's dtype and NHWC layout.  One entry per stage.
struct KaEntry {
  const void* x; const float* d; void* dx;
  int B, H, W, C, bf16;
};
struct KaTable { KaEntry e[KS_MAXS]; };

__global__ void __launch_bounds__(256) kdsvd_gram_apply_kernel(KaTable tab) {
  // D [w'][w] (row stride 64) and a 64-channel chunk of the slab in LDS;
  // thread (channel c = tid & 63, quarter wq = tid >> 6) owns outputs
  // w = wq*WQ .. +WQ of channel c: per w' one slab read and WQ FMAs against
  // wave-uniform (broadcast) D reads
  __shared__ float sd[KS_MAXW * 64];
  __shared__ float xs[KS_MAXW][64];
  const KaEntry& en = tab.e[blockIdx.y];
  const int H = en.H, W = en.W, C = en.C;
  const int slab = blockIdx.x;
  if (slab >= en.B * H) return;
  const int n = slab / H;
  const float* d = en.d + (int64_t)n * W * W;
  for (int t = threadIdx.x; t < W * W; t += 256) {
    const int a = t / W;
    sd[a * 64 + (t - a * W)] = d[t];
  }
  const int c = threadIdx.x & 63, wq = threadIdx.x >> 6;
  const int WQ = (W + 3) / 4;
  const int64_t base = (int64_t)slab * W * C;
  for (int c0 = 0; c0 < C; c0 += 64) {
    __syncthreads();
    for (int t = threadIdx.x; t < W * 64; t += 256) {
      const int w = t >> 6, cc = t & 63;
      xs[w][cc] = c0 + cc < C ? kg_load(en.x, base + (int64_t)w * C + c0 + cc, en.bf16) : 0.f;
    }
    __syncthreads();
    float acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    for (int w2 = 0; w2 < W; ++w2) {
      const float xv = xs[w2][c];
      const float* drow = sd + w2 * 64 + wq * WQ;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (i < WQ) acc[i] += xv * drow[i];
    }
    if (c0 + c < C) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int w = wq * WQ + i;
        if (i < WQ && w < W) {
          const int64_t o = base + (int64_t)w * C + c0 + c;
          if (en.bf16)
            ((bf16_t*)en.dx)[o] = f2bf(acc[i]);
          else
            ((float*)en.dx)[o] = acc[i];
        }
      }
    }
  }
}

}  // namespace

// vs / vt / lt / dvs: arrays of S device pointers (host memory); W: S ints.
// go == null: forward (loss_part[N] = each sample's loss / N); else backward
// (dvs written in full).
// ls / ds (may be null): student eigenvalue and D-output pointer arrays -- with
// ds the backward writes D = dG + dG^T of each stage (see the kernel) instead of dvs.
MDA_API int mda_kdsvd_post(const int64_t* vs, const int64_t* vt, const int64_t* lt, const int64_t* dvs,
                           const int64_t* W, int64_t S, int64_t N, int64_t k, float* loss_part,
                           const float* go, const int64_t* ls, const int64_t* ds, hipStream_t st) {
  if (S < 2 || S > KS_MAXS || k < 1 || k > KS_MAXK || N < 1) return (int)hipErrorInvalidValue;
  KsArgs a{};
  for (int i = 0; i < S; ++i) {
    if (W[i] < k + 3 || W[i] > KS_MAXW) return (int)hipErrorInvalidValue;
    a.vs[i] = (const float*)vs[i];
    a.vt[i] = (const float*)vt[i];
    a.lt[i] = (const float*)lt[i];
    a.dvs[i] = go && dvs ? (float*)dvs[i] : nullptr;
    a.ls[i] = ls ? (const float*)ls[i] : nullptr;
    a.ds[i] = go && ds ? (float*)ds[i] : nullptr;
    if (a.ds[i] && !a.ls[i]) return (int)hipErrorInvalidValue;
    a.W[i] = (int)W[i];
  }
  if (go == nullptr && loss_part == nullptr) return (int)hipErrorInvalidValue;
  a.S = (int)S; a.N = (int)N; a.k = (int)k;
  a.loss_part = loss_part;
  a.go = go;
  if (go && a.ds[0] == nullptr && a.dvs[0] == nullptr) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kdsvd_post_kernel, dim3((unsigned)N), dim3(256), 0, st, a);
  MDA_CHECK_LAUNCH();
}

// table int64 [E][8] rows (x, g, pstride, B, H, W, C, bf16), E <= 8; every
// block of entry e writes partial Gram ks at g + ks * pstride (ksplit parts).
MDA_API int mda_kdsvd_gram(const int64_t* table, int64_t E, int64_t ksplit, hipStream_t st) {
  if (E < 1 || E > KG_MAXE || ksplit < 1 || ksplit > 64) return (int)hipErrorInvalidValue;
  KgTable tab{};
  tab.ksplit = (int)ksplit;
  int bmax = 0, wmax = 0;
  for (int e = 0; e < E; ++e) {
    const int64_t* r = table + 8 * e;
    if (r[3] < 1 || r[3] > 65535 || r[4] < 1 || r[5] < 1 || r[5] > KS_MAXW || r[6] < 1)
      return (int)hipErrorInvalidValue;
    tab.e[e] = KgEntry{(const void*)r[0], (float*)r[1], r[2], (int)r[3], (int)r[4], (int)r[5],
                       (int)r[6], (int)r[7]};
    bmax = std::max(bmax, (int)r[3]);
    wmax = std::max(wmax, (int)r[5]);
  }
  if (ksplit == KG_WAVES) {
    bool mfma = true;
    for (int e = 0; e < E; ++e) {
      const KgEntry& k = tab.e[e];
      mfma = mfma && k.bf16 && k.W <= 32 && (k.W > 16 ? k.C % 16 == 0 : k.C % 32 == 0) &&
             ((uintptr_t)k.x & 15) == 0;
    }
    if (mfma) {
      hipLaunchKernelGGL(kdsvd_gram_mfma_kernel, dim3((unsigned)bmax, (unsigned)E), dim3(256), 0, st, tab);
      MDA_CHECK_LAUNCH();
    }
  }
  const dim3 grid((unsigned)bmax, (unsigned)E, (unsigned)ksplit);
  if (wmax * wmax <= 256)
    hipLaunchKernelGGL(kdsvd_gram_kernel<1>, grid, dim3(256), 0, st, tab);
  else if (wmax * wmax <= 1024)
    hipLaunchKernelGGL(kdsvd_gram_kernel<4>, grid, dim3(256), 0, st, tab);
  else
    hipLaunchKernelGGL(kdsvd_gram_kernel<16>, grid, dim3(256), 0, st, tab);
  MDA_CHECK_LAUNCH();
}

// table int64 [E][8] rows (x, d, dx, B, H, W, C, bf16), E <= 4.
MDA_API int mda_kdsvd_gram_apply(const int64_t* table, int64_t E, hipStream_t st) {
  if (E < 1 || E > KS_MAXS) return (int)hipErrorInvalidValue;
  KaTable tab{};
  int64_t smax = 0;
  for (int e = 0; e < E; ++e) {
    const int64_t* r = table + 8 * e;
    if (r[3] < 1 || r[4] < 1 || r[5] < 1 || r[5] > KS_MAXW || r[6] < 1) return (int)hipErrorInvalidValue;
    tab.e[e] = KaEntry{(const void*)r[0], (const float*)r[1], (void*)r[2], (int)r[3], (int)r[4],
                       (int)r[5], (int)r[6], (int)r[7]};
    smax = std::max(smax, r[3] * r[4]);
  }
  if (smax > 0x7fffffff) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kdsvd_gram_apply_kernel, dim3((unsigned)smax, (unsigned)E), dim3(256), 0, st, tab);
  MDA_CHECK_LAUNCH();
}
