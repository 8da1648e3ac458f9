// Relational distillation losses on the batch Gram (survey K11):
//   SP   `distillers/SP.py:12-24`   Ghat = rownorm(F F^T), sum (Ghat_t - Ghat_s)^2 / B^2
//   PKT  `distillers/PKT.py:8-35`   cosine kernel -> row-stochastic -> KL
//   RKD  `distillers/RKD.py:21-50`  pairwise distances and (i; j, k) angles, smooth-L1
// Every quantity these losses use is a function of the B x B Gram G = F F^T of
// the flattened features (row norms = sqrt(G_ii), distances^2 = G_ii + G_jj -
// 2 G_ij, difference-vector dot products = G_jk - G_ij - G_ik + G_ii), so the
// feature maps are read once by an MFMA Gram kernel and the B x D difference /
// normalised copies the reference materialises (B x B x D for the RKD angles)
// never exist.  The gradient goes back the same way: the loss kernels produce
// dL/dG, symmetrised into S = dG + dG^T, and dF = go * S F.
//
// Launches: gram_partial (MFMA 16x16x32 bf16, split over D) -> core (SP/PKT,
// one block) or rkd_angle (2B blocks) + rkd_finalize (one block) -> in the
// backward, gram_bwd.  Batch B <= 64 (one 64 x 64 Gram per tensor; larger
// batches take the PyTorch path).  All reductions are fixed-order.
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int RB = 64;        // Gram rows (max batch)
constexpr int GG = RB * RB;   // one Gram / partial
constexpr int LDG = RB + 1;   // LDS row stride

struct GramArgs {
  const bf16_t* a[2];   // [B, D_t] row-major bf16
  int64_t D[2];
  int64_t kc[2];        // columns per chunk (multiple of 32)
  int nchunk[2];
  int B;
  float* part;          // [nchunk[0] + nchunk[1]][64][64]
};

__device__ __forceinline__ bf16x8 row_frag(const bf16_t* A, int64_t D, int row, int64_t k, bool ok) {
  bf16x8 f;
  if (ok) {
    f = *(const bf16x8*)(A + (int64_t)row * D + k);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = (__bf16)0.f;
  }
  return f;
}

// Partial Gram of one D-chunk.  grid (max nchunk, 2), 4 waves; wave w owns
// rows 16w..16w+15 of the 64 x 64 tile and its four 16-column tiles.  MFMA
// 16x16x32: lane supplies 8 consecutive k of row (lane & 15) for both operands
// (the B operand of F F^T is F's rows again); lane holds G[4(lane>>4)+r][lane&15].
__global__ void __launch_bounds__(256) gram_partial_kernel(const GramArgs g) {
  const int t = blockIdx.y;
  if ((int)blockIdx.x >= g.nchunk[t]) return;
  const bf16_t* A = g.a[t];
  const int64_t D = g.D[t];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, kq = lane >> 4;
  const int64_t k0 = (int64_t)blockIdx.x * g.kc[t];
  const int64_t k1 = min(D, k0 + g.kc[t]);
  f32x4 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ra = 16 * w + r;
  for (int64_t k = k0; k < k1; k += 32) {
    const int64_t kk = k + 8 * kq;
    const bool kok = kk < k1;  // D % 8 == 0: an 8-column group is whole
    const bf16x8 fa = row_frag(A, D, ra, kk, kok && ra < g.B);
    bf16x8 fb[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) fb[c] = row_frag(A, D, 16 * c + r, kk, kok && 16 * c + r < g.B);
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[c], acc[c], 0, 0, 0);
  }
  float* out = g.part + (int64_t)(t == 0 ? blockIdx.x : g.nchunk[0] + blockIdx.x) * GG;
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) out[(16 * w + 4 * kq + i) * RB + 16 * c + r] = acc[c][i];
}

// Both Grams into LDS (fixed-order sum of the chunk partials, <= 16 chunks).
// float4 rows and every chunk's load issued together: a thread's loads are
// independent (one L2 round trip per 4 x 4 elements, not one per chunk).
__device__ void load_grams(const float* __restrict__ part, int nc0, int nc1, int B, float* Gs,
                           float* Gt) {
  const int B4 = (B + 3) / 4;
  for (int e = threadIdx.x; e < B * B4; e += blockDim.x) {
    const int i = e / B4, j0 = 4 * (e - i * B4);
    float4 s[16], u[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      s[c] = c < nc0 ? *(const float4*)(part + (int64_t)c * GG + i * RB + j0) : z;
      u[c] = c < nc1 ? *(const float4*)(part + (int64_t)(nc0 + c) * GG + i * RB + j0) : z;
    }
    float4 a = s[0], b = u[0];
#pragma unroll
    for (int c = 1; c < 16; ++c) {
      a.x += s[c].x; a.y += s[c].y; a.z += s[c].z; a.w += s[c].w;
      b.x += u[c].x; b.y += u[c].y; b.z += u[c].z; b.w += u[c].w;
    }
    const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (j0 + q < B) {
        Gs[i * LDG + j0 + q] = av[q];
        Gt[i * LDG + j0 + q] = bv[q];
      }
  }
}

__device__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// S = dG + dG^T (64-stride global)
__device__ void store_sym(const float* dG, int B, float* __restrict__ S) {
  for (int e = threadIdx.x; e < B * B; e += blockDim.x) {
    const int i = e / B, j = e - i * B;
    S[i * RB + j] = dG[i * LDG + j] + dG[j * LDG + i];
  }
}

__device__ __forceinline__ float sl1(float x) { return fabsf(x) < 1.f ? 0.5f * x * x : fabsf(x) - 0.5f; }
__device__ __forceinline__ float sl1_grad(float x) { return fabsf(x) < 1.f ? x : (x > 0.f ? 1.f : -1.f); }

constexpr int MODE_SP = 0, MODE_PKT = 1;

// SP / PKT: one block of 256 threads does the B x B algebra and its gradient.
__global__ void __launch_bounds__(256)
relation_core_kernel(const float* __restrict__ part, int nc0, int nc1, int B, int mode,
                     float* __restrict__ loss, float* __restrict__ S) {
  __shared__ float Gs[RB * LDG], Gt[RB * LDG], dG[RB * LDG];
  __shared__ float v0[RB], v1[RB], v2[RB], v3[RB], red[8];
  const int tid = threadIdx.x;
  load_grams(part, nc0, nc1, B, Gs, Gt);
  __syncthreads();
  const float invB2 = 1.f / ((float)B * (float)B);
  float acc = 0.f;
  if (mode == MODE_SP) {
    constexpr float EPS = 1e-12f;  // F.normalize
    if (tid < 2 * B) {  // row norms of both Grams
      const float* G = tid < B ? Gs : Gt;
      const int i = tid < B ? tid : tid - B;
      float s = 0.f;
      for (int j = 0; j < B; ++j) s += G[i * LDG + j] * G[i * LDG + j];
      (tid < B ? v0 : v1)[i] = fmaxf(sqrtf(s), EPS);
    }
    __syncthreads();
    for (int e = tid; e < B * B; e += blockDim.x) {
      const int i = e / B, j = e - i * B;
      const float d = Gt[i * LDG + j] / v1[i] - Gs[i * LDG + j] / v0[i];
      acc += d * d;
      dG[i * LDG + j] = -2.f * d * invB2;  // d loss / d Ghat_s
    }
    __syncthreads();
    if (tid < B) {
      float s = 0.f;
      for (int j = 0; j < B; ++j) s += dG[tid * LDG + j] * (Gs[tid * LDG + j] / v0[tid]);
      v2[tid] = s;
    }
    __syncthreads();
    for (int e = tid; e < B * B; e += blockDim.x) {
      const int i = e / B, j = e - i * B;
      // x / max(||x||, eps): the projection only where the norm is not clamped
      const float n = v0[i];
      const float gh = dG[i * LDG + j];
      dG[i * LDG + j] = n > EPS ? (gh - (Gs[i * LDG + j] / n) * v2[i]) / n : gh / n;
    }
  } else {  // PKT
    constexpr float EPS = 1e-7f;
    if (tid < 2 * B) {  // q_i = ||f_i|| + eps
      const float* G = tid < B ? Gs : Gt;
      const int i = tid < B ? tid : tid - B;
      (tid < B ? v0 : v1)[i] = sqrtf(fmaxf(G[i * LDG + i], 0.f)) + EPS;
    }
    __syncthreads();
    if (tid < 2 * B) {  // row sums of m = (C + 1) / 2
      const bool st = tid < B;
      const float* G = st ? Gs : Gt;
      const float* q = st ? v0 : v1;
      const int i = st ? tid : tid - B;
      float s = 0.f;
      for (int j = 0; j < B; ++j) s += 0.5f * (G[i * LDG + j] / (q[i] * q[j]) + 1.f);
      (st ? v2 : v3)[i] = s;
    }
    __syncthreads();
    for (int e = tid; e < B * B; e += blockDim.x) {
      const int i = e / B, j = e - i * B;
      const float ms = 0.5f * (Gs[i * LDG + j] / (v0[i] * v0[j]) + 1.f) / v2[i];
      const float ts = 0.5f * (Gt[i * LDG + j] / (v1[i] * v1[j]) + 1.f) / v3[i];
      acc += ts * logf((ts + EPS) / (ms + EPS));
      dG[i * LDG + j] = -ts / (ms + EPS) * invB2;  // d loss / d ms
    }
    __syncthreads();
    __shared__ float rd[RB];
    if (tid < B) {  // sum_k a_ik ms_ik
      float s = 0.f;
      for (int k = 0; k < B; ++k)
        s += dG[tid * LDG + k] * 0.5f * (Gs[tid * LDG + k] / (v0[tid] * v0[k]) + 1.f) / v2[tid];
      rd[tid] = s;
    }
    __syncthreads();
    for (int e = tid; e < B * B; e += blockDim.x) {  // dC = dm / 2, dm = (a - rowdot) / r
      const int i = e / B, j = e - i * B;
      dG[i * LDG + j] = 0.5f * (dG[i * LDG + j] - rd[i]) / v2[i];
    }
    __syncthreads();
    __shared__ float dq[RB];
    if (tid < B) {  // d q_i from C_ij = G_ij / (q_i q_j), as row and as column
      float s = 0.f;
      for (int j = 0; j < B; ++j) {
        s += dG[tid * LDG + j] * Gs[tid * LDG + j] / (v0[tid] * v0[j]);
        s += dG[j * LDG + tid] * Gs[j * LDG + tid] / (v0[j] * v0[tid]);
      }
      dq[tid] = -s / v0[tid];
    }
    __syncthreads();
    for (int e = tid; e < B * B; e += blockDim.x) {
      const int i = e / B, j = e - i * B;
      float v = dG[i * LDG + j] / (v0[i] * v0[j]);
      if (i == j) {
        const float n = v0[i] - EPS;  // sqrt(G_ii)
        if (n > 0.f) v += dq[i] / (2.f * n);
      }
      dG[i * LDG + j] = v;
    }
  }
  const float tot = block_sum(acc, red);
  __syncthreads();
  store_sym(dG, B, S);
  if (tid == 0) loss[0] = tot * invB2;
}

// ---------------------------------------------------------------- RKD
// r_ij = max(||x_j - x_i||, 1e-12) (F.normalize of the difference vectors)
__device__ void diff_norms(const float* G, int B, float* R) {
  for (int e = threadIdx.x; e < B * B; e += blockDim.x) {
    const int i = e / B, j = e - i * B;
    const float d2 = G[j * LDG + j] - 2.f * G[i * LDG + j] + G[i * LDG + i];
    R[i * LDG + j] = fmaxf(sqrtf(fmaxf(d2, 0.f)), 1e-12f);
  }
}

// cos angle (i; j, k) of one feature set
__device__ __forceinline__ float angle(const float* G, const float* R, int i, int j, int k) {
  const float n = (G[j * LDG + k] - G[i * LDG + j]) - (G[i * LDG + k] - G[i * LDG + i]);
  return n / (R[i * LDG + j] * R[i * LDG + k]);
}

// Blocks 0..B-1 (anchor i): per (i, j) P = sum_k dN_ijk, Rg = sum_k g_ijk a_ijk, and
// the block's angle-loss sum.  Blocks B..2B-1 (j): Q_jk = sum_i dN_ijk.
// g = smooth-L1'(a_s - a_t) * gscale; dN = g / (r_ij r_ik).  Terms with j == i
// or k == i are zero (zero difference vector: angle 0 in both sets, and their
// G-gradients cancel exactly), so they are skipped.
__global__ void __launch_bounds__(256)
rkd_angle_kernel(const float* __restrict__ part, int nc0, int nc1, int B, float gscale,
                 float* __restrict__ P, float* __restrict__ Rg, float* __restrict__ Q,
                 float* __restrict__ lossA) {
  __shared__ float Gs[RB * LDG], Gt[RB * LDG], Rs[RB * LDG], Rt[RB * LDG];
  __shared__ float s1[256], s2[256], s3[256], red[8];
  const int tid = threadIdx.x;
  load_grams(part, nc0, nc1, B, Gs, Gt);
  __syncthreads();
  diff_norms(Gs, B, Rs);
  diff_norms(Gt, B, Rt);
  __syncthreads();
  const int a = tid >> 2, seg = tid & 3;  // row a of the output, quarter seg of the loop
  const int per = (B + 3) / 4;
  float p = 0.f, rg = 0.f, l = 0.f;
  if ((int)blockIdx.x < B) {
    const int i = blockIdx.x, j = a;
    if (j < B && j != i) {
      for (int k = seg * per; k < min(B, seg * per + per); ++k) {
        if (k == i) continue;
        const float as = angle(Gs, Rs, i, j, k), at = angle(Gt, Rt, i, j, k);
        l += sl1(as - at);
        const float g = sl1_grad(as - at) * gscale;
        p += g / (Rs[i * LDG + j] * Rs[i * LDG + k]);
        rg += g * as;
      }
    }
  } else {
    const int j = blockIdx.x - B, k = a;
    if (k < B && k != j) {
      for (int i = seg * per; i < min(B, seg * per + per); ++i) {
        if (i == j || i == k) continue;
        const float as = angle(Gs, Rs, i, j, k), at = angle(Gt, Rt, i, j, k);
        p += sl1_grad(as - at) * gscale / (Rs[i * LDG + j] * Rs[i * LDG + k]);
      }
    }
  }
  s1[tid] = p;
  s2[tid] = rg;
  __syncthreads();
  if (seg == 0 && a < B) {
    const float ps = (s1[tid] + s1[tid + 1]) + (s1[tid + 2] + s1[tid + 3]);
    if ((int)blockIdx.x < B) {
      P[blockIdx.x * RB + a] = ps;
      Rg[blockIdx.x * RB + a] = (s2[tid] + s2[tid + 1]) + (s2[tid + 2] + s2[tid + 3]);
    } else {
      Q[(blockIdx.x - B) * RB + a] = ps;
    }
  }
  (void)s3;
  const float lt = block_sum(l, red);
  if ((int)blockIdx.x < B && tid == 0) lossA[blockIdx.x] = lt;
}

// Distances (with their positive-mean normalisation), the angle terms' G
// gradient from P / Rg / Q, the loss, and S.  One block.
__global__ void __launch_bounds__(256)
rkd_finalize_kernel(const float* __restrict__ part, int nc0, int nc1, int B, int squared,
                    float eps, float dist_w, float angle_w, const float* __restrict__ P,
                    const float* __restrict__ Rg, const float* __restrict__ Q,
                    const float* __restrict__ lossA, float* __restrict__ loss,
                    float* __restrict__ S) {
  __shared__ float Gs[RB * LDG], Gt[RB * LDG], dG[RB * LDG], Dd[RB * LDG], Td[RB * LDG];
  __shared__ float red[8], rowP[RB];
  const int tid = threadIdx.x;
  load_grams(part, nc0, nc1, B, Gs, Gt);
  __syncthreads();
  // pairwise distances of both sets (_pdist: clamp(min=eps), sqrt unless squared, zero diagonal)
  float cs = 0.f, ct = 0.f, ns = 0.f, nt = 0.f;
  for (int e = tid; e < B * B; e += blockDim.x) {
    const int i = e / B, j = e - i * B;
    float ds = 0.f, dt = 0.f;
    if (i != j) {
      ds = fmaxf(Gs[i * LDG + i] + Gs[j * LDG + j] - 2.f * Gs[i * LDG + j], eps);
      dt = fmaxf(Gt[i * LDG + i] + Gt[j * LDG + j] - 2.f * Gt[i * LDG + j], eps);
      if (!squared) { ds = sqrtf(ds); dt = sqrtf(dt); }
    }
    Dd[i * LDG + j] = ds;
    Td[i * LDG + j] = dt;
    if (ds > 0.f) { cs += ds; ns += 1.f; }
    if (dt > 0.f) { ct += dt; nt += 1.f; }
  }
  cs = block_sum(cs, red);
  ns = block_sum(ns, red);
  ct = block_sum(ct, red);
  nt = block_sum(nt, red);
  const float mu_s = cs / ns, mu_t = ct / nt;
  const float invB2 = 1.f / ((float)B * (float)B);
  // smooth-L1 of the normalised distances; d loss / d d_ij, and sum g d for the mean's gradient
  float ld = 0.f, gd = 0.f;
  for (int e = tid; e < B * B; e += blockDim.x) {
    const int i = e / B, j = e - i * B;
    const float x = Dd[i * LDG + j] / mu_s - Td[i * LDG + j] / mu_t;
    ld += sl1(x);
    const float g = sl1_grad(x) * invB2 * dist_w;
    dG[i * LDG + j] = g;  // temporarily d loss / d (d_ij / mu)
    gd += g * Dd[i * LDG + j];
  }
  ld = block_sum(ld, red);
  gd = block_sum(gd, red);
  __shared__ float Ps[RB * LDG];
  for (int e = tid; e < B * B; e += blockDim.x) {  // P into LDS: independent loads
    const int i = e / B, j = e - i * B;
    Ps[i * LDG + j] = P[i * RB + j];
  }
  __syncthreads();
  if (tid < B) {
    float s = 0.f;
    for (int j = 0; j < B; ++j) s += Ps[tid * LDG + j];
    rowP[tid] = s;
  }
  __syncthreads();
  // d loss / d d_kl = g_kl / mu - (sum g d) / mu^2 [d_kl > 0] / count
  for (int e = tid; e < B * B; e += blockDim.x) {
    const int i = e / B, j = e - i * B;
    const float d = Dd[i * LDG + j];
    float dd = dG[i * LDG + j] / mu_s - (d > 0.f ? gd / (mu_s * mu_s) / ns : 0.f);
    float dpre = 0.f;  // d loss / d (G_ii + G_jj - 2 G_ij)
    if (i != j) {
      const float pre = Gs[i * LDG + i] + Gs[j * LDG + j] - 2.f * Gs[i * LDG + j];
      if (pre > eps) dpre = squared ? dd : dd / (2.f * d);
    }
    dG[i * LDG + j] = dpre;  // applied below with the angle terms
  }
  __syncthreads();
  // assemble dG (row i owned by thread i: no write conflicts, fixed order)
  __shared__ float E[RB * LDG];
  for (int e = tid; e < B * B; e += blockDim.x) {
    const int i = e / B, j = e - i * B;
    // angle: +Q_ij (G_jk term, indices (j,k) -> (i,j)), -2 P_ij (G_ij and G_ik terms)
    float v = Q[i * RB + j] - 2.f * Ps[i * LDG + j];
    // distance: -2 dpre_ij on G_ij
    v -= 2.f * dG[i * LDG + j];
    // angle norms r_ij: dr = -2 Rg_ij / r_ij, dD2 = dr / (2 r): -2 dD2 on G_ij
    float dD2 = 0.f;
    if (i != j) {
      const float d2 = Gs[j * LDG + j] - 2.f * Gs[i * LDG + j] + Gs[i * LDG + i];
      const float r = sqrtf(fmaxf(d2, 0.f));
      if (r > 1e-12f) dD2 = (-2.f * Rg[i * RB + j] / r) / (2.f * r);
    }
    v -= 2.f * dD2;
    E[i * LDG + j] = dD2;
    Dd[i * LDG + j] = v;
  }
  __syncthreads();
  if (tid < B) {  // diagonal collects: sum_jk dN (rowP), dpre / dD2 of row and column pairs
    const int i = tid;
    float s = rowP[i];
    for (int j = 0; j < B; ++j) {
      if (j == i) continue;
      s += dG[i * LDG + j] + dG[j * LDG + i];  // distance: G_ii term of (i,j) and G_jj term of (j,i)
      s += E[i * LDG + j] + E[j * LDG + i];    // angle norms likewise
    }
    Dd[i * LDG + i] += s;
  }
  __syncthreads();
  store_sym(Dd, B, S);
  if (tid == 0) {
    float la = 0.f;
    for (int i = 0; i < B; ++i) la += lossA[i];
    loss[0] = dist_w * ld * invB2 + angle_w * la / ((float)B * (float)B * (float)B);
  }
}

// dF[i][d] = go * sum_j S[i][j] F[j][d]; S staged transposed in LDS so the
// inner loop reads one broadcast row per j.  grid ceil(D / 256); thread = column d.
__global__ void __launch_bounds__(256)
gram_bwd_kernel(const bf16_t* __restrict__ A, const float* __restrict__ S,
                const float* __restrict__ go, bf16_t* __restrict__ dA, int B, int64_t D) {
  __shared__ float St[RB * RB];
  for (int e = threadIdx.x; e < RB * RB; e += blockDim.x) {
    const int i = e / RB, j = e - i * RB;
    St[j * RB + i] = (i < B && j < B) ? S[i * RB + j] : 0.f;
  }
  __syncthreads();
  const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const float gs = go[0];
  // the thread's column: all rows' loads issued at once, parked in LDS
  __shared__ float Av[RB * 256];
  {
    float av[RB];
#pragma unroll
    for (int jj = 0; jj < RB; ++jj) av[jj] = (jj < B && d < D) ? bf2f(A[(int64_t)jj * D + d]) : 0.f;
#pragma unroll
    for (int jj = 0; jj < RB; ++jj) Av[jj * 256 + threadIdx.x] = av[jj];
  }
  if (d >= D) return;
  float acc[RB];
#pragma unroll
  for (int i = 0; i < RB; ++i) acc[i] = 0.f;
  for (int jj = 0; jj < B; ++jj) {
    const float a = Av[jj * 256 + threadIdx.x];
    const float4* srow = (const float4*)(St + jj * RB);
#pragma unroll
    for (int i4 = 0; i4 < RB / 4; ++i4) {
      const float4 sv = srow[i4];
      acc[4 * i4] += sv.x * a;
      acc[4 * i4 + 1] += sv.y * a;
      acc[4 * i4 + 2] += sv.z * a;
      acc[4 * i4 + 3] += sv.w * a;
    }
  }
#pragma unroll
  for (int i = 0; i < RB; ++i)
    if (i < B) dA[(int64_t)i * D + d] = f2bf(acc[i] * gs);
}

}  // namespace

// Chunk plan: ceil(D / kc) <= 16 chunks of a multiple of 32 columns.
MDA_API int mda_gram_plan(int64_t D, int64_t* kc, int64_t* nchunk) {
  int64_t c = (D + 15) / 16;
  c = (c + 31) / 32 * 32;
  if (c < 256) c = 256;
  *kc = c;
  *nchunk = (D + c - 1) / c;
  return 0;
}

// a_s [B, Ds], a_t [B, Dt] bf16 row-major (16-byte aligned rows: D % 8 == 0);
// part >= (nc_s + nc_t) * 4096 floats.
MDA_API int mda_gram_partial(const void* a_s, const void* a_t, float* part, int64_t B, int64_t Ds,
                             int64_t Dt, int64_t kc_s, int64_t kc_t, int64_t nc_s, int64_t nc_t,
                             hipStream_t st) {
  if (B < 1 || B > RB || Ds % 8 || Dt % 8 || kc_s % 32 || kc_t % 32 || nc_s < 1 || nc_t < 1)
    return (int)hipErrorInvalidValue;
  GramArgs g;
  g.a[0] = (const bf16_t*)a_s;
  g.a[1] = (const bf16_t*)a_t;
  g.D[0] = Ds; g.D[1] = Dt;
  g.kc[0] = kc_s; g.kc[1] = kc_t;
  g.nchunk[0] = (int)nc_s; g.nchunk[1] = (int)nc_t;
  g.B = (int)B;
  g.part = part;
  hipLaunchKernelGGL(gram_partial_kernel, dim3((unsigned)(nc_s > nc_t ? nc_s : nc_t), 2), dim3(256), 0,
                     st, g);
  MDA_CHECK_LAUNCH();
}

// mode 0 = SP, 1 = PKT: loss[0] and S [64][64] (rows/cols < B valid).
MDA_API int mda_relation_core(const float* part, int64_t nc_s, int64_t nc_t, int64_t B, int64_t mode,
                              float* loss, float* S, hipStream_t st) {
  if (B < 1 || B > RB || mode < 0 || mode > 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(relation_core_kernel, dim3(1), dim3(256), 0, st, part, (int)nc_s, (int)nc_t,
                     (int)B, (int)mode, loss, S);
  MDA_CHECK_LAUNCH();
}

// RKD: scratch P, Rg, Q >= 4096 floats each, lossA >= 64 floats.
MDA_API int mda_rkd_loss(const float* part, int64_t nc_s, int64_t nc_t, int64_t B, int64_t squared,
                         float eps, float dist_w, float angle_w, float* P, float* Rg, float* Q,
                         float* lossA, float* loss, float* S, hipStream_t st) {
  if (B < 2 || B > RB) return (int)hipErrorInvalidValue;
  const float gscale = angle_w / ((float)B * (float)B * (float)B);
  hipLaunchKernelGGL(rkd_angle_kernel, dim3((unsigned)(2 * B)), dim3(256), 0, st, part, (int)nc_s,
                     (int)nc_t, (int)B, gscale, P, Rg, Q, lossA);
  hipLaunchKernelGGL(rkd_finalize_kernel, dim3(1), dim3(256), 0, st, part, (int)nc_s, (int)nc_t,
                     (int)B, (int)squared, eps, dist_w, angle_w, P, Rg, Q, lossA, loss, S);
  MDA_CHECK_LAUNCH();
}

// dA [B, D] bf16 = go[0] * S A.
MDA_API int mda_gram_bwd(const void* a, const float* S, const float* go, void* da, int64_t B,
                         int64_t D, hipStream_t st) {
  if (B < 1 || B > RB || D < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(gram_bwd_kernel, dim3((unsigned)((D + 255) / 256)), dim3(256), 0, st,
                     (const bf16_t*)a, S, go, (bf16_t*)da, (int)B, D);
  MDA_CHECK_LAUNCH();
}
