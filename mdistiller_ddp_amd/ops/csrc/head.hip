// Classifier head and per-step metrics (survey K4/K5/K15).
//
//  * pool_fc  -- global average pool of the last NHWC feature map fused with
//    the Linear classifier: one block per image pools its HW x C tile into
//    LDS (fp32), writes the pooled feature and the J logits (fp32 weights,
//    fp32 accumulation, one thread per logit).  The backward is ONE launch:
//    blocks [0, J) produce dW/db rows (accumulated straight into the flat fp32
//    gradient views), blocks [J, J+N) produce d(feature map) = (dpooled +
//    dlogits @ W) / HW broadcast over the HW positions.  Replaces avg_pool2d +
//    hipBLASLt GEMM + bias/cast kernels (~8 launches per head per step at
//    batch 64) -- the reference runs F.avg_pool2d + nn.Linear
//    (models/cifar/resnet.py:123-124).
//  * meters_update -- top-1/top-5 hit counts (rank of the target logit), loss
//    sums, sample and step counts accumulated into one fp64 device buffer in a
//    single launch (reference: utils.accuracy + per-iteration all-reduces,
//    engine/utils.py:125-136, trainer.py:277-281).
#include "common.h"
#include "bnslot.h"

// optional BN-backward sums of the pooled map's producer (pool_fc_bwd_kernel)
struct HeadBn {
  const bf16_t* y; const bf16_t* res; const float* stats; BnRegion* reg; int act;
  const float* vres;  // res is a virtual residual (see BwdArgs::vres in bn.hip)
};

namespace {

// grid (N, ceil(J / 256)).  Phase 1: the block pools image n into LDS -- 8
// channels per thread with 16-byte loads, pixel groups reduced through LDS.
// Phase 2: one thread per logit, dot(pooled, W[j]) with 16-byte weight loads,
// 32 of them in flight per round.
template <typename T>
__global__ void __launch_bounds__(256)
pool_fc_fwd_kernel(const T* __restrict__ x, int HW, int C, const float* __restrict__ W,
                   const float* __restrict__ bias, T* __restrict__ pooled, T* __restrict__ logits,
                   int J, float inv_hw) {
  extern __shared__ float sh[];  // [C] pooled + [256 * 8] partials
  float* sp = sh;
  float* part = sh + C;
  const int n = blockIdx.x;
  const T* xn = x + (int64_t)n * HW * C;
  const int tid = threadIdx.x;
  constexpr int V = 16 / sizeof(T);  // elements per 16-byte load
  const int CG = C / V;
  if (C % V == 0 && CG <= 256) {
    const int P = 256 / CG;  // pixel groups
    const int cg = tid % CG, pg = tid / CG;
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
    if (pg < P) {
#pragma unroll 8
      for (int p = pg; p < HW; p += P) {
        const uint4 raw = *reinterpret_cast<const uint4*>(xn + (int64_t)p * C + cg * V);
        const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
        for (int i = 0; i < V; ++i) acc[i] += io<T>::ld(e, i);
      }
#pragma unroll
      for (int i = 0; i < V; ++i) part[pg * C + cg * V + i] = acc[i];
    }
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
      float s = 0.f;
      for (int q = 0; q < P; ++q) s += part[q * C + c];
      sp[c] = s * inv_hw;
    }
  } else {
    for (int c = tid; c < C; c += 256) {
      float s = 0.f;
      for (int p = 0; p < HW; ++p) s += io<T>::ld(xn, (int64_t)p * C + c);
      sp[c] = s * inv_hw;
    }
  }
  __syncthreads();
  // round to the storage dtype: the classifier consumes the stored feature,
  // as the unfused path (pool -> tensor -> Linear) does
  for (int c = tid; c < C; c += 256) {
    if (blockIdx.y == 0) io<T>::st(pooled, (int64_t)n * C + c, sp[c]);
    T r;
    io<T>::st(&r, 0, sp[c]);
    sp[c] = io<T>::ld(&r, 0);
  }
  __syncthreads();
  const int j = blockIdx.y * 256 + tid;
  if (j < J) {
    // thread per logit; 32 weight float4s in flight per round (a C = 256 row is
    // two L2 round trips), four independent accumulators
    const float* wj = W + (int64_t)j * C;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    int c = 0;
    if ((C & 3) == 0) {
      for (; c + 128 <= C; c += 128) {
        float4 w4[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) w4[u] = *reinterpret_cast<const float4*>(wj + c + 4 * u);
#pragma unroll
        for (int u = 0; u < 32; ++u) {
          const float4 s4 = *reinterpret_cast<const float4*>(sp + c + 4 * u);
          a[u & 3] += (s4.x * w4[u].x + s4.y * w4[u].y) + (s4.z * w4[u].z + s4.w * w4[u].w);
        }
      }
      for (; c < C; c += 4) {
        const float4 w4 = *reinterpret_cast<const float4*>(wj + c);
        a[0] += (sp[c] * w4.x + sp[c + 1] * w4.y) + (sp[c + 2] * w4.z + sp[c + 3] * w4.w);
      }
    }
    for (; c < C; ++c) a[0] += sp[c] * wj[c];
    io<T>::st(logits, (int64_t)n * J + j, ((a[0] + a[1]) + (a[2] + a[3])) + (bias ? bias[j] : 0.f));
  }
}

template <typename T>
__global__ void __launch_bounds__(256)
pool_fc_bwd_kernel(const T* __restrict__ dl, const T* __restrict__ dpooled,
                   const T* __restrict__ pooled, const float* __restrict__ W,
                   float* __restrict__ dW, float* __restrict__ db, T* __restrict__ dx, int N,
                   int HW, int C, int J, float inv_hw, int accum, HeadBn bn, int ksplit) {
  extern __shared__ float sh[];
  if ((int)blockIdx.x < J) {
    // ---- dW[j, :] = sum_n dl[n, j] * pooled[n, :];  db[j] = sum_n dl[n, j]
    const int j = blockIdx.x;
    for (int n = threadIdx.x; n < N; n += blockDim.x) sh[n] = io<T>::ld(dl, (int64_t)n * J + j);
    __syncthreads();
    if (dW != nullptr) {
      for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        int n = 0;
        for (; n + 32 <= N; n += 32) {  // 32 loads in flight per round
          float v[32];
#pragma unroll
          for (int u = 0; u < 32; ++u) v[u] = io<T>::ld(pooled, (int64_t)(n + u) * C + c);
#pragma unroll
          for (int u = 0; u < 32; ++u) a[u & 7] += sh[n + u] * v[u];
        }
        for (; n < N; ++n) a[0] += sh[n] * io<T>::ld(pooled, (int64_t)n * C + c);
        const float acc = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
        float* o = dW + (int64_t)j * C + c;
        *o = accum ? *o + acc : acc;
      }
    }
    if (db != nullptr && threadIdx.x < 64) {
      float acc = 0.f;
      for (int n = threadIdx.x; n < N; n += 64) acc += sh[n];
      acc = wave_sum(acc);
      if (threadIdx.x == 0) db[j] = accum ? db[j] + acc : acc;
    }
    return;
  }
  // ---- dx[n, p, :] = (dpooled[n, :] + dl[n, :] @ W) / HW   for every p;
  // ksplit blocks per image, each owning HW / ksplit pixels (the dx vector is
  // recomputed per block: W is L2-resident and the pixel loop is the cost)
  const int n = (blockIdx.x - J) / ksplit;
  const int part = (blockIdx.x - J) - n * ksplit;
  const int hw_b = HW / ksplit, p_lo = part * hw_b;
  float* sdl = sh;                                   // [J]
  float* sv = sh + (N > J ? N : J);                  // [C] the stored (rounded) dx value
  float* sred = sv + C;                              // [2][P][C] BN partials
  for (int j = threadIdx.x; j < J; j += blockDim.x) sdl[j] = io<T>::ld(dl, (int64_t)n * J + j);
  __syncthreads();
  T* dxn = dx + (int64_t)n * HW * C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int j = 0;
    for (; j + 32 <= J; j += 32) {  // 32 weight loads in flight per round
      float w[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) w[u] = W[(int64_t)(j + u) * C + c];
#pragma unroll
      for (int u = 0; u < 32; ++u) a[u & 7] += sdl[j + u] * w[u];
    }
    for (; j < J; ++j) a[0] += sdl[j] * W[(int64_t)j * C + c];
    const float acc = (dpooled ? io<T>::ld(dpooled, (int64_t)n * C + c) : 0.f) +
                      (((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7])));
    T r;
    io<T>::st(&r, 0, acc * inv_hw);
    sv[c] = io<T>::ld(&r, 0);
  }
  __syncthreads();
  const int CG = C / 8;
  if (sizeof(T) == 2 && (C & 7) == 0 && CG <= 256) {
    // 8 channels x a pixel group per thread: 16-byte dx stores and BN-input
    // loads (one scalar channel per thread walking all pixels took 39 us for
    // the 8x8x256 head of ResNet8x4)
    const int P = 256 / CG;
    const int cg = threadIdx.x % CG, pg = threadIdx.x / CG;
    const int c0 = cg * 8;
    float s1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, s2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (pg < P) {
      float d[8];
      uint32_t dw[4];
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = sv[c0 + e];
#pragma unroll
      for (int w = 0; w < 4; ++w) dw[w] = pack_bf16x2(d[2 * w], d[2 * w + 1]);
      const uint4 dv = make_uint4(dw[0], dw[1], dw[2], dw[3]);
      float mu[8], rs[8], sc[8], sf[8], vsc[8], vsh[8];
      if (bn.reg != nullptr) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          mu[e] = bn.stats[c0 + e]; rs[e] = bn.stats[C + c0 + e];
          sc[e] = bn.stats[2 * C + c0 + e]; sf[e] = bn.stats[3 * C + c0 + e];
          vsc[e] = bn.vres ? bn.vres[2 * C + c0 + e] : 1.f;
          vsh[e] = bn.vres ? bn.vres[3 * C + c0 + e] : 0.f;
        }
      }
      const bf16_t* yn = bn.y ? bn.y + (int64_t)n * HW * C : nullptr;
      const bf16_t* rn = bn.res ? bn.res + (int64_t)n * HW * C : nullptr;
      for (int p0 = p_lo + pg; p0 < p_lo + hw_b; p0 += 4 * P) {
        // up to 4 pixels' BN-input loads in flight before any math
        uint4 yv4[4], rv4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int p = p0 + k * P;
          const bool ok = bn.reg != nullptr && p < p_lo + hw_b;
          const int64_t o = (int64_t)(ok ? p : p_lo) * C + c0;
          yv4[k] = ok ? *(const uint4*)(yn + o) : make_uint4(0u, 0u, 0u, 0u);
          rv4[k] = (ok && rn) ? *(const uint4*)(rn + o) : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
        const int p = p0 + k * P;
        if (p >= p_lo + hw_b) break;
        const int64_t o = (int64_t)p * C + c0;
        *(uint4*)(dxn + o) = dv;
        if (bn.reg != nullptr) {
          const uint4 yv = yv4[k];
          const uint4 rv = rv4[k];
          const uint32_t yw[4] = {yv.x, yv.y, yv.z, yv.w}, rw[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const uint32_t u = yw[e >> 1], q = rw[e >> 1];
            const float yf = (e & 1) ? __uint_as_float(u & 0xffff0000u) : __uint_as_float(u << 16);
            float z = yf * sc[e] + sf[e];
            if (rn) z += ((e & 1) ? __uint_as_float(q & 0xffff0000u) : __uint_as_float(q << 16)) * vsc[e] + vsh[e];
            const float g = bn.act == 1 ? (z > 0.f ? d[e] : 0.f)
                            : bn.act == 2 ? ((z > 0.f && z < 6.f) ? d[e] : 0.f) : d[e];
            s1[e] += g;
            s2[e] += g * ((yf - mu[e]) * rs[e]);
          }
        }
        }
      }
    }
    if (bn.reg == nullptr) return;
    const int PP = 256 / CG;
    if (pg < PP) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sred[(0 * PP + pg) * C + c0 + e] = s1[e];
        sred[(1 * PP + pg) * C + c0 + e] = s2[e];
      }
    }
    __syncthreads();
    const int shard = (blockIdx.x - J) % slot_shards(C);
    for (int t = threadIdx.x; t < 2 * C; t += blockDim.x) {
      const int q = t / C, c = t - q * C;
      float a = 0.f;
      for (int r = 0; r < PP; ++r) a += sred[(q * PP + r) * C + c];
      acc_add(region_acc(bn.reg, C, shard, q) + c, (double)a);
    }
    return;
  }
  for (int c = threadIdx.x; c < C; c += blockDim.x) {  // (ksplit == 1 here)
    const float v = sv[c];
    for (int p = 0; p < HW; ++p) io<T>::st(dxn, (int64_t)p * C + c, v);
    if (bn.reg != nullptr) {
      // dx is the whole output gradient of the training BN that produced the
      // pooled map: its sum dz / sum dz*xhat over this sample's pixels
      const float d = v;  // the stored (rounded) value
      const float mu = bn.stats[c], rs = bn.stats[C + c], sc = bn.stats[2 * C + c],
                  shf = bn.stats[3 * C + c];
      float s1 = 0.f, s2 = 0.f;
      const bf16_t* yn = bn.y + (int64_t)n * HW * C;
      const bf16_t* rn = bn.res ? bn.res + (int64_t)n * HW * C : nullptr;
      for (int p = 0; p < HW; ++p) {
        const float yv = bf2f(yn[(int64_t)p * C + c]);
        float z = yv * sc + shf;
        if (rn) z += bn.vres ? bf2f(rn[(int64_t)p * C + c]) * bn.vres[2 * C + c] + bn.vres[3 * C + c]
                             : bf2f(rn[(int64_t)p * C + c]);
        const float g = bn.act == 1 ? (z > 0.f ? d : 0.f)
                        : bn.act == 2 ? ((z > 0.f && z < 6.f) ? d : 0.f) : d;
        s1 += g;
        s2 += g * ((yv - mu) * rs);
      }
      const int shard = n % slot_shards(C);
      acc_add(region_acc(bn.reg, C, shard, 0) + c, (double)s1);
      acc_add(region_acc(bn.reg, C, shard, 1) + c, (double)s2);
    }
  }
}

// One wave per row (lanes stride over the C classes; ImageNet's 1000-class
// rows took 100 us as one thread per row in a single block).  Hit counts are
// integers, so the per-block fp64 atomic adds are exact and order-free
// (deterministic); block 0 also adds the loss values and the sample/step
// counts.
template <typename T>
__global__ void __launch_bounds__(256)
meters_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target, int B, int C,
              const float* __restrict__ l0, const float* __restrict__ l1,
              const float* __restrict__ l2, const float* __restrict__ l3, int nloss,
              double* __restrict__ buf) {
  __shared__ int s_hits[2];
  if (threadIdx.x < 2) s_hits[threadIdx.x] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = blockIdx.x * 4 + wid;
  if (r < B) {
    const int64_t base = (int64_t)r * C;
    const int tg = (int)target[r];
    const float t = io<T>::ld(preds, base + tg);
    // rank of the target = classes ordered before it by topk: strictly larger
    // logits, plus EQUAL logits at a lower class index (ties are frequent with
    // bf16 logits and must not count as hits)
    int cnt = 0;
    for (int c = lane; c < C; c += 64) {
      const float v = io<T>::ld(preds, base + c);
      cnt += (v > t) || (v == t && c < tg);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if (lane == 0) {
      if (cnt < 1) atomicAdd(&s_hits[0], 1);
      if (cnt < 5) atomicAdd(&s_hits[1], 1);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_hits[0]) atomicAdd(&buf[nloss + 1], (double)s_hits[0]);
    if (s_hits[1]) atomicAdd(&buf[nloss + 2], (double)s_hits[1]);
    if (blockIdx.x == 0) {
      const float* ls[4] = {l0, l1, l2, l3};
      double total = 0.0;
      for (int i = 0; i < nloss; ++i) {
        const double v = (double)*ls[i];
        buf[1 + i] += v;
        total += v;
      }
      buf[0] += total;
      buf[nloss + 3] += (double)B;
      buf[nloss + 4] += 1.0;
    }
  }
}

// ---- tiled head backward for large heads (ImageNet: J = 1000, C = 512..2048)
// Two small GEMMs, one launch: blocks [0, nW) compute dW/db tiles
// (64 j x 64 c, reduction over the batch), blocks [nW, nW + nX) compute
// d(feature) tiles (16 n x 64 c, reduction over the J logits) and broadcast
// them over the HW positions.  Reduction operands are staged through LDS in
// chunks of 32; each thread owns a 4x4 (dW) or 1x4 (dx) register tile.
constexpr int HB_TJ = 64, HB_TC = 64, HB_TN = 16, HB_R = 32;

template <typename T>
__global__ void __launch_bounds__(256)
pool_fc_bwd_tiled_kernel(const T* __restrict__ dl, const T* __restrict__ dpooled,
                         const T* __restrict__ pooled, const float* __restrict__ W,
                         float* __restrict__ dW, float* __restrict__ db, T* __restrict__ dx, int N,
                         int HW, int C, int J, float inv_hw, int accum, int nW) {
  __shared__ float sa[HB_R][HB_TJ + 1];
  __shared__ float sb[HB_R][HB_TC + 4];
  const int tid = threadIdx.x;
  const int ctiles = (C + HB_TC - 1) / HB_TC;
  if ((int)blockIdx.x < nW) {
    if (dW == nullptr && db == nullptr) return;
    const int jt = blockIdx.x / ctiles, ct = blockIdx.x - jt * ctiles;
    const int j0 = jt * HB_TJ, c0 = ct * HB_TC;
    const int tj = (tid >> 4) * 4, tc = (tid & 15) * 4;
    float acc[4][4] = {};
    float dbacc = 0.f;
    for (int n0 = 0; n0 < N; n0 += HB_R) {
      for (int i = tid; i < HB_R * HB_TJ; i += 256) {
        const int r = i / HB_TJ, jj = i - r * HB_TJ;
        const int n = n0 + r, j = j0 + jj;
        sa[r][jj] = (n < N && j < J) ? io<T>::ld(dl, (int64_t)n * J + j) : 0.f;
      }
      for (int i = tid; i < HB_R * HB_TC; i += 256) {
        const int r = i / HB_TC, cc = i - r * HB_TC;
        const int n = n0 + r, c = c0 + cc;
        sb[r][cc] = (n < N && c < C) ? io<T>::ld(pooled, (int64_t)n * C + c) : 0.f;
      }
      __syncthreads();
#pragma unroll 4
      for (int r = 0; r < HB_R; ++r) {
        float a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) { a[u] = sa[r][tj + u]; b[u] = sb[r][tc + u]; }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int v = 0; v < 4; ++v) acc[u][v] += a[u] * b[v];
      }
      if (db != nullptr && ct == 0 && tid < HB_TJ)
        for (int r = 0; r < HB_R; ++r) dbacc += sa[r][tid];
      __syncthreads();
    }
    if (dW != nullptr) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int j = j0 + tj + u;
        if (j >= J) continue;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int c = c0 + tc + v;
          if (c >= C) continue;
          float* o = dW + (int64_t)j * C + c;
          *o = accum ? *o + acc[u][v] : acc[u][v];
        }
      }
    }
    if (db != nullptr && ct == 0 && tid < HB_TJ && j0 + tid < J)
      db[j0 + tid] = accum ? db[j0 + tid] + dbacc : dbacc;
    return;
  }
  // ---- dx tile: rows n0..n0+15, channels c0..c0+63
  const int b = blockIdx.x - nW;
  const int nt = b / ctiles, ct = b - nt * ctiles;
  const int n0 = nt * HB_TN, c0 = ct * HB_TC;
  const int tn = tid >> 4, tc = (tid & 15) * 4;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int r0 = 0; r0 < J; r0 += HB_R) {
    for (int i = tid; i < HB_R * HB_TN; i += 256) {
      const int r = i / HB_TN, nn = i - r * HB_TN;
      const int j = r0 + r, n = n0 + nn;
      sa[r][nn] = (n < N && j < J) ? io<T>::ld(dl, (int64_t)n * J + j) : 0.f;
    }
    for (int i = tid; i < HB_R * HB_TC; i += 256) {
      const int r = i / HB_TC, cc = i - r * HB_TC;
      const int j = r0 + r, c = c0 + cc;
      sb[r][cc] = (j < J && c < C) ? W[(int64_t)j * C + c] : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int r = 0; r < HB_R; ++r) {
      const float a = sa[r][tn];
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[v] += a * sb[r][tc + v];
    }
    __syncthreads();
  }
  const int n = n0 + tn;
  if (n >= N) return;
  T* dxn = dx + (int64_t)n * HW * C;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int c = c0 + tc + v;
    if (c >= C) continue;
    const float val = ((dpooled ? io<T>::ld(dpooled, (int64_t)n * C + c) : 0.f) + acc[v]) * inv_hw;
    for (int p = 0; p < HW; ++p) io<T>::st(dxn, (int64_t)p * C + c, val);
  }
}

}  // namespace

// x [N, HW, C] (NHWC) fp32|bf16; W [J, C] fp32; bias [J] fp32 or null;
// pooled [N, C], logits [N, J] in x's dtype.
MDA_API int mda_pool_fc_fwd(int64_t dt, const void* x, const float* W, const float* bias,
                            void* pooled, void* logits, int64_t N, int64_t HW, int64_t C,
                            int64_t J, hipStream_t st) {
  if (N <= 0 || C <= 0 || C > 8192 || J <= 0) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)(C + 256 * 8) * sizeof(float);
  const dim3 grid((unsigned)N, (unsigned)((J + 255) / 256));
  if (dt == DT_F32)
    hipLaunchKernelGGL(pool_fc_fwd_kernel<float>, grid, dim3(256), lds, st, (const float*)x,
                       (int)HW, (int)C, W, bias, (float*)pooled, (float*)logits, (int)J, 1.f / HW);
  else
    hipLaunchKernelGGL(pool_fc_fwd_kernel<bf16_t>, grid, dim3(256), lds, st, (const bf16_t*)x,
                       (int)HW, (int)C, W, bias, (bf16_t*)pooled, (bf16_t*)logits, (int)J, 1.f / HW);
  MDA_CHECK_LAUNCH();
}

// dl [N, J]; dpooled [N, C] or null; pooled [N, C]; W [J, C] fp32; dW [J, C] fp32 or
// null; db [J] fp32 or null; dx [N, HW, C].  accum: dW/db += instead of =.
MDA_API int mda_pool_fc_bwd_bn(int64_t dt, const void* dl, const void* dpooled, const void* pooled,
                               const float* W, float* dW, float* db, void* dx, int64_t N,
                               int64_t HW, int64_t C, int64_t J, int64_t accum, const void* bn_y,
                               const void* bn_res, const float* bn_stats, int64_t bn_act,
                               void* bn_region, const float* bn_vres, hipStream_t st);

MDA_API int mda_pool_fc_bwd(int64_t dt, const void* dl, const void* dpooled, const void* pooled,
                            const float* W, float* dW, float* db, void* dx, int64_t N, int64_t HW,
                            int64_t C, int64_t J, int64_t accum, hipStream_t st) {
  return mda_pool_fc_bwd_bn(dt, dl, dpooled, pooled, W, dW, db, dx, N, HW, C, J, accum, nullptr,
                            nullptr, nullptr, 0, nullptr, nullptr, st);
}

// mda_pool_fc_bwd that also adds the BN backward sums of the layer whose
// output was pooled (bn_*: its input, residual, [4][C] stats, activation and a
// fresh region; bf16 only, small heads only -- the caller checks
// mda_pool_fc_bwd_bn_ok).
MDA_API int mda_pool_fc_bwd_bn(int64_t dt, const void* dl, const void* dpooled, const void* pooled,
                               const float* W, float* dW, float* db, void* dx, int64_t N,
                               int64_t HW, int64_t C, int64_t J, int64_t accum, const void* bn_y,
                               const void* bn_res, const float* bn_stats, int64_t bn_act,
                               void* bn_region, const float* bn_vres, hipStream_t st) {
  if (N <= 0 || C <= 0 || J <= 0 || N > 16384 || J > 16384) return (int)hipErrorInvalidValue;
  HeadBn bn{(const bf16_t*)bn_y, (const bf16_t*)bn_res, bn_stats, (BnRegion*)bn_region, (int)bn_act,
            bn_res != nullptr ? bn_vres : nullptr};
  if (bn_region != nullptr && (dt == DT_F32 || (int64_t)J * C > (1 << 16) || C > SLOT_CMAX))
    return (int)hipErrorInvalidValue;
  if ((int64_t)J * C > (1 << 16)) {  // large head: tiled GEMM blocks
    const int ct = (int)((C + HB_TC - 1) / HB_TC);
    const int nW = (int)((J + HB_TJ - 1) / HB_TJ) * ct;
    const int nX = (int)((N + HB_TN - 1) / HB_TN) * ct;
    if (dt == DT_F32)
      hipLaunchKernelGGL(pool_fc_bwd_tiled_kernel<float>, dim3(nW + nX), dim3(256), 0, st,
                         (const float*)dl, (const float*)dpooled, (const float*)pooled, W, dW, db,
                         (float*)dx, (int)N, (int)HW, (int)C, (int)J, 1.f / HW, (int)accum, nW);
    else
      hipLaunchKernelGGL(pool_fc_bwd_tiled_kernel<bf16_t>, dim3(nW + nX), dim3(256), 0, st,
                         (const bf16_t*)dl, (const bf16_t*)dpooled, (const bf16_t*)pooled, W, dW,
                         db, (bf16_t*)dx, (int)N, (int)HW, (int)C, (int)J, 1.f / HW, (int)accum,
                         nW);
    MDA_CHECK_LAUNCH();
  }
  // [max(N, J)] dl column / row + [C] dx values + [2][256 / (C/8)][C] BN partials
  const int64_t pp = (C % 8 == 0 && C / 8 <= 256) ? 256 / (C / 8) : 0;
  const size_t lds = (size_t)((N > J ? N : J) + C + 2 * pp * C) * sizeof(float);
  if (lds > 64 * 1024) return (int)hipErrorInvalidValue;
  // images split over ksplit blocks (>= 16 pixels each) on the vector path
  static const int kmax = [] {
    const char* e = getenv("MDA_HEAD_KSPLIT");
    return e ? atoi(e) : 4;
  }();
  int ksplit = 1;
  if (dt != DT_F32 && pp > 0 && kmax > 1)
    for (int k = kmax; k > 1; k >>= 1)
      if (HW % k == 0 && HW / k >= 16) { ksplit = k; break; }
  const dim3 grid((unsigned)(J + N * ksplit));
  if (dt == DT_F32)
    hipLaunchKernelGGL(pool_fc_bwd_kernel<float>, grid, dim3(256), lds, st, (const float*)dl,
                       (const float*)dpooled, (const float*)pooled, W, dW, db, (float*)dx, (int)N,
                       (int)HW, (int)C, (int)J, 1.f / HW, (int)accum, bn, 1);
  else
    hipLaunchKernelGGL(pool_fc_bwd_kernel<bf16_t>, grid, dim3(256), lds, st, (const bf16_t*)dl,
                       (const bf16_t*)dpooled, (const bf16_t*)pooled, W, dW, db, (bf16_t*)dx,
                       (int)N, (int)HW, (int)C, (int)J, 1.f / HW, (int)accum, bn, ksplit);
  MDA_CHECK_LAUNCH();
}

// preds [B, C] fp32|bf16; target [B] int64; l0..l3 fp32 scalars (first nloss used);
// buf fp64 [1 + nloss + 4] = [total, per-loss..., top1, top5, samples, steps].
MDA_API int mda_meters_update(int64_t dt, const void* preds, const int64_t* target, int64_t B,
                              int64_t C, const float* l0, const float* l1, const float* l2,
                              const float* l3, int64_t nloss, double* buf, hipStream_t st) {
  if (nloss < 0 || nloss > 4 || B <= 0) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)((B + 3) / 4));
  if (dt == DT_F32)
    hipLaunchKernelGGL(meters_kernel<float>, grid, dim3(256), 0, st, (const float*)preds, target,
                       (int)B, (int)C, l0, l1, l2, l3, (int)nloss, buf);
  else
    hipLaunchKernelGGL(meters_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)preds,
                       target, (int)B, (int)C, l0, l1, l2, l3, (int)nloss, buf);
  MDA_CHECK_LAUNCH();
}
