// Depthwise KxK convolution on NHWC bf16 activations (survey K3: MobileNetV1
// `mobilenetv1.py:19-29`, MobileNetV2 `cifar/mobilenetv2.py:42-50`,
// ShuffleNetV1/V2 depthwise 3x3).  There is no reduction over input channels,
// so MFMA does not apply: this is a memory-bound stencil on the vector ALUs.
//
//  * forward   -- one thread owns V consecutive channels (V = 8/4/2/1 bf16, one
//    16/8/4/2-byte load) of OWT = 4 consecutive output columns; per filter row
//    the (OWT-1)*stride + K input columns it needs are loaded once into
//    registers and reused by all four outputs.  Fused epilogue (inference /
//    folded-BN teacher path): y = act(acc*scale + bias (+ res)), optional
//    pre-activation; training path: raw y (BN runs in bn.hip).
//  * dgrad     -- dx[h, w] = sum over taps whose (h + p - kh, w + p - kw) lands
//    on the stride grid of dy; same V x OWT thread tile.
//  * wgrad     -- per-block partial sums of dy * x for every (tap, channel),
//    reduced over pixel lanes through LDS by all threads (three taps per
//    round, (output, slice) pairs), then a
//    channel-parallel finalize kernel combines the blocks in fixed order and
//    writes/accumulates the fp32 [C, K, K] gradient (deterministic).
// Weights arrive as fp32 packed tap-major [KH*KW, C] (coalesced per-channel
// loads); folded teacher weights are packed once on the host.  3x3 kernels,
// stride 1 or 2 (every depthwise layer of the model zoo); others use PyTorch.
#include <cstdlib>

#include "common.h"
#include "bnslot.h"

namespace {

constexpr int OWT = 4;       // output (or input, for dgrad) columns per thread
constexpr int KS = 3;        // kernel size (every depthwise conv of the zoo is 3x3)

template <int V> struct vec;
template <> struct vec<8> { typedef uint4 t; };
template <> struct vec<4> { typedef uint2 t; };
template <> struct vec<2> { typedef uint32_t t; };
template <> struct vec<1> { typedef uint16_t t; };

template <int V>
__device__ __forceinline__ void ld_vec(const bf16_t* p, float (&o)[V]) {
  const typename vec<V>::t r = *reinterpret_cast<const typename vec<V>::t*>(p);
  const bf16_t* e = reinterpret_cast<const bf16_t*>(&r);
#pragma unroll
  for (int i = 0; i < V; ++i) o[i] = bf2f(e[i]);
}

template <int V>
__device__ __forceinline__ void st_vec(bf16_t* p, const float (&v)[V]) {
  typename vec<V>::t r;
  bf16_t* e = reinterpret_cast<bf16_t*>(&r);
#pragma unroll
  for (int i = 0; i < V; ++i) e[i] = f2bf(v[i]);
  *reinterpret_cast<typename vec<V>::t*>(p) = r;
}

// Raw (packed bf16) vector load with zero fill, and its unpack: the kernels
// below issue every load of a work item before any math (the layers of the
// CIFAR students are a few dozen blocks: latency, not bandwidth, bound).
template <int V>
__device__ __forceinline__ typename vec<V>::t ld_raw(const bf16_t* p, bool ok) {
  typename vec<V>::t r{};
  if (ok) r = *reinterpret_cast<const typename vec<V>::t*>(p);
  return r;
}

template <int V>
__device__ __forceinline__ void unpack(const typename vec<V>::t& r, float (&o)[V]) {
  const bf16_t* e = reinterpret_cast<const bf16_t*>(&r);
#pragma unroll
  for (int i = 0; i < V; ++i) o[i] = bf2f(e[i]);
}

// V consecutive fp32 weights of one tap (16-byte loads when V >= 4).
template <int V>
__device__ __forceinline__ void ld_w(const float* p, float (&o)[V]) {
  if constexpr (V >= 4) {
#pragma unroll
    for (int i = 0; i < V; i += 4) {
      const float4 t = *reinterpret_cast<const float4*>(p + i);
      o[i] = t.x; o[i + 1] = t.y; o[i + 2] = t.z; o[i + 3] = t.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) o[i] = p[i];
  }
}

__device__ __forceinline__ float act_fn(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) return fminf(fmaxf(v, 0.f), 6.f);
  return v;
}

struct DwParams {
  const bf16_t* x;      // [N, H, W, C]   (dgrad: dy [N, Ho, Wo, C])
  const float* w;       // [KH*KW, C] fp32
  const float* scale;   // [C] or null
  const float* bias;    // [C] or null
  const bf16_t* res;    // [N, Ho, Wo, C] or null
  bf16_t* y;            // output
  bf16_t* preact;       // or null
  int N, H, W, C, Ho, Wo, KH, KW, stride, pad, act;
  // training BN after the conv (round 3): the block's sum y / sum y^2 of the
  // stored bf16 output go into this region (csrc/bnslot.h) instead of a
  // separate statistics pass; needs a grid stride that is a multiple of C / V
  // (every thread keeps one channel group), see launch_fwd
  BnRegion* stats_slot;
};

// Block channel sums of the per-thread (channel group) partials st1/st2 into
// a region shard; deterministic: thread t always held channel group
// (blockIdx.x * 256 + t) % CG (grid stride a multiple of CG, launch_dw), and
// channel c sums the threads of its group in order.
template <int V>
__device__ __forceinline__ void dw_block_sums(BnRegion* slot, int C, const float (&st1)[V],
                                              const float (&st2)[V]) {
  const int CG = C / V;
  __shared__ float red[256][2 * V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    red[threadIdx.x][v] = st1[v];
    red[threadIdx.x][V + v] = st2[v];
  }
  __syncthreads();
  const int base = (int)(((int64_t)blockIdx.x * blockDim.x) % CG);
  const int shard = (int)blockIdx.x % slot_shards(C);
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int g = c / V, e = c - g * V;
    float a = 0.f, b = 0.f;
    for (int t = ((g - base) % CG + CG) % CG; t < (int)blockDim.x; t += CG) {
      a += red[t][e];
      b += red[t][V + e];
    }
    acc_add(region_acc(slot, C, shard, 0) + c, (double)a);
    acc_add(region_acc(slot, C, shard, 1) + c, (double)b);
  }
}

template <int V, int S>
__global__ void __launch_bounds__(256)
dw_fwd_kernel(const DwParams p) {
  constexpr int NCOLS = (OWT - 1) * S + KS;
  const int CG = p.C / V;
  const int WT = (p.Wo + OWT - 1) / OWT;
  const int64_t total = (int64_t)p.N * p.Ho * WT * CG;
  float st1[V], st2[V];
#pragma unroll
  for (int v = 0; v < V; ++v) st1[v] = st2[v] = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int cg = (int)(i % CG);
    int64_t r = i / CG;
    const int wt = (int)(r % WT);
    r /= WT;
    const int ho = (int)(r % p.Ho);
    const int n = (int)(r / p.Ho);
    const int c0 = cg * V;
    const int wo0 = wt * OWT;
    const int iw0 = wo0 * S - p.pad;
    float wv[KS * KS][V];
    (void)c0;
#pragma unroll
    for (int t = 0; t < KS * KS; ++t) ld_w<V>(p.w + t * p.C + c0, wv[t]);
    typename vec<V>::t raw[KS][NCOLS];
#pragma unroll
    for (int kh = 0; kh < KS; ++kh) {
      const int ih = ho * S - p.pad + kh;
      const bool okr = (unsigned)ih < (unsigned)p.H;
      const bf16_t* row = p.x + (((int64_t)n * p.H + (okr ? ih : 0)) * p.W) * p.C + c0;
#pragma unroll
      for (int q = 0; q < NCOLS; ++q) {
        const int iw = iw0 + q;
        raw[kh][q] = ld_raw<V>(row + (int64_t)iw * p.C, okr && (unsigned)iw < (unsigned)p.W);
      }
    }
    float acc[OWT][V];
#pragma unroll
    for (int j = 0; j < OWT; ++j)
#pragma unroll
      for (int v = 0; v < V; ++v) acc[j][v] = 0.f;
#pragma unroll
    for (int kh = 0; kh < KS; ++kh) {
      float xin[NCOLS][V];
#pragma unroll
      for (int q = 0; q < NCOLS; ++q) unpack<V>(raw[kh][q], xin[q]);
#pragma unroll
      for (int kw = 0; kw < KS; ++kw)
#pragma unroll
        for (int j = 0; j < OWT; ++j)
#pragma unroll
          for (int v = 0; v < V; ++v) acc[j][v] += xin[j * S + kw][v] * wv[kh * KS + kw][v];
    }
    float sc[V], bi[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      sc[v] = p.scale ? p.scale[c0 + v] : 1.f;
      bi[v] = p.bias ? p.bias[c0 + v] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < OWT; ++j) {
      const int wo = wo0 + j;
      if (wo >= p.Wo) break;
      const int64_t o = (((int64_t)n * p.Ho + ho) * p.Wo + wo) * p.C + c0;
      float t[V];
#pragma unroll
      for (int v = 0; v < V; ++v) t[v] = acc[j][v] * sc[v] + bi[v];
      if (p.res) {
        float rr[V];
        ld_vec<V>(p.res + o, rr);
#pragma unroll
        for (int v = 0; v < V; ++v) t[v] += rr[v];
      }
      if (p.preact) st_vec<V>(p.preact + o, t);
#pragma unroll
      for (int v = 0; v < V; ++v) t[v] = act_fn(t[v], p.act);
      st_vec<V>(p.y + o, t);
      if (p.stats_slot) {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const float q = bf2f(f2bf(t[v]));  // the stored value
          st1[v] += q;
          st2[v] += q * q;
        }
      }
    }
  }
  if (p.stats_slot == nullptr) return;
  dw_block_sums<V>(p.stats_slot, p.C, st1, st2);
}

// dx[n, h, w, c] = sum_{kh, kw} dy[n, (h + p - kh)/s, (w + p - kw)/s, c] * w[kh, kw, c]
// over taps landing on the stride grid.  p.x = dy, p.y = dx; H/W = input dims.
// S = 1: dx[h, w0 + j] = sum dy[h + p - kh, w0 + j + p - kw] * w[kh, kw], the
// OWT + 2 dy columns of each of the three rows loaded once, all up front.
template <int V, int S>
__global__ void __launch_bounds__(256)
dw_dgrad_kernel(const DwParams p) {
  const int CG = p.C / V;
  const int WT = (p.W + OWT - 1) / OWT;
  const int64_t total = (int64_t)p.N * p.H * WT * CG;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int cg = (int)(i % CG);
    int64_t r = i / CG;
    const int wt = (int)(r % WT);
    r /= WT;
    const int h = (int)(r % p.H);
    const int n = (int)(r / p.H);
    const int c0 = cg * V;
    const int w0 = wt * OWT;
    float acc[OWT][V];
#pragma unroll
    for (int j = 0; j < OWT; ++j)
#pragma unroll
      for (int v = 0; v < V; ++v) acc[j][v] = 0.f;
    if constexpr (S == 1) {
      constexpr int NC = OWT + KS - 1;
      float wv[KS * KS][V];
#pragma unroll
      for (int t = 0; t < KS * KS; ++t) ld_w<V>(p.w + t * p.C + c0, wv[t]);
      const int ow0 = w0 + p.pad - (KS - 1);
      typename vec<V>::t raw[KS][NC];
#pragma unroll
      for (int kh = 0; kh < KS; ++kh) {
        const int oh = h + p.pad - kh;
        const bool okr = (unsigned)oh < (unsigned)p.Ho;
        const bf16_t* row = p.x + (((int64_t)n * p.Ho + (okr ? oh : 0)) * p.Wo) * p.C + c0;
#pragma unroll
        for (int q = 0; q < NC; ++q) {
          const int ow = ow0 + q;
          raw[kh][q] = ld_raw<V>(row + (int64_t)ow * p.C, okr && (unsigned)ow < (unsigned)p.Wo);
        }
      }
#pragma unroll
      for (int kh = 0; kh < KS; ++kh) {
        float d[NC][V];
#pragma unroll
        for (int q = 0; q < NC; ++q) unpack<V>(raw[kh][q], d[q]);
#pragma unroll
        for (int kw = 0; kw < KS; ++kw)
#pragma unroll
          for (int j = 0; j < OWT; ++j)
#pragma unroll
            for (int v = 0; v < V; ++v) acc[j][v] += d[j + KS - 1 - kw][v] * wv[kh * KS + kw][v];
      }
    } else {
#pragma unroll
    for (int kh = 0; kh < KS; ++kh) {
      const int t = h + p.pad - kh;
      if (t < 0 || t % p.stride) continue;
      const int oh = t / p.stride;
      if (oh >= p.Ho) continue;
      const bf16_t* row = p.x + (((int64_t)n * p.Ho + oh) * p.Wo) * p.C + c0;
#pragma unroll
      for (int kw = 0; kw < KS; ++kw) {
        float wv[V];
        const float* wp = p.w + (kh * KS + kw) * p.C + c0;
#pragma unroll
        for (int v = 0; v < V; ++v) wv[v] = wp[v];
#pragma unroll
        for (int j = 0; j < OWT; ++j) {
          const int u = w0 + j + p.pad - kw;
          if (w0 + j >= p.W || u < 0 || u % p.stride) continue;
          const int ow = u / p.stride;
          if (ow >= p.Wo) continue;
          float d[V];
          ld_vec<V>(row + (int64_t)ow * p.C, d);
#pragma unroll
          for (int v = 0; v < V; ++v) acc[j][v] += d[v] * wv[v];
        }
      }
    }
    }
#pragma unroll
    for (int j = 0; j < OWT; ++j) {
      const int w = w0 + j;
      if (w >= p.W) break;
      st_vec<V>(p.y + (((int64_t)n * p.H + h) * p.W + w) * p.C + c0, acc[j]);
    }
  }
}

// Per-block partials of dW[tap, c] = sum_m dy[m, c] * x[src(m, tap), c].
// Thread = (channel group cg, lane); a lane's work item is OWT consecutive
// output pixels of one output row: it loads the 3 x ((OWT-1)*S + 3) input
// columns and OWT dy vectors once (~5.5 loads per pixel instead of 10, all
// independent), accumulating acc[9][V].  partial[blk][9][C].
template <int V, int S>
__global__ void __launch_bounds__(256)
dw_wgrad_partial_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                        float* __restrict__ partial, int N, int H, int W, int C, int Ho, int Wo,
                        int pad) {
  constexpr int NCOLS = (OWT - 1) * S + KS;
  constexpr int KK = KS * KS;
  constexpr int TG = 3;  // taps per reduction round
  __shared__ float red[TG * 256 * V];
  __shared__ float red2[1024];  // (output, slice) pair sums when SL > 1 (OUT*SL <= 1024)
  const int CG = C / V;
  const int PL = max(1, 256 / CG);  // lanes per block
  const int tid = threadIdx.x;
  const int cg = tid % CG, pl = tid / CG;
  const bool active = tid < CG * PL;
  const int c0 = cg * V;
  const int WT = (Wo + OWT - 1) / OWT;
  const int64_t items = (int64_t)N * Ho * WT;
  float acc[KK][V];
#pragma unroll
  for (int t = 0; t < KK; ++t)
#pragma unroll
    for (int v = 0; v < V; ++v) acc[t][v] = 0.f;
  if (active) {
    for (int64_t it = (int64_t)blockIdx.x * PL + pl; it < items; it += (int64_t)gridDim.x * PL) {
      const int wt = (int)(it % WT);
      const int64_t r = it / WT;
      const int ho = (int)(r % Ho);
      const int n = (int)(r / Ho);
      const int wo0 = wt * OWT;
      const int iw0 = wo0 * S - pad;
      typename vec<V>::t draw[OWT], raw[KS][NCOLS];
      const bf16_t* drow = dy + (((int64_t)n * Ho + ho) * Wo + wo0) * C + c0;
#pragma unroll
      for (int j = 0; j < OWT; ++j) draw[j] = ld_raw<V>(drow + (int64_t)j * C, wo0 + j < Wo);
#pragma unroll
      for (int kh = 0; kh < KS; ++kh) {
        const int ih = ho * S - pad + kh;
        const bool okr = (unsigned)ih < (unsigned)H;
        const bf16_t* row = x + (((int64_t)n * H + (okr ? ih : 0)) * W) * C + c0;
#pragma unroll
        for (int q = 0; q < NCOLS; ++q) {
          const int iw = iw0 + q;
          raw[kh][q] = ld_raw<V>(row + (int64_t)iw * C, okr && (unsigned)iw < (unsigned)W);
        }
      }
      float d[OWT][V];
#pragma unroll
      for (int j = 0; j < OWT; ++j) unpack<V>(draw[j], d[j]);
#pragma unroll
      for (int kh = 0; kh < KS; ++kh) {
        float xin[NCOLS][V];
#pragma unroll
        for (int q = 0; q < NCOLS; ++q) unpack<V>(raw[kh][q], xin[q]);
#pragma unroll
        for (int kw = 0; kw < KS; ++kw)
#pragma unroll
          for (int j = 0; j < OWT; ++j)
#pragma unroll
            for (int v = 0; v < V; ++v) acc[kh * KS + kw][v] += d[j][v] * xin[j * S + kw][v];
      }
    }
  }
  // Reduce over the PL lanes with every thread, three taps per round (LDS
  // red[3][PL][C], PL*C <= 256*V: 24.6 KB, so load-phase occupancy stays at
  // 5+ blocks/CU): (output, slice) pairs each sum PL/SL lanes (slice-major,
  // neighbouring threads read neighbouring channels), then each output sums
  // its SL slices -- fixed order.  (One thread per channel walking all PL
  // lanes tap by tap was ~1150 dependent LDS reads for C = 16, PL = 128.)
  const int OUT = TG * C;  // outputs per round
  int SL = 1;
  while (SL * 2 <= PL && OUT * SL * 2 <= 1024) SL *= 2;
#pragma unroll
  for (int g = 0; g < KK / TG; ++g) {
    if (active) {
#pragma unroll
      for (int t = 0; t < TG; ++t)
#pragma unroll
        for (int v = 0; v < V; ++v) red[(t * PL + pl) * C + c0 + v] = acc[g * TG + t][v];
    }
    __syncthreads();
    float* dst = partial + ((int64_t)blockIdx.x * KK + g * TG) * C;  // [blk][tap][c]
    for (int pr = tid; pr < OUT * SL; pr += blockDim.x) {
      const int s = pr / OUT, o = pr - s * OUT;
      const int t = o / C, c = o - t * C;
      float a = 0.f;
      for (int q = s; q < PL; q += SL) a += red[(t * PL + q) * C + c];
      if (SL == 1) dst[o] = a; else red2[pr] = a;
    }
    __syncthreads();
    if (SL > 1) {
      for (int o = tid; o < OUT; o += blockDim.x) {
        float a = 0.f;
        for (int j = 0; j < SL; ++j) a += red2[j * OUT + o];
        dst[o] = a;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// LDS-tiled depthwise forward / weight gradient (pad 1, stride 1 or 2).
// The register-tiled kernels above load every input vector ~4.5x through the
// cache hierarchy and need 150-256 VGPRs (1-3 waves per SIMD): latency bound
// at 15-25 % of HBM rate on the MobileNet layers.  Here a block stages the
// input rows of `tr` output rows (+ halo, zero padded) for `cc` channels ONCE
// in LDS (the weight gradient also the tile's dy), and each thread owns one
// channel of a pixel slice: 9 LDS reads + 9 FMAs per output (forward) or per
// dy pixel (weight gradient, 9 per-thread accumulators); slices reduce through
// LDS.  Block = (sample, row tile) x channel chunk; the weight-gradient
// partial rows keep the [blk][tap][C] layout of dw_wgrad_partial_kernel
// (same finalize / multi-layer reduce).
// LDS bytes per block (MDA_DW_TILE_KB, default 24: 6 blocks per CU; A/B 24 / 40 /
// 64 KB: R50->MV1 6.34 / 6.44 / 6.63 ms, VGG13->MV2 2.62 / 2.61 / 2.61,
// register kernels 6.41 / 2.70 -- profiles/r4_dw_fusion_ab.md)
inline int64_t dwt_budget() {
  static const int64_t b = [] {
    const char* e = getenv("MDA_DW_TILE_KB");
    const int64_t k = e ? atoll(e) : 24;
    return (k >= 8 && k <= 150 ? k : 24) * 1024;
  }();
  return b;
}

// x rows [ih0, ih0 + rin) x cols [-1, W] of channels [c0, c0 + cc) -> xs
// (zero outside the image).
__device__ __forceinline__ void dw_fill_x(const bf16_t* __restrict__ x, bf16_t* xs, int n, int H, int W,
                                          int C, int c0, int cc, int ih0, int rin) {
  const int Wp = W + 2, cv = cc / 8;
  for (int i = threadIdx.x; i < rin * Wp * cv; i += blockDim.x) {
    const int pos = i / cv, q = i - pos * cv;
    const int r = pos / Wp, col = pos - r * Wp;
    const int ih = ih0 + r, iw = col - 1;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
      v = *(const uint4*)(x + (((int64_t)n * H + ih) * W + iw) * C + c0 + 8 * q);
    *(uint4*)(xs + (size_t)pos * cc + 8 * q) = v;
  }
}

template <int S>
__global__ void __launch_bounds__(256) dw_wgrad_tile_kernel(const bf16_t* __restrict__ x,
                                                            const bf16_t* __restrict__ dy,
                                                            float* __restrict__ partial, int N, int H,
                                                            int W, int C, int Ho, int Wo, int tr, int cc) {
  extern __shared__ __attribute__((aligned(16))) bf16_t dwt_sm[];
  const int tid = threadIdx.x;
  const int nrt = (Ho + tr - 1) / tr;
  const int blk = blockIdx.x, n = blk / nrt, rt = blk - n * nrt;
  const int c0 = blockIdx.y * cc;
  const int ho0 = rt * tr, hon = min(tr, Ho - ho0);
  const int rin = (tr - 1) * S + 3, Wp = W + 2, cv = cc / 8;
  bf16_t* xs = dwt_sm;
  bf16_t* ds = dwt_sm + (size_t)rin * Wp * cc;
  dw_fill_x(x, xs, n, H, W, C, c0, cc, ho0 * S - 1, rin);
  for (int i = tid; i < tr * Wo * cv; i += 256) {
    const int pos = i / cv, q = i - pos * cv;
    const int r = pos / Wo, col = pos - r * Wo;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (r < hon) v = *(const uint4*)(dy + (((int64_t)n * Ho + ho0 + r) * Wo + col) * C + c0 + 8 * q);
    *(uint4*)(ds + (size_t)pos * cc + 8 * q) = v;
  }
  __syncthreads();
  const int c = tid % cc, sl = tid / cc, nsl = 256 / cc;
  float acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = 0.f;
  for (int r = 0; r < hon; ++r)
    for (int col = sl; col < Wo; col += nsl) {
      const float d = bf2f(ds[((size_t)r * Wo + col) * cc + c]);
      const bf16_t* xb = xs + ((size_t)(r * S) * Wp + col * S) * cc + c;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) acc[kh * 3 + kw] += d * bf2f(xb[((size_t)kh * Wp + kw) * cc]);
    }
  __syncthreads();  // the tiles are dead: the slice reduction reuses the LDS
  float* red = (float*)dwt_sm;  // [nsl][9][cc]
#pragma unroll
  for (int t = 0; t < 9; ++t) red[((size_t)sl * 9 + t) * cc + c] = acc[t];
  __syncthreads();
  for (int o = tid; o < 9 * cc; o += 256) {
    const int t = o / cc, ch = o - t * cc;
    float a = 0.f;
    for (int s2 = 0; s2 < nsl; ++s2) a += red[((size_t)s2 * 9 + t) * cc + ch];
    partial[((int64_t)blk * 9 + t) * C + c0 + ch] = a;
  }
}

// Training forward: raw bf16 output + the BN batch sums of the stored values
// into p.stats_slot (or no statistics).
template <int S>
__global__ void __launch_bounds__(256) dw_fwd_tile_kernel(const DwParams p, int tr, int cc) {
  extern __shared__ __attribute__((aligned(16))) bf16_t dwt_sm[];
  const int tid = threadIdx.x;
  const int nrt = (p.Ho + tr - 1) / tr;
  const int blk = blockIdx.x, n = blk / nrt, rt = blk - n * nrt;
  const int c0 = blockIdx.y * cc;
  const int ho0 = rt * tr, hon = min(tr, p.Ho - ho0);
  const int rin = (tr - 1) * S + 3, Wp = p.W + 2;
  bf16_t* xs = dwt_sm;
  dw_fill_x(p.x, xs, n, p.H, p.W, p.C, c0, cc, ho0 * S - 1, rin);
  __syncthreads();
  const int c = tid % cc, sl = tid / cc, nsl = 256 / cc;
  float wv[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) wv[t] = p.w[t * p.C + c0 + c];
  float st1 = 0.f, st2 = 0.f;
  for (int r = 0; r < hon; ++r) {
    bf16_t* yrow = p.y + (((int64_t)n * p.Ho + ho0 + r) * p.Wo) * p.C + c0 + c;
    for (int col = sl; col < p.Wo; col += nsl) {
      const bf16_t* xb = xs + ((size_t)(r * S) * Wp + col * S) * cc + c;
      float a = 0.f;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) a += wv[kh * 3 + kw] * bf2f(xb[((size_t)kh * Wp + kw) * cc]);
      const bf16_t o = f2bf(a);
      yrow[(int64_t)col * p.C] = o;
      const float q = bf2f(o);
      st1 += q;
      st2 += q * q;
    }
  }
  if (p.stats_slot == nullptr) return;
  __syncthreads();
  float* red = (float*)dwt_sm;  // [2][nsl][cc]
  red[(size_t)sl * cc + c] = st1;
  red[(size_t)(nsl + sl) * cc + c] = st2;
  __syncthreads();
  if (tid < 2 * cc) {
    const int qq = tid / cc, ch = tid - qq * cc;
    float a = 0.f;
    for (int s2 = 0; s2 < nsl; ++s2) a += red[(size_t)(qq * nsl + s2) * cc + ch];
    const int shard = (int)(blk + gridDim.x * blockIdx.y) % slot_shards(p.C);
    acc_add(region_acc(p.stats_slot, p.C, shard, qq) + c0 + ch, (double)a);
  }
}

// dgrad: dx[h, w] = sum_{kh,kw} w[2-kh, 2-kw] * dyd[h - 1 + kh, w - 1 + kw]
// with dyd the stride-dilated dy (dy[i/S, j/S] at multiples of S, else 0):
// the stride-1 forward's tile loop on a (dilated) dy tile with the flipped
// filter.  p.x = dy [N, Ho, Wo, C], p.y = dx [N, H, W, C].
template <int S>
__global__ void __launch_bounds__(256) dw_dgrad_tile_kernel(const DwParams p, int tr, int cc) {
  extern __shared__ __attribute__((aligned(16))) bf16_t dwt_sm[];
  const int tid = threadIdx.x;
  const int nrt = (p.H + tr - 1) / tr;
  const int blk = blockIdx.x, n = blk / nrt, rt = blk - n * nrt;
  const int c0 = blockIdx.y * cc;
  const int h0 = rt * tr, hon = min(tr, p.H - h0);
  const int rin = tr + 2, Wp = p.W + 2, cv = cc / 8;
  bf16_t* xs = dwt_sm;
  for (int i = tid; i < rin * Wp * cv; i += blockDim.x) {
    const int pos = i / cv, q = i - pos * cv;
    const int r = pos / Wp, col = pos - r * Wp;
    const int di = h0 - 1 + r, dj = col - 1;  // dilated dy coordinates
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (di >= 0 && dj >= 0 && di % S == 0 && dj % S == 0 && di / S < p.Ho && dj / S < p.Wo)
      v = *(const uint4*)(p.x + (((int64_t)n * p.Ho + di / S) * p.Wo + dj / S) * p.C + c0 + 8 * q);
    *(uint4*)(xs + (size_t)pos * cc + 8 * q) = v;
  }
  __syncthreads();
  const int c = tid % cc, sl = tid / cc, nsl = 256 / cc;
  float wv[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) wv[t] = p.w[(8 - t) * p.C + c0 + c];
  for (int r = 0; r < hon; ++r) {
    bf16_t* xrow = p.y + (((int64_t)n * p.H + h0 + r) * p.W) * p.C + c0 + c;
    for (int col = sl; col < p.W; col += nsl) {
      const bf16_t* xb = xs + ((size_t)r * Wp + col) * cc + c;
      float a = 0.f;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) a += wv[kh * 3 + kw] * bf2f(xb[((size_t)kh * Wp + kw) * cc]);
      xrow[(int64_t)col * p.C] = f2bf(a);
    }
  }
}

// Tile plan: output rows per block (tr) and channels per block (cc) so the
// block's LDS fits dwt_budget(); false = not served (the register kernels run).
inline bool dw_tile_plan(int H, int W, int C, int Ho, int Wo, int S, int pad, bool with_dy, int& tr,
                         int& cc) {
  static const bool on = [] {
    const char* e = getenv("MDA_DW_TILE");
    return !(e && e[0] == '0');
  }();
  cc = C % 64 == 0 ? 64 : C % 32 == 0 ? 32 : C % 16 == 0 ? 16 : 8;  // channels per block
  if (!on || pad != 1 || C % cc || (S != 1 && S != 2)) return false;
  for (int t = Ho < 16 ? Ho : 16; t >= 1; --t) {
    const int64_t rin = (int64_t)(t - 1) * S + 3;
    const int64_t bytes = (rin * (W + 2) + (with_dy ? (int64_t)t * Wo : 0)) * cc * 2;
    if (bytes <= dwt_budget()) {
      tr = t;
      return true;
    }
  }
  return false;
}

inline size_t dw_tile_lds(int W, int Wo, int S, int tr, int cc, bool with_dy) {
  const size_t rin = (size_t)(tr - 1) * S + 3;
  const size_t b = (rin * (W + 2) + (with_dy ? (size_t)tr * Wo : 0)) * cc * 2;
  const size_t red = (size_t)256 * 9 * 4;  // the slice reduction reuses the tile
  return b > red ? b : red;
}

// grad[c, tap] (+)= sum_blk partial[blk][tap][c]   (fixed order, fp64)
// Block = 32 elements x 8 block-slices: thread (e, s) sums the partial blocks
// b = s (mod 8) with four loads in flight, then slice sums combine in a fixed
// order through LDS.  (One thread per element walking all 512 blocks was
// latency-bound: ~22 us per MobileNet layer.)
__global__ void __launch_bounds__(256)
dw_wgrad_finalize_kernel(const float* __restrict__ partial, int nblk, int KK, int C,
                         float* __restrict__ grad, int accumulate) {
  __shared__ double red[8][32];
  const int64_t V = (int64_t)KK * C;
  const int e = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const int64_t i = (int64_t)blockIdx.x * 32 + e;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (i < V) {
    int b = sl;
    for (; b + 24 < nblk; b += 32) {
      s0 += (double)partial[(int64_t)(b + 0) * V + i];
      s1 += (double)partial[(int64_t)(b + 8) * V + i];
      s2 += (double)partial[(int64_t)(b + 16) * V + i];
      s3 += (double)partial[(int64_t)(b + 24) * V + i];
    }
    for (; b < nblk; b += 8) s0 += (double)partial[(int64_t)b * V + i];
  }
  red[sl][e] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (sl != 0 || i >= V) return;
  const double s = ((red[0][e] + red[1][e]) + (red[2][e] + red[3][e])) +
                   ((red[4][e] + red[5][e]) + (red[6][e] + red[7][e]));
  const int t = (int)(i / C), c = (int)(i - (int64_t)t * C);
  float* o = grad + (int64_t)c * KK + t;
  *o = accumulate ? *o + (float)s : (float)s;
}

// fp32 [C, KH, KW] -> fp32 [KH*KW, C] (optionally scaled per channel)
__global__ void dw_pack_kernel(const float* __restrict__ w, const float* __restrict__ scale,
                               float* __restrict__ out, int C, int KK) {
  const int total = C * KK;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int t = i / C, c = i - t * C;
    out[i] = w[c * KK + t] * (scale ? scale[c] : 1.f);
  }
}

// channels per thread, capped at MDA_DW_VMAX (default 4): the V = 8 kernels
// (16-byte vectors) need 234-256 VGPRs -- 1-2 waves per SIMD -- the V = 4 ones
// ~150 (3 waves); R50->MV1 6.55 -> 6.40 ms, VGG13->MV2 2.77 -> 2.68
// (profiles/r4_dw_fusion_ab.md)
inline int vwidth(int C) {
  static const int vmax = [] {
    const char* e = getenv("MDA_DW_VMAX");
    const int v = e ? atoi(e) : 4;
    return (v == 1 || v == 2 || v == 8) ? v : 4;
  }();
  const int v = (C % 8 == 0) ? 8 : (C % 4 == 0) ? 4 : (C % 2 == 0) ? 2 : 1;
  return v < vmax ? v : vmax;
}

inline int grid_for(int64_t work) {
  int64_t b = (work + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

// grid of a launch whose threads keep one channel group (region sums): a
// multiple of the stride period, at most 256 blocks per region shard
int region_grid(int nb, int C, int V) {
  const int CG = C / V;
  int a = CG, b = 256;
  while (b) { const int t = a % b; a = b; b = t; }
  const int unit = CG / a;  // blocks per stride period
  const int cap = 256 * slot_shards(C);
  nb = nb < cap ? nb : cap;
  return (nb + unit - 1) / unit * unit;
}

int launch_fwd(const DwParams& p, hipStream_t st) {
  int tr, cc;
  if (!p.scale && !p.bias && !p.res && !p.preact && p.act == 0 &&
      dw_tile_plan(p.H, p.W, p.C, p.Ho, p.Wo, p.stride, p.pad, false, tr, cc)) {
    const dim3 g((unsigned)(p.N * ((p.Ho + tr - 1) / tr)), (unsigned)(p.C / cc));
    const size_t lds = dw_tile_lds(p.W, p.Wo, p.stride, tr, cc, false);
    if (p.stride == 1) hipLaunchKernelGGL((dw_fwd_tile_kernel<1>), g, dim3(256), lds, st, p, tr, cc);
    else hipLaunchKernelGGL((dw_fwd_tile_kernel<2>), g, dim3(256), lds, st, p, tr, cc);
    return (int)hipGetLastError();
  }
  const int V = vwidth(p.C);
  const int64_t work = (int64_t)p.N * p.Ho * ((p.Wo + OWT - 1) / OWT) * (p.C / V);
  int nb = grid_for(work);
  // grid stride a multiple of CG (each thread keeps its channel group); at most
  // 256 blocks per region shard, so each region address sees few atomics
  if (p.stats_slot) nb = region_grid(nb, p.C, V);
  const dim3 g(nb);
#define DW_FWD(VV, SS) hipLaunchKernelGGL((dw_fwd_kernel<VV, SS>), g, dim3(256), 0, st, p)
  if (p.stride == 1) {
    if (V == 8) DW_FWD(8, 1); else if (V == 4) DW_FWD(4, 1); else if (V == 2) DW_FWD(2, 1); else DW_FWD(1, 1);
  } else {
    if (V == 8) DW_FWD(8, 2); else if (V == 4) DW_FWD(4, 2); else if (V == 2) DW_FWD(2, 2); else DW_FWD(1, 2);
  }
#undef DW_FWD
  return (int)hipGetLastError();
}

}  // namespace

MDA_API int mda_dw_pack(const float* w, const float* scale, float* out, int64_t C, int64_t KK,
                        hipStream_t st) {
  hipLaunchKernelGGL(dw_pack_kernel, dim3(grid_for(C * KK)), dim3(256), 0, st, w, scale, out,
                     (int)C, (int)KK);
  MDA_CHECK_LAUNCH();
}

// x [N,H,W,C] bf16; w packed [KH*KW, C] fp32; scale/bias [C] or null; res/preact or null.
MDA_API int mda_dw_fwd(const void* x, const float* w, const float* scale, const float* bias,
                       const void* res, void* y, void* preact, int64_t N, int64_t H, int64_t W,
                       int64_t C, int64_t Ho, int64_t Wo, int64_t KH, int64_t KW, int64_t stride,
                       int64_t pad, int64_t act, hipStream_t st) {
  if (KH != KS || KW != KS || stride < 1 || stride > 2) return (int)hipErrorInvalidValue;
  DwParams p{(const bf16_t*)x, w, scale, bias, (const bf16_t*)res, (bf16_t*)y, (bf16_t*)preact,
             (int)N, (int)H, (int)W, (int)C, (int)Ho, (int)Wo, (int)KH, (int)KW, (int)stride,
             (int)pad, (int)act};
  return launch_fwd(p, st);
}

namespace {
int launch_dgrad(const DwParams& p, hipStream_t st) {
  const int64_t N = p.N, H = p.H, W = p.W, C = p.C;
  const int stride = p.stride;
  int tr, cc;
  if (dw_tile_plan((int)H, (int)W, (int)C, (int)H, (int)W, 1, p.pad, false, tr, cc)) {
    const dim3 g((unsigned)(N * ((H + tr - 1) / tr)), (unsigned)(C / cc));
    const size_t lds = dw_tile_lds((int)W, (int)W, 1, tr, cc, false);
    if (stride == 1) hipLaunchKernelGGL((dw_dgrad_tile_kernel<1>), g, dim3(256), lds, st, p, tr, cc);
    else hipLaunchKernelGGL((dw_dgrad_tile_kernel<2>), g, dim3(256), lds, st, p, tr, cc);
    return (int)hipGetLastError();
  }
  const int V = vwidth((int)C);
  const int64_t work = N * H * ((W + OWT - 1) / OWT) * (C / V);
  const dim3 g(grid_for(work));
#define DW_DG(VV, SS) hipLaunchKernelGGL((dw_dgrad_kernel<VV, SS>), g, dim3(256), 0, st, p)
  if (stride == 1) {
    if (V == 8) DW_DG(8, 1); else if (V == 4) DW_DG(4, 1); else if (V == 2) DW_DG(2, 1); else DW_DG(1, 1);
  } else {
    if (V == 8) DW_DG(8, 2); else if (V == 4) DW_DG(4, 2); else if (V == 2) DW_DG(2, 2); else DW_DG(1, 2);
  }
#undef DW_DG
  MDA_CHECK_LAUNCH();
}
}  // namespace

// dy [N,Ho,Wo,C] bf16 -> dx [N,H,W,C] bf16.
MDA_API int mda_dw_dgrad(const void* dy, const float* w, void* dx, int64_t N, int64_t H, int64_t W,
                         int64_t C, int64_t Ho, int64_t Wo, int64_t KH, int64_t KW, int64_t stride,
                         int64_t pad, hipStream_t st) {
  if (KH != KS || KW != KS || stride < 1 || stride > 2) return (int)hipErrorInvalidValue;
  DwParams p{(const bf16_t*)dy, w, nullptr, nullptr, nullptr, (bf16_t*)dx, nullptr, (int)N,
             (int)H, (int)W, (int)C, (int)Ho, (int)Wo, (int)KH, (int)KW, (int)stride, (int)pad, 0};
  return launch_dgrad(p, st);
}

MDA_API int mda_dw_wgrad_blocks(int64_t N, int64_t Ho, int64_t Wo, int64_t C, int64_t* nblk);

// Partial rows of mda_dw_wgrad for this shape (the tile kernel's (sample,
// row tile) blocks when it serves the shape, else mda_dw_wgrad_blocks').
MDA_API int mda_dw_wgrad_blocks2(int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho, int64_t Wo,
                                 int64_t stride, int64_t pad, int64_t* nblk) {
  int tr, cc;
  if (dw_tile_plan((int)H, (int)W, (int)C, (int)Ho, (int)Wo, (int)stride, (int)pad, true, tr, cc)) {
    *nblk = N * ((Ho + tr - 1) / tr);
    return 0;
  }
  return mda_dw_wgrad_blocks(N, Ho, Wo, C, nblk);
}

MDA_API int mda_dw_wgrad_blocks(int64_t N, int64_t Ho, int64_t Wo, int64_t C, int64_t* nblk) {
  const int V = vwidth((int)C);
  const int64_t CG = C / V;
  const int64_t PL = CG >= 256 ? 1 : 256 / CG;
  const int64_t items = N * Ho * ((Wo + OWT - 1) / OWT);
  // ~ITEMS_PER_LANE work items (4 pixels each) per lane: enough blocks that the
  // lanes' independent load batches hide the memory latency (the finalize
  // reads the nblk partials in parallel)
  // (A/B, profiles/r2_misc_ab.md: 1 for CIFAR-size maps, 2 for 112^2 ImageNet ones)
  static const int64_t forced = [] {
    const char* e = getenv("MDA_DW_WG_IPL");
    return e ? (int64_t)atoi(e) : (int64_t)0;
  }();
  const int64_t ipl = forced > 0 ? forced : (N * Ho * ((Wo + OWT - 1) / OWT) < 200000 ? 1 : 2);
  int64_t b = (items + PL * ipl - 1) / (PL * ipl);
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  *nblk = b;
  return 0;
}

// x [N,H,W,C], dy [N,Ho,Wo,C] bf16; partial >= nblk*KH*KW*C floats;
// grad fp32 [C, KH, KW] (accumulated when accumulate != 0).
MDA_API int mda_dw_wgrad(const void* x, const void* dy, float* partial, float* grad, int64_t N,
                         int64_t H, int64_t W, int64_t C, int64_t Ho, int64_t Wo, int64_t KH,
                         int64_t KW, int64_t stride, int64_t pad, int64_t nblk,
                         int64_t accumulate, hipStream_t st) {
  if (KH != KS || KW != KS || stride < 1 || stride > 2 || nblk < 1) return (int)hipErrorInvalidValue;
  int tr, cc;
  if (dw_tile_plan((int)H, (int)W, (int)C, (int)Ho, (int)Wo, (int)stride, (int)pad, true, tr, cc)) {
    const int64_t nb = N * ((Ho + tr - 1) / tr);
    if (nb != nblk) return (int)hipErrorInvalidValue;  // partial rows sized by mda_dw_wgrad_blocks2
    const dim3 g((unsigned)nb, (unsigned)(C / cc));
    const size_t lds = dw_tile_lds((int)W, (int)Wo, (int)stride, tr, cc, true);
#define DW_WT(SS)                                                                              \
  hipLaunchKernelGGL((dw_wgrad_tile_kernel<SS>), g, dim3(256), lds, st, (const bf16_t*)x,        \
                     (const bf16_t*)dy, partial, (int)N, (int)H, (int)W, (int)C, (int)Ho, (int)Wo, \
                     tr, cc)
    if (stride == 1) DW_WT(1); else DW_WT(2);
#undef DW_WT
  } else {
  const int V = vwidth((int)C);
  if (C / V > 256) return (int)hipErrorInvalidValue;
#define DW_WG(VV, SS)                                                                       \
  hipLaunchKernelGGL((dw_wgrad_partial_kernel<VV, SS>), dim3(nblk), dim3(256), 0, st,          \
                     (const bf16_t*)x, (const bf16_t*)dy, partial, (int)N, (int)H, (int)W,      \
                     (int)C, (int)Ho, (int)Wo, (int)pad)
  if (stride == 1) {
    if (V == 8) DW_WG(8, 1); else if (V == 4) DW_WG(4, 1); else if (V == 2) DW_WG(2, 1); else DW_WG(1, 1);
  } else {
    if (V == 8) DW_WG(8, 2); else if (V == 4) DW_WG(4, 2); else if (V == 2) DW_WG(2, 2); else DW_WG(1, 2);
  }
#undef DW_WG
  }
  if (grad == nullptr) MDA_CHECK_LAUNCH();  // partials only (a deferred multi-layer reduce sums them)
  hipLaunchKernelGGL(dw_wgrad_finalize_kernel, dim3((unsigned)((KH * KW * C + 31) / 32)), dim3(256), 0, st,
                     partial, (int)nblk, (int)(KH * KW), (int)C, grad, (int)accumulate);
  MDA_CHECK_LAUNCH();
}

// Training depthwise conv whose blocks add the BN statistics of the stored
// output into `region` (the caller follows with mda_bn_apply_fin).
MDA_API int mda_dw_fwd_bnacc(const void* x, const float* w, void* y, void* region, int64_t N,
                             int64_t H, int64_t W, int64_t C, int64_t Ho, int64_t Wo, int64_t KH,
                             int64_t KW, int64_t stride, int64_t pad, hipStream_t st) {
  if (KH != KS || KW != KS || stride < 1 || stride > 2 || C > SLOT_CMAX || region == nullptr)
    return (int)hipErrorInvalidValue;
  DwParams p{(const bf16_t*)x, w, nullptr, nullptr, nullptr, (bf16_t*)y, nullptr, (int)N, (int)H,
             (int)W, (int)C, (int)Ho, (int)Wo, (int)KH, (int)KW, (int)stride, (int)pad, 0,
             (BnRegion*)region};
  return launch_fwd(p, st);
}
