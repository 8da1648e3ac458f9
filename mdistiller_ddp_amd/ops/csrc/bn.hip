// Training-mode BatchNorm (+ residual + activation) around the MFMA convs
// (survey K1, student side).  NHWC bf16 activations viewed as [M, C] with
// M = N*H*W; fp32 statistics.
//
// forward:   stats   (y -> mean, rstd, scale = g*rstd, shift = b - mean*scale,
//                     running-stat update)               one launch, last
//                                                          arriver finalises
//            apply   z = y*scale + shift (+ res) ; out = act(z) (+ preact z)
// backward:  reduce  dz = dout * act'(z) (+ dpreact) ; dbeta = sum dz,
//                     dgamma = sum dz*xhat  -> accumulated into the flat
//                     gradient buffer, last arriver finalises
//            apply   dy = scale * (dz - (dbeta + xhat*dgamma)/M) ; dres = dz
//
// versus MIOpen's 4 forward + 3 backward BN kernels plus separate add / ReLU
// (and its backward) launches per layer in the reference stack.
// Determinism: the partial-row kernels in this first part (stats /
// bn_bwd_reduce2 + a finalize) combine fixed per-block fp32 partials in a
// fixed order in fp64, so they are deterministic.  The default fused path
// below (one-shot BnRegion channel sums, csrc/bnslot.h) adds block partials
// with fp64 atomics, whose order varies run to run: its results agree to fp64
// rounding only.  EXPERIMENT.DETERMINISTIC selects the partial-row kernels
// (ops/hip_train.py set_deterministic).
#include "common.h"

namespace {


enum { ACT_NONE = 0, ACT_RELU = 1, ACT_RELU6 = 2 };

__device__ __forceinline__ float act_f(float v, int act) {
  if (act == ACT_RELU) return fmaxf(v, 0.f);
  if (act == ACT_RELU6) return fminf(fmaxf(v, 0.f), 6.f);
  return v;
}
__device__ __forceinline__ float act_grad(float z, int act) {
  if (act == ACT_RELU) return z > 0.f ? 1.f : 0.f;
  if (act == ACT_RELU6) return (z > 0.f && z < 6.f) ? 1.f : 0.f;
  return 1.f;
}

// Block-level per-channel partial sums of two quantities over rows, 8
// channels (16 bytes) per thread: thread t owns channel group t % C8 and row
// offset t / C8; rows are strided over the grid.  Writes partial[blk][2][C].
__device__ __forceinline__ void block_channel_partials(float (&a)[8], float (&b)[8], int C,
                                                       int rpi, float* __restrict__ partial) {
  __shared__ float sm[2][256 * 8];
  const int tid = threadIdx.x;
  const int C8 = C / 8;
  const int cg = tid % C8, r0 = tid / C8;
  if (r0 < rpi) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sm[0][r0 * C + cg * 8 + k] = a[k];
      sm[1][r0 * C + cg * 8 + k] = b[k];
    }
  }
  __syncthreads();
  for (int t = tid; t < 2 * C; t += blockDim.x) {
    const int q = t / C, c = t - q * C;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int r = 0;
    for (; r + 4 <= rpi; r += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += sm[q][(r + u) * C + c];
    }
    for (; r < rpi; ++r) acc[0] += sm[q][r * C + c];
    partial[(int64_t)blockIdx.x * 2 * C + t] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  }
}

// Deterministic two-level combine of the per-block partials partial[blk][V]
// (V = 2C): blocks arrive in groups of RED_GROUP; the last arriver of a group
// sums its group's rows in block order into gpart[group][V]; the last group
// to finish sums the group rows (fp64, fixed order) into tot[V] (LDS).  Every
// thread of the final block issues its <= 16 loads together, so the serial
// tail is two L2 round trips instead of one block walking nblk*V values.
// counters: [0] = top level, [1 + g] = group g (>= 1 + 256/RED_GROUP zeroed uints).
constexpr int RED_GROUP = 16;
constexpr int RED_MAX_BLOCKS = 256;

__device__ __forceinline__ bool combine_partials(float* __restrict__ partial, int V,
                                                 unsigned* __restrict__ counters,
                                                 double* __restrict__ tot) {
  const int nblk = gridDim.x;
  const int ngrp = (nblk + RED_GROUP - 1) / RED_GROUP;
  const int g = blockIdx.x / RED_GROUP;
  const int gsize = min(RED_GROUP, nblk - g * RED_GROUP);
  float* gpart = partial + (int64_t)nblk * V;
  if (!mda_arrive(counters + 1 + g, gsize)) return false;
  for (int v = threadIdx.x; v < V; v += blockDim.x) {
    float x[RED_GROUP];
#pragma unroll
    for (int i = 0; i < RED_GROUP; ++i)
      x[i] = i < gsize ? partial[(int64_t)(g * RED_GROUP + i) * V + v] : 0.f;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < RED_GROUP; ++i) acc += x[i];
    gpart[(int64_t)g * V + v] = acc;
  }
  if (!mda_arrive(counters, ngrp)) return false;
  for (int v = threadIdx.x; v < V; v += blockDim.x) {
    float x[RED_MAX_BLOCKS / RED_GROUP];
#pragma unroll
    for (int i = 0; i < RED_MAX_BLOCKS / RED_GROUP; ++i)
      x[i] = i < ngrp ? gpart[(int64_t)i * V + v] : 0.f;
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < RED_MAX_BLOCKS / RED_GROUP; ++i) acc += (double)x[i];
    tot[v] = acc;
  }
  __syncthreads();
  return true;
}

// Per-thread row loop over [M, C] bf16 rows: thread owns channel group cg
// and rows r0, r0 + rstride, ...; four 16-byte loads in flight per stream.
#define MDA_ROW_LOOP(...)                                                    \
  {                                                                          \
    const int rstride = gridDim.x * rpi;                                     \
    int m = blockIdx.x * rpi + r0;                                           \
    for (; m + 3 * rstride < M; m += 4 * rstride) {                          \
      _Pragma("unroll") for (int u = 0; u < 4; ++u) {                        \
        const int64_t o = (int64_t)(m + u * rstride) * C + cg * 8;           \
        __VA_ARGS__                                                          \
      }                                                                      \
    }                                                                        \
    for (; m < M; m += rstride) {                                            \
      const int64_t o = (int64_t)m * C + cg * 8;                             \
      __VA_ARGS__                                                            \
    }                                                                        \
  }

__global__ void __launch_bounds__(256)
bn_stats_kernel(const bf16_t* __restrict__ y, int M, int C, float* __restrict__ partial,
                unsigned* __restrict__ counter, const float* __restrict__ gamma,
                const float* __restrict__ beta, float* __restrict__ running_mean,
                float* __restrict__ running_var, float* __restrict__ mean_out,
                float* __restrict__ rstd_out, float* __restrict__ scale_out,
                float* __restrict__ shift_out, float momentum, float eps,
                int64_t* __restrict__ nbt) {
  const int C8 = C / 8;
  const int rpi = 256 / C8;  // rows per block-iteration
  const int cg = threadIdx.x % C8, r0 = threadIdx.x / C8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ss[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (r0 < rpi) {
    MDA_ROW_LOOP({
      const uint4 v = *(const uint4*)(y + o);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
_Pragma("unroll")
      for (int k = 0; k < 4; ++k) {
        const float f0 = __uint_as_float(w[k] << 16), f1 = __uint_as_float(w[k] & 0xffff0000u);
        s[2 * k] += f0; ss[2 * k] += f0 * f0;
        s[2 * k + 1] += f1; ss[2 * k + 1] += f1 * f1;
      }
    })
  }
  block_channel_partials(s, ss, C, rpi, partial);
  if (counter == nullptr) return;  // partials only; bn_finalize_kernel combines
  __shared__ double tot[2 * 2048];
  if (combine_partials(partial, 2 * C, counter, tot)) {
    if (threadIdx.x == 0 && nbt) nbt[0] += 1;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      const double mean = tot[c] / M;
      double var = tot[C + c] / M - mean * mean;
      if (var < 0) var = 0;
      const float rstd = (float)(1.0 / sqrt(var + (double)eps));
      const float g = gamma ? gamma[c] : 1.f;
      const float bb = beta ? beta[c] : 0.f;
      mean_out[c] = (float)mean;
      rstd_out[c] = rstd;
      scale_out[c] = g * rstd;
      shift_out[c] = bb - (float)mean * g * rstd;
      if (running_mean) {
        const double unbiased = M > 1 ? var * M / (M - 1) : var;
        running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unbiased;
      }
    }
  }
}

// 8 channels (16 bytes) per thread-iteration; C % 8 == 0.
__global__ void __launch_bounds__(256)
bn_apply_kernel(const bf16_t* __restrict__ y, const float* __restrict__ scale,
                const float* __restrict__ shift, const bf16_t* __restrict__ res,
                bf16_t* __restrict__ out, bf16_t* __restrict__ preact, int64_t M, int C, int act) {
  const int64_t total = M * C / 8;
  const int c8 = C / 8;
  // the grid stride is a multiple of C/8 (both powers of two or the launch
  // makes it so), so every thread keeps one channel group: load its params once
  const int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int c0 = (int)(i0 % c8) * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { sc[k] = scale[c0 + k]; sh[k] = shift[c0 + k]; }
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool fixed = (stride % c8) == 0;
  for (int64_t i = i0; i < total; i += stride) {
    if (!fixed) {
      const int cc = (int)(i % c8) * 8;
#pragma unroll
      for (int k = 0; k < 8; ++k) { sc[k] = scale[cc + k]; sh[k] = shift[cc + k]; }
    }
    uint4 yv = ((const uint4*)y)[i];
    uint4 rv = res ? ((const uint4*)res)[i] : make_uint4(0, 0, 0, 0);
    const bf16_t* yp = (const bf16_t*)&yv;
    const bf16_t* rp = (const bf16_t*)&rv;
    bf16_t o[8], z[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = bf2f(yp[k]) * sc[k] + sh[k];
      if (res) v += bf2f(rp[k]);
      z[k] = f2bf(v);
      o[k] = f2bf(act_f(v, act));
    }
    ((uint4*)out)[i] = *(uint4*)o;
    if (preact) ((uint4*)preact)[i] = *(uint4*)z;
  }
}

// dz = dout * act'(z) (+ dpre); sums of dz and dz*xhat per channel.
// z is recovered from y: z = y*scale + shift (+ res), so the ReLU mask needs
// no stored pre-activation.
__global__ void __launch_bounds__(256)
bn_bwd_reduce_kernel(const bf16_t* __restrict__ dout, const bf16_t* __restrict__ dpre,
                     const bf16_t* __restrict__ y, const bf16_t* __restrict__ res,
                     const float* __restrict__ scale, const float* __restrict__ shift,
                     const float* __restrict__ mean, const float* __restrict__ rstd, int M, int C,
                     int act, float* __restrict__ partial, unsigned* __restrict__ counter,
                     float* __restrict__ sums, float* __restrict__ dgamma,
                     float* __restrict__ dbeta) {
  const int C8 = C / 8;
  const int rpi = 256 / C8;
  const int cg = threadIdx.x % C8, r0 = threadIdx.x / C8;
  float sdz[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sdzx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (r0 < rpi) {
    float sc[8], sh[8], mu[8], rs[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = cg * 8 + k;
      sc[k] = scale[c]; sh[k] = shift[c]; mu[k] = mean[c]; rs[k] = rstd[c];
    }
    MDA_ROW_LOOP({
      uint4 yv = *(const uint4*)(y + o);
      uint4 dv = dout ? *(const uint4*)(dout + o) : make_uint4(0, 0, 0, 0);
      uint4 pv = dpre ? *(const uint4*)(dpre + o) : make_uint4(0, 0, 0, 0);
      uint4 rv = (res && act != ACT_NONE) ? *(const uint4*)(res + o) : make_uint4(0, 0, 0, 0);
      const bf16_t* ye = (const bf16_t*)&yv;
      const bf16_t* de = (const bf16_t*)&dv;
      const bf16_t* pe = (const bf16_t*)&pv;
      const bf16_t* re = (const bf16_t*)&rv;
_Pragma("unroll")
      for (int k = 0; k < 8; ++k) {
        const float yf = bf2f(ye[k]);
        float dz = bf2f(de[k]);
        if (act != ACT_NONE) {
          float z = yf * sc[k] + sh[k];
          if (res) z += bf2f(re[k]);
          dz *= act_grad(z, act);
        }
        if (dpre) dz += bf2f(pe[k]);
        sdz[k] += dz;
        sdzx[k] += dz * (yf - mu[k]) * rs[k];
      }
    })
  }
  block_channel_partials(sdz, sdzx, C, rpi, partial);
  if (counter == nullptr) return;  // partials only; bn_finalize_kernel combines
  __shared__ double tot[2 * 2048];
  if (combine_partials(partial, 2 * C, counter, tot)) {
    for (int t = threadIdx.x; t < 2 * C; t += blockDim.x) {
      const int q = t / C, c = t - q * C;
      const float v = (float)tot[t];
      sums[t] = v;  // [0, C): sum dz (= dbeta), [C, 2C): sum dz*xhat (= dgamma)
      if (q == 0 && dbeta) dbeta[c] += v;
      if (q == 1 && dgamma) dgamma[c] += v;
    }
  }
}

__global__ void __launch_bounds__(256)
bn_bwd_apply_kernel(const bf16_t* __restrict__ dout, const bf16_t* __restrict__ dpre,
                    const bf16_t* __restrict__ y, const bf16_t* __restrict__ res,
                    const float* __restrict__ scale, const float* __restrict__ shift,
                    const float* __restrict__ mean, const float* __restrict__ rstd,
                    const float* __restrict__ sums, bf16_t* __restrict__ dy,
                    bf16_t* __restrict__ dres, int64_t M, int C, int act) {
  const int64_t total = M * C / 8;
  const int c8 = C / 8;
  const float invM = 1.f / (float)M;
  const int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int c0 = (int)(i0 % c8) * 8;
  float sc[8], sh[8], mu[8], rs[8], s0[8], s1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = c0 + k;
    sc[k] = scale[c]; sh[k] = shift[c]; mu[k] = mean[c]; rs[k] = rstd[c];
    s0[k] = sums[c] * invM; s1[k] = sums[C + c] * invM;
  }
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool fixed = (stride % c8) == 0;
  for (int64_t i = i0; i < total; i += stride) {
    if (!fixed) {
      const int cc = (int)(i % c8) * 8;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = cc + k;
        sc[k] = scale[c]; sh[k] = shift[c]; mu[k] = mean[c]; rs[k] = rstd[c];
        s0[k] = sums[c] * invM; s1[k] = sums[C + c] * invM;
      }
    }
    uint4 yv = ((const uint4*)y)[i];
    uint4 dv = dout ? ((const uint4*)dout)[i] : make_uint4(0, 0, 0, 0);
    uint4 pv = dpre ? ((const uint4*)dpre)[i] : make_uint4(0, 0, 0, 0);
    uint4 rv = (res && act != ACT_NONE) ? ((const uint4*)res)[i] : make_uint4(0, 0, 0, 0);
    const bf16_t* yp = (const bf16_t*)&yv;
    const bf16_t* dp = (const bf16_t*)&dv;
    const bf16_t* pp = (const bf16_t*)&pv;
    const bf16_t* rp = (const bf16_t*)&rv;
    bf16_t o[8], r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float yf = bf2f(yp[k]);
      float dz = bf2f(dp[k]);
      if (act != ACT_NONE) {
        float z = yf * sc[k] + sh[k];
        if (res) z += bf2f(rp[k]);
        dz *= act_grad(z, act);
      }
      if (dpre) dz += bf2f(pp[k]);
      const float xhat = (yf - mu[k]) * rs[k];
      const float g = sc[k] * (dz - (s0[k] + xhat * s1[k]));
      o[k] = f2bf(g);
      r[k] = f2bf(dz);
    }
    ((uint4*)dy)[i] = *(uint4*)o;
    if (dres) ((uint4*)dres)[i] = *(uint4*)r;
  }
}

// Channel-parallel combine of the per-block partials partial[nblk][2C]:
// block b owns channels [8b, 8b+8); thread (v = tid % 16, g = tid / 16)
// sums rows g, g+16, ... of value v in fp64, then the 16 row groups are
// added in fixed order -- deterministic, no atomics, no cross-block hand-off.
// MODE 0: forward statistics (mean, rstd, scale, shift, running stats);
// MODE 1: backward sums (dbeta = sum dz, dgamma = sum dz*xhat).
template <int MODE>
__global__ void __launch_bounds__(256)
bn_finalize_kernel(const float* __restrict__ partial, int nblk, int M, int C,
                   const float* __restrict__ gamma, const float* __restrict__ beta,
                   float* __restrict__ running_mean, float* __restrict__ running_var,
                   float* __restrict__ mean_out, float* __restrict__ rstd_out,
                   float* __restrict__ scale_out, float* __restrict__ shift_out, float momentum,
                   float eps, int64_t* __restrict__ nbt, float* __restrict__ sums,
                   float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ double red[16][17];
  const int v = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int q = v >> 3, k = v & 7;
  const int c = blockIdx.x * 8 + k;
  double acc = 0.0;
  if (c < C) {
    // 8 independent loads in flight per round: a 512-row partial is 4 L2
    // round trips per thread instead of 8 (the finalize is latency-bound)
    const float* src = partial + q * C + c;
    float x[8];
    int r = g;
    for (; r + 112 < nblk; r += 128) {
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = src[(int64_t)(r + 16 * u) * 2 * C];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += (double)x[u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = r + 16 * u < nblk ? src[(int64_t)(r + 16 * u) * 2 * C] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += (double)x[u];  // + 0.0 is exact
  }
  red[g][v] = acc;
  __syncthreads();
  if (threadIdx.x >= 8) return;
  const int ch = blockIdx.x * 8 + threadIdx.x;
  if (ch >= C) return;
  double t0 = 0.0, t1 = 0.0;
  for (int i = 0; i < 16; ++i) {
    t0 += red[i][threadIdx.x];
    t1 += red[i][8 + threadIdx.x];
  }
  if (MODE == 0) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) nbt[0] += 1;
    const double mean = t0 / M;
    double var = t1 / M - mean * mean;
    if (var < 0) var = 0;
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    const float gm = gamma ? gamma[ch] : 1.f;
    const float bb = beta ? beta[ch] : 0.f;
    mean_out[ch] = (float)mean;
    rstd_out[ch] = rstd;
    scale_out[ch] = gm * rstd;
    shift_out[ch] = bb - (float)mean * gm * rstd;
    if (running_mean) {
      const double unbiased = M > 1 ? var * M / (M - 1) : var;
      running_mean[ch] = (1.f - momentum) * running_mean[ch] + momentum * (float)mean;
      running_var[ch] = (1.f - momentum) * running_var[ch] + momentum * (float)unbiased;
    }
  } else {
    sums[ch] = (float)t0;
    sums[C + ch] = (float)t1;
    if (dbeta) dbeta[ch] += (float)t0;
    if (dgamma) dgamma[ch] += (float)t1;
  }
}

int g_red_vpt = 8;       // sixteen-byte vectors per thread in the reduction kernels
int g_red_max = RED_MAX_BLOCKS;

inline int reduce_blocks(int64_t M, int64_t C, int vpt = 0, int max_blocks = 0) {
  // ~vpt sixteen-byte vectors per thread (issued 4 at a time)
  if (vpt <= 0) vpt = g_red_vpt;
  if (max_blocks <= 0) max_blocks = g_red_max;
  int64_t b = (M * (C / 8) + 256 * vpt - 1) / (256 * vpt);
  if (b < 1) b = 1;
  if (b > max_blocks) b = max_blocks;
  return (int)b;
}

// Measured on MI355X (scripts/bn_microbench.py, student shapes): the stats
// pass is load-bound and best at 8 vectors/thread; the backward reduce does
// ~3x the math per vector and is best at 4 vectors/thread (up to 512 blocks).
constexpr int STATS2_VPT = 8, STATS2_MAXB = 256;
constexpr int BWD2_VPT = 4, BWD2_MAXB = 512;
constexpr int RED2_MAX_BLOCKS = 512;  // workspace sizing: partial >= 2*C*512 floats

inline int ew_blocks(int64_t n8) {
  // power of two, so the grid stride is a multiple of C/8 (hoisted per-channel params)
  int64_t want = (n8 + 255) / 256;
  int64_t b = 1;
  while (b < want && b < 2048) b <<= 1;
  return (int)b;
}

}  // namespace

// Workspace: partial >= 2*C*(256+16) floats; counter: 17 zeroed uints.  C % 8 == 0, C <= 2048.
MDA_API int mda_bn_stats(const void* y, int64_t M, int64_t C, float* partial, unsigned* counter,
                         const float* gamma, const float* beta, float* running_mean,
                         float* running_var, float* mean, float* rstd, float* scale,
                         float* shift, float momentum, float eps, int64_t* nbt,
                         hipStream_t st) {
  if (C % 8 || C / 8 > 256 || C > 2048) return (int)hipErrorInvalidValue;
  dim3 grid(reduce_blocks(M, C));
  hipLaunchKernelGGL(bn_stats_kernel, grid, dim3(256), 0, st, (const bf16_t*)y, (int)M, (int)C,
                     partial, counter, gamma, beta, running_mean, running_var, mean, rstd, scale,
                     shift, momentum, eps, nbt);
  MDA_CHECK_LAUNCH();
}

MDA_API int mda_bn_apply(const void* y, const float* scale, const float* shift, const void* res,
                         void* out, void* preact, int64_t M, int64_t C, int64_t act,
                         hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_apply_kernel, dim3(ew_blocks(M * C / 8)), dim3(256), 0, st,
                     (const bf16_t*)y, scale, shift, (const bf16_t*)res, (bf16_t*)out,
                     (bf16_t*)preact, M, (int)C, (int)act);
  MDA_CHECK_LAUNCH();
}

// sums: 2*C floats out (sum dz, sum dz*xhat); dgamma/dbeta accumulated (may be null).
MDA_API int mda_bn_bwd_reduce(const void* dout, const void* dpre, const void* y, const void* res,
                              const float* scale, const float* shift, const float* mean,
                              const float* rstd, int64_t M, int64_t C, int64_t act,
                              float* partial, unsigned* counter, float* sums, float* dgamma,
                              float* dbeta, hipStream_t st) {
  if (C % 8 || C / 8 > 256 || C > 2048) return (int)hipErrorInvalidValue;
  dim3 grid(reduce_blocks(M, C));
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, grid, dim3(256), 0, st, (const bf16_t*)dout,
                     (const bf16_t*)dpre, (const bf16_t*)y, (const bf16_t*)res, scale, shift,
                     mean, rstd, (int)M, (int)C, (int)act, partial, counter, sums, dgamma, dbeta);
  MDA_CHECK_LAUNCH();
}

MDA_API int mda_bn_bwd_apply(const void* dout, const void* dpre, const void* y, const void* res,
                             const float* scale, const float* shift, const float* mean,
                             const float* rstd, const float* sums, void* dy, void* dres,
                             int64_t M, int64_t C, int64_t act, hipStream_t st) {
  if (C % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(ew_blocks(M * C / 8)), dim3(256), 0, st,
                     (const bf16_t*)dout, (const bf16_t*)dpre, (const bf16_t*)y,
                     (const bf16_t*)res, scale, shift, mean, rstd, sums, (bf16_t*)dy,
                     (bf16_t*)dres, M, (int)C, (int)act);
  MDA_CHECK_LAUNCH();
}

// Tuning hook (microbenchmarks): vectors per thread and max blocks of the
// reduction kernels.  The in-kernel hand-off variants require max <= 256.
MDA_API int mda_bn_tune(int64_t vpt, int64_t max_blocks) {
  if (vpt < 1 || max_blocks < 1 || max_blocks > 4096) return (int)hipErrorInvalidValue;
  g_red_vpt = (int)vpt;
  g_red_max = (int)max_blocks;
  return 0;
}

// Two-launch variants (the training path): partials kernel (no in-kernel
// hand-off) + channel-parallel finalize.  2-3x faster than the single-launch
// last-arriver combine at batch 64 (the agent-scope release/acquire hand-off
// serialises two L2 round trips into every call).  Workspace: partial >=
// 2*C*512 floats; no counters.
MDA_API int mda_bn_stats2(const void* y, int64_t M, int64_t C, float* partial,
                          const float* gamma, const float* beta, float* running_mean,
                          float* running_var, float* mean, float* rstd, float* scale,
                          float* shift, float momentum, float eps, int64_t* nbt,
                          hipStream_t st) {
  if (C % 8 || C / 8 > 256 || C > 2048) return (int)hipErrorInvalidValue;
  const int nblk = reduce_blocks(M, C, STATS2_VPT, STATS2_MAXB);
  hipLaunchKernelGGL(bn_stats_kernel, dim3(nblk), dim3(256), 0, st, (const bf16_t*)y, (int)M,
                     (int)C, partial, (unsigned*)nullptr, gamma, beta, running_mean, running_var,
                     mean, rstd, scale, shift, momentum, eps, nbt);
  hipLaunchKernelGGL(bn_finalize_kernel<0>, dim3((unsigned)((C + 7) / 8)), dim3(256), 0, st,
                     partial, nblk, (int)M, (int)C, gamma, beta, running_mean, running_var, mean,
                     rstd, scale, shift, momentum, eps, nbt, (float*)nullptr, (float*)nullptr,
                     (float*)nullptr);
  MDA_CHECK_LAUNCH();
}

MDA_API int mda_bn_bwd_reduce2(const void* dout, const void* dpre, const void* y, const void* res,
                               const float* scale, const float* shift, const float* mean,
                               const float* rstd, int64_t M, int64_t C, int64_t act,
                               float* partial, float* sums, float* dgamma, float* dbeta,
                               hipStream_t st) {
  if (C % 8 || C / 8 > 256 || C > 2048) return (int)hipErrorInvalidValue;
  const int nblk = reduce_blocks(M, C, BWD2_VPT, BWD2_MAXB);
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(nblk), dim3(256), 0, st, (const bf16_t*)dout,
                     (const bf16_t*)dpre, (const bf16_t*)y, (const bf16_t*)res, scale, shift,
                     mean, rstd, (int)M, (int)C, (int)act, partial, (unsigned*)nullptr, sums,
                     dgamma, dbeta);
  hipLaunchKernelGGL(bn_finalize_kernel<1>, dim3((unsigned)((C + 7) / 8)), dim3(256), 0, st,
                     partial, nblk, (int)M, (int)C, (const float*)nullptr, (const float*)nullptr,
                     (float*)nullptr, (float*)nullptr, (float*)nullptr, (float*)nullptr,
                     (float*)nullptr, (float*)nullptr, 0.f, 0.f, (int64_t*)nullptr, sums, dgamma,
                     dbeta);
  MDA_CHECK_LAUNCH();
}

// Channel-parallel finalize of externally produced statistics partials
// partial[nblk][2][C] (the conv epilogue's, csrc/conv_igemm.hip).
MDA_API int mda_bn_finalize(const float* partial, int64_t nblk, int64_t M, int64_t C,
                            const float* gamma, const float* beta, float* running_mean,
                            float* running_var, float* mean, float* rstd, float* scale,
                            float* shift, float momentum, float eps, int64_t* nbt,
                            hipStream_t st) {
  if (C % 8 || C > 2048 || nblk <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_finalize_kernel<0>, dim3((unsigned)((C + 7) / 8)), dim3(256), 0, st,
                     partial, (int)nblk, (int)M, (int)C, gamma, beta, running_mean, running_var,
                     mean, rstd, scale, shift, momentum, eps, nbt, (float*)nullptr,
                     (float*)nullptr, (float*)nullptr);
  MDA_CHECK_LAUNCH();
}

// ===========================================================================
// Fused training BN (round 3): channel sums through a one-shot BnRegion
// (csrc/bnslot.h) instead of partial rows + a finalize launch.
//
//   forward   conv (epilogue adds the block's sum y / sum y^2 into the region,
//             conv_igemm.hip mda_conv_fwd_bnacc)  or  bn_stats_acc_kernel
//             -> bn_apply_fin_kernel: every block finalizes the channels
//                from the region in its prologue (block 0 also writes mean /
//                rstd / scale / shift for the backward and the running stats),
//                applies z = y*scale + shift (+ res), act, preact.  2 launches
//   backward  bn_bwd_fused_kernel: dz = (dout + dout2) * act'(z) (+ dpre),
//             block sums -> region, grid barrier (<= 1 block per CU, resident
//             by construction), every block reads the totals, block 0
//             accumulates dgamma / dbeta into the flat gradient, then
//             dy = scale*(dz - (sum dz + xhat*sum dz*xhat)/M), dres = dz from
//             the values still in registers (HOLD) or re-read.  1 launch
//
// versus 3 forward (conv, finalize, apply) + 3 backward (reduce, finalize,
// apply) launches per layer before; dout2 folds the gradient add of a
// residual fork (two consumers of one activation) into the same pass.
#include "bnslot.h"
#include "bnbwd.h"
#include <cstdlib>

namespace {

// Block sums a[8], b[8] of the thread's channel group -> region shard.
__device__ __forceinline__ void region_block_add(BnRegion* r, float (&a)[8], float (&b)[8], int C,
                                                 int rpi) {
  __shared__ float sm[2][256 * 8];
  const int tid = threadIdx.x;
  const int C8 = C / 8;
  const int cg = tid % C8, r0 = tid / C8;
  if (r0 < rpi) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sm[0][r0 * C + cg * 8 + k] = a[k];
      sm[1][r0 * C + cg * 8 + k] = b[k];
    }
  }
  __syncthreads();
  const int shard = blockIdx.x % slot_shards(C);
  for (int t = tid; t < 2 * C; t += blockDim.x) {
    const int q = t / C, c = t - q * C;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int rr = 0;
    for (; rr + 4 <= rpi; rr += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += sm[q][(rr + u) * C + c];
    }
    for (; rr < rpi; ++rr) acc[0] += sm[q][rr * C + c];
    acc_add(region_acc(r, C, shard, q) + c, (double)((acc[0] + acc[1]) + (acc[2] + acc[3])));
  }
}

// Standalone statistics pass (y already materialised: depthwise convs,
// split-K convs, pre-activation BN): sums into the region, no finalize.
__global__ void __launch_bounds__(256)
bn_stats_acc_kernel(const bf16_t* __restrict__ y, int M, int C, BnRegion* __restrict__ reg) {
  const int C8 = C / 8;
  const int rpi = 256 / C8;
  const int cg = threadIdx.x % C8, r0 = threadIdx.x / C8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ss[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (r0 < rpi) {
    MDA_ROW_LOOP({
      const uint4 v = *(const uint4*)(y + o);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
_Pragma("unroll")
      for (int k = 0; k < 4; ++k) {
        const float f0 = __uint_as_float(w[k] << 16), f1 = __uint_as_float(w[k] & 0xffff0000u);
        s[2 * k] += f0; ss[2 * k] += f0 * f0;
        s[2 * k + 1] += f1; ss[2 * k + 1] += f1 * f1;
      }
    })
  }
  region_block_add(reg, s, ss, C, rpi);
}

// z = y*scale + shift (+ res); out = act(z); preact = z -- with the finalize
// of the region's sums in the prologue.  Grid stride is a multiple of C/8
// when C/8 is a power of two (power-of-two grid) so every thread keeps one
// channel group.



// z = y*scale + shift (+ res); out = act(z); preact = z -- with the finalize
// of the region's sums in the prologue.  The thread's V vectors of y
// (and res) are loaded BEFORE the prologue, so their latency overlaps the
// region loads; grids past V vectors per thread loop.
// rreg != null: `res` is the RAW output of another training conv whose BN
// (no activation: a projection shortcut) is applied here too -- its batch
// statistics are finalized from rreg in the same prologue (rf: its affine,
// running stats and [4][C] stats) and res contributes res*rscale + rshift, so
// that BN never runs an apply pass of its own.
// The per-channel operands live in dynamic LDS sized to C (2C or 4C floats):
// a static SLOT_CMAX-channel array held 16-32 KB whatever the layer's width.
// V = 16-byte vectors per thread (apply_vpt).
template <int V>
__global__ void __launch_bounds__(256)
bn_apply_fin_kernel(const bf16_t* __restrict__ y, BnRegion* __restrict__ reg, int64_t M, int C,
                    FinArgs f, const bf16_t* __restrict__ res, bf16_t* __restrict__ out,
                    bf16_t* __restrict__ preact, int act, BnRegion* __restrict__ rreg, FinArgs rf) {
  extern __shared__ float s_dyn[];
  bn_apply_fin_body<V>(FwdApply{y, reg, M, C, f, res, out, preact, act, rreg, rf}, s_dyn,
                       (int)blockIdx.x, (int)gridDim.x);
}

template <int VPT, bool HOLD>
__global__ void __launch_bounds__(256)
bn_bwd_fused_kernel(BwdArgs a) {
  dual_shift(a, blockIdx.y);
  __shared__ float s_m0[SLOT_CMAX], s_m1[SLOT_CMAX];
  const int C = a.C, M = a.M;
  const int C8 = C / 8;
  const int rpi = 256 / C8;
  const int cg = threadIdx.x % C8, r0 = threadIdx.x / C8;
  const bool active = r0 < rpi;
  const int c0 = cg * 8;
  float sc[8], sh[8], mu[8], rs[8], vsc[8], vsh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu[k] = a.stats[c0 + k]; rs[k] = a.stats[C + c0 + k];
    sc[k] = a.stats[2 * C + c0 + k]; sh[k] = a.stats[3 * C + c0 + k];
    vsc[k] = a.vres ? a.vres[2 * C + c0 + k] : 1.f;
    vsh[k] = a.vres ? a.vres[3 * C + c0 + k] : 0.f;
  }
  const int rstride = gridDim.x * rpi;
  float sdz[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sdzx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float hz[HOLD ? VPT : 1][8];
  uint4 hy[HOLD ? VPT : 1];
  auto accum = [&](const float (&dz)[8], const uint4& yv) {
    const uint32_t yw[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float yf = (e & 1) ? __uint_as_float(yw[e >> 1] & 0xffff0000u) : __uint_as_float(yw[e >> 1] << 16);
      sdz[e] += dz[e];
      sdzx[e] += dz[e] * (yf - mu[e]) * rs[e];
    }
  };
  if (HOLD) {
    // every load of the thread's rows in flight before any math
    Raw8 raw[HOLD ? VPT : 1];
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int m = blockIdx.x * rpi + r0 + k * rstride;
      const bool ok = active && m < M;
      bwd_load8(a, (int64_t)(ok ? m : 0) * C + c0, raw[k]);
    }
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int m = blockIdx.x * rpi + r0 + k * rstride;
      hy[k] = raw[k].y;
      if (active && m < M) {
        bwd_dz8(a, raw[k], sc, sh, hz[k], vsc, vsh);
        accum(hz[k], hy[k]);
      }
    }
  } else if (active) {
    int m = blockIdx.x * rpi + r0;
    for (; m + rstride < M; m += 2 * rstride) {
      Raw8 v0, v1;
      bwd_load8(a, (int64_t)m * C + c0, v0);
      bwd_load8(a, (int64_t)(m + rstride) * C + c0, v1);
      float dz[8];
      bwd_dz8(a, v0, sc, sh, dz, vsc, vsh);
      accum(dz, v0.y);
      bwd_dz8(a, v1, sc, sh, dz, vsc, vsh);
      accum(dz, v1.y);
    }
    if (m < M) {
      Raw8 v0;
      bwd_load8(a, (int64_t)m * C + c0, v0);
      float dz[8];
      bwd_dz8(a, v0, sc, sh, dz, vsc, vsh);
      accum(dz, v0.y);
    }
  }
  region_block_add(a.reg, sdz, sdzx, C, rpi);
  region_grid_barrier(a.reg, a.err);
  {
    const float invM = 1.f / (float)M;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      double d0, d1;
      region_channel<true>(a.reg, C, c, d0, d1);
      const float t0 = (float)d0, t1 = (float)d1;
      s_m0[c] = t0 * invM;
      s_m1[c] = t1 * invM;
      if (blockIdx.x == 0) {
        if (a.sums) { a.sums[c] = t0; a.sums[C + c] = t1; }
        if (a.dbeta) a.dbeta[c] += t0;
        if (a.dgamma) a.dgamma[c] += t1;
      }
    }
  }
  __syncthreads();
  float m0[8], m1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { m0[k] = s_m0[c0 + k]; m1[k] = s_m1[c0 + k]; }
  float r1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, r2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto emit = [&](int m, const float (&dz)[8], const uint4& yv) {
    const int64_t o = (int64_t)m * C + c0;
    const uint32_t yw[4] = {yv.x, yv.y, yv.z, yv.w};
    uint32_t go[4], ro[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      float g[2], r[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = 2 * w + h;
        const float yf = h ? __uint_as_float(yw[w] & 0xffff0000u) : __uint_as_float(yw[w] << 16);
        const float xhat = (yf - mu[e]) * rs[e];
        g[h] = sc[e] * (dz[e] - (m0[e] + xhat * m1[e]));
        r[h] = dz[e];
      }
      go[w] = pack_bf16x2(g[0], g[1]);
      ro[w] = pack_bf16x2(r[0], r[1]);
    }
    *(uint4*)(a.dy + o) = make_uint4(go[0], go[1], go[2], go[3]);
    if (a.dres) *(uint4*)(a.dres + o) = make_uint4(ro[0], ro[1], ro[2], ro[3]);
    if (a.rreg) rsum_add8(a, o, c0, ro, r1, r2);
  };
  if (HOLD) {
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int m = blockIdx.x * rpi + r0 + k * rstride;
      if (active && m < M) emit(m, hz[k], hy[k]);
    }
  } else if (active) {
    for (int m = blockIdx.x * rpi + r0; m < M; m += rstride) {
      Raw8 v0;
      bwd_load8(a, (int64_t)m * C + c0, v0);
      float dz[8];
      bwd_dz8(a, v0, sc, sh, dz, vsc, vsh);
      emit(m, dz, v0.y);
    }
  }
  if (a.rreg) {
    __syncthreads();  // the phase-1 reduction's shared buffer is reused
    region_block_add(a.rreg, r1, r2, C, rpi);
  }
}

// BN-backward channel sums (sum dz, sum dz*xhat) of a large tensor into the
// region: as many blocks as the reduction wants (no grid barrier, so no
// one-block-per-CU cap); mda_bn_bwd_apply_reg follows.  Used instead of the
// grid-barrier kernel when its rows do not fit in registers: that kernel
// re-read y / dout with 4 waves per CU (70 us for a 64 x 112^2 x 64 layer).
__global__ void __launch_bounds__(256)
bn_bwd_sums_kernel(BwdArgs a) {
  dual_shift(a, blockIdx.y);
  const int C = a.C, M = a.M;
  const int C8 = C / 8;
  const int rpi = 256 / C8;
  const int cg = threadIdx.x % C8, r0 = threadIdx.x / C8;
  const int c0 = cg * 8;
  float sc[8], sh[8], mu[8], rs[8], vsc[8], vsh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu[k] = a.stats[c0 + k]; rs[k] = a.stats[C + c0 + k];
    sc[k] = a.stats[2 * C + c0 + k]; sh[k] = a.stats[3 * C + c0 + k];
    vsc[k] = a.vres ? a.vres[2 * C + c0 + k] : 1.f;
    vsh[k] = a.vres ? a.vres[3 * C + c0 + k] : 0.f;
  }
  float sdz[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sdzx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (r0 < rpi) {
    MDA_ROW_LOOP({
      Raw8 v;
      bwd_load8(a, o, v);
      float dz[8];
      bwd_dz8(a, v, sc, sh, dz, vsc, vsh);
      const uint32_t yw[4] = {v.y.x, v.y.y, v.y.z, v.y.w};
_Pragma("unroll")
      for (int e = 0; e < 8; ++e) {
        const float yf = (e & 1) ? __uint_as_float(yw[e >> 1] & 0xffff0000u) : __uint_as_float(yw[e >> 1] << 16);
        sdz[e] += dz[e];
        sdzx[e] += dz[e] * (yf - mu[e]) * rs[e];
      }
    })
  }
  region_block_add(a.reg, sdz, sdzx, C, rpi);
}

// BN backward whose channel sums a producer already added into the region
// (the dgrad epilogue of the consuming conv, conv_igemm.hip
// mda_conv_dgrad_bnsum): one streaming pass (bnbwd.h bn_bwd_apply_body).
template <int V>
__global__ void __launch_bounds__(256)
bn_bwd_apply_reg_kernel(BwdArgs a) {
  extern __shared__ float s_dyn[];
  dual_shift(a, blockIdx.y);
  bn_bwd_apply_body<V>(a, s_dyn, (int)blockIdx.x, (int)gridDim.x);
}

int g_num_cus = 0;

int num_cus() {
  if (g_num_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      g_num_cus = n;
    else
      g_num_cus = 256;
  }
  return g_num_cus;
}


// Vectors per thread of a streaming apply launch.  Fewer vectors and more
// blocks for small layers (>= 2 blocks per CU) measured the same on the
// flagship and 2 % slower on R50 -> MV1 (profiles/r6_ab.md): kept at 4.
inline int apply_vpt(int64_t) { return 4; }

template <typename... A>
int launch_apply_fin(int v, dim3 g, size_t lds, hipStream_t st, A... args) {
  if (v != 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_apply_fin_kernel<4>, g, dim3(256), lds, st, args...);
  return (int)hipGetLastError();
}

int launch_bwd_apply(int v, dim3 g, int C, hipStream_t st, const BwdArgs& a) {
  if (v != 4) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)bn_apply_lds_bytes(C, 256, a.rreg != nullptr);
  hipLaunchKernelGGL(bn_bwd_apply_reg_kernel<4>, g, dim3(256), lds, st, a);
  return (int)hipGetLastError();
}

}  // namespace

// Bytes of the (zeroed, 64-byte aligned) region one BN call needs.
MDA_API int mda_bn_region_bytes(int64_t C, int64_t* out) {
  if (C <= 0 || C % 8 || C > SLOT_CMAX) return (int)hipErrorInvalidValue;
  *out = region_bytes((int)C);
  return 0;
}

MDA_API int mda_bn_stats_acc(const void* y, int64_t M, int64_t C, void* region, hipStream_t st) {
  if (C % 8 || C > SLOT_CMAX || M <= 0 || M >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  const int nblk = reduce_blocks(M, C, STATS2_VPT, STATS2_MAXB);
  hipLaunchKernelGGL(bn_stats_acc_kernel, dim3(nblk), dim3(256), 0, st, (const bf16_t*)y, (int)M,
                     (int)C, (BnRegion*)region);
  MDA_CHECK_LAUNCH();
}

MDA_API int mda_bn_apply_fin_vr(const void* y, void* region, int64_t M, int64_t C, const float* gamma,
                                const float* beta, float* running_mean, float* running_var,
                                float* stats, float momentum, float eps, int64_t* nbt,
                                const void* res, void* out, void* preact, int64_t act,
                                void* rregion, const float* rgamma, const float* rbeta,
                                float* rrunning_mean, float* rrunning_var, float* rstats,
                                float rmomentum, float reps, int64_t* rnbt, hipStream_t st) {
  if (C % 8 || C > SLOT_CMAX || M <= 0 || M >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  if (rregion != nullptr && (res == nullptr || rstats == nullptr)) return (int)hipErrorInvalidValue;
  FinArgs f{gamma, beta, running_mean, running_var, stats, momentum, eps, nbt};
  FinArgs rf{rgamma, rbeta, rrunning_mean, rrunning_var, rstats, rmomentum, reps, rnbt};
  const int v = apply_vpt(M * C / 8);
  const int nb = apply_blocks(M * C / 8, v);
  const size_t lds = (size_t)(rregion != nullptr ? 4 : 2) * C * sizeof(float);
  return launch_apply_fin(v, dim3(nb), lds, st, (const bf16_t*)y, (BnRegion*)region, M, (int)C, f,
                          (const bf16_t*)res, (bf16_t*)out, (bf16_t*)preact, (int)act,
                          (BnRegion*)rregion, rf);
}

MDA_API int mda_bn_apply_fin(const void* y, void* region, int64_t M, int64_t C, const float* gamma,
                             const float* beta, float* running_mean, float* running_var,
                             float* stats, float momentum, float eps, int64_t* nbt,
                             const void* res, void* out, void* preact, int64_t act,
                             hipStream_t st) {
  return mda_bn_apply_fin_vr(y, region, M, C, gamma, beta, running_mean, running_var, stats, momentum,
                             eps, nbt, res, out, preact, act, nullptr, nullptr, nullptr, nullptr,
                             nullptr, nullptr, 0.f, 0.f, nullptr, st);
}

// Fused BN backward (one launch) on a fresh (zeroed) region.  dout2
// (optional) is a second gradient of the BN output added to dout (residual
// fork); sums (optional) receives [sum dz | sum dz*xhat]; dgamma / dbeta
// (optional) are accumulated; err (optional) is set on a barrier timeout.
MDA_API int mda_bn_bwd_fused(const void* dout, const void* dout2, const void* dpre, const void* y,
                             const void* res, const float* stats, int64_t M, int64_t C,
                             int64_t act, void* region, void* err, void* dy, void* dres,
                             float* dgamma, float* dbeta, float* sums, const void* ry,
                             const float* rstats, void* rregion, const float* vres,
                             int64_t nsets, int64_t dd, int64_t dg, int64_t dr, hipStream_t st) {
  if (C % 8 || C > SLOT_CMAX || M <= 0 || M >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  if (rregion != nullptr && (dres == nullptr || ry == nullptr || rstats == nullptr ||
                             256 % (C / 8) != 0))
    return (int)hipErrorInvalidValue;
  if (nsets != 1 && (nsets != 2 || dr <= 0)) return (int)hipErrorInvalidValue;
  BwdArgs a{(const bf16_t*)dout, (const bf16_t*)dout2, (const bf16_t*)dpre, (const bf16_t*)y,
            (const bf16_t*)res, stats, (bf16_t*)dy, (bf16_t*)dres, dgamma, dbeta, sums,
            (BnRegion*)region, (unsigned*)err, (int)M, (int)C, (int)act, (const bf16_t*)ry,
            rstats, (BnRegion*)rregion, vres, dd, dg, dr};
  const int C8 = (int)C / 8;
  const int rpi = 256 / C8;
  const int64_t rows_iter = (M + rpi - 1) / rpi;       // block-iterations of work
  // at most one block per CU over BOTH sets: every block of each set's grid
  // barrier is resident
  const int maxb = std::max(1, num_cus() / (int)nsets);
  // small layers hold >= p row iterations per thread on rows_iter / p blocks:
  // a grid barrier over fewer blocks.  MDA_BN_BWD_PER (default 4; measured
  // ShuffleV2 DOT 3.80 -> 3.60 ms, ShuffleV1 3.54 -> 3.48, flagship unchanged)
  static const int min_per = [] {
    const char* e = getenv("MDA_BN_BWD_PER");
    const int v = e ? atoi(e) : 4;
    return v < 1 ? 1 : (v > 8 ? 8 : v);
  }();
  const int nb = (int)std::min<int64_t>((rows_iter + min_per - 1) / min_per, maxb);
  const int64_t per = (rows_iter + nb - 1) / nb;     // row iterations per thread
  const unsigned ns = (unsigned)nsets;
  if (per > 8) {
    // too many rows to hold: sums with a full grid, then one streaming pass
    const int nbr = reduce_blocks(M, C, BWD2_VPT, BWD2_MAXB);
    hipLaunchKernelGGL(bn_bwd_sums_kernel, dim3(nbr, ns), dim3(256), 0, st, a);
    { const int rc_ = (int)hipGetLastError(); if (rc_) return rc_; }
    a.err = nullptr;
    const int v = apply_vpt(M * C / 8);
    return launch_bwd_apply(v, dim3(apply_blocks(M * C / 8, v), ns), (int)C, st, a);
  }
  if (per <= 1) hipLaunchKernelGGL((bn_bwd_fused_kernel<1, true>), dim3(nb, ns), dim3(256), 0, st, a);
  else if (per <= 2) hipLaunchKernelGGL((bn_bwd_fused_kernel<2, true>), dim3(nb, ns), dim3(256), 0, st, a);
  else if (per <= 4) hipLaunchKernelGGL((bn_bwd_fused_kernel<4, true>), dim3(nb, ns), dim3(256), 0, st, a);
  else if (per <= 8) hipLaunchKernelGGL((bn_bwd_fused_kernel<8, true>), dim3(nb, ns), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((bn_bwd_fused_kernel<1, false>), dim3(nb, ns), dim3(256), 0, st, a);
  MDA_CHECK_LAUNCH();
}

// BN backward on sums already in `region` (a dgrad epilogue produced them,
// conv_igemm.hip mda_conv_dgrad_bnsum): one streaming launch.
MDA_API int mda_bn_bwd_apply_reg(const void* dout, const void* dpre, const void* y, const void* res,
                                 const float* stats, int64_t M, int64_t C, int64_t act,
                                 void* region, void* dy, void* dres, float* dgamma, float* dbeta,
                                 float* sums, const void* ry, const float* rstats, void* rregion,
                                 const float* vres, int64_t nsets, int64_t dd, int64_t dg,
                                 int64_t dr, hipStream_t st) {
  if (C % 8 || C > SLOT_CMAX || M <= 0 || M >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  if (nsets != 1 && (nsets != 2 || dr <= 0)) return (int)hipErrorInvalidValue;
  BwdArgs a{(const bf16_t*)dout, nullptr, (const bf16_t*)dpre, (const bf16_t*)y,
            (const bf16_t*)res, stats, (bf16_t*)dy, (bf16_t*)dres, dgamma, dbeta, sums,
            (BnRegion*)region, nullptr, (int)M, (int)C, (int)act, (const bf16_t*)ry, rstats,
            (BnRegion*)rregion, vres, dd, dg, dr};
  if (rregion != nullptr && (dres == nullptr || ry == nullptr || rstats == nullptr ||
                             256 % (C / 8) != 0))
    return (int)hipErrorInvalidValue;  // a thread must keep one channel group
  const int v = apply_vpt(M * C / 8);
  return launch_bwd_apply(v, dim3(apply_blocks(M * C / 8, v), (unsigned)nsets), (int)C, st, a);
}
