// Implicit-GEMM convolution on CDNA4 MFMA (bf16 in, fp32 accumulate) with a
// fused per-channel epilogue (survey K1/K2):
//
//   y[m, co] = act( acc[m, co] * scale[co] + bias[co] + residual[m, co] )
//
// GEMM view (NHWC activations, "B^T" weights):
//   M = N*Ho*Wo output pixels, N = Cout, K = KH*KW*Cin
//   A[m, k]  = x[n, oh*s - p + kh, ow*s - p + kw, ci]   (zero outside the image)
//   B[k, co] = w_packed[co, k]  with k = (kh*KW + kw)*Cin + ci, rows padded to Kp = ceil32(K)
//
// With frozen BN folded into (w, bias) this is the whole teacher layer
// (conv + BN + residual add + ReLU) in ONE launch; the reference runs 4-5
// kernels per layer (cuDNN conv, BN, add, ReLU).  ``preact`` optionally also
// stores the pre-activation tensor (feature distillers consume it).
//
// Tiling: 256 threads = 4 waves as 2x2; block tile BM x BN x 32, wave tile
// (BM/2) x (BN/2) built from 16x16x32 bf16 MFMAs.  A/B K-slices are staged
// global -> VGPR -> LDS with a register prefetch of step s+1 while step s
// computes, two LDS buffers, one barrier per K-step.  LDS rows are 80 B
// (32 bf16 + 16 B pad) so the 16-lane groups of each ds_read_b128 fragment
// read hit 16 disjoint 4-bank slots (conflict-free).
//
// Loader modes: FAST (Cin % 32 == 0: each 32-wide K-slice is one filter tap),
// VEC8 (Cin % 8 == 0: every 16-byte chunk lies inside one tap), SCALAR (any
// Cin, e.g. the 3-channel stem).
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int BK = 32;
constexpr int LDS_ROW = 40;  // bf16 elements per LDS row (32 + 8 pad)

enum { LOAD_FAST = 0, LOAD_VEC8 = 1, LOAD_SCALAR = 2 };
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_RELU6 = 2 };

struct ConvParams {
  const bf16_t* x;       // [N, H, W, Cin]
  const bf16_t* w;       // [Cout, Kp]
  const float* scale;    // [Cout] or null
  const float* bias;     // [Cout] or null
  const bf16_t* res;     // [M, Cout] or null
  bf16_t* y;             // [M, Cout]
  bf16_t* preact;        // [M, Cout] or null
  int N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, K, Kp, M, act;
};

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == ACT_RELU) return fmaxf(v, 0.f);
  if (act == ACT_RELU6) return fminf(fmaxf(v, 0.f), 6.f);
  return v;
}

template <int BM, int BN, int MODE>
__global__ void __launch_bounds__(256)
conv_fwd_kernel(const ConvParams p) {
  constexpr int MI = BM / 32;  // 16-row MFMA tiles per wave (wave tile = BM/2 rows)
  constexpr int NI = BN / 32;
  constexpr int AROWS = BM / 64;  // A rows loaded per thread per K-step
  constexpr int BLOADS = (BN * 4 + 255) / 256;

  __shared__ __attribute__((aligned(16))) bf16_t As[2][BM][LDS_ROW];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][BN][LDS_ROW];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int chunk = tid & 3;
  const int HoWo = p.Ho * p.Wo;

  // per-thread A rows: pixel coordinates, resolved once
  int a_n[AROWS], a_ih0[AROWS], a_iw0[AROWS];
  bool a_ok[AROWS];
#pragma unroll
  for (int j = 0; j < AROWS; ++j) {
    int m = m0 + (tid >> 2) + 64 * j;
    a_ok[j] = m < p.M;
    int mm = a_ok[j] ? m : 0;
    int n = mm / HoWo;
    int r = mm - n * HoWo;
    int oh = r / p.Wo;
    int ow = r - oh * p.Wo;
    a_n[j] = n;
    a_ih0[j] = oh * p.stride - p.pad;
    a_iw0[j] = ow * p.stride - p.pad;
  }

  uint4 ra[AROWS];
  uint4 rb[BLOADS];
  const int nsteps = p.Kp / BK;
  const int cin_blocks = p.Cin / BK;  // FAST mode only

  auto load_step = [&](int s) {
    // ---- A ----
    if (MODE == LOAD_FAST) {
      const int tap = s / cin_blocks;
      const int c0 = (s - tap * cin_blocks) * BK + chunk * 8;
      const int kh = tap / p.KW, kw = tap - (tap / p.KW) * p.KW;
#pragma unroll
      for (int j = 0; j < AROWS; ++j) {
        int ih = a_ih0[j] + kh, iw = a_iw0[j] + kw;
        bool ok = a_ok[j] && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        if (ok) {
          const bf16_t* src = p.x + (((int64_t)a_n[j] * p.H + ih) * p.W + iw) * p.Cin + c0;
          ra[j] = *(const uint4*)src;
        } else {
          ra[j] = make_uint4(0, 0, 0, 0);
        }
      }
    } else if (MODE == LOAD_VEC8) {
      const int k0 = s * BK + chunk * 8;
      const int tap = k0 / p.Cin;
      const int c0 = k0 - tap * p.Cin;
      const int kh = tap / p.KW, kw = tap - (tap / p.KW) * p.KW;
      const bool kok = k0 < p.K;
#pragma unroll
      for (int j = 0; j < AROWS; ++j) {
        int ih = a_ih0[j] + kh, iw = a_iw0[j] + kw;
        bool ok = kok && a_ok[j] && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        if (ok) {
          const bf16_t* src = p.x + (((int64_t)a_n[j] * p.H + ih) * p.W + iw) * p.Cin + c0;
          ra[j] = *(const uint4*)src;
        } else {
          ra[j] = make_uint4(0, 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < AROWS; ++j) {
        bf16_t v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          int k = s * BK + chunk * 8 + e;
          int tap = k / p.Cin;
          int c = k - tap * p.Cin;
          int kh = tap / p.KW, kw = tap - (tap / p.KW) * p.KW;
          int ih = a_ih0[j] + kh, iw = a_iw0[j] + kw;
          bool ok = k < p.K && a_ok[j] && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
          v[e] = ok ? p.x[(((int64_t)a_n[j] * p.H + ih) * p.W + iw) * p.Cin + c] : (bf16_t)0;
        }
        ra[j] = *(uint4*)v;
      }
    }
    // ---- B ----
#pragma unroll
    for (int j = 0; j < BLOADS; ++j) {
      int idx = tid + 256 * j;
      int row = idx >> 2, ch = idx & 3;
      int co = n0 + row;
      if (row < BN && co < p.Cout)
        rb[j] = *(const uint4*)(p.w + (int64_t)co * p.Kp + s * BK + ch * 8);
      else
        rb[j] = make_uint4(0, 0, 0, 0);
    }
  };

  auto store_step = [&](int buf) {
#pragma unroll
    for (int j = 0; j < AROWS; ++j)
      *(uint4*)&As[buf][(tid >> 2) + 64 * j][chunk * 8] = ra[j];
#pragma unroll
    for (int j = 0; j < BLOADS; ++j) {
      int idx = tid + 256 * j;
      int row = idx >> 2, ch = idx & 3;
      if (row < BN) *(uint4*)&Bs[buf][row][ch * 8] = rb[j];
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  load_step(0);
  store_step(0);
  __syncthreads();

  const int frow = lane & 15;
  const int fk = (lane >> 4) * 8;
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) load_step(s + 1);
    bf16x8 af[MI], bfr[NI];
#pragma unroll
    for (int i = 0; i < MI; ++i)
      af[i] = *(const bf16x8*)&As[buf][wm * (BM / 2) + i * 16 + frow][fk];
#pragma unroll
    for (int j = 0; j < NI; ++j)
      bfr[j] = *(const bf16x8*)&Bs[buf][wn * (BN / 2) + j * 16 + frow][fk];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (s + 1 < nsteps) store_step(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue ----
  const int ecol = lane & 15;
  const int erow = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int co = n0 + wn * (BN / 2) + j * 16 + ecol;
    if (co >= p.Cout) continue;
    const float sc = p.scale ? p.scale[co] : 1.f;
    const float bi = p.bias ? p.bias[co] : 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / 2) + i * 16 + erow + r;
        if (m >= p.M) continue;
        const int64_t o = (int64_t)m * p.Cout + co;
        float v = acc[i][j][r] * sc + bi;
        if (p.res) v += bf2f(p.res[o]);
        if (p.preact) p.preact[o] = f2bf(v);
        p.y[o] = f2bf(apply_act(v, p.act));
      }
    }
  }
}

template <int BM, int BN>
int launch_mode(const ConvParams& p, int mode, hipStream_t st) {
  dim3 grid((p.M + BM - 1) / BM, (p.Cout + BN - 1) / BN);
  if (mode == LOAD_FAST)
    hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, LOAD_FAST>), grid, dim3(256), 0, st, p);
  else if (mode == LOAD_VEC8)
    hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, LOAD_VEC8>), grid, dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, LOAD_SCALAR>), grid, dim3(256), 0, st, p);
  MDA_CHECK_LAUNCH();
}

}  // namespace

// tile: 0 = auto; otherwise BM*1000 + BN (e.g. 128064)
MDA_API int mda_conv_fwd(const void* x, const void* w, const float* scale, const float* bias,
                         const void* res, void* y, void* preact, int64_t N, int64_t H, int64_t W,
                         int64_t Cin, int64_t Ho, int64_t Wo, int64_t Cout, int64_t KH, int64_t KW,
                         int64_t stride, int64_t pad, int64_t Kp, int64_t act, int64_t tile,
                         hipStream_t st) {
  ConvParams p;
  p.x = (const bf16_t*)x; p.w = (const bf16_t*)w; p.scale = scale; p.bias = bias;
  p.res = (const bf16_t*)res; p.y = (bf16_t*)y; p.preact = (bf16_t*)preact;
  p.N = N; p.H = H; p.W = W; p.Cin = Cin; p.Ho = Ho; p.Wo = Wo; p.Cout = Cout; p.KH = KH;
  p.KW = KW; p.stride = stride; p.pad = pad; p.K = KH * KW * Cin; p.Kp = Kp; p.M = N * Ho * Wo;
  p.act = act;
  if (Kp % BK || Kp < p.K) return (int)hipErrorInvalidValue;
  int mode = (Cin % 32 == 0) ? LOAD_FAST : (Cin % 8 == 0 ? LOAD_VEC8 : LOAD_SCALAR);
  if (tile == 0) {
    // pick the largest tile that still gives >= ~2 blocks per CU (256 CUs)
    const int64_t target = 512;
    int bn = Cout <= 32 ? 32 : (Cout <= 64 ? 64 : 128);
    int bm = 128;
    auto blocks = [&](int bm_, int bn_) { return ((p.M + bm_ - 1) / bm_) * ((Cout + bn_ - 1) / bn_); };
    if (blocks(bm, bn) < target && bn == 128) bn = 64;
    if (blocks(bm, bn) < target) bm = 64;
    if (blocks(bm, bn) < target && bn == 64) bn = 32;
    tile = bm * 1000 + bn;
  }
  switch (tile) {
    case 128128: return launch_mode<128, 128>(p, mode, st);
    case 128064: return launch_mode<128, 64>(p, mode, st);
    case 128032: return launch_mode<128, 32>(p, mode, st);
    case 64128: return launch_mode<64, 128>(p, mode, st);
    case 64064: return launch_mode<64, 64>(p, mode, st);
    case 64032: return launch_mode<64, 32>(p, mode, st);
    default: return (int)hipErrorInvalidValue;
  }
}
