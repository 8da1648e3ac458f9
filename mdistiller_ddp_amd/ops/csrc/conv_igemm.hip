// Implicit-GEMM convolution on CDNA4 MFMA (bf16 in, fp32 accumulate) with a
// fused per-channel epilogue (survey K1/K2):
//
//   y[m, co] = act( acc[m, co] * scale[co] + bias[co] + residual[m, co] )
//
// GEMM view (NHWC activations, "B^T" weights):
//   M = N*Ho*Wo output pixels, N = Cout, K = KH*KW*Cin
//   A[m, k]  = x[n, oh*s - p + kh, ow*s - p + kw, ci]   (zero outside the image)
//   B[k, co] = w_packed[co, k]  with k = (kh*KW + kw)*Cin + ci, rows padded to Kp = ceil64(K)
//
// With frozen BN folded into (w, bias) this is the whole teacher layer
// (conv + BN + residual add + ReLU) in ONE launch; the reference runs 4-5
// kernels per layer (cuDNN conv, BN, add, ReLU).  ``preact`` optionally also
// stores the pre-activation tensor (feature distillers consume it).
//
// Tiling: 256 threads = 4 waves as 2x2; block tile BM x BN x 64, wave tile
// (BM/2) x (BN/2) built from 16x16x32 bf16 MFMAs (2 k-substeps per stage).
// A/B K-slices are staged global -> VGPR -> LDS with a register prefetch of
// stage s+1 while stage s computes; two LDS buffers, one barrier per stage.
// LDS rows are 144 B (64 bf16 + 16 B pad): row starts land on 16 distinct
// 4-bank slots, so every 16-lane group of a ds_read_b128 fragment read is
// conflict-free.
//
// Narrow-M layers (the 8x8 / 16x16 CIFAR stages at small batch) do not fill
// 256 CUs with output tiles alone, so the K loop is split over gridDim.z;
// partial fp32 tiles go to a workspace and a second launch sums them in a
// fixed order and applies the epilogue (deterministic, no float atomics).
//
// Loader modes: FAST (Cin % 64 == 0: each stage is one filter tap), VEC8
// (Cin % 8 == 0: every 16-byte chunk lies inside one tap), SCALAR (any Cin,
// e.g. the 3-channel stem).
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int BK = 64;
constexpr int LDS_ROW = 72;  // bf16 elements per LDS row (64 + 8 pad = 144 B)

enum { LOAD_FAST = 0, LOAD_VEC8 = 1, LOAD_SCALAR = 2, LOAD_DGRAD_FAST = 3, LOAD_DGRAD_VEC8 = 4 };
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_RELU6 = 2 };

struct ConvParams {
  const bf16_t* x;       // [N, H, W, Cin]
  const bf16_t* w;       // [Cout, Kp]
  const float* scale;    // [Cout] or null
  const float* bias;     // [Cout] or null
  const bf16_t* res;     // [M, Cout] or null
  bf16_t* y;             // [M, Cout]
  bf16_t* preact;        // [M, Cout] or null
  float* partial;        // [splits, M, Cout] when split-K
  int N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, K, Kp, M, act;
  int steps_per_split;
};

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == ACT_RELU) return fmaxf(v, 0.f);
  if (act == ACT_RELU6) return fminf(fmaxf(v, 0.f), 6.f);
  return v;
}

__device__ __forceinline__ void epilogue_store(const ConvParams& p, int m, int co, float acc) {
  const int64_t o = (int64_t)m * p.Cout + co;
  float v = acc * (p.scale ? p.scale[co] : 1.f) + (p.bias ? p.bias[co] : 0.f);
  if (p.res) v += bf2f(p.res[o]);
  if (p.preact) p.preact[o] = f2bf(v);
  p.y[o] = f2bf(apply_act(v, p.act));
}

template <int BM, int BN, int MODE>
__global__ void __launch_bounds__(256)
conv_fwd_kernel(const ConvParams p) {
  constexpr int MI = BM / 32;  // 16-row MFMA tiles per wave (wave tile = BM/2 rows)
  constexpr int NI = BN / 32;
  constexpr int AROWS = BM / 32;  // A rows loaded per thread per stage (8 chunks per row)
  constexpr int BLOADS = (BN * 8 + 255) / 256;

  __shared__ __attribute__((aligned(16))) bf16_t As[2][BM][LDS_ROW];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][BN][LDS_ROW];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int chunk = tid & 7;
  const int arow = tid >> 3;
  const int HoWo = p.Ho * p.Wo;

  int a_n[AROWS], a_ih0[AROWS], a_iw0[AROWS];
  bool a_ok[AROWS];
#pragma unroll
  for (int j = 0; j < AROWS; ++j) {
    int m = m0 + arow + 32 * j;
    a_ok[j] = m < p.M;
    int mm = a_ok[j] ? m : 0;
    int n = mm / HoWo;
    int r = mm - n * HoWo;
    int oh = r / p.Wo;
    int ow = r - oh * p.Wo;
    a_n[j] = n;
    if (MODE == LOAD_DGRAD_FAST || MODE == LOAD_DGRAD_VEC8) {
      // dgrad: output row = input-gradient pixel (ih, iw); taps gather dy at
      // oh = (ih + pad - kh) / stride when divisible and in range
      a_ih0[j] = oh + p.pad;
      a_iw0[j] = ow + p.pad;
    } else {
      a_ih0[j] = oh * p.stride - p.pad;
      a_iw0[j] = ow * p.stride - p.pad;
    }
  }

  uint4 ra[AROWS];
  uint4 rb[BLOADS];
  const int total_steps = p.Kp / BK;
  const int s_begin = blockIdx.z * p.steps_per_split;
  const int s_end = min(total_steps, s_begin + p.steps_per_split);
  const int cin_blocks = p.Cin / BK;  // FAST mode only

  auto load_step = [&](int s) {
    if (MODE == LOAD_FAST) {
      const int tap = s / cin_blocks;
      const int c0 = (s - tap * cin_blocks) * BK + chunk * 8;
      const int kh = tap / p.KW, kw = tap - kh * p.KW;
#pragma unroll
      for (int j = 0; j < AROWS; ++j) {
        int ih = a_ih0[j] + kh, iw = a_iw0[j] + kw;
        bool ok = a_ok[j] && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        ra[j] = ok ? *(const uint4*)(p.x + (((int64_t)a_n[j] * p.H + ih) * p.W + iw) * p.Cin + c0)
                   : make_uint4(0, 0, 0, 0);
      }
    } else if (MODE == LOAD_VEC8) {
      const int k0 = s * BK + chunk * 8;
      const int tap = k0 / p.Cin;
      const int c0 = k0 - tap * p.Cin;
      const int kh = tap / p.KW, kw = tap - kh * p.KW;
      const bool kok = k0 < p.K;
#pragma unroll
      for (int j = 0; j < AROWS; ++j) {
        int ih = a_ih0[j] + kh, iw = a_iw0[j] + kw;
        bool ok = kok && a_ok[j] && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        ra[j] = ok ? *(const uint4*)(p.x + (((int64_t)a_n[j] * p.H + ih) * p.W + iw) * p.Cin + c0)
                   : make_uint4(0, 0, 0, 0);
      }
    } else if (MODE == LOAD_DGRAD_FAST || MODE == LOAD_DGRAD_VEC8) {
      int tap, c0;
      bool kok = true;
      if (MODE == LOAD_DGRAD_FAST) {
        tap = s / cin_blocks;
        c0 = (s - tap * cin_blocks) * BK + chunk * 8;
      } else {
        const int k0 = s * BK + chunk * 8;
        tap = k0 / p.Cin;
        c0 = k0 - tap * p.Cin;
        kok = k0 < p.K;
      }
      const int kh = tap / p.KW, kw = tap - kh * p.KW;
#pragma unroll
      for (int j = 0; j < AROWS; ++j) {
        const int nh = a_ih0[j] - kh, nw = a_iw0[j] - kw;
        bool ok = kok && a_ok[j] && nh >= 0 && nw >= 0;
        int ih = 0, iw = 0;
        if (p.stride == 1) {
          ih = nh; iw = nw;
        } else {
          ok = ok && (nh % p.stride == 0) && (nw % p.stride == 0);
          ih = nh / p.stride; iw = nw / p.stride;
        }
        ok = ok && ih < p.H && iw < p.W;
        ra[j] = ok ? *(const uint4*)(p.x + (((int64_t)a_n[j] * p.H + ih) * p.W + iw) * p.Cin + c0)
                   : make_uint4(0, 0, 0, 0);
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
          int kh = tap / p.KW, kw = tap - kh * p.KW;
          int ih = a_ih0[j] + kh, iw = a_iw0[j] + kw;
          bool ok = k < p.K && a_ok[j] && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
          v[e] = ok ? p.x[(((int64_t)a_n[j] * p.H + ih) * p.W + iw) * p.Cin + c] : (bf16_t)0;
        }
        ra[j] = *(uint4*)v;
      }
    }
#pragma unroll
    for (int j = 0; j < BLOADS; ++j) {
      int idx = tid + 256 * j;
      int row = idx >> 3, ch = idx & 7;
      int co = n0 + row;
      rb[j] = (row < BN && co < p.Cout)
                  ? *(const uint4*)(p.w + (int64_t)co * p.Kp + s * BK + ch * 8)
                  : make_uint4(0, 0, 0, 0);
    }
  };

  auto store_step = [&](int buf) {
#pragma unroll
    for (int j = 0; j < AROWS; ++j) *(uint4*)&As[buf][arow + 32 * j][chunk * 8] = ra[j];
#pragma unroll
    for (int j = 0; j < BLOADS; ++j) {
      int idx = tid + 256 * j;
      int row = idx >> 3, ch = idx & 7;
      if (row < BN) *(uint4*)&Bs[buf][row][ch * 8] = rb[j];
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if (s_begin < s_end) {
    load_step(s_begin);
    store_step(0);
  }
  __syncthreads();

  const int frow = lane & 15;
  const int fk = (lane >> 4) * 8;
  for (int s = s_begin; s < s_end; ++s) {
    const int buf = (s - s_begin) & 1;
    const bool more = s + 1 < s_end;
    if (more) load_step(s + 1);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        af[i] = *(const bf16x8*)&As[buf][wm * (BM / 2) + i * 16 + frow][kk + fk];
#pragma unroll
      for (int j = 0; j < NI; ++j)
        bfr[j] = *(const bf16x8*)&Bs[buf][wn * (BN / 2) + j * 16 + frow][kk + fk];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) store_step(buf ^ 1);
    __syncthreads();
  }

  const int ecol = lane & 15;
  const int erow = (lane >> 4) * 4;
  const bool split = gridDim.z > 1;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int co = n0 + wn * (BN / 2) + j * 16 + ecol;
    if (co >= p.Cout) continue;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / 2) + i * 16 + erow + r;
        if (m >= p.M) continue;
        if (split)
          p.partial[((int64_t)blockIdx.z * p.M + m) * p.Cout + co] = acc[i][j][r];
        else
          epilogue_store(p, m, co, acc[i][j][r]);
      }
    }
  }
}

// Split-K combine: y = epilogue(sum_z partial[z]) in fixed z order.
__global__ void __launch_bounds__(256) conv_splitk_epilogue(const ConvParams p, int splits) {
  const int64_t total = (int64_t)p.M * p.Cout;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    float a = 0.f;
    for (int z = 0; z < splits; ++z) a += p.partial[(int64_t)z * total + i];
    const int m = (int)(i / p.Cout);
    const int co = (int)(i - (int64_t)m * p.Cout);
    epilogue_store(p, m, co, a);
  }
}

template <int BM, int BN>
int launch_tile(const ConvParams& p, int mode, int splits, hipStream_t st) {
  dim3 grid((p.M + BM - 1) / BM, (p.Cout + BN - 1) / BN, splits);
  if (mode == LOAD_FAST)
    hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, LOAD_FAST>), grid, dim3(256), 0, st, p);
  else if (mode == LOAD_VEC8)
    hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, LOAD_VEC8>), grid, dim3(256), 0, st, p);
  else if (mode == LOAD_DGRAD_FAST)
    hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, LOAD_DGRAD_FAST>), grid, dim3(256), 0, st, p);
  else if (mode == LOAD_DGRAD_VEC8)
    hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, LOAD_DGRAD_VEC8>), grid, dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, LOAD_SCALAR>), grid, dim3(256), 0, st, p);
  return (int)hipGetLastError();
}

}  // namespace

// Host-side tile / split-K choice (also used by Python to size the workspace).
// Returns tile code BM*1000+BN in *tile and the split count in *splits.
MDA_API int mda_conv_plan(int64_t M, int64_t Cout, int64_t Kp, int64_t* tile, int64_t* splits) {
  const int64_t target = 512;  // >= 2 workgroups per CU on 256 CUs
  int bn = Cout <= 32 ? 32 : (Cout <= 64 ? 64 : 128);
  int bm = 128;
  auto blocks = [&](int bm_, int bn_) { return ((M + bm_ - 1) / bm_) * ((Cout + bn_ - 1) / bn_); };
  if (blocks(bm, bn) < target && bn == 128) bn = 64;
  if (blocks(bm, bn) < target) bm = 64;
  int64_t nb = blocks(bm, bn);
  int64_t steps = Kp / BK;
  int64_t sp = 1;
  while (nb * sp < target && steps / (sp * 2) >= 4 && sp < 8) sp *= 2;
  *tile = bm * 1000 + bn;
  *splits = sp;
  return 0;
}

namespace {

int dispatch(ConvParams& p, int mode, int64_t tile, int64_t splits, hipStream_t st) {
  if (p.Kp % BK || p.Kp < p.K) return (int)hipErrorInvalidValue;
  if (tile == 0 || splits == 0) mda_conv_plan(p.M, p.Cout, p.Kp, &tile, &splits);
  if (splits > 1 && p.partial == nullptr) return (int)hipErrorInvalidValue;
  const int steps = p.Kp / BK;
  p.steps_per_split = (int)((steps + splits - 1) / splits);
  int rc;
  switch (tile) {
    case 128128: rc = launch_tile<128, 128>(p, mode, splits, st); break;
    case 128064: rc = launch_tile<128, 64>(p, mode, splits, st); break;
    case 128032: rc = launch_tile<128, 32>(p, mode, splits, st); break;
    case 64128: rc = launch_tile<64, 128>(p, mode, splits, st); break;
    case 64064: rc = launch_tile<64, 64>(p, mode, splits, st); break;
    case 64032: rc = launch_tile<64, 32>(p, mode, splits, st); break;
    default: return (int)hipErrorInvalidValue;
  }
  if (rc || splits <= 1) return rc;
  int64_t total = (int64_t)p.M * p.Cout;
  int blocks = (int)std::min<int64_t>((total + 255) / 256, 2048);
  hipLaunchKernelGGL(conv_splitk_epilogue, dim3(blocks), dim3(256), 0, st, p, (int)splits);
  return (int)hipGetLastError();
}

}  // namespace

// tile/splits: 0 = auto (mda_conv_plan).  partial: fp32 workspace of
// splits*M*Cout floats (may be null when splits == 1).
MDA_API int mda_conv_fwd(const void* x, const void* w, const float* scale, const float* bias,
                         const void* res, void* y, void* preact, float* partial, int64_t N,
                         int64_t H, int64_t W, int64_t Cin, int64_t Ho, int64_t Wo, int64_t Cout,
                         int64_t KH, int64_t KW, int64_t stride, int64_t pad, int64_t Kp,
                         int64_t act, int64_t tile, int64_t splits, hipStream_t st) {
  ConvParams p;
  p.x = (const bf16_t*)x; p.w = (const bf16_t*)w; p.scale = scale; p.bias = bias;
  p.res = (const bf16_t*)res; p.y = (bf16_t*)y; p.preact = (bf16_t*)preact; p.partial = partial;
  p.N = N; p.H = H; p.W = W; p.Cin = Cin; p.Ho = Ho; p.Wo = Wo; p.Cout = Cout; p.KH = KH;
  p.KW = KW; p.stride = stride; p.pad = pad; p.K = KH * KW * Cin; p.Kp = Kp; p.M = N * Ho * Wo;
  p.act = act;
  int mode = (Cin % BK == 0) ? LOAD_FAST : (Cin % 8 == 0 ? LOAD_VEC8 : LOAD_SCALAR);
  return dispatch(p, mode, tile, splits, st);
}

// Input gradient of a convolution (any stride): dx[N, H, W, Cin] =
// sum_{kh,kw,co} dy[N, (ih+pad-kh)/s, (iw+pad-kw)/s, co] * w[co, ci, kh, kw].
// wt: weights packed [Cin][Kp] with k = (kh*KW + kw)*Cout + co (mda_pack_conv_weights).
// dy: [N, Ho, Wo, Cout]; requires Cout % 8 == 0.
MDA_API int mda_conv_dgrad(const void* dy, const void* wt, void* dx, float* partial, int64_t N,
                           int64_t H, int64_t W, int64_t Cin, int64_t Ho, int64_t Wo,
                           int64_t Cout, int64_t KH, int64_t KW, int64_t stride, int64_t pad,
                           int64_t Kp, int64_t tile, int64_t splits, hipStream_t st) {
  if (Cout % 8) return (int)hipErrorInvalidValue;
  ConvParams p;
  p.x = (const bf16_t*)dy; p.w = (const bf16_t*)wt; p.scale = nullptr; p.bias = nullptr;
  p.res = nullptr; p.y = (bf16_t*)dx; p.preact = nullptr; p.partial = partial;
  // GEMM view: rows = dx pixels, cols = Cin, k = (tap, co); "input" image = dy
  p.N = N; p.H = Ho; p.W = Wo; p.Cin = Cout; p.Ho = H; p.Wo = W; p.Cout = Cin; p.KH = KH;
  p.KW = KW; p.stride = stride; p.pad = pad; p.K = KH * KW * Cout; p.Kp = Kp; p.M = N * H * W;
  p.act = 0;
  int mode = (Cout % BK == 0) ? LOAD_DGRAD_FAST : LOAD_DGRAD_VEC8;
  return dispatch(p, mode, tile, splits, st);
}
