// Streaming 1x1 convolution for the memory-bound pointwise layers (survey K2;
// the ResNet-50 bottleneck expand / reduce convs of the ImageNet teacher, and
// any 1x1 dgrad): y[m, co] = epilogue(sum_k x[m, k] * w[co, k]).
//
// At 56x56 x batch 64 a 64 -> 256 1x1 conv reads 25 MB and writes 100 MB for
// 6.6 GFLOP: output-bandwidth bound.  The implicit-GEMM kernels in
// conv_igemm.hip stage an fp32 C tile through LDS and re-read it for 16-byte
// row stores, and their blocks each load a fresh weight tile: 3-4x MIOpen on
// these shapes (profiles/r3_conv1x1_imagenet.md).  Here:
//
// * the GEMM is computed TRANSPOSED, C^T[co, m] = W[co, :] . X[m, :]^T, with
//   the 16x16x32 bf16 MFMA: a lane's accumulator holds 4 consecutive output
//   CHANNELS of one pixel, so the epilogue goes straight from the accumulators
//   to 8-byte global stores (4 bf16 channels), no C tile, no LDS round trip;
//   the four 16-channel subtiles a wave owns complete 128-byte lines of a
//   pixel row back to back, which L2 merges before HBM;
// * the block's weight slice (BN = 64*CI output channels x K <= 256) is loaded
//   ONCE into registers (A fragments) and stays there;
// * blocks are persistent over 64-pixel tiles (grid.x ~ resident blocks):
//   the next tile's X rows are loaded into registers while the current tile
//   is multiplied and stored, then written to the other LDS buffer.
//
// Epilogues: inference (per-channel scale / bias = folded BN, residual,
// activation, optional pre-activation), training forward (raw bf16 output +
// the BN batch sums of the stored values into a BnRegion), and dgrad (raw
// store + an optional residual-fork gradient add).  stride 1 or 2 (pad 0)
// forward; dgrad stride 1.
#include "common.h"
#include "bnslot.h"
#include "bnbwd.h"
#include <stdlib.h>

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int S_BM = 64;  // pixels per tile

struct S1Params {
  const bf16_t* x;     // [N, H, W, K] (dgrad: dy [N, H, W, Cout_fwd])
  const bf16_t* w;     // [Cout][Kp]
  const float* scale;  // [Cout] or null
  const float* bias;   // [Cout] or null
  const bf16_t* res;   // [M, Cout] or null
  bf16_t* y;           // [M, Cout]
  bf16_t* preact;      // [M, Cout] or null
  BnRegion* slot;      // training forward: BN sums of the stored y (raw output, no epilogue)
  int N, H, W, Ho, Wo, K, Kp, Cout, stride, M, act, ntiles;
};

__device__ __forceinline__ float s1_act(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) return fminf(fmaxf(v, 0.f), 6.f);
  return v;
}

// CI 16-channel subtiles per wave (block: 4 waves x 16*CI channels), KK
// 32-wide k slices (K = 32*KK)
template <int KK>
struct S1Smem { static constexpr int BYTES = 2 * S_BM * (32 * KK + 8) * 2; };

// Block (bx, by) of a (gx, gy) grid: bx strides the pixel tiles (persistent),
// by picks the channel slice.  The stand-alone kernel passes blockIdx /
// gridDim; the fused launch (mda_conv1x1_bnacc_apply) a linear block index.
template <int CI, int KK>
__device__ __forceinline__ void conv1x1_body(const S1Params& p, char* smem, int bx, int by, int gx,
                                             int gy) {
  constexpr int K = 32 * KK;
  constexpr int ROW = K + 8;                  // LDS row (bf16): 16-byte pad, conflict-free b128 reads
  constexpr int CH = S_BM * K / 8 / 256;      // 16-byte X chunks per thread per tile
  static_assert(S_BM * K / 8 % 256 == 0, "tile load");
  bf16_t (*xs)[S_BM * ROW] = (bf16_t (*)[S_BM * ROW])smem;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int q = lane >> 4, r16 = lane & 15;
  const int ch0 = by * (64 * CI) + wid * (16 * CI);   // this wave's first channel
  // Cout % 64 == 32 (CI == 1): the last channel slice's upper two waves have no
  // channels -- they still stage X tiles, but multiply and store nothing
  const bool live = ch0 < p.Cout;

  // resident A fragments: W[ch0 + 16 ci + r16][32 kk + 8 q .. + 8]
  bf16x8 af[CI][KK];
#pragma unroll
  for (int ci = 0; ci < CI; ++ci)
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
      af[ci][kk] = live ? *(const bf16x8*)(p.w + (int64_t)(ch0 + 16 * ci + r16) * p.Kp + 32 * kk + 8 * q)
                        : (bf16x8){};
  // this lane's output channels: ch0 + 16 ci + 4 q + e
  float sc[CI][4], bi[CI][4];
#pragma unroll
  for (int ci = 0; ci < CI; ++ci)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = ch0 + 16 * ci + 4 * q + e;
      sc[ci][e] = (p.scale && live) ? p.scale[c] : 1.f;
      bi[ci][e] = (p.bias && live) ? p.bias[c] : 0.f;
    }
  float s1[CI][4], s2[CI][4];
#pragma unroll
  for (int ci = 0; ci < CI; ++ci)
#pragma unroll
    for (int e = 0; e < 4; ++e) { s1[ci][e] = 0.f; s2[ci][e] = 0.f; }

  const int HoWo = p.Ho * p.Wo;
  // X rows of a tile -> registers (zero past M); row = output pixel, its input
  // pixel (n, s*oh, s*ow)
  auto load_tile = [&](int t, uint4 (&v)[CH]) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = tid + 256 * j;
      const int row = c / (K / 8), c8 = c - row * (K / 8);
      const int m = t * S_BM + row;
      uint4 val = make_uint4(0u, 0u, 0u, 0u);
      if (m < p.M) {
        int64_t src;
        if (p.stride == 1) {
          src = (int64_t)m * K;
        } else {
          const int n = m / HoWo, rr = m - n * HoWo, oh = rr / p.Wo, ow = rr - oh * p.Wo;
          src = ((int64_t)(n * p.H + oh * p.stride) * p.W + ow * p.stride) * K;
        }
        val = *(const uint4*)(p.x + src + c8 * 8);
      }
      v[j] = val;
    }
  };
  auto store_tile = [&](int buf, const uint4 (&v)[CH]) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = tid + 256 * j;
      const int row = c / (K / 8), c8 = c - row * (K / 8);
      *(uint4*)(&xs[buf][row * ROW + c8 * 8]) = v[j];
    }
  };

  int t = bx;
  if (t >= p.ntiles) goto done;
  {
    uint4 v[CH];
    load_tile(t, v);
    store_tile(0, v);
    __syncthreads();
    int buf = 0;
    for (; t < p.ntiles; t += gx) {
      const int tn = t + gx;
      if (tn < p.ntiles) load_tile(tn, v);   // in flight during this tile's MFMAs and stores
      f32x4 acc[CI][4];
#pragma unroll
      for (int ci = 0; ci < CI; ++ci)
#pragma unroll
        for (int pj = 0; pj < 4; ++pj) acc[ci][pj] = (f32x4){0.f, 0.f, 0.f, 0.f};
      const bf16_t* xb = xs[buf];
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        bf16x8 bfr[4];
#pragma unroll
        for (int pj = 0; pj < 4; ++pj)
          bfr[pj] = *(const bf16x8*)(xb + (16 * pj + r16) * ROW + 32 * kk + 8 * q);
#pragma unroll
        for (int ci = 0; ci < CI; ++ci)
#pragma unroll
          for (int pj = 0; pj < 4; ++pj)
            acc[ci][pj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ci][kk], bfr[pj], acc[ci][pj], 0, 0, 0);
      }
      // epilogue straight from the accumulators: lane = pixel 16 pj + r16,
      // channels ch0 + 16 ci + 4 q .. + 3 (8-byte stores)
#pragma unroll
      for (int pj = 0; pj < 4; ++pj) {
        const int m = t * S_BM + 16 * pj + r16;
        if (m >= p.M || !live) continue;
#pragma unroll
        for (int ci = 0; ci < CI; ++ci) {
          const int c = ch0 + 16 * ci + 4 * q;
          const int64_t o = (int64_t)m * p.Cout + c;
          float z[4];
          if (p.slot != nullptr) {
            const uint2 u = make_uint2(pack_bf16x2(acc[ci][pj][0], acc[ci][pj][1]),
                                       pack_bf16x2(acc[ci][pj][2], acc[ci][pj][3]));
            *(uint2*)(p.y + o) = u;
            const float a0 = __uint_as_float(u.x << 16), a1 = __uint_as_float(u.x & 0xffff0000u);
            const float a2 = __uint_as_float(u.y << 16), a3 = __uint_as_float(u.y & 0xffff0000u);
            s1[ci][0] += a0; s2[ci][0] += a0 * a0;
            s1[ci][1] += a1; s2[ci][1] += a1 * a1;
            s1[ci][2] += a2; s2[ci][2] += a2 * a2;
            s1[ci][3] += a3; s2[ci][3] += a3 * a3;
            continue;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) z[e] = acc[ci][pj][e] * sc[ci][e] + bi[ci][e];
          if (p.res) {
            const uint2 rv = *(const uint2*)(p.res + o);
            z[0] += __uint_as_float(rv.x << 16);
            z[1] += __uint_as_float(rv.x & 0xffff0000u);
            z[2] += __uint_as_float(rv.y << 16);
            z[3] += __uint_as_float(rv.y & 0xffff0000u);
          }
          if (p.preact)
            *(uint2*)(p.preact + o) = make_uint2(pack_bf16x2(z[0], z[1]), pack_bf16x2(z[2], z[3]));
          *(uint2*)(p.y + o) = make_uint2(pack_bf16x2(s1_act(z[0], p.act), s1_act(z[1], p.act)),
                                          pack_bf16x2(s1_act(z[2], p.act), s1_act(z[3], p.act)));
        }
      }
      if (tn < p.ntiles) store_tile(buf ^ 1, v);
      __syncthreads();  // next buffer written; this buffer's reads retired
      buf ^= 1;
    }
  }
done:
  if (p.slot != nullptr && live) {
    // the 16 lanes of a quad group hold the same channels: reduce over r16,
    // then one fp64 atomic per channel and block into shard blockIdx % SH
#pragma unroll
    for (int ci = 0; ci < CI; ++ci)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float a = s1[ci][e], b = s2[ci][e];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          a += __shfl_xor(a, o, 64);
          b += __shfl_xor(b, o, 64);
        }
        if (r16 == 0) {
          const int c = ch0 + 16 * ci + 4 * q + e;
          const int sh = (int)(bx + gx * by) % slot_shards(p.Cout);
          acc_add(region_acc(p.slot, p.Cout, sh, 0) + c, (double)a);
          acc_add(region_acc(p.slot, p.Cout, sh, 1) + c, (double)b);
        }
      }
  }
}

template <int CI, int KK>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
conv1x1_stream_kernel(const S1Params p) {
  __shared__ __attribute__((aligned(16))) char smem[S1Smem<KK>::BYTES];
  conv1x1_body<CI, KK>(p, smem, (int)blockIdx.x, (int)blockIdx.y, (int)gridDim.x, (int)gridDim.y);
}

// A residual block's projection-shortcut conv (training forward: raw output
// + BN sums) and the BN forward apply of conv1's output in ONE launch:
// neither reads the other's output (the shortcut reads the block input,
// the apply conv1's raw output) and back to back each ran on half the GPU.
// Blocks [0, gx * gy) are the conv's, the rest the apply's (bnbwd.h).
template <int CI, int KK>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
conv1x1_apply_kernel(const S1Params p, const FwdApply a, int gx, int gy) {
  __shared__ __attribute__((aligned(16))) char smem[S1Smem<KK>::BYTES];
  const int nw = gx * gy, b = blockIdx.x;
  if (b < nw) conv1x1_body<CI, KK>(p, smem, b % gx, b / gx, gx, gy);
  else bn_apply_fin_body<4>(a, (float*)smem, b - nw, (int)gridDim.x - nw);
}

int g_cus = 0;
int cus() {
  if (g_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      g_cus = n;
    else
      g_cus = 256;
  }
  return g_cus;
}

template <int CI, int KK>
int launch_ci(const S1Params& p, hipStream_t st, const FwdApply* fa) {
  const int ny = (p.Cout + 64 * CI - 1) / (64 * CI);
  // persistent: about two resident blocks per CU over all channel tiles
  int gx = (2 * cus() + ny - 1) / ny;
  if (gx > p.ntiles) gx = p.ntiles;
  if (gx < 1) gx = 1;
  if (fa != nullptr) {
    if (bn_fin_lds_bytes(fa->C, fa->rreg != nullptr) > S1Smem<KK>::BYTES) return -1;
    const int nbn = apply_blocks(fa->M * fa->C / 8, 4);
    hipLaunchKernelGGL((conv1x1_apply_kernel<CI, KK>), dim3(gx * ny + nbn), dim3(256), 0, st, p,
                       *fa, gx, ny);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL((conv1x1_stream_kernel<CI, KK>), dim3(gx, ny), dim3(256), 0, st, p);
  return (int)hipGetLastError();
}

template <int KK>
int launch_kk(const S1Params& p, hipStream_t st, const FwdApply* fa) {
  // widest channel slice without register spills (kernel-resource-usage:
  // <4, 2> 228 VGPRs, <2, 8> 248, <4, 4> spills)
  if constexpr (KK <= 2) {
    if (p.Cout % 256 == 0) return launch_ci<4, KK>(p, st, fa);
  }
  if (p.Cout % 128 == 0) return launch_ci<2, KK>(p, st, fa);
  if (p.Cout % 32 == 0) return launch_ci<1, KK>(p, st, fa);  // (Cout % 64 == 32: half-live slice)
  return (int)hipErrorInvalidValue;
}

}  // namespace

// Eligibility + launch (host side of conv_igemm.hip's dispatch): 1x1, pad 0,
// dense, K a multiple of 32 up to 256 (weight rows Kp >= K), Cout % 32 == 0, stride 1 (or 2
// for a forward), large M.  Returns -1 when the shape is not served.
static int conv1x1_try(const void* x, const void* w, const float* scale, const float* bias,
                       const void* res, void* y, void* preact, void* slot, int64_t N, int64_t H,
                       int64_t W, int64_t K, int64_t Kp, int64_t Ho, int64_t Wo, int64_t Cout,
                       int64_t stride, int64_t act, hipStream_t st, const FwdApply* fa,
                       int64_t min_m_override) {
  static const bool on = [] {
    const char* e = getenv("MDA_CONV1X1_STREAM");
    return !(e && e[0] == '0');
  }();
  static const int64_t min_m = [] {
    const char* e = getenv("MDA_CONV1X1_MIN_M");
    return e ? (int64_t)atoll(e) : (int64_t)16384;
  }();
  const int64_t M = N * Ho * Wo;
  static const int cmod = [] {
    const char* e = getenv("MDA_CONV1X1_C32");  // 0: Cout % 64 only (A/B)
    return (e && e[0] == '0') ? 64 : 32;
  }();
  if (!on || Kp < K || K % 32 || K > 256 || Cout % cmod ||
      M < (min_m_override > 0 ? min_m_override : min_m) || (stride != 1 && stride != 2))
    return -1;
  if (N * H * W * K >= ((int64_t)1 << 31) || M * Cout >= ((int64_t)1 << 31)) return -1;
  if (((uintptr_t)x | (uintptr_t)y | (uintptr_t)(res ? res : y) | (uintptr_t)(preact ? preact : y)) & 15)
    return -1;
  S1Params p;
  p.x = (const bf16_t*)x; p.w = (const bf16_t*)w; p.scale = scale; p.bias = bias;
  p.res = (const bf16_t*)res; p.y = (bf16_t*)y; p.preact = (bf16_t*)preact; p.slot = (BnRegion*)slot;
  p.N = (int)N; p.H = (int)H; p.W = (int)W; p.Ho = (int)Ho; p.Wo = (int)Wo; p.K = (int)K;
  p.Kp = (int)Kp; p.Cout = (int)Cout; p.stride = (int)stride; p.M = (int)M; p.act = (int)act;
  p.ntiles = (int)((M + S_BM - 1) / S_BM);
  switch (K) {
    case 32: return launch_kk<1>(p, st, fa);   // MobileNetV1's 32 -> 64 at 112^2 (output-bound)
    case 64: return launch_kk<2>(p, st, fa);
    case 96: return launch_kk<3>(p, st, fa);
    case 128: return launch_kk<4>(p, st, fa);
    case 160: return launch_kk<5>(p, st, fa);
    case 192: return launch_kk<6>(p, st, fa);
    case 224: return launch_kk<7>(p, st, fa);
    default: return launch_kk<8>(p, st, fa);
  }
}

extern "C" int mda_conv1x1_stream_try(const void* x, const void* w, const float* scale,
                                      const float* bias, const void* res, void* y, void* preact,
                                      void* slot, int64_t N, int64_t H, int64_t W, int64_t K,
                                      int64_t Kp, int64_t Ho, int64_t Wo, int64_t Cout,
                                      int64_t stride, int64_t act, hipStream_t st) {
  return conv1x1_try(x, w, scale, bias, res, y, preact, slot, N, H, W, K, Kp, Ho, Wo, Cout, stride,
                     act, st, nullptr, 0);
}

// A projection shortcut's training conv (1 x 1, stride 1 or 2, pad 0: raw
// bf16 output y + its BN batch sums into `slot`) and the BN forward apply of
// ANOTHER layer (conv1 of the same block: a_y its raw output, a_reg its
// region, the finalize operands, out / pre) in one launch
// (conv1x1_apply_kernel).  Every M is served (the apply fills the GPU the
// small conv leaves idle).  MDA_NOT_SERVED (nothing launched) when the conv
// is not a streaming-kernel shape.
MDA_API int mda_conv1x1_bnacc_apply(const void* x, const void* w, void* y, void* slot, int64_t N,
                                    int64_t H, int64_t W, int64_t K, int64_t Kp, int64_t Ho,
                                    int64_t Wo, int64_t Cout, int64_t stride, const void* a_y,
                                    void* a_reg, int64_t a_M, int64_t a_C, const float* gamma,
                                    const float* beta, float* running_mean, float* running_var,
                                    float* stats, float momentum, float eps, int64_t* nbt,
                                    const void* a_res, void* a_out, void* a_pre, int64_t a_act,
                                    hipStream_t st) {
  if (a_C % 8 || a_C > SLOT_CMAX || a_M <= 0 || a_M >= ((int64_t)1 << 31) || slot == nullptr ||
      a_reg == nullptr)
    return MDA_NOT_SERVED;
  const FwdApply fa{(const bf16_t*)a_y, (BnRegion*)a_reg, a_M, (int)a_C,
                    FinArgs{gamma, beta, running_mean, running_var, stats, momentum, eps, nbt},
                    (const bf16_t*)a_res, (bf16_t*)a_out, (bf16_t*)a_pre, (int)a_act, nullptr,
                    FinArgs{}};
  const int rc = conv1x1_try(x, w, nullptr, nullptr, nullptr, y, nullptr, slot, N, H, W, K, Kp,
                             Ho, Wo, Cout, stride, 0, st, &fa, 1);
  return rc == -1 ? MDA_NOT_SERVED : rc;
}
