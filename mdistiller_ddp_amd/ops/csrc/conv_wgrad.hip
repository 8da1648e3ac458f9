// Convolution weight gradient on MFMA + fp32 master-weight plumbing.
//
// wgrad:  dW[co, k] = sum_m dy[m, co] * A[m, k]     (A = im2col(x), k = (kh*KW+kw)*Cin + ci)
//
// The reduction runs over output pixels m, which is the OUTER (row) index of
// both NHWC operands, so both tiles are staged into LDS as natural
// [m][channel] rows (16-byte global loads) and the MFMA fragments -- which
// want 8 consecutive m per lane -- are read with the CDNA4 transposing LDS
// read ds_read_b64_tr_b16 (two per fragment).  Block tile 64 co x 64 k,
// 4 waves as 2x2 (32x32 per wave, 16x16x32 bf16 MFMA), 64 pixels per stage,
// register-prefetched double buffer.  The pixel range is split over
// gridDim.z (M = N*Ho*Wo is 65536 for a 32x32 stage at batch 64) and the
// fp32 partials are combined by mda_wgrad_reduce in a fixed order, which
// also scatters into the OIHW fp32 gradient and ACCUMULATES into it (the
// flat gradient buffer the optimizer reads) -- no separate grad cast/add.
//
// pack:   fp32 OIHW master weights -> bf16 [Cout][Kp] (forward operand) and,
//         optionally, bf16 [Cin][KpT] with k = (kh*KW+kw)*Cout + co (dgrad
//         operand), in one launch per conv per step.
#include "common.h"
#include "bnslot.h"
#include "bnbwd.h"

extern uint64_t* g_stamps;  // csrc/conv_igemm.hip (mda_conv_set_stamps)

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int TM = 64;       // pixels per stage
constexpr int TC = 64;       // co per block
constexpr int TK = 64;       // k per block
constexpr int ROW = 72;      // LDS row length (bf16), 144 B

enum { WG_FAST = 0, WG_VEC8 = 1, WG_SCALAR = 2 };

// Division by a runtime constant as multiply-high + shift (n < 2^31):
// q = (umulhi(n, mul) + n) >> shr with shr = ceil(log2 d),
// mul = floor(2^32 (2^shr - d) / d) + 1.
struct FastDiv {
  uint32_t d, mul, shr;
};
inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.shr = l;
  f.mul = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
  return f;
}
__device__ __forceinline__ int fdiv(int n, const FastDiv& f) {
  return (int)((__umulhi((uint32_t)n, f.mul) + (uint32_t)n) >> f.shr);
}

struct WgParams {
  const bf16_t* x;   // [N, H, W, Cin]
  const bf16_t* dy;  // [N, Ho, Wo, Cout]
  float* partial;    // [splits, Cout, Kp]
  int N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, K, Kp, M, m_per_split;
  int x_bytes, dy_bytes;
  FastDiv div_howo, div_wo;
  // splits per gradient set: gridDim.z = sets x zsp.  Set k (DOT single-pass
  // backward: two stacked cotangents) reads dy k*M*Cout elements in and owns
  // partial sets [k*zsp, (k+1)*zsp); x is shared.
  int zsp;
  // halo kernel: a 64-pixel stage is h_img whole images of h_rh rows (W = Wo)
  int h_rh, h_img;
  uint64_t* stamps;  // diagnostics: per-block phase stamps (mda_conv_set_stamps), else null
};

// A GEMM block's position in its (co tile, k tile, split) grid.  The
// stand-alone kernels take it from blockIdx; the fused launches
// (wgrad + BN-backward apply, mda_conv_wgrad_nored_bn) from the block's
// linear index, in the same x-fastest order.
struct VB {
  int x, y, z, gx, gy, gz;
  __device__ int lin() const { return x + gx * (y + gy * z); }
};
__device__ __forceinline__ VB vb_hw() {
  return VB{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z,
            (int)gridDim.x, (int)gridDim.y, (int)gridDim.z};
}
__device__ __forceinline__ VB vb_lin(int b, int gx, int gy, int gz) {
  return VB{b % gx, (b / gx) % gy, b / (gx * gy), gx, gy, gz};
}

__device__ __forceinline__ void wg_stamp(const WgParams& p, int k, const VB& vb) {
  if (p.stamps != nullptr && threadIdx.x == 0)
    p.stamps[(int64_t)vb.lin() * 8 + k] = __builtin_amdgcn_s_memrealtime();
}

constexpr uint32_t OOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* ptr, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(ptr), (short)0, bytes, 0x00020000);
}
// ok ? off : out-of-range, without a branch: the offset is always computed
// and bit 31 forces it past the descriptor range (every range is < 2 GiB).
// A select on a runtime condition made hipcc branch around each address
// computation and load, which also broke its vmcnt bookkeeping.
__device__ __forceinline__ uint32_t sel_off(bool ok, int off) {
  return (uint32_t)off | ((uint32_t)(!ok) << 31);
}
__device__ __forceinline__ uint4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ bf16x8 tr_frag(const bf16_t* tile, int r0, int c0, int lane) {
  // lane 16g + 4q + p supplies &tile[r0 + 8g + q (+4)][c0 + 4p]; receives column (lane & 15)
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const bf16_t* a0 = tile + (r0 + 8 * g + q) * ROW + c0 + 4 * p;
  const bf16_t* a1 = a0 + 4 * ROW;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  bf16x8 out;
  short* o = (short*)&out;
  o[0] = lo[0]; o[1] = lo[1]; o[2] = lo[2]; o[3] = lo[3];
  o[4] = hi[0]; o[5] = hi[1]; o[6] = hi[2]; o[7] = hi[3];
  return out;
}

constexpr int WG_REG_SMEM = 4 * TM * ROW * 2;  // Ds[2] + Xs[2] bf16 tiles

template <int MODE>
__device__ __forceinline__ void wgrad_reg_body(const WgParams& p, char* smem, const VB& vb) {
  bf16_t (*Ds)[TM * ROW] = (bf16_t (*)[TM * ROW])smem;                  // dy tile [m][co]
  bf16_t (*Xs)[TM * ROW] = (bf16_t (*)[TM * ROW])(smem + 2 * TM * ROW * 2);  // im2col tile [m][k]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int co0 = vb.x * TC;
  const int k0 = vb.y * TK;
  const int zset = vb.z / p.zsp;
  const int m_begin = (vb.z - zset * p.zsp) * p.m_per_split;
  const int m_end = min(p.M, m_begin + p.m_per_split);
  const int chunk = tid & 7, row = tid >> 3;  // 32 rows x 8 chunks per pass, 2 passes
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  const __amdgpu_buffer_rsrc_t dr = make_rsrc(p.dy + (int64_t)zset * p.M * p.Cout, p.dy_bytes);

  // this thread's im2col column (fixed for the whole block): tap and channel
  int tap, c;
  bool kok = true;
  if (MODE == WG_FAST) {
    tap = k0 / p.Cin;  // the whole 64-wide k tile is one tap
    c = k0 - tap * p.Cin + chunk * 8;
  } else {
    const int kk = k0 + chunk * 8;
    tap = kk / p.Cin;
    c = kk - tap * p.Cin;
    kok = kk < p.K;
  }
  const int kh = tap / p.KW, kw = tap - kh * p.KW;
  const int co = co0 + chunk * 8;
  const bool cok = co < p.Cout;

  auto load = [&](int mb, uint4 (&rd)[2], uint4 (&rx)[2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = mb + row + 32 * j;
      const bool mok = m < m_end;
      rd[j] = ld16(dr, sel_off(mok && cok, (m * p.Cout + co) * 2));
      const int n = fdiv(m, p.div_howo);
      const int rr = m - n * p.Ho * p.Wo;
      const int oh = fdiv(rr, p.div_wo);
      const int ow = rr - oh * p.Wo;
      if (MODE == WG_FAST || MODE == WG_VEC8) {
        const int ih = oh * p.stride - p.pad + kh, iw = ow * p.stride - p.pad + kw;
        const bool ok = kok && mok && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        rx[j] = ld16(xr, sel_off(ok, (((n * p.H + ih) * p.W + iw) * p.Cin + c) * 2));
      } else {
        uint32_t v[4];
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          uint32_t pair = 0;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int kk = k0 + chunk * 8 + 2 * e2 + h;
            const int tp = kk / p.Cin;
            const int ce = kk - tp * p.Cin;
            const int kh2 = tp / p.KW, kw2 = tp - kh2 * p.KW;
            const int ih = oh * p.stride - p.pad + kh2, iw = ow * p.stride - p.pad + kw2;
            const bool ok = kk < p.K && mok && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
            const uint32_t e = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(
                xr, (int)sel_off(ok, (((n * p.H + ih) * p.W + iw) * p.Cin + ce) * 2), 0, 0);
            pair |= e << (16 * h);
          }
          v[e2] = pair;
        }
        rx[j] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
  };
  auto store = [&](int buf, const uint4 (&rd)[2], const uint4 (&rx)[2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = row + 32 * j;
      *(uint4*)&Ds[buf][r * ROW + chunk * 8] = rd[j];
      *(uint4*)&Xs[buf][r * ROW + chunk * 8] = rx[j];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
#pragma unroll
    for (int kk = 0; kk < TM; kk += 32) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = tr_frag(Ds[buf], kk, wm * 32 + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = tr_frag(Xs[buf], kk, wn * 32 + j * 16, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // two register staging sets (stage s+2 in flight while s+1 is written to
  // LDS and s computed), loop unrolled by two to keep them static
  uint4 rd0[2], rx0[2], rd1[2], rx1[2];
  // loads are unconditional: past m_end every row is OOB and reads zeros,
  // so each iteration issues a fixed number of loads and the vmcnt waits
  // stay exact (conditional prefetches made the compiler wait on them)
  const int n = (m_end - m_begin + TM - 1) / TM;
  load(m_begin, rd0, rx0);
  load(m_begin + TM, rd1, rx1);
  store(0, rd0, rx0);
  __syncthreads();
  for (int t = 0; t < n; t += 2) {
    load(m_begin + (t + 2) * TM, rd0, rx0);
    compute(0);
    store(1, rd1, rx1);
    __syncthreads();
    if (t + 1 >= n) break;
    load(m_begin + (t + 3) * TM, rd1, rx1);
    compute(1);
    store(0, rd0, rx0);
    __syncthreads();
  }
  const int ecol = lane & 15, erow = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int oc = co0 + wm * 32 + i * 16 + erow + r;
        const int k = k0 + wn * 32 + j * 16 + ecol;
        if (oc < p.Cout && k < p.Kp)
          p.partial[((int64_t)vb.z * p.Cout + oc) * p.Kp + k] = acc[i][j][r];
      }
}

template <int MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
conv_wgrad_kernel(const WgParams p) {
  __shared__ __attribute__((aligned(16))) char smem[WG_REG_SMEM];
  wgrad_reg_body<MODE>(p, smem, vb_hw());
}

// ---------------------------------------------------------------------------
// LDS-DMA wgrad (FAST / VEC8 modes).  The register-staged kernel above held
// one stage in flight per block and one block per CU for the ImageNet layers
// (M = 100-200 K pixels, 9-64 (co, k) tiles -> ~300 blocks): every 64-pixel
// stage paid a global-load round trip, ~56 TFLOP/s on a ResNet-18 at batch
// 32.  Here both operands go global -> LDS with global_load_lds_dwordx4
// through a 3-buffer ring (two stages in flight, one barrier per stage, as
// conv_glds_kernel), the block tile grows to 128 x 128 where the layer allows
// (64 x 64 per wave: LDS reads at half the MFMA time), and the split count
// targets several blocks per CU.
//
// Stage layout: [64 px][64 ch] bf16 subtiles of 128-B rows, TCo/64 of dy then
// TKk/64 of im2col(x).  A DMA instruction of wave w writes rows
// 32 d + 8 w + (lane >> 3), slot lane & 7, which holds the global 16-B chunk
// slot ^ wg_swz(row).  The fragment reads are ds_read_b64_tr_b16: in each 32-
// lane group they touch rows {q, 8 + q} (+ 4) x a 32-B chunk pair; rows of
// one parity share a bank half, so the XOR (even, keeps the pair) separates
// rows whose bits 1 and 3 differ -> conflict-free.
constexpr int WG_NBUF = 3;
__device__ __attribute__((aligned(16))) uint32_t g_wg_zero16[4] = {0u, 0u, 0u, 0u};

__device__ __forceinline__ int wg_swz(int r) { return (((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1; }

__device__ __forceinline__ void wg_glds16(const void* src, uint32_t lds_wave_base) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds_wave_base)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wg_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"i"(N) : "memory");
}

template <int TCo, int TKk>
struct WgOcc { static constexpr int W = (TCo * TKk >= 16384) ? 1 : 3; };

template <int TCo, int TKk>
struct WgGlds { static constexpr int BYTES = WG_NBUF * (TCo / 64 + TKk / 64) * 64 * 128; };

template <int TCo, int TKk>
__device__ __forceinline__ void wgrad_glds_body(const WgParams& p, char* smem, const VB& vb) {
  constexpr int SC = TCo / 64, SK = TKk / 64;  // 64-wide subtiles of dy / im2col(x)
  constexpr int SUB = 64 * 128;                // bytes per [64 px][64 ch] subtile
  constexpr int STAGE = (SC + SK) * SUB;
  constexpr int NL = 2 * (SC + SK);            // DMA instructions per wave per stage
  constexpr int MI = TCo / 32, NI = TKk / 32;  // 16x16 tiles per wave (wave tile TCo/2 x TKk/2)
  typedef __attribute__((address_space(3))) char lds_char;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_char*)smem;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int co0 = vb.x * TCo;
  const int k0 = vb.y * TKk;
  const int zset = vb.z / p.zsp;
  const int m_begin = (vb.z - zset * p.zsp) * p.m_per_split;
  const int m_end = min(p.M, m_begin + p.m_per_split);
  const bf16_t* const dyp = p.dy + (int64_t)zset * p.M * p.Cout;
  const uint32_t wave_off = (uint32_t)__builtin_amdgcn_readfirstlane(wid) * 1024u;
  const bf16_t* const zero = (const bf16_t*)g_wg_zero16;

  // per-lane DMA geometry (fixed for the block): rows and swizzled chunks
  int drow[2], dch[2];
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    drow[d] = 32 * d + 8 * wid + (lane >> 3);
    dch[d] = (lane & 7) ^ wg_swz(drow[d]);
  }
  int dy_col[SC][2];
  bool dy_ok[SC][2];
  int x_kh[SK][2], x_kw[SK][2], x_c[SK][2];
  bool x_ok[SK][2];
#pragma unroll
  for (int d = 0; d < 2; ++d) {
#pragma unroll
    for (int sc = 0; sc < SC; ++sc) {
      const int col = co0 + 64 * sc + dch[d] * 8;
      dy_ok[sc][d] = col < p.Cout;
      dy_col[sc][d] = dy_ok[sc][d] ? col : 0;
    }
#pragma unroll
    for (int sk = 0; sk < SK; ++sk) {
      const int k = k0 + 64 * sk + dch[d] * 8;
      x_ok[sk][d] = k < p.K;
      const int kk = x_ok[sk][d] ? k : 0;
      const int tap = kk / p.Cin;
      x_c[sk][d] = kk - tap * p.Cin;
      x_kh[sk][d] = tap / p.KW;
      x_kw[sk][d] = tap - x_kh[sk][d] * p.KW;
    }
  }

  // every copy of the 64-pixel stage starting at mb into buffer buf (always NL per wave)
  auto issue = [&](int mb, int buf) {
    const uint32_t base = lds0 + (uint32_t)(buf * STAGE) + wave_off;
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      const int m = mb + drow[d];
      const bool mok = m < m_end;
      const int mm = mok ? m : 0;
      const int n = fdiv(mm, p.div_howo);
      const int rr = mm - n * p.Ho * p.Wo;
      const int oh = fdiv(rr, p.div_wo);
      const int ow = rr - oh * p.Wo;
#pragma unroll
      for (int sc = 0; sc < SC; ++sc) {
        const bf16_t* src = (mok && dy_ok[sc][d]) ? dyp + ((int64_t)mm * p.Cout + dy_col[sc][d]) : zero;
        wg_glds16(src, base + (uint32_t)(sc * SUB + d * 4096));
      }
#pragma unroll
      for (int sk = 0; sk < SK; ++sk) {
        const int ih = oh * p.stride - p.pad + x_kh[sk][d];
        const int iw = ow * p.stride - p.pad + x_kw[sk][d];
        const bool ok = mok && x_ok[sk][d] && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        const bf16_t* src = ok ? p.x + ((int64_t)((n * p.H + ih) * p.W + iw) * p.Cin + x_c[sk][d]) : zero;
        wg_glds16(src, base + (uint32_t)((SC + sk) * SUB + d * 4096));
      }
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // transposing fragment reads: lane 16g + 4q + p reads rows r0 + 8g + q (+4),
  // bf16 columns c0 + 4p .. +3 and receives column (lane & 15), rows r0 + 8g .. +7.
  // The swizzle depends on row bits 1 and 3 only (= q >> 1, g & 1): fixed per lane.
  const int fg = lane >> 4, fq = (lane >> 2) & 3, fp = lane & 3;
  const int fswz = ((fq >> 1) | ((fg & 1) << 1)) << 1;
  const int frow_off = (8 * fg + fq) * 128 + (fp & 1) * 8;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  auto frag = [&](const char* tile, int r0, int c0) {
    const char* a = tile + r0 * 128 + frow_off + ((((c0 >> 3) + (fp >> 1)) ^ fswz) << 4);
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + 4 * 128));
    bf16x8 out;
    short* o = (short*)&out;
    o[0] = lo[0]; o[1] = lo[1]; o[2] = lo[2]; o[3] = lo[3];
    o[4] = hi[0]; o[5] = hi[1]; o[6] = hi[2]; o[7] = hi[3];
    return out;
  };
  auto compute = [&](int buf) {
    const char* Ds = smem + buf * STAGE;
    const char* Xs = Ds + SC * SUB;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int c = wm * (TCo / 2) + i * 16;  // local co
        af[i] = frag(Ds + (c >> 6) * SUB, kk * 32, c & 63);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int c = wn * (TKk / 2) + j * 16;  // local k
        bfr[j] = frag(Xs + (c >> 6) * SUB, kk * 32, c & 63);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  const int n = (m_end - m_begin + 63) / 64;
  issue(m_begin, 0);
  issue(m_begin + 64, 1);
  int cbuf = 0;
  for (int t = 0; t < n; ++t) {
    wg_wait_barrier<NL>();  // stage t landed everywhere; stage t-1 reads retired everywhere
    const int ibuf = cbuf == 0 ? 2 : cbuf - 1;
    issue(m_begin + (t + 2) * 64, ibuf);
    compute(cbuf);
    cbuf = cbuf == 2 ? 0 : cbuf + 1;
  }
  wg_wait_barrier<0>();  // drain the zero-page prefetches before the block retires

  const int ecol = lane & 15, erow = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int oc = co0 + wm * (TCo / 2) + i * 16 + erow + r;
        const int k = k0 + wn * (TKk / 2) + j * 16 + ecol;
        if (oc < p.Cout && k < p.Kp)
          p.partial[((int64_t)vb.z * p.Cout + oc) * p.Kp + k] = acc[i][j][r];
      }
}

template <int TCo, int TKk>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WgOcc<TCo, TKk>::W)))
conv_wgrad_glds_kernel(const WgParams p) {
  __shared__ __attribute__((aligned(16))) char smem[WgGlds<TCo, TKk>::BYTES];
  wgrad_glds_body<TCo, TKk>(p, smem, vb_hw());
}

// ---------------------------------------------------------------------------
// Patch-reuse ("halo") weight gradient of a 3x3 / stride-1 / pad-1 conv
// (Cin, Cout multiples of 64, W in {8, 16, 32}: the CIFAR ResNet bodies).
// The im2col kernels above give each block one tap's 64-wide k tile, so every
// input pixel crosses L2 -> LDS nine times and the dy tile once per tap.
// Here a block owns 64 output channels x 64 input channels x ALL NINE taps:
// per 64-pixel stage (whole image rows) it stages the dy tile [64 px][64 co]
// and the input patch [(rows + 2) x (W + 2) px][64 ci] once, and forms the
// tap operands as shifted views of the patch (the transposing LDS read takes
// a per-lane row address, so a tap is only a row offset).
//
// 12 waves: three groups of four, group g owning the filter row kh = g (three
// taps, 48 accumulator VGPRs per wave) over the same 2 x 2 (co, ci) wave
// grid.  Three waves per SIMD keep the MFMA pipe busy while one waits on its
// LDS reads -- the 4-wave version (nine taps per wave, 144 accumulators, one
// wave per SIMD) ran its loop at ~38 % MFMA occupancy (rocprofv3
// SQ_VALU_MFMA_BUSY_CYCLES, scripts/wgrad_stamps.py).  Every wave issues 2-3
// of a stage's 28 DMA instructions.  Split partials as [splits][Cout][Kp] (the common reduce),
// staged through LDS so each thread stores 16-byte runs along k.
constexpr int WGH_PROWS = 160;                  // patch rows per stage (5 DMA rounds of 32)
constexpr int WGH_XB = WGH_PROWS * 128;         // dy tile offset within a stage
constexpr int WGH_STAGE = (64 + WGH_PROWS) * 128;  // patch + dy tile: 28 KB
constexpr int WGH_RING = 5;                     // 140 KB: four stages in flight
constexpr int WGH_CS = 68;                      // C staging row stride (floats)
constexpr int WGH_NT = 768;                     // threads per block
static_assert(3 * 64 * WGH_CS * 4 <= WGH_RING * WGH_STAGE, "C staging fits the ring");

// patch swizzle (even: keeps a lane's 32-B chunk pair): column bits 1 and 3,
// the latter XOR the image row's parity
__device__ __forceinline__ int wgh_swz(int ir, int ic) {
  return (((ic >> 1) & 1) | ((((ic >> 3) ^ ir) & 1) << 1)) << 1;
}

__device__ __forceinline__ void wgrad_halo_body(const WgParams& p, char* smem, const VB& vb) {
  typedef __attribute__((address_space(3))) char lds_char;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_char*)smem;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int kh = __builtin_amdgcn_readfirstlane(wid >> 2);  // this wave's filter row
  const int wq = wid & 3, wm = wq >> 1, wn = wq & 1;
  // XCD-aware block order: hardware block b runs on XCD b % 8; each XCD gets a
  // contiguous run of (co tile, ci tile, split) in that order, so the blocks
  // that read the same x chunk / dy chunk of a split share an L2
  const int gx = vb.gx, gy = vb.gy;
  const int nwg = gx * gy * vb.gz;
  const int bid = vb.lin();
  int wg = bid;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int bx = wg % gx, by = (wg / gx) % gy, bz = wg / (gx * gy);
  const int co0 = bx * 64;
  const int ci0 = by * 64;
  const int zset = bz / p.zsp;
  const int m_begin = (bz - zset * p.zsp) * p.m_per_split;
  const int m_end = min(p.M, m_begin + p.m_per_split);
  const bf16_t* const dyp = p.dy + (int64_t)zset * p.M * p.Cout;
  const bf16_t* const zero = (const bf16_t*)g_wg_zero16;
  const int W = p.W, H = p.H, HW = H * W;
  const int RH = p.h_rh, PW = W + 2, PHPW = (RH + 2) * PW, P = p.h_img * PHPW;
  wg_stamp(p, 0, vb);

  // Stage layout: patch rows [0, 160) (byte 0), dy rows after (byte WGH_XB).
  // A DMA instruction writes 8 rows of 128 B (lane-linear);
  // LDS slot tid & 7 of a row holds global 16-B chunk slot ^ swizzle.  dy rows
  // (read at aligned row groups) use wg_swz(row); patch rows use
  // wgh_swz(image row, column): the tap views read rows at any shift, and
  // keying the XOR on the pixel's column bits 1 / 3 and its image row's
  // parity keeps every 32-lane transposing read conflict-free for W = 8, 16
  // and 32 (a row-index key conflicts 2-way at W = 8).
  // Waves 0-3 issue the stage DMAs (7 per wave): round j of 32 rows covers
  // patch rows 32 j .. (j < 5), then dy rows (j = 5, 6).  (Spreading the 28
  // DMA instructions over all 12 waves measured slower: loop 10.0 vs 9.0 us.)
  const int trow = (tid & 255) >> 3, slot = tid & 7;
  const bool loader = wid < 4;
  const uint32_t wave_off = (uint32_t)__builtin_amdgcn_readfirstlane(wq) * 1024u;
  int d_off[2];
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    const int r = trow + 32 * d;
    d_off[d] = r * p.Cout + co0 + ((slot ^ wg_swz(r)) << 3);
  }
  int x_rel[5], x_ir[5];
  bool x_ok[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int pr = trow + 32 * j;
    const int img = pr / PHPW, rem = pr - img * PHPW;
    const int ir = rem / PW, ic = rem - ir * PW;
    x_ok[j] = pr < P && (unsigned)(ic - 1) < (unsigned)W;
    x_ir[j] = pr < P ? ir - 1 : -(1 << 20);
    x_rel[j] = ((img * H + ir - 1) * W + ic - 1) * p.Cin + ci0 + ((slot ^ wgh_swz(ir, ic)) << 3);
  }

  auto issue = [&](int mb, int buf) {  // stage of 64 pixels from mb (7 DMAs per loader wave)
    if (!loader) return;
    const uint32_t base = lds0 + (uint32_t)(buf * WGH_STAGE) + wave_off;
    const bool live = mb < m_end;
    const int mm = live ? mb : 0;
    const int n0 = mm / HW, oh0 = (mm - n0 * HW) / W;
    const bf16_t* xb = p.x + ((int64_t)n0 * HW + oh0 * W) * p.Cin;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const bool ok = live && x_ok[j] && (unsigned)(oh0 + x_ir[j]) < (unsigned)H;
      wg_glds16(ok ? xb + x_rel[j] : zero, base + (uint32_t)(j * 4096));
    }
#pragma unroll
    for (int d = 0; d < 2; ++d)
      wg_glds16(live ? dyp + ((int64_t)mm * p.Cout + d_off[d]) : zero,
                base + (uint32_t)(WGH_XB + d * 4096));
  };

  f32x4 acc[3][2][2];  // [kw][co 16-block][ci 16-block]
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[t][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // Transposing reads: lane 16 g + 4 q + pp supplies the address of pixel
  // 8 g + q (lo) / 8 g + q + 4 (hi) of a 32-pixel half, 8 bytes at column
  // c0 + 4 pp, and receives column c0 + (lane & 15) of pixels 8 g .. 8 g + 7.
  // Every address within a stage is fixed per lane, so they are made here.
  // The second 16-column fragment of a wave (chunk + 2) is the first one's
  // address XOR 32: the lane's chunk c has bit 1 clear and every swizzle is
  // even, so (c + 2) ^ s = (c ^ s) ^ 2.
  const int fg = lane >> 4, fq = (lane >> 2) & 3, fp = lane & 3;
  int xa[2][3][2];  // [kk][kw][lo/hi]: patch byte offsets of fragment 0
  int da[2][2];     // [kk][lo/hi]: dy byte offsets of fragment 0
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int m = kk * 32 + 8 * fg;  // 8 consecutive pixels in one image row (W % 8 == 0)
    const int img = m / (RH * W), rr = m - img * RH * W;
    const int r = rr / W, c = rr - r * W + fq;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ir = r + kh, ic = c + kw + 4 * h;
        const int row = img * PHPW + ir * PW + ic;
        xa[kk][kw][h] = row * 128 + (((wn * 4 + (fp >> 1)) ^ wgh_swz(ir, ic)) << 4) + (fp & 1) * 8;
      }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = kk * 32 + 8 * fg + fq + 4 * h;
      da[kk][h] = WGH_XB + row * 128 + (((wm * 4 + (fp >> 1)) ^ wg_swz(row)) << 4) + (fp & 1) * 8;
    }
  }
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  auto rd2 = [&](const char* base, int lo, int hi) {
    s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + lo));
    s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + hi));
    bf16x8 out;
    short* o = (short*)&out;
    o[0] = a[0]; o[1] = a[1]; o[2] = a[2]; o[3] = a[3];
    o[4] = b[0]; o[5] = b[1]; o[6] = b[2]; o[7] = b[3];
    return out;
  };
  auto compute = [&](const char* S) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[2];
      af[0] = rd2(S, da[kk][0], da[kk][1]);
      af[1] = rd2(S, da[kk][0] ^ 32, da[kk][1] ^ 32);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        bf16x8 bfr[2];
        bfr[0] = rd2(S, xa[kk][kw][0], xa[kk][kw][1]);
        bfr[1] = rd2(S, xa[kk][kw][0] ^ 32, xa[kk][kw][1] ^ 32);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[kw][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[kw][i][j], 0, 0, 0);
      }
    }
  };

  const int n = (m_end - m_begin + 63) / 64;
#pragma unroll
  for (int s0 = 0; s0 < WGH_RING - 1; ++s0) issue(m_begin + s0 * 64, s0);
  wg_stamp(p, 1, vb);
  int cbuf = 0;
  for (int t = 0; t < n; ++t) {
    // loaders: stage t landed (the 7 DMAs of each of the RING - 2 younger
    // stages still in flight); the barrier publishes it and retires every
    // wave's reads of the slot stage t + RING - 1 overwrites (stage t - 1's)
    wg_wait_barrier<7 * (WGH_RING - 2)>();
    if (t == 0) wg_stamp(p, 2, vb);
    const int ibuf = cbuf == 0 ? WGH_RING - 1 : cbuf - 1;  // (t + RING - 1) % RING
    issue(m_begin + (t + WGH_RING - 1) * 64, ibuf);
    compute(smem + cbuf * WGH_STAGE);
    cbuf = cbuf == WGH_RING - 1 ? 0 : cbuf + 1;
  }
  wg_wait_barrier<0>();  // zero-page prefetches drained, every fragment read retired
  wg_stamp(p, 3, vb);

  // partials: round kw stages the three taps (kh, kw) of all groups, then
  // 16-byte stores along k (partial[z][co][tap * Cin + ci])
  float* Cs = (float*)smem;
  const int ecol = lane & 15, erow = (lane >> 4) * 4;
  float* const dst0 = p.partial + ((int64_t)bz * p.Cout + co0) * p.Kp + ci0;
#pragma unroll
  for (int kw = 0; kw < 3; ++kw) {
    if (kw) __syncthreads();  // the previous round's stores have read the staging area
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Cs[(kh * 64 + wm * 32 + i * 16 + erow + r) * WGH_CS + wn * 32 + j * 16 + ecol] = acc[kw][i][j][r];
    __syncthreads();
    for (int f = tid; f < 3 * 1024; f += WGH_NT) {
      const int g = f >> 10, rem = f & 1023, row = rem >> 4, c4 = rem & 15;
      const float4 v = *(const float4*)&Cs[(g * 64 + row) * WGH_CS + 4 * c4];
      *(float4*)(dst0 + (int64_t)row * p.Kp + (3 * g + kw) * p.Cin + 4 * c4) = v;
    }
  }
  if (p.stamps != nullptr) {
    __syncthreads();
    wg_stamp(p, 4, vb);
  }
}

__global__ void __launch_bounds__(WGH_NT)
conv_wgrad_halo_kernel(const WgParams p) {
  __shared__ __attribute__((aligned(16))) char smem[WGH_RING * WGH_STAGE];
  wgrad_halo_body(p, smem, vb_hw());
}

// ---------------------------------------------------------------------------
// A weight-gradient GEMM and the streaming BN-backward apply of the layer
// below it in ONE launch (mda_conv_wgrad_nored_bn).  Neither depends on the
// other -- the GEMM reads this conv's dy and x, the apply reads the dgrad
// output of this conv -- and back to back each left most CUs idle (the
// flagship's backward: 128-512-block applies after 16-288-block GEMMs).
// Blocks [0, nw) are the GEMM's (x-fastest order of its 3-D grid), the rest
// the apply's; the apply runs with the GEMM's block size and reuses its LDS.
template <int MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
wgrad_reg_bn_kernel(const WgParams p, const BwdArgs a, int gx, int gy, int gz) {
  __shared__ __attribute__((aligned(16))) char smem[WG_REG_SMEM];
  const int nw = gx * gy * gz, b = blockIdx.x;
  if (b < nw) wgrad_reg_body<MODE>(p, smem, vb_lin(b, gx, gy, gz));
  else bn_bwd_apply_body<4>(a, (float*)smem, b - nw, (int)gridDim.x - nw);
}

template <int TCo, int TKk>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WgOcc<TCo, TKk>::W)))
wgrad_glds_bn_kernel(const WgParams p, const BwdArgs a, int gx, int gy, int gz) {
  __shared__ __attribute__((aligned(16))) char smem[WgGlds<TCo, TKk>::BYTES];
  const int nw = gx * gy * gz, b = blockIdx.x;
  if (b < nw) wgrad_glds_body<TCo, TKk>(p, smem, vb_lin(b, gx, gy, gz));
  else bn_bwd_apply_body<4>(a, (float*)smem, b - nw, (int)gridDim.x - nw);
}

__global__ void __launch_bounds__(WGH_NT)
wgrad_halo_bn_kernel(const WgParams p, const BwdArgs a, int gx, int gy, int gz) {
  __shared__ __attribute__((aligned(16))) char smem[WGH_RING * WGH_STAGE];
  const int nw = gx * gy * gz, b = blockIdx.x;
  if (b < nw) wgrad_halo_body(p, smem, vb_lin(b, gx, gy, gz));
  else bn_bwd_apply_body<4>(a, (float*)smem, b - nw, (int)gridDim.x - nw);
}

// grad[co][ci][kh][kw] (+)= scale * sum_s partial[s][co][(kh*KW+kw)*Cin+ci]
// Block = 16 float4 columns (64 packed (co, k) elements) x 16 set-slices:
// thread (c, sl) sums the partial sets s = sl (mod 16), two loads in flight,
// and the 16 slice sums combine in a fixed order (deterministic).  With up to
// 128 sets per layer the earlier 4-slice version walked ~30 dependent loads
// per thread (14 us per ResNet-18 layer); this one issues ~8.
// Slices per block adapt to the split count (round 3): S = 1 for <= 8 sets
// (each thread sums all sets of ONE float4 column: 256 columns per block),
// up to 16 for > 64 sets (16 columns per block, as before).  The flagship's
// deferred multi-layer reduce was 18,944 blocks of 64 elements each: 29 us.
__host__ __device__ __forceinline__ int wgr_slices(int splits) {
  return splits <= 8 ? 1 : splits <= 16 ? 2 : splits <= 32 ? 4 : splits <= 64 ? 8 : 16;
}
__host__ __device__ __forceinline__ int wgr_cols(int splits) { return 256 / wgr_slices(splits); }

__device__ __forceinline__ void wgrad_reduce_block(
    int64_t blk, const float* __restrict__ partial, float* __restrict__ grad, int splits, int Cout,
    int Cin, int KH, int KW, int Kp, float scale, int accumulate, int cin_keep, int groups) {
  __shared__ float4 red[256];
  const int S = wgr_slices(splits), CP = 256 / S;
  const int c = threadIdx.x % CP, sl = threadIdx.x / CP;
  const int64_t total4 = (int64_t)Cout * Kp / 4;
  const int64_t e4 = blk * CP + c;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e4 < total4) {
    const float4* src = (const float4*)partial + e4;
    float4 b = a;
    int s = sl;
    for (; s + S < splits; s += 2 * S) {
      const float4 u0 = src[(int64_t)s * total4], u1 = src[(int64_t)(s + S) * total4];
      a.x += u0.x; a.y += u0.y; a.z += u0.z; a.w += u0.w;
      b.x += u1.x; b.y += u1.y; b.z += u1.z; b.w += u1.w;
    }
    if (s < splits) {
      const float4 u = src[(int64_t)s * total4];
      a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
    }
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  float v[4] = {a.x, a.y, a.z, a.w};
  if (S > 1) {
    red[sl * CP + c] = a;
    __syncthreads();
    if (sl != 0 || e4 >= total4) return;
    v[0] = v[1] = v[2] = v[3] = 0.f;
    for (int q = 0; q < S; ++q) {
      const float4 r = red[q * CP + c];
      v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
    }
  } else if (e4 >= total4) {
    return;
  }
  const int K = Cin * KH * KW;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t e = e4 * 4 + q;
    const int co = (int)(e / Kp);
    const int k = (int)(e - (int64_t)co * Kp);   // packed order: (kh*KW + kw)*Cin + ci
    if (k >= K) continue;                        // padding columns
    const int tap = k / Cin, ci = k - tap * Cin;
    // channel-padded stems (Cin 3 -> 8): only the real input channels exist in grad
    if (ci >= cin_keep) continue;
    int ciw = ci, cin_w = cin_keep;
    if (groups > 1) {  // block-diagonal dense product: keep the co's own group
      const int cin_g = Cin / groups, g = co / (Cout / groups);
      if (ci / cin_g != g) continue;
      ciw = ci - g * cin_g;
      cin_w = cin_g;
    }
    const int64_t dst = ((int64_t)co * cin_w + ciw) * KH * KW + tap;
    grad[dst] = (accumulate ? grad[dst] : 0.f) + scale * v[q];
  }
}

__global__ void __launch_bounds__(256)
wgrad_reduce_kernel(const float* __restrict__ partial, float* __restrict__ grad, int splits,
                    int Cout, int Cin, int KH, int KW, int Kp, float scale, int accumulate,
                    int cin_keep, int groups) {
  wgrad_reduce_block(blockIdx.x, partial, grad, splits, Cout, Cin, KH, KW, Kp, scale, accumulate,
                     cin_keep, groups);
}

// The split reductions of up to WGRM_MAX layers in ONE launch (the deferred
// reduces of a captured backward: engine/step.py flushes them once the last
// weight-gradient GEMM is queued).  Layers passed by value; block b belongs to
// the layer whose [blk0, blk0 + blocks) range holds it.
constexpr int WGRM_MAX = 32;
struct WgrLayer {
  const float* partial;
  float* grad;
  int splits, Cout, Cin, KH, KW, Kp, accumulate, cin_keep, groups, blk0;
  float scale;
  int dw;  // depthwise layer: partial [splits][KH*KW][Cout] -> grad [Cout][KH*KW]
};

// Depthwise split sums (csrc/dwconv.hip dw_wgrad_finalize_kernel's reduction,
// same order: 8 slices x 32 elements, fp64), so a captured backward can defer
// them into the one multi-layer reduce as well.
__device__ __forceinline__ void dw_reduce_block(int64_t blk, const float* __restrict__ partial,
                                                int nblk, int KK, int C, float* __restrict__ grad,
                                                int accumulate) {
  __shared__ double dred[8][32];
  const int64_t V = (int64_t)KK * C;
  const int e = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const int64_t i = blk * 32 + e;
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
  dred[sl][e] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (sl != 0 || i >= V) return;
  const double sum = ((dred[0][e] + dred[1][e]) + (dred[2][e] + dred[3][e])) +
                     ((dred[4][e] + dred[5][e]) + (dred[6][e] + dred[7][e]));
  const int t = (int)(i / C), c = (int)(i - (int64_t)t * C);
  float* o = grad + (int64_t)c * KK + t;
  *o = accumulate ? *o + (float)sum : (float)sum;
}
struct WgrTable {
  WgrLayer l[WGRM_MAX];
  int n;
};

__global__ void __launch_bounds__(256) wgrad_reduce_multi_kernel(const WgrTable t) {
  int i = 0;
  while (i + 1 < t.n && (int)blockIdx.x >= t.l[i + 1].blk0) ++i;
  const WgrLayer& L = t.l[i];
  if (L.dw) {
    dw_reduce_block(blockIdx.x - L.blk0, L.partial, L.splits, L.KH * L.KW, L.Cout, L.grad,
                    L.accumulate);
    return;
  }
  wgrad_reduce_block(blockIdx.x - L.blk0, L.partial, L.grad, L.splits, L.Cout, L.Cin, L.KH, L.KW,
                     L.Kp, L.scale, L.accumulate, L.cin_keep, L.groups);
}

__global__ void __launch_bounds__(256)
pack_kernel(const float* __restrict__ w, bf16_t* __restrict__ wf, bf16_t* __restrict__ wt,
            int Cout, int Cin, int KH, int KW, int Kp, int KpT) {
  // one thread per packed-forward element (including the zero padding)
  const int64_t total = (int64_t)Cout * Kp;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int co = (int)(i / Kp);
    const int k = (int)(i - (int64_t)co * Kp);
    float v = 0.f;
    if (k < KH * KW * Cin) {
      const int tap = k / Cin, ci = k - (k / Cin) * Cin;
      const int kh = tap / KW, kw = tap - kh * KW;
      v = w[(((int64_t)co * Cin + ci) * KH + kh) * KW + kw];
      if (wt) wt[(int64_t)ci * KpT + tap * Cout + co] = f2bf(v);
    }
    wf[i] = f2bf(v);
  }
  if (wt) {  // zero the dgrad padding columns
    const int64_t pad = (int64_t)Cin * (KpT - KH * KW * Cout);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < pad;
         i += (int64_t)gridDim.x * blockDim.x) {
      const int w_ = KpT - KH * KW * Cout;
      const int ci = (int)(i / w_);
      const int j = (int)(i - (int64_t)ci * w_);
      wt[(int64_t)ci * KpT + KH * KW * Cout + j] = 0;
    }
  }
}

// All layers of a network in one launch, as tiled transposes through LDS.
// table[l] = {w, wf, wt (0 = none), Cout, Cin, KH, KW, Kp, KpT, tile0} (int64),
// tile0 = first tile of layer l.  A tile is T co x T ci x all taps
// (T = 32 for 1x1, 16 up to 3x3, 8 for larger kernels: many small blocks, the
// pack of a CIFAR student is only ~100 K weights), loaded with
// coalesced reads of the OIHW fp32 rows (taps contiguous per (co, ci)) and
// written as T-long contiguous runs of both packed layouts:
//   wf[co][tap*Cin + ci]   and   wt[ci][tap*Cout + co].
// Depthwise layers ride along (Cin = -1 rows): fp32 [C,1,3,3] -> tap-major
// [9, C] (csrc/dwconv.hip's operand), 256 elements per tile.  So does the
// rest of the step's prologue, each one launch less in the captured chain:
//   Cin = -2  channel-padded stem operand {w, wf, 0, Cout, -2, KH, KW, Kp,
//             C | Cp << 16}: wf[co][tap*Cp + ci], 256 elements per tile
//   Cin = -3  zero fill {ptr, nbytes (multiple of 4)}: 16 KB per tile (the
//             flat gradients and the step's BN-region arena)
//   Cin = -4  image pad {x, y, dt, M, -4, C}: [M, C] fp32/bf16 NHWC ->
//             [M, 8] bf16 (zeros beyond C), 256 pixels per tile
// Padding columns (k >= K, and the dgrad tail) are never touched: they are
// zeroed once by the per-layer pack at registration and stay zero.
// (The previous element-per-thread version scattered 2-byte stores at
// stride KpT and took 232 us for a ResNet-18.)
constexpr int PACK_MAX_LAYERS = 256;
constexpr int PACK_FIELDS = 10;
constexpr int PACK_LDS_FLOATS = 13056;  // >= max over T of T*(T*KHKW + 1)

__device__ __forceinline__ int pack_tile_dim(int khkw) {
  return khkw == 1 ? 32 : (khkw <= 9 ? 16 : 8);
}

// Dynamic LDS, sized on the host for THIS table (its rows and its largest
// tile): a CIFAR student's table + a 3x3 tile is ~10 KB, so many blocks share
// a CU and their load -> transpose -> store chains overlap (the static
// worst-case 72 KB allowed two blocks per CU: 22 us for a ResNet8x4).
__global__ void __launch_bounds__(256)
pack_multi_kernel(const int64_t* __restrict__ table, int L) {
  extern __shared__ __attribute__((aligned(16))) char pack_dyn[];
  int64_t* tb = (int64_t*)pack_dyn;
  float* sm = (float*)(pack_dyn + ((L * PACK_FIELDS * 8 + 15) / 16) * 16);
  for (int i = threadIdx.x; i < L * PACK_FIELDS; i += blockDim.x) tb[i] = table[i];
  __syncthreads();
  int l = 0;
  while (l + 1 < L && (int64_t)blockIdx.x >= tb[(l + 1) * PACK_FIELDS + 9]) ++l;
  const int64_t* e = tb + l * PACK_FIELDS;
  if (e[4] < 0) {  // block-uniform branches (l depends on blockIdx only)
    const int64_t t = (int64_t)blockIdx.x - e[9];
    if (e[4] == -1) {  // depthwise {w [C,1,3,3], dst fp32 [9, C], 0, C, -1}
      const float* w = (const float*)e[0];
      float* dst = (float*)e[1];
      const int C = (int)e[3];
      const int i = (int)t * 256 + threadIdx.x;
      if (i < 9 * C) dst[i] = w[(i % C) * 9 + i / C];
    } else if (e[4] == -2) {  // channel-padded stem operand
      const float* w = (const float*)e[0];
      bf16_t* wf = (bf16_t*)e[1];
      const int Cout = (int)e[3], KH = (int)e[5], KW = (int)e[6], Kp = (int)e[7];
      const int C = (int)(e[8] & 0xffff), Cp = (int)(e[8] >> 16);
      const int64_t i = t * 256 + threadIdx.x;
      if (i < (int64_t)Cout * Kp) {
        const int co = (int)(i / Kp), k = (int)(i - (int64_t)co * Kp);
        float v = 0.f;
        if (k < KH * KW * Cp) {
          const int tap = k / Cp, ci = k - tap * Cp;
          if (ci < C) v = w[(((int64_t)co * C + ci) * KH + tap / KW) * KW + tap % KW];
        }
        wf[i] = f2bf(v);
      }
    } else if (e[4] == -3) {  // zero fill: 16-byte stores, 4-byte tail
      char* base = (char*)e[0];
      const int64_t nb = e[1];
      const int64_t o0 = t * 16384;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t o = o0 + ((int64_t)r * 256 + threadIdx.x) * 16;
        if (o + 16 <= nb) {
          *(uint4*)(base + o) = make_uint4(0u, 0u, 0u, 0u);
        } else if (o < nb) {
          for (int64_t q = o; q < nb; q += 4) *(uint32_t*)(base + q) = 0u;
        }
      }
    } else {  // image pad to 8 channels
      const int64_t M = e[3];
      const int C = (int)e[5];
      const int64_t m = t * 256 + threadIdx.x;
      if (m < M) {
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (e[2] == DT_F32) {
          const float* x = (const float*)e[0];
          for (int c = 0; c < C; ++c) v[c] = x[m * C + c];
        } else {
          const bf16_t* x = (const bf16_t*)e[0];
          for (int c = 0; c < C; ++c) v[c] = bf2f(x[m * C + c]);
        }
        *(uint4*)((bf16_t*)e[1] + m * 8) = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                                      pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
      }
    }
    return;
  }
  const float* w = (const float*)e[0];
  bf16_t* wf = (bf16_t*)e[1];
  bf16_t* wt = (bf16_t*)e[2];
  const int Cout = (int)e[3], Cin = (int)e[4], KHKW = (int)(e[5] * e[6]);
  const int Kp = (int)e[7], KpT = (int)e[8];
  const int T = pack_tile_dim(KHKW);
  const int tci = (Cin + T - 1) / T;
  const int t = (int)(blockIdx.x - e[9]);
  const int co0 = (t / tci) * T, ci0 = (t - (t / tci) * tci) * T;
  const int nco = min(T, Cout - co0), nci = min(T, Cin - ci0);
  const int RS = T * KHKW + 1;  // LDS row stride (odd: conflict-free column walks)
  // load: rows co0..co0+nco, each a contiguous run of nci*KHKW floats
  const int run = nci * KHKW;
  for (int i = threadIdx.x; i < nco * run; i += blockDim.x) {
    const int r = i / run, c = i - (i / run) * run;
    sm[r * RS + c] = w[((int64_t)(co0 + r) * Cin + ci0) * KHKW + c];
  }
  __syncthreads();
  // wf[co][tap*Cin + ci]: runs over ci
  for (int i = threadIdx.x; i < nco * KHKW * nci; i += blockDim.x) {
    const int r = i / (KHKW * nci), rem = i - r * (KHKW * nci);
    const int tap = rem / nci, ci = rem - tap * nci;
    wf[(int64_t)(co0 + r) * Kp + tap * Cin + ci0 + ci] = f2bf(sm[r * RS + ci * KHKW + tap]);
  }
  if (wt) {  // wt[ci][tap*Cout + co]: runs over co
    for (int i = threadIdx.x; i < nci * KHKW * nco; i += blockDim.x) {
      const int ci = i / (KHKW * nco), rem = i - ci * (KHKW * nco);
      const int tap = rem / nco, r = rem - tap * nco;
      wt[(int64_t)(ci0 + ci) * KpT + tap * Cout + co0 + r] = f2bf(sm[r * RS + ci * KHKW + tap]);
    }
  }
}

// Stem support: the 3-channel image conv would gather 2-byte elements one
// at a time; padding the input to 8 channels (zeros) puts it on the 16-byte
// vector loaders, at 8/3 the (tiny) stem MFMA work.
// x: [M, C] NHWC fp32 or bf16 -> y: [M, Cp] bf16, channels >= C zero.
template <typename T>
__global__ void __launch_bounds__(256)
pad_channels_kernel(const T* __restrict__ x, bf16_t* __restrict__ y, int64_t M, int C, int Cp) {
  for (int64_t m = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; m < M;
       m += (int64_t)gridDim.x * blockDim.x) {
    if (Cp == 8) {
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int c = 0; c < C; ++c) v[c] = io<T>::ld(x, m * C + c);
      *(uint4*)(y + m * 8) = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                        pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
    } else {
      for (int c = 0; c < Cp; ++c) y[m * Cp + c] = f2bf(c < C ? io<T>::ld(x, m * C + c) : 0.f);
    }
  }
}

// forward operand of a channel-padded conv: wf[co][(kh*KW+kw)*Cp + ci] =
// w[co][ci][kh][kw] for ci < C, else 0; k >= KH*KW*Cp zero.
__global__ void __launch_bounds__(256)
pack_pad_kernel(const float* __restrict__ w, bf16_t* __restrict__ wf, int Cout, int C, int Cp,
                int KH, int KW, int Kp) {
  const int64_t total = (int64_t)Cout * Kp;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int co = (int)(i / Kp), k = (int)(i - (i / Kp) * Kp);
    float v = 0.f;
    if (k < KH * KW * Cp) {
      const int tap = k / Cp, ci = k - tap * Cp;
      if (ci < C) v = w[(((int64_t)co * C + ci) * KH + tap / KW) * KW + tap % KW];
    }
    wf[i] = f2bf(v);
  }
}

}  // namespace

MDA_API int mda_pad_channels(int64_t dt, const void* x, void* y, int64_t M, int64_t C, int64_t Cp,
                             hipStream_t st) {
  if (C > Cp || C > 8 || M <= 0) return (int)hipErrorInvalidValue;
  const int blocks = (int)std::min<int64_t>((M + 255) / 256, 4096);
  if (dt == DT_F32)
    hipLaunchKernelGGL(pad_channels_kernel<float>, dim3(blocks), dim3(256), 0, st,
                       (const float*)x, (bf16_t*)y, M, (int)C, (int)Cp);
  else
    hipLaunchKernelGGL(pad_channels_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st,
                       (const bf16_t*)x, (bf16_t*)y, M, (int)C, (int)Cp);
  MDA_CHECK_LAUNCH();
}

MDA_API int mda_pack_conv_weights_pad(const float* w, void* wf, int64_t Cout, int64_t C, int64_t Cp,
                                      int64_t KH, int64_t KW, int64_t Kp, hipStream_t st) {
  if (C > Cp || Kp < KH * KW * Cp) return (int)hipErrorInvalidValue;
  const int64_t total = Cout * Kp;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 1024);
  hipLaunchKernelGGL(pack_pad_kernel, dim3(blocks), dim3(256), 0, st, w, (bf16_t*)wf, (int)Cout,
                     (int)C, (int)Cp, (int)KH, (int)KW, (int)Kp);
  MDA_CHECK_LAUNCH();
}

// total = number of tiles over all layers (see pack_multi_kernel; mda_pack_tiles
// gives a layer's count).  The packed buffers' padding must already be zero.
// khkw_max: the largest KH*KW of the table's layers (sizes the LDS tile).
MDA_API int mda_pack_conv_weights_multi(const int64_t* table, int64_t L, int64_t total,
                                        int64_t khkw_max, hipStream_t st) {
  if (L <= 0 || L > PACK_MAX_LAYERS || total <= 0 || total > (1 << 30) || khkw_max < 1 ||
      khkw_max > 49)
    return (int)hipErrorInvalidValue;
  int tile_floats = 256;  // a depthwise row's tile needs none; keep a floor
  for (int kk = 1; kk <= khkw_max; ++kk) {
    const int T = kk == 1 ? 32 : (kk <= 9 ? 16 : 8);
    tile_floats = std::max(tile_floats, T * (T * kk + 1));
  }
  const size_t lds = ((size_t)L * PACK_FIELDS * 8 + 15) / 16 * 16 + (size_t)tile_floats * 4;
  hipLaunchKernelGGL(pack_multi_kernel, dim3((unsigned)total), dim3(256), lds, st, table, (int)L);
  MDA_CHECK_LAUNCH();
}

// Tiles of one layer in mda_pack_conv_weights_multi.
MDA_API int mda_pack_tiles(int64_t Cout, int64_t Cin, int64_t KH, int64_t KW, int64_t* tiles) {
  const int64_t khkw = KH * KW;
  const int64_t T = khkw == 1 ? 32 : (khkw <= 9 ? 16 : 8);
  if (khkw > 49) return (int)hipErrorInvalidValue;  // PACK_LDS_FLOATS sizing
  *tiles = ((Cout + T - 1) / T) * ((Cin + T - 1) / T);
  return 0;
}

// Kernel / block tile of a wgrad, from the kernel-level A/B on the ResNet
// CIFAR and ImageNet shapes (profiles/r2_wgrad_ab.md): the LDS-DMA kernel with
// 128 x 128 tiles for wide 1x1 layers (64 x 64 for narrow ones), 64 x 128 for
// 3x3 layers with >= 20 K pixels; the register-staged kernel (0) for small-M
// 3x3 layers and the scalar stem gather.  MDA_WG_TILE=<code> forces a tile,
// MDA_WG_GLDS=0 the register-staged kernel.
static int wg_tile(int64_t M, int64_t Cout, int64_t Cin, int64_t KH, int64_t KW, int64_t Kp) {
  static const int forced = [] {
    const char* e = getenv("MDA_WG_TILE");
    return e ? atoi(e) : -1;
  }();
  static const bool glds = [] {
    const char* e = getenv("MDA_WG_GLDS");
    return !(e && e[0] == '0');
  }();
  if (Cin % 8 || !glds) return 0;
  if (forced == 0 || forced == 64064 || forced == 64128 || forced == 128064 || forced == 128128) return forced;
  if (KH * KW == 1) return (Cout >= 128 && Kp >= 128) ? 128128 : 64064;
  return M >= 20000 ? 64128 : 0;
}

// The halo kernel's stage geometry: 64 output pixels = img whole images of
// rh rows (false: not served).
static bool wg_halo_geom(int64_t H, int64_t W, int64_t* rh, int64_t* img) {
  if (W % 8 || W > 32 || H <= 0) return false;
  if (H * W >= 64) {
    if (64 % W || H % (64 / W)) return false;
    *rh = 64 / W;
    *img = 1;
  } else {
    if (64 % (H * W)) return false;
    *rh = H;
    *img = 64 / (H * W);
  }
  return *img * (*rh + 2) * (W + 2) <= WGH_PROWS;
}

static bool wg_halo_ok(int64_t M, int64_t Cout, int64_t Cin, int64_t KH, int64_t KW, int64_t H,
                       int64_t W, int64_t stride, int64_t pad) {
  static const bool on = [] {
    const char* e = getenv("MDA_WG_HALO");
    return !(e && e[0] == '0');
  }();
  int64_t rh, img;
  return on && KH == 3 && KW == 3 && stride == 1 && pad == 1 && Cin % 64 == 0 && Cout % 64 == 0 &&
         M % 64 == 0 && wg_halo_geom(H, W, &rh, &img);
}

// halo kernel splits: MDA_WGH_BLOCKS (default 128) blocks, >= 2 stages each
// Target GEMM blocks of a halo wgrad: 64 since round 6.  Its GEMM now shares
// a launch with a BN-backward apply (mda_conv_wgrad_nored_bn), so fewer,
// longer blocks (half the split partials for the deferred reduce) won:
// flagship 0.7707 -> 0.7605 ms/step (0.7678 -> 0.7614 in a second set); the
// student alone 0.6130 -> 0.6208 (profiles/r6_ab.md).  MDA_WGH_BLOCKS: A/B.
static int64_t wg_halo_splits(int64_t M, int64_t Cout, int64_t Cin) {
  static const int64_t target = [] {
    const char* e = getenv("MDA_WGH_BLOCKS");
    return e ? (int64_t)atoi(e) : (int64_t)64;
  }();
  const int64_t tiles = (Cout / 64) * (Cin / 64), stages = M / 64;
  int64_t sp = (target + tiles - 1) / tiles;
  sp = std::min<int64_t>(sp, std::max<int64_t>(1, stages / 2));
  return std::max<int64_t>(1, std::min<int64_t>(sp, 128));
}

MDA_API int mda_wgrad_plan(int64_t M, int64_t Cout, int64_t Cin, int64_t KH, int64_t KW, int64_t Kp,
                           int64_t H, int64_t W, int64_t stride, int64_t pad, int64_t* splits) {
  if (wg_halo_ok(M, Cout, Cin, KH, KW, H, W, stride, pad)) {
    *splits = wg_halo_splits(M, Cout, Cin);
    return 0;
  }
  const int tile = wg_tile(M, Cout, Cin, KH, KW, Kp);
  int64_t sp = 1;
  if (tile == 0) {
    // register-staged kernel: >= 256 workgroups, >= 4 stages (256 pixels) per split
    const int64_t tiles = ((Cout + TC - 1) / TC) * ((Kp + TK - 1) / TK);
    while (tiles * sp < 256 && (M / (sp * 2)) >= 4 * TM && sp < 64) sp *= 2;
  } else {
    const int tc = tile / 1000, tk = tile % 1000;
    const int64_t tiles = ((Cout + tc - 1) / tc) * ((Kp + tk - 1) / tk);
    // one round of blocks over the CU slots (LDS-limited blocks per CU), each
    // split >= 8 stages of 64 pixels, at most 128 partial sets
    const int64_t occ = tile == 128128 ? 1 : (tile == 64064 ? 3 : 2);
    static const int64_t slots = [] {  // CU slots to fill (MDA_WG_SLOTS, A/B)
      const char* e = getenv("MDA_WG_SLOTS");
      return e ? (int64_t)atoi(e) : (int64_t)256;
    }();
    sp = (slots * occ + tiles - 1) / tiles;
    sp = std::min<int64_t>(sp, std::max<int64_t>(1, M / (8 * TM)));
    sp = std::max<int64_t>(1, std::min<int64_t>(sp, 128));
  }
  *splits = sp;
  return 0;
}

// partial: splits*Cout*Kp floats.  grad: fp32 OIHW, accumulated when accumulate != 0.
static int conv_wgrad_impl(const void* x, const void* dy, float* partial, float* grad, int64_t N,
                           int64_t H, int64_t W, int64_t Cin, int64_t Ho, int64_t Wo, int64_t Cout,
                           int64_t KH, int64_t KW, int64_t stride, int64_t pad, int64_t Kp,
                           int64_t splits, float scale, int64_t accumulate, int64_t cin_keep,
                           int64_t groups, hipStream_t st, bool reduce, int64_t nsets,
                           int64_t gstride, const BwdArgs* fuse = nullptr) {
  if (Cout % 8 || Kp % TK || nsets < 1 || nsets > 2) return (int)hipErrorInvalidValue;
  if (fuse != nullptr && (reduce || nsets != 1)) return MDA_NOT_SERVED;
  if (cin_keep <= 0 || cin_keep > Cin) cin_keep = Cin;
  if (groups > 1 && (Cin % groups || Cout % groups)) return (int)hipErrorInvalidValue;
  WgParams p;
  p.x = (const bf16_t*)x; p.dy = (const bf16_t*)dy; p.partial = partial;
  p.N = N; p.H = H; p.W = W; p.Cin = Cin; p.Ho = Ho; p.Wo = Wo; p.Cout = Cout; p.KH = KH;
  p.KW = KW; p.stride = stride; p.pad = pad; p.K = KH * KW * Cin; p.Kp = Kp; p.M = N * Ho * Wo;
  const int64_t xb = N * H * W * Cin * 2, db = N * Ho * Wo * Cout * 2;
  if (xb >= ((int64_t)1 << 31) || db >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  p.x_bytes = (int)xb;
  p.dy_bytes = (int)db;
  p.stamps = g_stamps;
  p.div_howo = make_fastdiv((uint32_t)(Ho * Wo));
  p.div_wo = make_fastdiv((uint32_t)Wo);
  if (splits <= 0) mda_wgrad_plan(p.M, Cout, Cin, KH, KW, Kp, H, W, stride, pad, &splits);
  p.m_per_split = (int)(((p.M + splits - 1) / splits + TM - 1) / TM * TM);
  p.zsp = (int)splits;
  const int mode = (Cin % TK == 0) ? WG_FAST : (Cin % 8 == 0 ? WG_VEC8 : WG_SCALAR);
  dim3 grid((int)((Cout + TC - 1) / TC), (int)(Kp / TK), (int)(splits * nsets));
  const int tile = mode == WG_SCALAR ? 0 : wg_tile(p.M, Cout, Cin, KH, KW, Kp);
  int64_t hrh = 0, himg = 0;
  // fused launch (fuse != null): the GEMM's blocks, then nbn apply blocks
  // of the next BN backward, if its operands fit the GEMM's LDS
  const int nbn = fuse ? apply_blocks((int64_t)fuse->M * fuse->C / 8, 4) : 0;
  auto fits = [&](int64_t lds, int nt) {
    return bn_apply_lds_bytes(fuse->C, nt, fuse->rreg != nullptr) <= lds;
  };
  if (groups <= 1 && cin_keep == Cin && Kp == 9 * Cin &&
      wg_halo_ok(p.M, Cout, Cin, KH, KW, H, W, stride, pad) && wg_halo_geom(H, W, &hrh, &himg)) {
    p.h_rh = (int)hrh;
    p.h_img = (int)himg;
    dim3 gh((int)(Cout / 64), (int)(Cin / 64), (int)(splits * nsets));
    if (fuse) {
      if (!fits(WGH_RING * WGH_STAGE, WGH_NT)) return MDA_NOT_SERVED;
      const int nw = (int)(gh.x * gh.y * gh.z);
      hipLaunchKernelGGL(wgrad_halo_bn_kernel, dim3(nw + nbn), dim3(WGH_NT), 0, st, p, *fuse,
                         (int)gh.x, (int)gh.y, (int)gh.z);
      return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(conv_wgrad_halo_kernel, gh, dim3(WGH_NT), 0, st, p);
  } else if (tile != 0 && fuse) {
    const int tc = tile / 1000, tk = tile % 1000;
    dim3 g2((int)((Cout + tc - 1) / tc), (int)((Kp + tk - 1) / tk), (int)(splits * nsets));
    const int nw = (int)(g2.x * g2.y * g2.z);
#define WG_FUSED_GLDS(TC_, TK_)                                                                  \
  if (!fits(WgGlds<TC_, TK_>::BYTES, 256)) return MDA_NOT_SERVED;                               \
  hipLaunchKernelGGL((wgrad_glds_bn_kernel<TC_, TK_>), dim3(nw + nbn), dim3(256), 0, st, p, *fuse, \
                     (int)g2.x, (int)g2.y, (int)g2.z);
    switch (tile) {
      case 128128: { WG_FUSED_GLDS(128, 128) break; }
      case 128064: { WG_FUSED_GLDS(128, 64) break; }
      case 64128: { WG_FUSED_GLDS(64, 128) break; }
      default: { WG_FUSED_GLDS(64, 64) break; }
    }
#undef WG_FUSED_GLDS
    return (int)hipGetLastError();
  } else if (fuse) {
    if (!fits(WG_REG_SMEM, 256)) return MDA_NOT_SERVED;
    const int nw = (int)(grid.x * grid.y * grid.z);
    if (mode == WG_FAST)
      hipLaunchKernelGGL(wgrad_reg_bn_kernel<WG_FAST>, dim3(nw + nbn), dim3(256), 0, st, p, *fuse,
                         (int)grid.x, (int)grid.y, (int)grid.z);
    else if (mode == WG_VEC8)
      hipLaunchKernelGGL(wgrad_reg_bn_kernel<WG_VEC8>, dim3(nw + nbn), dim3(256), 0, st, p, *fuse,
                         (int)grid.x, (int)grid.y, (int)grid.z);
    else
      hipLaunchKernelGGL(wgrad_reg_bn_kernel<WG_SCALAR>, dim3(nw + nbn), dim3(256), 0, st, p, *fuse,
                         (int)grid.x, (int)grid.y, (int)grid.z);
    return (int)hipGetLastError();
  } else if (tile != 0) {
    const int tc = tile / 1000, tk = tile % 1000;
    dim3 g2((int)((Cout + tc - 1) / tc), (int)((Kp + tk - 1) / tk), (int)(splits * nsets));
    switch (tile) {
      case 128128: hipLaunchKernelGGL((conv_wgrad_glds_kernel<128, 128>), g2, dim3(256), 0, st, p); break;
      case 128064: hipLaunchKernelGGL((conv_wgrad_glds_kernel<128, 64>), g2, dim3(256), 0, st, p); break;
      case 64128: hipLaunchKernelGGL((conv_wgrad_glds_kernel<64, 128>), g2, dim3(256), 0, st, p); break;
      default: hipLaunchKernelGGL((conv_wgrad_glds_kernel<64, 64>), g2, dim3(256), 0, st, p); break;
    }
  } else if (mode == WG_FAST)
    hipLaunchKernelGGL(conv_wgrad_kernel<WG_FAST>, grid, dim3(256), 0, st, p);
  else if (mode == WG_VEC8)
    hipLaunchKernelGGL(conv_wgrad_kernel<WG_VEC8>, grid, dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL(conv_wgrad_kernel<WG_SCALAR>, grid, dim3(256), 0, st, p);
  int rc = (int)hipGetLastError();
  if (rc || !reduce) return rc;
  const int64_t total4 = Cout * Kp / 4;  // Kp % 64 == 0
  const int cp = wgr_cols((int)splits);
  const int blocks = (int)((total4 + cp - 1) / cp);
  for (int64_t k = 0; k < nsets; ++k) {
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st,
                       partial + k * splits * Cout * Kp, grad + k * gstride,
                       (int)splits, (int)Cout, (int)Cin, (int)KH, (int)KW, (int)Kp, scale,
                       (int)accumulate, (int)cin_keep, (int)(groups > 1 ? groups : 1));
    const int rc2 = (int)hipGetLastError();
    if (rc2) return rc2;
  }
  return 0;
}

MDA_API int mda_conv_wgrad(const void* x, const void* dy, float* partial, float* grad, int64_t N,
                           int64_t H, int64_t W, int64_t Cin, int64_t Ho, int64_t Wo, int64_t Cout,
                           int64_t KH, int64_t KW, int64_t stride, int64_t pad, int64_t Kp,
                           int64_t splits, float scale, int64_t accumulate, int64_t cin_keep,
                           int64_t groups, int64_t nsets, int64_t gstride, hipStream_t st) {
  return conv_wgrad_impl(x, dy, partial, grad, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad,
                         Kp, splits, scale, accumulate, cin_keep, groups, st, true, nsets, gstride);
}

// The weight-gradient GEMM only: its split partials stay in `partial` for a
// later mda_wgrad_reduce_multi (same arguments; grad / scale / accumulate /
// cin_keep / groups are checked and then belong to that reduce).
MDA_API int mda_conv_wgrad_nored(const void* x, const void* dy, float* partial, float* grad,
                                 int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Ho,
                                 int64_t Wo, int64_t Cout, int64_t KH, int64_t KW, int64_t stride,
                                 int64_t pad, int64_t Kp, int64_t splits, float scale,
                                 int64_t accumulate, int64_t cin_keep, int64_t groups,
                                 int64_t nsets, hipStream_t st) {
  return conv_wgrad_impl(x, dy, partial, grad, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad,
                         Kp, splits, scale, accumulate, cin_keep, groups, st, false, nsets, 0);
}

// mda_conv_wgrad_nored and the streaming BN-backward apply of the next layer
// (csrc/bn.hip mda_bn_bwd_apply_reg's operands, b_*, one gradient set, no
// pre-activation gradient) in ONE launch.  MDA_NOT_SERVED (nothing launched)
// when the apply's LDS does not fit the GEMM kernel's or the shapes are not
// served; the caller then launches the two on their own.
MDA_API int mda_conv_wgrad_nored_bn(const void* x, const void* dy, float* partial, float* grad,
                                    int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Ho,
                                    int64_t Wo, int64_t Cout, int64_t KH, int64_t KW,
                                    int64_t stride, int64_t pad, int64_t Kp, int64_t splits,
                                    int64_t cin_keep, int64_t groups, const void* b_dout,
                                    const void* b_y, const void* b_res, const float* b_stats,
                                    int64_t b_M, int64_t b_C, int64_t b_act, void* b_region,
                                    void* b_dy, void* b_dres, float* b_dgamma, float* b_dbeta,
                                    float* b_sums, const void* b_ry, const float* b_rstats,
                                    void* b_rregion, const float* b_vres, hipStream_t st) {
  if (b_C % 8 || b_C > SLOT_CMAX || b_M <= 0 || b_M >= ((int64_t)1 << 31) || b_region == nullptr)
    return MDA_NOT_SERVED;
  if (b_rregion != nullptr && (b_dres == nullptr || b_ry == nullptr || b_rstats == nullptr ||
                               256 % (b_C / 8) != 0))
    return MDA_NOT_SERVED;  // a thread must keep one channel group
  const BwdArgs a{(const bf16_t*)b_dout, nullptr, nullptr, (const bf16_t*)b_y,
                  (const bf16_t*)b_res, b_stats, (bf16_t*)b_dy, (bf16_t*)b_dres, b_dgamma, b_dbeta,
                  b_sums, (BnRegion*)b_region, nullptr, (int)b_M, (int)b_C, (int)b_act,
                  (const bf16_t*)b_ry, b_rstats, (BnRegion*)b_rregion, b_vres, 0, 0, 0};
  return conv_wgrad_impl(x, dy, partial, grad, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad,
                         Kp, splits, 1.f, 1, cin_keep, groups, st, false, 1, 0, &a);
}

// rows: n x 11 int64 {partial, grad, splits, Cout, Cin, KH, KW, Kp, accumulate, cin_keep,
// groups} (host memory; scale 1).  Launches ceil(n / 16) multi-layer reduce kernels.
MDA_API int mda_wgrad_reduce_multi(const int64_t* rows, int64_t n, hipStream_t st) {
  for (int64_t b0 = 0; b0 < n; b0 += WGRM_MAX) {
    WgrTable t;
    t.n = (int)((n - b0) < WGRM_MAX ? (n - b0) : WGRM_MAX);
    int blk = 0;
    for (int i = 0; i < t.n; ++i) {
      const int64_t* r = rows + (b0 + i) * 11;
      WgrLayer& L = t.l[i];
      L.partial = (const float*)r[0];
      L.grad = (float*)r[1];
      L.splits = (int)r[2]; L.Cout = (int)r[3]; L.Cin = (int)r[4]; L.KH = (int)r[5];
      L.KW = (int)r[6]; L.Kp = (int)r[7]; L.accumulate = (int)r[8];
      L.cin_keep = (int)((r[9] <= 0 || r[9] > r[4]) ? r[4] : r[9]);
      L.groups = (int)(r[10] > 1 ? r[10] : 1);
      L.dw = r[10] == -1;  // groups = -1 marks a depthwise row (Cout = C, KH x KW taps)
      L.scale = 1.f;
      L.blk0 = blk;
      if (L.dw) {
        if (L.splits < 1 || L.Cout < 1) return (int)hipErrorInvalidValue;
        blk += (int)(((int64_t)L.KH * L.KW * L.Cout + 31) / 32);
        continue;
      }
      if (L.Cout % 8 || L.Kp % 64 || L.splits < 1) return (int)hipErrorInvalidValue;
      const int cp = wgr_cols(L.splits);
      blk += (int)(((int64_t)L.Cout * L.Kp / 4 + cp - 1) / cp);
    }
    hipLaunchKernelGGL(wgrad_reduce_multi_kernel, dim3((unsigned)blk), dim3(256), 0, st, t);
    const int rc = (int)hipGetLastError();
    if (rc) return rc;
  }
  return 0;
}

namespace {
// Grouped conv (groups G, not depthwise) as ONE dense GEMM on the block-
// diagonal weight: w fp32 [Cout, Cin/G, KH, KW] -> wf bf16 [Cout, Kp] with
// k = tap*Cin + ci (zero where ci is outside co's group, and k >= K) and,
// optionally, wt bf16 [Cin, KpT] with k = tap*Cout + co (padding zeroed).
// G x the MFMA work of a grouped kernel, but the grouped 1x1 convs this
// serves (ShuffleNetV1, G = 3) are a small part of their network's FLOPs.
__global__ void __launch_bounds__(256)
pack_grouped_kernel(const float* __restrict__ w, bf16_t* __restrict__ wf, bf16_t* __restrict__ wt,
                    int Cout, int Cin, int KH, int KW, int Kp, int KpT, int G) {
  const int cin_g = Cin / G, cout_g = Cout / G, KK = KH * KW, K = KK * Cin;
  const int64_t total = (int64_t)Cout * Kp;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int co = (int)(i / Kp), k = (int)(i - (i / Kp) * Kp);
    float v = 0.f;
    if (k < K) {
      const int tap = k / Cin, ci = k - tap * Cin;
      const int g = co / cout_g;
      if (ci / cin_g == g) v = w[((int64_t)co * cin_g + (ci - g * cin_g)) * KK + tap];
      if (wt) wt[(int64_t)ci * KpT + tap * Cout + co] = f2bf(v);
    }
    wf[i] = f2bf(v);
  }
  if (wt) {
    const int padw = KpT - KK * Cout;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (int64_t)Cin * padw;
         i += (int64_t)gridDim.x * blockDim.x) {
      const int ci = (int)(i / padw), j = (int)(i - (i / padw) * padw);
      wt[(int64_t)ci * KpT + KK * Cout + j] = 0;
    }
  }
}
// Compact operands of a grouped conv (group-aligned GEMM tiles,
// conv_igemm.hip mda_conv_fwd_bnacc_g / mda_conv_dgrad_bnsum_g): w fp32
// [Cout, Cin/G, KH, KW] ->
//   wf bf16 [Cout][Kp]:  k = tap * (Cin/G) + ci            (the group's K only)
//   wt bf16 [Cin][KpT]:  k = tap * (Cout/G) + co_in_group  (dgrad of the group)
__global__ void __launch_bounds__(256)
pack_gc_kernel(const float* __restrict__ w, bf16_t* __restrict__ wf, bf16_t* __restrict__ wt,
               int Cout, int cin_g, int KH, int KW, int Kp, int KpT, int G) {
  const int cout_g = Cout / G, KK = KH * KW, K = KK * cin_g;
  const int64_t total = (int64_t)Cout * Kp;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int co = (int)(i / Kp), k = (int)(i - (i / Kp) * Kp);
    float v = 0.f;
    if (k < K) {
      const int tap = k / cin_g, ci = k - tap * cin_g;
      v = w[((int64_t)co * cin_g + ci) * KK + tap];
      if (wt) {
        const int g = co / cout_g, cog = co - g * cout_g;
        wt[(int64_t)(g * cin_g + ci) * KpT + tap * cout_g + cog] = f2bf(v);
      }
    }
    wf[i] = f2bf(v);
  }
  if (wt) {
    const int padw = KpT - KK * cout_g;
    const int64_t rows = (int64_t)cin_g * G;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < rows * padw;
         i += (int64_t)gridDim.x * blockDim.x) {
      const int ci = (int)(i / padw), j = (int)(i - (i / padw) * padw);
      wt[(int64_t)ci * KpT + KK * cout_g + j] = 0;
    }
  }
}
}  // namespace

MDA_API int mda_pack_conv_weights_gc(const float* w, void* wf, void* wt, int64_t Cout, int64_t cin_g,
                                     int64_t KH, int64_t KW, int64_t Kp, int64_t KpT, int64_t G,
                                     hipStream_t st) {
  if (G < 1 || Cout % G || Kp < KH * KW * cin_g || (wt && KpT < KH * KW * (Cout / G)))
    return (int)hipErrorInvalidValue;
  const int64_t total = Cout * Kp;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 2048);
  hipLaunchKernelGGL(pack_gc_kernel, dim3(blocks), dim3(256), 0, st, w, (bf16_t*)wf, (bf16_t*)wt,
                     (int)Cout, (int)cin_g, (int)KH, (int)KW, (int)Kp, (int)KpT, (int)G);
  MDA_CHECK_LAUNCH();
}

MDA_API int mda_pack_conv_weights_grouped(const float* w, void* wf, void* wt, int64_t Cout, int64_t Cin,
                                          int64_t KH, int64_t KW, int64_t Kp, int64_t KpT, int64_t G,
                                          hipStream_t st) {
  if (G < 1 || Cin % G || Cout % G) return (int)hipErrorInvalidValue;
  const int64_t total = Cout * Kp;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 2048);
  hipLaunchKernelGGL(pack_grouped_kernel, dim3(blocks), dim3(256), 0, st, w, (bf16_t*)wf, (bf16_t*)wt,
                     (int)Cout, (int)Cin, (int)KH, (int)KW, (int)Kp, (int)KpT, (int)G);
  MDA_CHECK_LAUNCH();
}

// w fp32 [Cout, Cin, KH, KW] -> wf bf16 [Cout, Kp]; wt (optional) bf16 [Cin, KpT]
MDA_API int mda_pack_conv_weights(const float* w, void* wf, void* wt, int64_t Cout, int64_t Cin,
                                  int64_t KH, int64_t KW, int64_t Kp, int64_t KpT,
                                  hipStream_t st) {
  int64_t total = Cout * Kp;
  int blocks = (int)std::min<int64_t>((total + 255) / 256, 1024);
  hipLaunchKernelGGL(pack_kernel, dim3(blocks), dim3(256), 0, st, w, (bf16_t*)wf, (bf16_t*)wt,
                     (int)Cout, (int)Cin, (int)KH, (int)KW, (int)Kp, (int)KpT);
  MDA_CHECK_LAUNCH();
}
