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
// A/B K-slices are staged global -> VGPR -> LDS with two register sets
// (stage s+2 in flight while s+1 is written and s computed), two LDS
// buffers, one barrier per stage.  Global reads are buffer loads with 32-bit
// offsets; padding taps / tails read as zero through the descriptor range
// check instead of branching.  LDS rows are 144 B (64 bf16 + 16 B pad): row
// starts land on 16 distinct 4-bank slots, so every 16-lane group of a
// ds_read_b128 fragment read is conflict-free.  The epilogue goes through
// an fp32 LDS C tile so each thread stores 8 channels (16 B) per row.
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
#include "bnslot.h"
#include <stdlib.h>
#include <mutex>
#include <unordered_map>


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
  int x_bytes, w_bytes;  // buffer-descriptor ranges (< 2 GiB, checked on the host)
  int hrows, himgs, hpb; // halo kernels: output rows per image, images, pixels per block
  // strided dgrad by output parity (glds kernel): gridDim.z = par*par classes x
  // zsplits K-splits; class (ph, pw) owns the dx pixels whose (ih+pad) % par == ph
  // (resp. pw) and only the taps kh = ph (mod par), kw = pw (mod par): the
  // 1 - 1/par^2 of the taps that cannot contribute are never multiplied.
  int par, zsplits;
  // training BN: per-block per-channel sum / sum of squares of the stored
  // (bf16-rounded) output, stats_part[blockIdx.x][2][Cout] (raw output only:
  // no scale/bias/residual/activation, no split-K)
  float* stats_part;
  // training BN through a one-shot BnRegion (bnslot.h): the block's channel
  // sums are added into shard blockIdx.x % slot_shards(Cout) of it instead
  BnRegion* stats_slot;
  // diagnostics: per-block phase timestamps (s_memrealtime, 100 MHz), null in
  // normal runs (mda_conv_set_stamps)
  uint64_t* stamps;
  // BN-backward sums (dgrad only): this dgrad's output is the gradient dout of
  // a training BN layer's output act(y*scale + shift (+ bnb_res)); besides the
  // bf16 dout the epilogue adds that layer's sum dz and sum dz*xhat
  // (dz = dout * act'(z), xhat = (y - mean) * rstd) into shard
  // blockIdx.x % slot_shards(Cout) of bnb_slot, so the BN backward is one
  // streaming pass (csrc/bn.hip mda_bn_bwd_apply_reg) instead of a
  // reduction + grid barrier + apply.  bnb_stats: [4][Cout] mean, rstd,
  // scale, shift of that layer.
  const bf16_t* bnb_y;
  const bf16_t* bnb_res;
  const float* bnb_stats;
  BnRegion* bnb_slot;
  int bnb_act;
  // optional: bnb_res is the RAW input of another training BN applied inside
  // this layer's apply (mda_bn_apply_fin_vr): residual = res*vres[2C+c] + vres[3C+c]
  const float* bnb_vres;
  // DOT single-pass backward: dy / dx hold two stacked cotangents (2N images);
  // rows >= bnb_mh belong to set 1, read bnb_y / bnb_res at row - bnb_mh (the
  // forward's N images) and add their sums into the region bnb_rstride bytes
  // past bnb_slot.  0 = one set.
  int bnb_mh;
  int64_t bnb_rstride;
  // grouped conv (glds kernel only): Cin above is the channels of ONE group,
  // x rows hold ldx channels, each group owns cout_g consecutive output
  // channels, and a block's N tile never leaves its group (grid.y = groups x
  // tiles per group).  Dense: ldx = Cin, cout_g = Cout.
  int ldx, cout_g;
  int xcd;  // glds kernel: XCD-aware tile order (MDA_CONV_XCD, default on)
  // K-order rotation (MDA_CONV_KROT): block (mt, nt) starts its K loop at step
  // (mt + nt) mod steps, so the blocks of a wave of the grid do not all read
  // the same weight tile of the same L2 channel in the same step
  int krot;
  int perm8;  // halo kernels on 8-wide maps: pixel-permuted MFMA rows (perm8, MDA_HALO_PERM8)
  // halo kernels: multiply-shift divisions by W, H, W + 2, (rows + 2)(W + 2)
  // and rows (set by halo_geometry).  The prologue's ~20 integer divisions
  // by runtime values cost ~1.2 us per block (in-kernel stamps,
  // scripts/conv_stamps.py) -- as much as a third of a 16x16 conv's MFMA loop.
  uint32_t dv_W[2], dv_H[2], dv_PW[2], dv_PHPW[2], dv_RH[2];
  // glds kernel loader: the same multiply-shift divisions by Cin, KW, Cin / 64,
  // Ho * Wo, Wo and the stride (set by dispatch).  With generic integer
  // divisions (and the branches hipcc wraps around them) the per-stage address
  // math of the strided dgrad was ~1.6 us of VALU per K-step -- the whole
  // kernel time (scripts/dgrad_stamps.py)
  uint32_t dv_Cin[2], dv_KW[2], dv_cb[2], dv_HoWo[2], dv_Wo[2], dv_s[2];
  // strided dgrad (PAR) with a second, 1 x 1 / stride-par / pad-0 conv on the
  // same input folded in (a residual block's projection shortcut): parity
  // class cls2 -- the dx pixels that conv samples -- runs cin2 / 64 more
  // K-steps with A = x2 [N, H, W, cin2] at the class's dy pixel minus sh2
  // rows / columns and B = w2 [Cout][kp2] (that conv's dgrad operand), so dx
  // is the SUM of both input gradients in one launch
  const bf16_t* x2;
  const bf16_t* w2;
  int cin2, kp2, cls2, sh2;
};

// n / d for 0 <= n < 2^31 with the host-made (mul, shr) of d
__device__ __forceinline__ int hdiv(int n, const uint32_t (&dv)[2]) {
  return (int)((__umulhi((uint32_t)n, dv[0]) + (uint32_t)n) >> dv[1]);
}
inline void make_hdiv(uint32_t d, uint32_t (&dv)[2]) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  dv[1] = l;
  dv[0] = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
}

// first output channel past the group of the tile starting at n0
__device__ __forceinline__ int group_nlim(const ConvParams& p, int n0) {
  if (p.cout_g >= p.Cout) return p.Cout;
  const int e = (n0 / p.cout_g + 1) * p.cout_g;
  return e < p.Cout ? e : p.Cout;
}
// N tile -> first output channel of the tile (group-aligned tiles)
__device__ __forceinline__ int group_n0(const ConvParams& p, int ty, int BN) {
  if (p.cout_g >= p.Cout) return ty * BN;
  const int tpg = (p.cout_g + BN - 1) / BN;
  return (ty / tpg) * p.cout_g + (ty % tpg) * BN;
}

__device__ __forceinline__ void stamp(const ConvParams& p, int k) {
  if (p.stamps != nullptr && threadIdx.x == 0) {
    const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    p.stamps[(int64_t)b * 8 + k] = __builtin_amdgcn_s_memrealtime();
  }
}

// Parity class of the strided-dgrad decomposition.
struct ParClass {
  int ih0, iw0, Hc, Wc, Mc;    // first dx row/col of the class, class extent, rows
  int kh0, kw0, nkh, nkw;      // first tap and tap counts (step par)
};

__host__ __device__ __forceinline__ ParClass par_class(const ConvParams& p, int cls) {
  // GEMM view of dgrad: p.H/p.W = dy extent, p.Ho/p.Wo = dx extent, p.stride = s
  ParClass c;
  const int s = p.par;
  const int ph = cls / s, pw = cls - (cls / s) * s;
  c.ih0 = ((ph - p.pad) % s + s) % s;
  c.iw0 = ((pw - p.pad) % s + s) % s;
  c.Hc = p.Ho > c.ih0 ? (p.Ho - c.ih0 + s - 1) / s : 0;
  c.Wc = p.Wo > c.iw0 ? (p.Wo - c.iw0 + s - 1) / s : 0;
  c.Mc = p.N * c.Hc * c.Wc;
  c.kh0 = ph;
  c.kw0 = pw;
  c.nkh = p.KH > ph ? (p.KH - ph + s - 1) / s : 0;
  c.nkw = p.KW > pw ? (p.KW - pw + s - 1) / s : 0;
  return c;
}

// class row -> global dx pixel index
__device__ __forceinline__ int par_row(const ConvParams& p, const ParClass& c, int m) {
  const int hw = c.Hc * c.Wc;
  const int n = m / hw, r = m - n * hw;
  const int i = r / c.Wc, j = r - (r / c.Wc) * c.Wc;
  return (n * p.Ho + c.ih0 + p.par * i) * p.Wo + c.iw0 + p.par * j;
}

// Buffer loads: 32-bit per-lane byte offsets against a wave-uniform
// descriptor; an offset past the range returns zeros, which is how padding
// taps, tail rows and tail channels are zero-filled without exec-mask
// branches around every load.
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

// 8 consecutive channels [co, co+8) of row m (Cout % 8 == 0): 16-byte
// residual load, preact and output stores; sc/bi already hold the channels'
// scale and bias.
__device__ __forceinline__ void epilogue_store8(const ConvParams& p, int m, int co, const float* v,
                                                const float* sc, const float* bi,
                                                uint4 res_reg = make_uint4(0u, 0u, 0u, 0u),
                                                bool use_reg = false) {
  const int64_t o = (int64_t)m * p.Cout + co;
  float t[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = v[e] * sc[e] + bi[e];
  if (p.res) {
    const uint4 r = use_reg ? res_reg : *(const uint4*)(p.res + o);
    const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      t[2 * e] += __uint_as_float(rr[e] << 16);
      t[2 * e + 1] += __uint_as_float(rr[e] & 0xffff0000u);
    }
  }
  if (p.preact)
    *(uint4*)(p.preact + o) = make_uint4(pack_bf16x2(t[0], t[1]), pack_bf16x2(t[2], t[3]),
                                         pack_bf16x2(t[4], t[5]), pack_bf16x2(t[6], t[7]));
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = apply_act(t[e], p.act);
  *(uint4*)(p.y + o) = make_uint4(pack_bf16x2(t[0], t[1]), pack_bf16x2(t[2], t[3]),
                                  pack_bf16x2(t[4], t[5]), pack_bf16x2(t[6], t[7]));
}

__device__ __forceinline__ void load_scale_bias8(const ConvParams& p, int co, float* sc, float* bi) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = p.scale ? p.scale[co + e] : 1.f;
    bi[e] = p.bias ? p.bias[co + e] : 0.f;
  }
}

template <int BM, int BN>
struct ConvSmem {
  static constexpr int STAGE = 2 * (BM + BN) * LDS_ROW * 2;  // bytes, double-buffered A+B
  static constexpr int CS = BN + 4;                          // fp32 C-tile row (floats)
  static constexpr int CTILE = BM * CS * 4;
  static constexpr int BYTES = STAGE > CTILE ? STAGE : CTILE;
};

// Epilogue through LDS, shared by both conv kernels: the fp32 C tile is
// written in MFMA layout, then each thread owns 8 consecutive channels of a
// row -> 16-byte residual loads and output stores, scale/bias loaded once
// per thread.  Split-K blocks write fp32 partials instead.  The caller must
// have finished every read of `smem` (barrier) before calling.
// Phase 1 of the epilogue: one 4-wave group's MFMA accumulators (a BMg x BN
// tile, 2x2 waves) into the fp32 C tile at row offset `row0`.
// 8-wide maps (halo kernels): MFMA row f of a 16-pixel fragment reads output
// pixel perm8(f), so the ds_read_b128 lane groups {0-3,12-15 | 20-27} read the
// fragment's first output row with one k-chunk and its second row with the
// other -- 16 distinct 16-byte bank slots under the r & 6 patch swizzle (the
// identity order put both rows' pixels of a chunk on 8 slots: 2-way, 8 LDS
// cycles per read instead of 4).  The C tile is stored back in pixel order.
__device__ __forceinline__ int perm8(int f) { return f < 4 ? f : (f < 12 ? f + 4 : f - 8); }

template <int BMg, int BN>
__device__ __forceinline__ void store_c_tile(float* Cs, int CS, const f32x4 (&acc)[BMg / 32][BN / 32],
                                             int row0, int wid, int lane, bool p8 = false) {
  constexpr int MI = BMg / 32, NI = BN / 32;
  const int wm = wid >> 1, wn = wid & 1;
  const int ecol = lane & 15;
  const int erow = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int fr = p8 ? perm8(erow + r) : erow + r;
        Cs[(row0 + wm * (BMg / 2) + i * 16 + fr) * CS + wn * (BN / 2) + j * 16 + ecol] = acc[i][j][r];
      }
}

// Epilogue operands of one thread (its 8 channels' scale / bias and, when the
// row count is small, its residual rows), loaded at kernel start, BEFORE the
// first LDS-DMA is issued (older than every DMA, so the vmcnt-counted waits
// of the main loop stay exact).  Loaded after the main loop instead, their
// global latency serialises with the stores: in-kernel stamps put the halo
// conv epilogue at ~3.7 of ~11.4 us, one round trip of it being these loads.
template <int BM, int BN, int NT>
struct EpiPre {
  static constexpr int TPR = BN / 8;                  // threads per row
  static constexpr int RPP = NT / TPR;                // rows per pass
  static constexpr int RPT = (BM + RPP - 1) / RPP;    // passes
  static constexpr bool RES = RPT <= 4;               // residual rows held in registers
  float sc[8], bi[8];
  uint4 res[RES ? RPT : 1];
  bool have;                                          // sc / bi valid
  bool have_res;                                      // res valid
};

template <int BM, int BN, int NT>
__device__ __forceinline__ void epi_prefetch(const ConvParams& p, EpiPre<BM, BN, NT>& e, int m0, int n0,
                                             int rows, bool par) {
  using E = EpiPre<BM, BN, NT>;
  const int tid = threadIdx.x;
  const int c8 = tid % E::TPR, rr = tid / E::TPR;
  const int co = n0 + c8 * 8;
  const bool split = par ? p.zsplits > 1 : gridDim.z > 1;
  e.have = !split && p.stats_part == nullptr && p.stats_slot == nullptr && p.bnb_slot == nullptr &&
           (p.Cout & 7) == 0 && co < group_nlim(p, n0);
  e.have_res = false;
  if (!e.have) return;
  load_scale_bias8(p, co, e.sc, e.bi);
  if (E::RES && p.res != nullptr && !par) {
    e.have_res = true;
#pragma unroll
    for (int k = 0; k < (E::RES ? E::RPT : 1); ++k) {
      const int r0 = rr + k * E::RPP;
      const int m = m0 + r0;
      e.res[k] = (r0 < rows && m < p.M) ? *(const uint4*)(p.res + (int64_t)m * p.Cout + co)
                                        : make_uint4(0u, 0u, 0u, 0u);
    }
  }
}

template <int BM, int BN, int NT = 256>
__device__ __forceinline__ void conv_epilogue_rows(const ConvParams& p, char* smem, int m0, int n0,
                                                   int rows, const ParClass& pc, bool has_pc,
                                                   const EpiPre<BM, BN, NT>& pre);

__device__ __forceinline__ float bnb_act_grad(float z, int act) {
  if (act == ACT_RELU) return z > 0.f ? 1.f : 0.f;
  if (act == ACT_RELU6) return (z > 0.f && z < 6.f) ? 1.f : 0.f;
  return 1.f;
}

// BN-backward epilogue of a dgrad (see ConvParams::bnb_*): store
// dout = acc (+ res) in bf16, then sum dz and dz*xhat of the STORED values
// over the block's rows and add them into the region (what the streaming
// apply recomputes dz from).  Every load of a thread's rows (C tile, BN
// input y, its residual, the fork gradient) is issued before any math.
template <int BM, int BN, int NT>
__device__ __forceinline__ void conv_epilogue_bnb(const ConvParams& p, float* Cs, int m0, int n0,
                                                  int rows, const ParClass& pc, bool has_pc) {
  constexpr int CS = ConvSmem<BM, BN>::CS;
  constexpr int TPR = BN / 8;
  constexpr int RPP = NT / TPR;
  constexpr int RPT = (BM + RPP - 1) / RPP;
  const int tid = threadIdx.x;
  const int c8 = tid % TPR, rr = tid / TPR;
  const int co = n0 + c8 * 8;
  const int C = p.Cout;
  const int mlim = has_pc ? pc.Mc : p.M;
  const bool cok = co < group_nlim(p, n0);
  const bool zres = p.bnb_res != nullptr && p.bnb_act != ACT_NONE;
  float mu[8], rs[8], sc[8], sh[8], vsc[8], vsh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = cok ? p.bnb_stats[co + e] : 0.f;
    rs[e] = cok ? p.bnb_stats[C + co + e] : 0.f;
    sc[e] = cok ? p.bnb_stats[2 * C + co + e] : 0.f;
    sh[e] = cok ? p.bnb_stats[3 * C + co + e] : 0.f;
    vsc[e] = (cok && p.bnb_vres) ? p.bnb_vres[2 * C + co + e] : 1.f;
    vsh[e] = (cok && p.bnb_vres) ? p.bnb_vres[3 * C + co + e] : 0.f;
  }
  uint4 yv[RPT], rv[RPT], gv[RPT];
  int mrow[RPT];
  const int mh = p.bnb_mh;
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int r0 = rr + k * RPP;
    int m = m0 + r0;
    const bool ok = cok && r0 < rows && m < mlim;
    if (ok && has_pc) m = par_row(p, pc, m);
    mrow[k] = ok ? m : -1;
    const int ma = (mh > 0 && m >= mh) ? m - mh : m;  // the forward's row
    const int64_t o = (int64_t)(ok ? m : 0) * C + (cok ? co : 0);
    const int64_t oa = (int64_t)(ok ? ma : 0) * C + (cok ? co : 0);
    yv[k] = ok ? *(const uint4*)(p.bnb_y + oa) : make_uint4(0u, 0u, 0u, 0u);
    rv[k] = (ok && zres) ? *(const uint4*)(p.bnb_res + oa) : make_uint4(0u, 0u, 0u, 0u);
    gv[k] = (ok && p.res) ? *(const uint4*)(p.res + o) : make_uint4(0u, 0u, 0u, 0u);
  }
  float s1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, s2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float t1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, t2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    if (mrow[k] < 0) continue;
    const bool set1 = mh > 0 && mrow[k] >= mh;
    const int r0 = rr + k * RPP;
    const float4 lo = *(const float4*)&Cs[r0 * CS + c8 * 8];
    const float4 hi = *(const float4*)&Cs[r0 * CS + c8 * 8 + 4];
    float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    const uint32_t gw[4] = {gv[k].x, gv[k].y, gv[k].z, gv[k].w};
    const uint32_t yw[4] = {yv[k].x, yv[k].y, yv[k].z, yv[k].w};
    const uint32_t rw[4] = {rv[k].x, rv[k].y, rv[k].z, rv[k].w};
    uint32_t ow[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      if (p.res) {
        v[2 * w] += __uint_as_float(gw[w] << 16);
        v[2 * w + 1] += __uint_as_float(gw[w] & 0xffff0000u);
      }
      ow[w] = pack_bf16x2(v[2 * w], v[2 * w + 1]);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = 2 * w + h;
        float d = h ? __uint_as_float(ow[w] & 0xffff0000u) : __uint_as_float(ow[w] << 16);
        const float yf = h ? __uint_as_float(yw[w] & 0xffff0000u) : __uint_as_float(yw[w] << 16);
        if (p.bnb_act != ACT_NONE) {
          float z = yf * sc[e] + sh[e];
          if (zres) z += (h ? __uint_as_float(rw[w] & 0xffff0000u) : __uint_as_float(rw[w] << 16)) * vsc[e] + vsh[e];
          d *= bnb_act_grad(z, p.bnb_act);
        }
        const float xh = d * ((yf - mu[e]) * rs[e]);
        if (set1) { t1[e] += d; t2[e] += xh; } else { s1[e] += d; s2[e] += xh; }
      }
    }
    *(uint4*)(p.y + (int64_t)mrow[k] * C + co) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
  }
  __syncthreads();  // every read of the C tile is done: reuse it for the reduction
  float* red = Cs;  // [2][RPP][BN]
  const int nsets = mh > 0 ? 2 : 1;  // (block-uniform)
  for (int set = 0; set < nsets; ++set) {
    if (set) __syncthreads();  // set 0's reads of `red` are done
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(0 * RPP + rr) * BN + c8 * 8 + e] = set ? t1[e] : s1[e];
      red[(1 * RPP + rr) * BN + c8 * 8 + e] = set ? t2[e] : s2[e];
    }
    __syncthreads();
    if (tid < 2 * BN) {
      const int q = tid / BN, c = tid - q * BN;
      float a0 = 0.f, a1 = 0.f;
      for (int r = 0; r < RPP; r += 2) {
        a0 += red[(q * RPP + r) * BN + c];
        a1 += red[(q * RPP + r + 1) * BN + c];
      }
      BnRegion* slot = (BnRegion*)((char*)p.bnb_slot + (set ? p.bnb_rstride : 0));
      if (n0 + c < group_nlim(p, n0))
        acc_add(region_acc(slot, C, (int)blockIdx.x % slot_shards(C), q) + n0 + c, (double)(a0 + a1));
    }
  }
}

template <int BM, int BN>
__device__ __forceinline__ void conv_epilogue(const ConvParams& p, const f32x4 (&acc)[BM / 32][BN / 32],
                                              char* smem, int m0, int n0, int rows,
                                              const ParClass& pc, bool has_pc,
                                              const EpiPre<BM, BN, 256>& pre, bool p8 = false) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  store_c_tile<BM, BN>((float*)smem, ConvSmem<BM, BN>::CS, acc, 0, wid, lane, p8);
  __syncthreads();
  conv_epilogue_rows<BM, BN, 256>(p, smem, m0, n0, rows, pc, has_pc, pre);
}


// Phase 2: NT threads own 8 channels x rows of the C tile: bias / BN affine,
// residual, activation, preact and bf16 stores, split-K partials, or the raw
// output + BN statistics partials.  Every barrier is reached by all threads.
template <int BM, int BN, int NT>
__device__ __forceinline__ void conv_epilogue_rows(const ConvParams& p, char* smem, int m0, int n0,
                                                   int rows, const ParClass& pc, bool has_pc,
                                                   const EpiPre<BM, BN, NT>& pre) {
  constexpr int CS = ConvSmem<BM, BN>::CS;
  const int tid = threadIdx.x;
  float* const Cs = (float*)smem;
  constexpr int TPR = BN / 8;    // threads per row
  constexpr int RPP = NT / TPR;  // rows per pass
  const int c8 = tid % TPR;
  const int rr = tid / TPR;
  const int co = n0 + c8 * 8;
  const int zsplit = has_pc ? (int)blockIdx.z % p.zsplits : (int)blockIdx.z;
  const bool split = has_pc ? p.zsplits > 1 : gridDim.z > 1;
  const int mlim = has_pc ? pc.Mc : p.M;
  if (p.bnb_slot != nullptr) {
    conv_epilogue_bnb<BM, BN, NT>(p, Cs, m0, n0, rows, pc, has_pc);
    return;
  }
  if (p.stats_part != nullptr || p.stats_slot != nullptr) {
    // raw bf16 output + BN statistics partials of this block's rows.  No early
    // return before the barrier: threads past Cout just contribute zeros.
    float s1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, s2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const bool cok = co < group_nlim(p, n0);
    for (int r0 = rr; r0 < rows; r0 += RPP) {
      const int m = m0 + r0;
      if (m >= mlim || !cok) break;
      const float4 lo = *(const float4*)&Cs[r0 * CS + c8 * 8];
      const float4 hi = *(const float4*)&Cs[r0 * CS + c8 * 8 + 4];
      const uint4 o = make_uint4(pack_bf16x2(lo.x, lo.y), pack_bf16x2(lo.z, lo.w),
                                 pack_bf16x2(hi.x, hi.y), pack_bf16x2(hi.z, hi.w));
      *(uint4*)(p.y + (int64_t)m * p.Cout + co) = o;
      const uint32_t u[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a = __uint_as_float(u[e] << 16), b = __uint_as_float(u[e] & 0xffff0000u);
        s1[2 * e] += a; s2[2 * e] += a * a;
        s1[2 * e + 1] += b; s2[2 * e + 1] += b * b;
      }
    }
    __syncthreads();  // every read of the C tile is done: reuse it for the reduction
    float* red = Cs;  // [2][RPP][BN]
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(0 * RPP + rr) * BN + c8 * 8 + e] = s1[e];
      red[(1 * RPP + rr) * BN + c8 * 8 + e] = s2[e];
    }
    __syncthreads();
    if (tid < 2 * BN) {
      const int q = tid / BN, c = tid - q * BN;
      float a0 = 0.f, a1 = 0.f;
      for (int r = 0; r < RPP; r += 2) {
        a0 += red[(q * RPP + r) * BN + c];
        a1 += red[(q * RPP + r + 1) * BN + c];
      }
      if (n0 + c < group_nlim(p, n0)) {
        if (p.stats_slot != nullptr)
          acc_add(region_acc(p.stats_slot, p.Cout, (int)blockIdx.x % slot_shards(p.Cout), q) + n0 + c,
                  (double)(a0 + a1));
        else
          p.stats_part[((int64_t)(m0 / rows) * 2 + q) * p.Cout + n0 + c] = a0 + a1;
      }
    }
    return;
  }
  if ((p.Cout & 7) == 0) {
    if (co >= group_nlim(p, n0)) return;
    using E = EpiPre<BM, BN, NT>;
    if (pre.have) {
      // operands already in registers (epi_prefetch); fully unrolled so the
      // residual array stays in VGPRs
#pragma unroll
      for (int k = 0; k < E::RPT; ++k) {
        const int r0 = rr + k * RPP;
        int m = m0 + r0;
        if (r0 < rows && m < mlim) {  // (no break: keeps the loop fully unrolled)
          if (has_pc) m = par_row(p, pc, m);
          const float4 lo = *(const float4*)&Cs[r0 * CS + c8 * 8];
          const float4 hi = *(const float4*)&Cs[r0 * CS + c8 * 8 + 4];
          const float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
          epilogue_store8(p, m, co, v, pre.sc, pre.bi, pre.res[E::RES ? k : 0], pre.have_res);
        }
      }
      return;
    }
    float sc[8], bi[8];
    if (!split) load_scale_bias8(p, co, sc, bi);
#pragma unroll 2
    for (int r0 = rr; r0 < rows; r0 += RPP) {
      int m = m0 + r0;
      if (m >= mlim) break;
      if (has_pc) m = par_row(p, pc, m);
      const float4 lo = *(const float4*)&Cs[r0 * CS + c8 * 8];
      const float4 hi = *(const float4*)&Cs[r0 * CS + c8 * 8 + 4];
      if (split) {
        float* dst = p.partial + ((int64_t)zsplit * p.M + m) * p.Cout + co;
        *(float4*)dst = lo;
        *(float4*)(dst + 4) = hi;
      } else {
        const float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        epilogue_store8(p, m, co, v, sc, bi);
      }
    }
  } else {
    for (int r0 = rr; r0 < rows; r0 += RPP) {
      int m = m0 + r0;
      if (m >= mlim) break;
      if (has_pc) m = par_row(p, pc, m);
      for (int e = 0; e < 8; ++e) {
        if (co + e >= group_nlim(p, n0)) break;
        const float a = Cs[r0 * CS + c8 * 8 + e];
        if (split)
          p.partial[((int64_t)zsplit * p.M + m) * p.Cout + co + e] = a;
        else
          epilogue_store(p, m, co + e, a);
      }
    }
  }
}

// Occupancy hint: without it the compiler spends up to 512 registers on a
// 256-thread block (1 block per CU); two 4-wave blocks per CU keep the
// register budget at 256 (no spills except the 128x128 tile, left free).
template <int BM, int BN>
struct ConvOcc { static constexpr int W = (BM * BN >= 16384) ? 1 : 2; };

template <int BM, int BN, int MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ConvOcc<BM, BN>::W)))
conv_fwd_kernel(const ConvParams p) {
  constexpr int MI = BM / 32;  // 16-row MFMA tiles per wave (wave tile = BM/2 rows)
  constexpr int NI = BN / 32;
  constexpr int AROWS = BM / 32;  // A rows loaded per thread per stage (8 chunks per row)
  constexpr int BLOADS = (BN * 8 + 255) / 256;
  constexpr bool DGRAD = (MODE == LOAD_DGRAD_FAST || MODE == LOAD_DGRAD_VEC8);

  __shared__ __attribute__((aligned(16))) char smem[ConvSmem<BM, BN>::BYTES];
  bf16_t* const As = (bf16_t*)smem;                 // [2][BM][LDS_ROW]
  bf16_t* const Bs = As + 2 * BM * LDS_ROW;         // [2][BN][LDS_ROW]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  EpiPre<BM, BN, 256> pre;
  epi_prefetch(p, pre, m0, n0, BM, false);
  const int chunk = tid & 7;
  const int arow = tid >> 3;
  const int HoWo = p.Ho * p.Wo;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(p.x, p.x_bytes);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(p.w, p.w_bytes);

  // per A row: element offset of the image (n) and the window origin
  int a_img[AROWS], a_ih0[AROWS], a_iw0[AROWS];
#pragma unroll
  for (int j = 0; j < AROWS; ++j) {
    int m = m0 + arow + 32 * j;
    const bool ok = m < p.M;
    int mm = ok ? m : 0;
    int n = mm / HoWo;
    int r = mm - n * HoWo;
    int oh = r / p.Wo;
    int ow = r - oh * p.Wo;
    a_img[j] = n * p.H * p.W * p.Cin;
    if (DGRAD) {
      // dgrad: output row = input-gradient pixel (ih, iw); taps gather dy at
      // oh = (ih + pad - kh) / stride when divisible and in range
      a_ih0[j] = oh + p.pad;
      a_iw0[j] = ow + p.pad;
    } else {
      a_ih0[j] = oh * p.stride - p.pad;
      a_iw0[j] = ow * p.stride - p.pad;
    }
    if (!ok) a_ih0[j] = -(1 << 28);  // every tap out of range -> zero row
  }
  // B (weights) rows: per-lane byte offsets, OOB past Cout
  uint32_t b_off[BLOADS];
#pragma unroll
  for (int j = 0; j < BLOADS; ++j) {
    int idx = tid + 256 * j;
    int row = idx >> 3, ch = idx & 7;
    int co = n0 + row;
    b_off[j] = (row < BN && co < p.Cout) ? (uint32_t)((co * p.Kp + ch * 8) * 2) : OOB;
  }

  // two register staging sets: stage s+2 is in flight while stage s+1 is
  // being written to LDS and stage s is computed
  uint4 ra0[AROWS], rb0[BLOADS], ra1[AROWS], rb1[BLOADS];
  const int total_steps = p.Kp / BK;
  const int s_begin = blockIdx.z * p.steps_per_split;
  const int s_end = min(total_steps, s_begin + p.steps_per_split);
  const int cin_blocks = p.Cin / BK;  // FAST modes only

  // Every call issues the same number of loads, also past the end of the K
  // range (then all offsets are OOB and the loads return zeros without
  // touching memory): with a fixed per-iteration load count the compiler's
  // vmcnt waits are exact.  Conditional loads made it merge the paths
  // conservatively and wait on the just-issued prefetch every stage.
  auto load_step = [&](int s, uint4 (&ra)[AROWS], uint4 (&rb)[BLOADS]) {
    const bool live = s < s_end;
    s = live ? s : s_begin;
    if (MODE == LOAD_FAST || MODE == LOAD_VEC8) {
      int tap, c0;
      bool kok = live;
      if (MODE == LOAD_FAST) {
        tap = s / cin_blocks;  // wave-uniform
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
        const int ih = a_ih0[j] + kh, iw = a_iw0[j] + kw;
        const bool ok = kok && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        ra[j] = ld16(xr, sel_off(ok, (a_img[j] + (ih * p.W + iw) * p.Cin + c0) * 2));
      }
    } else if (DGRAD) {
      int tap, c0;
      bool kok = live;
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
        bool ok = kok && nh >= 0 && nw >= 0;
        int ih = nh, iw = nw;
        if (p.stride != 1) {
          ih = hdiv(max(nh, 0), p.dv_s);
          iw = hdiv(max(nw, 0), p.dv_s);
          ok = ok && ih * p.stride == nh && iw * p.stride == nw;
        }
        ok = ok && ih < p.H && iw < p.W;
        ra[j] = ld16(xr, sel_off(ok, (a_img[j] + (ih * p.W + iw) * p.Cin + c0) * 2));
      }
    } else {
#pragma unroll
      for (int j = 0; j < AROWS; ++j) {
        uint32_t v[4];
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          uint32_t pair = 0;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int k = s * BK + chunk * 8 + 2 * e2 + h;
            const int tap = k / p.Cin;
            const int c = k - tap * p.Cin;
            const int kh = tap / p.KW, kw = tap - kh * p.KW;
            const int ih = a_ih0[j] + kh, iw = a_iw0[j] + kw;
            const bool ok = live && k < p.K && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
            const uint32_t e = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(
                xr, (int)sel_off(ok, (a_img[j] + (ih * p.W + iw) * p.Cin + c) * 2), 0, 0);
            pair |= e << (16 * h);
          }
          v[e2] = pair;
        }
        ra[j] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
#pragma unroll
    for (int j = 0; j < BLOADS; ++j)
      rb[j] = ld16(wr, (b_off[j] + (uint32_t)(s * BK * 2)) | ((uint32_t)(!live) << 31));
  };

  auto store_step = [&](int buf, const uint4 (&ra)[AROWS], const uint4 (&rb)[BLOADS]) {
#pragma unroll
    for (int j = 0; j < AROWS; ++j)
      *(uint4*)&As[(buf * BM + arow + 32 * j) * LDS_ROW + chunk * 8] = ra[j];
#pragma unroll
    for (int j = 0; j < BLOADS; ++j) {
      int idx = tid + 256 * j;
      int row = idx >> 3, ch = idx & 7;
      if (row < BN) *(uint4*)&Bs[(buf * BN + row) * LDS_ROW + ch * 8] = rb[j];
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15;
  const int fk = (lane >> 4) * 8;
  auto compute = [&](int buf) {
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        af[i] = *(const bf16x8*)&As[(buf * BM + wm * (BM / 2) + i * 16 + frow) * LDS_ROW + kk + fk];
#pragma unroll
      for (int j = 0; j < NI; ++j)
        bfr[j] = *(const bf16x8*)&Bs[(buf * BN + wn * (BN / 2) + j * 16 + frow) * LDS_ROW + kk + fk];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  const int n = s_end - s_begin;
  load_step(s_begin, ra0, rb0);
  load_step(s_begin + 1, ra1, rb1);
  store_step(0, ra0, rb0);
  __syncthreads();
  // unrolled by two so both register sets stay statically indexed; loads
  // and LDS stores are unconditional (zeros past the end, see load_step)
  for (int t = 0; t < n; t += 2) {
    load_step(s_begin + t + 2, ra0, rb0);
    compute(0);
    store_step(1, ra1, rb1);
    __syncthreads();
    if (t + 1 >= n) break;
    load_step(s_begin + t + 3, ra1, rb1);
    compute(1);
    store_step(0, ra0, rb0);
    __syncthreads();
  }

  __syncthreads();  // (loop ended with a barrier; keeps the C tile write safe either way)
  conv_epilogue<BM, BN>(p, acc, smem, m0, n0, BM, ParClass{}, false, pre);
}

// ---------------------------------------------------------------------------
// LDS-DMA variant (all modes except SCALAR).  Tiles go global -> LDS with
// global_load_lds_dwordx4 (no VGPR staging), three LDS buffers, two stages in
// flight, ONE barrier per stage: at iteration t the wave waits until its own
// stage-t copies landed (vmcnt = loads of the one newer stage), the barrier
// makes every wave's copies visible AND retires every wave's reads of the
// buffer the next copy overwrites, then stage t+2 is issued and stage t
// computed.  The copies are inline asm, so hipcc neither counts them nor
// inserts vmcnt(0) drains of its own (CDNA HIP guide §5 "Pipelining across
// barriers", §5.7).  LDS rows are 128 B, lane-linear per wave (the DMA
// writes base + lane*16); bank conflicts of the fragment reads are removed
// by an XOR swizzle applied on the SOURCE side: LDS slot c of row r holds
// k-chunk c ^ ((r >> 1) & 7), so the 16 rows of a fragment read hit 16
// distinct 16-byte bank groups.  Padding taps, tail rows and dead stages
// read a 16-byte zero page instead of branching.
__device__ __attribute__((aligned(16))) uint32_t g_zero16[4] = {0u, 0u, 0u, 0u};

constexpr int GLDS_NBUF = 3;

// RING = 1: single-stage blocks (K <= 64, e.g. the 1x1 expand convs of a
// bottleneck): one LDS buffer, no dead prefetch stages, and a footprint of
// max(stage, C tile) so 2-4 blocks share a CU and one block's DMA wait / MFMA
// / epilogue overlap another's.  With three buffers a K = 64 block issued three
// stages of DMAs (two of them zero-page dummies) and held 74-98 KB of LDS, one
// block per CU, every phase serialised: 97 us for a 6.6 GFLOP 64->256 1x1 conv
// at 56x56 x 64 that moves 128 MB (MIOpen: 23 us).
template <int BM, int BN, int RING = GLDS_NBUF>
struct GldsSmem {
  static constexpr int STAGE = (BM + BN) * 128;  // bytes per stage: A rows then B rows
  static constexpr int PIPE = RING * STAGE;
  static constexpr int CTILE = ConvSmem<BM, BN>::CTILE;
  // the BN-statistics reduction of conv_epilogue_rows: [2][RPP][BN] floats
  // (256 threads: RPP * BN = 2048) -- larger than a small tile's single stage
  static constexpr int RED = 2 * 2048 * 4;
  static constexpr int BYTES0 = PIPE > CTILE ? PIPE : CTILE;
  static constexpr int BYTES = BYTES0 > RED ? BYTES0 : RED;
};

__device__ __forceinline__ void glds16(const void* src, uint32_t lds_wave_base) {
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
__device__ __forceinline__ void vm_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"i"(N) : "memory");
}

template <int BM, int BN, int RING = GLDS_NBUF>
struct GldsOcc {
  static constexpr int W = RING == 1 ? (BM * BN >= 16384 ? 2 : 4)
                                     : ((BM * BN >= 16384 || RING > GLDS_NBUF) ? 1 : 2);
};

// XCD-aware tile order: blocks b, b + 8, ... share an XCD (and its L2); each
// XCD gets a contiguous run of tiles in (m, n) order, so the N tiles of one
// block of rows -- which read the same A rows -- run on one L2 (bijective
// for any tile count; cdna_hip_programming.md T1)
__device__ __forceinline__ void glds_tile(bool xcd, int& mt, int& nt) {
  mt = blockIdx.x;
  nt = blockIdx.y;
  if (xcd) {
    const int nwg = gridDim.x * gridDim.y;
    const int bid = blockIdx.x + gridDim.x * blockIdx.y;
    const int x = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
    mt = wg / gridDim.y;
    nt = wg - mt * gridDim.y;
  }
}

template <int BM, int BN, int MODE, int RING>
__device__ __forceinline__ void glds_body(const ConvParams& p, char* smem, int mt, int nt);

template <int BM, int BN, int MODE, int RING = GLDS_NBUF>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GldsOcc<BM, BN, RING>::W)))
conv_glds_kernel(const ConvParams p) {
  __shared__ __attribute__((aligned(16))) char smem[GldsSmem<BM, BN, RING>::BYTES];
  int mt, nt;
  glds_tile(p.xcd != 0, mt, nt);
  glds_body<BM, BN, MODE, RING>(p, smem, mt, nt);
}

template <int BM, int BN, int MODE, int RING>
__device__ __forceinline__ void glds_body(const ConvParams& p, char* smem, int mt, int nt) {
  constexpr int MI = BM / 32, NI = BN / 32;
  constexpr int AROWS = BM / 32;
  constexpr int BLOADS = (BN * 8 + 255) / 256;
  constexpr int NL = AROWS + BLOADS;  // DMA instructions per stage per wave
  constexpr int STAGE = GldsSmem<BM, BN, RING>::STAGE;
  constexpr bool DGRAD = (MODE == LOAD_DGRAD_FAST || MODE == LOAD_DGRAD_VEC8);
  constexpr bool FASTK = (MODE == LOAD_FAST || MODE == LOAD_DGRAD_FAST);
  static_assert(MODE != LOAD_SCALAR, "SCALAR gathers use conv_fwd_kernel");
  static_assert(RING == 1 || RING >= GLDS_NBUF, "ring depth");

  typedef __attribute__((address_space(3))) char lds_char;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_char*)smem;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = mt * BM;
  const int n0 = group_n0(p, nt, BN);
  const int nlim = group_nlim(p, n0);
  const int xoff = (n0 / p.cout_g) * p.Cin;  // grouped: this group's first x channel
  const int trow = tid >> 3;                              // row within each 32-row slab
  const int chunk = (tid & 7) ^ ((trow >> 1) & 7);        // swizzled k-chunk this lane copies
  const uint32_t wave_off = (uint32_t)__builtin_amdgcn_readfirstlane(wid) * 1024u;
  const int HoWo = p.Ho * p.Wo;
  const bf16_t* const zero = (const bf16_t*)g_zero16;
  // strided-dgrad parity class (see ConvParams::par); unused otherwise
  const bool PAR = DGRAD && FASTK && p.par > 1;
  ParClass pcv{};
  if (PAR) {
    pcv = par_class(p, (int)blockIdx.z / p.zsplits);
    if (m0 >= pcv.Mc) return;                             // whole block past this class
  }
  const int mlim = PAR ? pcv.Mc : p.M;
  stamp(p, 0);
  EpiPre<BM, BN, 256> pre;
  epi_prefetch(p, pre, m0, n0, BM, PAR);

  // per A row: image base, and the input row / column of tap (0, 0) --
  // for a strided-dgrad class, the dy row / column of the class's first tap
  // (dy pixel of class tap (th, tw) = (a_ih0 - th, a_iw0 - tw): no division
  // per stage)
  int a_img[AROWS], a_ih0[AROWS], a_iw0[AROWS], a_img2[AROWS];
#pragma unroll
  for (int j = 0; j < AROWS; ++j) {
    const int m = m0 + trow + 32 * j;
    const bool ok = m < mlim;
    const int mm = ok ? (PAR ? par_row(p, pcv, m) : m) : 0;
    const int n = hdiv(mm, p.dv_HoWo);
    const int r = mm - n * HoWo;
    const int oh = hdiv(r, p.dv_Wo);
    const int ow = r - oh * p.Wo;
    a_img[j] = n * p.H * p.W * p.ldx + xoff;
    a_img2[j] = n * p.H * p.W * p.cin2;
    if (PAR) {
      // (oh + pad - kh0) is a non-negative multiple of the stride for every
      // pixel of the class (par_class), up to the tail rows masked below
      a_ih0[j] = hdiv(oh + p.pad - pcv.kh0 + p.par, p.dv_s) - 1;
      a_iw0[j] = hdiv(ow + p.pad - pcv.kw0 + p.par, p.dv_s) - 1;
    } else if (DGRAD) {
      a_ih0[j] = oh + p.pad;
      a_iw0[j] = ow + p.pad;
    } else {
      a_ih0[j] = oh * p.stride - p.pad;
      a_iw0[j] = ow * p.stride - p.pad;
    }
    if (!ok) a_ih0[j] = -(1 << 28);
  }
  const bf16_t* b_row[BLOADS];
  bool b_ok[BLOADS];
#pragma unroll
  for (int j = 0; j < BLOADS; ++j) {
    const int co = n0 + trow + 32 * j;
    b_ok[j] = (trow + 32 * j < BN) && co < nlim;
    b_row[j] = p.w + (int64_t)(b_ok[j] ? co : 0) * p.Kp + chunk * 8;
  }

  const int cin_blocks = p.Cin / BK;
  // the folded 1 x 1 conv's steps come after this class's own taps
  const int own_steps = PAR ? pcv.nkh * pcv.nkw * cin_blocks : p.Kp / BK;
  const bool X2 = PAR && p.x2 != nullptr && (int)blockIdx.z / p.zsplits == p.cls2;
  const int total_steps = own_steps + (X2 ? p.cin2 / BK : 0);
  const bf16_t* b_row2[BLOADS];
#pragma unroll
  for (int j = 0; j < BLOADS; ++j) {
    const int co = n0 + trow + 32 * j;
    b_row2[j] = X2 ? p.w2 + (int64_t)(b_ok[j] ? co : 0) * p.kp2 + chunk * 8 : zero;
  }
  const int zs = PAR ? (int)blockIdx.z % p.zsplits : (int)blockIdx.z;
  const int s_begin = zs * p.steps_per_split;
  const int s_end = min(total_steps, s_begin + p.steps_per_split);

  const int nst = s_end - s_begin;
  const int rot = (p.krot && nst > 1) ? (mt + nt) % nst : 0;
  // issue every copy of stage s into LDS buffer buf (always NL per wave)
  auto issue = [&](int s, int buf) {
    const bool live = s < s_end;
    if (live) {  // logical step -> rotated physical step
      s += rot;
      if (s >= s_end) s -= nst;
    } else {
      s = s_begin;
    }
    if (X2 && s >= own_steps) {  // the folded 1 x 1 conv: its dy pixel, its weights
      const int c2 = (s - own_steps) * BK + chunk * 8;
      const uint32_t abase2 = lds0 + (uint32_t)(buf * STAGE) + wave_off;
#pragma unroll
      for (int j = 0; j < AROWS; ++j) {
        const int ih = a_ih0[j] - p.sh2, iw = a_iw0[j] - p.sh2;
        const bool ok = live && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        const bf16_t* src = ok ? p.x2 + (a_img2[j] + (ih * p.W + iw) * p.cin2 + c2) : zero;
        glds16(src, abase2 + (uint32_t)(j * 32 * 128));
      }
      const uint32_t bbase2 = abase2 + (uint32_t)(BM * 128);
#pragma unroll
      for (int j = 0; j < BLOADS; ++j) {
        const bf16_t* src = (live && b_ok[j]) ? b_row2[j] + (s - own_steps) * BK : zero;
        glds16(src, bbase2 + (uint32_t)(j * 32 * 128));
      }
      return;
    }
    int tap, c0;
    bool kok = live;
    int th = 0, tw = 0;
    if (PAR) {  // class tap t -> real tap; the weight column follows the real tap
      const int t = hdiv(s, p.dv_cb), cb = s - t * cin_blocks;
      th = pcv.nkw == 2 ? (t >> 1) : (pcv.nkw == 1 ? t : t / max(pcv.nkw, 1));
      tw = t - th * pcv.nkw;
      tap = (pcv.kh0 + p.par * th) * p.KW + pcv.kw0 + p.par * tw;
      c0 = cb * BK + chunk * 8;
      s = tap * cin_blocks + cb;
    } else if (FASTK) {
      tap = hdiv(s, p.dv_cb);
      c0 = (s - tap * cin_blocks) * BK + chunk * 8;
    } else {
      const int k0 = s * BK + chunk * 8;
      tap = hdiv(k0, p.dv_Cin);
      c0 = k0 - tap * p.Cin;
      kok = kok && k0 < p.K;
    }
    const int kh = hdiv(tap, p.dv_KW), kw = tap - kh * p.KW;
    const uint32_t abase = lds0 + (uint32_t)(buf * STAGE) + wave_off;
#pragma unroll
    for (int j = 0; j < AROWS; ++j) {
      int ih, iw;
      bool ok = kok;
      if (PAR) {
        ih = a_ih0[j] - th;
        iw = a_iw0[j] - tw;
        ok = ok && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      } else if (DGRAD) {
        const int nh = a_ih0[j] - kh, nw = a_iw0[j] - kw;
        ok = ok && nh >= 0 && nw >= 0;
        ih = nh; iw = nw;
        if (p.stride != 1) {
          ih = hdiv(max(nh, 0), p.dv_s);
          iw = hdiv(max(nw, 0), p.dv_s);
          ok = ok && ih * p.stride == nh && iw * p.stride == nw;
        }
        ok = ok && ih < p.H && iw < p.W;
      } else {
        ih = a_ih0[j] + kh;
        iw = a_iw0[j] + kw;
        ok = ok && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      }
      const bf16_t* src = ok ? p.x + (a_img[j] + (ih * p.W + iw) * p.ldx + c0) : zero;
      glds16(src, abase + (uint32_t)(j * 32 * 128));
    }
    const uint32_t bbase = abase + (uint32_t)(BM * 128);
#pragma unroll
    for (int j = 0; j < BLOADS; ++j) {
      const bf16_t* src = (live && b_ok[j]) ? b_row[j] + s * BK : zero;
      glds16(src, bbase + (uint32_t)(j * 32 * 128));
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // fragment read offsets: row R, logical chunk q -> R*128 + ((q ^ ((R>>1)&7)) * 16);
  // every fragment row R = (multiple of 16) + (lane & 15), so the swizzle is per-lane
  const int frow = lane & 15;
  const int swz = (frow >> 1) & 7;
  const int g4 = lane >> 4;
  auto compute = [&](int buf) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + BM * 128;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int coff = ((kk * 4 + g4) ^ swz) * 16;
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        af[i] = *(const bf16x8*)(As + (wm * (BM / 2) + i * 16 + frow) * 128 + coff);
#pragma unroll
      for (int j = 0; j < NI; ++j)
        bfr[j] = *(const bf16x8*)(Bs + (wn * (BN / 2) + j * 16 + frow) * 128 + coff);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  const int n = s_end - s_begin;
  if constexpr (RING == 1) {
    for (int t = 0; t < n; ++t) {
      if (t) __syncthreads();  // every read of the previous stage retired
      issue(s_begin + t, 0);
      vm_wait_barrier<0>();    // landed everywhere
      compute(0);
    }
  } else {
    // RING - 1 stages in flight
#pragma unroll
    for (int s0 = 0; s0 < RING - 1; ++s0) issue(s_begin + s0, s0);
    stamp(p, 1);
    int cbuf = 0;
    for (int t = 0; t < n; ++t) {
      // stage t landed everywhere (RING - 2 younger stages may be in flight);
      // stage t-1 reads retired everywhere
      vm_wait_barrier<NL * (RING - 2)>();
      if (t == 0) stamp(p, 2);
      const int ibuf = cbuf == 0 ? RING - 1 : cbuf - 1;  // (t + RING - 1) % RING
      issue(s_begin + t + RING - 1, ibuf);
      compute(cbuf);
      cbuf = cbuf == RING - 1 ? 0 : cbuf + 1;
    }
  }
  vm_wait_barrier<0>();  // drain the zero-page prefetches; all reads done before the C tile
  stamp(p, 3);
  conv_epilogue<BM, BN>(p, acc, smem, m0, n0, BM, pcv, PAR, pre);
  if (p.stamps != nullptr) {
    __syncthreads();
    stamp(p, 4);
  }
}

// ---------------------------------------------------------------------------
// Halo-tiled 3x3 / stride-1 / pad-1 convolution (the CIFAR ResNet body).
// The implicit-GEMM kernels above gather im2col rows, so every input pixel
// crosses L2 -> LDS nine times: ~113 MB of L2 traffic for one 64->64 32x32
// conv at batch 64, which at ~70 GB/s per CU of L2-served gathers is the
// kernel's whole runtime.  Here a block owns BM = 128 output pixels made of
// whole output rows (R = 128 / W rows of one image, or 128 / (H*W) whole
// images), stages the (rows + 2) x (W + 2) input patch of one 64-channel
// chunk into LDS ONCE, and forms all nine taps from it: A traffic drops ~5x.
// K loop = channel chunks (runtime) x 9 taps (unrolled).  Per step the
// weight tile of (chunk, tap) arrives by LDS-DMA into a 3-deep ring; the next
// chunk's patch (7 DMA pieces of 32 rows) is spread over taps 0..6, so every
// step's DMA count -- and hence every counted vmcnt -- is a compile-time
// constant.  FLIP mirrors the taps (dgrad: dx = conv(dy, w^T flipped)).
constexpr int HALO_BM = 128;
constexpr int HALO_PIECES = 7;                        // patch DMA pieces (32 rows each)
constexpr int HALO_PROWS = HALO_PIECES * 32;          // 224 patch rows max
constexpr int HALO1_PIECES = 8;                       // single-chunk kernel: 256 rows
constexpr int HALO1_PROWS = HALO1_PIECES * 32;
// A block owns hpb <= 128 output pixels: hrows whole output rows of one
// image (W * hrows <= 128, hrows | H), or himgs whole images (H*W*himgs <=
// 128).  Maps whose width does not divide 128 (ImageNet 56 / 28 / 14 / 7)
// leave the MFMA rows past hpb idle (<= 23 %) instead of falling back to the
// im2col gather kernels, which re-read every input pixel 9 times.

// RING = weight tiles in flight + 1.  RING 3 (80 KB: two blocks per CU) is
// the generic kernel; RING 8 (120 KB, one block per CU, prefetch 7 taps
// ahead) is for grids of about one block per CU (the 16x16 / 8x8 CIFAR
// stages and ImageNet's deep stages), where nothing else hides the L2
// round trip of each tap's weight tile.
template <int BN, int RING = 3>
struct HaloSmem {
  static constexpr int PATCH = HALO_PROWS * 128;      // bytes per patch buffer
  static constexpr int BT = BN * 128;                 // bytes per weight tile
  static constexpr int PIPE = 2 * PATCH + RING * BT;
  static constexpr int CTILE = ConvSmem<HALO_BM, BN>::CTILE;
  static constexpr int BYTES = PIPE > CTILE ? PIPE : CTILE;
};

template <int BN, bool FLIP, int RING = 3>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu((BN >= 128 || RING > 3) ? 1 : 2)))
conv_halo_kernel(const ConvParams p) {
  constexpr int BM = HALO_BM;
  constexpr int MI = BM / 32, NI = BN / 32;
  constexpr int BLOADS = (BN * 8 + 255) / 256;
  constexpr int PATCH = HaloSmem<BN, RING>::PATCH;
  constexpr int BT = HaloSmem<BN, RING>::BT;

  __shared__ __attribute__((aligned(16))) char smem[HaloSmem<BN, RING>::BYTES];
  typedef __attribute__((address_space(3))) char lds_char;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_char*)smem;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int PB = p.hpb;                       // output pixels of this block (<= BM)
  const int m0 = blockIdx.x * PB;
  const int n0 = blockIdx.y * BN;
  const uint32_t wave_off = (uint32_t)__builtin_amdgcn_readfirstlane(wid) * 1024u;
  const bf16_t* const zero = (const bf16_t*)g_zero16;
  stamp(p, 0);

  // block geometry: IMGS images of RH output rows each
  const int W = p.W, H = p.H;
  const int IMGS = p.himgs;
  const int RH = p.hrows;
  const int PW = W + 2;                       // patch row length (pixels)
  const int PH = RH + 2;                      // patch rows per image
  const int grow0 = hdiv(m0, p.dv_W);                   // first global output row (n*H + oh)
  const int img0 = hdiv(grow0, p.dv_H);
  const int oh0 = grow0 - img0 * H;
  EpiPre<BM, BN, 256> pre;
  epi_prefetch(p, pre, m0, n0, PB, false);
  stamp(p, 5);

  // patch DMA: piece j covers patch rows 32j..32j+31; this thread's row/chunk
  const int trow = tid >> 3;
  // patch swizzle s(r) = r & 6 (rows mod 32j): any 16 consecutive patch rows
  // -- a fragment read at ANY tap offset -- hit 16 distinct 16-B slots of the
  // ds_read_b128 lane groups; the GEMM swizzle (r >> 1) & 7 assumed aligned
  // rows and cost ~1.75-way conflicts on the shifted tap views
  const int chunk = (tid & 7) ^ (trow & 6);
  int p_src[HALO_PIECES];                     // element offset of the patch pixel, or -1
  {
    const int P = IMGS * PH * PW;
#pragma unroll
    for (int j = 0; j < HALO_PIECES; ++j) {
      const int pr = 32 * j + trow;
      int off = -1;
      if (pr < P) {
        const int img = hdiv(pr, p.dv_PHPW);
        const int rem = pr - img * PH * PW;
        const int ir = hdiv(rem, p.dv_PW), ic = rem - ir * PW;
        const int n = img0 + img;
        const int ih = oh0 + ir - 1, iw = ic - 1;
        if (n < p.N && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
          off = ((n * H + ih) * W + iw) * p.Cin;
      }
      p_src[j] = off;
    }
  }
  // weight rows
  const bf16_t* b_row[BLOADS];
  bool b_ok[BLOADS];
#pragma unroll
  for (int j = 0; j < BLOADS; ++j) {
    const int co = n0 + trow + 32 * j;
    b_ok[j] = (trow + 32 * j < BN) && co < p.Cout;
    b_row[j] = p.w + (int64_t)(b_ok[j] ? co : 0) * p.Kp + chunk * 8;
  }

  stamp(p, 6);
  const int nchunks = p.Cin / BK;
  const int c_begin = blockIdx.z * p.steps_per_split;
  const int c_end = min(nchunks, c_begin + p.steps_per_split);
  const int nsteps = (c_end - c_begin) * 9;

  auto issue_b = [&](int step, int bbuf) {   // weight tile of step (chunk, tap)
    const bool live = step < nsteps;
    const int st = live ? step : 0;
    const int cc = c_begin + st / 9, tap = st - (st / 9) * 9;
    const int wtap = FLIP ? 8 - tap : tap;
    const uint32_t base = lds0 + 2 * PATCH + (uint32_t)(bbuf * BT) + wave_off;
#pragma unroll
    for (int j = 0; j < BLOADS; ++j) {
      const bf16_t* src = (live && b_ok[j]) ? b_row[j] + wtap * p.Cin + cc * BK : zero;
      glds16(src, base + (uint32_t)(j * 32 * 128));
    }
  };
  auto issue_piece = [&](int cc, int pbuf, int j) {  // patch piece j of chunk cc
    const bool live = cc < c_end;
    const int off = p_src[j];
    const bf16_t* src = (live && off >= 0) ? p.x + off + cc * BK + chunk * 8 : zero;
    glds16(src, lds0 + (uint32_t)(pbuf * PATCH) + wave_off + (uint32_t)(j * 32 * 128));
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // per A fragment: patch row of (pixel, tap 0,0)
  const int frow = lane & 15;
  const bool p8 = W == 8 && p.perm8 != 0;  // (see perm8)
  const int g4 = lane >> 4;
  int a_prow[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    int ml = wm * (BM / 2) + i * 16 + (p8 ? perm8(frow) : frow);  // local output pixel
    if (ml >= PB) ml = 0;                           // idle MFMA row (masked at the store)
    const int lr = hdiv(ml, p.dv_W), c = ml - lr * W;   // local output row, column
    const int img = hdiv(lr, p.dv_RH), r = lr - img * RH;
    a_prow[i] = (img * PH + r) * PW + c;
  }
  const int bswz = frow & 6;

  auto compute = [&](int pbuf, int bbuf, int tap) {
    const char* Ps = smem + pbuf * PATCH;
    const char* Bs = smem + 2 * PATCH + bbuf * BT;
    const int kh = tap / 3, kw = tap - (tap / 3) * 3;
    const int toff = kh * PW + kw;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int q = kk * 4 + g4;
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int pr = a_prow[i] + toff;
        af[i] = *(const bf16x8*)(Ps + pr * 128 + ((q ^ (pr & 6)) * 16));
      }
#pragma unroll
      for (int j = 0; j < NI; ++j)
        bfr[j] = *(const bf16x8*)(Bs + (wn * (BN / 2) + j * 16 + frow) * 128 + ((q ^ bswz) * 16));
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // prologue: patch of the first chunk, weight tiles of steps 0 and 1
#pragma unroll
  for (int j = 0; j < HALO_PIECES; ++j) issue_piece(c_begin, 0, j);
#pragma unroll
  for (int s0 = 0; s0 < RING - 1; ++s0) issue_b(s0, s0);
  stamp(p, 1);
  int pbuf = 0, bbuf = 0, step = 0;
  for (int cc = c_begin; cc < c_end; ++cc) {
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (RING == 3) {
        // DMAs issued after B(step): [piece(tap-2) if 0<=tap-2<7] B(step+1) [piece(tap-1) if 0<=tap-1<7]
        if (tap == 0) vm_wait_barrier<BLOADS>();
        else if (tap == 1) vm_wait_barrier<BLOADS + 1>();
        else if (tap <= 7) vm_wait_barrier<BLOADS + 2>();
        else vm_wait_barrier<BLOADS + 1>();
      } else {
        // B(step) is older than the RING-2 weight tiles issued after it, so
        // vmcnt((RING-2)*BLOADS) has it landed (counting no patch piece keeps
        // the count safe in the prologue steps too).  At tap 0 the patch of
        // this chunk (last piece issued at tap 6 of the previous chunk, two
        // weight tiles ago) must have landed as well.
        if (tap == 0) vm_wait_barrier<2 * BLOADS>();
        else vm_wait_barrier<(RING - 2) * BLOADS>();
      }
      if (step == 0) stamp(p, 2);
      int nb = bbuf + RING - 1;                  // (step + RING - 1) % RING
      if (nb >= RING) nb -= RING;
      issue_b(step + RING - 1, nb);
      if (tap < HALO_PIECES) issue_piece(cc + 1, pbuf ^ 1, tap);
      compute(pbuf, bbuf, tap);
      bbuf = bbuf == RING - 1 ? 0 : bbuf + 1;
      ++step;
    }
    pbuf ^= 1;
  }
  vm_wait_barrier<0>();
  stamp(p, 3);
  conv_epilogue<BM, BN>(p, acc, smem, m0, n0, PB, ParClass{}, false, pre, p8);
  if (p.stamps != nullptr) {
    __syncthreads();
    stamp(p, 4);
  }
}

// Single-chunk (Cin == 64) halo variant: the block's one patch is staged
// once (no second patch buffer, no dummy prefetch of a next chunk) and the
// freed LDS holds a RING-deep weight-tile ring, so weight tiles are fetched
// RING-1 taps ahead instead of 2 -- the 3-deep ring of the generic kernel
// leaves every tap waiting on an L2 round trip at these tiny per-tap MFMA
// workloads.  Still two blocks per CU.
template <int BN>
struct Halo1Smem {
  static constexpr int PATCH = HALO1_PROWS * 128;
  static constexpr int BT = BN * 128;
  static constexpr int RING = (81920 - PATCH) / BT > 9 ? 9 : (81920 - PATCH) / BT;
  static constexpr int PIPE = PATCH + RING * BT;
  static constexpr int CTILE = ConvSmem<HALO_BM, BN>::CTILE;
  static constexpr int BYTES = PIPE > CTILE ? PIPE : CTILE;
};

template <int BN, bool FLIP>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
conv_halo1_kernel(const ConvParams p) {
  constexpr int BM = HALO_BM;
  constexpr int MI = BM / 32, NI = BN / 32;
  constexpr int BLOADS = (BN * 8 + 255) / 256;
  constexpr int PATCH = Halo1Smem<BN>::PATCH;
  constexpr int BT = Halo1Smem<BN>::BT;
  constexpr int RING = Halo1Smem<BN>::RING;

  __shared__ __attribute__((aligned(16))) char smem[Halo1Smem<BN>::BYTES];
  typedef __attribute__((address_space(3))) char lds_char;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_char*)smem;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int PB = p.hpb;                       // output pixels of this block (<= BM)
  const int m0 = blockIdx.x * PB;
  const int n0 = blockIdx.y * BN;
  const uint32_t wave_off = (uint32_t)__builtin_amdgcn_readfirstlane(wid) * 1024u;
  const bf16_t* const zero = (const bf16_t*)g_zero16;

  // block geometry: IMGS images of RH output rows each
  const int W = p.W, H = p.H;
  const int IMGS = p.himgs;
  const int RH = p.hrows;
  const int PW = W + 2;                       // patch row length (pixels)
  const int PH = RH + 2;                      // patch rows per image
  const int grow0 = hdiv(m0, p.dv_W);                   // first global output row (n*H + oh)
  const int img0 = hdiv(grow0, p.dv_H);
  const int oh0 = grow0 - img0 * H;
  EpiPre<BM, BN, 256> pre;
  epi_prefetch(p, pre, m0, n0, PB, false);

  // patch DMA: piece j covers patch rows 32j..32j+31; this thread's row/chunk
  const int trow = tid >> 3;
  // patch swizzle s(r) = r & 6 (rows mod 32j): any 16 consecutive patch rows
  // -- a fragment read at ANY tap offset -- hit 16 distinct 16-B slots of the
  // ds_read_b128 lane groups; the GEMM swizzle (r >> 1) & 7 assumed aligned
  // rows and cost ~1.75-way conflicts on the shifted tap views
  const int chunk = (tid & 7) ^ (trow & 6);
  int p_src[HALO1_PIECES];                    // element offset of the patch pixel, or -1
  {
    const int P = IMGS * PH * PW;
#pragma unroll
    for (int j = 0; j < HALO1_PIECES; ++j) {
      const int pr = 32 * j + trow;
      int off = -1;
      if (pr < P) {
        const int img = hdiv(pr, p.dv_PHPW);
        const int rem = pr - img * PH * PW;
        const int ir = hdiv(rem, p.dv_PW), ic = rem - ir * PW;
        const int n = img0 + img;
        const int ih = oh0 + ir - 1, iw = ic - 1;
        if (n < p.N && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
          off = ((n * H + ih) * W + iw) * p.Cin;
      }
      p_src[j] = off;
    }
  }
  // weight rows
  const bf16_t* b_row[BLOADS];
  bool b_ok[BLOADS];
#pragma unroll
  for (int j = 0; j < BLOADS; ++j) {
    const int co = n0 + trow + 32 * j;
    b_ok[j] = (trow + 32 * j < BN) && co < p.Cout;
    b_row[j] = p.w + (int64_t)(b_ok[j] ? co : 0) * p.Kp + chunk * 8;
  }

  const int c_begin = 0, c_end = 1;  // Cin == 64: one channel chunk, 9 taps
  const int nsteps = 9;

  auto issue_b = [&](int step, int bbuf) {   // weight tile of step (chunk, tap)
    const bool live = step < nsteps;
    const int st = live ? step : 0;
    const int cc = c_begin + st / 9, tap = st - (st / 9) * 9;
    const int wtap = FLIP ? 8 - tap : tap;
    const uint32_t base = lds0 + PATCH + (uint32_t)(bbuf * BT) + wave_off;
#pragma unroll
    for (int j = 0; j < BLOADS; ++j) {
      const bf16_t* src = (live && b_ok[j]) ? b_row[j] + wtap * p.Cin + cc * BK : zero;
      glds16(src, base + (uint32_t)(j * 32 * 128));
    }
  };
  auto issue_piece = [&](int cc, int pbuf, int j) {  // patch piece j of chunk cc
    const bool live = cc < c_end;
    const int off = p_src[j];
    const bf16_t* src = (live && off >= 0) ? p.x + off + cc * BK + chunk * 8 : zero;
    glds16(src, lds0 + (uint32_t)(pbuf * PATCH) + wave_off + (uint32_t)(j * 32 * 128));
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // per A fragment: patch row of (pixel, tap 0,0)
  const int frow = lane & 15;
  const bool p8 = W == 8 && p.perm8 != 0;  // (see perm8)
  const int g4 = lane >> 4;
  int a_prow[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    int ml = wm * (BM / 2) + i * 16 + (p8 ? perm8(frow) : frow);  // local output pixel
    if (ml >= PB) ml = 0;                           // idle MFMA row (masked at the store)
    const int lr = hdiv(ml, p.dv_W), c = ml - lr * W;   // local output row, column
    const int img = hdiv(lr, p.dv_RH), r = lr - img * RH;
    a_prow[i] = (img * PH + r) * PW + c;
  }
  const int bswz = frow & 6;

  auto compute = [&](int pbuf, int bbuf, int tap) {
    const char* Ps = smem + pbuf * PATCH;
    const char* Bs = smem + PATCH + bbuf * BT;
    const int kh = tap / 3, kw = tap - (tap / 3) * 3;
    const int toff = kh * PW + kw;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int q = kk * 4 + g4;
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int pr = a_prow[i] + toff;
        af[i] = *(const bf16x8*)(Ps + pr * 128 + ((q ^ (pr & 6)) * 16));
      }
#pragma unroll
      for (int j = 0; j < NI; ++j)
        bfr[j] = *(const bf16x8*)(Bs + (wn * (BN / 2) + j * 16 + frow) * 128 + ((q ^ bswz) * 16));
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // prologue: the (only) patch, then weight tiles of steps 0 .. RING-2
#pragma unroll
  for (int j = 0; j < HALO1_PIECES; ++j) issue_piece(c_begin, 0, j);
#pragma unroll
  for (int s0 = 0; s0 < RING - 1; ++s0) issue_b(s0, s0);
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    // DMAs issued after B(tap): B(tap+1) .. B(tap+RING-2), always RING-2 tiles
    // (tiles past the last step are zero-page dummies, so counts stay constant)
    vm_wait_barrier<(RING - 2) * BLOADS>();
    issue_b(tap + RING - 1, (tap + RING - 1) % RING);
    compute(0, tap % RING, tap);
  }
  vm_wait_barrier<0>();
  conv_epilogue<BM, BN>(p, acc, smem, m0, n0, PB, ParClass{}, false, pre, p8);
}

// Split-K combine: y = epilogue(sum_z partial[z]) in fixed z order.
// Cout % 8 == 0: one thread per 8 channels (16-byte traffic).
__global__ void __launch_bounds__(256) conv_splitk_epilogue(const ConvParams p, int splits) {
  const int64_t total = (int64_t)p.M * p.Cout;
  if ((p.Cout & 7) == 0) {
    const int64_t t8 = total >> 3;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < t8;
         i += (int64_t)gridDim.x * blockDim.x) {
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int z = 0; z < splits; ++z) {
        const float* src = p.partial + (int64_t)z * total + i * 8;
        const float4 lo = *(const float4*)src, hi = *(const float4*)(src + 4);
        v[0] += lo.x; v[1] += lo.y; v[2] += lo.z; v[3] += lo.w;
        v[4] += hi.x; v[5] += hi.y; v[6] += hi.z; v[7] += hi.w;
      }
      const int m = (int)((i * 8) / p.Cout);
      const int co = (int)(i * 8 - (int64_t)m * p.Cout);
      float sc[8], bi[8];
      load_scale_bias8(p, co, sc, bi);
      epilogue_store8(p, m, co, v, sc, bi);
    }
    return;
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    float a = 0.f;
    for (int z = 0; z < splits; ++z) a += p.partial[(int64_t)z * total + i];
    const int m = (int)(i / p.Cout);
    const int co = (int)(i - (int64_t)m * p.Cout);
    epilogue_store(p, m, co, a);
  }
}

// 3x3 / stride 1 / pad 1 "same" conv with Cin % 64 == 0 whose block
// geometry (see HALO_BM) has a patch of at most `max_rows` rows; fills
// p.hrows / p.himgs / p.hpb.
bool halo_geometry(ConvParams& p, int max_rows, int cap = HALO_BM) {
  if (p.KH != 3 || p.KW != 3 || p.stride != 1 || p.pad != 1) return false;
  if (p.Ho != p.H || p.Wo != p.W || p.Cin % BK || p.Kp != 9 * p.Cin) return false;
  if (p.W > HALO_BM) return false;
  int imgs = 1, rows = 0;
  if (p.H * p.W <= cap) {
    imgs = cap / (p.H * p.W);
    while (imgs > 1 && imgs * (p.H + 2) * (p.W + 2) > max_rows) --imgs;
    rows = p.H;
  } else {
    for (int r = cap / p.W; r >= 1; --r)
      if (p.H % r == 0 && (r + 2) * (p.W + 2) <= max_rows) { rows = r; break; }
  }
  if (rows <= 0 || imgs * (rows + 2) * (p.W + 2) > max_rows) return false;
  const int pb = imgs * rows * p.W;
  if (4 * pb < 3 * cap && !(p.H * p.W <= HALO_BM)) return false;  // < 75 % rows busy
  p.hrows = rows;
  p.himgs = imgs;
  p.hpb = pb;
  make_hdiv((uint32_t)p.W, p.dv_W);
  make_hdiv((uint32_t)p.H, p.dv_H);
  make_hdiv((uint32_t)(p.W + 2), p.dv_PW);
  make_hdiv((uint32_t)((rows + 2) * (p.W + 2)), p.dv_PHPW);
  make_hdiv((uint32_t)rows, p.dv_RH);
  return true;
}

bool halo_eligible(ConvParams& p) {
  static const bool on = [] {
    const char* e = getenv("MDA_CONV_HALO");
    return !(e && e[0] == '0');
  }();
  if (!on) return false;
  return halo_geometry(p, p.Cin == BK ? HALO1_PROWS : HALO_PROWS);
}

// grouped convs: re-pick the N tile width for the group size (MDA_GROUPED_BN=0: off, A/B)
bool grouped_bn_fit() {
  static const bool on = [] {
    const char* e = getenv("MDA_GROUPED_BN");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool use_halo1() {
  static const bool on = [] {
    const char* e = getenv("MDA_CONV_HALO1");
    return !(e && e[0] == '0');
  }();
  return on;
}

// MDA_REG1X1_MIN_M: smallest M of a 1x1 forward conv sent to the register-staged kernel
int reg1x1_min_m() {
  static const int v = [] {
    const char* e = getenv("MDA_REG1X1_MIN_M");
    return e ? atoi(e) : 32768;
  }();
  return v;
}

bool use_xcd_remap() {
  static const bool on = [] {
    const char* e = getenv("MDA_CONV_XCD");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool use_krot() {
  static const bool on = [] {
    const char* e = getenv("MDA_CONV_KROT");
    return e && e[0] == '1';
  }();
  return on;
}

bool use_par_dgrad() {
  static const bool on = [] {
    const char* e = getenv("MDA_DGRAD_PARITY");
    return !(e && e[0] == '0');
  }();
  return on;
}

// MDA_HALO_RING: 3 (default) / 8 / 0 (= 8 for grids of <= 320 blocks); the deep
// ring measured no faster on the CIFAR step (1.295 vs 1.274 ms)
int halo_ring() {
  static const int v = [] {
    const char* e = getenv("MDA_HALO_RING");
    return e ? atoi(e) : 3;
  }();
  return v;
}

// largest per-block K-step count that takes the single-stage glds variant
int ring1_max() {
  static const int v = [] {
    const char* e = getenv("MDA_GLDS_RING1_MAX");
    return e ? atoi(e) : 4;
  }();
  return v;
}

bool use_glds() {
  static const bool on = [] {
    const char* e = getenv("MDA_CONV_GLDS");
    return !(e && e[0] == '0');
  }();
  return on;
}

#define DLAUNCH(K, G, B, S, ST, P) hipLaunchKernelGGL(K, G, B, S, ST, P)

template <int BM, int BN>
int launch_tile(const ConvParams& p, int mode, int splits, hipStream_t st) {
  const int ny = p.cout_g < p.Cout ? (p.Cout / p.cout_g) * ((p.cout_g + BN - 1) / BN)
                                   : (p.Cout + BN - 1) / BN;
  dim3 grid((p.M + BM - 1) / BM, ny, splits);
  if (p.cout_g < p.Cout && (mode == LOAD_SCALAR || !use_glds())) return (int)hipErrorInvalidValue;
  // large-M 1x1 forward convs are output-bandwidth bound: the register-staged
  // kernel streams them 1.2-1.4x faster than the LDS-DMA one
  // (profiles/r3_conv1x1_imagenet.md)
  // (also every short-K one: the CIFAR shortcuts, flagship 0.92-0.93 -> 0.913 ms)
  const bool reg1x1 = p.KH == 1 && p.KW == 1 && p.cout_g >= p.Cout &&
                      (p.M >= reg1x1_min_m() || p.Kp <= 4 * BK) &&
                      (mode == LOAD_FAST || mode == LOAD_VEC8);
  if (mode != LOAD_SCALAR && use_glds() && !reg1x1 && p.steps_per_split <= ring1_max()) {  // short-K blocks
    if (mode == LOAD_FAST)
      DLAUNCH((conv_glds_kernel<BM, BN, LOAD_FAST, 1>), grid, dim3(256), 0, st, p);
    else if (mode == LOAD_VEC8)
      DLAUNCH((conv_glds_kernel<BM, BN, LOAD_VEC8, 1>), grid, dim3(256), 0, st, p);
    else if (mode == LOAD_DGRAD_FAST)
      DLAUNCH((conv_glds_kernel<BM, BN, LOAD_DGRAD_FAST, 1>), grid, dim3(256), 0, st, p);
    else
      DLAUNCH((conv_glds_kernel<BM, BN, LOAD_DGRAD_VEC8, 1>), grid, dim3(256), 0, st, p);
    return (int)hipGetLastError();
  }
  if (mode != LOAD_SCALAR && use_glds() && !reg1x1) {
    if (mode == LOAD_FAST)
      DLAUNCH((conv_glds_kernel<BM, BN, LOAD_FAST>), grid, dim3(256), 0, st, p);
    else if (mode == LOAD_VEC8)
      DLAUNCH((conv_glds_kernel<BM, BN, LOAD_VEC8>), grid, dim3(256), 0, st, p);
    else if (mode == LOAD_DGRAD_FAST)
      DLAUNCH((conv_glds_kernel<BM, BN, LOAD_DGRAD_FAST>), grid, dim3(256), 0, st, p);
    else
      DLAUNCH((conv_glds_kernel<BM, BN, LOAD_DGRAD_VEC8>), grid, dim3(256), 0, st, p);
    return (int)hipGetLastError();
  }
  if (mode == LOAD_FAST)
    DLAUNCH((conv_fwd_kernel<BM, BN, LOAD_FAST>), grid, dim3(256), 0, st, p);
  else if (mode == LOAD_VEC8)
    DLAUNCH((conv_fwd_kernel<BM, BN, LOAD_VEC8>), grid, dim3(256), 0, st, p);
  else if (mode == LOAD_DGRAD_FAST)
    DLAUNCH((conv_fwd_kernel<BM, BN, LOAD_DGRAD_FAST>), grid, dim3(256), 0, st, p);
  else if (mode == LOAD_DGRAD_VEC8)
    DLAUNCH((conv_fwd_kernel<BM, BN, LOAD_DGRAD_VEC8>), grid, dim3(256), 0, st, p);
  else
    DLAUNCH((conv_fwd_kernel<BM, BN, LOAD_SCALAR>), grid, dim3(256), 0, st, p);
  return (int)hipGetLastError();
}

}  // namespace

uint64_t* g_stamps = nullptr;  // diagnostics (mda_conv_set_stamps)

// Diagnostics: subsequent conv launches write per-block phase timestamps into
// buf (8 x uint64 per block; instrumented kernels only); null turns it off.
MDA_API int mda_conv_set_stamps(void* buf) {
  g_stamps = (uint64_t*)buf;
  return 0;
}

// Host-side tile / split-K choice (also used by Python to size the workspace).
// Returns tile code BM*1000+BN in *tile and the split count in *splits.
MDA_API int mda_conv_plan(int64_t M, int64_t Cout, int64_t Kp, int64_t* tile, int64_t* splits) {
  // >= 1 workgroup per CU on 256 CUs before splitting K (MDA_CONV_TARGET overrides)
  static const int64_t target = [] {
    const char* e = getenv("MDA_CONV_TARGET");
    return e ? (int64_t)atoi(e) : (int64_t)256;  // A/B: profiles/r2_conv_target_ab.md
  }();
  int bn = Cout <= 32 ? 32 : (Cout <= 64 ? 64 : 128);
  int bm = 128;
  auto blocks = [&](int bm_, int bn_) { return ((M + bm_ - 1) / bm_) * ((Cout + bn_ - 1) / bn_); };
  int64_t steps = Kp / BK;
  if (steps <= ring1_max() && bn == 128) bn = 64;  // short K: 4 blocks per CU (see GldsSmem)
  if (blocks(bm, bn) < target && bn == 128) bn = 64;
  if (blocks(bm, bn) < target) bm = 64;
  int64_t nb = blocks(bm, bn);
  int64_t sp = 1;
  while (nb * sp < target && steps / (sp * 2) >= 4 && sp < 8) sp *= 2;
  *tile = bm * 1000 + bn;
  *splits = sp;
  return 0;
}

extern "C" int mda_conv1x1_stream_try(const void* x, const void* w, const float* scale,
                                      const float* bias, const void* res, void* y, void* preact,
                                      void* slot, int64_t N, int64_t H, int64_t W, int64_t K,
                                      int64_t Kp, int64_t Ho, int64_t Wo, int64_t Cout,
                                      int64_t stride, int64_t act, hipStream_t st);

namespace {

// loader constants of the glds kernel (XCD order, K rotation, multiply-shift divisors)
void glds_prep(ConvParams& p) {
  static const int perm8_on = [] {
    const char* e = getenv("MDA_HALO_PERM8");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  p.perm8 = perm8_on;
  p.xcd = use_xcd_remap() ? 1 : 0;
  p.krot = use_krot() ? 1 : 0;
  make_hdiv((uint32_t)std::max(p.Cin, 1), p.dv_Cin);
  make_hdiv((uint32_t)std::max(p.KW, 1), p.dv_KW);
  make_hdiv((uint32_t)std::max(p.Cin / BK, 1), p.dv_cb);
  make_hdiv((uint32_t)std::max(p.Ho * p.Wo, 1), p.dv_HoWo);
  make_hdiv((uint32_t)std::max(p.Wo, 1), p.dv_Wo);
  make_hdiv((uint32_t)std::max(p.stride, 1), p.dv_s);
}

int dispatch(ConvParams& p, int mode, int64_t tile, int64_t splits, hipStream_t st, int halo = 0) {
  if (p.Kp % BK || p.Kp < p.K) return (int)hipErrorInvalidValue;
  if (p.ldx <= 0) p.ldx = p.Cin;
  if (p.cout_g <= 0) p.cout_g = p.Cout;
  // memory-bound 1x1 convs (and stride-1 1x1 dgrads): the streaming kernel
  // (conv1x1.hip) -- transposed MFMA, resident weights, stores straight from
  // the accumulators; -1 = shape not served, fall through
  if (p.KH == 1 && p.KW == 1 && p.pad == 0 && p.cout_g >= p.Cout && p.ldx == p.Cin &&
      p.bnb_slot == nullptr && p.stats_part == nullptr && p.stamps == nullptr &&
      (mode == LOAD_FAST || mode == LOAD_VEC8 ||
       ((mode == LOAD_DGRAD_FAST || mode == LOAD_DGRAD_VEC8) && p.stride == 1))) {
    // (K = Cin a multiple of 32 is enough there: LOAD_VEC8 covers K = 32 / 96 / ...)
    const bool fwd = mode == LOAD_FAST || mode == LOAD_VEC8;
    const int rc = mda_conv1x1_stream_try(p.x, p.w, p.scale, p.bias, p.res, p.y, p.preact,
                                          p.stats_slot, p.N, p.H, p.W, p.Cin, p.Kp, p.Ho, p.Wo,
                                          p.Cout, fwd ? p.stride : 1, p.act, st);
    if (rc != -1) return rc;
  }
  glds_prep(p);
  if (p.cout_g < p.Cout) {  // grouped: group-aligned tiles on the glds kernel only
    if (p.Cout % p.cout_g || p.ldx != p.Cin * (p.Cout / p.cout_g) || p.cout_g % 8 || p.Cin % 8)
      return (int)hipErrorInvalidValue;
    halo = 0;
    p.par = 0;
  }
  const int64_t xb = (int64_t)p.N * p.H * p.W * p.ldx * 2, wb = (int64_t)p.Cout * p.Kp * 2;
  if (xb >= ((int64_t)1 << 31) || wb >= ((int64_t)1 << 31) || (int64_t)p.M * p.Cout >= ((int64_t)1 << 31))
    return (int)hipErrorInvalidValue;  // 32-bit buffer offsets
  p.x_bytes = (int)xb;
  p.w_bytes = (int)wb;
  if (tile == 0 || splits == 0) mda_conv_plan(p.M, p.Cout, p.Kp, &tile, &splits);
  if (splits > 1 && p.partial == nullptr) return (int)hipErrorInvalidValue;
  if (p.cout_g < p.Cout && grouped_bn_fit()) {
    // group-aligned N tiles: the tile width that pads a group least (the
    // plan's width is chosen for the whole Cout).  ShuffleNetV1's groups of
    // 24 / 72 / 80 / 160 channels waste 25-62 % of a 64 / 128-wide tile.
    const int cg = p.cout_g;
    int best = (int)(tile % 1000), best_pad = (cg + best - 1) / best * best;
    for (int bn : {128, 64, 32}) {
      const int pad = (cg + bn - 1) / bn * bn;
      if (pad * 8 <= cg * 9) { best = bn; best_pad = pad; break; }  // <= 12.5 % padding
      if (pad < best_pad) { best = bn; best_pad = pad; }
    }
    tile = tile / 1000 * 1000 + best;
  }
  int rc;
  if (p.x2 != nullptr && (halo || p.par <= 1 || splits != 1 || p.cin2 % BK || p.cls2 < 0 ||
                          p.cls2 >= p.par * p.par))
    return MDA_NOT_SERVED;  // a folded 1 x 1 conv needs the strided (parity) glds path
  if (halo) {
    const int nchunks = p.Cin / BK;
    // the multi-chunk kernel double-buffers patches of at most HALO_PROWS rows
    if (!(nchunks == 1 && splits == 1 && use_halo1()) &&
        p.himgs * (p.hrows + 2) * (p.W + 2) > HALO_PROWS)
      halo = 0;
  }
  if (halo) {  // halo kernel: split over 64-channel chunks, hpb pixels per block
    const int nchunks = p.Cin / BK;
    p.steps_per_split = (int)((nchunks + splits - 1) / splits);
    // (halving the channel tile of 8x8 convs with fewer blocks than CUs helped
    // the student alone but not beside the look-ahead teacher: deleted in
    // round 6, profiles/r6_ab.md)
    const int bn = p.Cout <= 32 ? 32 : 64;
    dim3 grid((p.M + p.hpb - 1) / p.hpb, (p.Cout + bn - 1) / bn, (int)splits);
    if (nchunks == 1 && splits == 1 && use_halo1()) {
      if (bn == 32) {
        if (halo == 2) DLAUNCH((conv_halo1_kernel<32, true>), grid, dim3(256), 0, st, p);
        else DLAUNCH((conv_halo1_kernel<32, false>), grid, dim3(256), 0, st, p);
      } else {
        if (halo == 2) DLAUNCH((conv_halo1_kernel<64, true>), grid, dim3(256), 0, st, p);
        else DLAUNCH((conv_halo1_kernel<64, false>), grid, dim3(256), 0, st, p);
      }
    } else {
      const int64_t nblocks = (int64_t)grid.x * grid.y * grid.z;
      const bool deep = halo_ring() == 8 || (halo_ring() == 0 && nblocks <= 320);
      if (bn == 32) {
        if (deep) {
          if (halo == 2) DLAUNCH((conv_halo_kernel<32, true, 8>), grid, dim3(256), 0, st, p);
          else DLAUNCH((conv_halo_kernel<32, false, 8>), grid, dim3(256), 0, st, p);
        } else {
          if (halo == 2) DLAUNCH((conv_halo_kernel<32, true>), grid, dim3(256), 0, st, p);
          else DLAUNCH((conv_halo_kernel<32, false>), grid, dim3(256), 0, st, p);
        }
      } else {
        if (deep) {
          if (halo == 2) DLAUNCH((conv_halo_kernel<64, true, 8>), grid, dim3(256), 0, st, p);
          else DLAUNCH((conv_halo_kernel<64, false, 8>), grid, dim3(256), 0, st, p);
        } else {
          if (halo == 2) DLAUNCH((conv_halo_kernel<64, true>), grid, dim3(256), 0, st, p);
          else DLAUNCH((conv_halo_kernel<64, false>), grid, dim3(256), 0, st, p);
        }
      }
    }
    rc = (int)hipGetLastError();
  } else if (p.par > 1) {
    // strided dgrad by parity class (glds kernel, Cout % 64 == 0 only)
    const int s2 = p.par * p.par;
    int steps = ((p.KH + p.par - 1) / p.par) * ((p.KW + p.par - 1) / p.par) * (p.Cin / BK);
    if (p.x2 != nullptr) {  // the folded 1 x 1 conv's class: its own taps + cin2 / 64
      const ParClass c = par_class(p, p.cls2);
      steps = std::max(steps, c.nkh * c.nkw * (p.Cin / BK) + p.cin2 / BK);
    }
    p.zsplits = (int)splits;
    p.steps_per_split = (int)((steps + splits - 1) / splits);
    const int bm = (int)(tile / 1000), bn = (int)(tile % 1000);
    const int mc = p.N * ((p.Ho + p.par - 1) / p.par) * ((p.Wo + p.par - 1) / p.par);
    dim3 grid((mc + bm - 1) / bm, (p.Cout + bn - 1) / bn, s2 * (int)splits);
    switch (tile) {
      case 128128: DLAUNCH((conv_glds_kernel<128, 128, LOAD_DGRAD_FAST>), grid, dim3(256), 0, st, p); break;
      case 128064: DLAUNCH((conv_glds_kernel<128, 64, LOAD_DGRAD_FAST>), grid, dim3(256), 0, st, p); break;
      case 128032: DLAUNCH((conv_glds_kernel<128, 32, LOAD_DGRAD_FAST>), grid, dim3(256), 0, st, p); break;
      case 64128: DLAUNCH((conv_glds_kernel<64, 128, LOAD_DGRAD_FAST>), grid, dim3(256), 0, st, p); break;
      case 64064: DLAUNCH((conv_glds_kernel<64, 64, LOAD_DGRAD_FAST>), grid, dim3(256), 0, st, p); break;
      case 64032: DLAUNCH((conv_glds_kernel<64, 32, LOAD_DGRAD_FAST>), grid, dim3(256), 0, st, p); break;
      default: return (int)hipErrorInvalidValue;
    }
    rc = (int)hipGetLastError();
  } else {
  const int steps = p.Kp / BK;
  p.steps_per_split = (int)((steps + splits - 1) / splits);
  switch (tile) {
    case 128128: rc = launch_tile<128, 128>(p, mode, splits, st); break;
    case 128064: rc = launch_tile<128, 64>(p, mode, splits, st); break;
    case 128032: rc = launch_tile<128, 32>(p, mode, splits, st); break;
    case 64128: rc = launch_tile<64, 128>(p, mode, splits, st); break;
    case 64064: rc = launch_tile<64, 64>(p, mode, splits, st); break;
    case 64032: rc = launch_tile<64, 32>(p, mode, splits, st); break;
    default: return (int)hipErrorInvalidValue;
  }
  }
  if (rc || splits <= 1) return rc;
  int64_t total = (int64_t)p.M * p.Cout;
  int64_t work = (p.Cout % 8 == 0) ? total / 8 : total;
  int blocks = (int)std::min<int64_t>((work + 255) / 256, 2048);
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
  ConvParams p{};
  p.x = (const bf16_t*)x; p.w = (const bf16_t*)w; p.scale = scale; p.bias = bias;
  p.res = (const bf16_t*)res; p.y = (bf16_t*)y; p.preact = (bf16_t*)preact; p.partial = partial;
  p.N = N; p.H = H; p.W = W; p.Cin = Cin; p.Ho = Ho; p.Wo = Wo; p.Cout = Cout; p.KH = KH;
  p.KW = KW; p.stride = stride; p.pad = pad; p.K = KH * KW * Cin; p.Kp = Kp; p.M = N * Ho * Wo;
  p.act = act;
  p.par = 0;
  p.zsplits = 1;
  p.stats_part = nullptr;
  p.stats_slot = nullptr;
  p.stamps = g_stamps;
  int mode = (Cin % BK == 0) ? LOAD_FAST : (Cin % 8 == 0 ? LOAD_VEC8 : LOAD_SCALAR);
  return dispatch(p, mode, tile, splits, st, halo_eligible(p) ? 1 : 0);
}

// Input gradient of a convolution (any stride): dx[N, H, W, Cin] =
// sum_{kh,kw,co} dy[N, (ih+pad-kh)/s, (iw+pad-kw)/s, co] * w[co, ci, kh, kw].
// wt: weights packed [Cin][Kp] with k = (kh*KW + kw)*Cout + co (mda_pack_conv_weights).
// dy: [N, Ho, Wo, Cout]; requires Cout % 8 == 0.
MDA_API int mda_conv_dgrad_res(const void* dy, const void* wt, void* dx, float* partial,
                               const void* res, int64_t N, int64_t H, int64_t W, int64_t Cin,
                               int64_t Ho, int64_t Wo, int64_t Cout, int64_t KH, int64_t KW,
                               int64_t stride, int64_t pad, int64_t Kp, int64_t tile,
                               int64_t splits, hipStream_t st);

MDA_API int mda_conv_dgrad_bnsum(const void* dy, const void* wt, void* dx, float* partial,
                                 const void* res, int64_t N, int64_t H, int64_t W, int64_t Cin,
                                 int64_t Ho, int64_t Wo, int64_t Cout, int64_t KH, int64_t KW,
                                 int64_t stride, int64_t pad, int64_t Kp, int64_t tile,
                                 int64_t splits, const void* bn_y, const void* bn_res,
                                 const float* bn_stats, int64_t bn_act, void* region,
                                 hipStream_t st);
MDA_API int mda_conv_dgrad_bnsum_g(const void* dy, const void* wt, void* dx, float* partial,
                                   const void* res, int64_t N, int64_t H, int64_t W, int64_t Cin,
                                   int64_t Ho, int64_t Wo, int64_t Cout, int64_t KH, int64_t KW,
                                   int64_t stride, int64_t pad, int64_t Kp, int64_t tile,
                                   int64_t splits, const void* bn_y, const void* bn_res,
                                   const float* bn_stats, int64_t bn_act, void* region,
                                   int64_t groups, const float* bn_vres, int64_t bn_mh,
                                   int64_t bn_rstride, hipStream_t st);

MDA_API int mda_conv_dgrad(const void* dy, const void* wt, void* dx, float* partial, int64_t N,
                           int64_t H, int64_t W, int64_t Cin, int64_t Ho, int64_t Wo,
                           int64_t Cout, int64_t KH, int64_t KW, int64_t stride, int64_t pad,
                           int64_t Kp, int64_t tile, int64_t splits, hipStream_t st) {
  return mda_conv_dgrad_res(dy, wt, dx, partial, nullptr, N, H, W, Cin, Ho, Wo, Cout, KH, KW,
                            stride, pad, Kp, tile, splits, st);
}

// dx = dgrad(dy) (+ res): the residual-add epilogue sums the gradient another
// consumer of the same activation produced (a residual fork), so autograd
// never launches that add.  res: [N, H, W, Cin] bf16 or null.
MDA_API int mda_conv_dgrad_res(const void* dy, const void* wt, void* dx, float* partial,
                               const void* res, int64_t N, int64_t H, int64_t W, int64_t Cin,
                               int64_t Ho, int64_t Wo, int64_t Cout, int64_t KH, int64_t KW,
                               int64_t stride, int64_t pad, int64_t Kp, int64_t tile,
                               int64_t splits, hipStream_t st) {
  return mda_conv_dgrad_bnsum(dy, wt, dx, partial, res, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride,
                              pad, Kp, tile, splits, nullptr, nullptr, nullptr, 0, nullptr, st);
}

// dx = dgrad(dy) (+ res) that also adds the BN-backward sums of the layer
// whose output gradient dx is (ConvParams::bnb_*): bn_y = that BN's input
// [N, H, W, Cin], bn_res = its residual (or null), bn_stats = its [4][Cin]
// mean / rstd / scale / shift, bn_act its activation, region a fresh zeroed
// BnRegion for Cin channels.  Requires splits == 1 (the split-K combine has
// no reduction epilogue) and Cin % 8 == 0.
MDA_API int mda_conv_dgrad_bnsum(const void* dy, const void* wt, void* dx, float* partial,
                                 const void* res, int64_t N, int64_t H, int64_t W, int64_t Cin,
                                 int64_t Ho, int64_t Wo, int64_t Cout, int64_t KH, int64_t KW,
                                 int64_t stride, int64_t pad, int64_t Kp, int64_t tile,
                                 int64_t splits, const void* bn_y, const void* bn_res,
                                 const float* bn_stats, int64_t bn_act, void* region,
                                 hipStream_t st) {
  return mda_conv_dgrad_bnsum_g(dy, wt, dx, partial, res, N, H, W, Cin, Ho, Wo, Cout, KH, KW,
                                stride, pad, Kp, tile, splits, bn_y, bn_res, bn_stats, bn_act,
                                region, 1, nullptr, 0, 0, st);
}

// Grouped dgrad (groups > 1): dx[.., g*Cin/G + ci] sums only group g's output
// channels; wt packed [Cin][KpT] with k = tap * (Cout/G) + co_in_group
// (mda_pack_conv_weights_gc).  The GEMM runs with group-aligned tiles.
static int conv_dgrad_impl(const void* dy, const void* wt, void* dx, float* partial,
                           const void* res, int64_t N, int64_t H, int64_t W, int64_t Cin,
                           int64_t Ho, int64_t Wo, int64_t Cout, int64_t KH, int64_t KW,
                           int64_t stride, int64_t pad, int64_t Kp, int64_t tile, int64_t splits,
                           const void* bn_y, const void* bn_res, const float* bn_stats,
                           int64_t bn_act, void* region, int64_t groups, const float* bn_vres,
                           int64_t bn_mh, int64_t bn_rstride, const void* x2, const void* w2,
                           int64_t cin2, int64_t kp2, hipStream_t st);

MDA_API int mda_conv_dgrad_bnsum_g(const void* dy, const void* wt, void* dx, float* partial,
                                   const void* res, int64_t N, int64_t H, int64_t W, int64_t Cin,
                                   int64_t Ho, int64_t Wo, int64_t Cout, int64_t KH, int64_t KW,
                                   int64_t stride, int64_t pad, int64_t Kp, int64_t tile,
                                   int64_t splits, const void* bn_y, const void* bn_res,
                                   const float* bn_stats, int64_t bn_act, void* region,
                                   int64_t groups, const float* bn_vres, int64_t bn_mh,
                                   int64_t bn_rstride, hipStream_t st) {
  return conv_dgrad_impl(dy, wt, dx, partial, res, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride,
                         pad, Kp, tile, splits, bn_y, bn_res, bn_stats, bn_act, region, groups,
                         bn_vres, bn_mh, bn_rstride, nullptr, nullptr, 0, 0, st);
}

// mda_conv_dgrad_bnsum_g of a stride-s conv with a 1 x 1 / stride-s / pad-0
// conv on the same input folded in (ConvParams::x2): dx = dgrad(dy; wt) +
// dgrad(dy2; wt2), dy2 [N, Ho, Wo, cin2] (the folded conv's output gradient,
// same extent as dy), wt2 its dgrad operand [Cin][kp2].  A residual block's
// conv1 and projection shortcut share their input: one launch for both input
// gradients, no parked gradient, no residual add.  Returns MDA_NOT_SERVED
// (nothing launched) when the shapes do not take the parity (strided glds) path.
MDA_API int mda_conv_dgrad_bnsum2(const void* dy, const void* wt, void* dx, int64_t N, int64_t H,
                                  int64_t W, int64_t Cin, int64_t Ho, int64_t Wo, int64_t Cout,
                                  int64_t KH, int64_t KW, int64_t stride, int64_t pad, int64_t Kp,
                                  const void* bn_y, const void* bn_res, const float* bn_stats,
                                  int64_t bn_act, void* region, const float* bn_vres,
                                  const void* dy2, const void* wt2, int64_t cin2, int64_t kp2,
                                  hipStream_t st) {
  if (dy2 == nullptr || wt2 == nullptr || cin2 <= 0 || cin2 % BK || kp2 < cin2 || kp2 % BK)
    return MDA_NOT_SERVED;
  int64_t tile = 0, splits = 0;
  mda_conv_plan(N * H * W, Cin, Kp, &tile, &splits);
  if (splits != 1) return MDA_NOT_SERVED;
  return conv_dgrad_impl(dy, wt, dx, nullptr, nullptr, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride,
                         pad, Kp, tile, splits, bn_y, bn_res, bn_stats, bn_act, region, 1, bn_vres,
                         0, 0, dy2, wt2, cin2, kp2, st);
}

static int conv_dgrad_impl(const void* dy, const void* wt, void* dx, float* partial,
                           const void* res, int64_t N, int64_t H, int64_t W, int64_t Cin,
                           int64_t Ho, int64_t Wo, int64_t Cout, int64_t KH, int64_t KW,
                           int64_t stride, int64_t pad, int64_t Kp, int64_t tile, int64_t splits,
                           const void* bn_y, const void* bn_res, const float* bn_stats,
                           int64_t bn_act, void* region, int64_t groups, const float* bn_vres,
                           int64_t bn_mh, int64_t bn_rstride, const void* x2, const void* w2,
                           int64_t cin2, int64_t kp2, hipStream_t st) {
  if (Cout % 8 || groups < 1 || Cin % groups || Cout % groups) return (int)hipErrorInvalidValue;
  if (region != nullptr && (splits != 1 || Cin % 8 || Cin > SLOT_CMAX || bn_y == nullptr ||
                            bn_stats == nullptr))
    return (int)hipErrorInvalidValue;
  // two stacked sets: dx rows [mh, 2 mh) are set 1 (N holds both sets' images)
  if (bn_mh != 0 && (region == nullptr || bn_mh * 2 != N * H * W || bn_rstride <= 0))
    return (int)hipErrorInvalidValue;
  ConvParams p{};
  p.bnb_mh = (int)bn_mh;
  p.bnb_rstride = bn_rstride;
  p.bnb_y = (const bf16_t*)bn_y;
  p.bnb_res = (const bf16_t*)bn_res;
  p.bnb_stats = bn_stats;
  p.bnb_slot = (BnRegion*)region;
  p.bnb_act = (int)bn_act;
  p.bnb_vres = bn_res != nullptr ? bn_vres : nullptr;
  p.x2 = (const bf16_t*)x2;
  p.w2 = (const bf16_t*)w2;
  p.cin2 = (int)cin2;
  p.kp2 = (int)kp2;
  p.cls2 = -1;
  p.sh2 = 0;
  p.x = (const bf16_t*)dy; p.w = (const bf16_t*)wt; p.scale = nullptr; p.bias = nullptr;
  p.res = (const bf16_t*)res; p.y = (bf16_t*)dx; p.preact = nullptr; p.partial = partial;
  // GEMM view: rows = dx pixels, cols = Cin, k = (tap, co); "input" image = dy
  p.N = N; p.H = Ho; p.W = Wo; p.Cin = Cout / groups; p.Ho = H; p.Wo = W; p.Cout = Cin; p.KH = KH;
  p.KW = KW; p.stride = stride; p.pad = pad; p.K = KH * KW * p.Cin; p.Kp = Kp; p.M = N * H * W;
  p.act = 0;
  p.ldx = (int)Cout;
  p.cout_g = (int)(Cin / groups);
  int mode = (p.Cin % BK == 0) ? LOAD_DGRAD_FAST : LOAD_DGRAD_VEC8;
  p.par = 0;
  p.zsplits = 1;
  p.stats_part = nullptr;
  p.stats_slot = nullptr;
  p.stamps = g_stamps;
  // strided dgrad: one GEMM per output-parity class with only its taps
  if (stride > 1 && mode == LOAD_DGRAD_FAST && use_glds() && use_par_dgrad() && groups == 1)
    p.par = (int)stride;
  if (x2 != nullptr) {
    if (p.par <= 1 || groups != 1 || bn_mh != 0) return MDA_NOT_SERVED;
    // the 1 x 1 / stride-s / pad-0 conv samples dx pixels (s i, s j): parity
    // class (pad mod s, pad mod s), whose dy pixel minus pad / s is (i, j)
    const int ph = (int)(pad % stride);
    p.cls2 = ph * (int)stride + ph;
    p.sh2 = (int)(pad / stride);
    if (tile == 0 || splits == 0) mda_conv_plan(p.M, p.Cout, p.Kp, &tile, &splits);
    if (splits != 1) return MDA_NOT_SERVED;
  }
  if (groups > 1 && (p.Cin % 8 || p.cout_g % 8)) return (int)hipErrorInvalidValue;
  // stride-1 3x3 pad-1 dgrad is a "same" conv of dy with the mirrored taps
  return dispatch(p, mode, tile, splits, st, (groups == 1 && halo_eligible(p)) ? 2 : 0);
}

// Training conv + BN statistics, two launches: the conv writes the raw bf16
// output AND per-block channel partials of its rows from the epilogue (the
// output is never re-read for statistics), then the channel-parallel finalize
// (csrc/bn.hip) produces mean / rstd / scale / shift and the running-stat
// update.  Falls back to conv + mda_bn_stats2 when the conv is split over K
// (the partial sums are only final after the split-K combine).
// partial: >= max(nblk * 2 * Cout, 2 * 2048 * 512) floats (the BN workspace).
extern "C" int mda_bn_finalize(const float* partial, int64_t nblk, int64_t M, int64_t C,
                               const float* gamma, const float* beta, float* running_mean,
                               float* running_var, float* mean, float* rstd, float* scale,
                               float* shift, float momentum, float eps, int64_t* nbt,
                               hipStream_t st);
extern "C" int mda_bn_stats2(const void* y, int64_t M, int64_t C, float* partial,
                             const float* gamma, const float* beta, float* running_mean,
                             float* running_var, float* mean, float* rstd, float* scale,
                             float* shift, float momentum, float eps, int64_t* nbt,
                             hipStream_t st);

MDA_API int mda_conv_fwd_bnstats(const void* x, const void* w, void* y, float* partial,
                                 float* bn_partial, int64_t bn_partial_cap, int64_t N, int64_t H,
                                 int64_t W, int64_t Cin, int64_t Ho, int64_t Wo, int64_t Cout,
                                 int64_t KH, int64_t KW, int64_t stride, int64_t pad, int64_t Kp,
                                 int64_t tile, int64_t splits, const float* gamma,
                                 const float* beta, float* running_mean, float* running_var,
                                 float* mean, float* rstd, float* scale, float* shift,
                                 float momentum, float eps, int64_t* nbt, hipStream_t st) {
  ConvParams p{};
  p.x = (const bf16_t*)x; p.w = (const bf16_t*)w; p.scale = nullptr; p.bias = nullptr;
  p.res = nullptr; p.y = (bf16_t*)y; p.preact = nullptr; p.partial = partial;
  p.N = N; p.H = H; p.W = W; p.Cin = Cin; p.Ho = Ho; p.Wo = Wo; p.Cout = Cout; p.KH = KH;
  p.KW = KW; p.stride = stride; p.pad = pad; p.K = KH * KW * Cin; p.Kp = Kp; p.M = N * Ho * Wo;
  p.act = 0;
  p.par = 0;
  p.zsplits = 1;
  p.stats_part = nullptr;
  p.stats_slot = nullptr;
  p.stamps = g_stamps;
  if (Cout % 8 || Cout > 2048) return (int)hipErrorInvalidValue;
  int mode = (Cin % BK == 0) ? LOAD_FAST : (Cin % 8 == 0 ? LOAD_VEC8 : LOAD_SCALAR);
  if (tile == 0 || splits == 0) mda_conv_plan(p.M, p.Cout, p.Kp, &tile, &splits);
  const int halo = halo_eligible(p) ? 1 : 0;
  // M-blocks of the launch that will run (see dispatch)
  int64_t nblk;
  if (halo && !(!((Cin / BK) == 1 && splits == 1 && use_halo1()) &&
                     p.himgs * (p.hrows + 2) * (p.W + 2) > HALO_PROWS))
    nblk = (p.M + p.hpb - 1) / p.hpb;
  else
    nblk = (p.M + tile / 1000 - 1) / (tile / 1000);
  const bool fused = splits == 1 && nblk * 2 * Cout <= bn_partial_cap;
  if (fused) p.stats_part = bn_partial;
  int rc = dispatch(p, mode, tile, splits, st, halo);
  if (rc) return rc;
  if (fused)
    return mda_bn_finalize(bn_partial, nblk, p.M, Cout, gamma, beta, running_mean, running_var,
                           mean, rstd, scale, shift, momentum, eps, nbt, st);
  return mda_bn_stats2(y, p.M, Cout, bn_partial, gamma, beta, running_mean, running_var, mean,
                       rstd, scale, shift, momentum, eps, nbt, st);
}

// Training conv whose epilogue adds the BN statistics of its raw bf16 output
// into a BnRegion (csrc/bnslot.h); the caller follows with mda_bn_apply_fin,
// whose prologue finalizes them (2 launches per conv + BN instead of 3).
// Split-K convs (sums only final after the combine) run the conv, then the
// standalone statistics pass into the same slot.
extern "C" int mda_bn_stats_acc(const void* y, int64_t M, int64_t C, void* region, hipStream_t st);

MDA_API int mda_conv_fwd_bnacc_g(const void* x, const void* w, void* y, float* partial,
                                 void* region, int64_t N, int64_t H, int64_t W, int64_t Cin,
                                 int64_t Ho, int64_t Wo, int64_t Cout, int64_t KH, int64_t KW,
                                 int64_t stride, int64_t pad, int64_t Kp, int64_t tile,
                                 int64_t splits, int64_t groups, hipStream_t st);

MDA_API int mda_conv_fwd_bnacc(const void* x, const void* w, void* y, float* partial, void* region,
                               int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Ho,
                               int64_t Wo, int64_t Cout, int64_t KH, int64_t KW, int64_t stride,
                               int64_t pad, int64_t Kp, int64_t tile, int64_t splits,
                               hipStream_t st) {
  return mda_conv_fwd_bnacc_g(x, w, y, partial, region, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride,
                              pad, Kp, tile, splits, 1, st);
}

// Grouped (groups > 1, Cin/G and Cout/G multiples of 8): w packed [Cout][Kp]
// over the Cin/G channels of each output channel's group (the OIHW weight of
// a grouped conv packed as if dense, mda_pack_conv_weights with Cin/G).
MDA_API int mda_conv_fwd_bnacc_g(const void* x, const void* w, void* y, float* partial,
                                 void* region, int64_t N, int64_t H, int64_t W, int64_t Cin,
                                 int64_t Ho, int64_t Wo, int64_t Cout, int64_t KH, int64_t KW,
                                 int64_t stride, int64_t pad, int64_t Kp, int64_t tile,
                                 int64_t splits, int64_t groups, hipStream_t st) {
  if (groups < 1 || Cin % groups || Cout % groups) return (int)hipErrorInvalidValue;
  ConvParams p{};
  p.ldx = (int)Cin;
  p.cout_g = (int)(Cout / groups);
  Cin /= groups;
  p.x = (const bf16_t*)x; p.w = (const bf16_t*)w; p.scale = nullptr; p.bias = nullptr;
  p.res = nullptr; p.y = (bf16_t*)y; p.preact = nullptr; p.partial = partial;
  p.N = N; p.H = H; p.W = W; p.Cin = Cin; p.Ho = Ho; p.Wo = Wo; p.Cout = Cout; p.KH = KH;
  p.KW = KW; p.stride = stride; p.pad = pad; p.K = KH * KW * Cin; p.Kp = Kp; p.M = N * Ho * Wo;
  p.act = 0;
  p.par = 0;
  p.zsplits = 1;
  p.stats_part = nullptr;
  p.stats_slot = nullptr;
  p.stamps = g_stamps;
  if (Cout % 8 || Cout > SLOT_CMAX) return (int)hipErrorInvalidValue;
  int mode = (Cin % BK == 0) ? LOAD_FAST : (Cin % 8 == 0 ? LOAD_VEC8 : LOAD_SCALAR);
  if (groups > 1 && mode == LOAD_SCALAR) return (int)hipErrorInvalidValue;
  if (tile == 0 || splits == 0) mda_conv_plan(p.M, p.Cout, p.Kp, &tile, &splits);
  const int halo = (groups == 1 && halo_eligible(p)) ? 1 : 0;
  if (splits == 1) p.stats_slot = (BnRegion*)region;
  int rc = dispatch(p, mode, tile, splits, st, halo);
  if (rc || splits == 1) return rc;
  return mda_bn_stats_acc(y, p.M, Cout, region, st);
}


