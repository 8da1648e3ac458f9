// Training-BN streaming passes shared by csrc/bn.hip (the BN kernels) and the
// fused launches that run them beside another kernel's blocks:
// csrc/conv_wgrad.hip (a weight-gradient GEMM and the NEXT layer's BN
// backward apply, mda_conv_wgrad_nored_bn) and csrc/conv1x1.hip (a residual
// block's projection-shortcut conv and conv1's BN forward apply,
// mda_conv1x1_bnacc_apply).
//
// bn_bwd_apply_body is the streaming pass of a BN backward whose channel sums
// a producer already added into the region (the consuming conv's dgrad
// epilogue): dz = dout * act'(z) (+ dpre), dy = scale*(dz - (sum dz +
// xhat*sum dz*xhat)/M), dres = dz; block 0 accumulates dgamma / dbeta.  It
// takes its block index and block count as arguments and works for any block
// size that is a multiple of 256, so a fused launch can run it on the blocks
// past the GEMM's.
#pragma once
#include "common.h"
#include "bnslot.h"

namespace {

__device__ __forceinline__ float bw_act_grad(float z, int act) {
  if (act == 1) return z > 0.f ? 1.f : 0.f;                 // relu
  if (act == 2) return (z > 0.f && z < 6.f) ? 1.f : 0.f;    // relu6
  return 1.f;
}

struct BwdArgs {
  const bf16_t* dout; const bf16_t* dout2; const bf16_t* dpre;
  const bf16_t* y; const bf16_t* res;
  const float* stats;    // [4][C] mean, rstd, scale, shift
  bf16_t* dy; bf16_t* dres;
  float* dgamma; float* dbeta; float* sums;   // accumulated / written by block 0 (each may be null)
  BnRegion* reg;
  unsigned* err;
  int M, C, act;
  // optional: the residual came from another training BN with no activation
  // (a projection shortcut): its dout IS dres, so this pass also adds that
  // layer's sum dres and sum dres*xhat_r (ry = its BN input, rstats = its
  // [4][C] stats) into rreg -- its backward is then one streaming pass too
  const bf16_t* ry; const float* rstats; BnRegion* rreg;
  // optional: `res` is the RAW input of another training BN (a projection
  // shortcut whose apply was folded into this layer's, mda_bn_apply_fin_vr):
  // the residual value is res * vres[2C + c] + vres[3C + c] (vres = that
  // layer's [4][C] stats)
  const float* vres;
  // DOT single-pass backward (two stacked cotangents): gridDim.y = 2 sets;
  // set 1's dout / dout2 / dpre / dy / dres start dd elements later, its
  // dgamma / dbeta / sums dg floats later (the other gradient set of the flat
  // buffer, may be negative) and its reg / rreg dr bytes later.  y, res, ry
  // and every stats operand are the forward's, shared by both sets.
  int64_t dd, dg, dr;
};

__device__ __forceinline__ void dual_shift(BwdArgs& a, unsigned set) {
  if (set == 0) return;
  if (a.dout) a.dout += a.dd;
  if (a.dout2) a.dout2 += a.dd;
  if (a.dpre) a.dpre += a.dd;
  if (a.dy) a.dy += a.dd;
  if (a.dres) a.dres += a.dd;
  if (a.dgamma) a.dgamma += a.dg;
  if (a.dbeta) a.dbeta += a.dg;
  if (a.sums) a.sums += a.dg;
  if (a.reg) a.reg = (BnRegion*)((char*)a.reg + a.dr);
  if (a.rreg) a.rreg = (BnRegion*)((char*)a.rreg + a.dr);
}

// res-producer sums of one 8-channel vector (dz = the stored dres values)
__device__ __forceinline__ void rsum_add8(const BwdArgs& a, int64_t o, int c0, const uint32_t (&ro)[4],
                                          float (&r1)[8], float (&r2)[8]) {
  const uint4 yv = *(const uint4*)(a.ry + o);
  const uint32_t yw[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int w = e >> 1;
    const float d = (e & 1) ? __uint_as_float(ro[w] & 0xffff0000u) : __uint_as_float(ro[w] << 16);
    const float yf = (e & 1) ? __uint_as_float(yw[w] & 0xffff0000u) : __uint_as_float(yw[w] << 16);
    r1[e] += d;
    r2[e] += d * ((yf - a.rstats[c0 + e]) * a.rstats[a.C + c0 + e]);
  }
}

struct Raw8 { uint4 y, d, d2, p, r; };

__device__ __forceinline__ void bwd_load8(const BwdArgs& a, int64_t o, Raw8& v) {
  v.y = *(const uint4*)(a.y + o);
  v.d = a.dout ? *(const uint4*)(a.dout + o) : make_uint4(0, 0, 0, 0);
  v.d2 = a.dout2 ? *(const uint4*)(a.dout2 + o) : make_uint4(0, 0, 0, 0);
  v.p = a.dpre ? *(const uint4*)(a.dpre + o) : make_uint4(0, 0, 0, 0);
  v.r = (a.res && a.act != 0) ? *(const uint4*)(a.res + o) : make_uint4(0, 0, 0, 0);
}

// dz of 8 channels (z recomputed from y: no stored mask)
__device__ __forceinline__ void bwd_dz8(const BwdArgs& a, const Raw8& v, const float* sc,
                                        const float* sh, float (&dz)[8], const float* vsc,
                                        const float* vsh) {
  const uint32_t yw[4] = {v.y.x, v.y.y, v.y.z, v.y.w}, dw[4] = {v.d.x, v.d.y, v.d.z, v.d.w};
  const uint32_t d2w[4] = {v.d2.x, v.d2.y, v.d2.z, v.d2.w}, pw[4] = {v.p.x, v.p.y, v.p.z, v.p.w};
  const uint32_t rw[4] = {v.r.x, v.r.y, v.r.z, v.r.w};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int w = k >> 1;
    const bool hi = k & 1;
    auto f = [&](uint32_t u) { return hi ? __uint_as_float(u & 0xffff0000u) : __uint_as_float(u << 16); };
    float d = f(dw[w]);
    if (a.dout2) d += f(d2w[w]);
    if (a.act != 0) {
      float z = f(yw[w]) * sc[k] + sh[k];
      if (a.res) z += a.vres ? f(rw[w]) * vsc[k] + vsh[k] : f(rw[w]);
      d *= bw_act_grad(z, a.act);
    }
    if (a.dpre) d += f(pw[w]);
    dz[k] = d;
  }
}

// Block sums a[8], b[8] of the thread's channel group (tid % (C/8)) -> shard
// `key` % SH of region r, through the caller's LDS scratch sm
// (2 * blockDim.x * 8 floats).
__device__ __forceinline__ void region_block_add_s(BnRegion* r, const float (&a)[8], const float (&b)[8],
                                                   int C, float* sm, int key) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const int C8 = C / 8;
  const int rpi = nt / C8;
  const int cg = tid % C8, r0 = tid / C8;
  float* const s0 = sm;
  float* const s1 = sm + nt * 8;
  if (r0 < rpi) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s0[r0 * C + cg * 8 + k] = a[k];
      s1[r0 * C + cg * 8 + k] = b[k];
    }
  }
  __syncthreads();
  const int shard = key % slot_shards(C);
  for (int t = tid; t < 2 * C; t += nt) {
    const int q = t / C, c = t - q * C;
    const float* sq = q ? s1 : s0;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int rr = 0;
    for (; rr + 4 <= rpi; rr += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += sq[(rr + u) * C + c];
    }
    for (; rr < rpi; ++rr) acc[0] += sq[rr * C + c];
    acc_add(region_acc(r, C, shard, q) + c, (double)((acc[0] + acc[1]) + (acc[2] + acc[3])));
  }
}

// LDS bytes bn_bwd_apply_body needs for C channels and nt threads per block.
__host__ __device__ __forceinline__ int64_t bn_apply_lds_bytes(int C, int nt, bool rreg) {
  const int64_t ops = (int64_t)8 * C * 4;
  const int64_t red = rreg ? (int64_t)2 * nt * 8 * 4 : 0;
  return ops > red ? ops : red;  // the reduction reuses the operand space after the pass
}

// The streaming BN-backward apply as block `bid` of `nblk`: V 16-byte
// vectors per thread loaded before the prologue reads the region, so both
// latencies overlap.  s_dyn: bn_apply_lds_bytes of LDS.
template <int V>
__device__ __forceinline__ void bn_bwd_apply_body(const BwdArgs& a, float* s_dyn, int bid, int nblk) {
  const int C = a.C;
  float* const s_m0 = s_dyn;
  float* const s_m1 = s_dyn + C;
  float* const s_st0 = s_dyn + 2 * C;  // [4][C] mean, rstd, scale, shift
  float* const s_vr0 = s_dyn + 6 * C;  // [2][C] virtual-residual scale, shift
  const int c8 = C / 8;
  const int64_t total = (int64_t)a.M * c8;
  const int64_t i0 = bid * (int64_t)blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)nblk * blockDim.x;
  Raw8 raw[V];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t i = i0 + k * stride;
    bwd_load8(a, (i < total ? i : 0) * 8, raw[k]);
  }
  {
    const float invM = 1.f / (float)a.M;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      double d0, d1;
      region_channel<false>(a.reg, C, c, d0, d1);
      const float t0 = (float)d0, t1 = (float)d1;
      s_m0[c] = t0 * invM;
      s_m1[c] = t1 * invM;
#pragma unroll
      for (int q = 0; q < 4; ++q) s_st0[q * C + c] = a.stats[q * C + c];
      s_vr0[c] = a.vres ? a.vres[2 * C + c] : 1.f;
      s_vr0[C + c] = a.vres ? a.vres[3 * C + c] : 0.f;
      if (bid == 0) {
        if (a.sums) { a.sums[c] = t0; a.sums[C + c] = t1; }
        if (a.dbeta) a.dbeta[c] += t0;
        if (a.dgamma) a.dgamma[c] += t1;
      }
    }
  }
  __syncthreads();
  float r1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, r2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto emit = [&](int64_t i, const Raw8& v) {
    const int c0 = (int)(i % c8) * 8;
    float sc[8], sh[8], mu[8], rs[8], dz[8], vsc[8], vsh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      mu[e] = s_st0[c0 + e]; rs[e] = s_st0[C + c0 + e];
      sc[e] = s_st0[2 * C + c0 + e]; sh[e] = s_st0[3 * C + c0 + e];
      vsc[e] = s_vr0[c0 + e]; vsh[e] = s_vr0[C + c0 + e];
    }
    bwd_dz8(a, v, sc, sh, dz, vsc, vsh);
    const uint32_t yw[4] = {v.y.x, v.y.y, v.y.z, v.y.w};
    uint32_t go[4], ro[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      float g[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = 2 * w + h;
        const float yf = h ? __uint_as_float(yw[w] & 0xffff0000u) : __uint_as_float(yw[w] << 16);
        const float xhat = (yf - mu[e]) * rs[e];
        g[h] = sc[e] * (dz[e] - (s_m0[c0 + e] + xhat * s_m1[c0 + e]));
      }
      go[w] = pack_bf16x2(g[0], g[1]);
      ro[w] = pack_bf16x2(dz[2 * w], dz[2 * w + 1]);
    }
    *(uint4*)(a.dy + i * 8) = make_uint4(go[0], go[1], go[2], go[3]);
    if (a.dres) *(uint4*)(a.dres + i * 8) = make_uint4(ro[0], ro[1], ro[2], ro[3]);
    if (a.rreg) rsum_add8(a, i * 8, c0, ro, r1, r2);  // (the host checks: fixed channel group)
  };
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t i = i0 + k * stride;
    if (i < total) emit(i, raw[k]);
  }
  for (int64_t i = i0 + V * stride; i < total; i += stride) {
    Raw8 v;
    bwd_load8(a, i * 8, v);
    emit(i, v);
  }
  if (a.rreg) {
    __syncthreads();  // every read of the operand LDS is done: it becomes the reduction scratch
    region_block_add_s(a.rreg, r1, r2, C, s_dyn, bid);
  }
}

// power-of-two block count for the streaming apply kernels
inline int apply_blocks(int64_t n8, int vpt) {
  const int64_t want = (n8 + 256 * (int64_t)vpt - 1) / (256 * (int64_t)vpt);
  int64_t b = 1;
  while (b < want && b < 1024) b <<= 1;
  return (int)b;
}

// ---------------------------------------------------------------------------
// Forward apply: z = y*scale + shift (+ res); out = act(z); preact = z, with
// the finalize of the region's sums in the prologue (every block finalizes
// the channels; block 0 also writes the [4][C] stats and the running
// statistics).  rreg != null: `res` is the RAW output of another training
// conv whose BN (no activation: a projection shortcut) is applied here too
// (VirtualBN).  V vectors per thread loaded BEFORE the prologue.
struct FwdApply {
  const bf16_t* y; BnRegion* reg; int64_t M; int C; FinArgs f;
  const bf16_t* res; bf16_t* out; bf16_t* preact; int act;
  BnRegion* rreg; FinArgs rf;
};

__device__ __forceinline__ float bw_act_f(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) return fminf(fmaxf(v, 0.f), 6.f);
  return v;
}

__device__ __forceinline__ void apply8(const uint4& yv, const uint4& rv, bool has_res, const float* sc,
                                       const float* sh, int act, uint4& out, uint4& z,
                                       const float* rsc = nullptr, const float* rsh = nullptr) {
  const uint32_t yw[4] = {yv.x, yv.y, yv.z, yv.w};
  const uint32_t rw[4] = {rv.x, rv.y, rv.z, rv.w};
  uint32_t zo[4], oo[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float v0 = __uint_as_float(yw[k] << 16) * sc[2 * k] + sh[2 * k];
    float v1 = __uint_as_float(yw[k] & 0xffff0000u) * sc[2 * k + 1] + sh[2 * k + 1];
    if (has_res) {
      const float r0 = __uint_as_float(rw[k] << 16), r1 = __uint_as_float(rw[k] & 0xffff0000u);
      if (rsc) {  // virtual residual: the raw input of another BN, applied here
        v0 += r0 * rsc[2 * k] + rsh[2 * k];
        v1 += r1 * rsc[2 * k + 1] + rsh[2 * k + 1];
      } else {
        v0 += r0;
        v1 += r1;
      }
    }
    zo[k] = pack_bf16x2(v0, v1);
    oo[k] = pack_bf16x2(bw_act_f(v0, act), bw_act_f(v1, act));
  }
  out = make_uint4(oo[0], oo[1], oo[2], oo[3]);
  z = make_uint4(zo[0], zo[1], zo[2], zo[3]);
}

// LDS floats bn_apply_fin_body needs for C channels
__host__ __device__ __forceinline__ int64_t bn_fin_lds_bytes(int C, bool rreg) {
  return (int64_t)(rreg ? 4 : 2) * C * 4;
}

template <int V>
__device__ __forceinline__ void bn_apply_fin_body(const FwdApply& a, float* s_dyn, int bid, int nblk) {
  const int C = a.C;
  float* const s_scale = s_dyn;
  float* const s_shift = s_dyn + C;
  float* const s_rscale = s_dyn + 2 * C;  // (rreg only)
  float* const s_rshift = s_dyn + 3 * C;
  const int64_t total = a.M * C / 8;
  const int c8 = C / 8;
  const int64_t i0 = bid * (int64_t)blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)nblk * blockDim.x;
  uint4 yv[V], rv[V];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t i = i0 + k * stride;
    const int64_t ii = i < total ? i : 0;
    yv[k] = ((const uint4*)a.y)[ii];
    rv[k] = a.res ? ((const uint4*)a.res)[ii] : make_uint4(0, 0, 0, 0);
  }
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    fin_channel_w<false>(a.reg, a.M, C, c, a.f, s_scale[c], s_shift[c], bid == 0);
    if (a.rreg) fin_channel_w<false>(a.rreg, a.M, C, c, a.rf, s_rscale[c], s_rshift[c], bid == 0);
  }
  if (bid == 0 && threadIdx.x == 0) {
    if (a.f.nbt) a.f.nbt[0] += 1;
    if (a.rreg && a.rf.nbt) a.rf.nbt[0] += 1;
  }
  __syncthreads();
  float sc[8], sh[8], rsc[8], rsh[8];
  const bool vr = a.rreg != nullptr;
  auto emit = [&](int64_t i, const uint4& y1, const uint4& r1) {
    const int cc = (int)(i % c8) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sc[e] = s_scale[cc + e]; sh[e] = s_shift[cc + e];
      rsc[e] = vr ? s_rscale[cc + e] : 1.f; rsh[e] = vr ? s_rshift[cc + e] : 0.f;
    }
    uint4 o, z;
    apply8(y1, r1, a.res != nullptr, sc, sh, a.act, o, z, vr ? rsc : nullptr, vr ? rsh : nullptr);
    ((uint4*)a.out)[i] = o;
    if (a.preact) ((uint4*)a.preact)[i] = z;
  };
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t i = i0 + k * stride;
    if (i < total) emit(i, yv[k], rv[k]);
  }
  for (int64_t i = i0 + V * stride; i < total; i += stride) {
    const uint4 y1 = ((const uint4*)a.y)[i];
    const uint4 r1 = a.res ? ((const uint4*)a.res)[i] : make_uint4(0, 0, 0, 0);
    emit(i, y1, r1);
  }
}

}  // namespace
