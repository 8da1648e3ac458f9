// Fused multi-head attention (FlashAttention-2 style) for the ViT students
// (reference mdistiller/models/imagenet/vit.py:99-133 -> timm Attention):
// head_dim 64, any sequence length (197 tokens at patch16 / 224^2), bf16 I/O,
// fp32 accumulation, no N x N matrix in memory.
//
// Forward, one 256-thread block per (64-query tile, batch*head), a wave per 16
// queries.  The scores are computed TRANSPOSED, S^T = K Q^T, with the queries
// on the MFMA N axis: in the 16x16x32 accumulator layout a lane then holds
// 16 keys of ONE query (lane & 15), so the online-softmax row statistics need
// only two cross-lane shuffles, and the probabilities feed O^T += V^T P^T as
// the MFMA B operand straight from the accumulators: the contraction order
// over keys is permuted to the accumulator's (keys 4g..4g+3, 16+4g..+3 of
// each 32), and the V^T operand is gathered in that order by
// ds_read_b64_tr_b16 with per-lane row addresses.  No register shuffles, no
// P round trip through LDS.  LSE (base 2) is kept for the backward.
//
// Backward: D = rowsum(dO o O) (one pass), then two kernels that recompute P
// from LSE: dK / dV per 64-key tile (a wave per 16 keys, looping over query
// tiles: S = Q K^T, dV^T += dO^T P, dP = dO V^T, dS = P (dP - D),
// dK^T += Q^T dS), and dQ per 64-query tile (S^T, dP^T = V dO^T,
// dQ^T += K^T dS^T).  Each gradient is written once (no atomics,
// deterministic).  q / k / v / dq / dk / dv are strided views of the fused
// [B, N, 3, H, 64] qkv projection, so the gradient lands in place for the
// qkv Linear's backward.
//
// LDS tiles are [64 rows][64 bf16] with 128-B rows; the 16-B chunk c of row r
// is stored at slot c ^ fa_swz(r).  fa_swz takes 8 distinct values on the 8
// same-parity rows of 16 consecutive rows (row-fragment ds_read_b128) and, for
// the rows a transposing read's 32-lane group touches ({4g + q}), distinct
// 32-B pair indices (ds_read_b64_tr_b16 reads 8 B inside one chunk, the pair
// {2i, 2i+1} is kept as a set).
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int FD = 64;                       // head dim
constexpr float LOG2E = 1.4426950408889634f;

struct FaParams {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  int64_t sb, sn, sh;                        // q/k/v element (b, n, h, d) at b*sb + n*sn + h*sh + d
  bf16_t* o;
  const bf16_t* dout;
  int64_t ob, on, oh;                        // o / dout strides
  float* lse;                                // [B*H][N], base 2
  float* dsum;                               // [B*H][N], rowsum(dO o O)
  bf16_t* dq;
  bf16_t* dk;
  bf16_t* dv;                                // gradient strides = q's
  int B, H, N;
  float scale;
};

__device__ __forceinline__ int fa_swz(int r) { return (((r >> 1) & 3) << 1) | ((r >> 3) & 1); }

// [64 rows][64 d] tile of rows r0.. of one (b, h) slice -> LDS (swizzled); rows >= N zero
__device__ __forceinline__ void fa_load_tile(char* lds, const bf16_t* base, int64_t sn, int r0, int N) {
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int row = i >> 3, c = i & 7;
    uint4 val = make_uint4(0u, 0u, 0u, 0u);
    if (r0 + row < N) val = *(const uint4*)(base + (int64_t)(r0 + row) * sn + c * 8);
    *(uint4*)(lds + row * 128 + ((c ^ fa_swz(row)) << 4)) = val;
  }
}

// A-operand fragment of 16 tile rows (rbase + lane&15) x 32 d (half kk)
__device__ __forceinline__ bf16x8 fa_row_frag(const char* lds, int rbase, int kk, int lane) {
  const int row = rbase + (lane & 15);
  const int c = 4 * kk + (lane >> 4);
  return *(const bf16x8*)(lds + row * 128 + ((c ^ fa_swz(row)) << 4));
}

// A-operand fragment of the TRANSPOSED tile: 16 columns (16*ct + lane&15) x 32
// contraction rows in the accumulator order of half s: rows 32s + 4g + {0..3}
// then 32s + 16 + 4g + {0..3}
__device__ __forceinline__ bf16x8 fa_tr_frag(const char* lds, int s, int ct, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int c = 2 * ct + (p >> 1);
  const int within = (p & 1) * 8;
  const int r0 = 32 * s + 4 * g + q, r1 = r0 + 16;
  const char* a0 = lds + r0 * 128 + ((c ^ fa_swz(r0)) << 4) + within;
  const char* a1 = lds + r1 * 128 + ((c ^ fa_swz(r1)) << 4) + within;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  bf16x8 out;
  short* o = (short*)&out;
  o[0] = lo[0]; o[1] = lo[1]; o[2] = lo[2]; o[3] = lo[3];
  o[4] = hi[0]; o[5] = hi[1]; o[6] = hi[2]; o[7] = hi[3];
  return out;
}

// B-operand fragment from two accumulator tiles (2s, 2s+1) of values owned by
// this lane's column: slots 0..3 = tile 2s rows 4g + r, 4..7 = tile 2s+1
__device__ __forceinline__ bf16x8 fa_acc_frag(const f32x4& t0, const f32x4& t1) {
  bf16x8 out;
  out[0] = (__bf16)t0[0]; out[1] = (__bf16)t0[1]; out[2] = (__bf16)t0[2]; out[3] = (__bf16)t0[3];
  out[4] = (__bf16)t1[0]; out[5] = (__bf16)t1[1]; out[6] = (__bf16)t1[2]; out[7] = (__bf16)t1[3];
  return out;
}

// 16 B of global row `row` (d chunk 4kk + lane>>4) as a B-operand fragment (column = lane & 15)
__device__ __forceinline__ bf16x8 fa_glob_frag(const bf16_t* base, int64_t sn, int row, int N, int kk, int lane) {
  bf16x8 f;
  if (row < N) {
    f = *(const bf16x8*)(base + (int64_t)row * sn + 32 * kk + 8 * (lane >> 4));
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = (__bf16)0.f;
  }
  return f;
}

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// A wave's transposed accumulator tile acc[4] = X^T[64 d][16 cols] (d = 16t + 4g + r,
// col = lane & 15) -> rows [16][64 d] of global memory at dst + col*sn (col < nvalid),
// through this wave's 2 KB LDS slice.
__device__ __forceinline__ void fa_store_T(char* wlds, const f32x4 (&acc)[4], float mul_per_lane,
                                           bf16_t* dst, int64_t sn, int nvalid, int lane) {
  const int col = lane & 15, g = lane >> 4;
  bf16_t* t = (bf16_t*)wlds;  // [16][64]
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) t[col * 64 + 16 * dt + 4 * g + r] = f2bf(acc[dt][r] * mul_per_lane);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = lane + 64 * i;  // 128 chunks: 16 rows x 8
    const int row = idx >> 3, c = idx & 7;
    if (row < nvalid) *(uint4*)(dst + (int64_t)row * sn + c * 8) = *(const uint4*)(t + row * 64 + c * 8);
  }
}

__global__ void __launch_bounds__(256) fa_fwd_kernel(const FaParams p) {
  __shared__ __attribute__((aligned(16))) char Ks[64 * 128];
  __shared__ __attribute__((aligned(16))) char Vs[64 * 128];
  __shared__ __attribute__((aligned(16))) char Ot[4][16 * 128];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int bh = blockIdx.y, b = bh / p.H, h = bh - b * p.H;
  const int64_t base = (int64_t)b * p.sb + (int64_t)h * p.sh;
  const int q0 = blockIdx.x * 64 + 16 * w;
  const int qi = q0 + (lane & 15);                 // this lane's query
  const float c2 = p.scale * LOG2E;
  bf16x8 qf[2];
  qf[0] = fa_glob_frag(p.q + base, p.sn, qi, p.N, 0, lane);
  qf[1] = fa_glob_frag(p.q + base, p.sn, qi, p.N, 1, lane);
  f32x4 acc_o[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc_o[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  const int g = lane >> 4;
  for (int kt = 0; kt < p.N; kt += 64) {
    __syncthreads();  // previous tile's reads done
    fa_load_tile(Ks, p.k + base, p.sn, kt, p.N);
    fa_load_tile(Vs, p.v + base, p.sn, kt, p.N);
    __syncthreads();
    f32x4 s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) s[t] = mfma(fa_row_frag(Ks, 16 * t, kk, lane), qf[kk], s[t]);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kt + 16 * t + 4 * g + r;
        const float v = key < p.N ? s[t][r] * c2 : -INFINITY;
        s[t][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    const float alpha = exp2f(m - mn);
    float rs = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = exp2f(s[t][r] - mn);
        s[t][r] = e;
        rs += e;
      }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    m = mn;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc_o[dt] *= alpha;
#pragma unroll
    for (int sh = 0; sh < 2; ++sh) {
      const bf16x8 pf = fa_acc_frag(s[2 * sh], s[2 * sh + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) acc_o[dt] = mfma(fa_tr_frag(Vs, sh, dt, lane), pf, acc_o[dt]);
    }
  }
  const float inv = 1.f / l;
  const int nvalid = min(16, p.N - q0);
  if (nvalid > 0)
    fa_store_T(Ot[w], acc_o, inv, p.o + (int64_t)b * p.ob + (int64_t)h * p.oh + (int64_t)q0 * p.on, p.on,
               nvalid, lane);
  if (g == 0 && qi < p.N) p.lse[(int64_t)bh * p.N + qi] = m + log2f(l);
}

// D[bh][n] = sum_d dO * O (fp32), one thread per (bh, n)
__global__ void __launch_bounds__(256) fa_dsum_kernel(const FaParams p) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)p.B * p.H * p.N;
  if (i >= total) return;
  const int bh = (int)(i / p.N), n = (int)(i - (int64_t)bh * p.N);
  const int b = bh / p.H, h = bh - b * p.H;
  const int64_t off = (int64_t)b * p.ob + (int64_t)n * p.on + (int64_t)h * p.oh;
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const uint4 x = *(const uint4*)(p.dout + off + 8 * c);
    const uint4 y = *(const uint4*)(p.o + off + 8 * c);
    const uint32_t xa[4] = {x.x, x.y, x.z, x.w}, ya[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc += __uint_as_float(xa[e] << 16) * __uint_as_float(ya[e] << 16);
      acc += __uint_as_float(xa[e] & 0xffff0000u) * __uint_as_float(ya[e] & 0xffff0000u);
    }
  }
  p.dsum[i] = acc;
}

// dK, dV of one 64-key tile; wave w owns keys kt + 16w .. +15
__global__ void __launch_bounds__(256) fa_bwd_dkv_kernel(const FaParams p) {
  __shared__ __attribute__((aligned(16))) char Qs[64 * 128];
  __shared__ __attribute__((aligned(16))) char Ds[64 * 128];  // dO tile
  __shared__ float Ls[64], Dd[64];
  __shared__ __attribute__((aligned(16))) char Ot[4][16 * 128];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int bh = blockIdx.y, b = bh / p.H, h = bh - b * p.H;
  const int64_t base = (int64_t)b * p.sb + (int64_t)h * p.sh;
  const int64_t obase = (int64_t)b * p.ob + (int64_t)h * p.oh;
  const int k0 = blockIdx.x * 64 + 16 * w;
  const int ki = k0 + (lane & 15);
  const int g = lane >> 4;
  const float c2 = p.scale * LOG2E;
  bf16x8 kf[2], vf[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    kf[kk] = fa_glob_frag(p.k + base, p.sn, ki, p.N, kk, lane);
    vf[kk] = fa_glob_frag(p.v + base, p.sn, ki, p.N, kk, lane);
  }
  f32x4 dk[4], dv[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) dk[t] = dv[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int qt = 0; qt < p.N; qt += 64) {
    __syncthreads();
    fa_load_tile(Qs, p.q + base, p.sn, qt, p.N);
    fa_load_tile(Ds, p.dout + obase, p.on, qt, p.N);
    if (threadIdx.x < 64) {
      const int qq = qt + threadIdx.x;
      Ls[threadIdx.x] = qq < p.N ? p.lse[(int64_t)bh * p.N + qq] : 0.f;
      Dd[threadIdx.x] = qq < p.N ? p.dsum[(int64_t)bh * p.N + qq] : 0.f;
    }
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = dp[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        s[t] = mfma(fa_row_frag(Qs, 16 * t, kk, lane), kf[kk], s[t]);   // S[q][key]
        dp[t] = mfma(fa_row_frag(Ds, 16 * t, kk, lane), vf[kk], dp[t]);  // dP[q][key]
      }
    }
    // P and dS in place (rows q = 16t + 4g + r, column = this lane's key)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = 16 * t + 4 * g + r;
        const bool ok = qt + ql < p.N && ki < p.N;
        const float pv = ok ? exp2f(s[t][r] * c2 - Ls[ql]) : 0.f;
        s[t][r] = pv;
        dp[t][r] = pv * (dp[t][r] - Dd[ql]);
      }
#pragma unroll
    for (int sh = 0; sh < 2; ++sh) {
      const bf16x8 pf = fa_acc_frag(s[2 * sh], s[2 * sh + 1]);
      const bf16x8 df = fa_acc_frag(dp[2 * sh], dp[2 * sh + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dv[dt] = mfma(fa_tr_frag(Ds, sh, dt, lane), pf, dv[dt]);  // dV^T[d][key] += dO^T P
        dk[dt] = mfma(fa_tr_frag(Qs, sh, dt, lane), df, dk[dt]);  // dK^T[d][key] += Q^T dS
      }
    }
  }
  const int nvalid = min(16, p.N - k0);
  if (nvalid > 0) {
    fa_store_T(Ot[w], dv, 1.f, p.dv + base + (int64_t)k0 * p.sn, p.sn, nvalid, lane);
    __builtin_amdgcn_wave_barrier();
    fa_store_T(Ot[w], dk, p.scale, p.dk + base + (int64_t)k0 * p.sn, p.sn, nvalid, lane);
  }
}

// dQ of one 64-query tile; wave w owns queries qt + 16w .. +15
__global__ void __launch_bounds__(256) fa_bwd_dq_kernel(const FaParams p) {
  __shared__ __attribute__((aligned(16))) char Ks[64 * 128];
  __shared__ __attribute__((aligned(16))) char Vs[64 * 128];
  __shared__ __attribute__((aligned(16))) char Ot[4][16 * 128];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int bh = blockIdx.y, b = bh / p.H, h = bh - b * p.H;
  const int64_t base = (int64_t)b * p.sb + (int64_t)h * p.sh;
  const int64_t obase = (int64_t)b * p.ob + (int64_t)h * p.oh;
  const int q0 = blockIdx.x * 64 + 16 * w;
  const int qi = q0 + (lane & 15);
  const int g = lane >> 4;
  const float c2 = p.scale * LOG2E;
  bf16x8 qf[2], of[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    qf[kk] = fa_glob_frag(p.q + base, p.sn, qi, p.N, kk, lane);
    of[kk] = fa_glob_frag(p.dout + obase, p.on, qi, p.N, kk, lane);
  }
  const float lse = qi < p.N ? p.lse[(int64_t)bh * p.N + qi] : 0.f;
  const float dsum = qi < p.N ? p.dsum[(int64_t)bh * p.N + qi] : 0.f;
  f32x4 dq[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) dq[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int kt = 0; kt < p.N; kt += 64) {
    __syncthreads();
    fa_load_tile(Ks, p.k + base, p.sn, kt, p.N);
    fa_load_tile(Vs, p.v + base, p.sn, kt, p.N);
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = dp[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        s[t] = mfma(fa_row_frag(Ks, 16 * t, kk, lane), qf[kk], s[t]);   // S^T[key][q]
        dp[t] = mfma(fa_row_frag(Vs, 16 * t, kk, lane), of[kk], dp[t]);  // dP^T[key][q]
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kt + 16 * t + 4 * g + r;
        const bool ok = key < p.N && qi < p.N;
        const float pv = ok ? exp2f(s[t][r] * c2 - lse) : 0.f;
        dp[t][r] = pv * (dp[t][r] - dsum);
      }
#pragma unroll
    for (int sh = 0; sh < 2; ++sh) {
      const bf16x8 df = fa_acc_frag(dp[2 * sh], dp[2 * sh + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dq[dt] = mfma(fa_tr_frag(Ks, sh, dt, lane), df, dq[dt]);  // dQ^T += K^T dS^T
    }
  }
  const int nvalid = min(16, p.N - q0);
  if (nvalid > 0) fa_store_T(Ot[w], dq, p.scale, p.dq + base + (int64_t)q0 * p.sn, p.sn, nvalid, lane);
}

bool fa_check(const FaParams& p) {
  // 16-B aligned rows: every stride and base a multiple of 8 elements
  auto al = [](const void* ptr) { return ((uintptr_t)ptr & 15) == 0; };
  return p.N > 0 && p.B > 0 && p.H > 0 && p.sn % 8 == 0 && p.sh % 8 == 0 && p.sb % 8 == 0 &&
         p.on % 8 == 0 && p.oh % 8 == 0 && p.ob % 8 == 0 && al(p.q) && al(p.k) && al(p.v) && al(p.o);
}

}  // namespace

// qkv: [B, N, 3, H, 64] bf16 (q / k / v interleaved as the fused projection
// writes them); o: [B, N, H, 64] bf16; lse: [B*H*N] fp32.
MDA_API int mda_attn_fwd(const void* qkv, void* o, float* lse, int64_t B, int64_t N, int64_t H,
                         float scale, hipStream_t st) {
  FaParams p{};
  const bf16_t* base = (const bf16_t*)qkv;
  p.q = base; p.k = base + H * FD; p.v = base + 2 * H * FD;
  p.sn = 3 * H * FD; p.sh = FD; p.sb = N * p.sn;
  p.o = (bf16_t*)o; p.on = H * FD; p.oh = FD; p.ob = N * p.on;
  p.lse = lse; p.B = (int)B; p.H = (int)H; p.N = (int)N; p.scale = scale;
  if (!fa_check(p) || N > (1 << 20)) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)((N + 63) / 64), (unsigned)(B * H));
  hipLaunchKernelGGL(fa_fwd_kernel, grid, dim3(256), 0, st, p);
  MDA_CHECK_LAUNCH();
}

// dqkv: [B, N, 3, H, 64] bf16 (written whole); dsum: [B*H*N] fp32 scratch.
MDA_API int mda_attn_bwd(const void* qkv, const void* o, const void* dout, const float* lse, float* dsum,
                         void* dqkv, int64_t B, int64_t N, int64_t H, float scale, hipStream_t st) {
  FaParams p{};
  const bf16_t* base = (const bf16_t*)qkv;
  p.q = base; p.k = base + H * FD; p.v = base + 2 * H * FD;
  p.sn = 3 * H * FD; p.sh = FD; p.sb = N * p.sn;
  p.o = (bf16_t*)o; p.dout = (const bf16_t*)dout; p.on = H * FD; p.oh = FD; p.ob = N * p.on;
  p.lse = (float*)lse; p.dsum = dsum;
  bf16_t* g = (bf16_t*)dqkv;
  p.dq = g; p.dk = g + H * FD; p.dv = g + 2 * H * FD;
  p.B = (int)B; p.H = (int)H; p.N = (int)N; p.scale = scale;
  if (!fa_check(p) || ((uintptr_t)dout & 15) || ((uintptr_t)dqkv & 15)) return (int)hipErrorInvalidValue;
  const int64_t rows = B * H * N;
  hipLaunchKernelGGL(fa_dsum_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, st, p);
  dim3 grid((unsigned)((N + 63) / 64), (unsigned)(B * H));
  hipLaunchKernelGGL(fa_bwd_dkv_kernel, grid, dim3(256), 0, st, p);
  hipLaunchKernelGGL(fa_bwd_dq_kernel, grid, dim3(256), 0, st, p);
  MDA_CHECK_LAUNCH();
}
