// Fused logit-distillation losses: CE + {KD | DKD} forward AND gradient in one
// pass over the logits (reference formulas: distillers/KD.py:8-13,
// distillers/DKD.py:8-32; survey K6/K7).
//
// One wave (64 lanes) owns one row of C classes; each lane keeps up to
// NPL = C/64 student and teacher logits in registers, so the row is read
// once from HBM and every softmax/log-softmax/KL term is computed in fp32.
// Per-block partial loss sums are reduced by the last-arriving block in a
// fixed order, so the scalar losses are deterministic (no float atomics).
//
// Outputs
//   losses[0] = ce_w * mean_b CE(s_b, y_b)
//   losses[1] = kd_w * w(epoch) * (KD | DKD) as defined by the reference,
//               w = min(epoch / warmup, 1) when an epoch pointer is given (else 1)
//   g_ce[b,c] = d losses[0] / d s[b,c]     (same dtype as s)
//   g_kd[b,c] = d losses[1] / d s[b,c]
//   g_sum[b,c] = g_ce + g_kd (optional, fp32 sum rounded once)
// The autograd backward combines them as go_ce*g_ce + go_kd*g_kd
// (mda_axpby) so the two-backward DOT trainer works unchanged; with the
// training step's constant unit seeds it returns g_sum (or g_ce) and
// launches nothing (ops/losses.py register_unit_seed).
#include "common.h"

namespace {

constexpr int ROWS_PER_BLOCK = 4;   // 4 waves per block, one row each
constexpr int MAXNPL = 32;          // C <= 2048

enum { MODE_CE = 0, MODE_KD = 1, MODE_DKD = 2 };

template <typename TS, typename TT, typename TG, int NPL, int MODE>
__global__ void __launch_bounds__(256)
logit_loss_kernel(const TS* __restrict__ s, const TT* __restrict__ t,
                  const int64_t* __restrict__ target, TG* __restrict__ g_ce,
                  TG* __restrict__ g_kd, float* __restrict__ partial,
                  unsigned* __restrict__ counter, float* __restrict__ losses,
                  int B, int C, float inv_T, float ce_w, float kd_w, float alpha,
                  float beta, const float* __restrict__ epoch, float warmup,
                  TG* __restrict__ g_sum) {
  // DKD/ReviewKD-style linear warm-up of the KD term, min(epoch / warmup, 1),
  // read from device memory so a replayed hipGraph sees the current epoch
  if (epoch != nullptr && warmup > 0.f) kd_w *= fminf(*epoch / warmup, 1.f);
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int row = blockIdx.x * ROWS_PER_BLOCK + wid;
  float ce_row = 0.f, kd_row = 0.f;
  const float T = 1.f / inv_T;
  const float invB = 1.f / (float)B;

  if (row < B) {
    const int64_t base = (int64_t)row * C;
    const int y = (int)target[row];
    float sv[NPL], tv[NPL];
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      int c = lane + 64 * i;
      bool ok = c < C;
      sv[i] = ok ? io<TS>::ld(s, base + c) : -INFINITY;
      tv[i] = (MODE != MODE_CE && ok) ? io<TT>::ld(t, base + c) : -INFINITY;
    }
    // ---- CE at temperature 1 ------------------------------------------
    float m1 = -INFINITY;
#pragma unroll
    for (int i = 0; i < NPL; ++i) m1 = fmaxf(m1, sv[i]);
    m1 = wave_max(m1);
    float z1 = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) z1 += __expf(sv[i] - m1);
    z1 = wave_sum(z1);
    const float lz1 = __logf(z1);
    float s_y = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i)
      if (lane + 64 * i == y) s_y = sv[i];
    s_y = wave_sum(s_y);
    ce_row = (m1 + lz1 - s_y);  // -log softmax(s)_y
    const float gce_scale = ce_w * invB;
    float gcv[NPL];
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      int c = lane + 64 * i;
      gcv[i] = 0.f;
      if (c < C) {
        float p = __expf(sv[i] - m1 - lz1);
        gcv[i] = gce_scale * (p - (c == y ? 1.f : 0.f));
        io<TG>::st(g_ce, base + c, gcv[i]);
      }
    }
    if (MODE == MODE_KD || MODE == MODE_DKD) {
      // ---- tempered softmaxes ------------------------------------------
      float ms = -INFINITY, mt = -INFINITY;
#pragma unroll
      for (int i = 0; i < NPL; ++i) {
        ms = fmaxf(ms, sv[i] * inv_T);
        mt = fmaxf(mt, tv[i] * inv_T);
      }
      ms = wave_max(ms);
      mt = wave_max(mt);
      if (MODE == MODE_KD) {
        float zs = 0.f, zt = 0.f;
#pragma unroll
        for (int i = 0; i < NPL; ++i) {
          zs += __expf(sv[i] * inv_T - ms);
          zt += __expf(tv[i] * inv_T - mt);
        }
        zs = wave_sum(zs);
        zt = wave_sum(zt);
        const float lzs = __logf(zs), lzt = __logf(zt);
        float kl = 0.f;
        const float gscale = kd_w * T * invB;  // d(T^2 KL / B)/ds = T (q - p) / B
#pragma unroll
        for (int i = 0; i < NPL; ++i) {
          int c = lane + 64 * i;
          if (c < C) {
            float lq = sv[i] * inv_T - ms - lzs;
            float lp = tv[i] * inv_T - mt - lzt;
            float p = __expf(lp);
            kl += p * (lp - lq);
            const float gk = gscale * (__expf(lq) - p);
            io<TG>::st(g_kd, base + c, gk);
            if (g_sum) io<TG>::st(g_sum, base + c, gcv[i] + gk);
          }
        }
        kd_row = wave_sum(kl) * T * T;
      } else {
        // ---- DKD: TCKD (binary gt/other) + NCKD (softmax over non-gt) ---
        // The non-target softmaxes are normalised by their OWN maxima (the
        // reference's -1000*gt_mask does the same): with a dominant target
        // logit (gap > ~88 at T = 1) every non-target exp under the full
        // maximum underflows to 0 and log(0) made the loss infinite.
        float ms_o = -INFINITY, mt_o = -INFINITY;
#pragma unroll
        for (int i = 0; i < NPL; ++i) {
          if (lane + 64 * i != y) {
            ms_o = fmaxf(ms_o, sv[i] * inv_T);
            mt_o = fmaxf(mt_o, tv[i] * inv_T);
          }
        }
        ms_o = wave_max(ms_o);
        mt_o = wave_max(mt_o);
        float zs_o = 0.f, zt_o = 0.f;
#pragma unroll
        for (int i = 0; i < NPL; ++i) {
          if (lane + 64 * i != y) {
            zs_o += __expf(sv[i] * inv_T - ms_o);
            zt_o += __expf(tv[i] * inv_T - mt_o);
          }
        }
        zs_o = wave_sum(zs_o);
        zt_o = wave_sum(zt_o);
        const float lzs_o = __logf(zs_o), lzt_o = __logf(zt_o);
        // binary (target, other) distributions in the log domain:
        // log P(other) = log sum_{j != y} exp(z_j) = m_o + log Z_o
        const float sy = s_y * inv_T;
        float ty = 0.f;
#pragma unroll
        for (int i = 0; i < NPL; ++i)
          if (lane + 64 * i == y) ty = tv[i] * inv_T;
        ty = wave_sum(ty);
        const float ls_o_raw = ms_o + lzs_o, lt_o_raw = mt_o + lzt_o;
        const float ls_n = fmaxf(sy, ls_o_raw) + __logf(1.f + __expf(-fabsf(sy - ls_o_raw)));
        const float lt_n = fmaxf(ty, lt_o_raw) + __logf(1.f + __expf(-fabsf(ty - lt_o_raw)));
        const float lps_g = sy - ls_n, lps_o = ls_o_raw - ls_n;
        const float lpt_g = ty - lt_n, lpt_o = lt_o_raw - lt_n;
        const float ps_g = __expf(lps_g), pt_g = __expf(lpt_g);
        float tckd = 0.f;
        if (pt_g > 0.f) tckd += pt_g * (lpt_g - lps_g);
        const float pt_o = __expf(lpt_o);
        if (pt_o > 0.f) tckd += pt_o * (lpt_o - lps_o);
        float nckd = 0.f;
        const float gs = kd_w * T * invB;
        const float tck = pt_g - ps_g;  // d TCKD / d z_j = q_j (pt_g - ps_g) for j != gt
#pragma unroll
        for (int i = 0; i < NPL; ++i) {
          int c = lane + 64 * i;
          if (c < C) {
            float gz;
            if (c == y) {
              gz = alpha * (ps_g - pt_g);
            } else {
              const float lq = sv[i] * inv_T - ms_o - lzs_o, lp = tv[i] * inv_T - mt_o - lzt_o;
              const float ph = __expf(lp), qh = __expf(lq);
              nckd += ph * (lp - lq);
              gz = alpha * qh * tck + beta * (qh - ph);
            }
            io<TG>::st(g_kd, base + c, gs * gz);
            if (g_sum) io<TG>::st(g_sum, base + c, gcv[i] + gs * gz);
          }
        }
        nckd = wave_sum(nckd);
        kd_row = (alpha * tckd + beta * nckd) * T * T;
      }
    }
  }
  // ---- deterministic batch reduction ------------------------------------
  __shared__ float red[2][ROWS_PER_BLOCK];
  if (lane == 0) {
    red[0][wid] = ce_row;
    red[1][wid] = kd_row;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f;
    for (int w = 0; w < ROWS_PER_BLOCK; ++w) { a += red[0][w]; b += red[1][w]; }
    partial[2 * blockIdx.x] = a;
    partial[2 * blockIdx.x + 1] = b;
  }
  if (mda_arrive(counter, gridDim.x)) {
    // fixed-order tree over blocks: wave 0 strides, then wave_sum
    if (wid == 0) {
      float a = 0.f, b = 0.f;
      for (int i = lane; i < (int)gridDim.x; i += 64) {
        a += partial[2 * i];
        b += partial[2 * i + 1];
      }
      a = wave_sum(a);
      b = wave_sum(b);
      if (lane == 0) {
        losses[0] = ce_w * a * invB;
        losses[1] = kd_w * b * invB;
      }
    }
  }
}

template <typename TS, typename TT, int MODE, int NPL>
int launch_t(const void* s, const void* t, const int64_t* y, void* gce, void* gkd, float* part,
             unsigned* cnt, float* losses, int B, int C, float invT, float cew, float kdw, float a,
             float b, const float* ep, float wu, void* gsum, hipStream_t st) {
  dim3 grid((B + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK);
  hipLaunchKernelGGL((logit_loss_kernel<TS, TT, TS, NPL, MODE>), grid, dim3(256), 0, st,
                     (const TS*)s, (const TT*)t, y, (TS*)gce, (TS*)gkd, part, cnt, losses, B, C,
                     invT, cew, kdw, a, b, ep, wu, (TS*)gsum);
  MDA_CHECK_LAUNCH();
}

template <typename TS, typename TT, int MODE>
int launch_npl(const void* s, const void* t, const int64_t* y, void* gce, void* gkd, float* part,
               unsigned* cnt, float* losses, int B, int C, float invT, float cew, float kdw,
               float a, float b, const float* ep, float wu, void* gsum, hipStream_t st) {
  int npl = (C + 63) / 64;
#define NPL_CASE(N)                                                                          \
  if (npl <= N)                                                                              \
    return launch_t<TS, TT, MODE, N>(s, t, y, gce, gkd, part, cnt, losses, B, C, invT, cew, \
                                     kdw, a, b, ep, wu, gsum, st);
  NPL_CASE(2) NPL_CASE(4) NPL_CASE(8) NPL_CASE(16) NPL_CASE(32)
#undef NPL_CASE
  return (int)hipErrorInvalidValue;
}

template <int MODE>
int launch_mode(int dts, int dtt, const void* s, const void* t, const int64_t* y, void* gce,
                void* gkd, float* part, unsigned* cnt, float* losses, int B, int C, float invT,
                float cew, float kdw, float a, float b, const float* ep, float wu, void* gs,
                hipStream_t st) {
  if (dts == DT_F32 && dtt == DT_F32)
    return launch_npl<float, float, MODE>(s, t, y, gce, gkd, part, cnt, losses, B, C, invT, cew, kdw, a, b, ep, wu, gs, st);
  if (dts == DT_BF16 && dtt == DT_BF16)
    return launch_npl<bf16_t, bf16_t, MODE>(s, t, y, gce, gkd, part, cnt, losses, B, C, invT, cew, kdw, a, b, ep, wu, gs, st);
  if (dts == DT_BF16 && dtt == DT_F32)
    return launch_npl<bf16_t, float, MODE>(s, t, y, gce, gkd, part, cnt, losses, B, C, invT, cew, kdw, a, b, ep, wu, gs, st);
  return launch_npl<float, bf16_t, MODE>(s, t, y, gce, gkd, part, cnt, losses, B, C, invT, cew, kdw, a, b, ep, wu, gs, st);
}

// out = (*a) * x + (*b) * y ; a/b are device scalars (graph-replay safe).
template <typename T>
__global__ void axpby_kernel(const float* __restrict__ a, const T* __restrict__ x,
                             const float* __restrict__ b, const T* __restrict__ y,
                             T* __restrict__ out, int64_t n) {
  const float av = a ? *a : 0.f, bv = b ? *b : 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    if (a) v += av * io<T>::ld(x, i);
    if (b) v += bv * io<T>::ld(y, i);
    io<T>::st(out, i, v);
  }
}

}  // namespace

// mode: 0 = CE only, 1 = CE + KD, 2 = CE + DKD
MDA_API int mda_logit_loss(int64_t mode, int64_t dts, int64_t dtt, const void* s, const void* t,
                           const int64_t* y, void* g_ce, void* g_kd, float* partial,
                           unsigned* counter, float* losses, int64_t B, int64_t C, float inv_T,
                           float ce_w, float kd_w, float alpha, float beta, const float* epoch,
                           float warmup, void* g_sum, hipStream_t st) {
  if (C > 64 * MAXNPL || B <= 0) return (int)hipErrorInvalidValue;
  if (mode == MODE_CE) g_sum = nullptr;
  if (mode == MODE_CE)
    return launch_mode<MODE_CE>(dts, dtt, s, t, y, g_ce, g_kd, partial, counter, losses, B, C, inv_T, ce_w, kd_w, alpha, beta, epoch, warmup, g_sum, st);
  if (mode == MODE_KD)
    return launch_mode<MODE_KD>(dts, dtt, s, t, y, g_ce, g_kd, partial, counter, losses, B, C, inv_T, ce_w, kd_w, alpha, beta, epoch, warmup, g_sum, st);
  return launch_mode<MODE_DKD>(dts, dtt, s, t, y, g_ce, g_kd, partial, counter, losses, B, C, inv_T, ce_w, kd_w, alpha, beta, epoch, warmup, g_sum, st);
}

MDA_API int mda_axpby(int64_t dt, const float* a, const void* x, const float* b, const void* y,
                      void* out, int64_t n, hipStream_t st) {
  int blocks = (int)((n + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  if (dt == DT_F32)
    hipLaunchKernelGGL(axpby_kernel<float>, dim3(blocks), dim3(256), 0, st, a, (const float*)x, b,
                       (const float*)y, (float*)out, n);
  else
    hipLaunchKernelGGL(axpby_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, a, (const bf16_t*)x,
                       b, (const bf16_t*)y, (bf16_t*)out, n);
  MDA_CHECK_LAUNCH();
}
