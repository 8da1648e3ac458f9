// Classifier head and per-step metrics (survey K4/K5/K15).
//
//  * pool_fc  -- global average pool of the last NHWC feature map fused with
//    the Linear classifier: one block per image pools its HW x C tile into
//    LDS (fp32), writes the pooled feature and the J logits (fp32 weights,
//    fp32 accumulation, one thread per logit).  The backward is ONE launch:
//    blocks [0, J) produce dW/db rows (accumulated straight into the flat fp32
//    gradient views), blocks [J, J+N) produce d(feature map) = (dpooled +
//    dlogits @ W) / HW broadcast over the HW positions.  Replaces avg_pool2d +
//    hipBLASLt GEMM + bias/cast kernels (~8 launches per head per step at
//    batch 64) -- the reference runs F.avg_pool2d + nn.Linear
//    (models/cifar/resnet.py:123-124).
//  * meters_update -- top-1/top-5 hit counts (rank of the target logit), loss
//    sums, sample and step counts accumulated into one fp64 device buffer in a
//    single launch (reference: utils.accuracy + per-iteration all-reduces,
//    engine/utils.py:125-136, trainer.py:277-281).
#include "common.h"

namespace {

// grid (N, ceil(J / 256)).  Phase 1: the block pools image n into LDS -- 8
// channels per thread with 16-byte loads, pixel groups reduced through LDS.
// Phase 2: one thread per logit, dot(pooled, W[j]) with 16-byte weight loads
// (independent loads, no serial cross-lane reductions).
template <typename T>
__global__ void __launch_bounds__(256)
pool_fc_fwd_kernel(const T* __restrict__ x, int HW, int C, const float* __restrict__ W,
                   const float* __restrict__ bias, T* __restrict__ pooled, T* __restrict__ logits,
                   int J, float inv_hw) {
  extern __shared__ float sh[];  // [C] pooled + [256 * 8] partials
  float* sp = sh;
  float* part = sh + C;
  const int n = blockIdx.x;
  const T* xn = x + (int64_t)n * HW * C;
  const int tid = threadIdx.x;
  constexpr int V = 16 / sizeof(T);  // elements per 16-byte load
  const int CG = C / V;
  if (C % V == 0 && CG <= 256) {
    const int P = 256 / CG;  // pixel groups
    const int cg = tid % CG, pg = tid / CG;
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
    if (pg < P) {
      for (int p = pg; p < HW; p += P) {
        const uint4 raw = *reinterpret_cast<const uint4*>(xn + (int64_t)p * C + cg * V);
        const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
        for (int i = 0; i < V; ++i) acc[i] += io<T>::ld(e, i);
      }
#pragma unroll
      for (int i = 0; i < V; ++i) part[pg * C + cg * V + i] = acc[i];
    }
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
      float s = 0.f;
      for (int q = 0; q < P; ++q) s += part[q * C + c];
      sp[c] = s * inv_hw;
    }
  } else {
    for (int c = tid; c < C; c += 256) {
      float s = 0.f;
      for (int p = 0; p < HW; ++p) s += io<T>::ld(xn, (int64_t)p * C + c);
      sp[c] = s * inv_hw;
    }
  }
  __syncthreads();
  // round to the storage dtype: the classifier consumes the stored feature,
  // as the unfused path (pool -> tensor -> Linear) does
  for (int c = tid; c < C; c += 256) {
    if (blockIdx.y == 0) io<T>::st(pooled, (int64_t)n * C + c, sp[c]);
    T r;
    io<T>::st(&r, 0, sp[c]);
    sp[c] = io<T>::ld(&r, 0);
  }
  __syncthreads();
  const int j = blockIdx.y * 256 + tid;
  if (j < J) {
    const float* wj = W + (int64_t)j * C;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int c = 0;
    if ((C & 3) == 0) {
      for (; c < C; c += 4) {
        const float4 w4 = *reinterpret_cast<const float4*>(wj + c);
        a0 += sp[c] * w4.x;
        a1 += sp[c + 1] * w4.y;
        a2 += sp[c + 2] * w4.z;
        a3 += sp[c + 3] * w4.w;
      }
    }
    for (; c < C; ++c) a0 += sp[c] * wj[c];
    io<T>::st(logits, (int64_t)n * J + j, ((a0 + a1) + (a2 + a3)) + (bias ? bias[j] : 0.f));
  }
}

template <typename T>
__global__ void __launch_bounds__(256)
pool_fc_bwd_kernel(const T* __restrict__ dl, const T* __restrict__ dpooled,
                   const T* __restrict__ pooled, const float* __restrict__ W,
                   float* __restrict__ dW, float* __restrict__ db, T* __restrict__ dx, int N,
                   int HW, int C, int J, float inv_hw, int accum) {
  extern __shared__ float sh[];
  if ((int)blockIdx.x < J) {
    // ---- dW[j, :] = sum_n dl[n, j] * pooled[n, :];  db[j] = sum_n dl[n, j]
    const int j = blockIdx.x;
    for (int n = threadIdx.x; n < N; n += blockDim.x) sh[n] = io<T>::ld(dl, (int64_t)n * J + j);
    __syncthreads();
    if (dW != nullptr) {
      for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float acc = 0.f;
        for (int n = 0; n < N; ++n) acc += sh[n] * io<T>::ld(pooled, (int64_t)n * C + c);
        float* o = dW + (int64_t)j * C + c;
        *o = accum ? *o + acc : acc;
      }
    }
    if (db != nullptr && threadIdx.x < 64) {
      float acc = 0.f;
      for (int n = threadIdx.x; n < N; n += 64) acc += sh[n];
      acc = wave_sum(acc);
      if (threadIdx.x == 0) db[j] = accum ? db[j] + acc : acc;
    }
    return;
  }
  // ---- dx[n, p, :] = (dpooled[n, :] + dl[n, :] @ W) / HW   for every p
  const int n = blockIdx.x - J;
  for (int j = threadIdx.x; j < J; j += blockDim.x) sh[j] = io<T>::ld(dl, (int64_t)n * J + j);
  __syncthreads();
  T* dxn = dx + (int64_t)n * HW * C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float acc = dpooled ? io<T>::ld(dpooled, (int64_t)n * C + c) : 0.f;
    for (int j = 0; j < J; ++j) acc += sh[j] * W[(int64_t)j * C + c];
    const float v = acc * inv_hw;
    for (int p = 0; p < HW; ++p) io<T>::st(dxn, (int64_t)p * C + c, v);
  }
}

template <typename T>
__global__ void __launch_bounds__(256)
meters_kernel(const T* __restrict__ preds, const int64_t* __restrict__ target, int B, int C,
              const float* __restrict__ l0, const float* __restrict__ l1,
              const float* __restrict__ l2, const float* __restrict__ l3, int nloss,
              double* __restrict__ buf) {
  __shared__ int s_hits[2];
  if (threadIdx.x < 2) s_hits[threadIdx.x] = 0;
  __syncthreads();
  int h1 = 0, h5 = 0;
  // one thread per row: C independent loads, no cross-lane reduction chain
  for (int r = threadIdx.x; r < B; r += blockDim.x) {
    const int64_t base = (int64_t)r * C;
    const int tg = (int)target[r];
    const float t = io<T>::ld(preds, base + tg);
    // rank of the target = classes ordered before it by topk: strictly larger
    // logits, plus EQUAL logits at a lower class index (ties are frequent with
    // bf16 logits and must not count as hits)
    int c0 = 0, c1 = 0, c2 = 0, c3 = 0, c = 0;
    for (; c + 4 <= tg; c += 4) {
      c0 += io<T>::ld(preds, base + c) >= t;
      c1 += io<T>::ld(preds, base + c + 1) >= t;
      c2 += io<T>::ld(preds, base + c + 2) >= t;
      c3 += io<T>::ld(preds, base + c + 3) >= t;
    }
    for (; c < tg; ++c) c0 += io<T>::ld(preds, base + c) >= t;
    for (c = tg + 1; c + 4 <= C; c += 4) {
      c0 += io<T>::ld(preds, base + c) > t;
      c1 += io<T>::ld(preds, base + c + 1) > t;
      c2 += io<T>::ld(preds, base + c + 2) > t;
      c3 += io<T>::ld(preds, base + c + 3) > t;
    }
    for (; c < C; ++c) c0 += io<T>::ld(preds, base + c) > t;
    const int cnt = c0 + c1 + c2 + c3;
    h1 += cnt < 1;
    h5 += cnt < 5;
  }
  if (h1) atomicAdd(&s_hits[0], h1);
  if (h5) atomicAdd(&s_hits[1], h5);
  __syncthreads();
  if (threadIdx.x == 0) {
    const float* ls[4] = {l0, l1, l2, l3};
    double total = 0.0;
    for (int i = 0; i < nloss; ++i) {
      const double v = (double)*ls[i];
      buf[1 + i] += v;
      total += v;
    }
    buf[0] += total;
    buf[nloss + 1] += (double)s_hits[0];
    buf[nloss + 2] += (double)s_hits[1];
    buf[nloss + 3] += (double)B;
    buf[nloss + 4] += 1.0;
  }
}

}  // namespace

// x [N, HW, C] (NHWC) fp32|bf16; W [J, C] fp32; bias [J] fp32 or null;
// pooled [N, C], logits [N, J] in x's dtype.
MDA_API int mda_pool_fc_fwd(int64_t dt, const void* x, const float* W, const float* bias,
                            void* pooled, void* logits, int64_t N, int64_t HW, int64_t C,
                            int64_t J, hipStream_t st) {
  if (N <= 0 || C <= 0 || C > 8192 || J <= 0) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)(C + 256 * 8) * sizeof(float);
  const dim3 grid((unsigned)N, (unsigned)((J + 255) / 256));
  if (dt == DT_F32)
    hipLaunchKernelGGL(pool_fc_fwd_kernel<float>, grid, dim3(256), lds, st, (const float*)x,
                       (int)HW, (int)C, W, bias, (float*)pooled, (float*)logits, (int)J, 1.f / HW);
  else
    hipLaunchKernelGGL(pool_fc_fwd_kernel<bf16_t>, grid, dim3(256), lds, st, (const bf16_t*)x,
                       (int)HW, (int)C, W, bias, (bf16_t*)pooled, (bf16_t*)logits, (int)J, 1.f / HW);
  MDA_CHECK_LAUNCH();
}

// dl [N, J]; dpooled [N, C] or null; pooled [N, C]; W [J, C] fp32; dW [J, C] fp32 or
// null; db [J] fp32 or null; dx [N, HW, C].  accum: dW/db += instead of =.
MDA_API int mda_pool_fc_bwd(int64_t dt, const void* dl, const void* dpooled, const void* pooled,
                            const float* W, float* dW, float* db, void* dx, int64_t N, int64_t HW,
                            int64_t C, int64_t J, int64_t accum, hipStream_t st) {
  if (N <= 0 || C <= 0 || J <= 0 || N > 16384 || J > 16384) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)(N > J ? N : J) * sizeof(float);
  const dim3 grid((unsigned)(J + N));
  if (dt == DT_F32)
    hipLaunchKernelGGL(pool_fc_bwd_kernel<float>, grid, dim3(256), lds, st, (const float*)dl,
                       (const float*)dpooled, (const float*)pooled, W, dW, db, (float*)dx, (int)N,
                       (int)HW, (int)C, (int)J, 1.f / HW, (int)accum);
  else
    hipLaunchKernelGGL(pool_fc_bwd_kernel<bf16_t>, grid, dim3(256), lds, st, (const bf16_t*)dl,
                       (const bf16_t*)dpooled, (const bf16_t*)pooled, W, dW, db, (bf16_t*)dx,
                       (int)N, (int)HW, (int)C, (int)J, 1.f / HW, (int)accum);
  MDA_CHECK_LAUNCH();
}

// preds [B, C] fp32|bf16; target [B] int64; l0..l3 fp32 scalars (first nloss used);
// buf fp64 [1 + nloss + 4] = [total, per-loss..., top1, top5, samples, steps].
MDA_API int mda_meters_update(int64_t dt, const void* preds, const int64_t* target, int64_t B,
                              int64_t C, const float* l0, const float* l1, const float* l2,
                              const float* l3, int64_t nloss, double* buf, hipStream_t st) {
  if (nloss < 0 || nloss > 4 || B <= 0) return (int)hipErrorInvalidValue;
  if (dt == DT_F32)
    hipLaunchKernelGGL(meters_kernel<float>, dim3(1), dim3(256), 0, st, (const float*)preds, target,
                       (int)B, (int)C, l0, l1, l2, l3, (int)nloss, buf);
  else
    hipLaunchKernelGGL(meters_kernel<bf16_t>, dim3(1), dim3(256), 0, st, (const bf16_t*)preds,
                       target, (int)B, (int)C, l0, l1, l2, l3, (int)nloss, buf);
  MDA_CHECK_LAUNCH();
}
