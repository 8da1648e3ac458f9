// Fused multi-tensor optimizers over ONE flat fp32 parameter buffer
// (survey K13/K14).  Every trainable tensor of the distiller is a view into
// a flat buffer, so each update is a single launch of float4 streams, and the
// learning rate / clip norm / Adam step live in device memory so a captured
// hipGraph replays the step with a new schedule value without re-capture.
//
//   SGD  (torch.optim.SGD, dampening 0, no nesterov):
//        d = s*g + wd*p ; buf = mu*buf + d ; p -= lr*buf
//   DOT  (reference engine/dot.py:15-55, survey §3.3), per element mask
//        bit0 = receives a task (CE) grad, bit1 = receives a KD grad:
//        task pass:  d = s*g_t + wd*p
//                    buf_t = first ? d : (both ? mu_t : (mu_t+mu_k)/2)*buf_t + d
//                    p -= lr*buf_t
//        kd pass:    both:    buf_k = first ? s*g_k : mu_k*buf_k + s*g_k
//                    kd only: buf_k = first ? s*g_k : (mu_t+mu_k)/2*buf_k + s*g_k + wd*p
//                    p -= lr*buf_k
//   Adam / AdamW (torch semantics, bias-corrected, step count on device).
// s = grad scale (1/world_size for a SUM all-reduce) times the optional
// clip coefficient min(1, max_norm / (||g|| + 1e-6)) read from *norm.
#include "common.h"

namespace {

__device__ __forceinline__ float clip_coef(const float* norm, float max_norm) {
  if (!norm || max_norm <= 0.f) return 1.f;
  float c = max_norm / (*norm + 1e-6f);
  return c < 1.f ? c : 1.f;
}

__global__ void __launch_bounds__(256)
sgd_kernel(float4* __restrict__ p, const float4* __restrict__ g, float4* __restrict__ buf,
           const float* __restrict__ lr_p, float mu, float wd, float gscale,
           const float* __restrict__ norm, float max_norm, int64_t n4) {
  const float lr = *lr_p;
  const float s = gscale * clip_coef(norm, max_norm);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 pv = p[i], gv = g[i];
    float4 d;
    d.x = s * gv.x + wd * pv.x; d.y = s * gv.y + wd * pv.y;
    d.z = s * gv.z + wd * pv.z; d.w = s * gv.w + wd * pv.w;
    if (mu != 0.f) {
      float4 b = buf[i];
      b.x = mu * b.x + d.x; b.y = mu * b.y + d.y; b.z = mu * b.z + d.z; b.w = mu * b.w + d.w;
      buf[i] = b;
      d = b;
    }
    pv.x -= lr * d.x; pv.y -= lr * d.y; pv.z -= lr * d.z; pv.w -= lr * d.w;
    p[i] = pv;
  }
}

__global__ void __launch_bounds__(256)
dot_kernel(float* __restrict__ p, const float* __restrict__ gt, const float* __restrict__ gk,
           float* __restrict__ bt, float* __restrict__ bk, const uint8_t* __restrict__ mask,
           const float* __restrict__ lr_p, float mu_t, float mu_k, float wd, float gscale,
           int first, int64_t n) {
  const float lr = *lr_p;
  const float mu_avg = 0.5f * (mu_t + mu_k);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t m = mask[i];
    const bool has_t = m & 1, has_k = m & 2;
    float pv = p[i];
    if (has_t) {
      float d = gscale * gt[i] + wd * pv;
      float b = first ? d : (has_k ? mu_t : mu_avg) * bt[i] + d;
      bt[i] = b;
      pv -= lr * b;
    }
    if (has_k) {
      float d = gscale * gk[i];
      float b;
      if (first) b = d;
      else if (has_t) b = mu_k * bk[i] + d;
      else b = mu_avg * bk[i] + d + wd * pv;
      bk[i] = b;
      pv -= lr * b;
    }
    p[i] = pv;
  }
}

__global__ void __launch_bounds__(256)
adam_kernel(float4* __restrict__ p, const float4* __restrict__ g, float4* __restrict__ m1,
            float4* __restrict__ m2, const float* __restrict__ lr_p,
            const float* __restrict__ step_p, float b1, float b2, float eps, float wd,
            int decoupled, float gscale, const float* __restrict__ norm, float max_norm,
            int64_t n4) {
  const float lr = *lr_p;
  const float t = *step_p;
  const float bc1 = 1.f - powf(b1, t), bc2 = 1.f - powf(b2, t);
  const float step = lr / bc1;
  const float rbc2 = rsqrtf(bc2);
  const float s = gscale * clip_coef(norm, max_norm);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float pa[4], ga[4], ma[4], va[4];
    *(float4*)pa = p[i]; *(float4*)ga = g[i]; *(float4*)ma = m1[i]; *(float4*)va = m2[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gv = s * ga[k];
      if (decoupled) pa[k] *= (1.f - lr * wd);
      else gv += wd * pa[k];
      ma[k] = b1 * ma[k] + (1.f - b1) * gv;
      va[k] = b2 * va[k] + (1.f - b2) * gv * gv;
      float denom = sqrtf(va[k]) * rbc2 + eps;
      pa[k] -= step * ma[k] / denom;
    }
    p[i] = *(float4*)pa; m1[i] = *(float4*)ma; m2[i] = *(float4*)va;
  }
}

// Deterministic ||x||_2 over a flat fp32 buffer: per-block partials, last
// arriver sums them in fixed order and writes sqrt to out[0].
__global__ void __launch_bounds__(256)
sq_norm_kernel(const float4* __restrict__ x, int64_t n4, float* __restrict__ partial,
               unsigned* __restrict__ counter, float* __restrict__ out, float scale) {
  float acc = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 v = x[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  acc = wave_sum(acc);
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
  if (mda_arrive(counter, gridDim.x)) {
    if (wid == 0) {
      float a = 0.f;
      for (int i = lane; i < (int)gridDim.x; i += 64) a += partial[i];
      a = wave_sum(a);
      if (lane == 0) out[0] = sqrtf(a) * scale;
    }
  }
}

__global__ void scale_kernel(float4* __restrict__ x, const float* __restrict__ s, int64_t n4) {
  const float sv = *s;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 v = x[i];
    v.x *= sv; v.y *= sv; v.z *= sv; v.w *= sv;
    x[i] = v;
  }
}

inline int grid_for(int64_t n, int cap = 1024) {
  int64_t b = (n + 255) / 256;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

MDA_API int mda_sgd_step(float* p, const float* g, float* buf, const float* lr, float mu,
                         float wd, float gscale, const float* norm, float max_norm, int64_t n,
                         hipStream_t st) {
  if (n % 4) return (int)hipErrorInvalidValue;
  int64_t n4 = n / 4;
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n4)), dim3(256), 0, st, (float4*)p,
                     (const float4*)g, (float4*)buf, lr, mu, wd, gscale, norm, max_norm, n4);
  MDA_CHECK_LAUNCH();
}

MDA_API int mda_dot_step(float* p, const float* gt, const float* gk, float* bt, float* bk,
                         const uint8_t* mask, const float* lr, float mu_t, float mu_k, float wd,
                         float gscale, int64_t first, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(dot_kernel, dim3(grid_for(n)), dim3(256), 0, st, p, gt, gk, bt, bk, mask,
                     lr, mu_t, mu_k, wd, gscale, (int)first, n);
  MDA_CHECK_LAUNCH();
}

MDA_API int mda_adam_step(float* p, const float* g, float* m1, float* m2, const float* lr,
                          const float* step, float b1, float b2, float eps, float wd,
                          int64_t decoupled, float gscale, const float* norm, float max_norm,
                          int64_t n, hipStream_t st) {
  if (n % 4) return (int)hipErrorInvalidValue;
  int64_t n4 = n / 4;
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n4)), dim3(256), 0, st, (float4*)p,
                     (const float4*)g, (float4*)m1, (float4*)m2, lr, step, b1, b2, eps, wd,
                     (int)decoupled, gscale, norm, max_norm, n4);
  MDA_CHECK_LAUNCH();
}

// out[0] = scale * ||x||_2 ; partial must hold >= 512 floats, counter zeroed once.
MDA_API int mda_sq_norm(const float* x, int64_t n, float* partial, unsigned* counter, float* out,
                        float scale, hipStream_t st) {
  if (n % 4) return (int)hipErrorInvalidValue;
  int64_t n4 = n / 4;
  hipLaunchKernelGGL(sq_norm_kernel, dim3(grid_for(n4, 512)), dim3(256), 0, st,
                     (const float4*)x, n4, partial, counter, out, scale);
  MDA_CHECK_LAUNCH();
}

MDA_API int mda_scale_inplace(float* x, const float* s, int64_t n, hipStream_t st) {
  if (n % 4) return (int)hipErrorInvalidValue;
  int64_t n4 = n / 4;
  hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n4)), dim3(256), 0, st, (float4*)x, s, n4);
  MDA_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Multi-tensor device copy: up to 16 (src, dst, bytes) pairs in ONE launch --
// the replayed step's input + teacher-output copies (engine/step.py
// _step_split), which torch._foreach_copy_ issues as one blit per tensor.
// 16-byte vectors where both ends are aligned, bytes otherwise.
namespace {
constexpr int MCOPY_MAX = 16;
struct MultiCopy {
  const char* src[MCOPY_MAX];
  char* dst[MCOPY_MAX];
  int64_t bytes[MCOPY_MAX];
  int64_t blk0[MCOPY_MAX + 1];  // first block of each pair (prefix sums)
  int n;
};
constexpr int MCOPY_CHUNK = 256 * 16 * 4;  // bytes per block

__global__ void __launch_bounds__(256) multi_copy_kernel(MultiCopy a) {
  int t = 0;
  while (t + 1 < a.n && (int64_t)blockIdx.x >= a.blk0[t + 1]) ++t;
  const int64_t base = ((int64_t)blockIdx.x - a.blk0[t]) * MCOPY_CHUNK;
  const int64_t end = min(base + (int64_t)MCOPY_CHUNK, a.bytes[t]);
  const char* s = a.src[t];
  char* d = a.dst[t];
  const bool vec = (((uintptr_t)s | (uintptr_t)d) & 15) == 0;
  if (vec) {
    const int64_t vend = base + ((end - base) / 16) * 16;
    for (int64_t o = base + threadIdx.x * 16; o < vend; o += 256 * 16)
      *(uint4*)(d + o) = *(const uint4*)(s + o);
    for (int64_t o = vend + threadIdx.x; o < end; o += 256) d[o] = s[o];
  } else {
    for (int64_t o = base + threadIdx.x; o < end; o += 256) d[o] = s[o];
  }
}
}  // namespace

// table: n x 3 int64 {src, dst, bytes} in host memory.
MDA_API int mda_multi_copy(const int64_t* table, int64_t n, hipStream_t st) {
  if (n < 1 || n > MCOPY_MAX) return (int)hipErrorInvalidValue;
  MultiCopy a{};
  a.n = (int)n;
  int64_t blk = 0;
  for (int i = 0; i < n; ++i) {
    a.src[i] = (const char*)table[3 * i];
    a.dst[i] = (char*)table[3 * i + 1];
    a.bytes[i] = table[3 * i + 2];
    a.blk0[i] = blk;
    blk += (a.bytes[i] + MCOPY_CHUNK - 1) / MCOPY_CHUNK;
  }
  a.blk0[n] = blk;
  if (blk <= 0) return 0;
  if (blk > (1 << 30)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(multi_copy_kernel, dim3((unsigned)blk), dim3(256), 0, st, a);
  MDA_CHECK_LAUNCH();
}
