// CRD contrastive memory (reference distillers/CRD.py:144-220; survey K10).
//
// scores:  e[b, k] = exp( <memory[idx[b, k]], v[b]> / T )            (B x (K+1))
// grad:    gv[b]   = sum_k  g[b, k] * e[b, k] / T * memory[idx[b, k]]
// update:  memory[y[b]] = normalize( m * memory[y[b]] + (1 - m) * v[b] )
//
// The reference materialises index_select(memory, idx) as a
// B x (K+1) x D tensor (537 MB per bank per step at B=64, K=16384, D=128)
// and runs a bmm over it, twice per bank (forward and backward).  Here the
// rows are streamed straight from the bank (L2 / Infinity Cache resident:
// 25.6 MB per bank on CIFAR) and consumed in registers: 16 lanes per row,
// 8 floats per lane (two 16-byte loads), 4 rows per wave instruction.
#include "common.h"

namespace {

constexpr int LPR = 16;  // lanes per row

template <int D>
__global__ void __launch_bounds__(256)
crd_scores_kernel(const float* __restrict__ mem, const int64_t* __restrict__ idx,
                  const float* __restrict__ v, float* __restrict__ e, int K1, float invT) {
  constexpr int VPL = D / LPR;  // floats per lane
  const int b = blockIdx.y;
  const int sub = threadIdx.x & (LPR - 1);
  const int group = (blockIdx.x * blockDim.x + threadIdx.x) / LPR;
  const int ngroups = gridDim.x * blockDim.x / LPR;
  float vr[VPL];
#pragma unroll
  for (int i = 0; i < VPL; i += 4) *(float4*)&vr[i] = *(const float4*)&v[(int64_t)b * D + sub * VPL + i];
  for (int k = group; k < K1; k += ngroups) {
    const int64_t row = idx[(int64_t)b * K1 + k];
    const float* w = mem + row * D + sub * VPL;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; i += 4) {
      float4 x = *(const float4*)&w[i];
      acc += x.x * vr[i] + x.y * vr[i + 1] + x.z * vr[i + 2] + x.w * vr[i + 3];
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (sub == 0) e[(int64_t)b * K1 + k] = __expf(acc * invT);
  }
}

// partial[b, chunk, :] = sum over this chunk's k of coef[b,k] * mem[idx[b,k]]
template <int D>
__global__ void __launch_bounds__(256)
crd_grad_kernel(const float* __restrict__ mem, const int64_t* __restrict__ idx,
                const float* __restrict__ g, const float* __restrict__ e,
                float* __restrict__ partial, int K1, float invT) {
  constexpr int VPL = D / LPR;
  const int b = blockIdx.y;
  const int chunk = blockIdx.x;
  const int nchunks = gridDim.x;
  const int sub = threadIdx.x & (LPR - 1);
  const int grp = threadIdx.x / LPR;          // 16 groups per block
  const int per = (K1 + nchunks - 1) / nchunks;
  const int k0 = chunk * per, k1 = min(K1, k0 + per);
  float acc[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) acc[i] = 0.f;
  for (int k = k0 + grp; k < k1; k += 256 / LPR) {
    const int64_t o = (int64_t)b * K1 + k;
    const float c = g[o] * e[o] * invT;
    const float* w = mem + idx[o] * D + sub * VPL;
#pragma unroll
    for (int i = 0; i < VPL; i += 4) {
      float4 x = *(const float4*)&w[i];
      acc[i] += c * x.x; acc[i + 1] += c * x.y; acc[i + 2] += c * x.z; acc[i + 3] += c * x.w;
    }
  }
  __shared__ float red[256 / LPR][D];
#pragma unroll
  for (int i = 0; i < VPL; ++i) red[grp][sub * VPL + i] = acc[i];
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float s = 0.f;
    for (int q = 0; q < 256 / LPR; ++q) s += red[q][d];
    partial[((int64_t)b * nchunks + chunk) * D + d] = s;
  }
}

template <int D>
__global__ void crd_grad_reduce(const float* __restrict__ partial, float* __restrict__ gv,
                                int nchunks) {
  const int b = blockIdx.x;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float s = 0.f;
    for (int c = 0; c < nchunks; ++c) s += partial[((int64_t)b * nchunks + c) * D + d];
    gv[(int64_t)b * D + d] = s;
  }
}

// one wave per updated row
__global__ void __launch_bounds__(256)
crd_update_kernel(float* __restrict__ mem, const int64_t* __restrict__ y,
                  const float* __restrict__ v, int B, int D, float momentum) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  float* row = mem + y[b] * (int64_t)D;
  const float* vb = v + (int64_t)b * D;
  float ss = 0.f;
  for (int d = lane; d < D; d += 64) {
    float l = momentum * row[d] + (1.f - momentum) * vb[d];
    ss += l * l;
  }
  ss = wave_sum(ss);
  const float inv = rsqrtf(ss);
  for (int d = lane; d < D; d += 64) {
    float l = momentum * row[d] + (1.f - momentum) * vb[d];
    row[d] = l * inv;
  }
}

}  // namespace

MDA_API int mda_crd_scores(const float* mem, const int64_t* idx, const float* v, float* e,
                           int64_t B, int64_t K1, int64_t D, float invT, hipStream_t st) {
  dim3 grid((int)std::min<int64_t>(64, (K1 * LPR + 255) / 256), (int)B);
  if (D == 128)
    hipLaunchKernelGGL(crd_scores_kernel<128>, grid, dim3(256), 0, st, mem, idx, v, e, (int)K1, invT);
  else if (D == 64)
    hipLaunchKernelGGL(crd_scores_kernel<64>, grid, dim3(256), 0, st, mem, idx, v, e, (int)K1, invT);
  else if (D == 256)
    hipLaunchKernelGGL(crd_scores_kernel<256>, grid, dim3(256), 0, st, mem, idx, v, e, (int)K1, invT);
  else
    return (int)hipErrorInvalidValue;
  MDA_CHECK_LAUNCH();
}

// partial: B * nchunks * D floats (nchunks = 16)
MDA_API int mda_crd_grad(const float* mem, const int64_t* idx, const float* g, const float* e,
                         float* partial, float* gv, int64_t B, int64_t K1, int64_t D, float invT,
                         hipStream_t st) {
  const int nchunks = 16;
  dim3 grid(nchunks, (int)B);
#define CRD_G(DD)                                                                              \
  hipLaunchKernelGGL(crd_grad_kernel<DD>, grid, dim3(256), 0, st, mem, idx, g, e, partial,     \
                     (int)K1, invT);                                                           \
  hipLaunchKernelGGL(crd_grad_reduce<DD>, dim3((int)B), dim3(128), 0, st, partial, gv, nchunks);
  if (D == 128) { CRD_G(128) }
  else if (D == 64) { CRD_G(64) }
  else if (D == 256) { CRD_G(256) }
  else return (int)hipErrorInvalidValue;
#undef CRD_G
  MDA_CHECK_LAUNCH();
}

MDA_API int mda_crd_update(float* mem, const int64_t* y, const float* v, int64_t B, int64_t D,
                           float momentum, hipStream_t st) {
  hipLaunchKernelGGL(crd_update_kernel, dim3((int)((B + 3) / 4)), dim3(256), 0, st, mem, y, v,
                     (int)B, (int)D, momentum);
  MDA_CHECK_LAUNCH();
}
