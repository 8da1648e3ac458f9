// Shared helpers for the CDNA4 (gfx950) kernels of mdistiller_ddp_amd.
// bf16 is carried as raw uint16_t (upper half of an fp32) so every kernel can
// be templated on {float, bf16} storage with fp32 math.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MDA_API extern "C" __attribute__((visibility("default")))
// status of an optional fused launcher that did not launch (shape / mode not
// served): the caller takes the unfused path.  Distinct from every hipError_t.
#define MDA_NOT_SERVED (-1)

typedef uint16_t bf16_t;

struct bf16x { bf16_t v; };  // tag type for templates

__device__ __forceinline__ float bf2f(bf16_t b) {
  return __uint_as_float(((uint32_t)b) << 16);
}
// gfx950 converts natively (v_cvt_pk_bf16_f32: round-to-nearest-even, NaN kept)
__device__ __forceinline__ bf16_t f2bf(float f) {
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}
typedef __attribute__((ext_vector_type(2))) __bf16 mda_bf16x2;
// two floats -> packed bf16 pair (lo = a), one instruction
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  mda_bf16x2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

template <typename T> struct io;
template <> struct io<float> {
  static __device__ __forceinline__ float ld(const float* p, int64_t i) { return p[i]; }
  static __device__ __forceinline__ void st(float* p, int64_t i, float v) { p[i] = v; }
};
template <> struct io<bf16_t> {
  static __device__ __forceinline__ float ld(const bf16_t* p, int64_t i) { return bf2f(p[i]); }
  static __device__ __forceinline__ void st(bf16_t* p, int64_t i, float v) { p[i] = f2bf(v); }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// dtype codes shared with the Python side (ops/_ext.py)
enum { DT_F32 = 0, DT_BF16 = 1 };

#define MDA_CHECK_LAUNCH() return (int)hipGetLastError()

// ---------------------------------------------------------------------------
// Deterministic cross-block "last arriver reduces" hand-off (agent-scope
// release/acquire; see the CDNA HIP guide, Guideline 16 recipe).
// Each block writes its partials with plain stores, then calls
// mda_arrive(); the block that returns true may read every partial.
__device__ __forceinline__ bool mda_arrive(unsigned* counter, unsigned nblocks) {
  __shared__ unsigned s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == nblocks - 1) ? 1u : 0u;
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // reset for the next launch (the buffer starts zeroed)
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  return s_last != 0;
}
