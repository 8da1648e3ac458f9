// BatchNorm channel-sum "region": the cross-block reduction of ONE training
// BN (forward statistics or backward sums), accumulated by device-scope fp64
// atomics instead of per-block partial rows + a separate finalize launch
// (round 3, csrc/bn.hip "fused BN").
//
//   producer (conv epilogue, stats pass, or the first phase of the fused
//   backward): each block adds its 2*C per-channel sums into shard
//   blockIdx % SH of acc (non-returning global_atomic_add_f64);
//   consumer (the next launch, or the same launch behind a grid barrier):
//   every block sums the SH shards of the channels it needs.
//
// Regions are used ONCE: the training step hands each BN call its own region
// of a per-device arena that one memset zeroes at the start of every step
// (ops/hip_train.py::bn_step_begin, captured into the step's hipGraph), so
// no kernel has to clean up after itself -- no departure ticket, no reset
// fan-in (a single 256-512-way counter costs 3-6 us at device scope).
//
// Shards: per-address atomics serialise (~12 ns each at device scope), so the
// blocks of one launch are spread over SH = clamp(1024 / C, 1, 8) copies.
// fp64 sums of fp32 block partials: order-independent to fp64 rounding, i.e.
// bitwise-stable in fp32 in all but vanishing cases (docs/DESIGN.md 3.3).
#pragma once
#include "common.h"

constexpr int SLOT_CMAX = 2048;
constexpr int SLOT_SHMAX = 8;
constexpr int BAR_GROUPS = 8;  // grid-barrier arrival groups (blockIdx % 8)

struct BnRegion {
  unsigned grp[BAR_GROUPS];  // per-group arrival counters
  unsigned top;              // groups complete
  unsigned pad[7];
  double acc[1];             // [SH][2][C]: q 0 = sum a, q 1 = sum b
};

__host__ __device__ __forceinline__ int slot_shards(int C) {
  const int s = 1024 / (C > 0 ? C : 1);
  return s < 1 ? 1 : (s > SLOT_SHMAX ? SLOT_SHMAX : s);
}

__host__ __device__ __forceinline__ int64_t region_bytes(int C) {
  return 64 + (int64_t)slot_shards(C) * 2 * C * 8;
}

__device__ __forceinline__ double* region_acc(BnRegion* r, int C, int shard, int q) {
  return r->acc + (shard * 2 + q) * C;
}

__device__ __forceinline__ void acc_add(double* a, double v) {
  __hip_atomic_fetch_add(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double acc_load(const double* a) {
  return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Grid-wide barrier for grids that are resident by construction (the fused
// BN backward launches at most one small block per CU) on a fresh region.
// Everything a block published before it are device-scope atomics, drained
// by vmcnt(0) before its arrival, and every read after it is a device-coherent
// load, so no L2 write-back / invalidate fence is needed (CDNA HIP guide G16,
// sc1 form).  XCD-style hierarchy: blocks arrive on one of 8 group counters;
// the last of a group bumps `top`; thread 0 of every block polls `top`.
// Spins are bounded (~2 s): on timeout *err is set and the kernel
// completes with wrong values instead of hanging the GPU.
// nb blocks in the grid, bid = this block's linear index (2-D / 3-D grids).
__device__ __forceinline__ void region_grid_barrier_n(BnRegion* r, unsigned* err, unsigned nb,
                                                      unsigned bid) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = bid % BAR_GROUPS;
    const unsigned ngroups = nb < BAR_GROUPS ? nb : BAR_GROUPS;
    const unsigned gsize = (nb - g + BAR_GROUPS - 1) / BAR_GROUPS;
    const unsigned t = __hip_atomic_fetch_add(&r->grp[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gsize - 1) __hip_atomic_fetch_add(&r->top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(&r->top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < ngroups) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 100 MHz clock: 2 s
        if (err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void region_grid_barrier(BnRegion* r, unsigned* err) {
  region_grid_barrier_n(r, err, gridDim.x, blockIdx.x);
}

// Finalize / running-stat operands of one training BN (forward).
struct FinArgs {
  const float* gamma; const float* beta;
  float* running_mean; float* running_var;
  float* stats;          // [4][C]: mean, rstd, scale, shift (written by one block)
  float momentum, eps;
  int64_t* nbt;
};

// Channel c's totals over the SH shards (plain loads when the sums come from
// an earlier launch, device-coherent ones behind an in-kernel barrier): all
// 2*SH loads of a channel in flight together.
template <bool COHERENT>
__device__ __forceinline__ void region_channel(BnRegion* r, int C, int c, double& t0, double& t1) {
  const int SH = slot_shards(C);
  double a[SLOT_SHMAX], b[SLOT_SHMAX];
#pragma unroll
  for (int k = 0; k < SLOT_SHMAX; ++k) {
    const double* pa = region_acc(r, C, k, 0) + c;
    const double* pb = region_acc(r, C, k, 1) + c;
    a[k] = k < SH ? (COHERENT ? acc_load(pa) : *pa) : 0.0;
    b[k] = k < SH ? (COHERENT ? acc_load(pb) : *pb) : 0.0;
  }
  t0 = 0.0;
  t1 = 0.0;
#pragma unroll
  for (int k = 0; k < SLOT_SHMAX; ++k) { t0 += a[k]; t1 += b[k]; }
}

// Batch statistics of channel c from a region -> scale / shift; `writer`
// (one block per channel) also stores the [4][C] stats of the backward and
// updates the running statistics.
template <bool COHERENT>
__device__ __forceinline__ void fin_channel_w(BnRegion* reg, int64_t M, int C, int c, const FinArgs& f,
                                              float& sc, float& sh, bool writer) {
  double t0, t1;
  region_channel<COHERENT>(reg, C, c, t0, t1);
  const double mean = t0 / (double)M;
  double var = t1 / (double)M - mean * mean;
  if (var < 0) var = 0;
  const float rstd = (float)(1.0 / sqrt(var + (double)f.eps));
  const float g = f.gamma ? f.gamma[c] : 1.f;
  const float bb = f.beta ? f.beta[c] : 0.f;
  sc = g * rstd;
  sh = bb - (float)mean * sc;
  if (writer) {
    f.stats[c] = (float)mean;
    f.stats[C + c] = rstd;
    f.stats[2 * C + c] = sc;
    f.stats[3 * C + c] = sh;
    if (f.running_mean) {
      const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
      f.running_mean[c] = (1.f - f.momentum) * f.running_mean[c] + f.momentum * (float)mean;
      f.running_var[c] = (1.f - f.momentum) * f.running_var[c] + f.momentum * (float)unbiased;
    }
  }
}
