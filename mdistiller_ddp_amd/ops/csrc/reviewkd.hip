// ReviewKD hot paths (survey K9; reference distillers/ReviewKD.py:11-28 HCL,
// :106-144 ABF).
//
//  * HCL (hierarchical context loss), every level in ONE launch:
//      L_i = ( mse(fs, ft) + sum_{l in 4,2,1; l < h} c_l * mse(P_l fs, P_l ft) ) / tot_i
//    with P_l = adaptive_avg_pool2d(., l), c_l = 1/2, 1/4, 1/8 (only levels
//    with l < h count), tot_i = 1 + sum c_l.  A block owns one image and CPB
//    channels of one level: it stages d = fs - ft for its (h*w, CPB) slab in
//    LDS (fp32), reduces the squared error and every adaptive-pool cell with
//    fixed-order tree reductions (deterministic), writes dL/dfs for the slab
//    (the pooled terms' gradients spread back over each cell, overlapping
//    adaptive bins included) and one loss partial.  A finalize kernel sums
//    the partials in fixed order.  Replaces ~12 PyTorch kernels per level
//    forward + backward (pools, MSEs, means, casts, fills).
//  * ABF attention fusion (below): out = x * s0 + up(y) * s1 with
//    (s0, s1) = sigmoid(W [x; up(y)] + b), nearest upsampling folded into the
//    indexing, forward and backward without materialising the concat.
#include "common.h"

namespace {

// ---------------------------------------------------------------------------
// HCL
constexpr int HCL_FIELDS = 10;
constexpr int HCL_MAX_LEVELS = 8;
// level table (int64): fs, ft, grad, N, H, W, C, CPB, first_block, nblocks.
// Passed BY VALUE as a kernel argument: a hipGraph captures it with the
// launch, so per-step activation pointers need no device-side table upload.
struct HclTable {
  int64_t v[HCL_MAX_LEVELS * HCL_FIELDS];
};

__device__ __forceinline__ int bin_start(int i, int h, int l) { return (i * h) / l; }
__device__ __forceinline__ int bin_end(int i, int h, int l) { return ((i + 1) * h + l - 1) / l; }

// fixed-order block reduction of one float per thread (256 threads)
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0) t = (scratch[0] + scratch[1]) + (scratch[2] + scratch[3]);
  return t;  // valid in thread 0
}

__device__ __forceinline__ float kd_factor(float weight, const float* epoch, float warmup) {
  float f = weight;
  if (epoch != nullptr && warmup > 0.f) f *= fminf(*epoch / warmup, 1.f);
  return f;
}

// level index t in {0: l=4, 1: l=2, 2: l=1} owning flattened cell `cell`
__device__ __forceinline__ int cell_level(int cell, const int (&off)[3], const float (&cnt)[3]) {
  const int ls[3] = {4, 2, 1};
  for (int t = 0; t < 3; ++t)
    if (cnt[t] > 0.f && cell >= off[t] && cell < off[t] + ls[t] * ls[t]) return t;
  return 2;
}

constexpr int HCL_MAX_CPB = 32;
constexpr int HCL_BINS = 7;  // x-bins of the three levels: 4 + 2 + 1

// VW consecutive bf16 (VW in 1, 2, 4, 8) <-> floats
template <int VW>
__device__ __forceinline__ void ld_bf16(const bf16_t* p, float* v) {
  if constexpr (VW == 8) {
    const uint4 u = *(const uint4*)p;
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[2 * e] = __uint_as_float(w[e] << 16); v[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u); }
  } else if constexpr (VW == 4) {
    const uint2 u = *(const uint2*)p;
    v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  } else if constexpr (VW == 2) {
    const uint32_t u = *(const uint32_t*)p;
    v[0] = __uint_as_float(u << 16); v[1] = __uint_as_float(u & 0xffff0000u);
  } else {
    v[0] = bf2f(*p);
  }
}
template <int VW>
__device__ __forceinline__ void st_bf16(bf16_t* p, const float* v) {
  if constexpr (VW == 8) {
    *(uint4*)p = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                            pack_bf16x2(v[6], v[7]));
  } else if constexpr (VW == 4) {
    *(uint2*)p = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
  } else if constexpr (VW == 2) {
    *(uint32_t*)p = pack_bf16x2(v[0], v[1]);
  } else {
    *p = f2bf(v[0]);
  }
}

// One block = one image x CPB channels of one level.  Phases (fixed order ->
// deterministic): stage d = fs - ft in LDS with VW-wide loads; row-bin sums
// R[y][b][k] over each level's x-bins; cell sums over each cell's y-bin of R
// (separable: every serial sum is <= one bin wide, where summing a whole
// 56x56 map per thread made this one kernel 290 us of a ResNet-34 step);
// loss partial; gradient with VW-wide stores.
template <int VW>
__device__ __forceinline__ void hcl_block(const int64_t* e, int local, float* partial, float weight,
                                          const float* epoch, float warmup, float* sd, float* scratch,
                                          float* cells) {
  const bf16_t* fs = (const bf16_t*)e[0];
  const bf16_t* ft = (const bf16_t*)e[1];
  bf16_t* grad = (bf16_t*)e[2];
  const int N = (int)e[3], H = (int)e[4], W = (int)e[5], C = (int)e[6], CPB = (int)e[7];
  const int groups = C / CPB;
  const int n = local / groups;
  const int c0 = (local - n * groups) * CPB;
  const int HW = H * W;
  const int tid = threadIdx.x;
  float* const R = sd + HW * CPB;  // [H][HCL_BINS][CPB]
  const int64_t base = (int64_t)n * HW * C + c0;
  // ---- stage d = fs - ft
  float sq = 0.f;
  const int nv = HW * CPB / VW;
  for (int q = tid; q < nv; q += blockDim.x) {
    const int e0 = q * VW;
    const int p = e0 / CPB, k = e0 - p * CPB;
    const int64_t o = base + (int64_t)p * C + k;
    float a[VW], b[VW];
    ld_bf16<VW>(fs + o, a);
    ld_bf16<VW>(ft + o, b);
#pragma unroll
    for (int v = 0; v < VW; ++v) {
      const float d = a[v] - b[v];
      sd[e0 + v] = d;
      sq += d * d;
    }
  }
  const float sqsum = block_sum(sq, scratch);  // also orders the LDS writes
  // ---- levels l = 4, 2, 1 with l < H (and l < W)
  const int levels[3] = {4, 2, 1};
  const int bin0[3] = {0, 4, 6};
  int cell_off[3];
  float cnt[3];
  float tot = 1.f, cw = 1.f;
  int ncell = 0;
  for (int t = 0; t < 3; ++t) {
    const int l = levels[t];
    cell_off[t] = ncell;
    cnt[t] = 0.f;
    if (l < H && l < W) {  // reference: `if l >= h: continue` (square maps)
      cw *= 0.5f;
      cnt[t] = cw;
      tot += cw;
      ncell += l * l;
    }
  }
  // ---- row-bin sums
  for (int q = tid; q < H * HCL_BINS * CPB; q += blockDim.x) {
    const int y = q / (HCL_BINS * CPB);
    const int rem = q - y * (HCL_BINS * CPB);
    const int b = rem / CPB, k = rem - b * CPB;
    const int t = b < 4 ? 0 : (b < 6 ? 1 : 2);
    const int l = levels[t], ix = b - bin0[t];
    float s = 0.f;
    if (cnt[t] > 0.f) {
      const int x0 = bin_start(ix, W, l), x1 = bin_end(ix, W, l);
      for (int xx = x0; xx < x1; ++xx) s += sd[(y * W + xx) * CPB + k];
    }
    R[q] = s;
  }
  __syncthreads();
  // ---- cell means
  for (int q = tid; q < ncell * CPB; q += blockDim.x) {
    const int cell = q / CPB, k = q - cell * CPB;
    const int t = cell_level(cell, cell_off, cnt);
    const int l = levels[t];
    const int ci = cell - cell_off[t];
    const int iy = ci / l, ix = ci - iy * l;
    const int y0 = bin_start(iy, H, l), y1 = bin_end(iy, H, l);
    const int x0 = bin_start(ix, W, l), x1 = bin_end(ix, W, l);
    float s = 0.f;
    for (int yy = y0; yy < y1; ++yy) s += R[(yy * HCL_BINS + bin0[t] + ix) * CPB + k];
    cells[cell * CPB + k] = s / (float)((y1 - y0) * (x1 - x0));  // mean difference
  }
  __syncthreads();
  // ---- loss partial: (sum d^2 / numel + sum_l c_l * sum_cells D^2 / (N*C*l*l)) / tot
  const float numel = (float)N * C * HW;
  float cl = 0.f;
  for (int q = tid; q < ncell * CPB; q += blockDim.x) {
    const int cell = q / CPB;
    const int t = cell_level(cell, cell_off, cnt);
    const int l = levels[t];
    const float D = cells[q];
    cl += cnt[t] * D * D / ((float)N * C * l * l);
  }
  const float cellsum = block_sum(cl, scratch);
  const float f = kd_factor(weight, epoch, warmup);
  if (tid == 0) partial[blockIdx.x] = (sqsum / numel + cellsum) / tot;
  // ---- gradient of the weighted, warmed-up loss w.r.t. fs
  const float inv_tot = f / tot;
  for (int q = tid; q < nv; q += blockDim.x) {
    const int e0 = q * VW;
    const int p = e0 / CPB, k0 = e0 - p * CPB;
    const int yy = p / W, xx = p - yy * W;
    float g[VW];
#pragma unroll
    for (int v = 0; v < VW; ++v) g[v] = 2.f * sd[e0 + v] / numel;
    for (int t = 0; t < 3; ++t) {
      if (cnt[t] == 0.f) continue;
      const int l = levels[t];
      const float scale = cnt[t] * 2.f / ((float)N * C * l * l);
      // adaptive bins may overlap: visit every cell containing (yy, xx)
      const int iy_lo = (yy * l) / H > 0 ? (yy * l) / H - 1 : 0;
      const int ix_lo = (xx * l) / W > 0 ? (xx * l) / W - 1 : 0;
      for (int iy = iy_lo; iy < l && bin_start(iy, H, l) <= yy; ++iy) {
        if (yy >= bin_end(iy, H, l)) continue;
        const int ah = bin_end(iy, H, l) - bin_start(iy, H, l);
        for (int ix = ix_lo; ix < l && bin_start(ix, W, l) <= xx; ++ix) {
          if (xx >= bin_end(ix, W, l)) continue;
          const int aw = bin_end(ix, W, l) - bin_start(ix, W, l);
          const float* cp = cells + (cell_off[t] + iy * l + ix) * CPB + k0;
          const float sc = scale / (float)(ah * aw);
#pragma unroll
          for (int v = 0; v < VW; ++v) g[v] += sc * cp[v];
        }
      }
    }
#pragma unroll
    for (int v = 0; v < VW; ++v) g[v] *= inv_tot;
    st_bf16<VW>(grad + base + (int64_t)p * C + k0, g);
  }
}

__global__ void __launch_bounds__(256)
hcl_kernel(const HclTable table, int L, float* __restrict__ partial, float weight,
           const float* __restrict__ epoch, float warmup) {
  extern __shared__ float sd[];  // [HW][CPB] differences, then [H][HCL_BINS][CPB] row-bin sums
  __shared__ float scratch[4];
  __shared__ float cells[21 * HCL_MAX_CPB];  // 4x4 + 2x2 + 1x1 cells
  const int64_t* tb = table.v;
  int lv = 0;
  while (lv + 1 < L && (int64_t)blockIdx.x >= tb[(lv + 1) * HCL_FIELDS + 8]) ++lv;
  const int64_t* e = tb + lv * HCL_FIELDS;
  const int local = blockIdx.x - (int)e[8];
  const int CPB = (int)e[7];
  if (CPB >= 8) hcl_block<8>(e, local, partial, weight, epoch, warmup, sd, scratch, cells);
  else if (CPB == 4) hcl_block<4>(e, local, partial, weight, epoch, warmup, sd, scratch, cells);
  else if (CPB == 2) hcl_block<2>(e, local, partial, weight, epoch, warmup, sd, scratch, cells);
  else hcl_block<1>(e, local, partial, weight, epoch, warmup, sd, scratch, cells);
}

__global__ void __launch_bounds__(256)
hcl_finalize_kernel(const float* __restrict__ partial, int nblk, float weight,
                    const float* __restrict__ epoch, float warmup, float* __restrict__ loss) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < nblk; i += blockDim.x) s += (double)partial[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = (float)red[0] * kd_factor(weight, epoch, warmup);
}

// ---------------------------------------------------------------------------
// ABF attention fusion.  x [N, h, w, C], y [N, hy, wy, C] (nearest-upsampled
// to h x w by index), Wt [2, 2C] fp32, bias [2].  One group of G = C/8
// threads per pixel (G power of two <= 64); 16-byte channel vectors.
__device__ __forceinline__ int up_src(int i, int out, int in) {
  // PyTorch 'nearest': src = floor(dst * in / out)
  return (int)(((int64_t)i * in) / out);
}

__device__ __forceinline__ void ld8(const bf16_t* p, float (&o)[8]) {
  const uint4 r = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    o[2 * k] = __uint_as_float(w[k] << 16);
    o[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}
__device__ __forceinline__ void st8(bf16_t* p, const float (&v)[8]) {
  *reinterpret_cast<uint4*>(p) = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                            pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
}
__device__ __forceinline__ float group_sum(float v, int G) {
  for (int o = G >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(256)
abf_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ y,
               const float* __restrict__ Wt, const float* __restrict__ bias,
               bf16_t* __restrict__ out, float* __restrict__ att, int N, int h, int w, int hy,
               int wy, int C) {
  const int G = C / 8;
  const int ppb = 256 / G;  // pixels per block pass
  const int g = threadIdx.x % G, pl = threadIdx.x / G;
  const int c0 = g * 8;
  const int64_t P = (int64_t)N * h * w;
  float wx0[8], wx1[8], wy0[8], wy1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    wx0[k] = Wt[c0 + k];
    wy0[k] = Wt[C + c0 + k];
    wx1[k] = Wt[2 * C + c0 + k];
    wy1[k] = Wt[3 * C + c0 + k];
  }
  const float b0 = bias ? bias[0] : 0.f, b1 = bias ? bias[1] : 0.f;
  for (int64_t p = (int64_t)blockIdx.x * ppb + pl; p < P; p += (int64_t)gridDim.x * ppb) {
    const int xx = (int)(p % w);
    const int64_t r = p / w;
    const int yy = (int)(r % h);
    const int n = (int)(r / h);
    const int64_t py = ((int64_t)n * hy + up_src(yy, h, hy)) * wy + up_src(xx, w, wy);
    float xv[8], yv[8];
    ld8(x + p * C + c0, xv);
    ld8(y + py * C + c0, yv);
    float z0 = 0.f, z1 = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      z0 += wx0[k] * xv[k] + wy0[k] * yv[k];
      z1 += wx1[k] * xv[k] + wy1[k] * yv[k];
    }
    z0 = group_sum(z0, G) + b0;
    z1 = group_sum(z1, G) + b1;
    const float s0 = 1.f / (1.f + __expf(-z0)), s1 = 1.f / (1.f + __expf(-z1));
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = xv[k] * s0 + yv[k] * s1;
    st8(out + p * C + c0, o);
    if (g == 0 && att) {
      att[2 * p] = s0;
      att[2 * p + 1] = s1;
    }
  }
}

// Per pixel: dz_k = (sum_c dout*[x|y]_c) * s_k (1 - s_k); dx = dout*s0 + dz0*Wx0 + dz1*Wx1;
// dyup (fp32, full res) = dout*s1 + dz0*Wy0 + dz1*Wy1; block partials of
// dW[k][c] = sum dz_k * [x|y]_c and db_k = sum dz_k -> partial[blk][4C + 2].
__global__ void __launch_bounds__(256)
abf_bwd_kernel(const bf16_t* __restrict__ dout, const bf16_t* __restrict__ x,
               const bf16_t* __restrict__ y, const float* __restrict__ att,
               const float* __restrict__ Wt, bf16_t* __restrict__ dx, float* __restrict__ dyup,
               float* __restrict__ partial, int N, int h, int w, int hy, int wy, int C) {
  extern __shared__ float red[];  // [ppb][4C + 2]
  const int G = C / 8;
  const int ppb = 256 / G;
  const int g = threadIdx.x % G, pl = threadIdx.x / G;
  const int c0 = g * 8;
  const int64_t P = (int64_t)N * h * w;
  const int V = 4 * C + 2;
  float wx0[8], wx1[8], wy0[8], wy1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    wx0[k] = Wt[c0 + k];
    wy0[k] = Wt[C + c0 + k];
    wx1[k] = Wt[2 * C + c0 + k];
    wy1[k] = Wt[3 * C + c0 + k];
  }
  float aw0x[8], aw0y[8], aw1x[8], aw1y[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) aw0x[k] = aw0y[k] = aw1x[k] = aw1y[k] = 0.f;
  float adb0 = 0.f, adb1 = 0.f;
  for (int64_t p = (int64_t)blockIdx.x * ppb + pl; p < P; p += (int64_t)gridDim.x * ppb) {
    const int xx = (int)(p % w);
    const int64_t r = p / w;
    const int yy = (int)(r % h);
    const int n = (int)(r / h);
    const int64_t py = ((int64_t)n * hy + up_src(yy, h, hy)) * wy + up_src(xx, w, wy);
    float xv[8], yv[8], dv[8];
    ld8(x + p * C + c0, xv);
    ld8(y + py * C + c0, yv);
    ld8(dout + p * C + c0, dv);
    const float s0 = att[2 * p], s1 = att[2 * p + 1];
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      a0 += dv[k] * xv[k];
      a1 += dv[k] * yv[k];
    }
    a0 = group_sum(a0, G);
    a1 = group_sum(a1, G);
    const float dz0 = a0 * s0 * (1.f - s0), dz1 = a1 * s1 * (1.f - s1);
    float ox[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      ox[k] = dv[k] * s0 + dz0 * wx0[k] + dz1 * wx1[k];
      float* dyp = dyup + p * C + c0;
      dyp[k] = dv[k] * s1 + dz0 * wy0[k] + dz1 * wy1[k];
      aw0x[k] += dz0 * xv[k];
      aw0y[k] += dz0 * yv[k];
      aw1x[k] += dz1 * xv[k];
      aw1y[k] += dz1 * yv[k];
    }
    st8(dx + p * C + c0, ox);
    adb0 += dz0;
    adb1 += dz1;
  }
  // block partials: reduce over the ppb pixel lanes in fixed order
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[pl * V + c0 + k] = aw0x[k];
    red[pl * V + C + c0 + k] = aw0y[k];
    red[pl * V + 2 * C + c0 + k] = aw1x[k];
    red[pl * V + 3 * C + c0 + k] = aw1y[k];
  }
  if (g == 0) {
    red[pl * V + 4 * C] = adb0;
    red[pl * V + 4 * C + 1] = adb1;
  }
  __syncthreads();
  for (int v = threadIdx.x; v < V; v += blockDim.x) {
    float s = 0.f;
    for (int q = 0; q < ppb; ++q) s += red[q * V + v];
    partial[(int64_t)blockIdx.x * V + v] = s;
  }
}

// dy[n, iy, ix, c] = sum of dyup over the h x w pixels whose nearest source is (iy, ix)
__global__ void __launch_bounds__(256)
abf_dy_gather_kernel(const float* __restrict__ dyup, bf16_t* __restrict__ dy, int N, int h, int w,
                     int hy, int wy, int C) {
  const int C8 = C / 8;
  const int64_t total = (int64_t)N * hy * wy * C8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int cg = (int)(i % C8);
    int64_t r = i / C8;
    const int ix = (int)(r % wy);
    r /= wy;
    const int iy = (int)(r % hy);
    const int n = (int)(r / hy);
    // destination rows/cols mapping to (iy, ix): floor(d * in / out) == i
    const int ya = (int)(((int64_t)iy * h + hy - 1) / hy), yb = (int)(((int64_t)(iy + 1) * h + hy - 1) / hy);
    const int xa = (int)(((int64_t)ix * w + wy - 1) / wy), xb = (int)(((int64_t)(ix + 1) * w + wy - 1) / wy);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int yy = ya; yy < yb && yy < h; ++yy)
      for (int xx = xa; xx < xb && xx < w; ++xx) {
        const float* s = dyup + ((((int64_t)n * h + yy) * w + xx) * C) + cg * 8;
        const float4 lo = *reinterpret_cast<const float4*>(s);
        const float4 hi = *reinterpret_cast<const float4*>(s + 4);
        acc[0] += lo.x; acc[1] += lo.y; acc[2] += lo.z; acc[3] += lo.w;
        acc[4] += hi.x; acc[5] += hi.y; acc[6] += hi.z; acc[7] += hi.w;
      }
    st8(dy + ((((int64_t)n * hy + iy) * wy + ix) * C) + cg * 8, acc);
  }
}

// dW [2, 2C] / db [2] (+)= fixed-order sum of the block partials.  A block
// owns 64 consecutive outputs; its 16 wavefronts each sum a fixed stride-16
// subset of the nblk partial rows (coalesced 256-B rows), then wave 0 adds
// the 16 sub-sums in order: deterministic, and 16x the parallelism of one
// serial loop per output (which left this kernel at ~68 us for C = 256).
constexpr int ABF_FIN_G = 16;
__global__ void __launch_bounds__(64 * ABF_FIN_G)
abf_wgrad_finalize_kernel(const float* __restrict__ partial, int nblk, int C,
                          float* __restrict__ dW, float* __restrict__ db, int accumulate) {
  __shared__ double red[ABF_FIN_G][64];
  const int V = 4 * C + 2;
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int v = blockIdx.x * 64 + lane;
  double s = 0.0;
  if (v < V)
    for (int b = g; b < nblk; b += ABF_FIN_G) s += (double)partial[(int64_t)b * V + v];
  red[g][lane] = s;
  __syncthreads();
  if (g != 0 || v >= V) return;
  double t = 0.0;
#pragma unroll
  for (int i = 0; i < ABF_FIN_G; ++i) t += red[i][lane];
  float* o = nullptr;
  // partial layout: [x-part k0 | y-part k0 | x-part k1 | y-part k1 | db0 db1]
  if (v < 4 * C) {
    if (dW) o = dW + v;  // == [k][2C] row-major: k0 -> [0, 2C), k1 -> [2C, 4C)
  } else if (db) {
    o = db + (v - 4 * C);
  }
  if (o) *o = accumulate ? *o + (float)t : (float)t;
}

}  // namespace

// table: L levels x 10 int64 (fs, ft, grad, N, H, W, C, CPB, first_block, nblocks);
// partial >= total blocks floats; loss [1] = weight * w(epoch) * sum_i L_i and the
// grads hold d loss / d fs_i (w = min(epoch / warmup, 1) when epoch is given).
// table: HOST array of L x 10 int64.
MDA_API int mda_hcl_loss(const int64_t* table, int64_t L, int64_t nblk, int64_t lds_floats,
                         float* partial, float weight, const float* epoch, float warmup,
                         float* loss, hipStream_t st) {
  if (L < 1 || L > HCL_MAX_LEVELS || nblk < 1 || lds_floats * 4 > 150 * 1024)
    return (int)hipErrorInvalidValue;
  HclTable tb{};
  for (int64_t i = 0; i < L * HCL_FIELDS; ++i) tb.v[i] = table[i];
  for (int64_t l = 0; l < L; ++l) {  // shape sanity before touching device memory
    const int64_t* e = tb.v + l * HCL_FIELDS;
    const int64_t cpb = e[7];
    if (cpb < 1 || cpb > HCL_MAX_CPB || (cpb & (cpb - 1)) || e[6] % cpb ||
        (e[4] * e[5] + e[4] * HCL_BINS) * cpb > lds_floats ||
        e[9] != e[3] * (e[6] / e[7]))
      return (int)hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(hcl_kernel, dim3((unsigned)nblk), dim3(256), lds_floats * sizeof(float), st,
                     tb, (int)L, partial, weight, epoch, warmup);
  hipLaunchKernelGGL(hcl_finalize_kernel, dim3(1), dim3(256), 0, st, partial, (int)nblk, weight,
                     epoch, warmup, loss);
  MDA_CHECK_LAUNCH();
}

MDA_API int mda_abf_fwd(const void* x, const void* y, const float* Wt, const float* bias, void* out,
                        float* att, int64_t N, int64_t h, int64_t w, int64_t hy, int64_t wy,
                        int64_t C, hipStream_t st) {
  const int64_t G = C / 8;
  if (C % 8 || G > 64 || (G & (G - 1))) return (int)hipErrorInvalidValue;
  const int64_t ppb = 256 / G;
  int64_t blocks = (N * h * w + ppb - 1) / ppb;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(abf_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const bf16_t*)x,
                     (const bf16_t*)y, Wt, bias, (bf16_t*)out, att, (int)N, (int)h, (int)w,
                     (int)hy, (int)wy, (int)C);
  MDA_CHECK_LAUNCH();
}

MDA_API int mda_abf_bwd_blocks(int64_t N, int64_t h, int64_t w, int64_t C, int64_t* nblk) {
  const int64_t ppb = 256 / (C / 8);
  int64_t b = (N * h * w + ppb * 8 - 1) / (ppb * 8);  // ~8 pixels per lane
  if (b > 512) b = 512;
  if (b < 1) b = 1;
  *nblk = b;
  return 0;
}

// dyup: N*h*w*C fp32 scratch; partial: nblk*(4C+2) floats.
MDA_API int mda_abf_bwd(const void* dout, const void* x, const void* y, const float* att,
                        const float* Wt, void* dx, void* dy, float* dyup, float* partial,
                        float* dW, float* db, int64_t N, int64_t h, int64_t w, int64_t hy,
                        int64_t wy, int64_t C, int64_t nblk, int64_t accumulate, hipStream_t st) {
  const int64_t G = C / 8;
  if (C % 8 || G > 64 || (G & (G - 1)) || nblk < 1) return (int)hipErrorInvalidValue;
  const int64_t ppb = 256 / G;
  const size_t lds = (size_t)ppb * (4 * C + 2) * sizeof(float);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(abf_bwd_kernel, dim3((unsigned)nblk), dim3(256), lds, st,
                     (const bf16_t*)dout, (const bf16_t*)x, (const bf16_t*)y, att, Wt,
                     (bf16_t*)dx, dyup, partial, (int)N, (int)h, (int)w, (int)hy, (int)wy, (int)C);
  if (dy) {
    int64_t tot = N * hy * wy * G;
    int64_t blocks = (tot + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(abf_dy_gather_kernel, dim3((unsigned)blocks), dim3(256), 0, st, dyup,
                       (bf16_t*)dy, (int)N, (int)h, (int)w, (int)hy, (int)wy, (int)C);
  }
  if (dW || db) {
    int64_t V = 4 * C + 2;
    hipLaunchKernelGGL(abf_wgrad_finalize_kernel, dim3((unsigned)((V + 63) / 64)), dim3(64 * ABF_FIN_G),
                       0, st, partial, (int)nblk, (int)C, dW, db, (int)accumulate);
  }
  MDA_CHECK_LAUNCH();
}
