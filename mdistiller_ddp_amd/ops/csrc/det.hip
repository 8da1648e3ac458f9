// Detection ops for the RCNN distillation path (reference detection/ leans on
// Detectron2's CUDA ROIAlign and NMS).
//
// ROIAlign (Detectron2 "ROIAlignV2" semantics: aligned=1 shifts by -0.5 px,
// adaptive sampling grid ceil(roi/bin) when sampling_ratio <= 0) over
// channels-last (NHWC) feature maps -- the layout every conv of this framework
// produces -- so one bilinear tap of 64 consecutive lanes reads 64 consecutive
// channels (coalesced), and the pooled output is written NHWC as well.
// One launch pools ALL FPN levels: each RoI carries its level index, so the
// per-level nonzero()/index_select/scatter of a Python pooler (and its host
// syncs) disappear.  Backward scatters with fp32 atomics shaped as 256-byte
// contiguous channel runs per wave instruction.
//
// NMS on wave64: a whole wavefront scores one box i against 64 candidate boxes
// (one per lane) and __ballot() packs the suppression decisions straight into
// the 64-bit mask word -- the wave width IS the mask width.  The greedy scan
// runs on the device in a single wave (no mask copy to the host).
#include "common.h"

namespace {

constexpr int MAXLEV = 5;

struct Levels {
  const void* x[MAXLEV];  // NHWC feature maps (fwd) / fp32 NHWC grad buffers (bwd)
  int H[MAXLEV], W[MAXLEV];
  float scale[MAXLEV];
};

struct RoiGeom {
  float x1, y1, bw, bh;
  int gh, gw;
  float inv_count;
};

__device__ __forceinline__ RoiGeom roi_geom(const float* roi, float scale, int PH, int PW,
                                            int sampling, int aligned) {
  RoiGeom g;
  const float off = aligned ? 0.5f : 0.f;
  g.x1 = roi[1] * scale - off;
  g.y1 = roi[2] * scale - off;
  float rw = roi[3] * scale - off - g.x1;
  float rh = roi[4] * scale - off - g.y1;
  if (!aligned) {  // legacy: force malformed RoIs to 1x1
    rw = fmaxf(rw, 1.f);
    rh = fmaxf(rh, 1.f);
  }
  g.bh = rh / PH;
  g.bw = rw / PW;
  g.gh = sampling > 0 ? sampling : (int)ceilf(rh / PH);
  g.gw = sampling > 0 ? sampling : (int)ceilf(rw / PW);
  g.gh = max(g.gh, 0);
  g.gw = max(g.gw, 0);
  g.inv_count = 1.f / (float)max(g.gh * g.gw, 1);
  return g;
}

// bilinear corner indices + weights; returns false for samples outside the map
__device__ __forceinline__ bool bilinear(float y, float x, int H, int W, int& o1, int& o2, int& o3,
                                         int& o4, float& w1, float& w2, float& w3, float& w4) {
  if (y < -1.f || y > (float)H || x < -1.f || x > (float)W) return false;
  y = fmaxf(y, 0.f);
  x = fmaxf(x, 0.f);
  int yl = (int)y, xl = (int)x, yh, xh;
  if (yl >= H - 1) { yh = yl = H - 1; y = (float)yl; } else { yh = yl + 1; }
  if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else { xh = xl + 1; }
  const float ly = y - yl, lx = x - xl, hy = 1.f - ly, hx = 1.f - lx;
  w1 = hy * hx; w2 = hy * lx; w3 = ly * hx; w4 = ly * lx;
  o1 = yl * W + xl; o2 = yl * W + xh; o3 = yh * W + xl; o4 = yh * W + xh;
  return true;
}

// grid (R, PH); 256 threads stride over (pw, c), c fastest
template <typename T>
__global__ void __launch_bounds__(256)
roi_align_fwd_kernel(Levels lv, const float* __restrict__ rois, const int* __restrict__ levels,
                     T* __restrict__ out, int C, int PH, int PW, int sampling, int aligned) {
  const int r = blockIdx.x, ph = blockIdx.y;
  const float* roi = rois + (int64_t)r * 5;
  const int l = levels ? levels[r] : 0;
  const int H = lv.H[l], W = lv.W[l];
  const int b = (int)roi[0];
  const T* x = (const T*)lv.x[l] + (int64_t)b * H * W * C;
  const RoiGeom g = roi_geom(roi, lv.scale[l], PH, PW, sampling, aligned);
  T* o = out + ((int64_t)r * PH + ph) * PW * C;
  for (int e = threadIdx.x; e < PW * C; e += blockDim.x) {
    const int pw = e / C, c = e - pw * C;
    float acc = 0.f;
    for (int iy = 0; iy < g.gh; ++iy) {
      const float y = g.y1 + ph * g.bh + (iy + 0.5f) * g.bh / g.gh;
      for (int ix = 0; ix < g.gw; ++ix) {
        const float xx = g.x1 + pw * g.bw + (ix + 0.5f) * g.bw / g.gw;
        int o1, o2, o3, o4;
        float w1, w2, w3, w4;
        if (!bilinear(y, xx, H, W, o1, o2, o3, o4, w1, w2, w3, w4)) continue;
        acc += w1 * io<T>::ld(x, (int64_t)o1 * C + c) + w2 * io<T>::ld(x, (int64_t)o2 * C + c) +
               w3 * io<T>::ld(x, (int64_t)o3 * C + c) + w4 * io<T>::ld(x, (int64_t)o4 * C + c);
      }
    }
    io<T>::st(o, e, acc * g.inv_count);
  }
}

// scatter-add of the pooled gradient into fp32 NHWC level buffers
template <typename T>
__global__ void __launch_bounds__(256)
roi_align_bwd_kernel(Levels lv, const float* __restrict__ rois, const int* __restrict__ levels,
                     const T* __restrict__ dout, int C, int PH, int PW, int sampling, int aligned) {
  const int r = blockIdx.x, ph = blockIdx.y;
  const float* roi = rois + (int64_t)r * 5;
  const int l = levels ? levels[r] : 0;
  const int H = lv.H[l], W = lv.W[l];
  const int b = (int)roi[0];
  float* dx = (float*)lv.x[l] + (int64_t)b * H * W * C;
  const RoiGeom g = roi_geom(roi, lv.scale[l], PH, PW, sampling, aligned);
  const T* d = dout + ((int64_t)r * PH + ph) * PW * C;
  for (int e = threadIdx.x; e < PW * C; e += blockDim.x) {
    const int pw = e / C, c = e - pw * C;
    const float gv = io<T>::ld(d, e) * g.inv_count;
    if (gv == 0.f) continue;
    for (int iy = 0; iy < g.gh; ++iy) {
      const float y = g.y1 + ph * g.bh + (iy + 0.5f) * g.bh / g.gh;
      for (int ix = 0; ix < g.gw; ++ix) {
        const float xx = g.x1 + pw * g.bw + (ix + 0.5f) * g.bw / g.gw;
        int o1, o2, o3, o4;
        float w1, w2, w3, w4;
        if (!bilinear(y, xx, H, W, o1, o2, o3, o4, w1, w2, w3, w4)) continue;
        atomicAdd(dx + (int64_t)o1 * C + c, gv * w1);
        atomicAdd(dx + (int64_t)o2 * C + c, gv * w2);
        atomicAdd(dx + (int64_t)o3 * C + c, gv * w3);
        atomicAdd(dx + (int64_t)o4 * C + c, gv * w4);
      }
    }
  }
}

// mask[i, blk] bit j: IoU(box i, box blk*64+j) > thr, j > i.  Boxes sorted by
// score.  Grid (col blocks, row blocks), one wave per block.
__global__ void __launch_bounds__(64)
nms_mask_kernel(const float* __restrict__ boxes, int n, float thr,
                unsigned long long* __restrict__ mask, int nblk) {
  const int rb = blockIdx.y, cb = blockIdx.x;
  const int lane = threadIdx.x;
  const int ri = rb * 64 + lane;
  if (cb < rb) {  // strictly-lower blocks are never read; keep them defined
    if (ri < n) mask[(int64_t)ri * nblk + cb] = 0ull;
    return;
  }
  __shared__ float rows[64][4];
  if (ri < n) {
    const float4 bx = *(const float4*)(boxes + (int64_t)ri * 4);
    rows[lane][0] = bx.x; rows[lane][1] = bx.y; rows[lane][2] = bx.z; rows[lane][3] = bx.w;
  }
  __syncthreads();
  const int j = cb * 64 + lane;
  float4 cbx = make_float4(0.f, 0.f, 0.f, 0.f);
  if (j < n) cbx = *(const float4*)(boxes + (int64_t)j * 4);
  const float carea = (cbx.z - cbx.x) * (cbx.w - cbx.y);
  const int nrows = min(64, n - rb * 64);
  unsigned long long mine = 0ull;
  for (int t = 0; t < nrows; ++t) {
    const int i = rb * 64 + t;
    const float x1 = rows[t][0], y1 = rows[t][1], x2 = rows[t][2], y2 = rows[t][3];
    const float iw = fminf(x2, cbx.z) - fmaxf(x1, cbx.x);
    const float ih = fminf(y2, cbx.w) - fmaxf(y1, cbx.y);
    const float inter = fmaxf(iw, 0.f) * fmaxf(ih, 0.f);
    const float uni = (x2 - x1) * (y2 - y1) + carea - inter;
    const bool sup = (j < n) && (j > i) && inter > 0.f && inter > thr * uni;
    const unsigned long long word = __ballot(sup);
    if (lane == t) mine = word;
  }
  if (ri < n) mask[(int64_t)ri * nblk + cb] = mine;
}

// greedy scan in one wave: lane w owns removed-words w, w+64, ...
__global__ void __launch_bounds__(64)
nms_reduce_kernel(const unsigned long long* __restrict__ mask, int n, int nblk, int max_keep,
                  uint8_t* __restrict__ keep, int* __restrict__ count) {
  extern __shared__ unsigned long long removed[];
  const int lane = threadIdx.x;
  for (int w = lane; w < nblk; w += 64) removed[w] = 0ull;
  for (int i = lane; i < n; i += 64) keep[i] = 0;
  __syncthreads();
  int kept = 0;
  for (int i = 0; i < n; ++i) {
    const bool rem = (removed[i >> 6] >> (i & 63)) & 1ull;
    if (rem) continue;
    if (kept >= max_keep) break;
    ++kept;
    if (lane == 0) keep[i] = 1;
    const unsigned long long* row = mask + (int64_t)i * nblk;
    for (int w = (i >> 6) + lane; w < nblk; w += 64) removed[w] |= row[w];
    __syncthreads();
  }
  if (lane == 0) *count = kept;
}

}  // namespace

// x_ptrs / dims / scales are HOST arrays (nlev entries; dims = H,W pairs).
// levels: device int32 [R] (nullptr when nlev == 1).  out: NHWC [R, PH, PW, C].
MDA_API int mda_roi_align_fwd(int64_t dt, int64_t nlev, const int64_t* x_ptrs, const int64_t* dims,
                              const float* scales, const float* rois, const int* levels, void* out,
                              int64_t R, int64_t C, int64_t PH, int64_t PW, int64_t sampling,
                              int64_t aligned, hipStream_t st) {
  if (nlev < 1 || nlev > MAXLEV) return (int)hipErrorInvalidValue;
  if (R == 0) return 0;
  Levels lv{};
  for (int l = 0; l < nlev; ++l) {
    lv.x[l] = (const void*)x_ptrs[l];
    lv.H[l] = (int)dims[2 * l];
    lv.W[l] = (int)dims[2 * l + 1];
    lv.scale[l] = scales[l];
  }
  dim3 grid((unsigned)R, (unsigned)PH);
  if (dt == DT_F32)
    hipLaunchKernelGGL(roi_align_fwd_kernel<float>, grid, dim3(256), 0, st, lv, rois, levels,
                       (float*)out, (int)C, (int)PH, (int)PW, (int)sampling, (int)aligned);
  else
    hipLaunchKernelGGL(roi_align_fwd_kernel<bf16_t>, grid, dim3(256), 0, st, lv, rois, levels,
                       (bf16_t*)out, (int)C, (int)PH, (int)PW, (int)sampling, (int)aligned);
  MDA_CHECK_LAUNCH();
}

// dx_ptrs: fp32 NHWC gradient buffers per level (zeroed by the caller).
MDA_API int mda_roi_align_bwd(int64_t dt, int64_t nlev, const int64_t* dx_ptrs, const int64_t* dims,
                              const float* scales, const float* rois, const int* levels,
                              const void* dout, int64_t R, int64_t C, int64_t PH, int64_t PW,
                              int64_t sampling, int64_t aligned, hipStream_t st) {
  if (nlev < 1 || nlev > MAXLEV) return (int)hipErrorInvalidValue;
  if (R == 0) return 0;
  Levels lv{};
  for (int l = 0; l < nlev; ++l) {
    lv.x[l] = (const void*)dx_ptrs[l];
    lv.H[l] = (int)dims[2 * l];
    lv.W[l] = (int)dims[2 * l + 1];
    lv.scale[l] = scales[l];
  }
  dim3 grid((unsigned)R, (unsigned)PH);
  if (dt == DT_F32)
    hipLaunchKernelGGL(roi_align_bwd_kernel<float>, grid, dim3(256), 0, st, lv, rois, levels,
                       (const float*)dout, (int)C, (int)PH, (int)PW, (int)sampling, (int)aligned);
  else
    hipLaunchKernelGGL(roi_align_bwd_kernel<bf16_t>, grid, dim3(256), 0, st, lv, rois, levels,
                       (const bf16_t*)dout, (int)C, (int)PH, (int)PW, (int)sampling, (int)aligned);
  MDA_CHECK_LAUNCH();
}

// boxes: fp32 [n, 4] sorted by descending score.  mask: u64 [n, ceil(n/64)].
// keep: u8 [n] (1 = kept), count: int32 [1].  At most max_keep boxes are kept.
MDA_API int mda_nms(const float* boxes, int64_t n, float thr, void* mask, int64_t max_keep,
                    uint8_t* keep, int* count, hipStream_t st) {
  if (n <= 0) return (int)hipMemsetAsync(count, 0, sizeof(int), st);
  const int nblk = (int)((n + 63) / 64);
  if ((size_t)nblk * 8 > 64 * 1024) return (int)hipErrorInvalidValue;  // > 512k boxes
  hipLaunchKernelGGL(nms_mask_kernel, dim3(nblk, nblk), dim3(64), 0, st, boxes, (int)n, thr,
                     (unsigned long long*)mask, nblk);
  hipLaunchKernelGGL(nms_reduce_kernel, dim3(1), dim3(64), (size_t)nblk * 8, st,
                     (const unsigned long long*)mask, (int)n, nblk,
                     (int)(max_keep > 0 ? max_keep : n), keep, count);
  MDA_CHECK_LAUNCH();
}
