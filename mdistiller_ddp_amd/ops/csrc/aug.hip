// Device-side CIFAR-style augmentation over a device-resident uint8 dataset
// (survey K16): gather the batch rows, RandomCrop(32, padding=4) with zero
// padding, RandomHorizontalFlip, ToTensor (/255) and Normalize, written as
// channels-last (NHWC) fp32 or bf16 -- the layout the conv kernels read.
// The whole CIFAR-100 train set is 150 MB of HBM; with this kernel the data
// pipeline never touches the host (the reference decodes PIL images in
// CPU workers, and its NUM_WORKERS //= world_size drops to 0 workers at
// world >= 3).
#include "common.h"

namespace {

template <typename TO>
__global__ void __launch_bounds__(256)
crop_flip_norm_kernel(const uint8_t* __restrict__ data, const int64_t* __restrict__ idx,
                      const int32_t* __restrict__ offs, const uint8_t* __restrict__ flip,
                      const float* __restrict__ mean, const float* __restrict__ inv_std,
                      TO* __restrict__ out, int B, int H, int W, int C, int pad) {
  const int64_t total = (int64_t)B * H * W;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(p / (H * W));
    const int r = (int)(p - (int64_t)b * H * W);
    const int y = r / W, x = r - (r / W) * W;
    const int xs = flip[b] ? (W - 1 - x) : x;
    const int sy = y + offs[2 * b] - pad, sx = xs + offs[2 * b + 1] - pad;
    const bool ok = (unsigned)sy < (unsigned)H && (unsigned)sx < (unsigned)W;
    const uint8_t* src = data + ((idx[b] * H + (ok ? sy : 0)) * W + (ok ? sx : 0)) * C;
    TO* dst = out + p * C;
    for (int c = 0; c < C; ++c) {
      float v = ok ? src[c] * (1.f / 255.f) : 0.f;
      io<TO>::st(dst, c, (v - mean[c]) * inv_std[c]);
    }
  }
}

}  // namespace

// data [N, H, W, C] uint8; idx [B]; offs [B, 2] int32 in [0, 2*pad]; flip [B] uint8;
// out [B, H, W, C] (NHWC) fp32 (dt 0) or bf16 (dt 1).
MDA_API int mda_crop_flip_norm(const uint8_t* data, const int64_t* idx, const int32_t* offs,
                               const uint8_t* flip, const float* mean, const float* inv_std,
                               void* out, int64_t dt, int64_t B, int64_t H, int64_t W, int64_t C,
                               int64_t pad, hipStream_t st) {
  int64_t total = B * H * W;
  int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
  if (dt == DT_F32)
    hipLaunchKernelGGL(crop_flip_norm_kernel<float>, dim3(blocks), dim3(256), 0, st, data, idx,
                       offs, flip, mean, inv_std, (float*)out, (int)B, (int)H, (int)W, (int)C, (int)pad);
  else
    hipLaunchKernelGGL(crop_flip_norm_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, data, idx,
                       offs, flip, mean, inv_std, (bf16_t*)out, (int)B, (int)H, (int)W, (int)C, (int)pad);
  MDA_CHECK_LAUNCH();
}
