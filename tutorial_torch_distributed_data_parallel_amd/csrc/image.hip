// On-device image preprocessing: the reference's torchvision chain Resize(224) ->
// RandomHorizontalFlip -> ToTensor -> Normalize(mean, std) (REF/data_and_toy_model.py:8-38), run
// in ONE pass over the uint8 batch the host loader copied to the GPU (csrc/loader.h). One thread
// per output pixel, all channels: reads hit L2 (the 32x32 source is 3 KB per image), the float
// output is written once, coalesced along the output row.
//
// Bilinear with half-pixel centres and edge clamping (torch upsample_bilinear2d,
// align_corners=False), which for upsampling is the triangle filter PIL's Resize applies;
// round_u8 then rounds to the nearest integer like PIL's uint8 output before ToTensor's /255.
#include "common.h"
#include "kernels.h"

namespace tdp {
namespace {

template <int C, bool CL>
__global__ __launch_bounds__(256) void image_transform_kernel(
    const uint8_t* __restrict__ x, const uint8_t* __restrict__ flip, float* __restrict__ out,
    int B, int Hs, int Ws, int Ho, int Wo, float sh, float sw, ImageNorm nrm, int round_u8) {
  const long total = (long)B * Ho * Wo;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int w = (int)(i % Wo);
    const long bh = i / Wo;
    const int h = (int)(bh % Ho);
    const int b = (int)(bh / Ho);
    const int ws = (flip != nullptr && flip[b]) ? Wo - 1 - w : w;
    float fy = fmaxf((h + 0.5f) * sh - 0.5f, 0.f);
    float fx = fmaxf((ws + 0.5f) * sw - 0.5f, 0.f);
    const int y0 = min((int)fy, Hs - 1), x0 = min((int)fx, Ws - 1);
    const int y1 = min(y0 + 1, Hs - 1), x1 = min(x0 + 1, Ws - 1);
    const float ly = fy - y0, lx = fx - x0;
    const uint8_t* img = x + (long)b * Hs * Ws * C;
    const uint8_t* p00 = img + ((long)y0 * Ws + x0) * C;
    const uint8_t* p01 = img + ((long)y0 * Ws + x1) * C;
    const uint8_t* p10 = img + ((long)y1 * Ws + x0) * C;
    const uint8_t* p11 = img + ((long)y1 * Ws + x1) * C;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float top = (float)p00[c] + lx * ((float)p01[c] - (float)p00[c]);
      const float bot = (float)p10[c] + lx * ((float)p11[c] - (float)p10[c]);
      float v = top + ly * (bot - top);
      if (round_u8) v = rintf(v);
      v = (v * (1.f / 255.f) - nrm.mean[c]) * nrm.inv_std[c];
      if (CL) out[i * C + c] = v;                                          // [B][Ho][Wo][C]
      else out[(((long)b * C + c) * Ho + h) * Wo + w] = v;                 // [B][C][Ho][Wo]
    }
  }
}

}  // namespace

template <int C, bool CL>
static void launch_image(const uint8_t* x, const uint8_t* flip, float* out, int B, int Hs, int Ws,
                         int Ho, int Wo, const ImageNorm& nrm, int round_u8, hipStream_t s) {
  const long total = (long)B * Ho * Wo;
  long g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL((image_transform_kernel<C, CL>), dim3((unsigned)g), dim3(256), 0, s, x, flip,
                     out, B, Hs, Ws, Ho, Wo, (float)Hs / (float)Ho, (float)Ws / (float)Wo, nrm,
                     round_u8);
}

void image_transform(const uint8_t* x, const uint8_t* flip, float* out, int B, int Hs, int Ws,
                     int C, int Ho, int Wo, const ImageNorm& nrm, bool round_u8,
                     bool channels_last, hipStream_t s) {
  if ((long)B * Ho * Wo <= 0) return;
  const int r = round_u8 ? 1 : 0;
  if (C == 3) {
    if (channels_last) launch_image<3, true>(x, flip, out, B, Hs, Ws, Ho, Wo, nrm, r, s);
    else launch_image<3, false>(x, flip, out, B, Hs, Ws, Ho, Wo, nrm, r, s);
  } else if (C == 1) {
    if (channels_last) launch_image<1, true>(x, flip, out, B, Hs, Ws, Ho, Wo, nrm, r, s);
    else launch_image<1, false>(x, flip, out, B, Hs, Ws, Ho, Wo, nrm, r, s);
  } else if (C == 4) {
    if (channels_last) launch_image<4, true>(x, flip, out, B, Hs, Ws, Ho, Wo, nrm, r, s);
    else launch_image<4, false>(x, flip, out, B, Hs, Ws, Ho, Wo, nrm, r, s);
  }
}

}  // namespace tdp
