// f1 — device-side training augmentation of the two-view datasets.
//
// Replaces the host pipeline of DS_mds.__getitem__ (datasets/dataset_mds.py:
// 41-201) per view: fliplr (utils/augment.py:216-227) -> noisy_mean (:261-267)
// -> affine crop/scale/rotate to inpRes (:86-138, skimage resize + rotate) ->
// image_colorNorm (utils/process.py:151-160).  The images stay resident in HBM
// as uint8 BGR [N][H][W][3] (what cv2.imread gives, utils/process.py:86-88);
// one launch writes a whole batch of augmented views as float32 NCHW.
//
// Geometry: output pixel (x, y) samples the flipped, noise-adjusted source at
// M (x, y, 1), M = the reference's pixel chain composed on the host
// (augment.warp_matrix): skimage.resize's pixel centres of the stripped crop,
// the rotation pad, skimage.transform.rotate's inverse map about the padded
// crop's centre, the integer crop corners transform([0,0] / res, invert=1)
// (utils/augment.py:103-137), and the flip (source column W-1-x).  The
// keypoints go through transform() with the same float32 operands on the host
// (utils/augment.py:150-156).  Bilinear sampling (skimage order 1) with zero
// outside the image (skimage's constant 0 padding).  Not reproduced: the
// reference resamples twice (rotate, then resize) where this samples once,
// skimage.resize's Gaussian anti-aliasing when a view is scaled down (<= 25 %
// here) and its reflect-mode edges — skimage is not in this image, so the
// pixels have statistical, not bitwise, parity.
//
// noisy_mean: v' = clamp(alpha * (v - mu) + mu + beta, 0, 1) on the [0,1]
// source pixels with mu the image mean over all channels and pixels
// (ubpl_image_mean_u8); applied to source pixels, before the warp, as the
// reference does (the padding stays 0).  colorNorm: minus the per-channel
// means (RGB-ordered means on BGR channels, the reference's quirk), no std.
//
// Memory: one output float per thread (HBM-write bound: 3 * Ho * Wo * 4 B
// per view); the 4 bilinear taps of 3 channels read a 196 KB source image
// that stays in L2 across the launch.
#include "common.h"

namespace {

__global__ void __launch_bounds__(256) image_mean_kernel(const uint8_t* __restrict__ imgs, int64_t n_per,
                                                         float* __restrict__ out) {
    __shared__ double red[16];
    const uint8_t* p = imgs + (int64_t)blockIdx.x * n_per;
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < n_per; i += blockDim.x) s += (double)p[i];
    s = ubpl::block_sum(s, red);
    if (threadIdx.x == 0) out[blockIdx.x] = (float)(s / (double)n_per / 255.0);
}

__device__ __forceinline__ float tap(const uint8_t* img, int H, int W, int x, int y, int c, float a, float mu,
                                     float b, bool noisy) {
    if (x < 0 || x >= W || y < 0 || y >= H) return 0.f;
    float v = (float)img[((int64_t)y * W + x) * 3 + c] * (1.f / 255.f);
    if (noisy) v = fminf(fmaxf(a * (v - mu) + mu + b, 0.f), 1.f);
    return v;
}

__global__ void __launch_bounds__(256) augment_warp_kernel(const uint8_t* __restrict__ imgs, int H, int W,
                                                           const int* __restrict__ src_idx,
                                                           const float* __restrict__ mat,
                                                           const float* __restrict__ noise,
                                                           const float* __restrict__ img_mean,
                                                           const float* __restrict__ chan_mean, int Ho, int Wo,
                                                           float* __restrict__ out) {
    const int v = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= Ho * Wo) return;
    const int y = p / Wo, x = p - y * Wo;
    const float* m = mat + 6 * v;
    const float sx = m[0] * (float)x + m[1] * (float)y + m[2];
    const float sy = m[3] * (float)x + m[4] * (float)y + m[5];
    const uint8_t* img = imgs + (int64_t)src_idx[v] * H * W * 3;
    const bool noisy = noise[3 * v + 2] > 0.f;
    const float a = noise[3 * v], b = noise[3 * v + 1], mu = img_mean[src_idx[v]];
    const float fx = floorf(sx), fy = floorf(sy);
    const int x0 = (int)fx, y0 = (int)fy;
    const float wx = sx - fx, wy = sy - fy;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float v00 = tap(img, H, W, x0, y0, c, a, mu, b, noisy);
        const float v01 = tap(img, H, W, x0 + 1, y0, c, a, mu, b, noisy);
        const float v10 = tap(img, H, W, x0, y0 + 1, c, a, mu, b, noisy);
        const float v11 = tap(img, H, W, x0 + 1, y0 + 1, c, a, mu, b, noisy);
        const float top = v00 + wx * (v01 - v00), bot = v10 + wx * (v11 - v10);
        out[((int64_t)v * 3 + c) * Ho * Wo + p] = top + wy * (bot - top) - chan_mean[c];
    }
}

}  // namespace

UBPL_API int ubpl_image_mean_u8(const uint8_t* imgs, int N, int64_t n_per_image, float* out, void* stream) {
    if (N <= 0) return 0;
    hipLaunchKernelGGL(image_mean_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, imgs, n_per_image, out);
    UBPL_LAUNCH_CHECK();
    return 0;
}

UBPL_API int ubpl_augment_warp(const uint8_t* imgs, int H, int W, const int* src_idx, const float* mat,
                               const float* noise, const float* img_mean, const float* chan_mean, int V, int Ho,
                               int Wo, float* out, void* stream) {
    if (V <= 0) return 0;
    if (H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0) return (int)hipErrorInvalidValue;
    dim3 grid((Ho * Wo + 255) / 256, V);
    hipLaunchKernelGGL(augment_warp_kernel, grid, dim3(256), 0, (hipStream_t)stream, imgs, H, W, src_idx, mat, noise,
                       img_mean, chan_mean, Ho, Wo, out);
    UBPL_LAUNCH_CHECK();
    return 0;
}
