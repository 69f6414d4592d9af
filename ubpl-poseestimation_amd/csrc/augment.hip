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

// The reference's two resamplings (utils/augment.py:119-137), ubpl_augment_chain.
// Stage 1 — skimage.transform.rotate (scikit-image 0.20: order 1, mode
// 'constant' 0, clip) of the padded integer crop, pad stripped: stripped pixel
// (r, c) is padded pixel (R, C) = (r + pad, c + pad), which samples the padded
// crop at s = Rot(angle) ((C, R) - ctr) + ctr, ctr = (Wp/2 - 0.5, Hp/2 - 0.5),
// bilinear between the floor and ceil neighbours; a neighbour outside the
// padded crop, or inside it but outside the (flipped) image, reads 0.  Bilinear
// weights are a convex combination, so rotate's clip to the crop's range is
// the identity.  geo int [V][8] = (src, flip, ul_x, ul_y, Hp, Wp, Hc, Wc),
// cs [V][2] = (cos, sin) of the angle (1, 0 and pad 0 when it is 0).
__global__ void __launch_bounds__(256) augment_rotate_kernel(const uint8_t* __restrict__ imgs, int H, int W,
                                                             const int* __restrict__ geo,
                                                             const float* __restrict__ cs,
                                                             const float* __restrict__ noise,
                                                             const float* __restrict__ img_mean, int Hm, int Wm,
                                                             float* __restrict__ inter) {
    const int v = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const int* g = geo + 8 * v;
    const int src = g[0], flip = g[1], ulx = g[2], uly = g[3], Hp = g[4], Wp = g[5], Hc = g[6], Wc = g[7];
    if (p >= Hc * Wc) return;
    const int r = p / Wc, c = p - r * Wc;
    const int pad = (Hp - Hc) >> 1;
    const float R = (float)(r + pad), C = (float)(c + pad);
    const float cx = 0.5f * (float)Wp - 0.5f, cy = 0.5f * (float)Hp - 0.5f;
    const float co = cs[2 * v], si = cs[2 * v + 1];
    const float sx = co * (C - cx) - si * (R - cy) + cx;
    const float sy = si * (C - cx) + co * (R - cy) + cy;
    const float fx = floorf(sx), fy = floorf(sy);
    const int x0 = (int)fx, y0 = (int)fy, x1 = (int)ceilf(sx), y1 = (int)ceilf(sy);
    const float dx = sx - fx, dy = sy - fy;
    const uint8_t* img = imgs + (int64_t)src * H * W * 3;
    const bool noisy = noise[3 * v + 2] > 0.f;
    const float a = noise[3 * v], b = noise[3 * v + 1], mu = img_mean[src];
    // padded-crop pixel (y, x) -> the flipped image's (y + uly, x + ulx); 0 outside either
    auto px = [&](int y, int x, int ch) -> float {
        if (x < 0 || x >= Wp || y < 0 || y >= Hp) return 0.f;
        const int iy = y + uly, ix = x + ulx;
        return tap(img, H, W, flip ? W - 1 - ix : ix, iy, ch, a, mu, b, noisy);   // (tap: 0 outside)
    };
    const int64_t plane = (int64_t)Hm * Wm;
    float* o = inter + (int64_t)v * 3 * plane + (int64_t)r * Wm + c;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        const float top = (1.f - dx) * px(y0, x0, ch) + dx * px(y0, x1, ch);
        const float bot = (1.f - dx) * px(y1, x0, ch) + dx * px(y1, x1, ch);
        o[ch * plane] = (1.f - dy) * top + dy * bot;
    }
}

// Stage 2 — skimage.transform.resize of the Hc x Wc stage-1 image to Ho x Wo
// (scikit-image 0.20: a Gaussian of sigma = max(0, (in/out - 1) / 2) when the
// axis shrinks, then scipy.ndimage.zoom(order=1, mode='mirror',
// grid_mode=True), clip).  The loaders' crops are at most 1.25 * 256 = 320
// pixels: sigma <= 0.125, radius int(4 sigma + 0.5) <= 1 with a neighbour weight
// exp(-32) = 1.3e-14 — the identity in f32, not applied.  Output pixel (i, j)
// samples ((j + 0.5) Wc/Wo - 0.5, (i + 0.5) Hc/Ho - 0.5), bilinear, an index
// past either edge mirrored (-1 -> 1, n -> n - 2); convex weights: clip is the
// identity.  Minus chan_mean (colorNorm).
__device__ __forceinline__ int mirror_idx(int i, int n) {
    if (n == 1) return 0;
    return i < 0 ? -i : (i >= n ? 2 * (n - 1) - i : i);
}

__global__ void __launch_bounds__(256) augment_resize_kernel(const float* __restrict__ inter,
                                                             const int* __restrict__ geo, int Hm, int Wm,
                                                             const float* __restrict__ chan_mean, int Ho, int Wo,
                                                             float* __restrict__ out) {
    const int v = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= Ho * Wo) return;
    const int i = p / Wo, j = p - i * Wo;
    const int Hc = geo[8 * v + 6], Wc = geo[8 * v + 7];
    const float sy = ((float)i + 0.5f) * ((float)Hc / (float)Ho) - 0.5f;
    const float sx = ((float)j + 0.5f) * ((float)Wc / (float)Wo) - 0.5f;
    const float fy = floorf(sy), fx = floorf(sx);
    const float wy = sy - fy, wx = sx - fx;
    const int y0 = mirror_idx((int)fy, Hc), y1 = mirror_idx((int)fy + 1, Hc);
    const int x0 = mirror_idx((int)fx, Wc), x1 = mirror_idx((int)fx + 1, Wc);
    const int64_t plane = (int64_t)Hm * Wm;
    const float* s = inter + (int64_t)v * 3 * plane;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        const float* q = s + ch * plane;
        const float top = (1.f - wx) * q[(int64_t)y0 * Wm + x0] + wx * q[(int64_t)y0 * Wm + x1];
        const float bot = (1.f - wx) * q[(int64_t)y1 * Wm + x0] + wx * q[(int64_t)y1 * Wm + x1];
        out[((int64_t)v * 3 + ch) * Ho * Wo + p] = (1.f - wy) * top + wy * bot - chan_mean[ch];
    }
}

// Random occlusion (utils/udaap/utils_augment.py:21-25,116-163: augment_occlu ->
// occlude_with_objects -> resize_by_factor + paste_over) on views already in
// HBM.  An occluder bank: RGBA float [h][w][4] images (values in [0,1]) packed
// at bank + off[o], sizes hw[2o] = h, hw[2o+1] = w.  A paste (one int row of
// PASTE_INTS): view, occluder, resized w1 / h1, destination rectangle
// [x0, x1) x [y0, y1), source start (sx0, sy0) in the resized occluder — the
// host draws them with the reference's RNG calls and paste_over's clipping.
// The resize is cv2.INTER_AREA's pixel-area relation (factors 0.2-0.8 are
// downscales): resized pixel (rx, ry) averages the original over
// [rx*w/w1, (rx+1)*w/w1) x [ry*h/h1, (ry+1)*h/h1) with fractional-overlap
// weights.  The blend alpha*color + (1-alpha)*dst is applied to the colorNorm'ed
// view (out = v - m): alpha*(color - m) + (1-alpha)*(v - m) is the same image
// normalised after the paste.  Each output pixel walks its view's pastes in
// draw order (later pastes over earlier ones), so a launch is deterministic.
constexpr int PASTE_INTS = 9;

__global__ void __launch_bounds__(256) occlude_kernel(float* __restrict__ out, int H, int W,
                                                      const float* __restrict__ bank,
                                                      const int64_t* __restrict__ off, const int* __restrict__ hw,
                                                      const int* __restrict__ pastes,
                                                      const int* __restrict__ view_first,
                                                      const float* __restrict__ chan_mean) {
    const int v = blockIdx.y;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= H * W) return;
    const int y = p / W, x = p - y * W;
    const int q0 = view_first[v], q1 = view_first[v + 1];
    if (q0 == q1) return;
    float* o = out + (int64_t)v * 3 * H * W + p;
    float px[3] = {o[0], o[(int64_t)H * W], o[2 * (int64_t)H * W]};
    bool hit = false;
    for (int q = q0; q < q1; ++q) {
        const int* pr = pastes + (int64_t)q * PASTE_INTS;
        const int x0 = pr[4], y0 = pr[5], x1 = pr[6], y1 = pr[7];
        if (x < x0 || x >= x1 || y < y0 || y >= y1) continue;
        const int oc = pr[1], w1 = pr[2], h1 = pr[3];
        const int sx0 = pr[8] & 0xFFFF, sy0 = pr[8] >> 16;
        const int h = hw[2 * oc], w = hw[2 * oc + 1];
        const float* src = bank + off[oc];
        const int rx = sx0 + (x - x0), ry = sy0 + (y - y0);
        const float fx = (float)w / (float)w1, fy = (float)h / (float)h1;
        const float ax0 = rx * fx, ax1 = (rx + 1) * fx, ay0 = ry * fy, ay1 = (ry + 1) * fy;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        for (int sy = (int)ay0; sy < h && (float)sy < ay1; ++sy) {
            const float wy = fminf(ay1, (float)(sy + 1)) - fmaxf(ay0, (float)sy);
            for (int sx = (int)ax0; sx < w && (float)sx < ax1; ++sx) {
                const float wgt = wy * (fminf(ax1, (float)(sx + 1)) - fmaxf(ax0, (float)sx));
                const float4 c = *reinterpret_cast<const float4*>(src + ((int64_t)sy * w + sx) * 4);
                acc[0] += wgt * c.x;
                acc[1] += wgt * c.y;
                acc[2] += wgt * c.z;
                acc[3] += wgt * c.w;
            }
        }
        const float inv = 1.f / (fx * fy);
        const float a = acc[3] * inv;
#pragma unroll
        for (int c = 0; c < 3; ++c) px[c] = a * (acc[c] * inv - chan_mean[c]) + (1.f - a) * px[c];
        hit = true;
    }
    if (!hit) return;
    o[0] = px[0];
    o[(int64_t)H * W] = px[1];
    o[2 * (int64_t)H * W] = px[2];
}

}  // namespace

UBPL_API int ubpl_occlude(float* out, int V, int H, int W, const float* bank, const int64_t* off, const int* hw,
                          const int* pastes, const int* view_first, const float* chan_mean, void* stream) {
    if (V <= 0 || H <= 0 || W <= 0) return V < 0 ? (int)hipErrorInvalidValue : 0;
    if ((((uintptr_t)bank) & 15) != 0) return (int)hipErrorInvalidValue;
    dim3 grid((H * W + 255) / 256, V);
    hipLaunchKernelGGL(occlude_kernel, grid, dim3(256), 0, (hipStream_t)stream, out, H, W, bank, off, hw, pastes,
                       view_first, chan_mean);
    UBPL_LAUNCH_CHECK();
    return 0;
}

UBPL_API int ubpl_augment_chain(const uint8_t* imgs, int H, int W, const int* geo, const float* cs,
                               const float* noise, const float* img_mean, const float* chan_mean, int V, int Hm,
                               int Wm, float* inter, int Ho, int Wo, float* out, void* stream) {
    if (V <= 0 || Ho <= 0 || Wo <= 0) return V < 0 ? (int)hipErrorInvalidValue : 0;
    if (Hm <= 0 || Wm <= 0) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(augment_rotate_kernel, dim3((Hm * Wm + 255) / 256, V), dim3(256), 0, (hipStream_t)stream,
                       imgs, H, W, geo, cs, noise, img_mean, Hm, Wm, inter);
    UBPL_LAUNCH_CHECK();
    hipLaunchKernelGGL(augment_resize_kernel, dim3((Ho * Wo + 255) / 256, V), dim3(256), 0, (hipStream_t)stream,
                       inter, geo, Hm, Wm, chan_mean, Ho, Wo, out);
    UBPL_LAUNCH_CHECK();
    return 0;
}

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
