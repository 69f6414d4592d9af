// R1 — per-keypoint Gaussian heatmap targets.
//
// Replaces ProcessUtils.kps_heatmap / kps_heatmap_mulKps / heatmap_gaussian
// (utils/process.py:252-318, 393-397), which the reference runs on the host
// inside DataLoader.__getitem__, one sample at a time.  Here one workgroup
// renders one (sample, keypoint) map straight into HBM.
//
// Arithmetic is the reference's: visibility from the int32-truncated keypoint
// (float32 ul/br), centre = trunc(kp) / stride in float64, value
// exp(-D2 / 2 / sigma / sigma) in float64, >1 -> 1, <cutoff -> 0, stored as
// float32.  Outside the cutoff radius the value is provably below the cutoff,
// so the exp is skipped there (the write stays).
#include "common.h"

namespace {

__global__ void __launch_bounds__(256) render_kernel(const float* __restrict__ kps, float* __restrict__ hm,
                                                     float* __restrict__ kps_out, int K, int img_h, int img_w,
                                                     double stride, int size_h, int size_w, float sig,
                                                     double cutoff, double d2_skip) {
    const int map = blockIdx.x;  // n * K + k
    const float* kp = kps + (int64_t)map * 3;
    const float kx = kp[0], ky = kp[1];
    const int ix = (int)kx, iy = (int)ky;  // torch .to(int32): truncation
    if (threadIdx.x == 0 && kps_out != nullptr) {
        const int ul0 = (int)((float)ix - sig), ul1 = (int)((float)iy - sig);
        const int br0 = (int)((float)ix + sig + 1.0f), br1 = (int)((float)iy + sig + 1.0f);
        const int vis = (br0 >= img_w || br1 >= img_h || ul0 < 0 || ul1 < 0) ? 0 : 1;
        kps_out[(int64_t)map * 3 + 0] = kx;
        kps_out[(int64_t)map * 3 + 1] = ky;
        kps_out[(int64_t)map * 3 + 2] = kp[2] * (float)vis;
    }
    const double cx = (double)ix * 1.0 / stride;
    const double cy = (double)iy * 1.0 / stride;
    const double s = (double)sig;
    float* out = hm + (int64_t)map * size_h * size_w;
    const int npix = size_h * size_w;
    for (int p = threadIdx.x; p < npix; p += blockDim.x) {
        const int gy = p / size_w, gx = p - gy * size_w;
        const double dx = (double)gx - cx, dy = (double)gy - cy;
        const double d2 = dx * dx + dy * dy;
        float v = 0.0f;
        if (d2 <= d2_skip) {
            double e = exp(-d2 / 2.0 / s / s);
            if (e > 1.0) e = 1.0;
            if (e < cutoff) e = 0.0;
            v = (float)e;
        }
        out[p] = v;
    }
}

}  // namespace

// kps [N,K,3] f32 (x, y, vis) in input-image pixels; hm [N,K,size_h,size_w];
// kps_out [N,K,3] receives kps with vis *= visible (may alias kps).
UBPL_API int ubpl_render_heatmaps(const float* kps, float* hm, float* kps_out, int N, int K, int img_h,
                                  int img_w, int inp_res, int out_res, float kernel_size, float sigma,
                                  float cutoff, void* stream) {
    if (N <= 0 || K <= 0) return 0;
    const double stride = (double)inp_res / (double)out_res;
    const int size_h = (int)(img_h / stride), size_w = (int)(img_w / stride);
    const float sig = sigma * kernel_size;
    // exp(-d2/(2 s^2)) < cutoff  <=>  d2 > -2 s^2 ln(cutoff); keep a margin so the
    // skipped region is strictly below the cutoff.
    const double d2_skip = cutoff > 0 ? (-2.0 * (double)sig * sig * log((double)cutoff)) * (1.0 + 1e-9) + 1e-9
                                      : 1e300;
    hipLaunchKernelGGL(render_kernel, dim3(N * K), dim3(256), 0, (hipStream_t)stream, kps, hm, kps_out, K,
                       img_h, img_w, stride, size_h, size_w, sig, (double)cutoff, d2_skip);
    UBPL_LAUNCH_CHECK();
    return 0;
}
