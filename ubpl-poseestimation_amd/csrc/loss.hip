// L1-L6 — heatmap MSE / consistency / UBPL pseudo-label mask / FDL.
//
// The reference computes every loss as mean_px((a - t)^2) per (sample, stack,
// keypoint) row, then weights rows (gate, sample weight, confidence mask) and
// counts rows with per-element Python loops over device tensors
// (utils/losses.py:8-286, utils/process.py:381-383) — ~8k host syncs per
// MT_UBPL step.  Here:
//   row_stats  one workgroup per row: sum of squares, max of a, max of the
//              (model-averaged) target, in one HBM pass;
//   finalize   one workgroup per loss: weights, mask, sum and every count on
//              device (no host sync);
//   row_grad   d/da = w_row * g * 2 (a - t) / HW written (or accumulated) in
//              one pass, g read from device memory (autograd's grad_output).
// Row geometry is given by strides so that stack slices ([:, -1]) and teacher
// stacks ([M, B, S, K, R, R]) are consumed in place, without copies.
#include "common.h"

namespace {

struct RowGeom {
    const float* a;
    int64_t a_sb, a_ss;  // a row (b,s,k) at a + b*a_sb + s*a_ss + k*HW
    const float* t;
    int64_t t_sb, t_ss, t_sm;  // target row (b,s,k) = mean over m of t + m*t_sm + b*t_sb + s*t_ss + k*HW
    int M;
};

__device__ __forceinline__ float target_at(const RowGeom& g, const float* trow, int64_t i) {
    float acc = trow[i];
    for (int m = 1; m < g.M; ++m) acc += trow[(int64_t)m * g.t_sm + i];
    return g.M == 1 ? acc : acc / (float)g.M;
}

__global__ void __launch_bounds__(256) row_stats_kernel(RowGeom g, int S, int K, int HW, float* __restrict__ sq_mean,
                                                       float* __restrict__ amax, float* __restrict__ tmax) {
    __shared__ float red[16];
    const int row = blockIdx.x;  // (b*S + s)*K + k
    const int k = row % K, s = (row / K) % S, b = row / (K * S);
    const float* arow = g.a + b * g.a_sb + s * g.a_ss + (int64_t)k * HW;
    const float* trow = g.t + b * g.t_sb + s * g.t_ss + (int64_t)k * HW;
    float sq = 0.f, am = -INFINITY, tm = -INFINITY;
    for (int i = threadIdx.x; i < HW; i += blockDim.x) {
        const float av = arow[i];
        const float tv = target_at(g, trow, i);
        const float d = av - tv;
        sq = fmaf(d, d, sq);
        am = fmaxf(am, av);
        tm = fmaxf(tm, tv);
    }
    sq = ubpl::block_sum(sq, red);
    am = ubpl::block_max(am, red);
    tm = ubpl::block_max(tm, red);
    if (threadIdx.x == 0) {
        sq_mean[row] = sq / (float)HW;
        if (amax) amax[row] = am;
        if (tmax) tmax[row] = tm;
    }
}

__global__ void __launch_bounds__(256) row_grad_kernel(RowGeom g, int S, int K, int HW, const float* __restrict__ w,
                                                      const float* __restrict__ gscale, float extra,
                                                      float* __restrict__ da, int accumulate) {
    const int row = blockIdx.x;
    const float wr = w[row];
    const int k = row % K, s = (row / K) % S, b = row / (K * S);
    const int64_t off = b * g.a_sb + s * g.a_ss + (int64_t)k * HW;
    float* drow = da + off;
    if (wr == 0.f) {  // zero-weight rows still need their gradient written (or left) as 0
        if (!accumulate)
            for (int i = threadIdx.x; i < HW; i += blockDim.x) drow[i] = 0.f;
        return;
    }
    const float c = wr * (gscale ? gscale[0] : 1.f) * extra;
    const float* arow = g.a + off;
    const float* trow = g.t + b * g.t_sb + s * g.t_ss + (int64_t)k * HW;
    for (int i = threadIdx.x; i < HW; i += blockDim.x) {
        const float v = c * (arow[i] - target_at(g, trow, i));
        drow[i] = accumulate ? drow[i] + v : v;
    }
}

// kind 0: MSE / consistency   w = gate? * sw?                     (utils/losses.py:16-53)
// kind 1: teacher-confidence  w = gate? * sw? * [tmax >= thr]     (utils/losses.py:255-286)
// kind 2: UBPL pseudo mask    w = sw * [amax >= thr] * [tmax >= thr]  (utils/losses.py:176-210)
// cnt[0] = S * #{gate > 0}, cnt[1] = n_pseudo = #{pre-mask loss > 0},
// cnt[2] = n_sel = #{mask > 0}, cnt[3] = #{rows with sw > 0}.
__global__ void __launch_bounds__(256) finalize_kernel(int kind, const float* __restrict__ sq_mean,
                                                      const float* __restrict__ amax,
                                                      const float* __restrict__ tmax,
                                                      const float* __restrict__ gate, const float* __restrict__ sw,
                                                      int use_gate, int use_sw, int B, int S, int K, float thr,
                                                      float* __restrict__ out_sum, int* __restrict__ out_cnt,
                                                      float* __restrict__ out_score, float* __restrict__ out_w) {
    __shared__ double dred[16];
    __shared__ int ired[16];
    const int rows = B * S * K;
    double lsum = 0.0;
    int n_pos = 0, n_sel = 0, n_gate = 0;
    for (int r = threadIdx.x; r < rows; r += blockDim.x) {
        const int k = r % K, b = r / (K * S);
        const float gv = gate ? gate[b * K + k] : 1.f;
        const float sv = sw ? sw[b] : 1.f;
        float l = sq_mean[r];
        float m = 1.f;
        if (kind == 2) {
            if (sw) l = l * sv;
            m = (amax[r] >= thr ? 1.f : 0.f) * (tmax[r] >= thr ? 1.f : 0.f);
        } else {
            if (use_gate) l = l * gv;
            if (use_sw && sw) l = l * sv;
            if (kind == 1) m = tmax[r] >= thr ? 1.f : 0.f;
        }
        n_pos += l > 0.f;
        n_sel += m > 0.f;
        lsum += (double)(l * m);
        float wv = m;
        if (kind == 2) {
            if (sw) wv *= sv;
        } else {
            if (use_gate) wv *= gv;
            if (use_sw && sw) wv *= sv;
        }
        out_w[r] = wv;
    }
    for (int r = threadIdx.x; r < B * K; r += blockDim.x) n_gate += (gate ? gate[r] : 1.f) > 0.f;
    lsum = ubpl::block_sum(lsum, dred);
    n_pos = ubpl::block_sum(n_pos, ired);
    n_sel = ubpl::block_sum(n_sel, ired);
    n_gate = ubpl::block_sum(n_gate, ired);
    int n_rows = 0;
    for (int b = 0; b < B; ++b) n_rows += (sw ? sw[b] : 1.f) > 0.f;
    if (threadIdx.x == 0) {
        out_sum[0] = (float)lsum;
        out_cnt[0] = S * n_gate;
        out_cnt[1] = n_pos;
        out_cnt[2] = n_sel;
        out_cnt[3] = n_rows;
    }
    // per-keypoint confidence score over rows with sw > 0 (utils/losses.py:196-208, :275-285)
    if (out_score != nullptr && kind != 0) {
        for (int k = threadIdx.x; k < K; k += blockDim.x) {
            float acc_s = 0.f;
            for (int s = 0; s < S; ++s) {
                float sa = 0.f, st = 0.f;
                for (int b = 0; b < B; ++b) {
                    if ((sw ? sw[b] : 1.f) > 0.f) {
                        const int r = (b * S + s) * K + k;
                        if (kind == 2) sa += amax[r];
                        st += tmax[r];
                    }
                }
                const float ma = n_rows > 0 ? sa / (float)n_rows : 0.f;
                const float mt = n_rows > 0 ? st / (float)n_rows : 0.f;
                acc_s += kind == 2 ? (ma + mt) / 2.f : mt;
            }
            out_score[k] = acc_s / (float)S;
        }
    }
}

// ---------------------------------------------------------------- FDL (L5)
// Per (b, s, c) row of two feature maps: centred means and the unbiased
// covariance (utils/process.py:18-31); rows whose sample is not selected
// (rowmask[b] <= 0) produce cov = 0 and are excluded downstream.
__global__ void __launch_bounds__(256) cov_rows_kernel(const float* __restrict__ f1, const float* __restrict__ f2,
                                                      const float* __restrict__ rowmask, int S, int C, int HW,
                                                      float* __restrict__ cov, float* __restrict__ mu1,
                                                      float* __restrict__ mu2) {
    __shared__ float red[16];
    const int row = blockIdx.x;  // (b*S + s)*C + c
    const int b = row / (S * C);
    if (rowmask && !(rowmask[b] > 0.f)) {
        if (threadIdx.x == 0) cov[row] = mu1[row] = mu2[row] = 0.f;
        return;
    }
    const float* x = f1 + (int64_t)row * HW;
    const float* y = f2 + (int64_t)row * HW;
    float sx = 0.f, sy = 0.f;
    for (int i = threadIdx.x; i < HW; i += blockDim.x) {
        sx += x[i];
        sy += y[i];
    }
    const float mx = ubpl::block_sum(sx, red) / (float)HW;
    const float my = ubpl::block_sum(sy, red) / (float)HW;
    float sxy = 0.f;
    for (int i = threadIdx.x; i < HW; i += blockDim.x) sxy = fmaf(x[i] - mx, y[i] - my, sxy);
    sxy = ubpl::block_sum(sxy, red);
    if (threadIdx.x == 0) {
        cov[row] = sxy / (float)(HW - 1);
        mu1[row] = mx;
        mu2[row] = my;
    }
}

__global__ void __launch_bounds__(256) cov_finalize_kernel(const float* __restrict__ cov,
                                                          const float* __restrict__ rowmask, int B, int S, int C,
                                                          float* __restrict__ out_val, int* __restrict__ out_cnt) {
    __shared__ double dred[16];
    double acc = 0.0;
    int nsel = 0;
    for (int b = 0; b < B; ++b) nsel += (rowmask ? rowmask[b] : 1.f) > 0.f;
    const int rows = B * S * C;
    for (int r = threadIdx.x; r < rows; r += blockDim.x) {
        const int b = r / (S * C);
        if (!rowmask || rowmask[b] > 0.f) acc += fabs((double)cov[r]);
    }
    acc = ubpl::block_sum(acc, dred);
    if (threadIdx.x == 0) {
        const int n = nsel * S * C;
        out_val[0] = n > 0 ? (float)(acc / (double)n) : NAN;
        out_cnt[0] = n;
    }
}

__global__ void __launch_bounds__(256) cov_grad_kernel(const float* __restrict__ f1, const float* __restrict__ f2,
                                                      const float* __restrict__ rowmask,
                                                      const float* __restrict__ cov, const float* __restrict__ mu1,
                                                      const float* __restrict__ mu2, const int* __restrict__ cnt,
                                                      const float* __restrict__ gscale, int S, int C, int HW,
                                                      float* __restrict__ d1, float* __restrict__ d2, int accumulate) {
    const int row = blockIdx.x;
    const int b = row / (S * C);
    const int64_t off = (int64_t)row * HW;
    const bool on = !rowmask || rowmask[b] > 0.f;
    const float cv = cov[row];
    const float sgn = (cv > 0.f) ? 1.f : ((cv < 0.f) ? -1.f : 0.f);
    const int n = cnt[0];
    const float c = on && n > 0 ? (gscale ? gscale[0] : 1.f) * sgn / (float)n / (float)(HW - 1) : 0.f;
    const float m1 = mu1[row], m2 = mu2[row];
    for (int i = threadIdx.x; i < HW; i += blockDim.x) {
        const float x = f1[off + i], y = f2[off + i];
        const float g1 = c * (y - m2), g2 = c * (x - m1);
        if (d1) d1[off + i] = accumulate ? d1[off + i] + g1 : g1;
        if (d2) d2[off + i] = accumulate ? d2[off + i] + g2 : g2;
    }
}

}  // namespace

UBPL_API int ubpl_heatmap_row_stats(const float* a, int64_t a_sb, int64_t a_ss, const float* t, int64_t t_sb,
                                    int64_t t_ss, int64_t t_sm, int M, int B, int S, int K, int HW, float* sq_mean,
                                    float* amax, float* tmax, void* stream) {
    if (B * S * K == 0) return 0;
    RowGeom g{a, a_sb, a_ss, t, t_sb, t_ss, t_sm, M};
    hipLaunchKernelGGL(row_stats_kernel, dim3(B * S * K), dim3(256), 0, (hipStream_t)stream, g, S, K, HW, sq_mean,
                       amax, tmax);
    UBPL_LAUNCH_CHECK();
    return 0;
}

UBPL_API int ubpl_heatmap_row_grad(const float* a, int64_t a_sb, int64_t a_ss, const float* t, int64_t t_sb,
                                   int64_t t_ss, int64_t t_sm, int M, int B, int S, int K, int HW, const float* w,
                                   const float* gscale, float extra, float* da, int accumulate, void* stream) {
    if (B * S * K == 0) return 0;
    RowGeom g{a, a_sb, a_ss, t, t_sb, t_ss, t_sm, M};
    hipLaunchKernelGGL(row_grad_kernel, dim3(B * S * K), dim3(256), 0, (hipStream_t)stream, g, S, K, HW, w, gscale,
                       extra, da, accumulate);
    UBPL_LAUNCH_CHECK();
    return 0;
}

UBPL_API int ubpl_loss_finalize(int kind, const float* sq_mean, const float* amax, const float* tmax,
                                const float* gate, const float* sw, int use_gate, int use_sw, int B, int S, int K,
                                float thr, float* out_sum, int* out_cnt, float* out_score, float* out_w,
                                void* stream) {
    hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, kind, sq_mean, amax, tmax, gate,
                       sw, use_gate, use_sw, B, S, K, thr, out_sum, out_cnt, out_score, out_w);
    UBPL_LAUNCH_CHECK();
    return 0;
}

UBPL_API int ubpl_fdl_cov_forward(const float* f1, const float* f2, const float* rowmask, int B, int S, int C,
                                  int HW, float* cov, float* mu1, float* mu2, float* out_val, int* out_cnt,
                                  void* stream) {
    if (B * S * C == 0) return 0;
    hipLaunchKernelGGL(cov_rows_kernel, dim3(B * S * C), dim3(256), 0, (hipStream_t)stream, f1, f2, rowmask, S, C,
                       HW, cov, mu1, mu2);
    UBPL_LAUNCH_CHECK();
    hipLaunchKernelGGL(cov_finalize_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, cov, rowmask, B, S, C,
                       out_val, out_cnt);
    UBPL_LAUNCH_CHECK();
    return 0;
}

UBPL_API int ubpl_fdl_cov_backward(const float* f1, const float* f2, const float* rowmask, const float* cov,
                                   const float* mu1, const float* mu2, const int* cnt, const float* gscale, int B,
                                   int S, int C, int HW, float* d1, float* d2, int accumulate, void* stream) {
    if (B * S * C == 0) return 0;
    hipLaunchKernelGGL(cov_grad_kernel, dim3(B * S * C), dim3(256), 0, (hipStream_t)stream, f1, f2, rowmask, cov,
                       mu1, mu2, cnt, gscale, S, C, HW, d1, d2, accumulate);
    UBPL_LAUNCH_CHECK();
    return 0;
}
