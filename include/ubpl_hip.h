/*
 * ubpl_hip.h — C-ABI of libubpl_hip.so, the MI355X (gfx950) hot path of
 * Qi2019KB/UBPL-PoseEstimation's semi-supervised pose training step.
 *
 * Conventions
 *   - plain pointers to DEVICE memory, sizes as int / int64_t, no torch types;
 *   - every function enqueues on `stream` (a hipStream_t, NULL = default
 *     stream), never synchronises, never allocates: scratch is caller-owned;
 *   - return 0 on success, otherwise a hipError_t code (e.g. 1 =
 *     hipErrorInvalidValue for an unsupported shape);
 *   - layouts are the reference's: NCHW float32 tensors, contiguous.
 *
 * Reference interfaces replaced (paths relative to the reference root) are
 * cited per entry.
 *
 * Argument annotations: the comment `/ *@ name:type[extent] ... * /` right
 * before a declaration gives each pointer argument its element type (f32,
 * f64, i32, i64, u16 = bf16 pieces, u8) and the number of elements the call
 * may touch, as a C expression of the integer arguments ("?" = not derivable
 * from them).  csrc/gen_torch_ops.py turns them into the torch ops' argument
 * checks (dtype, contiguity, storage extent), so a short tensor raises there
 * instead of being written out of bounds.  The Python host layer (ubpl-poseestimation_amd/ubpl_amd)
 * binds these through ctypes and re-exposes the reference's module API.
 */
#ifndef UBPL_HIP_H
#define UBPL_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- R1 ----
 * ProcessUtils.kps_heatmap / kps_heatmap_mulKps (utils/process.py:252-318).
 * kps [N,K,3] (x, y, vis) in image pixels -> hm [N,K,size_h,size_w] with
 * size = int(img / (inp_res/out_res)); kps_out[...,2] = vis * visible
 * (may alias kps: the reference mutates kpsMap in place, :267). */
/*@ kps:f32[N*K*3] hm:f32[(int64_t)N*K*(int)(img_h/((double)inp_res/out_res))*(int)(img_w/((double)inp_res/out_res))] kps_out:f32[N*K*3] */
int ubpl_render_heatmaps(const float* kps, float* hm, float* kps_out, int N, int K, int img_h, int img_w,
                         int inp_res, int out_res, float kernel_size, float sigma, float cutoff, void* stream);

/* ---------------------------------------------------------------- L1-L4 --
 * Row statistics of mean_px((a - t)^2): a row (b,s,k) at a + b*a_sb + s*a_ss + k*HW;
 * target = mean over m < M of t + m*t_sm + b*t_sb + s*t_ss + k*HW.
 * Outputs [B*S*K]: sq_mean; amax = max_px a (nullable); tmax = max_px target (nullable).
 * JointMSELoss / JointDistLoss / JointDistLoss_mt2 / JointPseudoLoss3 forward
 * (utils/losses.py:16-53, 255-286, 176-210). */
/*@ a:f32[(B-1)*a_sb+(S-1)*a_ss+(int64_t)K*HW] t:f32[(M-1)*t_sm+(B-1)*t_sb+(S-1)*t_ss+(int64_t)K*HW] sq_mean:f32[B*S*K] amax:f32[B*S*K] tmax:f32[B*S*K] */
int ubpl_heatmap_row_stats(const float* a, int64_t a_sb, int64_t a_ss, const float* t, int64_t t_sb, int64_t t_ss,
                           int64_t t_sm, int M, int B, int S, int K, int HW, float* sq_mean, float* amax,
                           float* tmax, void* stream);
/* Loss reduction + counts on device.  kind 0 MSE/consistency, 1 teacher-
 * confidence mask (mt2), 2 UBPL pseudo mask.  out_sum[1] f32; out_cnt[4] int32 =
 * {nStack*#gate>0, n_pseudo, n_sel, #rows sw>0}; out_score[K] (kinds 1,2);
 * out_w[B*S*K] per-row weight for the backward. */
/*@ sq_mean:f32[B*S*K] amax:f32[B*S*K] tmax:f32[B*S*K] gate:f32[B*K] sw:f32[B] out_sum:f32[1] out_cnt:i32[4] out_score:f32[K] out_w:f32[B*S*K] */
int ubpl_loss_finalize(int kind, const float* sq_mean, const float* amax, const float* tmax, const float* gate,
                       const float* sw, int use_gate, int use_sw, int B, int S, int K, float thr, float* out_sum,
                       int* out_cnt, float* out_score, float* out_w, void* stream);
/* d a (+)= w_row * (*gscale) * extra * (a - target); gscale device scalar (nullable = 1). */
/*@ a:f32[(B-1)*a_sb+(S-1)*a_ss+(int64_t)K*HW] t:f32[(M-1)*t_sm+(B-1)*t_sb+(S-1)*t_ss+(int64_t)K*HW] w:f32[B*S*K] gscale:f32[1] da:f32[(B-1)*a_sb+(S-1)*a_ss+(int64_t)K*HW] */
int ubpl_heatmap_row_grad(const float* a, int64_t a_sb, int64_t a_ss, const float* t, int64_t t_sb, int64_t t_ss,
                          int64_t t_sm, int M, int B, int S, int K, int HW, const float* w, const float* gscale,
                          float extra, float* da, int accumulate, void* stream);

/* ---------------------------------------------------------------- L5 ----
 * ProcessUtils.features_cov (utils/process.py:18-31) over rows whose
 * rowmask[b] > 0 (the caller's labeled-row selection, projects/MT_UBPL.py:309-320).
 * f1,f2 [B,S,C,HW]; cov/mu1/mu2 [B*S*C] scratch; out_val[1] = mean |cov|;
 * out_cnt[1] = #selected * S * C. */
/*@ f1:f32[(int64_t)B*S*C*HW] f2:f32[(int64_t)B*S*C*HW] rowmask:f32[B] cov:f32[B*S*C] mu1:f32[B*S*C] mu2:f32[B*S*C] out_val:f32[1] out_cnt:i32[1] */
int ubpl_fdl_cov_forward(const float* f1, const float* f2, const float* rowmask, int B, int S, int C, int HW,
                         float* cov, float* mu1, float* mu2, float* out_val, int* out_cnt, void* stream);
/*@ f1:f32[(int64_t)B*S*C*HW] f2:f32[(int64_t)B*S*C*HW] rowmask:f32[B] cov:f32[B*S*C] mu1:f32[B*S*C] mu2:f32[B*S*C] cnt:i32[1] gscale:f32[1] d1:f32[(int64_t)B*S*C*HW] d2:f32[(int64_t)B*S*C*HW] */
int ubpl_fdl_cov_backward(const float* f1, const float* f2, const float* rowmask, const float* cov, const float* mu1,
                          const float* mu2, const int* cnt, const float* gscale, int B, int S, int C, int HW,
                          float* d1, float* d2, int accumulate, void* stream);

/* ---------------------------------------------------------------- D1-D4 --
 * get_preds + final_preds + kps_fromHeatmap (utils/udaap/evaluation.py:13-30,215-238;
 * utils/process.py:320-327).  tinv [N,6] f64 = rows 0-1 of inv(get_transform)
 * (nullable: no transform).  raw/preds [N,K,2], scores [N,K] (each nullable). */
/*@ hm:f32[(int64_t)N*K*H*W] tinv:f64[N*6] raw:f32[N*K*2] preds:f32[N*K*2] scores:f32[N*K] */
int ubpl_decode_heatmaps(const float* hm, int N, int K, int H, int W, const double* tinv, float* raw, float* preds,
                         float* scores, void* stream);
/* EvaluationUtils.acc_pck (utils/evaluation.py:91-139).  errs/accs [K+1];
 * hits/valid [K] int32 (nullable) for cross-rank aggregation. */
/*@ preds:f32[N*K*2] gts:f32[N*K*3] errs:f32[K+1] accs:f32[K+1] hits:i32[K] valid:i32[K] */
int ubpl_pck(const float* preds, const float* gts, int N, int K, int ref0, int ref1, float thr, float* errs,
             float* accs, int* hits, int* valid, void* stream);

/* ---------------------------------------------------------------- E1 ----
 * update_ema_variables (utils/parameters.py:4-8) on a flat parameter buffer. */
/*@ ema:f32[n] p:f32[n] */
int ubpl_ema_update(float* ema, const float* p, int64_t n, double alpha, void* stream);
/* torch.optim.AdamW step (the optimizer projects/MT_UBPL.py:48 builds) on flat buffers. */
/*@ p:f32[n] g:f32[n] m:f32[n] v:f32[n] */
int ubpl_adamw_step(float* p, const float* g, float* m, float* v, int64_t n, double lr, double beta1, double beta2,
                    double eps, double weight_decay, int64_t step, void* stream);
/* The same step with the 1-based step count on the device (incremented by the
 * call), so a captured HIP graph of the training step replays it; coef: 4 floats. */
/*@ p:f32[n] g:f32[n] m:f32[n] v:f32[n] step:i64[1] coef:f32[4] */
int ubpl_adamw_step_dev(float* p, const float* g, float* m, float* v, int64_t n, double lr, double beta1,
                        double beta2, double eps, double weight_decay, int64_t* step, float* coef, void* stream);
/* ubpl_adamw_step_dev on p[0, nlive) fused with ubpl_ema_update(ema, p, n) in
 * one pass (the optimizer step of projects/MT_UBPL.py:338-340 followed by
 * update_ema_variables, utils/parameters.py:4-8); bit-identical to the two
 * calls.  nlive, n multiples of 4; buffers 16-B aligned. */
/*@ p:f32[n] g:f32[nlive] m:f32[nlive] v:f32[nlive] step:i64[1] coef:f32[4] ema:f32[n] */
int ubpl_adamw_ema_step_dev(float* p, const float* g, float* m, float* v, int64_t nlive, double lr, double beta1,
                            double beta2, double eps, double weight_decay, int64_t* step, float* coef, float* ema,
                            int64_t n, double alpha, void* stream);
/*@ x:f32[n] */
int ubpl_scale_(float* x, int64_t n, float s, void* stream);

/* ---------------------------------------------------------------- H2-H4 --
 * BatchNorm2d (models/base/layers.py:41,57-61), train-mode statistics.
 * part: scratch of ubpl_bn_part_doubles(B,C) doubles, ZEROED before its first
 * use (arrival counters for C <= 512 channels at its head, which each call
 * leaves at zero, then the partial sums; one call at a time per scratch).  rmean/rvar updated with momentum
 * (nullable).  scale = gamma*invstd, shift = beta - mean*scale. */
int ubpl_bn_splits(int B, int C);
int64_t ubpl_bn_part_doubles(int B, int C);
/*@ x:f32[(int64_t)B*C*HW] gamma:f32[C] beta:f32[C] rmean:f32[C] rvar:f32[C] part:f64[ubpl_bn_part_doubles(B,C)] mean_out:f32[C] invstd_out:f32[C] scale:f32[C] shift:f32[C] */
int ubpl_bn_forward_stats(const float* x, int B, int C, int HW, const float* gamma, const float* beta, float eps,
                          float momentum, float* rmean, float* rvar, double* part, float* mean_out,
                          float* invstd_out, float* scale, float* shift, void* stream);
/*@ gamma:f32[C] beta:f32[C] rmean:f32[C] rvar:f32[C] scale:f32[C] shift:f32[C] */
int ubpl_bn_eval_coeffs(const float* gamma, const float* beta, const float* rmean, const float* rvar, float eps,
                        int C, float* scale, float* shift, void* stream);
/*@ x:f32[(int64_t)B*C*HW] scale:f32[C] shift:f32[C] y:f32[(int64_t)B*C*HW] */
int ubpl_bn_apply(const float* x, int B, int C, int HW, const float* scale, const float* shift, int relu, float* y,
                  void* stream);
/* Statistics from 64-pixel partials: part [C][ceil(N/64)][2] f32 = (S, M2) =
 * (sum y, sum (y - S/n)^2) over each 64-pixel slice of the flat (b, p) pixels of
 * y [B,C,P] (Chan's parallel form); the conv kernels write it from their
 * accumulators (stat_part arguments), ubpl_bn_partials from a tensor.
 * ubpl_bn_stats_from_partials: outputs as ubpl_bn_forward_stats, f64 combine. */
int64_t ubpl_bn_partial_floats(int C, int64_t N);
/*@ y:f32[(int64_t)B*C*P] part:f32[ubpl_bn_partial_floats(C,(int64_t)B*P)] */
int ubpl_bn_partials(const float* y, int B, int C, int P, float* part, void* stream);
/*@ part:f32[ubpl_bn_partial_floats(C,N)] gamma:f32[C] beta:f32[C] rmean:f32[C] rvar:f32[C] mean_out:f32[C] invstd_out:f32[C] scale:f32[C] shift_out:f32[C] */
int ubpl_bn_stats_from_partials(const float* part, int C, int64_t N, const float* gamma,
                                const float* beta, float eps, float momentum, float* rmean, float* rvar,
                                float* mean_out, float* invstd_out, float* scale, float* shift_out, void* stream);
/* Backward of y = [relu](bn(x)); dgamma/dbeta accumulate; dx = add1 + add2 + dL/dx.
 * Statistics: one launch over `scratch` (ubpl_bn_part_doubles(B, C) doubles,
 * zeroed before first use, as ubpl_bn_forward_stats), or — part != nullptr —
 * from backward partials dz's producer wrote: per (channel, 64-pixel slice)
 * (S1, S2) = (sum g, sum g*(x - mean)), g = dz under the recomputed ReLU mask,
 * ubpl_bn_partial_floats(C, B*HW) floats (a conv epilogue's bn_part argument,
 * or ubpl_bn_backward_partials); coef: 3*C floats of scratch. */
/*@ dz:f32[(int64_t)B*C*HW] x:f32[(int64_t)B*C*HW] gamma:f32[C] mean:f32[C] invstd:f32[C] scale:f32[C] shift:f32[C] scratch:f64[ubpl_bn_part_doubles(B,C)] part:f32[ubpl_bn_partial_floats(C,(int64_t)B*HW)] coef:f32[3*C] dgamma:f32[C] dbeta:f32[C] add1:f32[(int64_t)B*C*HW] add2:f32[(int64_t)B*C*HW] dx:f32[(int64_t)B*C*HW] */
int ubpl_bn_backward(const float* dz, const float* x, int B, int C, int HW, const float* gamma, const float* mean,
                     const float* invstd, const float* scale, const float* shift, int relu, double* scratch,
                     const float* part, float* coef, float* dgamma, float* dbeta, const float* add1,
                     const float* add2, float* dx, void* stream);
/* The same backward with dx delivered only as PSA planes (ubpl_split_activation
 * layout, border `pad`, npieces 1, 2 or 3) — the operand of a split-path 3x3 data /
 * weight gradient; no addends; C % 16 == 0.  npieces 2 (2xfp16): the statistics
 * pass also bounds |dx| and picks the power-of-two scale of the fp16 pieces,
 * written to coef[3C] (coef: 3C + 1 floats) for the consumers (act_scale of
 * ubpl_conv2d_forward_psa / dscale of ubpl_wgrad3_psa); not with `part`. */
/*@ dz:f32[(int64_t)B*C*H*W] x:f32[(int64_t)B*C*H*W] gamma:f32[C] mean:f32[C] invstd:f32[C] scale:f32[C] shift:f32[C] scratch:f64[ubpl_bn_part_doubles(B,C)] part:f32[ubpl_bn_partial_floats(C,(int64_t)B*H*W)] coef:f32[3*C+1] dgamma:f32[C] dbeta:f32[C] dst:u16[(npieces-1)*plane+(int64_t)B*C*(H+2*pad)*(W+2*pad)] */
int ubpl_bn_backward_split(const float* dz, const float* x, int B, int C, int H, int W, const float* gamma,
                           const float* mean, const float* invstd, const float* scale, const float* shift, int relu,
                           double* scratch, const float* part, float* coef, float* dgamma, float* dbeta, int pad,
                           int npieces, uint16_t* dst, int64_t plane, void* stream);
/* The backward statistics partials alone (the layout above). */
/*@ dz:f32[(int64_t)B*C*HW] x:f32[(int64_t)B*C*HW] scale:f32[C] shift:f32[C] mean:f32[C] part:f32[ubpl_bn_partial_floats(C,(int64_t)B*HW)] */
int ubpl_bn_backward_partials(const float* dz, const float* x, int B, int C, int HW, const float* scale,
                              const float* shift, const float* mean, int relu, float* part, void* stream);

/* Conv (models/base/layers.py:31-50): 1x1/s1, 3x3/s1, 7x7/s2, pad (KS-1)/2,
 * optional fused pre-activation relu(x*pscale + pshift), bias, residual add
 * (res may alias y).  MFMA f32 implicit GEMM over a grouped tap-major K,
 * k = (ci/G)*G*T + tap*G + ci%G (T = KS*KS, G = 16 if 16 | Cin else Cin):
 * for KS > 1 the weights must be in the layout ubpl_conv_weight_tapmajor makes,
 * [Cout][Cin/G][T][G] (for KS == 1 that is the reference layout itself).
 * Small grids split K over workgroups: slab = ubpl_conv2d_forward_workspace
 * floats (nullable when that is 0). */
int64_t ubpl_conv2d_forward_workspace(int B, int Cin, int Cout, int KS, int Ho, int Wo);
/*@ x:f32[(int64_t)B*Cin*H*W] w:f32[(int64_t)Cout*Cin*KS*KS] bias:f32[Cout] pscale:f32[Cin] pshift:f32[Cin] res:f32[(int64_t)B*Cout*Ho*Wo] y:f32[(int64_t)B*Cout*Ho*Wo] slab:f32[ubpl_conv2d_forward_workspace(B,Cin,Cout,KS,Ho,Wo)] */
int ubpl_conv2d_forward(const float* x, int B, int Cin, int H, int W, const float* w, const float* bias, int Cout,
                        int KS, int stride, const float* pscale, const float* pshift, const float* res, float* y,
                        int Ho, int Wo, float* slab, void* stream);
/*@ w:f32[(int64_t)Cout*Cin*KS*KS] wt:f32[(int64_t)Cout*Cin*KS*KS] */
int ubpl_conv_weight_tapmajor(const float* w, int Cout, int Cin, int KS, float* wt, void* stream);
/* 1x1 stride-1 conv fed by LDS-DMA, k-major weights wk [Cin][Cout] (the
 * data-gradient re-layout of the conv; for a data gradient, the reference
 * weights themselves): same semantics as ubpl_conv2d_forward with KS = 1.
 * Cin % 16 == 0, Cout % 4 == 0, P % 4 == 0, x / wk 16-B aligned, Cin <= 256 with a
 * prologue. */
int64_t ubpl_conv1x1_kmajor_workspace(int B, int Cin, int Cout, int P);
/*@ x:f32[(int64_t)B*Cin*P] wk:f32[(int64_t)Cin*Cout] bias:f32[Cout] pscale:f32[Cin] pshift:f32[Cin] res:f32[(int64_t)B*Cout*P] y:f32[(int64_t)B*Cout*P] slab:f32[ubpl_conv1x1_kmajor_workspace(B,Cin,Cout,P)] stat_part:f32[ubpl_bn_partial_floats(Cout,(int64_t)B*P)] */
int ubpl_conv1x1_forward_kmajor(const float* x, int B, int Cin, int P, const float* wk, const float* bias, int Cout,
                                const float* pscale, const float* pshift, const float* res, float* y, float* slab,
                                float* stat_part, void* stream);
/* Weight gradient (+ bias gradient), reference weight layout. */
int64_t ubpl_conv2d_wgrad_workspace(int B, int Cin, int Cout, int KS, int Ho, int Wo);
/*@ dy:f32[(int64_t)B*Cout*Ho*Wo] x:f32[(int64_t)B*Cin*H*W] pscale:f32[Cin] pshift:f32[Cin] slab:f32[ubpl_conv2d_wgrad_workspace(B,Cin,Cout,KS,Ho,Wo)] dw:f32[(int64_t)Cout*Cin*KS*KS] db:f32[Cout] */
int ubpl_conv2d_wgrad(const float* dy, const float* x, int B, int Cin, int H, int W, int Cout, int KS, int stride,
                      const float* pscale, const float* pshift, int Ho, int Wo, float* slab, float* dw, float* db,
                      int accumulate, void* stream);
/* Data-gradient weights (stride 1): the forward layout of the flipped,
 * transposed kernel ([Cin][Cout/G][T][G], G from Cout), so
 * dx = ubpl_conv2d_forward(dy, wt). */
/*@ w:f32[(int64_t)Cout*Cin*KS*KS] wt:f32[(int64_t)Cout*Cin*KS*KS] */
int ubpl_conv_weight_flip(const float* w, int Cout, int Cin, int KS, float* wt, void* stream);
/* Reduce a weight-gradient slab [splits][Cout][Cin*T + 1] (columns n = tap*Cin + ci,
 * last = bias) into dw (reference layout, (+)=) and db (nullable). */
/*@ slab:f32[(int64_t)splits*Cout*((int64_t)Cin*T+1)] dw:f32[(int64_t)Cout*Cin*T] db:f32[Cout] */
int ubpl_wgrad_slab_reduce(const float* slab, int splits, int Cout, int Cin, int T, int with_bias, float* dw,
                           float* db, int accumulate, void* stream);
/* Both re-layouts for many convs in one launch: table int64 [nseg][5] =
 * (src_off, dst_off, Cout, Cin, KS*KS) in floats; mode 0 tap-major, 1 dgrad. */
/*@ src:f32[?] dst:f32[?] table:i64[nseg*5] */
int ubpl_conv_weights_relayout(const float* src, float* dst, const int64_t* table, int nseg, int mode, void* stream);

/* Split MFMA path of the same Conv (conv_split.hip): every f32 operand carried
 * as npieces 16-bit pieces, the piece products with pa + pb < npieces summed by
 * the 32x32x16 MFMA in f32: npieces 3 = three bf16 pieces ("6xbf16", exact
 * operands, 6 products), 2 = two fp16 pieces of the operand times a power-of-two
 * scale ("2xfp16", 3 products on v_mfma_f32_32x32x16_f16; weights scaled by
 * 2^(9 + ceil(log2 sqrt K)) for contraction length K, activations by 32, the
 * accumulators unscaled exactly before the stores), 1 = bf16 operands.  Weights:
 * ubpl_conv_weights_split writes npieces planes (`plane` elements apart)
 * of the mode-0 (forward, grouped tap-major) or mode-1 (data-gradient) layout
 * for many convs in one launch (table as above, dst_off % 8 == 0).
 * ubpl_conv2d_forward_split (the register-staged kernel, npieces 3): (KS, stride)
 * in {(1,1), (3,1)}, Cin % 16 == 0, wsplit 16-B aligned; other arguments as
 * ubpl_conv2d_forward. */
/*@ src:f32[?] dst:u16[npieces*plane] table:i64[nseg*5] */
int ubpl_conv_weights_split(const float* src, uint16_t* dst, int64_t plane, const int64_t* table, int nseg, int mode,
                            int npieces, void* stream);
int64_t ubpl_conv2d_forward_split_workspace(int B, int Cin, int Cout, int KS, int Ho, int Wo, int npieces);
/*@ x:f32[(int64_t)B*Cin*H*W] wsplit:u16[(npieces-1)*plane+(int64_t)Cout*Cin*KS*KS] bias:f32[Cout] pscale:f32[Cin] pshift:f32[Cin] res:f32[(int64_t)B*Cout*Ho*Wo] y:f32[(int64_t)B*Cout*Ho*Wo] slab:f32[ubpl_conv2d_forward_split_workspace(B,Cin,Cout,KS,Ho,Wo,npieces)] */
int ubpl_conv2d_forward_split(const float* x, int B, int Cin, int H, int W, const uint16_t* wsplit, int64_t plane,
                              const float* bias, int Cout, int KS, int stride, const float* pscale,
                              const float* pshift, const float* res, float* y, int Ho, int Wo, float* slab,
                              int npieces, void* stream);
/* Pre-split activations ("PSA"): npieces 16-bit planes (`plane` elements apart)
 * of [B][C/16][H+2pad][W+2pad][16] holding relu(x*pscale + pshift) (or x when
 * pscale is null) with a zero border; C % 16 == 0.  npieces 2 (2xfp16): the
 * pieces of v * 32; dst3 (nullable, npieces 2 only): also the 3-piece bf16
 * image of v (planes `plane3` apart) from the same read. */
/*@ x:f32[(int64_t)B*C*H*W] pscale:f32[C] pshift:f32[C] dst:u16[(npieces-1)*plane+(int64_t)B*C*(H+2*pad)*(W+2*pad)] dst3:u16[2*plane3+(int64_t)B*C*(H+2*pad)*(W+2*pad)] */
int ubpl_split_activation(const float* x, int B, int C, int H, int W, const float* pscale, const float* pshift,
                          int pad, int npieces, uint16_t* dst, int64_t plane, uint16_t* dst3, int64_t plane3,
                          void* stream);
/* Stride-1 conv (KS 1 or 3) of PSA activations (pad >= (KS-1)/2) with split
 * weights: both operands DMA'd global -> LDS; y = conv + bias (+ res, may alias y). */
int64_t ubpl_conv2d_forward_psa_workspace(int B, int Cin, int Cout, int KS, int H, int W, int npieces);
/* Test hook (host-only): the 3x3 input-halo kernel dispatch of
 * ubpl_conv2d_forward_psa.  halo_mode -1 default, 0 off, 1 on where eligible,
 * 2 on and required (an ineligible 3x3 launch returns hipErrorInvalidValue),
 * 3 the one-buffer variant required; teams -1 default, 1 / 2 teams per
 * workgroup.  The environment (UBPL_PSA_HALO = 0 / 1, UBPL_PSA_TEAMS) sets the
 * initial values, read once; (-2, -2) returns to the environment's values. */
int ubpl_set_psa_dispatch(int halo_mode, int teams);
/* 3x3 weight gradient (+ bias gradient, db nullable) on the split path from PSA
 * operands with a 1-pixel border: dys = split(dy), xs = split(conv input),
 * npieces 3 (6xbf16), 1 (bf16) or 2 (2xfp16: dys the pieces of dy * *dscale —
 * ubpl_bn_backward_split's coef[3C] — and xs of x * 32, the forward's image;
 * dscale required exactly then); Cin % 64 == 0, Cout % 64 == 0, W % 16 == 0. */
int64_t ubpl_wgrad3_psa_workspace(int B, int Cin, int Cout, int H, int W);
/*@ dys:u16[(npieces-1)*dplane+(int64_t)B*Cout*(H+2)*(W+2)] xs:u16[(npieces-1)*xplane+(int64_t)B*Cin*(H+2)*(W+2)] slab:f32[ubpl_wgrad3_psa_workspace(B,Cin,Cout,H,W)] dw:f32[(int64_t)Cout*Cin*9] db:f32[Cout] dscale:f32[1] */
int ubpl_wgrad3_psa(const uint16_t* dys, int64_t dplane, const uint16_t* xs, int64_t xplane, int B, int Cin,
                    int Cout, int H, int W, float* slab, float* dw, float* db, int accumulate, int npieces,
                    const float* dscale, void* stream);
/* The 7x7 stride-2 stem's weight gradient (+ bias gradient, db nullable) on the
 * split path, as the weight gradient of its space-to-depth form (replaces the
 * exact-f32 ubpl_conv2d_wgrad for models/pose/hourglass.py pre.0 / layers.py:31-50):
 * dys = split(dy) (PSA, pad 1, Cout channels at the H x W output), xs = the
 * forward's phase image (ubpl_stem_s2d_split, 16 channels, pad 2); KS = 7, C <= 4
 * input channels, Cout % 64 == 0, W % 16 == 0, npieces 3 or 1.  _workspace: slab floats. */
int64_t ubpl_wgrad_stem_psa_workspace(int B, int Cout, int H, int W);
/*@ dys:u16[(npieces-1)*dplane+(int64_t)B*Cout*(H+2)*(W+2)] xs:u16[(npieces-1)*xplane+(int64_t)B*16*(H+4)*(W+4)] slab:f32[ubpl_wgrad_stem_psa_workspace(B,Cout,H,W)] dw:f32[(int64_t)Cout*C*KS*KS] db:f32[Cout] */
int ubpl_wgrad_stem_psa(const uint16_t* dys, int64_t dplane, const uint16_t* xs, int64_t xplane, int B, int C,
                        int Cout, int H, int W, int KS, float* slab, float* dw, float* db, int accumulate,
                        int npieces, void* stream);
/* 1x1 weight gradient (+ bias gradient, db nullable) on the split path with
 * both f32 operands (dy [B,Cout,P], x [B,Cin,P], prologue relu(x*pscale +
 * pshift) when pscale != nullptr) split while staged: npieces 3 = 6xbf16,
 * 1 = bf16 operands with f32 accumulation.  _workspace: slab floats,
 * 0 = shape not supported (needs Cin % 64 == 0, Cout % 64 == 0, P % 16 == 0). */
int64_t ubpl_wgrad1x1_split_load_workspace(int B, int Cin, int Cout, int P);
/*@ dy:f32[(int64_t)B*Cout*P] x:f32[(int64_t)B*Cin*P] pscale:f32[Cin] pshift:f32[Cin] slab:f32[ubpl_wgrad1x1_split_load_workspace(B,Cin,Cout,P)] dw:f32[(int64_t)Cout*Cin] db:f32[Cout] */
int ubpl_wgrad1x1_split_load(const float* dy, const float* x, int B, int Cin, int Cout, int P, const float* pscale,
                             const float* pshift, float* slab, float* dw, float* db, int accumulate, int npieces,
                             void* stream);
/*@ xs:u16[(npieces-1)*xplane+(int64_t)B*Cin*(H+2*pad)*(W+2*pad)] wsplit:u16[(npieces-1)*wplane+(int64_t)Cout*Cin*KS*KS] bias:f32[Cout] res:f32[(int64_t)B*Cout*H*W] y:f32[(int64_t)B*Cout*H*W] slab:f32[ubpl_conv2d_forward_psa_workspace(B,Cin,Cout,KS,H,W,npieces)] stat_part:f32[ubpl_bn_partial_floats(Cout,(int64_t)B*H*W)] bn_x:f32[(int64_t)B*Cout*H*W] bn_coef:f32[3*Cout] bn_part:f32[ubpl_bn_partial_floats(Cout,(int64_t)B*H*W)] act_scale:f32[1] */
int ubpl_conv2d_forward_psa(const uint16_t* xs, int64_t xplane, int B, int Cin, int H, int W, int pad,
                            const uint16_t* wsplit, int64_t wplane, const float* bias, int Cout, int KS,
                            const float* res, float* y, float* slab, int npieces, float* stat_part,
                            const float* bn_x, const float* bn_coef, int bn_relu, float* bn_part,
                            const float* act_scale, void* stream);
/* bn_part (nullable; with bn_x [B,Cout,P], bn_coef = scale|shift|mean, Cout
 * floats each, bn_relu): when y is the data gradient dz of a BatchNorm(+ReLU)
 * with input bn_x, its backward statistics partials (ubpl_bn_backward layout),
 * from the epilogue — then ubpl_bn_backward(..., part_ready = 1) needs no pass.
 * act_scale (nullable, npieces 2 only): the device-side scale of xs's pieces (a
 * data gradient's, ubpl_bn_backward_split coef[3C]); null: xs from
 * ubpl_split_activation (scale 32). */
/* The 7x7 stride-2 stem (Cin <= 4) on the split path by space-to-depth: the
 * phase images of x as a 16-channel PSA image with a `pad` (>= 2) border, and
 * the equivalent 4x4 stride-1 weights (Cin' = 16, KS' = 4) split into npieces
 * (3: 6xbf16; 1: the bf16 precision) planes of Cout*256 bf16; then
 * ubpl_conv2d_forward_psa(..., KS = 4). */
/*@ x:f32[(int64_t)B*C*H*W] dst:u16[(npieces-1)*plane+(int64_t)B*16*(H/2+2*pad)*(W/2+2*pad)] */
int ubpl_stem_s2d_split(const float* x, int B, int C, int H, int W, int pad, int npieces, uint16_t* dst,
                        int64_t plane, void* stream);
/*@ w:f32[(int64_t)Cout*C*KS*KS] dst:u16[(npieces-1)*plane+(int64_t)Cout*256] */
int ubpl_stem_weight_s2d_split(const float* w, int Cout, int C, int KS, int npieces, uint16_t* dst, int64_t plane,
                               void* stream);
/* 1x1 stride-1 conv on the split path with the f32 activations split while
 * they are staged (no pre-split image): y = conv(relu(x*pscale + pshift) or x)
 * + bias (+ res, may alias y); wsplit = npieces planes of [Cout][Cin] from
 * ubpl_conv_weights_split (KS = 1); npieces 3 = 6xbf16, 2 = 2xfp16 (no epilogue
 * partials), 1 = bf16 operands (one plane; no epilogue partials).  Cin % 16 == 0, Cout % 16 == 0, P % 4 == 0.
 * stat_part (nullable): BatchNorm partials of y (ubpl_bn_partials layout).
 * _preferred: 1 when the shape is supported and fills the chip. */
int ubpl_conv1x1_split_load_preferred(int B, int Cin, int Cout, int P);
/*@ x:f32[(int64_t)B*Cin*P] wsplit:u16[(npieces-1)*wplane+(int64_t)Cout*Cin] bias:f32[Cout] pscale:f32[Cin] pshift:f32[Cin] res:f32[(int64_t)B*Cout*P] y:f32[(int64_t)B*Cout*P] stat_part:f32[ubpl_bn_partial_floats(Cout,(int64_t)B*P)] bn_x:f32[(int64_t)B*Cout*P] bn_coef:f32[3*Cout] bn_part:f32[ubpl_bn_partial_floats(Cout,(int64_t)B*P)] */
int ubpl_conv1x1_forward_split_load(const float* x, int B, int Cin, int P, const uint16_t* wsplit, int64_t wplane,
                                    const float* bias, int Cout, const float* pscale, const float* pshift,
                                    const float* res, float* y, float* stat_part, const float* bn_x,
                                    const float* bn_coef, int bn_relu, float* bn_part, int npieces, void* stream);

/* MaxPool2d(2,2) (models/base/layers.py:93), Upsample(x2, nearest) + add
 * (layers.py:110-111), AvgPool2d(2,2) projection (models/pose/hourglass.py:226). */
/*@ x:f32[planes*H*W] y:f32[planes*(H/2)*(W/2)] */
int ubpl_maxpool2x2_forward(const float* x, int64_t planes, int H, int W, float* y, void* stream);
/*@ x:f32[planes*H*W] dy:f32[planes*(H/2)*(W/2)] dx:f32[planes*H*W] */
int ubpl_maxpool2x2_backward(const float* x, const float* dy, int64_t planes, int H, int W, float* dx,
                             int accumulate, void* stream);
/*@ x:f32[planes*H*W] y:f32[planes*(H/2)*(W/2)] */
int ubpl_avgpool2x2_forward(const float* x, int64_t planes, int H, int W, float* y, void* stream);
/*@ dy:f32[planes*(H/2)*(W/2)] dx:f32[planes*H*W] */
int ubpl_avgpool2x2_backward(const float* dy, int64_t planes, int H, int W, float* dx, int accumulate, void* stream);
/*@ up:f32[planes*H*W] low:f32[planes*(H/2)*(W/2)] out:f32[planes*H*W] */
int ubpl_upsample2x_add_forward(const float* up, const float* low, int64_t planes, int H, int W, float* out,
                                void* stream);
/*@ dout:f32[planes*H*W] dlow:f32[planes*(H/2)*(W/2)] */
int ubpl_upsample2x_add_backward(const float* dout, int64_t planes, int H, int W, float* dlow, int accumulate,
                                 void* stream);
/*@ a:f32[n] b:f32[n] out:f32[n] */
int ubpl_add(const float* a, const float* b, int64_t n, float* out, void* stream);
/* The same forwards + BatchNorm partials of the output for the BN that
 * consumes it (ubpl_bn_partials layout); output planes of a multiple of 64 pixels. */
/*@ x:f32[(int64_t)B*C*H*W] y:f32[(int64_t)B*C*(H/2)*(W/2)] part:f32[ubpl_bn_partial_floats(C,(int64_t)B*(H/2)*(W/2))] */
int ubpl_maxpool2x2_forward_stats(const float* x, int B, int C, int H, int W, float* y, float* part, void* stream);
/*@ up:f32[(int64_t)B*C*H*W] low:f32[(int64_t)B*C*(H/2)*(W/2)] out:f32[(int64_t)B*C*H*W] part:f32[ubpl_bn_partial_floats(C,(int64_t)B*H*W)] */
int ubpl_upsample2x_add_forward_stats(const float* up, const float* low, int B, int C, int H, int W, float* out,
                                      float* part, void* stream);

/* ---------------------------------------------------------------- f1 ----
 * Two-view training augmentation (DS_mds.__getitem__, datasets/dataset_mds.py:41-201:
 * fliplr utils/augment.py:216-227, noisy_mean :261-267, affine :86-156,
 * image_colorNorm utils/process.py:151-160) on images resident in HBM.
 * imgs uint8 BGR [N][H][W][3].  ubpl_image_mean_u8: out[n] = mean of image n / 255
 * (the noisy_mean mu).  ubpl_augment_warp: view v samples image src_idx[v] at
 * (mat[6v..6v+2] . (x,y,1), mat[6v+3..6v+5] . (x,y,1)) — flip and the inverse
 * crop/scale/rotate transform folded by the host — bilinear, zero outside;
 * noise[3v..3v+2] = (alpha, beta, enabled) of noisy_mean; out [V][3][Ho][Wo]
 * float32 minus chan_mean[3]. */
/*@ imgs:u8[N*n_per_image] out:f32[N] */
int ubpl_image_mean_u8(const uint8_t* imgs, int N, int64_t n_per_image, float* out, void* stream);
/*@ imgs:u8[?] src_idx:i32[V] mat:f32[6*V] noise:f32[3*V] img_mean:f32[?] chan_mean:f32[3] out:f32[(int64_t)V*3*Ho*Wo] */
int ubpl_augment_warp(const uint8_t* imgs, int H, int W, const int* src_idx, const float* mat, const float* noise,
                      const float* img_mean, const float* chan_mean, int V, int Ho, int Wo, float* out, void* stream);

/* ubpl_augment_chain: the same views with the reference's TWO resamplings
 * (utils/augment.py:119-137) instead of one: stage 1, skimage.transform.rotate
 * (order 1, constant 0) of the integer crop of the flipped, noise-adjusted image
 * about the padded crop's centre, pad stripped, into inter [V][3][Hm][Wm]
 * (Hc x Wc used per view); stage 2, skimage.transform.resize to Ho x Wo (order
 * 1, pixel centres, mirror edges), minus chan_mean[3] -> out [V][3][Ho][Wo].
 * geo int [V][8] = (src_idx, flip, ul_x, ul_y, Hp, Wp, Hc, Wc): the grown crop
 * box corner and size, the stripped size (Hp - Hc = Wp - Wc = 2 * pad, Hc <= Hm,
 * Wc <= Wm); cs [V][2] = (cos, sin) of the angle; noise as ubpl_augment_warp. */
/*@ imgs:u8[?] geo:i32[8*V] cs:f32[2*V] noise:f32[3*V] img_mean:f32[?] chan_mean:f32[3] inter:f32[(int64_t)V*3*Hm*Wm] out:f32[(int64_t)V*3*Ho*Wo] */
int ubpl_augment_chain(const uint8_t* imgs, int H, int W, const int* geo, const float* cs, const float* noise,
                       const float* img_mean, const float* chan_mean, int V, int Hm, int Wm, float* inter, int Ho,
                       int Wo, float* out, void* stream);

/* Random occlusion of augmented views (utils/udaap/utils_augment.py:21-25,116-163:
 * augment_occlu / occlude_with_objects / resize_by_factor / paste_over), after
 * ubpl_augment_warp: out [V][3][H][W] (colorNorm'ed) gets, in draw order, each
 * paste alpha * (color - chan_mean) + (1 - alpha) * out.  bank: RGBA float
 * occluders (16-B aligned, [h][w][4] each at bank + off[o], hw[2o..2o+1] = h, w);
 * pastes int [P][9] = (view, occluder, w1, h1, x0, y0, x1, y1, sx0 | sy0 << 16)
 * sorted by view, view_first [V+1] the first paste of each view; the occluder is
 * resized to w1 x h1 by pixel-area averaging (cv2.INTER_AREA). */
/*@ out:f32[(int64_t)V*3*H*W] bank:f32[?] off:i64[?] hw:i32[?] pastes:i32[?] view_first:i32[V+1] chan_mean:f32[3] */
int ubpl_occlude(float* out, int V, int H, int W, const float* bank, const int64_t* off, const int* hw,
                 const int* pastes, const int* view_first, const float* chan_mean, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* UBPL_HIP_H */
