"""Tensor-level wrappers over the C-ABI (no autograd here).

Each wrapper validates device / dtype / contiguity, allocates outputs with
the torch caching allocator on the input's device and enqueues on torch's
current stream.  Nothing here computes on the host.
"""
import os

import torch

from . import _lib
from ._lib import call

F32 = torch.float32


def _p(t):
    """A device-pointer argument of a C-ABI entry: the tensor itself (its op
    passes data_ptr()), or None for NULL."""
    return t


def _chk(t, name, dtype=F32):
    if t is None:
        return
    _lib.require_gpu(t)
    if t.dtype != dtype:
        raise TypeError("ubpl_amd: %s must be %s, got %s" % (name, dtype, t.dtype))
    if not t.is_contiguous():
        raise ValueError("ubpl_amd: %s must be contiguous" % name)


# ------------------------------------------------------------------ R1
def render_heatmaps(kps, img_hw, inp_res, out_res, kernel_size=3.0, sigma=1.0, cutoff=0.01, kps_out=None):
    """kps [N,K,3] -> (hm [N,K,Rh,Rw], kps_out [N,K,3] with vis applied)."""
    _chk(kps, "kps")
    N, K, _ = kps.shape
    stride = inp_res / out_res
    rh, rw = int(img_hw[0] / stride), int(img_hw[1] / stride)
    hm = torch.empty((N, K, rh, rw), device=kps.device, dtype=F32)
    if kps_out is None:
        kps_out = torch.empty_like(kps)
    call("ubpl_render_heatmaps", _p(kps), _p(hm), _p(kps_out), N, K, int(img_hw[0]), int(img_hw[1]),
         int(inp_res), int(out_res), float(kernel_size), float(sigma), float(cutoff))
    return hm, kps_out


# ------------------------------------------------------------------ L1-L4
class RowGeom:
    """Row geometry of a (pred, target) pair for the heatmap loss kernels.
    a rows (b,s,k): a + b*a_sb + s*a_ss + k*HW; target rows: mean over m of
    t + m*t_sm + b*t_sb + s*t_ss + k*HW (strides in elements)."""

    def __init__(self, a, a_sb, a_ss, t, t_sb, t_ss, t_sm, M, B, S, K, HW):
        self.a, self.t = a, t
        self.a_off = 0
        self.args = (a_sb, a_ss, t_sb, t_ss, t_sm, M, B, S, K, HW)
        self.B, self.S, self.K, self.HW = B, S, K, HW
        self.a_ptr = a          # row base pointers as tensors (views at an element offset)
        self.t_ptr = t


def geom_stack(a, t, S, t_mode):
    """a: [B,S,K,R,R] (or [B,K,R,R] with S==1), contiguous.
    t_mode 'gt'    t [B,K,R,R] broadcast over stacks;
           'same'  t has a's layout;
           'ens'   t [M,B,St,K,R,R] (or [M,B,K,R,R]): mean over M of the LAST stack."""
    _chk(a, "preds")
    _chk(t, "targets")
    B = a.shape[0]
    K = a.shape[-3]
    HW = a.shape[-1] * a.shape[-2]
    a_sb, a_ss = S * K * HW, K * HW
    if t_mode == "gt":
        return RowGeom(a, a_sb, a_ss, t, K * HW, 0, 0, 1, B, S, K, HW)
    if t_mode == "same":
        return RowGeom(a, a_sb, a_ss, t, a_sb, a_ss, 0, 1, B, S, K, HW)
    M = t.shape[0]
    St = t.shape[2] if t.dim() == 6 else 1
    g = RowGeom(a, a_sb, a_ss, t, St * K * HW, 0, B * St * K * HW, M, B, S, K, HW)
    g.t_ptr = t.reshape(-1)[(St - 1) * K * HW:]
    return g


def geom_rows(a, a_base_elems, a_sb, t, t_base_elems, t_sb, B, K, HW, t_sm=0, M=1):
    """Single-stack rows with explicit base offsets/strides (e.g. last-stack slices)."""
    g = RowGeom(a, a_sb, 0, t, t_sb, 0, t_sm, M, B, 1, K, HW)
    g.a_ptr = a.reshape(-1)[a_base_elems:]
    g.t_ptr = t.reshape(-1)[t_base_elems:]
    return g


def row_stats(g, want_amax=False, want_tmax=False):
    dev = g.a.device
    rows = g.B * g.S * g.K
    sq = torch.empty(rows, device=dev, dtype=F32)
    am = torch.empty(rows, device=dev, dtype=F32) if want_amax else None
    tm = torch.empty(rows, device=dev, dtype=F32) if want_tmax else None
    a_sb, a_ss, t_sb, t_ss, t_sm, M, B, S, K, HW = g.args
    call("ubpl_heatmap_row_stats", g.a_ptr, a_sb, a_ss, g.t_ptr, t_sb, t_ss, t_sm, M, B, S, K, HW,
         _p(sq), _p(am), _p(tm))
    return sq, am, tm


def loss_finalize(kind, sq, amax, tmax, gate, sw, use_gate, use_sw, B, S, K, thr):
    dev = sq.device
    out_sum = torch.empty(1, device=dev, dtype=F32)
    out_cnt = torch.empty(4, device=dev, dtype=torch.int32)
    score = torch.empty(K, device=dev, dtype=F32) if kind != 0 else None
    w = torch.empty(B * S * K, device=dev, dtype=F32)
    call("ubpl_loss_finalize", int(kind), _p(sq), _p(amax), _p(tmax), _p(gate), _p(sw), int(use_gate),
         int(use_sw), B, S, K, float(thr), _p(out_sum), _p(out_cnt), _p(score), _p(w))
    return out_sum, out_cnt, score, w


def row_grad(g, w, gscale, extra, da, accumulate=False):
    a_sb, a_ss, t_sb, t_ss, t_sm, M, B, S, K, HW = g.args
    call("ubpl_heatmap_row_grad", g.a_ptr, a_sb, a_ss, g.t_ptr, t_sb, t_ss, t_sm, M, B, S, K, HW, _p(w),
         _p(gscale), float(extra), _p(da), int(accumulate))
    return da


# ------------------------------------------------------------------ L5
def fdl_cov_forward(f1, f2, rowmask=None):
    _chk(f1, "f1")
    _chk(f2, "f2")
    B, S, C = f1.shape[:3]
    HW = f1[0, 0, 0].numel()
    dev = f1.device
    cov = torch.empty(B * S * C, device=dev, dtype=F32)
    mu1, mu2 = torch.empty_like(cov), torch.empty_like(cov)
    val = torch.empty(1, device=dev, dtype=F32)
    cnt = torch.empty(1, device=dev, dtype=torch.int32)
    call("ubpl_fdl_cov_forward", _p(f1), _p(f2), _p(rowmask), B, S, C, HW, _p(cov), _p(mu1), _p(mu2), _p(val),
         _p(cnt))
    return val, cnt, (cov, mu1, mu2)


def fdl_cov_backward(f1, f2, rowmask, saved, cnt, gscale, d1=None, d2=None, accumulate=False):
    B, S, C = f1.shape[:3]
    HW = f1[0, 0, 0].numel()
    cov, mu1, mu2 = saved
    call("ubpl_fdl_cov_backward", _p(f1), _p(f2), _p(rowmask), _p(cov), _p(mu1), _p(mu2), _p(cnt), _p(gscale),
         B, S, C, HW, _p(d1), _p(d2), int(accumulate))
    return d1, d2


# ------------------------------------------------------------------ D1-D4
def decode_heatmaps(hm, tinv=None):
    """hm [N,K,H,W] -> (raw [N,K,2], preds [N,K,2] or None, scores [N,K])."""
    _chk(hm, "heatmap")
    N, K, H, W = hm.shape
    dev = hm.device
    raw = torch.empty((N, K, 2), device=dev, dtype=F32)
    preds = torch.empty((N, K, 2), device=dev, dtype=F32) if tinv is not None else None
    scores = torch.empty((N, K), device=dev, dtype=F32)
    if tinv is not None:
        _chk(tinv, "tinv", torch.float64)
    call("ubpl_decode_heatmaps", _p(hm), N, K, H, W, _p(tinv), _p(raw), _p(preds), _p(scores))
    return raw, preds, scores


def pck(preds, gts, ref, thr):
    _chk(preds, "preds")
    _chk(gts, "gts")
    N, K, _ = preds.shape
    dev = preds.device
    errs = torch.empty(K + 1, device=dev, dtype=F32)
    accs = torch.empty(K + 1, device=dev, dtype=F32)
    hits = torch.empty(K, device=dev, dtype=torch.int32)
    valid = torch.empty(K, device=dev, dtype=torch.int32)
    call("ubpl_pck", _p(preds), _p(gts), N, K, int(ref[0]), int(ref[1]), float(thr), _p(errs), _p(accs), _p(hits),
         _p(valid))
    return errs, accs, hits, valid


# ------------------------------------------------------------------ E1
def ema_update_(ema, p, alpha):
    _chk(ema, "ema")
    _chk(p, "param")
    assert ema.numel() == p.numel()
    call("ubpl_ema_update", _p(ema), _p(p), ema.numel(), float(alpha))


def adamw_step_(p, g, m, v, lr, beta1, beta2, eps, weight_decay, step):
    for t, n in ((p, "p"), (g, "g"), (m, "m"), (v, "v")):
        _chk(t, n)
    call("ubpl_adamw_step", _p(p), _p(g), _p(m), _p(v), p.numel(), float(lr), float(beta1), float(beta2),
         float(eps), float(weight_decay), int(step))



def adamw_step_dev_(p, g, m, v, lr, beta1, beta2, eps, weight_decay, step_t, coef):
    """AdamW with the step count in device memory (int64 scalar, incremented);
    replayable inside a captured HIP graph.  coef: 4-float scratch."""
    call("ubpl_adamw_step_dev", _p(p), _p(g), _p(m), _p(v), p.numel(), float(lr), float(beta1), float(beta2),
         float(eps), float(weight_decay), _p(step_t), _p(coef))

def adamw_ema_step_dev_(p, g, m, v, nlive, lr, beta1, beta2, eps, weight_decay, step_t, coef, ema, alpha):
    """adamw_step_dev_ on p[:nlive] and ema_update_(ema, p, alpha) over all of p, one pass."""
    if ema.numel() != p.numel() or nlive > p.numel():
        raise ValueError("adamw_ema_step_dev_: ema / p / nlive sizes disagree")
    call("ubpl_adamw_ema_step_dev", _p(p), _p(g), _p(m), _p(v), int(nlive), float(lr), float(beta1), float(beta2),
         float(eps), float(weight_decay), _p(step_t), _p(coef), _p(ema), p.numel(), float(alpha))


def scale_(x, s):
    _chk(x, "x")
    call("ubpl_scale_", _p(x), x.numel(), float(s))


# ------------------------------------------------------------------ BN
def bn_splits(B, C):
    return _lib.lib().ubpl_bn_splits(B, C)


def bn_part(B, C, device):
    """Zeroed BN scratch (partial sums + self-resetting arrival counters)."""
    return torch.zeros(int(_lib.lib().ubpl_bn_part_doubles(B, C)), dtype=torch.float64, device=device)


def bn_forward_stats(x, gamma, beta, eps, momentum, rmean, rvar, part, mean, invstd, scale, shift):
    B, C = x.shape[:2]
    HW = x[0, 0].numel()
    call("ubpl_bn_forward_stats", _p(x), B, C, HW, _p(gamma), _p(beta), float(eps), float(momentum), _p(rmean),
         _p(rvar), _p(part), _p(mean), _p(invstd), _p(scale), _p(shift))


def bn_eval_coeffs(gamma, beta, rmean, rvar, eps, scale, shift):
    call("ubpl_bn_eval_coeffs", _p(gamma), _p(beta), _p(rmean), _p(rvar), float(eps), gamma.numel(), _p(scale),
         _p(shift))


def bn_apply(x, scale, shift, relu, out=None):
    B, C = x.shape[:2]
    HW = x[0, 0].numel()
    y = torch.empty_like(x) if out is None else out
    call("ubpl_bn_apply", _p(x), B, C, HW, _p(scale), _p(shift), int(relu), _p(y))
    return y


def bn_partial_buffer(C, N, device):
    return torch.empty(int(_lib.lib().ubpl_bn_partial_floats(C, N)), device=device, dtype=F32)


def bn_partials(y, part):
    B, C = y.shape[:2]
    call("ubpl_bn_partials", _p(y), B, C, y[0, 0].numel(), _p(part))
    return part


def bn_stats_from_partials(part, C, N, gamma, beta, eps, momentum, rmean, rvar, mean, invstd, scale, shift_out):
    call("ubpl_bn_stats_from_partials", _p(part), C, int(N), _p(gamma), _p(beta), float(eps), float(momentum),
         _p(rmean), _p(rvar), _p(mean), _p(invstd), _p(scale), _p(shift_out))


def bn_backward_split(dz, x, gamma, mean, invstd, scale, shift, relu, scratch, coef, dgamma, dbeta, npieces, pad,
                      part=None):
    """bn_backward with dx delivered as a SplitAct (PSA planes) only.  npieces 2
    (2xfp16): the pieces of dx times the power of two its bound asks for, kept on
    the device at coef[3C] — the SplitAct's `scale`, read by its consumers (so coef
    must not be reused before they are enqueued: stream order)."""
    B, C, H, W = x.shape
    plane = B * C * (H + 2 * pad) * (W + 2 * pad)
    out = torch.empty(npieces * plane, device=x.device, dtype=torch.int16)
    call("ubpl_bn_backward_split", _p(dz), _p(x), B, C, H, W, _p(gamma), _p(mean), _p(invstd), _p(scale), _p(shift),
         int(relu), _p(scratch), _p(part), _p(coef), _p(dgamma), _p(dbeta), int(pad), int(npieces), _p(out),
         int(plane))
    return SplitAct(out, plane, B, C, H, W, pad, npieces, coef[3 * C:3 * C + 1] if npieces == 2 else None)


def bn_backward(dz, x, gamma, mean, invstd, scale, shift, relu, scratch, coef, dgamma, dbeta, add1=None, add2=None,
                out=None, part=None):
    """BatchNorm(+ReLU) backward.  scratch: bn_part(B, C) (zeroed double
    scratch of the one-launch statistics); part: the backward partials dz's
    producer wrote (bn_bwd_partials layout) — then only the finalize runs."""
    B, C = x.shape[:2]
    HW = x[0, 0].numel()
    dx = dz if out is None else out
    call("ubpl_bn_backward", _p(dz), _p(x), B, C, HW, _p(gamma), _p(mean), _p(invstd), _p(scale), _p(shift),
         int(relu), _p(scratch), _p(part), _p(coef), _p(dgamma), _p(dbeta), _p(add1), _p(add2), _p(dx))
    return dx


def bn_bwd_partials(dz, x, scale, shift, mean, relu):
    """Backward statistics partials (S1, S2) per (channel, 64-pixel slice)."""
    B, C = x.shape[:2]
    HW = x[0, 0].numel()
    part = bn_partial_buffer(C, B * HW, x.device)
    call("ubpl_bn_backward_partials", _p(dz), _p(x), B, C, HW, _p(scale), _p(shift), _p(mean), int(relu), _p(part))
    return part


# ------------------------------------------------------------------ conv
def conv_out_hw(H, W, KS, stride):
    pad = (KS - 1) // 2
    return (H + 2 * pad - KS) // stride + 1, (W + 2 * pad - KS) // stride + 1


def conv_weight_tapmajor(w):
    Cout, Cin, KS, _ = w.shape
    wt = torch.empty((Cout, KS * KS, Cin), device=w.device, dtype=F32)
    call("ubpl_conv_weight_tapmajor", _p(w), Cout, Cin, KS, _p(wt))
    return wt


def conv2d_forward(x, w, bias, stride=1, pscale=None, pshift=None, res=None, out=None, w_tap=None):
    """w: reference layout [Cout,Cin,KS,KS] (re-laid out here for KS > 1) — or
    pass w_tap, an already re-laid-out copy viewed as [Cout,KS*KS,Cin] (its
    element order is ubpl_conv_weight_tapmajor's grouped tap-major layout)."""
    B, Cin, H, W = x.shape
    if w_tap is not None:
        Cout, T, wc = w_tap.shape
        KS = int(round(T ** 0.5))
        wk = w_tap
    else:
        Cout, wc, KS, _ = w.shape
        wk = w if KS == 1 else conv_weight_tapmajor(w)
    if wc != Cin:
        raise AssertionError("{} {}".format(Cin, wc))  # models/base/layers.py:44
    Ho, Wo = conv_out_hw(H, W, KS, stride)
    y = torch.empty((B, Cout, Ho, Wo), device=x.device, dtype=F32) if out is None else out
    nws = _lib.lib().ubpl_conv2d_forward_workspace(B, Cin, Cout, KS, Ho, Wo)
    slab = torch.empty(int(nws), device=x.device, dtype=F32) if nws > 0 else None
    call("ubpl_conv2d_forward", _p(x), B, Cin, H, W, _p(wk), _p(bias), Cout, KS, stride, _p(pscale), _p(pshift),
         _p(res), _p(y), Ho, Wo, _p(slab))
    return y


def conv1x1_kmajor_ok(x, cout):
    """Shapes / alignment the LDS-DMA 1x1 kernel takes (x: its B operand)."""
    return (x.shape[1] % 16 == 0 and cout % 4 == 0 and (x.shape[2] * x.shape[3]) % 4 == 0
            and x.data_ptr() % 16 == 0)


def conv1x1_forward_kmajor(x, wk, bias, pscale=None, pshift=None, res=None, out=None, stat_part=None):
    """1x1 stride-1 conv with k-major weights wk (Cin*Cout floats, [Cin][Cout]):
    y = conv(relu(x*pscale + pshift) or x) + bias (+ res; res may alias out);
    stat_part: BatchNorm partials of y (bn_partial_buffer)."""
    B, Cin, H, W = x.shape
    Cout = wk.numel() // Cin
    y = torch.empty((B, Cout, H, W), device=x.device, dtype=F32) if out is None else out
    nws = _lib.lib().ubpl_conv1x1_kmajor_workspace(B, Cin, Cout, H * W)
    slab = torch.empty(int(nws), device=x.device, dtype=F32) if nws > 0 else None
    call("ubpl_conv1x1_forward_kmajor", _p(x), B, Cin, H * W, _p(wk), _p(bias), Cout, _p(pscale), _p(pshift),
         _p(res), _p(y), _p(slab), _p(stat_part))
    return y


def conv2d_wgrad(dy, x, KS, stride, dw, db, pscale=None, pshift=None, accumulate=True):
    B, Cin, H, W = x.shape
    Cout, Ho, Wo = dy.shape[1], dy.shape[2], dy.shape[3]
    n = _lib.lib().ubpl_conv2d_wgrad_workspace(B, Cin, Cout, KS, Ho, Wo)
    slab = torch.empty(int(n), device=x.device, dtype=F32)
    call("ubpl_conv2d_wgrad", _p(dy), _p(x), B, Cin, H, W, Cout, KS, stride, _p(pscale), _p(pshift), Ho, Wo,
         _p(slab), _p(dw), _p(db), int(accumulate))


def wgrad1x1_split_load_ok(dy, x):
    B, Cin, H, W = x.shape
    return (dy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0
            and _lib.lib().ubpl_wgrad1x1_split_load_workspace(B, Cin, dy.shape[1], H * W) > 0)


def conv2d_wgrad1x1_split_load(dy, x, dw, db, pscale=None, pshift=None, accumulate=True, npieces=3):
    """1x1 weight (+ bias) gradient on the split path (npieces 3: 6xbf16; 1: bf16
    operands, f32 accumulation), f32 operands split on load (v = relu(x*pscale +
    pshift) when pscale is given)."""
    B, Cin, H, W = x.shape
    Cout = dy.shape[1]
    n = _lib.lib().ubpl_wgrad1x1_split_load_workspace(B, Cin, Cout, H * W)
    slab = torch.empty(int(n), device=x.device, dtype=F32)
    call("ubpl_wgrad1x1_split_load", _p(dy), _p(x), B, Cin, Cout, H * W, _p(pscale), _p(pshift), _p(slab), _p(dw),
         _p(db), int(accumulate), int(npieces))


def conv_weight_flip(w):
    """Data-gradient weights (stride 1), viewed as [Cin, KS*KS, Cout]."""
    Cout, Cin, KS, _ = w.shape
    wt = torch.empty((Cin, KS * KS, Cout), device=w.device, dtype=F32)
    call("ubpl_conv_weight_flip", _p(w), Cout, Cin, KS, _p(wt))
    return wt


def conv_weights_relayout(src, dst, table, mode):
    """table: int64 [nseg,5] device tensor (src_off, dst_off, Cout, Cin, T)."""
    call("ubpl_conv_weights_relayout", _p(src), _p(dst), _p(table), int(table.shape[0]), int(mode))


# Conv arithmetic: "f32" = exact-f32 MFMA (v_mfma_f32_32x32x2_f32); "6xbf16" =
# split-bf16 MFMA with 3 bf16 pieces per f32 operand (6 piece products, f32
# accumulation: exact operands); "2xfp16" = the forward convs (students' and
# teachers') with 2 fp16 pieces per operand of the power-of-two-scaled value (3
# piece products on the fp16 MFMA, operands to 2^-22: conv_split.hip / common.h
# split2), the backward (data and weight gradients, whose operands have no
# known range) on 6xbf16; "bf16" = one piece, i.e. both operands rounded to bf16
# (RNE) with f32 accumulation — the throughput precision of BASELINE config 5
# (8 stacks, 384x384), not parity-grade.  Value = the forward's pieces (0 for f32).
CONV_PRECISIONS = {"f32": 0, "bf16": 1, "2xfp16": 2, "6xbf16": 3}
# (round 6: 2xfp16 the default — every network-level parity test green on it, the step 17 % faster)
DEFAULT_CONV_PRECISION = "2xfp16"


def backward_pieces(pieces):
    """Pieces of the data / weight gradients' split operands for a precision's
    forward pieces (2xfp16: the backward runs on 6xbf16)."""
    return 3 if pieces == 2 else pieces


def conv_precision_name(name=None):
    import os
    return name or os.environ.get("UBPL_CONV_PRECISION", DEFAULT_CONV_PRECISION)


def conv_precision_pieces(name=None):
    """Pieces for a precision name (default: $UBPL_CONV_PRECISION or DEFAULT_CONV_PRECISION)."""
    import os
    name = name or os.environ.get("UBPL_CONV_PRECISION", DEFAULT_CONV_PRECISION)
    if name not in CONV_PRECISIONS:
        raise ValueError("conv precision %r not in %s" % (name, sorted(CONV_PRECISIONS)))
    return CONV_PRECISIONS[name]


class SplitWeights:
    """One conv's weights as `npieces` bf16 planes (conv_split.hip): a view into
    a shared buffer `buf` (int16, planes `plane` elements apart) at element
    offset `off`; shape = (rows, KS*KS, cols) of the GEMM A operand."""

    __slots__ = ("buf", "plane", "off", "shape", "npieces")

    def __init__(self, buf, plane, off, shape, npieces):
        self.buf, self.plane, self.off, self.shape, self.npieces = buf, plane, off, shape, npieces

    def ptr(self):
        """The planes' base as a tensor view at element offset `off`."""
        return self.buf[self.off:]


def conv_weights_split(src, dst, plane, table, mode, npieces):
    """Batched split re-layout (table as conv_weights_relayout, dst int16)."""
    call("ubpl_conv_weights_split", _p(src), _p(dst), int(plane), _p(table), int(table.shape[0]), int(mode),
         int(npieces))


def conv_weight_split(w, mode, npieces):
    """Single conv: SplitWeights for the forward (mode 0) or data gradient (mode 1)."""
    Cout, Cin, KS, _ = w.shape
    n = w.numel()
    plane = (n + 7) // 8 * 8
    buf = torch.empty(npieces * plane, device=w.device, dtype=torch.int16)
    tbl = torch.tensor([[0, 0, Cout, Cin, KS * KS]], dtype=torch.int64).to(w.device)
    conv_weights_split(w.contiguous(), buf, plane, tbl, mode, npieces)
    shape = (Cout, KS * KS, Cin) if mode == 0 else (Cin, KS * KS, Cout)
    return SplitWeights(buf, plane, 0, shape, npieces)


def conv2d_forward_split(x, ws, bias, pscale=None, pshift=None, res=None, out=None):
    """Split-bf16 MFMA conv (stride 1, KS in {1, 3}, Cin % 16 == 0); ws: SplitWeights."""
    B, Cin, H, W = x.shape
    Cout, T, wc = ws.shape
    KS = int(round(T ** 0.5))
    if wc != Cin:
        raise AssertionError("{} {}".format(Cin, wc))
    Ho, Wo = conv_out_hw(H, W, KS, 1)
    y = torch.empty((B, Cout, Ho, Wo), device=x.device, dtype=F32) if out is None else out
    nws = _lib.lib().ubpl_conv2d_forward_split_workspace(B, Cin, Cout, KS, Ho, Wo, ws.npieces)
    slab = torch.empty(int(nws), device=x.device, dtype=F32) if nws > 0 else None
    call("ubpl_conv2d_forward_split", _p(x), B, Cin, H, W, ws.ptr(), int(ws.plane), _p(bias), Cout, KS, 1,
         _p(pscale), _p(pshift), _p(res), _p(y), Ho, Wo, _p(slab), int(ws.npieces))
    return y


class SplitAct:
    """Pre-split activations (conv_split.hip PSA layout): `npieces` 16-bit planes of
    [B][C/16][H+2pad][W+2pad][16] in an int16 buffer, planes `plane` elements apart
    (3: bf16 pieces; 2: fp16 pieces of v * 32, the 2xfp16 path; 1: bf16(v))."""

    __slots__ = ("buf", "plane", "B", "C", "H", "W", "pad", "npieces", "scale")

    def __init__(self, buf, plane, B, C, H, W, pad, npieces, scale=None):
        self.buf, self.plane, self.B, self.C, self.H, self.W = buf, plane, B, C, H, W
        self.pad, self.npieces = pad, npieces
        # 2xfp16 images whose power-of-two scale lives on the device (a data gradient's: a
        # one-float tensor); None: the fixed activation scale (32) or no scale
        self.scale = scale


def split_activation(x, npieces, pad, pscale=None, pshift=None, out=None, with3=False):
    """x [B,C,H,W] f32 -> SplitAct of relu(x*pscale + pshift) (or x), zero border `pad`.
    with3 (npieces 2): (the 2xfp16 image, the 3-piece 6xbf16 image) from one read — the
    2xfp16 forward's conv input and the 6xbf16 weight gradient's operand."""
    B, C, H, W = x.shape
    plane = B * C * (H + 2 * pad) * (W + 2 * pad)
    if out is None:
        out = torch.empty(npieces * plane, device=x.device, dtype=torch.int16)
    out3 = None
    if with3:
        if npieces != 2:
            raise ValueError("with3: the 2xfp16 split only")
        out3 = torch.empty(3 * plane, device=x.device, dtype=torch.int16)
    call("ubpl_split_activation", _p(x), B, C, H, W, _p(pscale), _p(pshift), int(pad), int(npieces), _p(out),
         int(plane), _p(out3), int(plane))
    xs = SplitAct(out, plane, B, C, H, W, pad, npieces)
    return (xs, SplitAct(out3, plane, B, C, H, W, pad, 3)) if with3 else xs


def conv2d_forward_psa(xs, ws, bias, res=None, out=None, stat_part=None, bwd=None):
    """Stride-1 conv of pre-split activations xs (SplitAct) with SplitWeights ws;
    stat_part: BatchNorm partials of the output (bn_partial_buffer); bwd =
    (x, coef, relu, part): the output is dz of a BN with input x — its backward
    statistics partials into part."""
    Cout, T, wc = ws.shape
    KS = int(round(T ** 0.5))
    if wc != xs.C or ws.npieces != xs.npieces:
        raise AssertionError("{} {} / pieces {} {}".format(xs.C, wc, xs.npieces, ws.npieces))
    B, H, W = xs.B, xs.H, xs.W
    y = torch.empty((B, Cout, H, W), device=xs.buf.device, dtype=F32) if out is None else out
    nws = _lib.lib().ubpl_conv2d_forward_psa_workspace(B, xs.C, Cout, KS, H, W, ws.npieces)
    slab = torch.empty(int(nws), device=xs.buf.device, dtype=F32) if nws > 0 else None
    call("ubpl_conv2d_forward_psa", _p(xs.buf), int(xs.plane), B, xs.C, H, W, int(xs.pad), ws.ptr(), int(ws.plane),
         _p(bias), Cout, KS, _p(res), _p(y), _p(slab), int(ws.npieces), _p(stat_part), *_bnb(bwd), _p(xs.scale))
    return y


def stem_s2d_ok(x):
    B, C, H, W = x.shape
    return C <= 4 and H % 2 == 0 and W % 2 == 0 and (B * (H // 2) * (W // 2)) % 256 == 0


def stem_s2d_split(x, pad=2, npieces=3):
    """7x7/s2 stem input as the 16-channel PSA image of its 4 phase images
    (space-to-depth; channels c*4 + 2ph + pw, the rest zero), border `pad`;
    npieces 3 (6xbf16) or 1 (bf16)."""
    B, C, H, W = x.shape
    Ho, Wo = H // 2, W // 2
    plane = B * (Ho + 2 * pad) * (Wo + 2 * pad) * 16
    buf = torch.empty(npieces * plane, device=x.device, dtype=torch.int16)
    call("ubpl_stem_s2d_split", _p(x), B, C, H, W, int(pad), int(npieces), _p(buf), int(plane))
    return SplitAct(buf, plane, B, 16, Ho, Wo, pad, npieces)


def stem_weight_s2d_split(w, npieces=3):
    """The stem's 7x7 weights as the split 4x4 weights of its space-to-depth conv."""
    Cout, C, KS, _ = w.shape
    plane = Cout * 16 * 16
    buf = torch.empty(npieces * plane, device=w.device, dtype=torch.int16)
    call("ubpl_stem_weight_s2d_split", _p(w.contiguous()), Cout, C, KS, int(npieces), _p(buf), int(plane))
    return SplitWeights(buf, plane, 0, (Cout, 16, 16), npieces)


_NO_SOL = os.environ.get("UBPL_NO_SOL") == "1"      # diagnostic: every 1x1 on the exact-f32 kernels


# small=True (a model on the 2xfp16 precision): the split-load 1x1 also on grids below the chip's
# CU count, down to this many workgroups — the smaller planes' 1x1 convs were on the exact-f32
# kernel at 1/16 of the bf16 MFMA rate (-1 % step, profiles/r06_v8_sol_small_ab.txt); 0, and the
# other precisions: only grids that fill the chip (ubpl_conv1x1_split_load_preferred)
_SOL_MINWG = int(os.environ.get("UBPL_SOL_MINWG", "32"))


def conv1x1_split_load_ok(x, ws, small=False):
    """The split-on-load 1x1 kernel (6xbf16, 2xfp16 or bf16) takes this shape and fills the chip
    (small: on grids of >= _SOL_MINWG workgroups)."""
    B, Cin, H, W = x.shape
    ok = (not _NO_SOL and ws is not None and ws.npieces in (1, 2, 3) and ws.shape[1] == 1 and ws.shape[2] == Cin
          and x.data_ptr() % 16 == 0)
    if not ok:
        return False
    if small and _SOL_MINWG > 0 and ws.npieces in (2, 3):
        Cout, P = ws.shape[0], H * W
        N = B * P
        if not (Cin % 16 == 0 and Cout % 16 == 0 and P % 4 == 0 and N >= 4):
            return False
        bm = 128 if Cout % 128 == 0 and ((N + 255) // 256) * (Cout // 128) >= 256 else 64
        return ((N + 255) // 256) * ((Cout + bm - 1) // bm) >= _SOL_MINWG
    return bool(_lib.lib().ubpl_conv1x1_split_load_preferred(B, Cin, ws.shape[0], H * W))


def _bnb(bwd):
    """bwd = (x, coef, relu, part): backward BN partials from the epilogue (see
    ubpl_conv2d_forward_psa); coef = scale|shift|mean (3*C contiguous floats)."""
    if bwd is None:
        return None, None, 0, None
    x, coef, relu, part = bwd
    return _p(x), _p(coef), int(relu), _p(part)


def conv1x1_forward_split_load(x, ws, bias, pscale=None, pshift=None, res=None, out=None, stat_part=None,
                               bwd=None):
    """1x1 stride-1 conv on the split path (ws.npieces 3: 6xbf16; 2: 2xfp16; 1: bf16 operands)
    with x (NCHW f32) split while it is staged: y = conv(relu(x*pscale + pshift) or x, ws) + bias (+ res; res may
    alias out); ws = SplitWeights (rows, 1, Cin) — a forward (mode 0) or a data
    gradient (mode 1, x = dy) table; stat_part: BatchNorm partials of y."""
    B, Cin, H, W = x.shape
    Cout, T, wc = ws.shape
    if T != 1 or wc != Cin or ws.npieces not in (1, 2, 3) or (ws.npieces != 3 and (stat_part is not None or
                                                                               bwd is not None)):
        raise AssertionError("split-load 1x1: weights {} / pieces {} for {} input channels".format(
            ws.shape, ws.npieces, Cin))
    y = torch.empty((B, Cout, H, W), device=x.device, dtype=F32) if out is None else out
    call("ubpl_conv1x1_forward_split_load", _p(x), B, Cin, H * W, ws.ptr(), int(ws.plane), _p(bias), Cout,
         _p(pscale), _p(pshift), _p(res), _p(y), _p(stat_part), *_bnb(bwd), int(ws.npieces))
    return y


def wgrad3_psa_ok(ys, xs):
    return (ys.npieces in (1, 2, 3) and xs.npieces == ys.npieces and (ys.npieces != 2 or ys.scale is not None) and ys.pad == 1 and xs.pad == 1 and xs.C % 64 == 0
            and ys.C % 64 == 0 and xs.W % 16 == 0 and (ys.B, ys.H, ys.W) == (xs.B, xs.H, xs.W))


def conv2d_wgrad3_psa(ys, xs, dw, db, accumulate=True):
    """3x3 weight (+ bias) gradient from PSA operands: ys = split(dy), xs = split(conv input), pad 1."""
    n = _lib.lib().ubpl_wgrad3_psa_workspace(xs.B, xs.C, ys.C, xs.H, xs.W)
    slab = torch.empty(int(n), device=xs.buf.device, dtype=F32)
    call("ubpl_wgrad3_psa", _p(ys.buf), int(ys.plane), _p(xs.buf), int(xs.plane), xs.B, xs.C, ys.C, xs.H, xs.W,
         _p(slab), _p(dw), _p(db), int(accumulate), int(xs.npieces), _p(ys.scale))


def wgrad_stem_psa_ok(ys, xs, w):
    Cout, C, KS = w.shape[0], w.shape[1], w.shape[2]
    return (ys.npieces in (1, 3) and xs.npieces == ys.npieces and ys.pad == 1 and xs.pad == 2 and xs.C == 16 and KS == 7
            and C <= 4 and Cout % 64 == 0 and ys.C == Cout and ys.W % 16 == 0
            and (ys.B, ys.H, ys.W) == (xs.B, xs.H, xs.W))


def conv2d_wgrad_stem_psa(ys, xs, dw, db, accumulate=True):
    """The 7x7/s2 stem's weight (+ bias) gradient from PSA operands: ys = split(dy) (pad 1),
    xs = the forward's space-to-depth phase image (stem_s2d_split, pad 2)."""
    Cout, C, KS = dw.shape[0], dw.shape[1], dw.shape[2]
    n = _lib.lib().ubpl_wgrad_stem_psa_workspace(ys.B, Cout, ys.H, ys.W)
    slab = torch.empty(int(n), device=ys.buf.device, dtype=F32)
    call("ubpl_wgrad_stem_psa", _p(ys.buf), int(ys.plane), _p(xs.buf), int(xs.plane), ys.B, C, Cout, ys.H, ys.W, KS,
         _p(slab), _p(dw), _p(db), int(accumulate), int(ys.npieces))


def conv2d_dgrad(dy, w, res=None, out=None, wt=None):
    """dx of a stride-1 conv = conv(dy, flip(w)^T); res/out allow accumulation."""
    if wt is None:
        wt = conv_weight_flip(w)
    return conv2d_forward(dy, None, None, 1, res=res, out=out, w_tap=wt)


# ------------------------------------------------------------------ pool / upsample
def maxpool2x2(x, out=None, stat_part=None):
    """stat_part: BatchNorm partials of the output (bn_partial_buffer; needs
    (H/2)*(W/2) % 64 == 0, see stats_ok)."""
    B, C, H, W = x.shape
    y = torch.empty((B, C, H // 2, W // 2), device=x.device, dtype=F32) if out is None else out
    if stat_part is not None:
        call("ubpl_maxpool2x2_forward_stats", _p(x), B, C, H, W, _p(y), _p(stat_part))
    else:
        call("ubpl_maxpool2x2_forward", _p(x), B * C, H, W, _p(y))
    return y


def stats_ok(H, W):
    """Elementwise producers (max-pool, upsample-add) emit BatchNorm partials for planes of 64k pixels."""
    return (H * W) % 64 == 0


def maxpool2x2_backward(x, dy, dx, accumulate):
    B, C, H, W = x.shape
    call("ubpl_maxpool2x2_backward", _p(x), _p(dy), B * C, H, W, _p(dx), int(accumulate))
    return dx


def avgpool2x2(x, out=None):
    B, C, H, W = x.shape
    y = torch.empty((B, C, H // 2, W // 2), device=x.device, dtype=F32) if out is None else out
    call("ubpl_avgpool2x2_forward", _p(x), B * C, H, W, _p(y))
    return y


def avgpool2x2_backward(dy, dx, accumulate):
    B, C, H, W = dx.shape
    call("ubpl_avgpool2x2_backward", _p(dy), B * C, H, W, _p(dx), int(accumulate))
    return dx


def upsample2x_add(up, low, out=None, stat_part=None):
    """stat_part: BatchNorm partials of the output (H*W % 64 == 0)."""
    B, C, H, W = up.shape
    y = torch.empty_like(up) if out is None else out
    if stat_part is not None:
        call("ubpl_upsample2x_add_forward_stats", _p(up), _p(low), B, C, H, W, _p(y), _p(stat_part))
    else:
        call("ubpl_upsample2x_add_forward", _p(up), _p(low), B * C, H, W, _p(y))
    return y


def upsample2x_add_backward(dout, dlow, accumulate):
    B, C, H, W = dout.shape
    call("ubpl_upsample2x_add_backward", _p(dout), B * C, H, W, _p(dlow), int(accumulate))
    return dlow


def add(a, b, out=None):
    y = torch.empty_like(a) if out is None else out
    call("ubpl_add", _p(a), _p(b), a.numel(), _p(y))
    return y


# ------------------------------------------------------------------ f1
def image_mean_u8(imgs):
    """imgs uint8 [N,H,W,3] -> per-image mean / 255 (noisy_mean's mu), float32 [N]."""
    _chk(imgs, "imgs", torch.uint8)
    out = torch.empty(imgs.shape[0], device=imgs.device, dtype=F32)
    call("ubpl_image_mean_u8", _p(imgs), imgs.shape[0], imgs[0].numel(), _p(out))
    return out


def augment_warp(imgs, src_idx, mat, noise, img_mean, chan_mean, out):
    """One launch for V augmented views (see augment.hip): out [V,3,Ho,Wo]."""
    _chk(imgs, "imgs", torch.uint8)
    _chk(src_idx, "src_idx", torch.int32)
    for t, n in ((mat, "mat"), (noise, "noise"), (img_mean, "img_mean"), (chan_mean, "chan_mean"), (out, "out")):
        _chk(t, n)
    V, _, Ho, Wo = out.shape
    if mat.numel() != 6 * V or noise.numel() != 3 * V or src_idx.numel() != V:
        raise ValueError("augment_warp: per-view tables do not match %d views" % V)
    call("ubpl_augment_warp", _p(imgs), imgs.shape[1], imgs.shape[2], _p(src_idx), _p(mat), _p(noise),
         _p(img_mean), _p(chan_mean), V, Ho, Wo, _p(out))
    return out


def augment_chain(imgs, geo, cs, noise, img_mean, chan_mean, Hm, Wm, out):
    """The reference's two resamplings per view (see augment.hip
    ubpl_augment_chain): geo int32 [V,8] (src, flip, ul_x, ul_y, Hp, Wp, Hc, Wc),
    cs float32 [V,2] (cos, sin); out [V,3,Ho,Wo].  Stage-1 scratch [V,3,Hm,Wm]."""
    _chk(imgs, "imgs", torch.uint8)
    _chk(geo, "geo", torch.int32)
    for t, n in ((cs, "cs"), (noise, "noise"), (img_mean, "img_mean"), (chan_mean, "chan_mean"), (out, "out")):
        _chk(t, n)
    V, _, Ho, Wo = out.shape
    if geo.numel() != 8 * V or cs.numel() != 2 * V or noise.numel() != 3 * V:
        raise ValueError("augment_chain: per-view tables do not match %d views" % V)
    g = geo.reshape(V, 8).cpu() if geo.is_cuda else geo.reshape(V, 8)
    if (g[:, 6] > Hm).any() or (g[:, 7] > Wm).any() or (g[:, 6] < 1).any() or (g[:, 7] < 1).any() or \
            (g[:, 0] < 0).any() or (g[:, 0] >= imgs.shape[0]).any():
        raise ValueError("augment_chain: a view's stripped crop exceeds %dx%d or its source index is out of range"
                         % (Hm, Wm))
    # skimage.transform.resize anti-aliases a downscale with a Gaussian of sigma = (s - 1) / 2
    # (s = crop / output); the device resize omits it, which is exact to f32 only while its
    # off-centre weight exp(-1 / (2 sigma^2)) stays below f32 rounding: s <= 1.3 (2e-10 there;
    # the loaders' defaults draw s <= 1.25).  A larger crop would silently leave the reference.
    s = max(float((g[:, 6].double() / Ho).max()), float((g[:, 7].double() / Wo).max()))
    if s > 1.3:
        raise ValueError("augment_chain: a crop %.3fx the output size needs skimage's anti-aliasing blur "
                         "(sigma %.3f px), which the device resize does not run; crops up to 1.3x are exact"
                         % (s, (s - 1) / 2))
    inter = torch.empty((V, 3, Hm, Wm), device=out.device, dtype=F32)
    call("ubpl_augment_chain", _p(imgs), imgs.shape[1], imgs.shape[2], _p(geo), _p(cs), _p(noise), _p(img_mean),
         _p(chan_mean), V, int(Hm), int(Wm), _p(inter), Ho, Wo, _p(out))
    return out


def _occlude_check(V, H, W, nbank, off, hw, pastes, view_first):
    """Every index occlude_kernel derives from a paste row stays inside its
    buffer (host copies of the small tables; occlusion is opt-in)."""
    if not pastes.numel():
        return
    noff = off.numel()
    pr = pastes.reshape(-1, 9).cpu().numpy().astype("int64")
    vf = view_first.cpu().numpy().astype("int64")
    hwh = hw.reshape(-1, 2).cpu().numpy().astype("int64")
    if vf[0] != 0 or (vf[1:] < vf[:-1]).any() or vf[-1] != len(pr):
        raise ValueError("occlude: view_first is not a running count of %d paste rows" % len(pr))
    v, oc, w1, h1, x0, y0, x1, y1 = (pr[:, i] for i in range(8))
    sx0, sy0 = pr[:, 8] & 0xFFFF, pr[:, 8] >> 16
    bad = ((v < 0) | (v >= V) | (oc < 0) | (oc >= min(noff, len(hwh))) | (w1 <= 0) | (h1 <= 0)
           | (x0 < 0) | (y0 < 0) | (x1 > W) | (y1 > H) | (x1 < x0) | (y1 < y0)
           | (sx0 + (x1 - x0) > w1) | (sy0 + (y1 - y0) > h1))
    if bad.any():
        raise ValueError("occlude: paste row %d is out of range for %dx%d views / %d occluders" % (
            int(bad.nonzero()[0][0]), H, W, noff))
    h, w = hwh[oc, 0], hwh[oc, 1]
    if (h <= 0).any() or (w <= 0).any():
        raise ValueError("occlude: an occluder of the bank has an empty size")
    offh = off.cpu().numpy().astype("int64")[oc]
    if (offh < 0).any() or (offh + h * w * 4 > nbank).any():
        raise ValueError("occlude: an occluder reaches past the end of the bank")


def occlude(out, bank, off, hw, pastes, view_first, chan_mean):
    """Random occlusion pastes onto augmented views in place (see augment.hip
    occlude_kernel): out [V,3,H,W]; bank / off / hw: the occluder bank;
    pastes int32 [P,9] sorted by view; view_first int32 [V+1]."""
    _chk(out, "out")
    _chk(bank, "bank")
    _chk(off, "off", torch.int64)
    _chk(hw, "hw", torch.int32)
    _chk(pastes, "pastes", torch.int32)
    _chk(view_first, "view_first", torch.int32)
    _chk(chan_mean, "chan_mean")
    V, _, H, W = out.shape
    if view_first.numel() != V + 1 or (pastes.numel() and pastes.shape[-1] != 9):
        raise ValueError("occlude: paste table does not match %d views" % V)
    _occlude_check(V, H, W, bank.numel(), off, hw, pastes, view_first)
    call("ubpl_occlude", _p(out), V, H, W, _p(bank), _p(off), _p(hw), _p(pastes), _p(view_first), _p(chan_mean))
    return out
