"""utils.losses drop-in: heatmap losses on the HIP kernels (L1-L4, L6).

Same class names, constructor arguments, call signatures and return tuples as
utils/losses.py (JointMSELoss :8, JointDistLoss :32, JointFeatureDistLoss :56,
JointPseudoLoss3 :169, JointDistLoss_mt2 :246, AvgCounter(s) :357-396).  Rows
follow the reference's reshape semantics exactly: with nStack == 1 a row is
(sample, preds.size(1)) — for a [B,1,K,R,R] model output that is one row per
sample over K*R*R pixels, as `preds.reshape((bs, k, -1))` makes it.

Counts are returned as Python ints, as the reference returns them; that costs
one device->host copy per call (the reference pays one per element).  The
fused training step (ubpl_amd.train) keeps counts on device instead.
"""
import torch
from torch import nn

from . import _lib
from . import kernels as Kn


def _rows_of(preds, nstack):
    """(B, S, K, HW) of the reference's reshape((bs, k, -1)) per stack."""
    B = preds.shape[0]
    if nstack == 1:
        K = preds.shape[1]
        return B, 1, K, preds.numel() // (B * K)
    K = preds.shape[2]
    return B, nstack, K, preds.numel() // (B * nstack * K)


def _geom(a, S, K, HW, t, t_sb, t_ss, t_sm, M, t_base=0):
    B = a.shape[0]
    g = Kn.RowGeom(a, S * K * HW, K * HW, t, t_sb, t_ss, t_sm, M, B, S, K, HW)
    g.t_ptr = t.reshape(-1)[t_base:]
    return g


class _RowLoss(torch.autograd.Function):
    """forward: (sum, cnt[4] int32, score[K]) on device; backward: d preds
    (and d targets for a same-layout target that requires grad)."""

    @staticmethod
    def forward(ctx, a, t, spec, gate, sw):
        kind, S, K, HW, tg, use_gate, use_sw, thr = spec
        g = _geom(a, S, K, HW, t, *tg)
        sq, am, tm = Kn.row_stats(g, want_amax=(kind == 2), want_tmax=(kind != 0))
        s, cnt, score, w = Kn.loss_finalize(kind, sq, am, tm, gate, sw, use_gate, use_sw, a.shape[0], S, K, thr)
        ctx.save_for_backward(a, t, w)
        ctx.spec = spec
        ctx.t_grad = t.requires_grad and tg[3] == 1 and tg[2] == 0
        outs = (s.view(()), cnt) + ((score,) if score is not None else (s.new_empty(0),))
        ctx.mark_non_differentiable(*outs[1:])
        return outs

    @staticmethod
    def backward(ctx, gs, _gc, _gsc):
        a, t, w = ctx.saved_tensors
        kind, S, K, HW, tg, _, _, _ = ctx.spec
        g = _geom(a, S, K, HW, t, *tg)
        da = torch.empty_like(a)
        Kn.row_grad(g, w, gs.reshape(1).contiguous().float(), 2.0 / HW, da)
        dt = -da if ctx.t_grad else None
        return da, dt, None, None, None


def _f32c(t):
    return None if t is None else t.detach().float().contiguous()


def _gate_rows(kpsGate, B, K, S):
    """Gate per loss row.  With nStack == 1 and [B,1,...] predictions the
    reference's rows are per sample (K == 1) while the gate is [B,Kg]:
    `loss.mul(kpsGate)` broadcasts [B,1] x [B,Kg] (utils/losses.py:25), i.e.
    each sample's loss is weighted by the SUM of its gates, and the count is
    still #{gate > 0} over the full gate (:18-19).  Returns (gate rows, count
    override or None)."""
    gate = _f32c(kpsGate)
    if gate is None or gate.shape[-1] == K:
        return gate, None
    if K != 1:
        raise RuntimeError("kpsGate %s does not broadcast against %d rows per sample" % (tuple(gate.shape), K))
    count = S * int((gate > 0).sum().item())
    return gate.reshape(B, -1).sum(1, keepdim=True).contiguous(), count


def _sw_vec(sw):
    return None if sw is None else sw.detach().float().reshape(-1).contiguous()


class JointMSELoss(nn.Module):
    """utils/losses.py:8-29 -> (sum over stacks/rows of the per-map pixel mean, nStack*#{gate>0})."""

    def __init__(self, nStack=1, useKPsGate=False, useSampleWeight=False):
        super().__init__()
        self.nStack, self.useKPsGate, self.useSampleWeight = nStack, useKPsGate, useSampleWeight

    def forward(self, preds, gts, kpsGate=None, sampleWeight=None):
        _lib.require_gpu(preds)
        a = preds.contiguous()
        B, S, K, HW = _rows_of(a, self.nStack)
        t = gts.detach().contiguous()
        if t.numel() != B * K * HW:
            raise RuntimeError("gts do not match preds rows")
        gate, count = _gate_rows(kpsGate, B, K, S)
        sw = _sw_vec(sampleWeight) if self.useSampleWeight else None
        spec = (0, S, K, HW, (K * HW, 0, 0, 1), bool(self.useKPsGate and gate is not None),
                bool(self.useSampleWeight and sw is not None), 0.0)
        s, cnt, _ = _RowLoss.apply(a, t, spec, gate, sw)
        return s, count if count is not None else int(cnt[0].item())


class JointDistLoss(nn.Module):
    """utils/losses.py:32-53 (Mean-Teacher consistency)."""

    def __init__(self, nStack=1, useKPsGate=False, useSampleWeight=False):
        super().__init__()
        self.nStack, self.useKPsGate, self.useSampleWeight = nStack, useKPsGate, useSampleWeight

    def forward(self, preds1, preds2, kpsGate=None, sampleWeight=None):
        _lib.require_gpu(preds1)
        a = preds1.contiguous()
        B, S, K, HW = _rows_of(a, self.nStack)
        t = preds2.contiguous()
        gate, count = _gate_rows(kpsGate, B, K, S)
        sw = _sw_vec(sampleWeight) if self.useSampleWeight else None
        spec = (0, S, K, HW, (S * K * HW, K * HW, 0, 1), bool(self.useKPsGate and gate is not None),
                bool(self.useSampleWeight and sw is not None), 0.0)
        s, cnt, _ = _RowLoss.apply(a, t, spec, gate, sw)
        return s, count if count is not None else int(cnt[0].item())


class JointDistLoss_mt2(nn.Module):
    """utils/losses.py:246-286: consistency kept where the second input's
    (teacher's) per-map max >= scoreThr.  Returns (sum, nStack*#gate,
    n_pseudo, n_sel, score[K])."""

    def __init__(self, nStack=1, useKPsGate=False, useSampleWeight=False, scoreThr=0.5):
        super().__init__()
        self.nStack, self.useKPsGate, self.useSampleWeight, self.scoreThr = nStack, useKPsGate, useSampleWeight, scoreThr

    def forward(self, preds1, preds2, kpsGate=None, sampleWeight=None):
        _lib.require_gpu(preds1)
        a = preds1.contiguous()
        B, S, K, HW = _rows_of(a, self.nStack)
        t = preds2.contiguous()
        gate = _f32c(kpsGate)
        sw = _sw_vec(sampleWeight)
        use_sw = bool(self.useSampleWeight and sw is not None)
        spec = (1, S, K, HW, (S * K * HW, K * HW, 0, 1), bool(self.useKPsGate and gate is not None), use_sw,
                float(self.scoreThr))
        # rows feeding the score are those with sampleWeight > 0 (utils/losses.py:276)
        s, cnt, score = _RowLoss.apply(a, t, spec, gate, sw if use_sw else sw)
        c = cnt.tolist()
        if c[3] == 0:
            raise RuntimeError("stack expects a non-empty TensorList")  # utils/losses.py:279
        return s, c[0], c[1], c[2], score


class JointPseudoLoss3(nn.Module):
    """utils/losses.py:169-210 — the UBPL ensemble pseudo-label loss with the
    per-(sample, keypoint) confidence mask."""

    def __init__(self, nStack=1, scoreThr=0.5):
        super().__init__()
        self.nStack, self.scoreThr = nStack, scoreThr

    def forward(self, preds, targets, sampleWeight):
        _lib.require_gpu(preds)
        a = preds.contiguous()
        B, S, K, HW = _rows_of(a, self.nStack)
        t = targets.detach().contiguous()
        M = t.shape[0]
        if self.nStack == 1:
            tg = (K * HW, 0, t.numel() // M, M)
            base = 0
        else:
            St = t.shape[2]
            tg = (St * K * HW, 0, B * St * K * HW, M)
            base = (St - 1) * K * HW
        sw = _sw_vec(sampleWeight)
        spec = (2, S, K, HW, tg + (base,), False, True, float(self.scoreThr))
        s, cnt, score = _RowLoss.apply(a, t, spec, None, sw)
        c = cnt.tolist()
        if c[3] == 0:
            raise RuntimeError("stack expects a non-empty TensorList")  # utils/losses.py:201
        return s, c[1], c[2], score, self.scoreThr, self.scoreThr


class JointFeatureDistLoss(nn.Module):
    """utils/losses.py:56-70 (FDL_type 'distance')."""

    def forward(self, inp1, inp2):
        _lib.require_gpu(inp1)
        bs, n, c = inp1.shape[:3]
        a = inp1.contiguous()
        t = inp2.contiguous()
        HW = a.numel() // (bs * n * c)
        spec = (0, 1, n * c, HW, (n * c * HW, 0, 0, 1), False, False, 0.0)
        s, _, _ = _RowLoss.apply(a, t, spec, None, None)
        return s, bs * n


class _FeaturesCov(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f1, f2, rowmask):
        val, cnt, saved = Kn.fdl_cov_forward(f1, f2, rowmask)
        ctx.save_for_backward(f1, f2, cnt, *saved)
        ctx.rowmask = rowmask
        ctx.mark_non_differentiable(cnt)
        return val.view(()), cnt

    @staticmethod
    def backward(ctx, gv, _gc):
        f1, f2, cnt, cov, mu1, mu2 = ctx.saved_tensors
        d1 = torch.empty_like(f1) if ctx.needs_input_grad[0] else None
        d2 = torch.empty_like(f2) if ctx.needs_input_grad[1] else None
        Kn.fdl_cov_backward(f1, f2, ctx.rowmask, (cov, mu1, mu2), cnt, gv.reshape(1).contiguous().float(), d1, d2)
        return d1, d2, None


def features_cov(inp1, inp2, rowmask=None):
    """ProcessUtils.features_cov (utils/process.py:18-31) on device.  With a
    rowmask [B] (>0 = selected) the selection of projects/MT_UBPL.py:309-320 is
    fused in; the count is returned as a device int32[1]."""
    _lib.require_gpu(inp1)
    return _FeaturesCov.apply(inp1.contiguous(), inp2.contiguous(), _f32c(rowmask))


class AvgCounter(object):
    """utils/losses.py:357-371 (host-side running mean)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = 0. if self.count == 0 else self.sum / self.count


class AvgCounters(object):
    """utils/losses.py:374-396."""

    def __init__(self, num=1):
        self.counters = [AvgCounter() for _ in range(num)]
        self.reset()

    def reset(self):
        for c in self.counters:
            c.reset()

    def update(self, idx, val, n=1):
        self.check_idx(idx)
        self.counters[idx].update(val, n)

    def avg(self):
        return [c.avg for c in self.counters]

    def sum(self):
        return [c.sum for c in self.counters]

    def check_idx(self, idx):
        while len(self.counters) < idx + 1:
            self.counters.append(AvgCounter())
