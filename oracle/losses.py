"""L1-L7 — heatmap losses, UBPL pseudo mask, FDL, sample weights (oracle).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Torch CPU float32 restatements (autograd supplies the gradients the HIP
backward kernels are checked against).  Counts are returned as Python ints,
as the reference returns them.  Each function is vectorised over rows instead
of the reference's per-element Python loops; the semantics (which rows count,
which rows feed the score mean) are the reference's, cited per line.
"""
import torch


def _rows(x, nstack_axis, S, B, K):
    """[B,S,K,R,R] (or [B,K,R,R] when S==1 without a stack axis) -> [B,S,K,HW]."""
    if nstack_axis:
        return x.reshape(B, S, K, -1)
    return x.reshape(B, 1, K, -1)


def joint_mse(preds, gts, nstack=1, gate=None, sw=None, use_gate=False, use_sw=False):
    """JointMSELoss.forward (utils/losses.py:16-29).  preds [B,S,K,R,R]
    (or [B,K,R,R] when nstack == 1), gts [B,K,R,R], gate [B,K], sw [B,1].
    Returns (sum over s,b,k of the per-map pixel mean, nstack * #{gate>0})."""
    B = preds.shape[0]
    K = preds.shape[1] if nstack == 1 else preds.shape[2]
    g = torch.ones(B, K) if gate is None else gate.detach()           # :18
    n = int((g.reshape(-1) > 0).sum())                                 # utils/process.py:381-383
    p = _rows(preds, nstack != 1, nstack, B, K)
    t = gts.reshape(B, 1, K, -1)
    loss = ((p - t) ** 2).mean(-1)                                     # :24  [B,S,K]
    if use_gate:
        loss = loss * g[:, None, :]                                    # :25
    if use_sw and sw is not None:
        loss = loss * sw.reshape(B, 1, 1)                              # :26
    return loss.sum(), nstack * n                                      # :29


def joint_dist(p1, p2, nstack=1, gate=None, sw=None, use_gate=False, use_sw=False):
    """JointDistLoss.forward (utils/losses.py:40-53): MSE between two heatmap
    stacks; the count is nstack * #{gate>0} with gate = ones when None."""
    B = p1.shape[0]
    K = p1.shape[1] if nstack == 1 else p1.shape[2]
    g = torch.ones(B, K) if gate is None else gate.detach()
    n = int((g.reshape(-1) > 0).sum())
    a = _rows(p1, nstack != 1, nstack, B, K)
    b = _rows(p2, nstack != 1, nstack, B, K)
    loss = ((a - b) ** 2).mean(-1)
    if use_gate:
        loss = loss * g[:, None, :]
    if use_sw and sw is not None:
        loss = loss * sw.reshape(B, 1, 1)
    return loss.sum(), nstack * n


def joint_dist_mt2(p1, p2, nstack=1, gate=None, sw=None, use_gate=False, use_sw=False, thr=0.5):
    """JointDistLoss_mt2.forward (utils/losses.py:255-286): consistency masked by
    the TEACHER's per-map max >= thr.  n_pseudo counts rows whose weighted loss
    is > 0 before the mask (:273); n_sel counts mask rows (:274); the score is
    the mean teacher max over rows with sw > 0 (:275-280).  Raises RuntimeError
    (torch.stack of an empty list) when no row has sw > 0, as the reference."""
    B = p1.shape[0]
    K = p1.shape[1] if nstack == 1 else p1.shape[2]
    g = torch.ones(B, K) if gate is None else gate.detach()
    n = int((g.reshape(-1) > 0).sum())
    a = _rows(p1, nstack != 1, nstack, B, K)
    b = _rows(p2, nstack != 1, nstack, B, K)
    loss = ((a - b) ** 2).mean(-1)                                     # [B,S,K]
    if use_gate:
        loss = loss * g[:, None, :]
    if use_sw and sw is not None:
        loss = loss * sw.reshape(B, 1, 1)
    score = b.max(-1).values                                           # :270
    mask = (score >= thr).float()                                      # :271
    n_pseudo = int((loss > 0).sum())
    n_sel = int((mask > 0).sum())
    rows = sw.reshape(-1) > 0
    if int(rows.sum()) == 0:
        torch.stack([])                                                # :279 raises
    score_mean = score[rows].mean(0).mean(0)                           # :280, :285
    return (loss * mask).sum(), nstack * n, n_pseudo, n_sel, score_mean


def joint_pseudo3(preds, targets, sw, nstack=1, thr=0.5):
    """JointPseudoLoss3.forward (utils/losses.py:176-210) — the UBPL ensemble
    pseudo-label mask.  targets [M,B,S,K,R,R] (or [M,B,K,R,R] at nstack 1):
    T = mean over models of the last stack (:179); per stack s the loss
    mean_px((p_s - T)^2) * sw is kept where max_px(p_s) >= thr AND
    max_px(T) >= thr (:187-193).  Returns (sum, n_pseudo, n_sel, score[K],
    thr, thr)."""
    B = preds.shape[0]
    K = preds.shape[1] if nstack == 1 else preds.shape[2]
    T = (targets if nstack == 1 else targets[:, :, -1]).mean(0)        # :179
    Tr = T.reshape(B, 1, K, -1)
    p = _rows(preds, nstack != 1, nstack, B, K)
    loss = ((p - Tr) ** 2).mean(-1)                                    # :184  [B,S,K]
    if sw is not None:
        loss = loss * sw.reshape(B, 1, 1)                              # :185
    s1 = p.max(-1).values                                              # :187
    s2 = Tr.max(-1).values.expand(B, p.shape[1], K)                    # :190
    mask = (s1 >= thr).float() * (s2 >= thr).float()                   # :188-193
    n_pseudo = int((loss > 0).sum())                                   # :194
    n_sel = int((mask > 0).sum())                                      # :195
    rows = sw.reshape(-1) > 0                                          # :197
    if int(rows.sum()) == 0:
        torch.stack([])                                                # :201 raises
    per_s = (s1[rows].mean(0) + s2[rows].mean(0)) / 2                  # :203  [S,K]
    return (loss * mask).sum(), n_pseudo, n_sel, per_s.mean(0), thr, thr


def joint_feature_dist(f1, f2):
    """JointFeatureDistLoss.forward (utils/losses.py:61-70)."""
    bs, n = f1.shape[0], f1.shape[1]
    a = f1.reshape(bs, n, f1.shape[2], -1)
    b = f2.reshape(bs, n, f2.shape[2], -1)
    return ((a - b) ** 2).mean(-1).sum(), bs * n


def features_cov(f1, f2):
    """ProcessUtils.features_cov / torch_cov (utils/process.py:18-31): unbiased
    covariance of the two feature maps per (b, s, c), mean of |cov| over all
    (b, s, c); count = b*s*c."""
    bs, n, c = f1.shape[0], f1.shape[1], f1.shape[2]
    a = f1.reshape(bs, n, c, -1)
    b = f2.reshape(bs, n, c, -1)
    hw = a.shape[-1]
    ac = a - a.mean(-1, keepdim=True)
    bc = b - b.mean(-1, keepdim=True)
    cov = (ac * bc).sum(-1) / (hw - 1)
    return cov.abs().mean(), bs * n * c


# L7 sample weights (projects/tools.py:13-54), from islabeled [B] bool
def sample_weight(isl):
    return torch.where(isl, torch.ones(isl.shape[0]), torch.zeros(isl.shape[0]))[:, None]


def sample_weight_nega(isl, pw):
    return torch.where(isl, torch.zeros(isl.shape[0]), pw * torch.ones(isl.shape[0]))[:, None]


def sample_weight_cons(isl, pw):
    return torch.where(isl, torch.ones(isl.shape[0]), pw * torch.ones(isl.shape[0]))[:, None]
