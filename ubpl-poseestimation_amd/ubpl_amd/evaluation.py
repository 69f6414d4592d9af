"""utils.evaluation drop-in: PCK on the HIP kernel (D4), plus the
utils/udaap/evaluation.py decoder entry points (D1-D2).
"""
import torch

from . import _lib
from . import kernels as Kn
from .process import inverse_transforms


def get_preds(scores):
    """utils/udaap/evaluation.py:13-30 (1-based argmax, zeroed where max <= 0)."""
    _lib.require_gpu()
    dev = scores.device
    raw, _, _ = Kn.decode_heatmaps(scores.detach().to("cuda", torch.float32).contiguous(), None)
    return raw.to(dev)


def final_preds(output, center, scale, res):
    """utils/udaap/evaluation.py:215-238."""
    _lib.require_gpu()
    dev = output.device
    tinv = inverse_transforms(center, scale, res).to("cuda")
    _, preds, _ = Kn.decode_heatmaps(output.detach().to("cuda", torch.float32).contiguous(), tinv)
    return preds.to(dev)


class EvaluationUtils:
    @classmethod
    def acc_pck(cls, preds, gts, pck_ref, pck_thr):
        """utils/evaluation.py:91-115 -> (errs [K+1], accs [K+1])."""
        errs, accs, _, _ = cls.acc_pck_counts(preds, gts, pck_ref, pck_thr)
        return errs, accs

    @classmethod
    def acc_pck_counts(cls, preds, gts, pck_ref, pck_thr):
        """acc_pck plus per-keypoint integer (hits, valid) counts for exact
        cross-rank aggregation."""
        _lib.require_gpu()
        dev = preds.device
        p = preds.detach().to("cuda", torch.float32).contiguous()
        g = gts.detach().to("cuda", torch.float32).contiguous()
        errs, accs, hits, valid = Kn.pck(p, g, pck_ref, pck_thr)
        return errs.to(dev), accs.to(dev), hits.to(dev), valid.to(dev)
