"""D1-D5 — argmax decoder, affine back-transform, PCK (oracle).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

get_preds      utils/udaap/evaluation.py:13-30
final_preds    utils/udaap/evaluation.py:215-238 (+ transforms.py:119-168)
acc_pck        utils/evaluation.py:91-139
AvgCounter(s)  utils/losses.py:357-396
"""
import numpy as np
import torch


def get_preds(scores):
    """[B,K,R,R] -> [B,K,2] float32 1-based (col, row), zeroed where the map max
    is not > 0.  torch.max returns the FIRST maximal index (:18)."""
    B, K, H, W = scores.shape
    flat = scores.reshape(B, K, -1)
    maxval, idx = torch.max(flat, 2)
    idx = idx.float() + 1                                            # :21
    preds = torch.stack([(idx - 1) % W + 1, torch.floor((idx - 1) / W) + 1], -1)   # :25-26
    return preds * (maxval > 0).float()[..., None]                    # :28-29


def transform_matrix(center, scale, res):
    """get_transform (transforms.py:119-148) at rot=0 with the reference's
    precision: scale is a float32 tensor, so h = 200*scale and every entry is
    float32 arithmetic, stored into a float64 matrix."""
    s = torch.as_tensor(scale, dtype=torch.float32)
    h = 200 * s                                                       # :125
    t = np.zeros((3, 3))
    t[0, 0] = float(res[1]) / h
    t[1, 1] = float(res[0]) / h
    t[0, 2] = res[1] * (-float(center[0]) / h + .5)
    t[1, 2] = res[0] * (-float(center[1]) / h + .5)
    t[2, 2] = 1
    return t


def inverse_transform(center, scale, res):
    """np.linalg.inv of the matrix above (transforms.py:155)."""
    return np.linalg.inv(transform_matrix(center, scale, res))


def transform_point(pt, tinv):
    """transforms.py:156-158: tinv . [x-1, y-1, 1], astype(int) (truncation), +1."""
    v = np.array([np.float64(pt[0]) - 1, np.float64(pt[1]) - 1, 1.])
    r = np.dot(tinv, v)
    return r[:2].astype(int) + 1


def final_preds(output, center, scale, res):
    """utils/udaap/evaluation.py:215-238 -> [B,K,2] float32 (integer valued)."""
    coords = get_preds(output)
    preds = coords.clone()
    for i in range(coords.shape[0]):
        tinv = inverse_transform(center[i], scale[i], res)
        for p in range(coords.shape[1]):
            preds[i, p] = torch.from_numpy(transform_point(coords[i, p].numpy(), tinv).astype(np.float32))
    return preds


def kps_from_heatmap(heatmap, center, scale, res):
    """ProcessUtils.kps_fromHeatmap mode 'batch' (utils/process.py:320-327)."""
    preds = final_preds(heatmap, center, scale, res)
    scores = torch.from_numpy(np.max(heatmap.numpy(), axis=(2, 3)).astype(np.float32))
    return preds, scores


def acc_pck(preds, gts, pck_ref, pck_thr):
    """EvaluationUtils.acc_pck (utils/evaluation.py:91-115) with _acc_calDists
    (:118-131) and _acc_counting (:134-139).  The per-keypoint error average
    divides by B INCLUDING the -1 sentinels of invalid rows (:99-101)."""
    B, K, _ = preds.shape
    dists = torch.zeros(K, B)
    dref = torch.zeros(K, B)
    for b in range(B):
        norm = torch.dist(gts[b, pck_ref[0], 0:2], gts[b, pck_ref[1], 0:2])
        for k in range(K):
            if gts[b, k, 0] > 1 and gts[b, k, 1] > 1:
                d = torch.dist(preds[b, k, 0:2], gts[b, k, 0:2])
                dists[k, b] = d
                dref[k, b] = d / norm
            else:
                dists[k, b] = -1
                dref[k, b] = -1
    errs = torch.zeros(K + 1)
    esum, enum = 0, 0
    for k in range(K):
        errs[k] = dists[k].sum() / B
        esum += errs[k]
        enum += 1
    errs[-1] = esum / enum
    accs = torch.zeros(K + 1)
    asum, anum = 0, 0
    for k in range(K):
        v = dref[k][dref[k] != -1]
        accs[k] = (1.0 * (v < pck_thr).sum().item() / len(v)) if len(v) > 0 else -1
        if accs[k] >= 0:
            asum += accs[k]
            anum += 1
    if anum != 0:
        accs[-1] = asum / anum
    return errs, accs


class AvgCounter:
    """utils/losses.py:357-371."""

    def __init__(self):
        self.val = self.avg = self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = 0. if self.count == 0 else self.sum / self.count
