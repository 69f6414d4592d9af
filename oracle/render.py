"""R1 — per-keypoint Gaussian heatmap rendering (oracle).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates ProcessUtils.kps_heatmap / kps_heatmap_mulKps / heatmap_gaussian
(utils/process.py:252-278, 288-318, 393-397).  Arithmetic follows the
reference: visibility from the int32-truncated keypoint, centre from
int()-truncated coordinates divided by the stride, a full-grid float64
exp(-D2 / (2 sigma^2)), clamp >1 -> 1, zero below 0.01, cast to float32.
"""
import math

import numpy as np


def render_one(kps, img_hw, inp_res, out_res, kernel_size=3.0, sigma=1.0):
    """One sample.  kps: float32 [K,3] (x, y, vis); returns (hm [K,R,R] f32,
    kps with kps[:,2] *= visible) — the reference mutates kps in place
    (utils/process.py:267), this returns the updated copy."""
    kps = np.array(kps, dtype=np.float32, copy=True)
    h, w = img_hw
    stride = inp_res / out_res                      # utils/process.py:255
    size_h, size_w = int(h / stride), int(w / stride)
    sig = sigma * kernel_size                       # utils/process.py:258
    K = kps.shape[0]
    hm = np.zeros((K, size_h, size_w), np.float32)
    gy, gx = np.mgrid[0:size_h, 0:size_w]
    for k in range(K):
        # kp_int = kps.to(int32): truncation toward zero (utils/process.py:263)
        kx, ky = int(np.float32(kps[k, 0])), int(np.float32(kps[k, 1]))
        # int32 tensor - python float -> float32 tensor, int() truncates (:264-265)
        ul = (int(float(np.float32(kx - sig))), int(float(np.float32(ky - sig))))
        br = (int(float(np.float32(kx + sig + 1))), int(float(np.float32(ky + sig + 1))))
        vis = 0 if (br[0] >= w or br[1] >= h or ul[0] < 0 or ul[1] < 0) else 1
        kps[k, 2] = np.float32(kps[k, 2] * vis)       # :267
        cx = int(kps[k, 0]) * 1.0 / stride              # :270-271
        cy = int(kps[k, 1]) * 1.0 / stride
        d2 = (gx - cx) ** 2 + (gy - cy) ** 2            # :395 (float64)
        ker = np.exp(-d2 / 2.0 / sig / sig)
        ker[ker > 1] = 1                                # :274-275
        ker[ker < 0.01] = 0
        hm[k] = ker                                     # float64 -> float32
    return hm, kps


def render_batch(kps_b, img_hw, inp_res, out_res, kernel_size=3.0, sigma=1.0):
    """[B,K,3] -> ([B,K,R,R], kps_after [B,K,3]); the DataLoader renders one
    sample at a time (datasets/dataset_mds.py:115) and collates."""
    hms, ks = zip(*[render_one(k, img_hw, inp_res, out_res, kernel_size, sigma) for k in kps_b])
    return np.stack(hms), np.stack(ks)


def kps_heatmap_torch(kpsMap, imgShape, inpRes, outRes, kernelSize=3.0, sigma=1.0):
    """Same call shape as ProcessUtils.kps_heatmap (utils/process.py:253): torch
    in, (torch heatmap, torch kps) out; the kps tensor is updated in place."""
    import torch
    hm, k = render_one(kpsMap.numpy(), (imgShape[1], imgShape[2]), inpRes, outRes, kernelSize, sigma)
    kpsMap[:, 2] = torch.from_numpy(k[:, 2])
    return torch.from_numpy(hm), kpsMap
