"""f1 — two-view augmentation of DS_mds on the device (augment.hip).

Per view, in the reference's order and with its random draws
(datasets/dataset_mds.py:88-113): fliplr with p 0.5 (utils/augment.py:216-227;
keypoints x -> W - x, centre x -> W - x), noisy_mean with p 0.5 (alpha
U(0.8, 1.2), beta U(-0.2, 0.2); :261-267), affine with scale =
scale0 * clamp(1 + sf * N(0,1), 1 - sf, 1 + sf) and angle = clamp(rf * N(0,1),
-rf, rf) (:86-98) — keypoints through utils/udaap/transforms.py:transform
(float64 matrix, int truncation, only where y > 0: utils/augment.py:150-156),
pixels through the same matrix inverted, folded with the flip into one 2x3
matrix per view for ubpl_augment_warp — and colorNorm (means, no std).  The
images never leave HBM; the host draws the random numbers and builds the
matrices (a few scalars per view), as the reference's loader does.
"""
import random

import numpy as np
import torch

from . import kernels as Kn


def get_transform(center, scale, res, rot=0.0):
    """utils/udaap/transforms.py:119-148 (float64)."""
    h = 200 * scale
    t = np.zeros((3, 3))
    t[0, 0] = float(res[1]) / h
    t[1, 1] = float(res[0]) / h
    t[0, 2] = res[1] * (-float(center[0]) / h + .5)
    t[1, 2] = res[0] * (-float(center[1]) / h + .5)
    t[2, 2] = 1
    if rot != 0:
        r = -rot * np.pi / 180
        sn, cs = np.sin(r), np.cos(r)
        rm = np.array([[cs, -sn, 0], [sn, cs, 0], [0, 0, 1.]])
        tm = np.eye(3)
        tm[0, 2], tm[1, 2] = -res[1] / 2, -res[0] / 2
        ti = tm.copy()
        ti[:2, 2] *= -1
        t = ti @ (rm @ (tm @ t))                                         # np.dot nesting of :147
    return t


def transform_point(pt, t):
    """utils/udaap/transforms.py:151-158 with a prebuilt matrix."""
    p = t @ np.array([pt[0] - 1, pt[1] - 1, 1.])
    return p[:2].astype(int) + 1


class DeviceAugment:
    """imgs: uint8 BGR [N,H,W,3] (numpy or device tensor); means: RGB-ordered
    channel means (MouseData.getSemiData)."""

    def __init__(self, imgs, means, inp_res=256, sf=0.25, rf=30.0, use_flip=True, use_noise=True, device="cuda"):
        self.imgs = torch.as_tensor(imgs).to(device).contiguous()
        self.N, self.H, self.W = self.imgs.shape[:3]
        self.res = inp_res
        self.sf, self.rf, self.use_flip, self.use_noise = sf, rf, use_flip, use_noise
        self.dev = torch.device(device)
        self.chan_mean = torch.tensor(means, dtype=torch.float32, device=self.dev)
        self.img_mean = Kn.image_mean_u8(self.imgs)

    def _draw(self, kps):
        """One view's random draws and keypoints (numpy [K,3] in, [K,3] out)."""
        W, H = self.W, self.H
        kps = kps.copy()
        center = [int(W / 2), int(H / 2)]                                # utils/process.py:218-221
        flip = False
        if self.use_flip and random.random() <= 0.5:                      # augment.py:218
            kps[:, 0] = W - kps[:, 0]                                      # process.py:239-242
            center[0] = W - center[0]
            flip = True
        noise = (1.0, 0.0, 0.0)
        if random.random() <= 0.5:                                        # augment.py:262
            a = random.uniform(0.8, 1.2)
            b = random.uniform(-0.2, 0.2)
            noise = (a, b, 1.0 if self.use_noise else 0.0)
        scale0 = self.res / 200.0
        scale = scale0 * float(torch.randn(1).mul_(self.sf).add_(1).clamp(1 - self.sf, 1 + self.sf)[0])
        angle = float(torch.randn(1).mul_(self.rf).clamp(-self.rf, self.rf)[0]) if random.random() <= 1.0 else 0.
        t = get_transform(center, scale, [self.res, self.res], rot=angle)
        for k in range(kps.shape[0]):
            if kps[k, 1] > 0:                                             # augment.py:153
                kps[k, :2] = transform_point(kps[k, :2], t)
        ti = np.linalg.inv(t)                                             # output (x, y) -> source, 0-based
        m = ti[:2].copy()
        if flip:                                                          # the source image is mirrored
            m[0] = -m[0]
            m[0, 2] += W - 1
        return m.reshape(-1), noise, kps

    def views(self, idx, kps):
        """idx: source image per view [V]; kps: numpy [V,K,3] pixel keypoints.
        -> (images [V,3,res,res] on the device, keypoints [V,K,3] on the device)."""
        mats, noises, out_k = [], [], []
        for k in kps:
            m, n, kk = self._draw(np.asarray(k, np.float32))
            mats.append(m)
            noises.append(n)
            out_k.append(kk)
        V = len(idx)
        idx = np.asarray(idx, np.int32)
        if idx.min() < 0 or idx.max() >= self.N:
            raise IndexError("DeviceAugment: source image index out of range")
        src = torch.tensor(idx, device=self.dev)
        mat = torch.tensor(np.array(mats, np.float32), device=self.dev)
        noise = torch.tensor(np.array(noises, np.float32), device=self.dev)
        out = torch.empty((V, 3, self.res, self.res), device=self.dev)
        Kn.augment_warp(self.imgs, src, mat, noise, self.img_mean, self.chan_mean, out)
        return out, torch.tensor(np.array(out_k, np.float32), device=self.dev)
