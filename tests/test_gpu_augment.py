"""f1 — device augmentation (augment.hip) against a numpy statement of the
same map: bilinear sampling of the (flipped, noisy_mean-adjusted) uint8 BGR
source at the host-built 2x3 matrix, zero outside, minus the channel means.
skimage (the reference's resize/rotate) is absent here, so parity with the
reference's pixels is statistical; the keypoint map is pinned
bit-exact on the CPU (test_cpu_host.py::test_augment_geometry_...)."""
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref_warp(img, m, noise, mu, means):
    H, W, _ = img.shape
    v = img.astype(np.float64) / 255.
    a, b, on = noise
    if on > 0:
        v = np.clip(a * (v - mu) + mu + b, 0, 1)
    out = np.zeros((3, 256, 256))
    ys, xs = np.mgrid[0:256, 0:256].astype(np.float64)
    sx = m[0] * xs + m[1] * ys + m[2]
    sy = m[3] * xs + m[4] * ys + m[5]
    x0, y0 = np.floor(sx).astype(int), np.floor(sy).astype(int)
    wx, wy = sx - x0, sy - y0

    def tap(x, y):
        ok = (x >= 0) & (x < W) & (y >= 0) & (y < H)
        r = np.zeros((256, 256, 3))
        r[ok] = v[y[ok], x[ok]]
        return r
    t00, t01, t10, t11 = tap(x0, y0), tap(x0 + 1, y0), tap(x0, y0 + 1), tap(x0 + 1, y0 + 1)
    top = t00 + wx[..., None] * (t01 - t00)
    bot = t10 + wx[..., None] * (t11 - t10)
    val = top + wy[..., None] * (bot - top)
    return np.transpose(val, (2, 0, 1)) - np.array(means)[:, None, None]


def test_augment_views_match_numpy_statement():
    from ubpl_amd.augment import DeviceAugment
    rs = np.random.RandomState(0)
    imgs = rs.randint(0, 256, (5, 256, 256, 3)).astype(np.uint8)
    means = [0.45, 0.5, 0.55]
    aug = DeviceAugment(imgs, means, device="cuda")
    random.seed(3)
    torch.manual_seed(3)
    kps = np.zeros((6, 9, 3), np.float32)
    kps[:, :, :2] = rs.randint(20, 236, (6, 9, 2))
    kps[:, :, 2] = 1
    kps[5] = 0                                                # an unlabeled row stays unlabeled
    idx = [0, 1, 2, 3, 4, 0]
    random.seed(11)
    torch.manual_seed(11)
    draws = [aug._draw(k) for k in kps]
    random.seed(11)
    torch.manual_seed(11)
    out, kout = aug.views(idx, kps)
    mu = aug.img_mean.cpu().numpy()
    assert np.allclose(mu, imgs.reshape(5, -1).mean(1) / 255., rtol=1e-6)
    o = out.cpu().numpy()
    for v, (m, noise, kk) in enumerate(draws):
        ref = _ref_warp(imgs[idx[v]], m.astype(np.float32).astype(np.float64), noise, float(mu[idx[v]]), means)
        assert np.abs(o[v] - ref).max() < 1e-4, v          # float32 source coordinates in the kernel
        assert np.array_equal(kout[v].cpu().numpy(), kk)
    assert np.array_equal(kout[5].cpu().numpy()[:, 1:], np.zeros((9, 2), np.float32))


def test_identity_view_is_the_normalised_image():
    from ubpl_amd.augment import DeviceAugment
    rs = np.random.RandomState(1)
    imgs = rs.randint(0, 256, (2, 256, 256, 3)).astype(np.uint8)
    means = [0.4920829] * 3
    aug = DeviceAugment(imgs, means, sf=0.0, rf=0.0, use_flip=False, use_noise=False, device="cuda")
    out, _ = aug.views([1, 0], np.zeros((2, 9, 3), np.float32))
    want = np.transpose(imgs[[1, 0]].astype(np.float32) / 255., (0, 3, 1, 2)) - np.float32(0.4920829)
    assert np.abs(out.cpu().numpy() - want).max() < 1e-6
