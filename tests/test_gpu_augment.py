"""f1 — device augmentation (augment.hip).  The default two-stage path
(ubpl_augment_chain: the reference's integer crop -> skimage rotate -> skimage
resize, utils/augment.py:119-137) against oracle/augment_chain.py, the numpy /
scipy.ndimage restatement of scikit-image 0.20's two functions (skimage itself
is absent here: that restatement is unpinned against skimage, see its
header); the single-warp path (ubpl_augment_warp) against a numpy statement of
its own map.  The keypoint map is pinned bit-exact on the CPU
(test_cpu_host.py::test_augment_geometry_...)."""
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
    aug = DeviceAugment(imgs, means, device="cuda", two_stage=False)
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
    for two in (True, False):
        aug = DeviceAugment(imgs, means, sf=0.0, rf=0.0, use_flip=False, use_noise=False, device="cuda",
                            two_stage=two)
        out, _ = aug.views([1, 0], np.zeros((2, 9, 3), np.float32))
        want = np.transpose(imgs[[1, 0]].astype(np.float32) / 255., (0, 3, 1, 2)) - np.float32(0.4920829)
        assert np.abs(out.cpu().numpy() - want).max() < 1e-6, two


def test_two_stage_views_match_the_reference_chain():
    """Default path: each view equals the reference's own pixel chain (flip ->
    noisy_mean -> integer crop -> skimage rotate -> strip pad -> skimage resize
    -> colorNorm) as oracle/augment_chain.py restates it, to f32 rounding of the
    sample coordinates (crops up to 451 px: ~3e-5 px)."""
    from oracle import augment_chain as AC
    from ubpl_amd.augment import DeviceAugment
    rs = np.random.RandomState(5)
    # smooth images with sharp edges (a natural image's mix), not white noise
    yy, xx = np.mgrid[0:256, 0:256]
    imgs = np.stack([np.stack([(127 + 120 * np.sin(xx / (7.0 + 3 * i + c)) * np.cos(yy / (11.0 + i))
                                + 60 * ((xx + 2 * yy + 17 * i) % 97 < 40)).clip(0, 255)
                               for c in range(3)], -1) for i in range(4)]).astype(np.uint8)
    means = [0.45, 0.5, 0.55]
    aug = DeviceAugment(imgs, means, device="cuda")
    kps = np.zeros((8, 9, 3), np.float32)
    kps[:, :, :2] = rs.randint(20, 236, (8, 9, 2))
    kps[:, :, 2] = 1
    idx = [0, 1, 2, 3, 0, 1, 2, 3]
    random.seed(21)
    torch.manual_seed(21)
    draws = [aug._draw_geo(k) for k in kps]
    random.seed(21)
    torch.manual_seed(21)
    out, kout = aug.views(idx, kps)
    o = out.cpu().numpy()
    mu = aug.img_mean.cpu().numpy()
    rotated = 0
    for v, (_, noise, kk, ((flip, ulx, uly, Hp, Wp, Hc, Wc), (cs, sn))) in enumerate(draws):
        src = imgs[idx[v]].astype(np.float32) / np.float32(255.)
        if flip:
            src = src[:, ::-1]
        a, b, on = noise
        if on > 0:
            src = np.clip(np.float32(a) * (src - np.float32(mu[idx[v]])) + np.float32(mu[idx[v]]) + np.float32(b),
                          0, 1)
        pad = (Hp - Hc) // 2
        rotated += pad > 0
        angle = float(np.rad2deg(np.arctan2(sn, cs))) if pad else 0.0
        ref = AC.affine_view(src.astype(np.float64), (ulx, uly), (ulx + Wp, uly + Hp), pad, angle)
        ref = np.transpose(ref, (2, 0, 1)) - np.array(means)[:, None, None]
        d = np.abs(o[v] - ref)
        assert d.max() < 2e-4 and d.mean() < 2e-6, (v, d.max(), d.mean())
        assert np.array_equal(kout[v].cpu().numpy(), kk)
    assert rotated >= 4


def _area_resize(occ, w1, h1):
    """cv2.INTER_AREA's pixel-area relation (numpy, float64): resized pixel (rx, ry)
    averages the source over [rx*w/w1, (rx+1)*w/w1) x [ry*h/h1, (ry+1)*h/h1)."""
    h, w = occ.shape[:2]
    fx, fy = w / w1, h / h1

    def weights(n_out, n_in, f):
        m = np.zeros((n_out, n_in))
        for r in range(n_out):
            a0, a1 = r * f, (r + 1) * f
            for s in range(int(a0), min(n_in, int(np.ceil(a1)))):
                m[r, s] = min(a1, s + 1) - max(a0, s)
        return m / f
    return np.einsum("ys,sxc->yxc", weights(h1, h, fy), np.einsum("xs,ysc->yxc", weights(w1, w, fx), occ))


def test_occlusion_kernel_matches_numpy_statement():
    """f1 occlusion on the device (augment.hip occlude_kernel) against a numpy
    statement: each view gets its pastes in draw order, each paste the occluder
    resized by pixel-area averaging and alpha-blended onto the colorNorm'ed view;
    a paste at the occluder's own size equals the reference's paste_over
    (tests/golden/occlusion.npz, CPU test) on the normalised image."""
    from ubpl_amd import kernels as Kn
    from ubpl_amd import augment as AU
    from ubpl_amd.augment import OcclusionBank, draw_occlusion
    rs = np.random.RandomState(3)
    occ = [rs.uniform(0, 1, (h, w, 4)).astype(np.float32) for h, w in ((40, 31), (77, 64), (12, 20))]
    for o in occ:
        o[..., 3] = rs.choice([0.0, 192 / 255., 1.0], o.shape[:2])
    bank = OcclusionBank(occ, device="cuda")
    V, H, W = 5, 64, 80
    means = np.array([0.45, 0.5, 0.55], np.float32)
    base = rs.uniform(-0.5, 0.5, (V, 3, H, W)).astype(np.float32)
    random.seed(4)
    np.random.seed(4)
    pastes, first = [], [0]
    for v in range(V):
        ps = draw_occlusion(W, H, bank.sizes, aug_rate=1.0 if v < 4 else 0.0)
        if v == 0:                                    # plus a full-size paste (w1 = w, h1 = h: no resize)
            ps.append((1, 64, 77) + AU.paste_rect(np.array([35.0, 43.5]), 64, 77, W, H))
        pastes += [(v,) + p for p in ps]
        first.append(len(pastes))
    out = torch.from_numpy(base.copy()).cuda()
    pt = np.array([p[:8] + (p[8] | (p[9] << 16),) for p in pastes], np.int32)
    Kn.occlude(out, bank.bank, bank.off, bank.hw, torch.from_numpy(pt).cuda(),
               torch.tensor(first, dtype=torch.int32).cuda(), torch.from_numpy(means).cuda())
    ref = base.astype(np.float64).copy()
    for v, o, w1, h1, x0, y0, x1, y1, sx, sy in pastes:
        src = _area_resize(occ[o].astype(np.float64), w1, h1)[sy:sy + y1 - y0, sx:sx + x1 - x0]
        a = src[..., 3]
        for c in range(3):
            ref[v, c, y0:y1, x0:x1] = a * (src[..., c] - means[c]) + (1 - a) * ref[v, c, y0:y1, x0:x1]
    got = out.cpu().numpy()
    assert np.abs(got - ref).max() < 2e-5, np.abs(got - ref).max()
    assert np.array_equal(got[4], base[4])                        # a view without pastes is untouched
    assert len(pastes) > 6
