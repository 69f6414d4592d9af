"""Test infrastructure (never imported by the product): a numpy restatement of
the reference's PIXEL path for one augmented view (utils/augment.py:86-137,
affine_image) with the two scikit-image resamplings it calls, so the device's
single bilinear warp (augment.hip, ubpl_amd/augment.py:warp_matrix) can be
measured against it.

scikit-image is not installed here (the reference pins scikit-image==0.20.0,
requirements.txt:39); its two functions are restated from their published
0.20 algorithms, on scipy.ndimage where skimage itself calls scipy.ndimage:

* skimage.transform.rotate(img, angle) (order 1, mode 'constant', cval 0,
  clip True): inverse map about c = (cols/2 - 0.5, rows/2 - 0.5),
  src = R(angle) (dst - c) + c with R = [[cos, -sin], [sin, cos]] on (col,
  row); bilinear from the floor / ceil neighbours, a neighbour outside the
  image reads cval; the result clipped to [min(img.min(), 0), max(img.max(),
  0)].
* skimage.transform.resize(img, (256, 256)) (order 1, mode 'reflect' ->
  ndimage 'mirror', clip True, anti_aliasing when any axis shrinks): a
  Gaussian of sigma_i = max(0, (in_i/out_i - 1) / 2) per axis (truncate 4,
  mirror edges), then ndimage.zoom(..., order=1, mode='mirror',
  grid_mode=True) — output pixel i samples (i + 0.5) * in/out - 0.5 — and the
  result clipped to the input's [min, max].

Parity of this restatement with skimage itself is unpinned (no skimage in the
image); the keypoint geometry it shares with the device path is pinned to the
reference's own transform() (tests/golden/augment.npz).
"""
import numpy as np


def crop_padded(image, ul, br):
    """The integer crop with zero fill of affine_image (utils/augment.py:119-129):
    image [H, W, C] float, ul / br the grown corners (ints)."""
    new = np.zeros((br[1] - ul[1], br[0] - ul[0], image.shape[2]))
    nx = max(0, -ul[0]), min(br[0], image.shape[1]) - ul[0]
    ny = max(0, -ul[1]), min(br[1], image.shape[0]) - ul[1]
    ox = max(0, ul[0]), min(image.shape[1], br[0])
    oy = max(0, ul[1]), min(image.shape[0], br[1])
    new[ny[0]:ny[1], nx[0]:nx[1]] = image[oy[0]:oy[1], ox[0]:ox[1]]
    return new


def sk_rotate(img, angle):
    """skimage.transform.rotate(img, angle) with its defaults (see module doc)."""
    rows, cols = img.shape[:2]
    cx, cy = cols / 2.0 - 0.5, rows / 2.0 - 0.5
    th = np.deg2rad(angle)
    r, c = np.mgrid[0:rows, 0:cols].astype(np.float64)
    sx = np.cos(th) * (c - cx) - np.sin(th) * (r - cy) + cx
    sy = np.sin(th) * (c - cx) + np.cos(th) * (r - cy) + cy
    x0, y0 = np.floor(sx).astype(int), np.floor(sy).astype(int)
    x1, y1 = np.ceil(sx).astype(int), np.ceil(sy).astype(int)
    dx, dy = sx - x0, sy - y0

    def px(y, x):
        ok = (y >= 0) & (y < rows) & (x >= 0) & (x < cols)
        out = np.zeros(y.shape + img.shape[2:])
        out[ok] = img[y[ok], x[ok]]
        return out
    w = (lambda a: a[..., None]) if img.ndim == 3 else (lambda a: a)
    top = (1 - w(dx)) * px(y0, x0) + w(dx) * px(y0, x1)
    bot = (1 - w(dx)) * px(y1, x0) + w(dx) * px(y1, x1)
    out = (1 - w(dy)) * top + w(dy) * bot
    return np.clip(out, min(img.min(), 0.0), max(img.max(), 0.0))


def sk_resize(img, shape):
    """skimage.transform.resize(img, shape) with its defaults (see module doc)."""
    from scipy import ndimage as ndi
    out_shape = tuple(shape) + img.shape[2:]
    factors = np.divide(img.shape, out_shape)
    lo, hi = img.min(), img.max()
    if any(o < i for o, i in zip(out_shape, img.shape)):
        img = ndi.gaussian_filter(img, np.maximum(0, (factors - 1) / 2), mode="mirror")
    out = ndi.zoom(img, [1 / f for f in factors], order=1, mode="mirror", grid_mode=True)
    return np.clip(out, lo, hi)


def affine_view(image, ul, br, pad, angle, res=(256, 256)):
    """affine_image's pixel path (utils/augment.py:103-137) for sf < 2 (no
    pre-resize: every scale the loaders draw, 256/200 * [0.75, 1.25]):
    crop with the grown box, rotate when angle != 0 and strip the pad, resize
    to res.  image [H, W, C] float in [0, 1] (flip and colour noise already
    applied, as the loader does before affine_mulKps)."""
    new = crop_padded(image, ul, br)
    if angle != 0:
        new = sk_rotate(new, angle)
        new = new[pad:-pad, pad:-pad]
    return sk_resize(new, res)


def single_warp(image, m, res=(256, 256)):
    """The device path's numpy twin (augment.hip augment_warp_kernel): one
    bilinear sample per output pixel through the 2x3 map m, zero outside."""
    H, W = image.shape[:2]
    ys, xs = np.mgrid[0:res[0], 0:res[1]].astype(np.float64)
    sx = m[0] * xs + m[1] * ys + m[2]
    sy = m[3] * xs + m[4] * ys + m[5]
    x0, y0 = np.floor(sx).astype(int), np.floor(sy).astype(int)
    wx, wy = (sx - x0)[..., None], (sy - y0)[..., None]

    def tap(x, y):
        ok = (x >= 0) & (x < W) & (y >= 0) & (y < H)
        r = np.zeros(res + image.shape[2:])
        r[ok] = image[y[ok], x[ok]]
        return r
    t00, t01, t10, t11 = tap(x0, y0), tap(x0 + 1, y0), tap(x0, y0 + 1), tap(x0 + 1, y0 + 1)
    top = t00 + wx * (t01 - t00)
    bot = t10 + wx * (t11 - t10)
    return top + wy * (bot - top)
