"""f1 — two-view augmentation of DS_mds on the device (augment.hip).

Per view, in the reference's order and with its random draws
(datasets/dataset_mds.py:88-113): fliplr with p 0.5 (utils/augment.py:216-227;
keypoints x -> W - x, centre x -> W - x), noisy_mean with p 0.5 (alpha
U(0.8, 1.2), beta U(-0.2, 0.2); :261-267), affine with scale =
scale0 * clamp(1 + sf * N(0,1), 1 - sf, 1 + sf) and angle = clamp(rf * N(0,1),
-rf, rf) (:18-22) — float32 TENSORS, as the loader builds them
(dataset_mds.py:60-61) — keypoints through utils/udaap/transforms.py:transform
with the reference's operand types (float32 matrix entries and sin/cos,
float64 products, int truncation, only where y > 0: utils/augment.py:150-156),
pixels through the reference's crop -> rotate -> resize geometry
(utils/augment.py:103-137) folded with the flip into one 2x3 matrix per view
for ubpl_augment_warp — and colorNorm (means, no std).  The images never
leave HBM; the host draws the random numbers and builds the matrices (a few
scalars per view), as the reference's loader does.
"""
import random

import numpy as np
import torch

from . import kernels as Kn

F32 = torch.float32


def get_transform(center, scale, res, rot=0.0):
    """utils/udaap/transforms.py:119-148 with the loader's operand types:
    scale and rot are float32 0-d tensors (datasets/dataset_mds.py:60-61,
    utils/augment.py:19-20), so h = 200*scale, every matrix entry and
    sin/cos(rot) are float32 values (torch's `float / tensor` is reciprocal(tensor)
    * float; numpy's float32 sin/cos on the tensor), stored into the float64
    matrix whose products (np.dot) are float64.  Python floats are promoted to
    float32 tensors the same way."""
    scale = torch.as_tensor(scale, dtype=F32)
    h = 200 * scale
    t = np.zeros((3, 3))
    t[0, 0] = float(float(res[1]) / h)
    t[1, 1] = float(float(res[0]) / h)
    t[0, 2] = float(res[1] * (-float(center[0]) / h + .5))
    t[1, 2] = float(res[0] * (-float(center[1]) / h + .5))
    t[2, 2] = 1
    rot = torch.as_tensor(rot, dtype=F32)
    if not bool(rot == 0):
        r = -rot
        r = r * np.pi / 180
        sn, cs = float(np.sin(r.numpy())), float(np.cos(r.numpy()))    # numpy float32 sin/cos, as on the tensor
        rm = np.zeros((3, 3))
        rm[0, :2] = [cs, -sn]
        rm[1, :2] = [sn, cs]
        rm[2, 2] = 1
        tm = np.eye(3)
        tm[0, 2], tm[1, 2] = -res[1] / 2, -res[0] / 2
        ti = tm.copy()
        ti[:2, 2] *= -1
        t = np.dot(ti, np.dot(rm, np.dot(tm, t)))                        # :147
    return t


def transform_point(pt, t, invert=False):
    """utils/udaap/transforms.py:151-158 with a prebuilt matrix: pt is a row of
    the float32 keypoint tensor, so pt - 1 is a float32 subtraction; the
    product is float64, truncated to int, + 1."""
    if invert:
        t = np.linalg.inv(t)
    if torch.is_tensor(pt):
        x, y = float(pt[0] - 1), float(pt[1] - 1)
    else:
        x, y = pt[0] - 1, pt[1] - 1
    p = np.dot(t, np.array([x, y, 1.]))
    return p[:2].astype(int) + 1


def crop_box(center, scale, res, angle):
    """The integer crop of affine_image (utils/augment.py:103-129): corners
    ul = transform([0, 0], invert=1), br = transform(res, invert=1) of the
    UNROTATED transform, then grown by pad = int(|br - ul| / 2 - (br_y - ul_y)
    / 2) on every side when angle != 0.  Returns (ul, br, pad) as ints (ul, br
    after the growth)."""
    ti = np.linalg.inv(get_transform(center, scale, res, 0))
    ul = transform_point([0, 0], ti)
    br = transform_point(list(res), ti)
    pad = int(np.linalg.norm(br - ul) / 2 - float(br[1] - ul[1]) / 2)
    if not bool(torch.as_tensor(angle, dtype=F32) == 0):
        ul = ul - pad
        br = br + pad
    else:
        pad = 0
    return ul, br, pad


def warp_matrix(center, scale, res, angle, W, flip=False):
    """2x3 map from output pixel (x, y) (0-based) to the source pixel it
    samples (0-based, of the unflipped source image of width W) — the
    reference's pixel path composed into one affine map
    (utils/augment.py:103-137):
      1. resize of the stripped crop (Hc x Wc) to res, skimage's pixel-centre
         convention: src = (dst + 0.5) * (crop / res) - 0.5;
      2. strip of the rotation pad: + pad;
      3. skimage.transform.rotate(angle) of the padded crop (H' x W'): inverse
         map about c = ((W'-1)/2, (H'-1)/2), p = c + R(angle) (q - c),
         R = [[cos, -sin], [sin, cos]];
      4. the integer crop: + (ul_x, ul_y) of the grown box;
      5. the fliplr that happened before it: x -> W - 1 - x.
    What one bilinear sample cannot restate (two resamplings in the
    reference, skimage's anti-aliasing Gaussian when the crop is larger than
    res, reflect-mode edges of the resize) is documented in DESIGN.md §1 f1."""
    ul, br, pad = crop_box(center, scale, res, angle)
    Hp, Wp = br[1] - ul[1], br[0] - ul[0]                  # the (padded) crop
    Hc, Wc = Hp - 2 * pad, Wp - 2 * pad                   # after stripping the pad
    M = np.array([[Wc / res[1], 0, 0.5 * Wc / res[1] - 0.5],
                  [0, Hc / res[0], 0.5 * Hc / res[0] - 0.5], [0, 0, 1.]])
    M = np.array([[1, 0, pad], [0, 1, pad], [0, 0, 1.]]) @ M
    if pad:
        th = np.deg2rad(float(torch.as_tensor(angle, dtype=F32)))
        c = np.array([(Wp - 1) / 2.0, (Hp - 1) / 2.0])
        R = np.array([[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1.]])
        Tc = np.array([[1, 0, c[0]], [0, 1, c[1]], [0, 0, 1.]])
        Tm = np.array([[1, 0, -c[0]], [0, 1, -c[1]], [0, 0, 1.]])
        M = Tc @ R @ Tm @ M
    M = np.array([[1, 0, ul[0]], [0, 1, ul[1]], [0, 0, 1.]]) @ M
    if flip:
        M = np.array([[-1, 0, W - 1], [0, 1, 0], [0, 0, 1.]]) @ M
    return M[:2]


def chain_geometry(center, scale, res, angle, flip):
    """The per-view table of ubpl_augment_chain (the reference's two
    resamplings): (flip, ul_x, ul_y, Hp, Wp, Hc, Wc) — the grown integer crop
    box of affine_image (corner, padded size) and its size after the pad is
    stripped — and (cos, sin) of the angle in float64 from its float32 value
    (skimage.transform.rotate's SimilarityTransform)."""
    ul, br, pad = crop_box(center, scale, res, angle)
    Hp, Wp = int(br[1] - ul[1]), int(br[0] - ul[0])
    th = np.deg2rad(float(torch.as_tensor(angle, dtype=F32))) if pad else 0.0
    return ((int(flip), int(ul[0]), int(ul[1]), Hp, Wp, Hp - 2 * pad, Wp - 2 * pad),
            (float(np.cos(th)), float(np.sin(th))))


def draw_view(kps, W, H, res_in, sf, rf, use_flip=True, use_noise=True, with_geometry=False):
    """One view's random draws (python `random`, then torch's CPU
    generator, in the reference loader's order) and keypoints (numpy [K,3]
    in, [K,3] out), with the loader's types: keypoints float32 tensors,
    centre ints, scale and angle float32 0-d tensors.  Host-only (no GPU):
    -> (2x3 warp matrix flattened, noisy_mean (alpha, beta, on), keypoints)."""
    kps = torch.tensor(np.asarray(kps, np.float32))
    center = [int(W / 2), int(H / 2)]                                # utils/process.py:218-221
    flip = False
    if use_flip and random.random() <= 0.5:                      # augment.py:218
        kps[:, 0] = W - kps[:, 0]                                      # process.py:239-242 (float32)
        center[0] = W - center[0]
        flip = True
    noise = (1.0, 0.0, 0.0)
    if random.random() <= 0.5:                                        # augment.py:262
        a = random.uniform(0.8, 1.2)
        b = random.uniform(-0.2, 0.2)
        noise = (a, b, 1.0 if use_noise else 0.0)
    scale = torch.tensor(res_in / 200.0)                            # dataset_mds.py:61 (float32)
    scale = scale * torch.randn(1).mul_(sf).add_(1).clamp(1 - sf, 1 + sf)[0]   # augment.py:19
    angle = torch.tensor(0.)                                          # dataset_mds.py:60
    angle = angle + torch.randn(1).mul_(rf).clamp(-rf, rf)[0] \
        if random.random() <= 1.0 else 0.                              # augment.py:20
    res = [res_in, res_in]
    t = get_transform(center, scale, res, rot=angle)
    out = kps.clone()
    for k in range(kps.shape[0]):
        if kps[k, 1] > 0:                                             # augment.py:153
            out[k, :2] = torch.from_numpy(transform_point(kps[k, :2], t))
    m = warp_matrix(center, scale, res, angle, W, flip)
    if with_geometry:
        return m.reshape(-1), noise, out.numpy(), chain_geometry(center, scale, res, angle, flip)
    return m.reshape(-1), noise, out.numpy()


# ---------------------------------------------------------------------------
# random occlusion (utils/udaap/utils_augment.py) — off by default in the
# reference (useOcclusion False, projects/MT_UBPL.py:473)
# ---------------------------------------------------------------------------
def _ellipse_8x8():
    """cv2.getStructuringElement(cv2.MORPH_ELLIPSE, (8, 8)) (OpenCV's row-span rule:
    r = c = 4, row i spans c -+ round(sqrt(r^2 - (i - r)^2)))."""
    k = np.zeros((8, 8), bool)
    for i in range(8):
        dy = i - 4
        dx = int(round(4 * np.sqrt((16 - dy * dy) / 16.0)))
        k[i, max(4 - dx, 0):min(4 + dx + 1, 8)] = True
    return k


def _erode(mask, k):
    """cv2.erode with kernel k, anchor at its centre, constant border = +inf."""
    from scipy.ndimage import grey_erosion
    return grey_erosion(mask, footprint=k, mode="constant", cval=255, origin=(-0, -0))


def _area_half(img):
    """cv2.resize(..., fx=fy=0.5, INTER_AREA) of a uint8 image: 2x2 means, (s + 2) >> 2."""
    h, w = img.shape[0] // 2, img.shape[1] // 2
    s = (img[0:2 * h:2, 0:2 * w:2].astype(np.int32) + img[1:2 * h:2, 0:2 * w:2] + img[0:2 * h:2, 1:2 * w:2] +
         img[1:2 * h:2, 1:2 * w:2])
    return ((s + 2) >> 2).astype(np.uint8)


class OcclusionBank:
    """The occluders of Augment (utils/udaap/utils_augment.py:13-88), resident on
    the device: RGBA float images in [0,1] (the object's pixels + a mask whose
    border ring is 192, downscaled by 0.5).  `from_voc` restates load_occluders
    on a Pascal VOC 2012 tree (segmented objects that are not cat / dog / cow /
    horse / sheep / person, >= 500 mask pixels); cv2 is not in this image, so
    the 8x8 elliptic erosion and the INTER_AREA halving are restated (parity
    unpinned).  Any list of RGBA float arrays works as a bank."""

    def __init__(self, occluders, device="cuda"):
        if not occluders:
            raise ValueError("OcclusionBank: no occluders")
        offs, flat, o = [], [], 0
        for a in occluders:
            a = np.ascontiguousarray(a, np.float32)
            if a.ndim != 3 or a.shape[2] != 4:
                raise ValueError("OcclusionBank: occluders are [h, w, 4] RGBA")
            offs.append(o)
            flat.append(a.reshape(-1))
            o += a.size
        self.sizes = [tuple(a.shape[:2]) for a in occluders]
        self.dev = torch.device(device)
        self.bank = torch.from_numpy(np.concatenate(flat)).to(self.dev)
        self.off = torch.tensor(offs, dtype=torch.int64, device=self.dev)
        self.hw = torch.tensor([v for hw in self.sizes for v in hw], dtype=torch.int32, device=self.dev)

    @classmethod
    def from_voc(cls, voc_root, device="cuda"):
        import os
        import xml.etree.ElementTree as ET
        from PIL import Image
        k = _ellipse_8x8()
        skip = {"cat", "dog", "cow", "horse", "sheep", "person"}
        occ = []
        ann = os.path.join(voc_root, "Annotations")
        for name in sorted(os.listdir(ann)):
            root = ET.parse(os.path.join(ann, name)).getroot()
            if root.find("segmented").text == "0":
                continue
            boxes = [(i, [int(o.find("bndbox").find(t).text) for t in ("xmin", "ymin", "xmax", "ymax")])
                     for i, o in enumerate(root.findall("object")) if o.find("name").text not in skip]
            if not boxes:
                continue
            fn = root.find("filename").text
            im = np.asarray(Image.open(os.path.join(voc_root, "JPEGImages", fn)))
            labels = np.asarray(Image.open(os.path.join(voc_root, "SegmentationObject", fn.replace("jpg", "png"))))
            for i, (x0, y0, x1, y1) in boxes:
                mask = (labels[y0:y1, x0:x1] == i + 1).astype(np.uint8) * 255
                if int((mask > 0).sum()) < 500:
                    continue
                mask[_erode(mask, k) < mask] = 192
                rgba = np.concatenate([im[y0:y1, x0:x1], mask[..., None]], axis=-1)
                occ.append(_area_half(rgba).astype(np.float32) / 255.0)
        return cls(occ, device)


def draw_occlusion(W, H, sizes, aug_rate=0.5, num_occluder=8):
    """One view's occlusion draws with the reference's RNG calls, in its order
    (augment_occlu :21-25, occlude_with_objects :116-129, resize_by_factor
    :166-171, paste_over's clipping :131-163): [] when the view is not
    occluded, else a list of (occluder, w1, h1, x0, y0, x1, y1, sx0, sy0)."""
    if not np.random.uniform(0, 1) < aug_rate:
        return []
    out = []
    count = np.random.randint(1, num_occluder)
    for _ in range(count):
        o = random.choice(range(len(sizes)))                               # random.choice(self.occluders)
        f = np.random.uniform(0.2, 0.8)
        h, w = sizes[o]
        w1, h1 = (int(v) for v in np.round(np.array([w, h]) * f).astype(int))
        r = paste_rect(np.random.uniform([0, 0], [W, H]), w1, h1, W, H)
        if r is not None:
            out.append((o, w1, h1) + r)
    return out


def paste_rect(center, w1, h1, W, H):
    """paste_over's geometry (utils/udaap/utils_augment.py:146-157): the
    destination rectangle (x0, y0, x1, y1) and the source start (sx0, sy0) of a
    w1 x h1 occluder centred at round(center) in a W x H image; None if nothing
    lands inside."""
    center = np.round(center).astype(np.int32)
    wh = np.array([w1, h1])
    raw0 = center - wh // 2
    raw1 = raw0 + wh
    d0 = np.clip(raw0, 0, [W, H])
    d1 = np.clip(raw1, 0, [W, H])
    s0 = d0 - raw0
    if w1 <= 0 or h1 <= 0 or not (d1 > d0).all():
        return None
    return int(d0[0]), int(d0[1]), int(d1[0]), int(d1[1]), int(s0[0]), int(s0[1])


class DeviceAugment:
    """imgs: uint8 BGR [N,H,W,3] (numpy or device tensor); means: RGB-ordered
    channel means (MouseData.getSemiData).  two_stage (default): the
    reference's pixels — skimage rotate, then resize (ubpl_augment_chain);
    False: one bilinear sample through the composed map (ubpl_augment_warp,
    the round-2/3 path; its deviation from the chain is in DESIGN.md §1 f1)."""

    def __init__(self, imgs, means, inp_res=256, sf=0.25, rf=30.0, use_flip=True, use_noise=True, device="cuda",
                 two_stage=True):
        self.two_stage = two_stage
        self.imgs = torch.as_tensor(imgs).to(device).contiguous()
        self.N, self.H, self.W = self.imgs.shape[:3]
        self.res = inp_res
        self.sf, self.rf, self.use_flip, self.use_noise = sf, rf, use_flip, use_noise
        self.dev = torch.device(device)
        self.chan_mean = torch.tensor(means, dtype=torch.float32, device=self.dev)
        self.img_mean = Kn.image_mean_u8(self.imgs)

    def _draw(self, kps):
        return draw_view(kps, self.W, self.H, self.res, self.sf, self.rf, self.use_flip, self.use_noise)

    def _draw_geo(self, kps):
        return draw_view(kps, self.W, self.H, self.res, self.sf, self.rf, self.use_flip, self.use_noise,
                         with_geometry=True)

    def views(self, idx, kps, occlusion=None, occ_rate=0.5, num_occluder=8):
        """idx: source image per view [V]; kps: numpy [V,K,3] pixel keypoints;
        occlusion: an OcclusionBank (DS_mds useOcclusion, datasets/dataset_mds.py:
        104-109: drawn after each view's affine, as the loader does).
        -> (images [V,3,res,res] on the device, keypoints [V,K,3] on the device)."""
        mats, noises, out_k, geos, css = [], [], [], [], []
        pastes, first = [], [0]
        for v, k in enumerate(kps):
            m, n, kk, (geo, cs) = self._draw_geo(np.asarray(k, np.float32))
            geos.append((int(idx[v]),) + geo)
            css.append(cs)
            mats.append(m)
            noises.append(n)
            out_k.append(kk)
            if occlusion is not None:
                pastes += [(v,) + p for p in draw_occlusion(self.res, self.res, occlusion.sizes, occ_rate,
                                                            num_occluder)]
                first.append(len(pastes))
        V = len(idx)
        idx = np.asarray(idx, np.int32)
        if idx.min() < 0 or idx.max() >= self.N:
            raise IndexError("DeviceAugment: source image index out of range")
        src = torch.tensor(idx, device=self.dev)
        mat = torch.tensor(np.array(mats, np.float32), device=self.dev)
        noise = torch.tensor(np.array(noises, np.float32), device=self.dev)
        out = torch.empty((V, 3, self.res, self.res), device=self.dev)
        if self.two_stage:
            g = np.array(geos, np.int32)
            Kn.augment_chain(self.imgs, torch.from_numpy(g).to(self.dev),
                             torch.tensor(np.array(css, np.float32), device=self.dev), noise, self.img_mean,
                             self.chan_mean, int(g[:, 6].max()), int(g[:, 7].max()), out)
        else:
            Kn.augment_warp(self.imgs, src, mat, noise, self.img_mean, self.chan_mean, out)
        if occlusion is not None and pastes:
            pt = np.array([p[:8] + (p[8] | (p[9] << 16),) for p in pastes], np.int32)
            Kn.occlude(out, occlusion.bank, occlusion.off, occlusion.hw, torch.from_numpy(pt).to(self.dev),
                       torch.tensor(first, dtype=torch.int32, device=self.dev), self.chan_mean)
        return out, torch.tensor(np.array(out_k, np.float32), device=self.dev)
