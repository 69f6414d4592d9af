"""Mouse datasource: the reference's semi-supervised split and
its images, as device batches for train() / validate().

Drop-in for MouseData (datasources/mouse.py:13-123): same attributes (inpRes
256, outRes 64, pck_ref [1, 2], pck_thr 0.2, 9 keypoints) and the same
getSemiData(trainCount, validCount, labelRatio) 8-tuple, read from the
reference's cached split (datasources/temp_data/Mouse_<t>_<v>_<r>.json, the
file getSemiData itself returns, :38-48 / :114-123) with its `D:/...` image
paths remapped to a local image directory.  Reference quirks kept:

* images are BGR (cv2.imread, utils/process.py:86-88; read here with PIL and
  flipped) while the means are RGB-ordered: per-channel means of the BGR
  pixels, then reversed (:72-90, `means.reverse()`), subtracted channel by
  channel from the BGR image without the std (utils/process.py:151-160);
* validation centre = [int(w/2), int(h/2)], scale = inpRes/200 as float32
  (datasets/dataset.py:33-35, utils/process.py:218-221).

GPU boxes do not have the reference tree: tools/pack_mouse.py writes the split
and its 600 images into one .npz (`write_pack`), which `from_pack` reads.
"""
import json
import os

import numpy as np
import torch

PACK_NAME = "mouse_100_500_0.3.npz"
DEFAULT_PACK = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "data",
                            PACK_NAME)


def _bgr(path):
    from PIL import Image
    return np.asarray(Image.open(path).convert("RGB"), dtype=np.uint8)[:, :, ::-1].copy()


def norm_params(imgs_bgr):
    """MouseData._getNormParams (datasources/mouse.py:72-90) on uint8 BGR
    images [N,H,W,3]: the reference stacks them as [H,W,C,N], takes float32
    means / stds per channel over that layout, then reverses (BGR -> RGB order)."""
    imgs = np.ascontiguousarray(np.transpose(imgs_bgr, (1, 2, 3, 0))).astype(np.float32) / 255.
    means, stds = [], []
    for i in range(3):
        px = imgs[:, :, i, :].ravel()
        means.append(float(np.mean(px)))
        stds.append(float(np.std(px)))
    means.reverse()
    stds.reverse()
    return means, stds


class MouseData:
    """datasources/mouse.py:13-123 (the cached-split path of getSemiData)."""

    def __init__(self, root=None, split_dir=None, pack=None):
        self.imgPath = None if root is None else os.path.join(root, "images")
        self.split_dir = split_dir
        self.inpRes, self.outRes = 256, 64
        self.pck_ref, self.pck_thr = [1, 2], 0.2
        self.selKpIdxs = list(range(9))
        self.kpsCount = 9
        self.imgType = "png"
        self._pack = pack

    @classmethod
    def from_pack(cls, path=DEFAULT_PACK):
        if not os.path.exists(path):
            raise FileNotFoundError("%s missing: run tools/pack_mouse.py in a tree with the reference data" % path)
        with np.load(path, allow_pickle=False) as z:
            pack = {k: z[k] for k in z.files}
        return cls(pack=pack)

    # -- the reference's API ----------------------------------------------
    def _split(self, trainCount, validCount, labelRatio):
        name = "Mouse_{}_{}_{}.json".format(trainCount, validCount, labelRatio)
        with open(os.path.join(self.split_dir, name)) as f:
            semi, valid, lab, unlab, lidx, uidx = json.load(f)
        for item in semi + valid + lab + unlab:
            item["imagePath"] = os.path.join(self.imgPath, item["imageName"])
        return semi, valid, lab, unlab, lidx, uidx

    def getSemiData(self, trainCount, validCount, labelRatio, reMean=True):
        """-> semiTrainData, validData, labeledData, unlabeledData, labeledIdxs,
        unlabeledIdxs, means, stds (datasources/mouse.py:38-48)."""
        if self._pack is not None:
            return self._semi_from_pack(reMean)
        semi, valid, lab, unlab, lidx, uidx = self._split(trainCount, validCount, labelRatio)
        if reMean:
            means, stds = norm_params(np.stack([_bgr(it["imagePath"]) for it in semi + valid]))
        else:
            means, stds = [0.4920829] * 3, [0.16629942] * 3
        return semi, valid, lab, unlab, lidx, uidx, means, stds

    # -- pack -------------------------------------------------------------
    def write_pack(self, path, trainCount, validCount, labelRatio):
        semi, valid, lab, unlab, lidx, uidx, means, stds = self.getSemiData(trainCount, validCount, labelRatio)
        np.savez_compressed(
            path,
            train_imgs=np.stack([_bgr(it["imagePath"]) for it in semi]),
            valid_imgs=np.stack([_bgr(it["imagePath"]) for it in valid]),
            train_kps=np.array([it["kps"] for it in semi], np.float32),
            train_kps_test=np.array([it["kps_test"] for it in semi], np.float32),
            train_islabeled=np.array([it["islabeled"] for it in semi], np.int64),
            valid_kps=np.array([it["kps"] for it in valid], np.float32),
            train_ids=np.array([it["imageID"] for it in semi]), valid_ids=np.array([it["imageID"] for it in valid]),
            labeledIdxs=np.array(lidx, np.int64), unlabeledIdxs=np.array(uidx, np.int64),
            means=np.array(means, np.float64), stds=np.array(stds, np.float64))

    def _semi_from_pack(self, reMean=True):
        p = self._pack

        def items(prefix, n):
            out = []
            for i in range(n):
                kps = p[prefix + "_kps"][i].tolist()
                out.append({"islabeled": int(p["train_islabeled"][i]) if prefix == "train" else 1,
                            "imageID": str(p[prefix + "_ids"][i]), "index": i, "split": prefix, "kps": kps,
                            "kps_test": p["train_kps_test"][i].tolist() if prefix == "train" else kps})
            return out
        semi = items("train", len(p["train_ids"]))
        valid = items("valid", len(p["valid_ids"]))
        lidx = p["labeledIdxs"].tolist()
        uidx = p["unlabeledIdxs"].tolist()
        means = p["means"].tolist() if reMean else [0.4920829] * 3
        stds = p["stds"].tolist() if reMean else [0.16629942] * 3
        return semi, valid, [semi[i] for i in lidx], [semi[i] for i in uidx], lidx, uidx, means, stds

    def images(self, split):
        """uint8 BGR [N,256,256,3] of 'train' (semiTrain order) or 'valid'."""
        if self._pack is not None:
            return self._pack[split + "_imgs"]
        semi, valid = self._split(100, 500, 0.3)[:2]
        return np.stack([_bgr(it["imagePath"]) for it in (semi if split == "train" else valid)])


def to_device_images(imgs_bgr, means, device):
    """uint8 BGR [N,H,W,3] -> float32 [N,3,H,W] on the device: /255, minus the
    (RGB-ordered) means channel by channel (utils/process.py:151-160, useStd False)."""
    x = torch.from_numpy(np.ascontiguousarray(imgs_bgr)).to(device).permute(0, 3, 1, 2).float().div_(255.)
    m = torch.tensor(means, dtype=torch.float32, device=device).view(1, 3, 1, 1)
    return (x - m).contiguous()


def valid_batches(data, batch, device, rank=0, world=1):
    """validate()'s loader over the validation split (datasets/dataset.py:21-146
    with isAug False), images resident on the device: (imgMap, None, meta) with
    meta center [B,2] int64, scale [B] float32, kpsMap [B,K,3].  Under data
    parallelism rank r takes every world-th batch (validate() then restores the
    single-device batch order, see train.validate)."""
    _, valid, _, _, _, _, means, _ = data.getSemiData(100, 500, 0.3)
    x = to_device_images(data.images("valid"), means, device)
    kps = torch.tensor([it["kps"] for it in valid], dtype=torch.float32)
    out = []
    for bi, s in enumerate(range(0, x.shape[0], batch)):
        if bi % world != rank:
            continue
        e = min(s + batch, x.shape[0])
        n = e - s
        meta = {"center": torch.tensor([[x.shape[3] // 2, x.shape[2] // 2]] * n, dtype=torch.int64),
                "scale": torch.full((n,), data.inpRes / 200.0, dtype=torch.float32),
                "kpsMap": kps[s:e].clone(), "batch_index": bi}
        out.append((x[s:e], None, meta))
    return out
