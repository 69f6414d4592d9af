"""utils.process drop-in (hot-path subset of ProcessUtils, utils/process.py).

kps_heatmap / kps_heatmap_mulKps (:252-318)  -> HIP renderer (render.hip)
kps_fromHeatmap (:320-327)                    -> HIP argmax + affine (decode.hip)
features_cov (:18-31)                         -> HIP covariance (loss.hip)
kps_getLabeledCount (:381-383)                -> one device reduction

Results come back on the device of the input (a CPU keypoint tensor from a
Dataset gets a CPU heatmap back, as the reference returns), the computation
always runs on the GPU.  render_batch() is the batched, device-resident form
the fused training step uses.
"""
import numpy as np
import torch

from . import _lib
from . import kernels as Kn
from . import losses as L


def inverse_transforms(center, scale, res):
    """rows 0-1 of inv(get_transform(center, scale, res)) per sample, float64
    [N,6], with the reference's precision (utils/udaap/transforms.py:119-155):
    h = 200*scale in float32 tensor arithmetic, entries float32, np.linalg.inv
    in float64.  Host-side setup, O(N) scalars."""
    center = torch.as_tensor(center)
    scale = torch.as_tensor(scale, dtype=torch.float32).reshape(-1)
    N = center.shape[0]
    out = np.zeros((N, 6), np.float64)
    for i in range(N):
        h = 200 * scale[i]
        t = np.zeros((3, 3))
        t[0, 0] = float(res[1]) / h
        t[1, 1] = float(res[0]) / h
        t[0, 2] = res[1] * (-float(center[i][0]) / h + .5)
        t[1, 2] = res[0] * (-float(center[i][1]) / h + .5)
        t[2, 2] = 1
        ti = np.linalg.inv(t)
        out[i] = ti[:2].reshape(-1)
    return torch.from_numpy(out)


def render_batch(kps, img_hw, inp_res, out_res, kernel_size=3.0, sigma=1.0):
    """kps [B,K,3] on device -> (heatmaps [B,K,R,R], kps with vis applied)."""
    return Kn.render_heatmaps(kps.contiguous(), img_hw, inp_res, out_res, kernel_size, sigma)


class ProcessUtils:
    @classmethod
    def kps_heatmap(cls, kpsMap, imgShape, inpRes, outRes, kernelSize=3.0, sigma=1.0):
        _lib.require_gpu()
        dev = kpsMap.device
        k = kpsMap.detach().to("cuda", torch.float32).reshape(1, -1, 3).contiguous()
        hm, kout = Kn.render_heatmaps(k, (imgShape[1], imgShape[2]), inpRes, outRes, kernelSize, sigma)
        kpsMap[:, 2] = kout[0, :, 2].to(dev, kpsMap.dtype)          # in place, utils/process.py:267
        return hm[0].to(dev), kpsMap

    @classmethod
    def kps_heatmap_mulKps(cls, kpsMapArray, imgShape, inpRes, outRes, kernelSize=3.0, sigma=1.0):
        hms, news = [], []
        for k in kpsMapArray:
            hm, kk = cls.kps_heatmap(k, imgShape, inpRes, outRes, kernelSize, sigma)
            hms.append(hm)
            news.append(kk)
        return hms, news

    @classmethod
    def kps_fromHeatmap(cls, heatmap, cenMap, scale, res, mode="batch"):
        if mode == "single":
            p, _ = cls.kps_fromHeatmap(heatmap.unsqueeze(0), torch.as_tensor(cenMap).unsqueeze(0),
                                       torch.as_tensor(scale).reshape(1), res)
            return p[0]
        _lib.require_gpu()
        dev = heatmap.device
        hm = heatmap.detach().to("cuda", torch.float32).contiguous()
        tinv = inverse_transforms(cenMap, scale, res).to("cuda")
        _, preds, scores = Kn.decode_heatmaps(hm, tinv)
        return preds.to(dev), scores.to(dev)

    @classmethod
    def features_cov(cls, inp1, inp2):
        val, cnt = L.features_cov(inp1, inp2)
        return val, int(cnt.item())

    @classmethod
    def kps_getLabeledCount(cls, kpsGate):
        return int((kpsGate.detach() > 0).sum().item())
