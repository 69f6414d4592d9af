"""projects.tools drop-in: ProjectTools (projects/tools.py:10-71).

Per-sample weight vectors [bs, 1] from the `islabeled` flags (L7).  They are
built on device without autograd leaves: the reference wraps them (and the
images/heatmaps) in Variable(requires_grad=True) (:56-61), which only makes
autograd compute gradients nobody reads.
"""
import torch


def _where(isl, lab, unlab, device):
    isl = isl.to(device, non_blocking=True)
    one = torch.ones(isl.shape[0], device=device)
    return torch.where(isl > 0, lab * one, unlab * one).unsqueeze(-1)


class ProjectTools:
    @classmethod
    def getSampleWeight(cls, isLabeledArray, args):                    # :13-19  labeled 1, else 0
        return [_where(i, 1.0, 0.0, args.device) for i in isLabeledArray]

    @classmethod
    def getSampleWeight_nega(cls, isLabeledArray, args):               # :21-28  labeled 0, else pseudoWeight
        return [_where(i, 0.0, args.pseudoWeight, args.device) for i in isLabeledArray]

    @classmethod
    def getSampleWeight_mt(cls, islabeled, args):                      # :30-36
        return _where(islabeled, 1.0, 0.0, args.device)

    @classmethod
    def getSampleWeight_mt_nega(cls, islabeled, args):                 # :38-45
        return _where(islabeled, 0.0, args.pseudoWeight, args.device)

    @classmethod
    def getSampleWeight_mt_cons(cls, islabeled, args):                 # :47-54  labeled 1, else pseudoWeight
        return _where(islabeled, 1.0, args.pseudoWeight, args.device)

    @classmethod
    def setVariable(cls, tensor, deviceID, toVariable=True, requires_grad=True):
        return tensor.to(deviceID, non_blocking=True)

    @classmethod
    def setContent(cls, dataArray, fmt):
        return ", ".join(format(v, fmt) for v in dataArray)
