"""ubpl_amd — MI355X-native (gfx950) hot path of UBPL-PoseEstimation.

The semi-supervised pose training step — stacked-hourglass forward/backward,
Gaussian heatmap targets, heatmap MSE / consistency losses, the UBPL
pseudo-label confidence mask, the feature-decorrelation loss, the Mean-Teacher
EMA update and the argmax + PCK decoder — on hand-written HIP kernels
(libubpl_hip.so, C-ABI in include/ubpl_hip.h), behind the reference's module
API (models.PoseModel, utils.losses, utils.parameters, utils.mt.data,
utils.process, utils.evaluation, projects.tools).

There is no CPU fallback: every compute entry point raises without the HIP
library or a GPU.
"""
from . import _lib  # noqa: F401

__all__ = ["hourglass", "losses", "parameters", "process", "evaluation", "sampler", "tools", "train", "dist"]
