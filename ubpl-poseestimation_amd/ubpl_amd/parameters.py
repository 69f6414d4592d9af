"""utils.parameters drop-in: Mean-Teacher EMA (E1) and loss-weight ramps (E2).

update_ema_variables (utils/parameters.py:4-8) runs ONE HIP kernel over each
model's flat parameter buffer (the reference issues 2 ops x 454 tensors).
alpha = min(1 - 1/(epo+1), ema_decay) is keyed on the EPOCH; BN running
statistics are not averaged (the teacher keeps its own, projects/MT_UBPL.py:169).
"""
import numpy as np

from . import kernels as Kn
from .hourglass import StackedHourglass


def ema_alpha(epo, ema_decay):
    return min(1 - 1 / (epo + 1), ema_decay)


def update_ema_variables(model, ema_model, args):
    if not (isinstance(model, StackedHourglass) and isinstance(ema_model, StackedHourglass)):
        raise TypeError("update_ema_variables: both models must be ubpl_amd StackedHourglass (flat buffers)")
    if model.n_total != ema_model.n_total:
        raise ValueError("teacher/student architectures differ")
    Kn.ema_update_(ema_model.flat_params, model.flat_params, ema_alpha(args.epo, args.ema_decay))


def _sigmoid_rampup(current, rampup_length):
    """utils/parameters.py:108-113."""
    if rampup_length == 0:
        return 1.0
    current = np.clip(current, 0.0, rampup_length)
    phase = 1.0 - current / rampup_length
    return float(np.exp(-5.0 * phase * phase))


def _value_increase(epo, maxValue, minValue, rampup):
    return minValue + (maxValue - minValue) * _sigmoid_rampup(epo, rampup)


def _value_decrease(epo, maxValue, minValue, rampup):
    return minValue + (maxValue - minValue) * (1.0 - _sigmoid_rampup(epo, rampup))


def consWeight_increase(epo, args):
    return _value_increase(epo, args.consWeight_max, args.consWeight_min, args.consWeight_rampup)


def pseudoWeight_increase(epo, args):
    return _value_increase(epo, args.pseudoWeight_max, args.pseudoWeight_min, args.pseudoWeight_rampup)


def FDLWeight_decrease(epo, args):
    return _value_decrease(epo, args.FDLWeight_max, args.FDLWeight_min, args.FDLWeight_rampup)


def FDLWeight_increase(epo, args):
    return _value_increase(epo, args.FDLWeight_max, args.FDLWeight_min, args.FDLWeight_rampup)
