"""E1 EMA teacher update, E2 ramps, S1 TwoStreamBatchSampler (oracle).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
"""
import itertools

import numpy as np
import torch


def ema_alpha(epo, ema_decay):
    """utils/parameters.py:6 — alpha keyed on the EPOCH index."""
    return min(1 - 1 / (epo + 1), ema_decay)


def ema_update(ema_params, params, epo, ema_decay):
    """utils/parameters.py:4-8: ema = ema*alpha, then += (1-alpha)*p, in place,
    parameters only (BN running stats are not averaged)."""
    a = ema_alpha(epo, ema_decay)
    with torch.no_grad():
        for e, p in zip(ema_params, params):
            e.mul_(a).add_(p, alpha=1 - a)


def sigmoid_rampup(current, rampup_length):
    """utils/parameters.py:108-113."""
    if rampup_length == 0:
        return 1.0
    current = np.clip(current, 0.0, rampup_length)
    phase = 1.0 - current / rampup_length
    return float(np.exp(-5.0 * phase * phase))


def value_increase(epo, vmax, vmin, rampup):
    return vmin + (vmax - vmin) * sigmoid_rampup(epo, rampup)          # :100-101


def value_decrease(epo, vmax, vmin, rampup):
    return vmin + (vmax - vmin) * (1.0 - sigmoid_rampup(epo, rampup))  # :104-105


def two_stream_batches(primary, secondary, batch_size, secondary_batch_size):
    """TwoStreamBatchSampler.__iter__ (utils/mt/data.py:117-125) with the same
    numpy RNG consumption order: one permutation of the primary indices at
    iteration start, then secondary permutations drawn lazily as batches are
    pulled."""
    pbs = batch_size - secondary_batch_size
    perm = np.random.permutation(primary)

    def eternal():
        while True:
            yield np.random.permutation(secondary)

    sec = itertools.chain.from_iterable(eternal())
    pit = iter(perm)
    out = []
    for _ in range(len(primary) // pbs):
        pb = tuple(next(pit) for _ in range(pbs))
        sb = tuple(next(sec) for _ in range(secondary_batch_size))
        out.append(pb + sb)
    return out
