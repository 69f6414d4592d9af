"""Data parallelism for the training step over RCCL (torch.distributed
backend "nccl" = RCCL on ROCm), one process per GPU.

The reference runs on a single device (projects/MT_UBPL.py:435).  Here each
rank owns a disjoint shard of the labeled/unlabeled index sets
(TwoStreamBatchSampler.shard) and a full replica of both students, both
teachers and the renderer.  Per step there are exactly two exchanges:

1. one tiny all-reduce of the loss sums and row counts (after the forward),
   so that every normaliser (pec_count, n_pseudo, fdc_count) is the GLOBAL
   batch's — the sharded step then computes the same gradient as one device
   running the global batch with per-rank BatchNorm statistics;
2. one SUM all-reduce of each student's flat grad-carrying buffer (26.3 MB
   fp32 per student at 2 stacks) after the backward.

Teachers stay replica-local: identical initial weights (same seed, plus a
broadcast at wrap time) and identical averaged updates keep them identical.
BatchNorm running statistics are per-rank (train-mode teachers keep their
own); `broadcast_buffers` syncs them from rank 0 before validation or a
checkpoint.
"""
import os

import torch
import torch.distributed as dist

# UBPL_DIST_WORLD1=1: the distributed step (its two collectives, the segmented capture of
# train._StepGraph) also on a one-rank process group — how the RCCL path is exercised on a
# one-GPU box (tests/test_gpu_dist.py; RCCL refuses two ranks on one device)
_WORLD1 = os.environ.get("UBPL_DIST_WORLD1") == "1"


def is_dist():
    return dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or _WORLD1)


def rank():
    return dist.get_rank() if is_dist() else 0


def world():
    return dist.get_world_size() if is_dist() else 1


def allreduce_(t):
    """In-place SUM all-reduce (no-op on one rank)."""
    if is_dist():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def broadcast_params(models, src=0):
    """Make every replica start from rank `src`'s weights (flat buffers)."""
    if not is_dist():
        return
    for m in models:
        dist.broadcast(m.flat_params, src)
        dist.broadcast(m.flat_stats, src)


def broadcast_buffers(models, src=0):
    if not is_dist():
        return
    for m in models:
        dist.broadcast(m.flat_stats, src)


def allreduce_grads(models):
    """SUM of each student's grad-carrying prefix (the losses are already
    normalised by global counts)."""
    if not is_dist():
        return
    for m in models:
        dist.all_reduce(m.live_grads(), op=dist.ReduceOp.SUM)
