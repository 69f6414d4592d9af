"""T1 — the training step of each project on the HIP path.

Same signatures, batch formats and returned records as the reference
train() functions (projects/MT_UBPL.py:157-352, projects/DualPose_UBPL.py:
156-295, projects/MT.py:161-268, projects/supervised.py:135-175), so a
project's epoch loop can call these instead.  What changes is where the work
happens:

* every loss sum AND every count stays on the device (the reference syncs
  per element, ~8k host round trips per MT_UBPL step at B=32); the step makes
  ONE device->host copy, at its end, for the records / the per-batch line;
* heatmap targets can be rendered on the device inside the step (meta["kps"]
  instead of rendered heatmaps), as the benchmark does;
* the optimiser step and the EMA teacher update are single kernels over the
  flat parameter buffers (FlatAdamW, update_ema_variables);
* under torch.distributed every normaliser is global (one tiny all-reduce of
  sums+counts after the forward) and the student gradients are SUM-reduced
  once after the backward (ubpl_amd.dist).

Reference semantics that look like bugs are kept: teachers run in train mode
and keep their own BN statistics; EMA alpha is keyed on the epoch; the FDL
term is added to both students' totals (its gradient applied twice); the
pseudo-loss normaliser counts rows with a positive weighted loss.
"""
import contextlib
import os

import torch

from . import dist as D
from . import kernels as Kn
from .losses import AvgCounter, _RowLoss, features_cov
from .parameters import update_ema_variables
from .process import render_batch


# ---------------------------------------------------------------------------
# device-count loss helpers (same row semantics as ubpl_amd.losses)
# ---------------------------------------------------------------------------
def _mse(preds, gts, S, gate, sw):
    """JointMSELoss(nStack=S, useKPsGate=True, useSampleWeight=True): (sum, cnt[4])."""
    B, K = preds.shape[0], preds.shape[2]
    HW = preds.shape[-1] * preds.shape[-2]
    spec = (0, S, K, HW, (K * HW, 0, 0, 1), gate is not None, sw is not None, 0.0)
    s, c, _ = _RowLoss.apply(preds, gts, spec, gate, sw)
    return s, c


def _mse_plain(preds, gts, S):
    """JointMSELoss(nStack=S) without gate/weights (projects/supervised.py:138);
    nStack == 1 keeps the reference's per-sample rows (reshape((bs, k, -1)))."""
    B = preds.shape[0]
    if S == 1:
        K = preds.shape[1]
        HW = preds.numel() // (B * K)
        spec = (0, 1, K, HW, (K * HW, 0, 0, 1), False, False, 0.0)
    else:
        K = preds.shape[2]
        HW = preds.shape[-1] * preds.shape[-2]
        spec = (0, S, K, HW, (K * HW, 0, 0, 1), False, False, 0.0)
    s, c, _ = _RowLoss.apply(preds, gts, spec, None, None)
    return s, c


def _dist_last(preds, tpreds):
    """JointDistLoss() on the last stack of both (projects/MT_UBPL.py:250)."""
    a = preds[:, -1].contiguous()
    t = tpreds[:, -1].contiguous()
    K = a.shape[1]
    HW = a.shape[-1] * a.shape[-2]
    spec = (0, 1, K, HW, (K * HW, K * HW, 0, 1), False, False, 0.0)
    s, c, _ = _RowLoss.apply(a, t, spec, None, None)
    return s, c


def _dist_mt2_last(preds, tpreds, sw, thr):
    """JointDistLoss_mt2(useSampleWeight=True, scoreThr) on the last stacks
    (projects/DualPose_UBPL.py:163,203)."""
    a = preds[:, -1].contiguous()
    t = tpreds[:, -1].contiguous()
    K = a.shape[1]
    HW = a.shape[-1] * a.shape[-2]
    spec = (1, 1, K, HW, (K * HW, K * HW, 0, 1), False, True, float(thr))
    return _RowLoss.apply(a, t, spec, None, sw)


def _pseudo(preds, targets, sw, S, thr):
    """JointPseudoLoss3(nStack=S, scoreThr) with targets [M,B,S,K,R,R]."""
    B, K = preds.shape[0], preds.shape[2]
    HW = preds.shape[-1] * preds.shape[-2]
    M, St = targets.shape[0], targets.shape[2]
    spec = (2, S, K, HW, (St * K * HW, 0, B * St * K * HW, M, (St - 1) * K * HW), False, True, float(thr))
    return _RowLoss.apply(preds, targets, spec, None, sw)


def _norm(s, n):
    """(s / n) if n > 0 else s — with n a device tensor."""
    n = n.float()
    return torch.where(n > 0, s / n.clamp(min=1.0), s)


def _fdl_view(fa, fb, rowmask, args):
    """One view of the multi-view feature decorrelation term (projects/MT_UBPL.py:
    301-330, DualPose_UBPL.py:246-270) over the selected rows (rowmask > 0):
    returns (kind, value, n_loc) with n_loc a device float[1].

    'covariance' (FDL_type default): value = ProcessUtils.features_cov of the
    selected rows = their MEAN |cov| (0 when no row of this rank is selected),
    n_loc = rows * S * C.  Any other FDL_type: the reference's else branch,
    JointFeatureDistLoss (utils/losses.py:56-70): value = SUM over the selected
    (sample, stack, channel) rows of the pixel-mean squared distance, n_loc =
    rows * S.  The value of a covariance view is a mean, so under data
    parallelism _fdl_total rescales it by n_loc / N_glob before summing."""
    if args.FDL_type == "covariance":
        v, c = features_cov(fa, fb, rowmask)
        n = c.float()
        return "cov", torch.where(n[0] > 0, v, torch.zeros_like(v)), n
    B, S, C = fa.shape[:3]
    HW = fa[0, 0, 0].numel()
    spec = (0, 1, S * C, HW, (S * C * HW, 0, 0, 1), False, True, 0.0)
    s, _, _ = _RowLoss.apply(fa.contiguous(), fb.contiguous(), spec, None, rowmask.reshape(-1).contiguous())
    return "dist", s, ((rowmask > 0).sum() * S).float().reshape(1)


def _fdl_total(views, gcounts_v, W, weight):
    """fdc = FDLWeight * (sum_a value_a) / (sum_a N_a) with global counts N_a
    (MT_UBPL.py:329).  A covariance view is a mean over this rank's rows;
    value_a * n_loc_a / N_a is its share of the global-batch mean (exactly
    value_a on one rank), so the SUM all-reduce of the gradients gives the
    single-device gradient."""
    terms = []
    for (kind, v, n_loc), N_a in zip(views, gcounts_v):
        if kind == "cov" and W > 1:
            v = v * (n_loc[0] / N_a.clamp(min=1.0))
        terms.append(v)
    return weight * _norm(sum(terms), sum(gcounts_v))


def _fdl_record_sums(views):
    """What each rank contributes to the all-reduced FDL record: the local
    SUM (covariance: mean * rows)."""
    return [v.detach() * n[0] if kind == "cov" else v.detach() for kind, v, n in views]


def _fdl_record(views, gsums_v, gcounts_v, W, weight):
    if W == 1:
        vals = [v.detach() for _, v, _ in views]
    else:
        vals = [s / N.clamp(min=1.0) if kind == "cov" else s
                for (kind, _, _), s, N in zip(views, gsums_v, gcounts_v)]
    return weight * _norm(sum(vals), sum(gcounts_v))


def _islabeled(meta_isl, dev):
    return meta_isl.to(dev, non_blocking=True).reshape(-1)


def _w(isl, lab, unlab):
    one = torch.ones(isl.shape[0], device=isl.device)
    return torch.where(isl > 0, lab * one, unlab * one).contiguous()


def _targets(imgs, hms, meta, A, dev, args):
    """Heatmaps and gates per view: either given (reference batch format) or
    rendered on the device from meta['kps'] (list of [B,K,3] per view)."""
    if hms is not None:
        hs = [h[0].to(dev, non_blocking=True).float().contiguous() for h in hms]
        gs = [kw[0].to(dev, non_blocking=True).float().contiguous() for kw in meta["kpsWeights"]]
        return hs, gs
    hs, gs = [], []
    inp = imgs[0].shape[-1]
    for a in range(A):
        hm, kk = render_batch(meta["kps"][a].to(dev).float(), (imgs[a].shape[-2], imgs[a].shape[-1]), inp,
                              args.outRes if hasattr(args, "outRes") else inp // 4)
        hs.append(hm)
        gs.append(kk[:, :, 2].contiguous())
    return hs, gs


def _sync_stats(local_sums, counts):
    """One small all-reduce: returns (global counts, global sums) — identity
    on one rank."""
    if not D.is_dist():
        return counts, local_sums
    pack = torch.cat([counts.float(), local_sums.detach().float()])
    D.allreduce_(pack)
    n = counts.numel()
    return pack[:n], pack[n:]


# ---------------------------------------------------------------------------
# MT_UBPL
# ---------------------------------------------------------------------------
# a student's second-view backward on its teacher's stream (UBPL_SPLIT_BWD=0: one stream per student)
_SPLIT_BWD = os.environ.get("UBPL_SPLIT_BWD", "1") != "0"
# teachers' forwards on their own streams (UBPL_TEACHER_STREAMS=0: on their students' streams)
_TEACHER_STREAMS = os.environ.get("UBPL_TEACHER_STREAMS", "1") != "0"


# Invariant of the networks' phases (fork -> join): no PyTorch arithmetic kernel
# is enqueued — PyTorch's elementwise kernels carry packed-FP32 instructions,
# which this hardware mis-executed beside concurrent matrix work (DESIGN.md §6;
# the library itself is built without them, csrc/Makefile NOPK).  With
# UBPL_STREAM_CHECK=1 every phase runs under _PhaseCheck, which records each
# aten op on a floating-point device tensor that is not a view, an allocation
# or a copy, and join() raises naming them (tests/test_gpu_race.py runs the
# step so).
_STREAM_CHECK = os.environ.get("UBPL_STREAM_CHECK") == "1"
# data movement and metadata: no arithmetic
_PHASE_OK = {"empty", "empty_strided", "empty_like", "zeros", "zeros_like", "zero_", "fill_", "copy_", "clone",
             "_to_copy", "to", "cat", "stack", "detach", "alias", "view", "_unsafe_view", "reshape", "as_strided",
             "expand", "select", "slice", "unsqueeze", "squeeze", "permute", "t", "transpose", "unbind", "split",
             "contiguous", "record_stream", "set_", "resize_", "lift_fresh", "new_empty", "new_zeros",
             "new_empty_strided", "split_with_sizes", "narrow", "view_as", "_reshape_alias", "unfold", "flatten",
             "is_same_size"}


def _phase_violation(func, args, kwargs, on_device):
    """The aten op's name if it is arithmetic on a floating-point device tensor."""
    if func.namespace != "aten":
        return None
    name = func.__name__.split(".")[0]
    if name in _PHASE_OK:
        return None
    ts = [a for a in list(args) + list((kwargs or {}).values()) if torch.is_tensor(a)]
    ts += [x for a in args if isinstance(a, (list, tuple)) for x in a if torch.is_tensor(x)]
    if any(on_device(t) and t.is_floating_point() for t in ts):
        return name
    return None


class _PhaseCheck:
    """Records the aten arithmetic ops enqueued while the networks' streams are
    forked (see _STREAM_CHECK).  on_device: which tensors count (the tests use
    CPU tensors to check the classifier itself)."""

    def __init__(self, on_device=lambda t: t.is_cuda):
        from torch.utils._python_dispatch import TorchDispatchMode
        seen = self.seen = []

        class Mode(TorchDispatchMode):
            def __torch_dispatch__(self, func, types, args=(), kwargs=None):
                v = _phase_violation(func, args, kwargs, on_device)
                if v is not None:
                    seen.append(v)
                return func(*args, **(kwargs or {}))
        self.mode = Mode()

    def __enter__(self):
        self.mode.__enter__()
        return self

    def __exit__(self, *a):
        return self.mode.__exit__(*a)


class _ModelStreams:
    """One HIP stream per network (students 0..M-1, then their teachers).  The
    networks are independent until the losses, and their small hourglass
    levels (<= 16x16: a few dozen workgroups per launch) leave most of the
    chip idle, so several networks in flight fill it.  Autograd runs each
    network's backward on its forward's stream (PyTorch stream semantics of
    backward), so the backward overlaps the same way.  UBPL_MODEL_STREAMS=0
    runs everything on the current stream."""
    _cache = {}

    def __init__(self, M, dev):
        self.main = torch.cuda.current_stream(dev)
        key = (M, dev.index)
        if key not in self._cache:
            self._cache[key] = [torch.cuda.Stream(device=dev) for _ in range(2 * M)]
        self.side = self._cache[key]
        self.M = M
        self._check = None
        self.fork()

    @staticmethod
    def make(M, dev):
        if M < 2 or os.environ.get("UBPL_MODEL_STREAMS", "1") == "0":
            return None
        return _ModelStreams(M, dev)

    # diagnostic: UBPL_ONE_SIDE=1 runs every network on ONE side stream (still not main)
    _one = os.environ.get("UBPL_ONE_SIDE") == "1"

    def on(self, mi):
        return torch.cuda.stream(self.side[0 if self._one else mi])

    def on_teacher(self, mi):
        return torch.cuda.stream(self.side[0 if self._one else self.M + mi])

    def stream(self, i):
        """side stream of network i (students 0..M-1, their teachers M..2M-1)"""
        return self.side[0 if self._one else i]

    def fork(self):
        """Every network stream waits for main: the start of a networks' phase
        (in a segment captured on its own it also brings the streams into the
        capture)."""
        for s in self.side:
            s.wait_stream(self.main)
        if _STREAM_CHECK and self._check is None:
            self._check = _PhaseCheck().__enter__()
            _OPEN_CHECKS.append(self)

    def end_check(self):
        """Leave the phase's _PhaseCheck mode (if one is on); returns what it saw."""
        if self._check is None:
            return ()
        chk, self._check = self._check, None
        chk.__exit__(None, None, None)
        if self in _OPEN_CHECKS:
            _OPEN_CHECKS.remove(self)
        return chk.seen

    def join(self, tensors=()):
        seen = self.end_check()
        for s in self.side:
            self.main.wait_stream(s)
        if seen:                          # (main has joined every network stream first)
            raise RuntimeError("ubpl_amd: PyTorch arithmetic enqueued while the network streams run "
                               "(UBPL_STREAM_CHECK): %s" % sorted(set(seen)))
        if torch.cuda.is_current_stream_capturing():
            return                        # the graph's own dependencies order them
        for t in tensors:                 # produced on a side stream, used on main
            if t is not None and t.is_cuda:
                t.record_stream(self.main)


# phases whose _PhaseCheck mode is on (UBPL_STREAM_CHECK): a step that raised between a
# fork and its join leaves its mode on the dispatch stack; the step drivers close them
_OPEN_CHECKS = []


def _close_phase_checks():
    while _OPEN_CHECKS:
        _OPEN_CHECKS[-1].end_check()


# The students' gradient all-reduce runs after the network streams have joined,
# with nothing else on the device beside it.  torch's RCCL gfx950 reduce kernels
# carry packed-FP32 adds (runTreeUpDown<float, FuncSum>, ReduceScatter PAT f32:
# tools/rccl_pk_check.py, profiles/r05_rccl_packed_fp32.txt), the instruction this
# hardware mis-executed beside concurrent matrix work, so round 3's
# overlap of student i's all-reduce with the other networks' backward (worth < 1 %
# of the step) is gone.
def _join_merge(mstreams, models):
    """Join the network streams and merge every student's second-view gradients
    (projects/MT_UBPL.py:334-336 accumulate both views into .grad)."""
    if mstreams:
        mstreams.join()
    for m in models:
        m.merge_alt_grads()


# ---------------------------------------------------------------------------
# collectives of a step generator
# ---------------------------------------------------------------------------
# The MT_UBPL and DualPose steps (_mt_ubpl_core, _dualpose_core) are generators: it YIELDS its two exchanges —
# ("sum", t): SUM all-reduce of the packed loss sums and counts in place (dist.py
# exchange 1), ("grads", models): the students' gradient all-reduce (exchange 2)
# — and whoever drives them performs them.  Eagerly they run at once (_drive); the
# captured step under torch.distributed captures the device work between them as
# graph segments and runs the collectives between the segments' replays
# (_StepGraph), so the exchanges are never inside a captured graph.
def _collective(req):
    kind, obj = req
    if kind == "sum":
        D.allreduce_(obj)
    elif kind == "grads":
        D.allreduce_grads(obj)
    else:
        raise ValueError("unknown collective %r" % (kind,))


def _drive(gen):
    """Run a step generator eagerly: each yielded collective is performed at once."""
    try:
        req = gen.send(None)
        while True:
            _collective(req)
            req = gen.send(None)
    except StopIteration as e:
        return e.value
    finally:
        _close_phase_checks()


# AdamW + the EMA teacher update in one pass per model (FlatAdamW.step_and_ema);
# UBPL_FUSED_EMA=0 runs the optimizer step and update_ema_variables separately.
_FUSED_EMA = os.environ.get("UBPL_FUSED_EMA", "1") != "0"


def _step_and_ema(models, models_ema, optims, args):
    """optims[i].step() for every student, then update_ema_variables(student,
    teacher) (projects/MT_UBPL.py:338-344, DualPose_UBPL.py:281-287); the
    teacher of model i depends only on student i's updated weights, so the
    per-model fused pass gives the same bits."""
    from .parameters import ema_alpha
    if _FUSED_EMA and all(hasattr(o, "step_and_ema") and o.model is m for o, m in zip(optims, models)):
        a = ema_alpha(args.epo, args.ema_decay)
        for o, e in zip(optims, models_ema):
            o.step_and_ema(e, a)
        return
    for o in optims:
        o.step()
    for mi, m in enumerate(models):
        update_ema_variables(m, models_ema[mi], args)


class _OnMain(torch.autograd.Function):
    """Identity applied on the main stream to a network output produced on a
    side stream.  Autograd sums the several loss gradients of a tensor on the
    stream of the node that consumes them; without this node that is the
    network's stream, reading summands the loss backward allocated on main,
    which the caching allocator hands back to main once autograd drops them —
    while the side stream may still be reading them (a race that only shows
    when main is not the legacy null stream, i.e. in the captured step and
    its warm-up).  With it, the sum happens on main and the network's backward
    receives one tensor that lives until its node has run."""

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g


def _backward_all(totals, outputs=None, mstreams=None):
    """The reference runs total_i.backward(retain_graph=True) once per student
    (projects/MT_UBPL.py:334-336): the shared FDL term makes every call reach
    every student, so each network's backward would run M times with gradients
    that are then summed into .grad.  Backward is linear, so one traversal of
    sum_i total_i accumulates the same gradients with each network's backward
    run once (its upstream gradients summed first).

    outputs (the networks' outputs the losses read): two phases — first every
    loss gradient w.r.t. those outputs, on the main stream, then the networks'
    backwards from them, on their own streams — so no PyTorch elementwise
    kernel (autograd's gradient sums, the loss backward) runs beside the
    networks' matrix work: PyTorch's kernels use packed-FP32 instructions,
    which this hardware mis-executed beside concurrent matrix work (csrc/Makefile
    NOPK)."""
    if outputs is None:
        torch.autograd.backward(totals)
        return
    outs = [t for t in outputs if t is not None and t.requires_grad]
    grads = torch.autograd.grad(totals, outs, allow_unused=True)
    pairs = [(t, g) for t, g in zip(outs, grads) if g is not None]
    if mstreams is not None:
        mstreams.fork()                   # the networks' phase (a captured segment's streams join here)
    torch.autograd.backward([t for t, _ in pairs], [g for _, g in pairs])


# ---------------------------------------------------------------------------
# HIP-graph capture of a whole training step
# ---------------------------------------------------------------------------
def _flatten(obj, leaves):
    """Tiny pytree flatten of a batch: tensors become leaves; lists, tuples and
    dicts recurse; anything else is a constant kept in the spec."""
    if torch.is_tensor(obj):
        leaves.append(obj)
        return ("T", len(leaves) - 1, tuple(obj.shape), str(obj.dtype))
    if isinstance(obj, (list, tuple)):
        return (type(obj).__name__, tuple(_flatten(v, leaves) for v in obj))
    if isinstance(obj, dict):
        return ("dict", tuple((k, _flatten(v, leaves)) for k, v in obj.items()))
    return ("C", repr(obj), obj)


def _spec_key(spec):
    if spec[0] == "C":
        return ("C", spec[1])
    if spec[0] == "T":
        return spec
    if spec[0] == "dict":
        return ("dict", tuple((k, _spec_key(v)) for k, v in spec[1]))
    return (spec[0], tuple(_spec_key(v) for v in spec[1]))


def _unflatten(spec, leaves):
    kind = spec[0]
    if kind == "T":
        return leaves[spec[1]]
    if kind == "C":
        return spec[2]
    if kind == "dict":
        return {k: _unflatten(v, leaves) for k, v in spec[1]}
    vals = [_unflatten(v, leaves) for v in spec[1]]
    return tuple(vals) if kind == "tuple" else vals


class _KeepAll:
    """Diagnostic (UBPL_GRAPH_KEEPALL=1): keeps every tensor any torch op
    allocates during the capture alive until the graph is released, so no
    memory block is reused inside the captured step."""

    def __enter__(self):
        from torch.utils._python_dispatch import TorchDispatchMode
        kept = self.kept = []

        class Mode(TorchDispatchMode):
            def __torch_dispatch__(self, func, types, args=(), kwargs=None):
                out = func(*args, **(kwargs or {}))
                kept.append(out)
                return out
        self.mode = Mode()
        self.mode.__enter__()
        return self

    def __exit__(self, *a):
        return self.mode.__exit__(*a)


class _StepGraph:
    """Runs a device-only step function (a *_core below) and, once the batch
    shapes repeat, replays it from a captured HIP graph: ~6k kernel launches
    per MT_UBPL step become one graph launch, so the host no longer paces the
    GPU.  The first WARM steps run eagerly on a side stream (graph warm-up
    rule); the next step is captured (capture records, it does not execute)
    and then replayed for that batch and every later one, its tensors copied
    into the graph's static inputs first.  Everything the step reads from the
    host — args, learning rates — is part of the cache key, so a change
    re-captures; per-step state (AdamW step counts, BN counters) lives on the
    device.  Under torch.distributed the step is captured as segments — the
    device work before, between and after its two collectives, in one memory
    pool, replayed in capture order — and the collectives run eagerly between
    the replays (no collective inside a graph).  Verified bit-identical to the
    eager step on gloo (two ranks, tests/test_gpu_dist.py) and on RCCL with one
    rank on the GPU (UBPL_DIST_WORLD1: both collectives through RCCL between the
    replays, test_rccl_segmented_graph_matches_eager); RCCL with more than one rank
    needs a multi-GPU box and is the driver's scaling run.  UBPL_STEP_GRAPH=0
    disables."""
    WARM = 2
    _cache = {}

    def __init__(self, core, models, models_ema, optims, args):
        self.core, self.models, self.emas, self.optims, self.args = core, models, models_ema, optims, args
        # default: captured, with or without per-network streams (rounds 1-3 kept
        # it off with streams for a divergence whose cause — packed-FP32
        # instructions beside concurrent matrix work — round 4 removed: DESIGN.md
        # §6); UBPL_STEP_GRAPH=0 disables it.
        env = os.environ.get("UBPL_STEP_GRAPH")
        want = env != "0"
        self.enabled = want and all(hasattr(o, "_step_t") for o in optims)
        self.hkey = None
        self.n_eager = 0
        self.graphs = None                 # the captured segments (one without torch.distributed)
        self.reqs = []                     # the collective after each segment but the last
        self.key = None
        self.static = None
        self.out = None
        self.side = None

    _force_eager = False

    @classmethod
    def eager(cls):
        """Context: run steps eagerly (e.g. to time individual kernels with host
        events, which a captured graph cannot record)."""
        import contextlib

        @contextlib.contextmanager
        def ctx():
            old = cls._force_eager
            cls._force_eager = True
            try:
                yield
            finally:
                cls._force_eager = old
        return ctx()

    @classmethod
    def get(cls, core, models, models_ema, optims, args):
        """One runner per (step function, networks, optimisers).  The host
        constants the captured step bakes in (args: loss weights, epoch ->
        EMA alpha; the learning rates) change every epoch: then the old graph
        and its memory pool are released and the next step re-captures."""
        key = (core.__name__, tuple(map(id, models)), tuple(map(id, models_ema)), tuple(map(id, optims)))
        hkey = (repr(sorted(vars(args).items())) if hasattr(args, "__dict__") else repr(args),
                repr([o.param_groups for o in optims]))
        r = cls._cache.get(key)
        if r is None:
            cls.clear()                      # one runner: an old one would pin its networks and pool
            r = cls._cache[key] = cls(core, models, models_ema, optims, args)
            r.hkey = hkey
        if r.hkey != hkey:
            r.release()
            r.args, r.hkey = args, hkey
        return r

    @classmethod
    def clear(cls):
        for r in cls._cache.values():
            r.release()
        cls._cache.clear()

    def release(self):
        """Drop the captured graph, its static inputs and outputs (its private
        memory pool goes with them)."""
        if self.graphs is not None:
            for g in self.graphs:
                g.reset()
            self.graphs, self.reqs, self.key, self.static, self.out = None, [], None, None, None
            torch.cuda.empty_cache()

    @property
    def graph(self):
        return self.graphs

    def _eager(self, batch):
        return _drive(self.core(self.models, self.emas, self.optims, self.args, *batch))

    def _replay(self):
        for i, g in enumerate(self.graphs):
            g.replay()
            if i < len(self.reqs):
                _collective(self.reqs[i])

    def _capture(self, sbatch):
        """Capture the step: one graph, or under torch.distributed one graph per
        stretch between collectives (shared pool, replayed in this order)."""
        gen = self.core(self.models, self.emas, self.optims, self.args, *sbatch)
        keep = _KeepAll() if os.environ.get("UBPL_GRAPH_KEEPALL") == "1" else contextlib.nullcontext()
        if not D.is_dist():
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g), keep:
                self.out = _drive(gen)
            self._kept = getattr(keep, "kept", None)
            self.graphs, self.reqs = [g], []
            return
        pool = torch.cuda.graph_pool_handle()
        graphs, reqs, done = [], [], False
        try:
            while not done:
                g = torch.cuda.CUDAGraph()
                # thread_local: the process group's own threads may query HIP while a segment captures
                with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
                    try:
                        req = gen.send(None)
                    except StopIteration as e:
                        self.out, done = e.value, True
                graphs.append(g)
                if not done:
                    reqs.append(req)
        finally:
            _close_phase_checks()
        self.graphs, self.reqs = graphs, reqs

    def run(self, batch, dev):
        if not self.enabled or self._force_eager:
            return self._eager(batch)
        leaves = []
        spec = _flatten(batch, leaves)
        key = _spec_key(spec)
        if self.graphs is not None and key == self.key:
            for dst, src in zip(self.static, leaves):
                dst.copy_(src, non_blocking=True)
            self._replay()
            return self.out
        if self.n_eager < self.WARM or self.graphs is not None:
            # warm-up (or a batch of another shape): eager, on a side stream
            if self.side is None:
                self.side = torch.cuda.Stream(device=dev)
            main = torch.cuda.current_stream(dev)
            self.side.wait_stream(main)
            with torch.cuda.stream(self.side):
                out = self._eager(batch)
            main.wait_stream(self.side)
            self.n_eager += 1
            return out
        self.static = [l.to(dev).clone() for l in leaves]
        sbatch = _unflatten(spec, self.static)
        torch.cuda.synchronize(dev)
        self._capture(sbatch)
        self.key = key
        self._replay()
        return self.out


def _mt_ubpl_core(models, models_ema, optims, args, augs_imgMap, augs_heatmaps, meta):
    """One MT_UBPL step (projects/MT_UBPL.py:188-336) on the device with no
    host synchronisation, as a generator: under torch.distributed it yields
    its two exchanges (see _collective), and it returns the packed records
    [3M+1 losses | counts | pseudo scores] as ONE device tensor and the
    host-side constants needed to unpack them.  Run it with _drive (eager) or
    _StepGraph (captured: one graph on one rank, one graph segment per
    collective-free stretch under torch.distributed)."""
    M = len(models)
    dev = models[0].flat_params.device
    S = args.nStack
    for o in optims:
        o.zero_grad()
    A = len(augs_imgMap)
    imgs = [x.to(dev, non_blocking=True).float().contiguous() for x in augs_imgMap]
    hms, gates = _targets(imgs, augs_heatmaps, meta, A, dev, args)
    isl = _islabeled(meta["islabeled"][0], dev)
    sw = _w(isl, 1.0, 0.0)                                   # getSampleWeight
    nega = _w(isl, 0.0, args.pseudoWeight)                   # getSampleWeight_nega
    B = imgs[0].shape[0]
    outs, feats, outs_ema = [], [], []
    mstreams = _ModelStreams.make(M, dev)
    split_bwd = mstreams is not None and _SPLIT_BWD
    for mi in range(M):                                      # :228-243
        oa, fa, ea = [], [], []
        with (mstreams.on(mi) if mstreams else contextlib.nullcontext()):
            for a in range(A):
                # views >= 1: their backward runs on the teacher's stream (idle by
                # then) into the alternate gradient buffer, beside view 0's
                models[mi]._bwd_stream = mstreams.side[M + mi] if split_bwd and a >= 1 else None
                o, f = models[mi](imgs[a])
                models[mi]._bwd_stream = None
                oa.append(o)
                fa.append(f)
        with (mstreams.on_teacher(mi) if mstreams and _TEACHER_STREAMS else
              mstreams.on(mi) if mstreams else contextlib.nullcontext()):
            for a in range(A):
                with torch.no_grad():
                    ea.append(models_ema[mi](imgs[a])[0])
        outs.append(oa)
        feats.append(fa)
        outs_ema.append(ea)
    if mstreams:
        mstreams.join([t for grp in (outs, feats, outs_ema) for ts in grp for t in ts])
        # the losses' gradients for each student output are summed on main
        outs = [[_OnMain.apply(t) for t in ts] for ts in outs]
        feats = [[None if t is None else _OnMain.apply(t) for t in ts] for ts in feats]
    K = outs[0][0].shape[2]
    use_ep = getattr(args, "useEnsemblePseudo", True)        # :271 (False: epc = 0, no print)
    zero = torch.zeros((), device=dev)
    zcnt = torch.zeros(4, dtype=torch.int32, device=dev)
    # ---- loss sums / counts on device
    sums = []
    ps_scores = []
    for mi in range(M):
        ms = []
        for a in range(A):
            s_d, _ = _dist_last(outs[mi][a], outs_ema[mi][a])
            s_p, c_p = _mse(outs[mi][a], hms[a], S, gates[a], sw.reshape(-1, 1))
            if use_ep:
                tg = torch.stack([outs_ema[j][a] for j in range(M)])
                s_e, c_e, sc_e = _pseudo(outs[mi][a], tg, nega, S, args.pseudoScoreThr)
                ps_scores.append(sc_e)
            else:
                s_e, c_e = zero, zcnt
            ms.append((s_d, s_p, c_p, s_e, c_e))
        sums.append(ms)
    fd = []
    if args.FDLWeight > 0:
        rowmask = _fdl_rows(sw, args)
        for a in range(A):                                   # :301-330 selected rows
            fd.append(_fdl_view(feats[0][a], feats[1][a], rowmask, args))
    # pack: per model [mtc_sum, pec_sum, epc_sum], counts [pec_n, epc_n, n_sel]; per FDL view sum / count
    loc = []
    cn = []
    for mi in range(M):
        loc += [sum(x[0] for x in sums[mi]), sum(x[1] for x in sums[mi]), sum(x[3] for x in sums[mi])]
        cn += [sum(x[2][0] for x in sums[mi]), sum(x[4][1] for x in sums[mi]), sum(x[4][2] for x in sums[mi])]
    loc += _fdl_record_sums(fd)
    cn += [n[0] for _, _, n in fd]
    counts = torch.stack([c.float() for c in cn])
    local = torch.stack([l.float() for l in loc])
    if D.is_dist():
        pack = torch.cat([counts, local.detach()])
        yield ("sum", pack)                                  # exchange 1: global sums / counts
        gcounts, gsums = pack[:counts.numel()], pack[counts.numel():]
    else:
        gcounts, gsums = _sync_stats(local, counts)
    W = D.world()
    mtc_n = A * B * K * W
    nf = len(fd)
    totals = []
    fdc = _fdl_total(fd, gcounts[3 * M:], W, args.FDLWeight) if fd else 0.
    for mi in range(M):
        mtc = args.consWeight * (loc[3 * mi] / mtc_n)
        pec = args.poseWeight * _norm(loc[3 * mi + 1], gcounts[3 * mi])
        epc = args.ensemblePseudoWeight * _norm(loc[3 * mi + 2], gcounts[3 * mi + 1]) if use_ep else 0.
        totals.append(pec + mtc + epc + fdc)
    _backward_all(totals, [t for grp in (outs, feats) for ts in grp for t in ts] if mstreams else None,
                  mstreams)                                                                    # :334-336
    _join_merge(mstreams, models)
    if D.is_dist():
        yield ("grads", models)                              # exchange 2: SUM of the students' gradients
    _step_and_ema(models, models_ema, optims, args)
    # ---- records: one device->host copy
    g_rec = []
    for mi in range(M):
        g_rec += [args.poseWeight * _norm(gsums[3 * mi + 1], gcounts[3 * mi]),
                  args.consWeight * gsums[3 * mi] / mtc_n,
                  args.ensemblePseudoWeight * _norm(gsums[3 * mi + 2], gcounts[3 * mi + 1]) if use_ep else zero]
    g_rec.append(_fdl_record(fd, gsums[3 * M:], gcounts[3 * M:], W, args.FDLWeight) if fd else zero)
    score = torch.stack(ps_scores).mean(0) if use_ep else torch.zeros(K, device=dev)
    packed = torch.cat([torch.stack([r.float() for r in g_rec]), gcounts, score])
    return packed, (nf, mtc_n, B, len(cn), use_ep)


class _LaggedRecords:
    """A step's records reach the host one step late: the device->host copy of
    step k goes into pinned memory asynchronously right behind step k's work,
    and the host reads it (waiting on its event) only after step k+1 has been
    enqueued — so the GPU never idles while the host enqueues the next step
    (a blocking .cpu() per step drained the queue every step: the next step's
    ~5k launches then started from an empty queue).  The records, their order
    and every printed line are those of the blocking form; `consume` runs in
    step order.  UBPL_LAG_RECORDS=0: consume each step's records at once."""
    _on = os.environ.get("UBPL_LAG_RECORDS", "1") != "0"

    def __init__(self):
        self.pending = None

    def push(self, packed, consume):
        dev_t = packed.detach().reshape(-1)
        host = torch.empty(dev_t.shape, dtype=dev_t.dtype, pin_memory=True)
        host.copy_(dev_t, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev_t.device))    # the stream the copy went on
        prev, self.pending = self.pending, (host, ev, consume)
        if prev is not None:
            self._run(prev)
        if not self._on:
            self.flush()

    def flush(self):
        prev, self.pending = self.pending, None
        if prev is not None:
            self._run(prev)

    @contextlib.contextmanager
    def flushing(self):
        """Flush on exit — also when the loader raised mid-epoch (the last
        step's records); then an error the flush itself raises (a wait on a
        step a GPU error left half-done) does not replace the one already
        propagating."""
        try:
            yield self
        except BaseException:
            try:
                self.flush()
            except Exception:
                pass
            raise
        self.flush()

    @staticmethod
    def _run(item):
        host, ev, consume = item
        ev.synchronize()
        consume(host.tolist())


def train_mt_ubpl(trainLoader, models, models_ema, optims, args, verbose=True):
    """projects/MT_UBPL.py:157-352 -> (pec_records, mtc_records, epc_records, fdc_record).
    Steps after the first two are replayed from a captured HIP graph when the
    batch shapes repeat (UBPL_STEP_GRAPH=0: every step eager)."""
    M = len(models)
    pec_c = [AvgCounter() for _ in range(M)]
    mtc_c = [AvgCounter() for _ in range(M)]
    epc_c = [AvgCounter() for _ in range(M)]
    fdc_c = AvgCounter()
    dev = models[0].flat_params.device
    for m in models:
        m.train()
    for e in models_ema:
        e.train()
    runner = _StepGraph.get(_mt_ubpl_core, models, models_ema, optims, args)
    lag = _LaggedRecords()
    with lag.flushing():
        for bat, (augs_imgMap, augs_heatmaps, meta) in enumerate(trainLoader):
            packed, meta_h = runner.run((augs_imgMap, augs_heatmaps, meta), dev)
            # the step's one device->host copy, read after the next step is enqueued
            lag.push(packed, lambda host, bat=bat, meta_h=meta_h: _mt_ubpl_records(
                host, bat, meta_h, M, pec_c, mtc_c, epc_c, fdc_c, args, verbose))
    return ([c.avg for c in pec_c], [c.avg for c in mtc_c], [c.avg for c in epc_c], fdc_c.avg)


def _mt_ubpl_records(host, bat, meta_h, M, pec_c, mtc_c, epc_c, fdc_c, args, verbose):
    """One MT_UBPL step's host records -> the AvgCounters and the batch line."""
    nf, mtc_n, B, ncn, use_ep = meta_h
    nrec = 3 * M + 1
    for mi in range(M):
        pec_c[mi].update(host[3 * mi], int(host[nrec + 3 * mi]))
        mtc_c[mi].update(host[3 * mi + 1], mtc_n)
        # useEnsemblePseudo False: epc_counter.update(0., outs.shape[2]) (:292-293; outs.shape[2] = B)
        epc_c[mi].update(host[3 * mi + 2], int(host[nrec + 3 * mi + 1]) if use_ep else B)
    if nf:
        fdc_c.update(host[3 * M], int(sum(host[nrec + 3 * M:nrec + 3 * M + nf])))
    else:
        fdc_c.update(0., B)
    if use_ep:
        n_ps = int(sum(host[nrec + 3 * mi + 1] for mi in range(M)))
        n_sel = int(sum(host[nrec + 3 * mi + 2] for mi in range(M)))
        # the reference's batch line divides by the pseudo-label count whether or not it
        # prints anywhere (projects/MT_UBPL.py:292-293, integer counts): a step with none
        # raises ZeroDivisionError there, and here when its records are consumed
        rate = _pseudo_rate(n_sel, n_ps)
        if verbose:
            sc = host[nrec + ncn:]
            print("batch.{} (scoreThr:{}): {} ({}/{}), pseudo-score: [{}]".format(
                format(bat + 1, "5d"), format(args.pseudoScoreThr, ".2f"),
                format(rate, ".2f"), format(n_sel, "5d"), format(n_ps, "5d"),
                ", ".join(format(v, ".3f") for v in sc)))


def _pseudo_rate(n_sel, n_ps):
    """n_sel / n_ps as the reference's batch line computes it: Python ints, so a step
    without pseudo labels raises ZeroDivisionError (projects/MT_UBPL.py:292-293,
    DualPose_UBPL.py:212-213,238-239)."""
    return int(n_sel) / int(n_ps)


def _fdl_rows(sw, args):
    if args.FDL_label == "labeled":
        return (sw > 0).float()
    if args.FDL_label == "unlabeled":
        return (sw == 0).float()
    return torch.ones_like(sw)


# ---------------------------------------------------------------------------
# DualPose_UBPL
# ---------------------------------------------------------------------------
def _dualpose_core(models, models_ema, optims, args, stu_imgMap, stu_heatmap, ema_imgMap, meta):
    """One DualPose_UBPL step (projects/DualPose_UBPL.py:170-290) on the device
    with no host synchronisation, as a generator like _mt_ubpl_core: it yields
    its two exchanges under torch.distributed and returns the packed records
    [3M+1 losses | counts | consistency scores | pseudo scores] and the
    host-side constants that unpack them."""
    M = len(models)
    dev = models[0].flat_params.device
    S = args.nStack
    for o in optims:
        o.zero_grad()
    si = stu_imgMap.to(dev, non_blocking=True).float().contiguous()
    ei = ema_imgMap.to(dev, non_blocking=True).float().contiguous()
    if stu_heatmap is None:
        hm, kk = render_batch(meta["kps"].to(dev).float(), (si.shape[-2], si.shape[-1]), si.shape[-1],
                              si.shape[-1] // 4)
        gate = kk[:, :, 2].contiguous()
    else:
        hm = stu_heatmap.to(dev, non_blocking=True).float().contiguous()
        gate = meta["kpsWeight"].to(dev, non_blocking=True).float().contiguous()
    isl = _islabeled(meta["islabeled"], dev)
    sw = _w(isl, 1.0, 0.0)
    nega = _w(isl, 0.0, args.pseudoWeight)
    cons = _w(isl, 1.0, args.pseudoWeight)
    outs, feats, ema_l = [], [], []
    mstreams = _ModelStreams.make(M, dev)                    # one HIP stream per network
    for mi in range(M):                                       # :185-196
        with (mstreams.on(mi) if mstreams else contextlib.nullcontext()):
            o, f = models[mi](si)
        outs.append(o)
        feats.append(f)
        with (mstreams.on_teacher(mi) if mstreams else contextlib.nullcontext()), torch.no_grad():
            ema_l.append(models_ema[mi](ei)[0])
    if mstreams:
        mstreams.join(outs + feats + ema_l)
        outs = [_OnMain.apply(t) for t in outs]
        feats = [None if t is None else _OnMain.apply(t) for t in feats]
    outs_ema = torch.stack(ema_l)
    use_ep = getattr(args, "useEnsemblePseudo", True)    # :224 (False: epc = 0, no print)
    K = outs[0].shape[2]
    zero = torch.zeros((), device=dev)
    loc, cn, cons_sc, ps_sc = [], [], [], []
    for mi in range(M):
        s_c, c_c, sc_c = _dist_mt2_last(outs[mi], outs_ema[mi], cons, args.pseudoScoreThr)
        s_p, c_p = _mse(outs[mi], hm, S, gate, sw.reshape(-1, 1))
        if use_ep:
            s_e, c_e, sc_e = _pseudo(outs[mi], outs_ema, nega, S, args.pseudoScoreThr)
            ps_sc.append(sc_e)
        else:
            s_e, c_e = zero, torch.zeros(4, dtype=torch.int32, device=dev)
        loc += [s_c, s_p, s_e]
        cn += [c_c[0], c_p[0], c_e[1], c_c[1], c_c[2], c_e[2]]
        cons_sc.append(sc_c)
    fd = []
    if args.FDLWeight > 0:                                     # :246-270 (one view)
        fd.append(_fdl_view(feats[0], feats[1], _fdl_rows(sw, args), args))
    loc += _fdl_record_sums(fd)
    cn += [n[0] for _, _, n in fd]
    counts = torch.stack([c.float() for c in cn])
    local = torch.stack([l.float() for l in loc])
    if D.is_dist():
        pack = torch.cat([counts, local.detach()])
        yield ("sum", pack)                                  # exchange 1: global sums / counts
        gcounts, gsums = pack[:counts.numel()], pack[counts.numel():]
    else:
        gcounts, gsums = _sync_stats(local, counts)
    W = D.world()
    fdc = _fdl_total(fd, gcounts[6 * M:], W, args.FDLWeight) if fd else 0.
    totals = []
    for mi in range(M):
        mtc = args.consWeight * _norm(loc[3 * mi], gcounts[6 * mi])
        pec = args.poseWeight * _norm(loc[3 * mi + 1], gcounts[6 * mi + 1])
        epc = args.ensemblePseudoWeight * _norm(loc[3 * mi + 2], gcounts[6 * mi + 2]) if use_ep else 0.
        totals.append(pec + mtc + epc + fdc)
    _backward_all(totals, outs + feats if mstreams else None, mstreams)   # DualPose_UBPL.py:277-279
    _join_merge(mstreams, models)
    if D.is_dist():
        yield ("grads", models)                              # exchange 2: SUM of the students' gradients
    _step_and_ema(models, models_ema, optims, args)
    g_rec = []
    for mi in range(M):
        g_rec += [args.poseWeight * _norm(gsums[3 * mi + 1], gcounts[6 * mi + 1]),
                  args.consWeight * _norm(gsums[3 * mi], gcounts[6 * mi]),
                  args.ensemblePseudoWeight * _norm(gsums[3 * mi + 2], gcounts[6 * mi + 2]) if use_ep else zero]
    g_rec.append(_fdl_record(fd, gsums[3 * M:], gcounts[6 * M:], W, args.FDLWeight) if fd else zero)
    packed = torch.cat([torch.stack([r.float() for r in g_rec]), gcounts, torch.stack(cons_sc).mean(0),
                        torch.stack(ps_sc).mean(0) if use_ep else torch.zeros(K, device=dev)])
    return packed, (len(cn), K, use_ep, len(fd))


def train_dualpose_ubpl(trainLoader, models, models_ema, optims, args, verbose=True):
    """projects/DualPose_UBPL.py:156-295.  Like train_mt_ubpl, steps after the
    first two replay a captured HIP graph when the batch shapes repeat."""
    M = len(models)
    pec_c = [AvgCounter() for _ in range(M)]
    mtc_c = [AvgCounter() for _ in range(M)]
    epc_c = [AvgCounter() for _ in range(M)]
    fdc_c = AvgCounter()
    dev = models[0].flat_params.device
    S = args.nStack
    for m in models:
        m.train()
    for e in models_ema:
        e.train()
    runner = _StepGraph.get(_dualpose_core, models, models_ema, optims, args)
    lag = _LaggedRecords()
    with lag.flushing():
        for bat, (stu_imgMap, stu_heatmap, ema_imgMap, meta) in enumerate(trainLoader):
            packed, (ncn, K, use_ep, nfd) = runner.run((stu_imgMap, stu_heatmap, ema_imgMap, meta), dev)
            lag.push(packed, lambda host, bat=bat, ncn=ncn, K=K, use_ep=use_ep, nfd=nfd: _dualpose_records(
                host, bat, ncn, K, use_ep, nfd, M, S, pec_c, mtc_c, epc_c, fdc_c, args, verbose))
    return ([c.avg for c in pec_c], [c.avg for c in mtc_c], [c.avg for c in epc_c], fdc_c.avg)


def _dualpose_records(host, bat, ncn, K, use_ep, nfd, M, S, pec_c, mtc_c, epc_c, fdc_c, args, verbose):
    """One DualPose_UBPL step's host records -> the AvgCounters and the batch lines."""
    nrec = 3 * M + 1
    cbase = nrec
    for mi in range(M):
        pec_c[mi].update(host[3 * mi], int(host[cbase + 6 * mi + 1]))
        mtc_c[mi].update(host[3 * mi + 1], int(host[cbase + 6 * mi]))
        # useEnsemblePseudo False: epc_counter.update(0., outs.shape[2]) (:244-245; outs.shape[2] = nStack)
        epc_c[mi].update(host[3 * mi + 2], int(host[cbase + 6 * mi + 2]) if use_ep else S)
    if nfd:
        fdc_c.update(host[3 * M], int(host[cbase + 6 * M]))
    else:
        fdc_c.update(0., S)                                   # :249 outs.shape[2] = nStack
    off = cbase + ncn
    c_ps = int(sum(host[cbase + 6 * mi + 3] for mi in range(M)))
    c_sel = int(sum(host[cbase + 6 * mi + 4] for mi in range(M)))
    e_ps = int(sum(host[cbase + 6 * mi + 2] for mi in range(M)))
    e_sel = int(sum(host[cbase + 6 * mi + 5] for mi in range(M)))
    c_rate = _pseudo_rate(c_sel, c_ps)                        # (the reference's lines raise on a zero count)
    e_rate = _pseudo_rate(e_sel, e_ps) if use_ep else None
    if verbose:
        print("batch.{} consist-pseudo (scoreThr:{}): {} ({}/{}), pseudo-score: [{}]".format(
            format(bat + 1, "5d"), format(args.pseudoScoreThr, ".2f"),
            format(c_rate, ".2f"), format(c_sel, "5d"), format(c_ps, "5d"),
            ", ".join(format(v, ".3f") for v in host[off:off + K])))
        if use_ep:
            print("batch.{} ensemble-pseudo (scoreThr:{}): {} ({}/{}), pseudo-score: [{}]".format(
                format(bat + 1, "5d"), format(args.pseudoScoreThr, ".2f"),
                format(e_rate, ".2f"), format(e_sel, "5d"), format(e_ps, "5d"),
                ", ".join(format(v, ".3f") for v in host[off + K:off + 2 * K])))


# ---------------------------------------------------------------------------
# MT and supervised
# ---------------------------------------------------------------------------
def train_mt(trainLoader, model, model_ema, optim, args):
    """projects/MT.py:161-268 -> (pec_avg, mtc_avg)."""
    pec_c, mtc_c = AvgCounter(), AvgCounter()
    dev = model.flat_params.device
    S = args.nStack
    model.train()
    model_ema.train()
    pick = (lambda r: r) if args.feature_mode == "default" else (lambda r: r[0])
    for bat, (augs_imgMap, augs_heatmaps, meta) in enumerate(trainLoader):
        optim.zero_grad()
        A = len(augs_imgMap)
        imgs = [x.to(dev, non_blocking=True).float().contiguous() for x in augs_imgMap]
        hms, gates = _targets(imgs, augs_heatmaps, meta, A, dev, args)
        sw = _w(_islabeled(meta["islabeled"][0], dev), 1.0, 0.0)
        outs, outs_ema = [], []
        for a in range(A):
            outs.append(pick(model(imgs[a])))
            with torch.no_grad():
                outs_ema.append(pick(model_ema(imgs[a])))
        B, K = outs[0].shape[0], outs[0].shape[2]
        sd = sum(_dist_last(outs[a], outs_ema[a])[0] for a in range(A))
        ps = [_mse(outs[a], hms[a], S, gates[a], sw.reshape(-1, 1)) for a in range(A)]
        sp = sum(p[0] for p in ps)
        cp = sum(p[1][0] for p in ps)
        counts, sums = _sync_stats(torch.stack([sd, sp]), cp.float().reshape(1))
        mtc_n = A * B * K * D.world()
        mtc = args.consWeight * (sd / mtc_n)
        pec = args.poseWeight * _norm(sp, counts[0])
        (pec + mtc).backward()
        D.allreduce_grads([model])
        optim.step()
        update_ema_variables(model, model_ema, args)
        host = torch.stack([args.poseWeight * _norm(sums[1], counts[0]), args.consWeight * sums[0] / mtc_n,
                            counts[0]]).cpu().tolist()
        mtc_c.update(host[1], mtc_n)
        pec_c.update(host[0], int(host[2]))
    return pec_c.avg, mtc_c.avg


def train_supervised(trainLoader, model, optim, args):
    """projects/supervised.py:135-175 -> pec_avg."""
    pec_c = AvgCounter()
    dev = model.flat_params.device
    model.train()
    pick = (lambda r: r) if args.feature_mode == "default" else (lambda r: r[0])
    for bat, (imgMap, heatmap, meta) in enumerate(trainLoader):
        optim.zero_grad()
        img = imgMap.to(dev, non_blocking=True).float().contiguous()
        hm = heatmap.to(dev, non_blocking=True).float().contiguous()
        out = pick(model(img))
        s, c = _mse_plain(out, hm, args.nStack)
        counts, sums = _sync_stats(s.reshape(1), c[0].float().reshape(1))
        pec = args.poseWeight * _norm(s, counts[0])
        pec.backward()
        D.allreduce_grads([model])
        optim.step()
        host = torch.stack([args.poseWeight * _norm(sums[0], counts[0]), counts[0]]).cpu().tolist()
        pec_c.update(host[0], int(host[1]))
    return pec_c.avg


# ---------------------------------------------------------------------------
# validate: teachers in eval mode -> decode -> PCK (D1-D5)
# ---------------------------------------------------------------------------
def gather_valid_rows(rows):
    """Validation rows (batch_index or None, bs, k, host row) of this rank ->
    the rows to fold, in the single-device batch order.

    Under torch.distributed the rows of all ranks are gathered and ordered by
    batch_index only when EVERY row of every rank carries one (the sharded
    loader, mouse.valid_batches, sets meta['batch_index']).  A loader without
    it gives no global order — every rank may have iterated the whole set, or
    a DistributedSampler reuses indices 0..n on each rank — so then each rank
    keeps its own rows in its own order (per-rank records) and a warning says
    so.  One device: the rows as iterated."""
    if not D.is_dist():
        return rows
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
    tagged = torch.tensor([float(all(r[0] is not None for r in rows))], device=dev)
    dist.all_reduce(tagged, op=dist.ReduceOp.MIN)
    if tagged.item() < 1:
        import warnings
        warnings.warn("ubpl_amd.validate under torch.distributed: the loader sets no meta['batch_index'], "
                      "so the records are this rank's own (not gathered)", RuntimeWarning)
        return rows
    allrows = [None] * D.world()
    dist.all_gather_object(allrows, [(bi, bs, k, h.tolist()) for bi, bs, k, h in rows])
    return sorted(((int(bi), bs, k, torch.tensor(h)) for part in allrows for bi, bs, k, h in part),
                  key=lambda r: r[0])


def validate(validLoader, models_ema, args):
    """projects/MT_UBPL.py:355-408 -> (predsArray, accs_records, errs_records);
    entries per teacher plus their mean (brNum + 1).

    Teachers in eval mode, heatmaps decoded and scored on the device (D1-D4);
    one device->host copy per batch.  Batches are (imgMap, heatmap or None,
    meta) with meta center / scale / kpsMap.  Under torch.distributed every
    rank validates its share of the batches (mouse.valid_batches: batch i on
    rank i % world, meta['batch_index'] = i) with rank 0's teacher BatchNorm
    statistics (broadcast first: train-mode teachers keep per-rank running
    statistics); the per-batch (errs, accs, bs) rows are gathered and folded
    into the AvgCounters in the single-device batch order, so the records are
    exactly what one device computes (projects/MT_UBPL.py:393-397 weights:
    bs per keypoint entry, bs*k for the mean entry)."""
    from .evaluation import EvaluationUtils
    from .losses import AvgCounters
    from .process import inverse_transforms
    n = len(models_ema) + 1
    D.broadcast_buffers(models_ema)
    for e in models_ema:
        e.eval()
    dev = models_ema[0].flat_params.device
    rows = []                                    # (batch index, bs, k, host row, preds)
    with torch.no_grad():
        for bat, (imgMap, heatmap, meta) in enumerate(validLoader):
            img = imgMap.to(dev, non_blocking=True).float().contiguous()
            bs, k = meta["kpsMap"].shape[:2]
            tinv = inverse_transforms(meta["center"], meta["scale"], [args.outRes, args.outRes]).to(dev)
            pm = []
            for e in models_ema:
                o = e(img)
                o = o[0] if isinstance(o, tuple) else o
                _, p, _ = Kn.decode_heatmaps(o[:, -1].contiguous(), tinv)
                pm.append(p)
            pm.append(torch.stack(pm, -1).mean(-1))                   # :387 preds_mean
            gts = meta["kpsMap"].to(dev).float().contiguous()
            outs = [EvaluationUtils.acc_pck(p, gts, args.pck_ref, args.pck_thr) for p in pm]
            host = torch.cat([torch.cat([er, ac]) for er, ac in outs] + [p.reshape(-1) for p in pm]).cpu()
            rows.append((meta.get("batch_index"), bs, k, host))
    rows = gather_valid_rows(rows)
    accs_c = [AvgCounters() for _ in range(n)]
    errs_c = [AvgCounters() for _ in range(n)]
    preds_arr = [[] for _ in range(n)]
    for _, bs, k, host in rows:
        for mi in range(n):
            errs = host[mi * 2 * (k + 1):mi * 2 * (k + 1) + k + 1]
            accs = host[mi * 2 * (k + 1) + k + 1:(mi + 1) * 2 * (k + 1)]
            for idx in range(k + 1):
                accs_c[mi].update(idx, accs[idx].item(), bs if idx < k else bs * k)
                errs_c[mi].update(idx, errs[idx].item(), bs if idx < k else bs * k)
        base = n * 2 * (k + 1)
        for mi in range(n):
            preds_arr[mi] += host[base + mi * bs * k * 2:base + (mi + 1) * bs * k * 2].reshape(bs, k, 2).tolist()
    for e in models_ema:
        e.train()
    return preds_arr, [c.avg() for c in accs_c], [c.avg() for c in errs_c]
