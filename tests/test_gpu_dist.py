"""§8e on the real step: MT_UBPL data parallelism with the HIP kernels.

Two ranks (torch.distributed, gloo, both on the one GPU of the box) each run
train_mt_ubpl on half of the golden mt_ubpl batch (one unlabeled + one
labeled row each).  Checked:
* both ranks end with bit-identical students and teachers (the SUM
  all-reduce gives every rank the same gradient, the EMA is replica-local);
* the all-reduced gradient equals, bit for bit, the sum of the two shard
  gradients computed here in ONE process with the global normalisers
  (train._sync_stats returning the sum of both shards' counts — dist.py
  exchange 1 — and world() = 2 for the consistency normaliser and the FDL
  share, train.py _fdl_total);
* the records are the global-batch records.
BatchNorm statistics are per rank, so the sharded step is not
the single-device B=4 step; this is the exact statement of what it is.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import seeds

pytestmark = pytest.mark.gpu
CASE = "mt_ubpl"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard(obj, rows):
    if torch.is_tensor(obj):
        return obj[rows].clone() if obj.dim() and obj.shape[0] == 4 else obj
    if isinstance(obj, (list, tuple)):
        return type(obj)(_shard(v, rows) for v in obj)
    if isinstance(obj, dict):
        return {k: _shard(v, rows) for k, v in obj.items()}
    return obj


ROWS = [[0, 2], [1, 3]]            # unlabeled rows 0-1, labeled rows 2-3 (TwoStreamBatchSampler order)


def _setup(rows, case=CASE):
    from ubpl_amd.hourglass import StackedHourglass
    from ubpl_amd.optim import FlatAdamW
    from oracle import render as OR
    cfg = seeds.step_cases()[case]
    models, emas, _ = seeds.step_models(lambda k, s, m: StackedHourglass(k, s, m), cfg, device="cuda")
    optims = [FlatAdamW(m, lr=cfg["lr"], weight_decay=0) for m in models]
    loader, args = seeds.step_batch(cfg, OR.kps_heatmap_torch)
    return models, emas, optims, [_shard(loader[0], rows)], args


def _snap_grads(T, models, store, mp_, orig):
    def snap(*a, **k):
        torch.cuda.synchronize()
        store.extend(m.flat_grads.detach().cpu().clone() for m in models)
        return orig(*a, **k)
    mp_.setattr(T, "_step_and_ema", snap)


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import contextlib
        import io
        from ubpl_amd import train as T
        mpatch = pytest.MonkeyPatch()
        models, emas, optims, loader, args = _setup(ROWS[rank])
        grads = []
        _snap_grads(T, models, grads, mpatch, T._step_and_ema)
        with contextlib.redirect_stdout(io.StringIO()):
            rec = T.train_mt_ubpl(loader, models, emas, optims, args)
        torch.cuda.synchronize()
        torch.save({"rec": rec, "grads": grads, "params": [m.flat_params.cpu() for m in models + emas],
                    "stats": [m.flat_stats.cpu() for m in models]}, os.path.join(out, "rank%d.pt" % rank))
        mpatch.undo()
    finally:
        dist.destroy_process_group()


def _single_process_shards(monkeypatch):
    """Each shard's gradient in one process with the global normalisers."""
    from ubpl_amd import dist as D
    from ubpl_amd import train as T
    import contextlib
    import io
    seen = []
    orig_sync, orig_step = T._sync_stats, T._step_and_ema
    monkeypatch.setattr(T, "_sync_stats", lambda s, c: (seen.append((s.clone(), c.clone())), (c, s))[1])
    for rows in ROWS:                                          # pass 1: each shard's local sums / counts
        models, emas, optims, loader, args = _setup(rows)
        with contextlib.redirect_stdout(io.StringIO()):
            T.train_mt_ubpl(loader, models, emas, optims, args)
    gsum, gcnt = seen[0][0] + seen[1][0], seen[0][1] + seen[1][1]
    monkeypatch.setattr(T, "_sync_stats", lambda s, c: (gcnt, gsum))
    monkeypatch.setattr(D, "world", lambda: 2)
    shard_grads, recs = [], []
    for rows in ROWS:                                          # pass 2: global normalisers
        models, emas, optims, loader, args = _setup(rows)
        g = []
        _snap_grads(T, models, g, monkeypatch, orig_step)
        with contextlib.redirect_stdout(io.StringIO()):
            recs.append(T.train_mt_ubpl(loader, models, emas, optims, args))
        shard_grads.append(g)
    monkeypatch.setattr(T, "_sync_stats", orig_sync)
    return shard_grads, recs


@pytest.mark.timeout(300)
def test_dp_two_ranks_real_step(tmp_path, monkeypatch):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    r0 = torch.load(os.path.join(tmp_path, "rank0.pt"), weights_only=True)
    r1 = torch.load(os.path.join(tmp_path, "rank1.pt"), weights_only=True)
    for a, b in zip(r0["params"], r1["params"]):
        assert torch.equal(a, b)                               # replicas stay identical
    for a, b in zip(r0["grads"], r1["grads"]):
        assert torch.equal(a, b)
    shard_grads, recs = _single_process_shards(monkeypatch)
    for mi in range(2):
        n = r0["grads"][mi].numel()
        want = shard_grads[0][mi] + shard_grads[1][mi]
        live = slice(0, n)
        assert torch.equal(r0["grads"][mi][live], want[live]), \
            float((r0["grads"][mi] - want).abs().max())
    # the records are the global ones (each pass-2 shard reports the global records)
    flat = lambda r: np.array([v for x in r for v in (x if isinstance(x, list) else [x])], np.float64)  # noqa: E731
    np.testing.assert_allclose(flat(r0["rec"]), flat(recs[0]), rtol=1e-6)


def _worker_graph(rank, world, port, out, case=CASE, backend="gloo"):
    """Four MT_UBPL (or DualPose_UBPL) steps per rank, eager and then captured
    (2 eager warm-up steps, the capture as graph segments around the two
    collectives, replays), each from freshly seeded networks.  backend "nccl"
    (RCCL): one rank with the distributed path forced on (UBPL_DIST_WORLD1)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if backend == "nccl":
        os.environ["UBPL_DIST_WORLD1"] = "1"
    import torch.distributed as dist
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import contextlib
        import io
        from ubpl_amd import train as T
        from ubpl_amd import dist as D
        assert D.is_dist()
        res = {}
        for mode in ("0", "1"):
            os.environ["UBPL_STEP_GRAPH"] = mode
            T._StepGraph.clear()
            models, emas, optims, loader, args = _setup(ROWS[rank] if world > 1 else [0, 1, 2, 3], case)
            dual = seeds.step_cases()[case]["project"] == "DualPose_UBPL"
            train, core = (T.train_dualpose_ubpl, T._dualpose_core) if dual else (T.train_mt_ubpl, T._mt_ubpl_core)
            with contextlib.redirect_stdout(io.StringIO()):
                rec = train(loader * 4, models, emas, optims, args)
            runner = T._StepGraph.get(core, models, emas, optims, args)
            torch.cuda.synchronize()
            res[mode] = {"rec": rec, "segments": len(runner.graph) if runner.graph else 0,
                         "params": [m.flat_params.cpu() for m in models + emas],
                         "stats": [m.flat_stats.cpu() for m in models + emas]}
            T._StepGraph.clear()
        torch.save(res, os.path.join(out, "graph_rank%d.pt" % rank))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("case", ["mt_ubpl", "dualpose"])
def test_dp_two_ranks_segmented_graph_matches_eager(tmp_path, case):
    """under torch.distributed the step is captured as
    graph segments (forward + losses | backward + merge | AdamW + EMA +
    records) with the two collectives run eagerly between their replays, for
    the MT_UBPL and the DualPose_UBPL steps.  Two gloo ranks: after 4 steps
    every rank's networks, BN statistics and records are bit-identical to its
    4 eager steps, and the replicas agree."""
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker_graph, args=(r, 2, port, str(tmp_path), case)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    rs = [torch.load(os.path.join(tmp_path, "graph_rank%d.pt" % r), weights_only=True) for r in range(2)]
    for r in rs:
        assert r["0"]["segments"] == 0 and r["1"]["segments"] == 3
        for what in ("params", "stats"):
            for a, b in zip(r["0"][what], r["1"][what]):
                assert torch.equal(a, b), what
        assert r["0"]["rec"] == r["1"]["rec"]
    for a, b in zip(rs[0]["1"]["params"], rs[1]["1"]["params"]):
        assert torch.equal(a, b)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("case", ["mt_ubpl", "dualpose"])
def test_rccl_segmented_graph_matches_eager(tmp_path, case):
    """the captured step under torch.distributed on the backend that runs
    it in production, RCCL ("nccl"): one rank (RCCL takes one rank per device; the
    box has one GPU) with the distributed path forced on, so both collectives run
    through RCCL between the segment replays — ProcessGroupNCCL's watchdog thread
    beside the thread_local captures, the synchronous all-reduce ordered between
    replays, recordStream on tensors of the graph's pool.  After 4 steps the
    captured run (3 segments) equals the eager run bit for bit: networks, BN
    statistics and records."""
    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_worker_graph, args=(0, 1, _free_port(), str(tmp_path), case, "nccl"))
    p.start()
    p.join(timeout=240)
    assert p.exitcode == 0
    r = torch.load(os.path.join(tmp_path, "graph_rank0.pt"), weights_only=True)
    assert r["0"]["segments"] == 0 and r["1"]["segments"] == 3
    for what in ("params", "stats"):
        for a, b in zip(r["0"][what], r["1"][what]):
            assert torch.equal(a, b), what
    assert r["0"]["rec"] == r["1"]["rec"]
