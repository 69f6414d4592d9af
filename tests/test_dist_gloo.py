"""N>1 data-parallel logic on the CPU (gloo, world_size 2, 127.0.0.1).

Checks the two exchanges of ubpl_amd.train / ubpl_amd.dist:
1. global normalisers: each rank divides its LOCAL loss sum by the GLOBAL
   count (_sync_stats), so after a SUM all-reduce of the gradients the
   sharded step has exactly the single-process global-batch gradient;
2. broadcast of the flat parameter / statistics buffers from rank 0.
The loss is the oracle's JointMSELoss restatement on a tiny 1x1-conv
"network", so the test needs no GPU.
"""
import os
import socket
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    g = torch.Generator().manual_seed(0)
    B, C, K, R = 8, 6, 4, 8
    x = torch.randn(B, C, R, R, generator=g)
    gts = torch.rand(B, K, R, R, generator=g)
    gate = (torch.rand(B, K, generator=g) > 0.3).float()
    isl = torch.tensor([0, 1, 0, 1, 1, 0, 1, 1], dtype=torch.bool)
    gate[~isl] = 0
    w0 = torch.randn(K, C, 1, 1, generator=g)
    return x, gts, gate, isl, w0


def _loss_parts(w, x, gts, gate, isl):
    from oracle import losses as OL
    preds = torch.nn.functional.conv2d(x, w).unsqueeze(1).repeat(1, 2, 1, 1, 1)   # 2 "stacks"
    sw = isl.float()[:, None]
    return OL.joint_mse(preds, gts, 2, gate, sw, True, True)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ubpl_amd import dist as D
        from ubpl_amd.train import _norm, _sync_stats
        x, gts, gate, isl, w0 = _data()
        sl = slice(rank, None, world)
        w = w0.clone().requires_grad_(True)
        s, n = _loss_parts(w, x[sl], gts[sl], gate[sl], isl[sl])
        counts, sums = _sync_stats(s.detach().reshape(1), torch.tensor([float(n)]))
        loss = 10.0 * _norm(s, counts[0])
        loss.backward()
        g = w.grad.clone()
        D.allreduce_(g)
        glob = 10.0 * _norm(sums[0], counts[0])
        # flat-buffer broadcast from rank 0
        fake = types.SimpleNamespace(flat_params=torch.full((5,), float(rank + 1)),
                                     flat_stats=torch.full((3,), float(rank + 7)))
        D.broadcast_params([fake])
        # plain lists: a tensor would travel as a shared-memory fd that dies with this process
        q.put((rank, g.tolist(), float(glob), fake.flat_params.tolist(), fake.flat_stats.tolist(),
               D.world(), D.rank()))
    finally:
        dist.destroy_process_group()


def test_dp_global_normalisers_match_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    x, gts, gate, isl, w0 = _data()
    w = w0.clone().requires_grad_(True)
    s, n = _loss_parts(w, x, gts, gate, isl)
    loss = 10.0 * (s / n)
    loss.backward()
    for rank, g, glob, fp, fs, world, rk in res:
        assert world == 2 and rk == rank
        torch.testing.assert_close(torch.tensor(g), w.grad, rtol=1e-5, atol=1e-7)
        assert abs(glob - loss.item()) <= 1e-5 * abs(loss.item())
        assert fp == [1.0] * 5 and fs == [7.0] * 3


def _fdl_data():
    g = torch.Generator().manual_seed(3)
    B, C, S, Cf, R = 8, 5, 2, 6, 4
    x = torch.randn(B, C, R, R, generator=g)
    isl = torch.tensor([1, 0, 1, 1, 0, 0, 1, 0], dtype=torch.bool)   # rank 1 (odd rows) has 1 labeled row
    wa = torch.randn(S * Cf, C, 1, 1, generator=g)
    wb = torch.randn(S * Cf, C, 1, 1, generator=g)
    return x, isl, wa, wb, (S, Cf)


def _feats(w, x, S, Cf):
    y = torch.nn.functional.conv2d(x, w)
    return y.reshape(x.shape[0], S, Cf, y.shape[-2], y.shape[-1])


def _fdl_local_views(wa, wb, x, isl, S, Cf, kind):
    """The per-view (kind, value, n_loc) triples train._fdl_view produces,
    computed with the oracle's restatement on this rank's selected rows."""
    from oracle import losses as OL
    fa, fb = _feats(wa, x, S, Cf), _feats(wb, x, S, Cf)
    views = []
    for a in range(2):                                   # two views: the second one shifted
        f1, f2 = (fa, fb) if a == 0 else (fa * 0.5 + 0.1, fb - 0.2)
        rows = isl
        n_rows = int(rows.sum())
        if kind == "cov":
            if n_rows:
                v, n = OL.features_cov(f1[rows], f2[rows])
            else:
                v, n = torch.zeros(()) * wa.sum(), 0
            views.append(("cov", v, torch.tensor([float(n)])))
        else:
            v, n = OL.joint_feature_dist(f1[rows], f2[rows]) if n_rows else (torch.zeros(()) * wa.sum(), 0)
            views.append(("dist", v, torch.tensor([float(n)])))
    return views


def _fdl_worker(rank, world, port, q, kind):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ubpl_amd import dist as D
        from ubpl_amd.train import _fdl_record, _fdl_record_sums, _fdl_total, _sync_stats
        x, isl, wa0, wb0, (S, Cf) = _fdl_data()
        sl = slice(rank, None, world)
        wa, wb = wa0.clone().requires_grad_(True), wb0.clone().requires_grad_(True)
        views = _fdl_local_views(wa, wb, x[sl], isl[sl], S, Cf, kind)
        counts = torch.stack([n[0] for _, _, n in views])
        gcounts, gsums = _sync_stats(torch.stack(_fdl_record_sums(views)), counts)
        fdc = _fdl_total(views, gcounts, world, 1.5)
        fdc.backward()
        ga, gb = wa.grad.clone(), wb.grad.clone()
        D.allreduce_(ga)
        D.allreduce_(gb)
        rec = _fdl_record(views, gsums, gcounts, world, 1.5)
        q.put((rank, ga.tolist(), gb.tolist(), float(rec)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["cov", "dist"])
def test_dp_fdl_matches_single_process(kind):
    """FDL under data parallelism: a covariance view is a MEAN over
    each rank's rows; _fdl_total rescales it by n_loc / N_glob so the SUM
    all-reduced gradient and the record equal one device running the global
    batch (projects/MT_UBPL.py:301-330), also with unequal labeled rows per rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fdl_worker, args=(r, 2, port, q, kind)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from ubpl_amd.train import _fdl_record, _fdl_total
    x, isl, wa0, wb0, (S, Cf) = _fdl_data()
    wa, wb = wa0.clone().requires_grad_(True), wb0.clone().requires_grad_(True)
    views = _fdl_local_views(wa, wb, x, isl, S, Cf, kind)
    counts = torch.stack([n[0] for _, _, n in views])
    # the reference: fdc = W * sum_a value_a / sum_a n_a on one device
    ref = 1.5 * sum(v for _, v, _ in views) / counts.sum()
    ref.backward()
    ours = _fdl_total(views, counts, 1, 1.5)
    assert abs(float(ours) - float(ref)) <= 1e-6 * abs(float(ref))
    rec1 = _fdl_record(views, None, counts, 1, 1.5)
    assert abs(float(rec1) - float(ref)) <= 1e-6 * abs(float(ref))
    for rank, ga, gb, rec in res:
        torch.testing.assert_close(torch.tensor(ga), wa.grad, rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(torch.tensor(gb), wb.grad, rtol=1e-5, atol=1e-7)
        assert abs(rec - float(ref)) <= 1e-5 * abs(float(ref)), (rec, float(ref))


def test_single_process_helpers_are_identity():
    from ubpl_amd import dist as D
    from ubpl_amd.train import _sync_stats
    t = torch.tensor([1.0, 2.0])
    assert D.allreduce_(t) is t and D.world() == 1 and D.rank() == 0
    c, s = _sync_stats(torch.tensor([3.0]), torch.tensor([4.0]))
    assert float(c[0]) == 4.0 and float(s[0]) == 3.0


def _valid_rows_worker(rank, world, port, q, tagged):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import warnings
        from ubpl_amd.train import gather_valid_rows
        # sharded loader: rank r holds batches r, r + world, ... (mouse.valid_batches);
        # plain loader: every rank iterates batches 0..3 itself (no batch_index)
        idx = range(rank, 5, world) if tagged else range(4)
        rows = [(i if tagged else None, 2, 3, torch.full((4,), float(10 * i + (rank if not tagged else 0))))
                for i in idx]
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            out = gather_valid_rows(rows)
        q.put((rank, [(bi, h.tolist()) for bi, _, _, h in out], len(w)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("tagged", [True, False])
def test_validate_rows_gather_only_with_batch_index(tagged):
    """validate() folds the gathered rows in batch_index
    order only when every rank's loader tags them; a plain loader keeps each
    rank's own rows (no W-fold duplication, no interleaving) and warns."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_valid_rows_worker, args=(r, 2, port, q, tagged)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, rows, nwarn in res:
        if tagged:
            assert [bi for bi, _ in rows] == [0, 1, 2, 3, 4] and nwarn == 0
            assert [h[0] for _, h in rows] == [0.0, 10.0, 20.0, 30.0, 40.0]
        else:
            assert [bi for bi, _ in rows] == [None] * 4 and nwarn == 1
            assert [h[0] for _, h in rows] == [10.0 * i + rank for i in range(4)]
