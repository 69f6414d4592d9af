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


def test_single_process_helpers_are_identity():
    from ubpl_amd import dist as D
    from ubpl_amd.train import _sync_stats
    t = torch.tensor([1.0, 2.0])
    assert D.allreduce_(t) is t and D.world() == 1 and D.rank() == 0
    c, s = _sync_stats(torch.tensor([3.0]), torch.tensor([4.0]))
    assert float(c[0]) == 4.0 and float(s[0]) == 3.0
