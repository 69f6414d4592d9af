"""Split MFMA convolutions (conv_split.hip) vs float64 references.

The exact-f32 MFMA path (conv.hip) is the yardstick: on the same inputs the
3-piece bf16 path (npieces=3, "6xbf16", exact operands) and the 2-piece fp16
path (npieces=2, "2xfp16": operands to 2^-22, 3 products) must land within
F16_BAR / 2x the f32 path's own error against float64.  Weight re-layout,
prologue, padding, residual, split-K and the data-gradient layout are all
exercised.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ubpl_amd import _lib
    _lib.load()


@pytest.fixture()
def _lib_dispatch():
    """The C library (ctypes) for the halo-dispatch test hook; the dispatch the
    process started with (the environment's UBPL_PSA_HALO / UBPL_PSA_TEAMS) is
    restored after the test."""
    from ubpl_amd import _lib
    lib = _lib.lib()
    yield lib
    assert lib.ubpl_set_psa_dispatch(-2, -2) == 0


def _rel(a, ref):
    a = a.detach().cpu().double()
    return float((a - ref).norm() / ref.norm())


# the bar of the 2xfp16 path against float64: F16_BAR x the exact-f32 kernel's own error, or its
# representation floor — each fp16-piece operand is carried to 2^-22 (the f32 input itself to
# 2^-24), so a layer's output sits near 2^-22 relative whatever K; the exact-f32 chain's error
# grows with K instead (tools/experiments/f16_split_numerics.hip: at K = 1152 the 2xfp16 sum is
# 0.44x the f32 chain's error, at K = 128-256 1x1 convs 0.5-3.5x).  6xbf16: 2x, no floor.
F16_BAR = 4.0
F16_FLOOR = 2.0 ** -21


def _bar(npieces):
    return F16_BAR if npieces == 2 else 2.0


def _ok(esp, e32, npieces):
    return esp <= _bar(npieces) * e32 + 1e-8 or (npieces == 2 and esp <= F16_FLOOR)


# (B, Cin, H, Cout, KS, prologue, residual): the hourglass shapes (1x1 and 3x3
# at the large and the split-K-sized planes, Cout 16 / 64 / 128 / 256)
CASES = [
    (2, 128, 64, 128, 3, True, False),
    (4, 128, 8, 128, 3, True, False),     # small grid: split-K + reduce
    (2, 64, 32, 64, 3, True, False),
    (2, 256, 16, 128, 1, True, False),
    (2, 128, 16, 256, 1, True, True),
    (2, 256, 64, 16, 1, False, False),    # preds head (Cout 16)
    (2, 16, 32, 256, 1, False, True),     # merge_preds (Cin 16)
    (3, 256, 4, 256, 1, True, True),
]


@pytest.mark.parametrize("npieces", [3])
@pytest.mark.parametrize("case", CASES)
def test_split_forward_and_dgrad_vs_f64(case, npieces):
    from ubpl_amd import kernels as Kn
    B, Cin, H, Cout, KS, pro, resid = case
    gen = torch.Generator().manual_seed(11 + hash(case) % 1000)
    x = torch.randn(B, Cin, H, H, generator=gen, dtype=torch.float64)
    w = torch.randn(Cout, Cin, KS, KS, generator=gen, dtype=torch.float64) / np.sqrt(Cin * KS * KS)
    b = torch.randn(Cout, generator=gen, dtype=torch.float64)
    sc = torch.rand(Cin, generator=gen, dtype=torch.float64) + 0.5
    sh = torch.randn(Cin, generator=gen, dtype=torch.float64) * 0.5
    res = torch.randn(B, Cout, H, H, generator=gen, dtype=torch.float64) if resid else None
    # the f32 inputs both paths see, and the float64 result on exactly those
    x32, w32, b32, sc32, sh32 = (t.float() for t in (x, w, b, sc, sh))
    res32 = res.float() if resid else None
    inp = F.relu(x32.double() * sc32.double()[None, :, None, None] + sh32.double()[None, :, None, None]) if pro \
        else x32.double()
    yref = F.conv2d(inp, w32.double(), b32.double(), 1, (KS - 1) // 2)
    if resid:
        yref = yref + res32.double()
    d = lambda t: None if t is None else t.to(DEV)
    ps, ph = (d(sc32), d(sh32)) if pro else (None, None)
    y_f32 = Kn.conv2d_forward(d(x32), d(w32), d(b32), 1, ps, ph, res=d(res32))
    ws = Kn.conv_weight_split(d(w32), 0, npieces)
    y_sp = Kn.conv2d_forward_split(d(x32), ws, d(b32), ps, ph, res=d(res32))
    e32, esp = _rel(y_f32, yref), _rel(y_sp, yref)
    print("fwd %s np=%d: f32 %.2e split %.2e" % (case, npieces, e32, esp))
    if npieces == 3:
        assert esp <= 2 * e32 + 1e-8, (esp, e32)
    else:
        assert esp <= 4e-5, (esp, e32)
    # data gradient: dx = conv(dy, flip(w)^T) through the mode-1 split layout
    dy = torch.randn(B, Cout, H, H, generator=gen, dtype=torch.float64).float()
    dxref = torch.nn.grad.conv2d_input((B, Cin, H, H), w32.double(), dy.double(), 1, (KS - 1) // 2)
    wd = Kn.conv_weight_split(d(w32), 1, npieces)
    dx_sp = Kn.conv2d_forward_split(d(dy), wd, None)
    dx_f32 = Kn.conv2d_dgrad(d(dy), d(w32))
    e32, esp = _rel(dx_f32, dxref), _rel(dx_sp, dxref)
    print("dgrad %s np=%d: f32 %.2e split %.2e" % (case, npieces, e32, esp))
    if npieces == 3:
        assert esp <= 2 * e32 + 1e-8, (esp, e32)
    else:
        assert esp <= 4e-5, (esp, e32)


def test_split_weights_reconstruct():
    """The pieces sum back to the f32 weight: exactly for 3 bf16 pieces; for 2 fp16
    pieces to 2^-22 of each weight, after the power-of-two weight scale
    2^(9 + ceil(log2 sqrt K)) (K = 144 here: 2^13)."""
    from ubpl_amd import kernels as Kn
    gen = torch.Generator().manual_seed(3)
    w = torch.randn(32, 16, 3, 3, generator=gen) / 12.0
    # grouped tap-major order: wt[co][ci/16][tap][ci%16]
    ref = w.reshape(32, 1, 16, 9).permute(0, 1, 3, 2).reshape(-1).double()
    for npieces in (2, 3):
        ws = Kn.conv_weight_split(w.to(DEV), 0, npieces)
        planes = ws.buf.view(npieces, ws.plane)[:, :w.numel()].cpu()
        if npieces == 3:
            f = lambda p: (planes[p].to(torch.int32) << 16).view(torch.float32)
            tot = sum(f(p).double() for p in range(npieces))
            assert torch.equal(tot, ref)
        else:
            tot = (planes[0].view(torch.float16).double() + planes[1].view(torch.float16).double()) / 2.0 ** 13
            err = float(((tot - ref).abs() / ref.abs().clamp_min(1e-30)).max())
            assert err <= 2.0 ** -22, err


@pytest.mark.parametrize("npieces", [2, 3])
@pytest.mark.parametrize("case", CASES)
def test_psa_forward_and_dgrad_vs_f64(case, npieces):
    """Pre-split activations (fused BN+ReLU+split pass) + LDS-DMA conv: same bar
    as the register-staged split path (2xfp16: F16_BAR)."""
    from ubpl_amd import kernels as Kn
    B, Cin, H, Cout, KS, pro, resid = case
    gen = torch.Generator().manual_seed(23 + hash(case) % 1000)
    x32 = torch.randn(B, Cin, H, H, generator=gen)
    w32 = torch.randn(Cout, Cin, KS, KS, generator=gen) / np.sqrt(Cin * KS * KS)
    b32 = torch.randn(Cout, generator=gen)
    sc32 = torch.rand(Cin, generator=gen) + 0.5
    sh32 = torch.randn(Cin, generator=gen) * 0.5
    res32 = torch.randn(B, Cout, H, H, generator=gen) if resid else None
    inp = F.relu(x32.double() * sc32.double()[None, :, None, None] + sh32.double()[None, :, None, None]) if pro \
        else x32.double()
    yref = F.conv2d(inp, w32.double(), b32.double(), 1, (KS - 1) // 2)
    if resid:
        yref = yref + res32.double()
    d = lambda t: None if t is None else t.to(DEV)
    ps, ph = (d(sc32), d(sh32)) if pro else (None, None)
    y_f32 = Kn.conv2d_forward(d(x32), d(w32), d(b32), 1, ps, ph, res=d(res32))
    for pad in sorted({(KS - 1) // 2, 1}):
        xs = Kn.split_activation(d(x32), npieces, pad, ps, ph)
        ws = Kn.conv_weight_split(d(w32), 0, npieces)
        y_sp = Kn.conv2d_forward_psa(xs, ws, d(b32), res=d(res32))
        e32, esp = _rel(y_f32, yref), _rel(y_sp, yref)
        print("psa fwd %s np=%d pad=%d: f32 %.2e split %.2e" % (case, npieces, pad, e32, esp))
        assert _ok(esp, e32, npieces), (esp, e32)
    dy = torch.randn(B, Cout, H, H, generator=gen)
    dxref = torch.nn.grad.conv2d_input((B, Cin, H, H), w32.double(), dy.double(), 1, (KS - 1) // 2)
    ys = Kn.split_activation(d(dy), npieces, (KS - 1) // 2)
    wd = Kn.conv_weight_split(d(w32), 1, npieces)
    dx_sp = Kn.conv2d_forward_psa(ys, wd, None)
    dx_f32 = Kn.conv2d_dgrad(d(dy), d(w32))
    e32, esp = _rel(dx_f32, dxref), _rel(dx_sp, dxref)
    print("psa dgrad %s np=%d: f32 %.2e split %.2e" % (case, npieces, e32, esp))
    assert _ok(esp, e32, npieces), (esp, e32)


@pytest.mark.parametrize("case", CASES)
def test_bf16_psa_forward_and_dgrad_vs_rounded_f64(case):
    """The "bf16" precision (one piece per operand): the PSA kernels with NP = 1
    compute the conv of the bf16-rounded (RNE) operands with f32 accumulation —
    against float64 on exactly those rounded operands, to f32 summation error."""
    from ubpl_amd import kernels as Kn
    B, Cin, H, Cout, KS, pro, resid = case
    gen = torch.Generator().manual_seed(29 + hash(case) % 1000)
    x32 = torch.randn(B, Cin, H, H, generator=gen)
    w32 = torch.randn(Cout, Cin, KS, KS, generator=gen) / np.sqrt(Cin * KS * KS)
    b32 = torch.randn(Cout, generator=gen)
    sc32 = torch.rand(Cin, generator=gen) + 0.5
    sh32 = torch.randn(Cin, generator=gen) * 0.5
    res32 = torch.randn(B, Cout, H, H, generator=gen) if resid else None
    bf = lambda t: t.to(torch.bfloat16).double()
    inp = F.relu((x32.double() * sc32.double()[None, :, None, None] + sh32.double()[None, :, None, None]).float()) \
        if pro else x32
    yref = F.conv2d(bf(inp), bf(w32), b32.double(), 1, (KS - 1) // 2)
    if resid:
        yref = yref + res32.double()
    d = lambda t: None if t is None else t.to(DEV)
    ps, ph = (d(sc32), d(sh32)) if pro else (None, None)
    for pad in sorted({(KS - 1) // 2, 1}):
        xs = Kn.split_activation(d(x32), 1, pad, ps, ph)
        ws = Kn.conv_weight_split(d(w32), 0, 1)
        y = Kn.conv2d_forward_psa(xs, ws, d(b32), res=d(res32))
        e = _rel(y, yref)
        print("bf16 psa fwd %s pad=%d: %.2e" % (case, pad, e))
        assert e <= 2e-6, (pad, e)
    dy = torch.randn(B, Cout, H, H, generator=gen)
    dxref = torch.nn.grad.conv2d_input((B, Cin, H, H), bf(w32), bf(dy), 1, (KS - 1) // 2)
    ys = Kn.split_activation(d(dy), 1, (KS - 1) // 2)
    wd = Kn.conv_weight_split(d(w32), 1, 1)
    e = _rel(Kn.conv2d_forward_psa(ys, wd, None), dxref)
    print("bf16 psa dgrad %s: %.2e" % (case, e))
    assert e <= 2e-6, e


@pytest.mark.parametrize("case", [(2, 128, 128, 64, 64), (2, 64, 64, 32, 32), (3, 128, 64, 16, 32)])
def test_bf16_wgrad3_psa_vs_rounded_f64(case):
    """3x3 weight gradient with NP = 1 operands vs float64 of the bf16-rounded operands."""
    from ubpl_amd import kernels as Kn
    B, Cin, Cout, H, W = case
    gen = torch.Generator().manual_seed(43 + hash(case) % 1000)
    x = torch.randn(B, Cin, H, W, generator=gen)
    dy = torch.randn(B, Cout, H, W, generator=gen)
    sc, sh = torch.rand(Cin, generator=gen) + 0.5, torch.randn(Cin, generator=gen) * 0.5
    bf = lambda t: t.to(torch.bfloat16).double()
    inp = F.relu((x.double() * sc.double()[None, :, None, None] + sh.double()[None, :, None, None]).float())
    dwref = torch.nn.grad.conv2d_weight(bf(inp), (Cout, Cin, 3, 3), bf(dy), 1, 1)
    dbref = bf(dy).sum((0, 2, 3))
    d = lambda t: t.to(DEV)
    xs = Kn.split_activation(d(x), 1, 1, d(sc), d(sh))
    ys = Kn.split_activation(d(dy), 1, 1)
    assert Kn.wgrad3_psa_ok(ys, xs)
    dw, db = torch.zeros(Cout, Cin, 3, 3, device=DEV), torch.zeros(Cout, device=DEV)
    Kn.conv2d_wgrad3_psa(ys, xs, dw, db, accumulate=False)
    e = _rel(dw, dwref)
    print("bf16 wgrad3 %s: %.2e" % (case, e))
    assert e <= 2e-6, e
    assert _rel(db, dbref) <= 1e-5


@pytest.mark.parametrize("case", [(2, 256, 64, 128, True, True), (2, 128, 32, 256, True, False),
                                  (3, 64, 16, 64, False, True)])
def test_bf16_conv1x1_split_load_vs_rounded_f64(case):
    """conv1x1_sol_kernel with NP = 1 (the "bf16" precision's 1x1 convs where the
    plane fills the chip: no pre-split pass): forward with prologue / residual
    and the data gradient equal float64 on the bf16-rounded (RNE) operands to
    f32 summation error, like the PSA kernels with NP = 1."""
    from ubpl_amd import kernels as Kn
    B, Cin, H, Cout, pro, resid = case
    gen = torch.Generator().manual_seed(61 + hash(case) % 1000)
    x32 = torch.randn(B, Cin, H, H, generator=gen)
    w32 = torch.randn(Cout, Cin, 1, 1, generator=gen) / np.sqrt(Cin)
    b32 = torch.randn(Cout, generator=gen)
    sc32 = torch.rand(Cin, generator=gen) + 0.5
    sh32 = torch.randn(Cin, generator=gen) * 0.5
    res32 = torch.randn(B, Cout, H, H, generator=gen) if resid else None
    bf = lambda t: t.to(torch.bfloat16).double()
    inp = F.relu((x32.double() * sc32.double()[None, :, None, None] + sh32.double()[None, :, None, None]).float()) \
        if pro else x32
    yref = F.conv2d(bf(inp), bf(w32), b32.double())
    if resid:
        yref = yref + res32.double()
    d = lambda t: None if t is None else t.to(DEV)
    ps, ph = (d(sc32), d(sh32)) if pro else (None, None)
    y = Kn.conv1x1_forward_split_load(d(x32), Kn.conv_weight_split(d(w32), 0, 1), d(b32), ps, ph, res=d(res32))
    e = _rel(y, yref)
    print("bf16 sol fwd %s: %.2e" % (case, e))
    assert e <= 2e-6, e
    if Cin % 64 == 0:
        dy = torch.randn(B, Cout, H, H, generator=gen)
        dxref = torch.nn.grad.conv2d_input((B, Cin, H, H), bf(w32), bf(dy))
        dx = Kn.conv1x1_forward_split_load(d(dy), Kn.conv_weight_split(d(w32), 1, 1), None)
        e = _rel(dx, dxref)
        print("bf16 sol dgrad %s: %.2e" % (case, e))
        assert e <= 2e-6, e


@pytest.mark.parametrize("case", [(2, 256, 128, 64, True), (3, 128, 256, 16, False), (2, 64, 128, 32, True),
                                  (2, 64, 64, 16, False)])
def test_bf16_wgrad1x1_split_load_vs_rounded_f64(case):
    """1x1 weight gradient with NP = 1 (bf16 operands, f32 accumulation) vs
    float64 of the bf16-rounded operands; the bias gradient sums the f32 dy."""
    from ubpl_amd import kernels as Kn
    B, Cin, Cout, H, pro = case
    gen = torch.Generator().manual_seed(67 + hash(case) % 1000)
    x = torch.randn(B, Cin, H, H, generator=gen)
    dy = torch.randn(B, Cout, H, H, generator=gen)
    sc, sh = torch.rand(Cin, generator=gen) + 0.5, torch.randn(Cin, generator=gen) * 0.5
    bf = lambda t: t.to(torch.bfloat16).double()
    inp = F.relu((x.double() * sc.double()[None, :, None, None] + sh.double()[None, :, None, None]).float()) \
        if pro else x
    dwref = torch.nn.grad.conv2d_weight(bf(inp), (Cout, Cin, 1, 1), bf(dy))
    dbref = dy.double().sum((0, 2, 3))
    d = lambda t: t.to(DEV)
    ps, ph = (d(sc), d(sh)) if pro else (None, None)
    dw, db = torch.zeros(Cout, Cin, 1, 1, device=DEV), torch.zeros(Cout, device=DEV)
    Kn.conv2d_wgrad1x1_split_load(d(dy), d(x), dw, db, ps, ph, accumulate=False, npieces=1)
    e = _rel(dw, dwref)
    print("bf16 wgrad1 %s: %.2e" % (case, e))
    assert e <= 2e-6, e
    assert _rel(db, dbref) <= 1e-5


def test_split_activation_layout():
    """PSA image: pieces sum back to relu(x*s+h) exactly, border zero, [B][C/16][Hp][Wp][16]."""
    from ubpl_amd import kernels as Kn
    gen = torch.Generator().manual_seed(4)
    x = torch.randn(2, 32, 5, 7, generator=gen)
    sc, sh = torch.rand(32, generator=gen) + 0.5, torch.randn(32, generator=gen)
    xs = Kn.split_activation(x.to(DEV), 3, 1, sc.to(DEV), sh.to(DEV))
    planes = xs.buf.view(3, xs.plane).cpu()
    f = lambda p: (planes[p].to(torch.int32) << 16).view(torch.float32).double()
    tot = (f(0) + f(1) + f(2)).view(2, 2, 7, 9, 16)
    # fmaf(x, s, h) = the f64 value of x*s + h rounded once to f32
    v = F.relu((x.double() * sc.double()[None, :, None, None] + sh.double()[None, :, None, None]).float()).double()
    ref = torch.zeros(2, 2, 7, 9, 16, dtype=torch.float64)
    ref[:, :, 1:6, 1:8, :] = v.view(2, 2, 16, 5, 7).permute(0, 1, 3, 4, 2)
    assert torch.equal(tot, ref)


@pytest.mark.parametrize("case", [(2, 128, 128, 64, 64), (3, 128, 128, 16, 32), (2, 256, 128, 32, 16),
                                  (2, 128, 256, 16, 16), (2, 64, 64, 32, 32), (2, 64, 128, 16, 16),
                                  (3, 128, 64, 16, 32)])
def test_wgrad3_psa_vs_f64(case):
    """3x3 weight + bias gradient from PSA operands (transposed LDS reads,
    split-K slab) within 2x the exact-f32 kernel's error against float64."""
    from ubpl_amd import kernels as Kn
    B, Cin, Cout, H, W = case
    gen = torch.Generator().manual_seed(41 + hash(case) % 1000)
    x = torch.randn(B, Cin, H, W, generator=gen)
    dy = torch.randn(B, Cout, H, W, generator=gen)
    sc, sh = torch.rand(Cin, generator=gen) + 0.5, torch.randn(Cin, generator=gen) * 0.5
    inp = F.relu((x.double() * sc.double()[None, :, None, None] + sh.double()[None, :, None, None]).float())
    dwref = torch.nn.grad.conv2d_weight(inp.double(), (Cout, Cin, 3, 3), dy.double(), 1, 1)
    dbref = dy.double().sum((0, 2, 3))
    d = lambda t: t.to(DEV)
    xs = Kn.split_activation(d(x), 3, 1, d(sc), d(sh))
    ys = Kn.split_activation(d(dy), 3, 1)
    assert Kn.wgrad3_psa_ok(ys, xs)
    dw = torch.full((Cout, Cin, 3, 3), 0.25, device=DEV)
    db = torch.full((Cout,), -0.5, device=DEV)
    Kn.conv2d_wgrad3_psa(ys, xs, dw, db, accumulate=True)
    dw32, db32 = torch.zeros(Cout, Cin, 3, 3, device=DEV), torch.zeros(Cout, device=DEV)
    Kn.conv2d_wgrad(d(dy), d(x), 3, 1, dw32, db32, d(sc), d(sh), accumulate=False)
    e32, esp = _rel(dw32, dwref), _rel(dw - 0.25, dwref)
    print("wgrad3 %s: f32 %.2e split %.2e" % (case, e32, esp))
    assert esp <= 2 * e32 + 1e-8, (esp, e32)
    assert _rel(db + 0.5, dbref) <= 1e-5


def test_bn_backward_split_matches_f32_then_split():
    """bn_backward_split == split_activation(bn_backward(...)) bit for bit (same
    per-element formula), dgamma/dbeta identical."""
    from ubpl_amd import kernels as Kn
    gen = torch.Generator().manual_seed(9)
    B, C, H, W = 2, 32, 8, 16
    d = lambda t: t.to(DEV)
    dz, x = d(torch.randn(B, C, H, W, generator=gen)), d(torch.randn(B, C, H, W, generator=gen))
    gamma = d(torch.rand(C, generator=gen) + 0.5)
    mean, istd = d(torch.randn(C, generator=gen) * 0.1), d(torch.rand(C, generator=gen) + 0.5)
    sc, sh = gamma * istd, d(torch.randn(C, generator=gen)) - mean * gamma * istd
    part = torch.zeros(int(__import__("ubpl_amd")._lib.lib().ubpl_bn_part_doubles(B, C)), dtype=torch.float64,
                       device=DEV)
    for npieces in (3, 1):
        outs = []
        for mode in ("f32", "split"):
            coef = torch.empty(3 * C + 1, device=DEV)
            dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
            if mode == "f32":
                dx = Kn.bn_backward(dz, x, gamma, mean, istd, sc, sh, 1, part, coef, dg, db,
                                    out=torch.empty_like(dz))
                ys = Kn.split_activation(dx, npieces, 1)
            else:
                ys = Kn.bn_backward_split(dz, x, gamma, mean, istd, sc, sh, 1, part, coef, dg, db, npieces, 1)
            outs.append((ys.buf.cpu(), dg.cpu(), db.cpu()))
        for a, b in zip(*outs):
            assert torch.equal(a, b), npieces


@pytest.mark.parametrize("mag", [1.0, 1e-6, 3e3])
@pytest.mark.parametrize("shape", [(2, 32, 8, 16), (4, 128, 16, 16), (2, 64, 64, 64)])
def test_bn_backward_split_2xfp16_scale(shape, mag):
    """bn_backward_split with npieces 2: the statistics pass bounds |dx| and picks a
    power-of-two scale s (coef[3C]) with 2^8 <= max|dx| * s <= 2^14, so the fp16
    pieces neither overflow nor sit in the subnormal range; the pieces carry dx * s
    to 2^-22 of each element (dx as bn_backward computes it), whatever the
    gradient's magnitude (mag scales dz); dgamma / dbeta as the 3-piece call's."""
    from ubpl_amd import kernels as Kn
    B, C, H, W = shape
    gen = torch.Generator().manual_seed(19 + C)
    d = lambda t: t.to(DEV)
    dz, x = d(torch.randn(B, C, H, W, generator=gen) * mag), d(torch.randn(B, C, H, W, generator=gen))
    gamma = d(torch.rand(C, generator=gen) + 0.5)
    mean, istd = d(torch.randn(C, generator=gen) * 0.1), d(torch.rand(C, generator=gen) + 0.5)
    sc, sh = gamma * istd, d(torch.randn(C, generator=gen)) - mean * gamma * istd
    part = torch.zeros(int(__import__("ubpl_amd")._lib.lib().ubpl_bn_part_doubles(B, C)), dtype=torch.float64,
                       device=DEV)
    coef = torch.full((3 * C + 1,), -1.0, device=DEV)
    dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    dx = Kn.bn_backward(dz, x, gamma, mean, istd, sc, sh, 1, part, coef, dg, db, out=torch.empty_like(dz))
    dg2, db2 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    ys = Kn.bn_backward_split(dz, x, gamma, mean, istd, sc, sh, 1, part, coef, dg2, db2, 2, 1)
    torch.cuda.synchronize()
    assert torch.equal(dg, dg2) and torch.equal(db, db2)
    s = float(ys.scale.item())
    m, e = np.frexp(s)
    assert m == 0.5, s                                          # a power of two
    amax = float(dx.abs().max())
    assert 2.0 ** 8 <= amax * s <= 2.0 ** 14, (amax, s)
    planes = ys.buf.view(2, ys.plane).cpu()
    img = (planes[0].view(torch.float16).double() + planes[1].view(torch.float16).double()) / s
    img = img.view(B, C // 16, H + 2, W + 2, 16)[:, :, 1:-1, 1:-1].permute(0, 1, 4, 2, 3).reshape(B, C, H, W)
    ref = dx.double().cpu()
    assert float(((img - ref).abs() - 2.0 ** -22 * ref.abs()).max()) <= 2.0 ** -26 * amax


@pytest.mark.parametrize("case", [(2, 128, 128, 64, 64), (3, 128, 128, 16, 32), (2, 64, 64, 32, 32),
                                  (2, 128, 128, 8, 8)])
def test_2xfp16_3x3_gradients_vs_f64(case):
    """The 2xfp16 backward of a 3x3 conv: dy through bn_backward_split (npieces 2, its
    device-side scale), the data gradient on the mode-1 fp16 weights and the weight
    gradient against the forward's fp16 image of the conv input, each within F16_BAR
    of the exact-f32 kernels' error against float64 (dy scaled small, as real
    gradients are)."""
    from ubpl_amd import kernels as Kn
    B, Cin, Cout, H, W = case
    gen = torch.Generator().manual_seed(61 + H)
    d = lambda t: t.to(DEV)
    x = torch.randn(B, Cin, H, W, generator=gen)
    w = torch.randn(Cout, Cin, 3, 3, generator=gen) / np.sqrt(Cin * 9)
    sc, sh = torch.rand(Cin, generator=gen) + 0.5, torch.randn(Cin, generator=gen) * 0.5
    # dy as the BN backward produces it (identity-like BN coefficients), magnitude ~1e-5
    dz = torch.randn(B, Cout, H, W, generator=gen) * 1e-5
    xb = torch.randn(B, Cout, H, W, generator=gen)
    gamma = torch.rand(Cout, generator=gen) + 0.5
    mean, istd = torch.randn(Cout, generator=gen) * 0.1, torch.rand(Cout, generator=gen) + 0.5
    bsc, bsh = gamma * istd, torch.randn(Cout, generator=gen) - mean * gamma * istd
    part = torch.zeros(int(__import__("ubpl_amd")._lib.lib().ubpl_bn_part_doubles(B, Cout)), dtype=torch.float64,
                       device=DEV)
    coef = torch.empty(3 * Cout + 1, device=DEV)
    dg, db_ = torch.zeros(Cout, device=DEV), torch.zeros(Cout, device=DEV)
    dy = Kn.bn_backward(d(dz), d(xb), d(gamma), d(mean), d(istd), d(bsc), d(bsh), 1, part, coef, dg, db_,
                        out=torch.empty(B, Cout, H, W, device=DEV))
    ys = Kn.bn_backward_split(d(dz), d(xb), d(gamma), d(mean), d(istd), d(bsc), d(bsh), 1, part, coef, None, None,
                              2, 1)
    dy64 = dy.double().cpu()
    # data gradient
    dxref = torch.nn.grad.conv2d_input((B, Cin, H, W), w.double(), dy64, 1, 1)
    dx = Kn.conv2d_forward_psa(ys, Kn.conv_weight_split(d(w), 1, 2), None)
    dx32 = Kn.conv2d_dgrad(dy, d(w))
    e32, e16 = _rel(dx32, dxref), _rel(dx, dxref)
    print("2xfp16 dgrad %s: f32 %.2e 2xfp16 %.2e" % (case, e32, e16))
    assert _ok(e16, e32, 2), (e16, e32)
    # weight gradient from the forward's 2xfp16 image
    inp = F.relu((x.double() * sc.double()[None, :, None, None] + sh.double()[None, :, None, None]).float())
    dwref = torch.nn.grad.conv2d_weight(inp.double(), (Cout, Cin, 3, 3), dy64, 1, 1)
    xs = Kn.split_activation(d(x), 2, 1, d(sc), d(sh))
    if Kn.wgrad3_psa_ok(ys, xs):
        dw, dbw = torch.zeros(Cout, Cin, 3, 3, device=DEV), torch.zeros(Cout, device=DEV)
        Kn.conv2d_wgrad3_psa(ys, xs, dw, dbw, accumulate=False)
        dw32, db32 = torch.zeros(Cout, Cin, 3, 3, device=DEV), torch.zeros(Cout, device=DEV)
        Kn.conv2d_wgrad(dy, d(x), 3, 1, dw32, db32, d(sc), d(sh), accumulate=False)
        e32, e16 = _rel(dw32, dwref), _rel(dw, dwref)
        print("2xfp16 wgrad %s: f32 %.2e 2xfp16 %.2e" % (case, e32, e16))
        assert _ok(e16, e32, 2), (e16, e32)
        assert _rel(dbw, dy64.sum((0, 2, 3))) <= 1e-5


# (B, Cin, H, Cout, prologue, residual): 128- and 64-row tiles, a pixel tail
# (N % 256 != 0) and 256-pixel tiles spanning several images (P < 256)
SOL_CASES = [
    (2, 256, 64, 128, True, False),
    (2, 128, 64, 256, True, True),
    (3, 64, 32, 64, True, True),
    (5, 256, 8, 256, False, True),
    (3, 128, 6, 128, True, False),
    (16, 128, 64, 256, True, True),       # 256-row 8-wave tiles (one pixel tile per CU)
    (32, 256, 64, 128, True, True),       # the headline 64x64 level: 512-pixel 8-wave tiles, 3-stage ring
    (37, 256, 60, 128, True, False),      # the same with a pixel tail (N % 512 = 80)
]


@pytest.mark.parametrize("npieces", [2, 3])
@pytest.mark.parametrize("case", SOL_CASES)
def test_conv1x1_split_load_vs_f64(case, npieces):
    """conv1x1_sol_kernel: forward (prologue, residual, BN partials on 6xbf16) and
    the data gradient through the mode-1 table, within 2x (2xfp16: F16_BAR) the f32
    path's error."""
    from ubpl_amd import kernels as Kn
    B, Cin, H, Cout, pro, resid = case
    npc = npieces
    gen = torch.Generator().manual_seed(5 + hash(case) % 1000)
    x32 = torch.randn(B, Cin, H, H, generator=gen)
    w32 = torch.randn(Cout, Cin, 1, 1, generator=gen) / np.sqrt(Cin)
    b32 = torch.randn(Cout, generator=gen)
    sc32 = torch.rand(Cin, generator=gen) + 0.5
    sh32 = torch.randn(Cin, generator=gen) * 0.5
    res32 = torch.randn(B, Cout, H, H, generator=gen) if resid else None
    inp = F.relu(x32.double() * sc32.double()[None, :, None, None] + sh32.double()[None, :, None, None]) if pro \
        else x32.double()
    yref = F.conv2d(inp, w32.double(), b32.double())
    if resid:
        yref = yref + res32.double()
    d = lambda t: None if t is None else t.to(DEV)
    ps, ph = (d(sc32), d(sh32)) if pro else (None, None)
    y_f32 = Kn.conv2d_forward(d(x32), d(w32), d(b32), 1, ps, ph, res=d(res32))
    part = Kn.bn_partial_buffer(Cout, B * H * H, DEV) if npc == 3 else None
    y = Kn.conv1x1_forward_split_load(d(x32), Kn.conv_weight_split(d(w32), 0, npc), d(b32), ps, ph, res=d(res32),
                                      stat_part=part)
    e32, esp = _rel(y_f32, yref), _rel(y, yref)
    print("sol fwd %s np=%d: f32 %.2e split-load %.2e" % (case, npc, e32, esp))
    assert _ok(esp, e32, npc), (esp, e32)
    # without the partials epilogue: the same K order and chunking, so the same
    # bits — except with a residual, which that kernel adds in its transposed
    # epilogue instead of seeding the accumulators with it (UBPL_SOL_TEPI)
    y2 = Kn.conv1x1_forward_split_load(d(x32), Kn.conv_weight_split(d(w32), 0, npc), d(b32), ps, ph,
                                       res=d(res32))
    if resid:
        assert _ok(_rel(y2, yref), e32, npc), (_rel(y2, yref), e32)
    else:
        assert torch.equal(y2, y)
    if resid:   # residual aliasing the output
        o = d(res32).clone()
        Kn.conv1x1_forward_split_load(d(x32), Kn.conv_weight_split(d(w32), 0, npc), d(b32), ps, ph, res=o, out=o)
        assert torch.equal(o, y2)
    if npc == 2:
        return      # (the data gradient runs on 6xbf16 under the 2xfp16 precision)
    # BN statistics from the epilogue partials
    gamma, beta = torch.ones(Cout, device=DEV), torch.zeros(Cout, device=DEV)
    rm, rv = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
    mu, istd, s_, h_ = (torch.empty(Cout, device=DEV) for _ in range(4))
    Kn.bn_stats_from_partials(part, Cout, B * H * H, gamma, beta, 1e-5, 0.1, rm, rv, mu, istd, s_, h_)
    yd = y.double().cpu()
    torch.testing.assert_close(mu.double().cpu(), yd.mean((0, 2, 3)), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(istd.double().cpu(), 1.0 / torch.sqrt(yd.var((0, 2, 3), unbiased=False) + 1e-5),
                               rtol=1e-5, atol=0)
    # data gradient (x = dy, mode-1 weights [Cin][Cout]); Cin plays the output role
    if Cin % 64 == 0:
        dy = torch.randn(B, Cout, H, H, generator=gen)
        dxref = torch.nn.grad.conv2d_input((B, Cin, H, H), w32.double(), dy.double())
        dx = Kn.conv1x1_forward_split_load(d(dy), Kn.conv_weight_split(d(w32), 1, 3), None)
        dx32 = Kn.conv2d_dgrad(d(dy), d(w32))
        e32, esp = _rel(dx32, dxref), _rel(dx, dxref)
        print("sol dgrad %s: f32 %.2e split-load %.2e" % (case, e32, esp))
        assert esp <= 2 * e32 + 1e-8, (esp, e32)


@pytest.mark.parametrize("npieces", [2, 3])
@pytest.mark.parametrize("case", [(4, 256, 32, 16, False), (8, 256, 16, 16, True), (2, 16, 32, 256, False)])
def test_conv1x1_split_load_16_channels(case, npieces):
    """The heatmap projection (256 -> K = 16) and its data gradient (K = 16 output
    channels of the merge_preds dgrad) on conv1x1_sol_kernel: one 64-row tile,
    rows past Cout clamped on load and never stored; within 2x the f32 path's error."""
    from ubpl_amd import kernels as Kn
    B, Cin, H, Cout, pro = case
    gen = torch.Generator().manual_seed(41 + hash(case) % 1000)
    x32 = torch.randn(B, Cin, H, H, generator=gen)
    w32 = torch.randn(Cout, Cin, 1, 1, generator=gen) / np.sqrt(Cin)
    b32 = torch.randn(Cout, generator=gen)
    sc32, sh32 = torch.rand(Cin, generator=gen) + 0.5, torch.randn(Cin, generator=gen) * 0.5
    inp = F.relu(x32.double() * sc32.double()[None, :, None, None] + sh32.double()[None, :, None, None]) if pro \
        else x32.double()
    yref = F.conv2d(inp, w32.double(), b32.double())
    d = lambda t: t.to(DEV)
    ps, ph = (d(sc32), d(sh32)) if pro else (None, None)
    assert Kn.conv1x1_split_load_ok(d(x32), Kn.conv_weight_split(d(w32), 0, npieces)) or B * H * H < 256 * 256
    y_f32 = Kn.conv2d_forward(d(x32), d(w32), d(b32), 1, ps, ph)
    y = Kn.conv1x1_forward_split_load(d(x32), Kn.conv_weight_split(d(w32), 0, npieces), d(b32), ps, ph)
    e32, esp = _rel(y_f32, yref), _rel(y, yref)
    print("sol16 fwd %s np=%d: f32 %.2e split-load %.2e" % (case, npieces, e32, esp))
    assert _ok(esp, e32, npieces), (esp, e32)
    if npieces == 2:
        return
    dy = torch.randn(B, Cout, H, H, generator=gen)
    dxref = torch.nn.grad.conv2d_input((B, Cin, H, H), w32.double(), dy.double())
    dx = Kn.conv1x1_forward_split_load(d(dy), Kn.conv_weight_split(d(w32), 1, 3), None)
    dx32 = Kn.conv2d_dgrad(d(dy), d(w32))
    e32, esp = _rel(dx32, dxref), _rel(dx, dxref)
    print("sol16 dgrad %s: f32 %.2e split-load %.2e" % (case, e32, esp))
    assert esp <= 2 * e32 + 1e-8, (esp, e32)


@pytest.mark.parametrize("case", [(2, 256, 128, 64, True), (2, 128, 256, 32, True), (3, 256, 256, 16, False),
                                  (4, 128, 128, 4, True), (2, 64, 64, 32, True), (2, 64, 128, 32, False),
                                  (3, 128, 64, 16, True), (2, 64, 64, 128, True)])
def test_wgrad1x1_split_load_vs_f64(case):
    """1x1 weight + bias gradient with both operands split on load, within 2x
    the exact-f32 kernel's error against float64 or 8 f32 unit roundoffs
    (2^-21), whichever is larger; accumulate adds.  The floor: the split path's
    relative error on random data is ~6 u whatever K (each 16-pixel chunk's
    MFMA sum is rounded once at the chunk's magnitude, the chunks' errors add
    at random sign), while the exact-f32 kernel's short split-K fmaf chains
    reach ~2.5 u at K = 32k pixels (the 64-channel convs at 128x128: K = B*16384)."""
    from ubpl_amd import kernels as Kn
    B, Cin, Cout, H, pro = case
    gen = torch.Generator().manual_seed(17 + hash(case) % 1000)
    x = torch.randn(B, Cin, H, H, generator=gen)
    dy = torch.randn(B, Cout, H, H, generator=gen)
    sc, sh = torch.rand(Cin, generator=gen) + 0.5, torch.randn(Cin, generator=gen) * 0.5
    inp = F.relu((x.double() * sc.double()[None, :, None, None] + sh.double()[None, :, None, None]).float()) \
        if pro else x
    dwref = torch.nn.grad.conv2d_weight(inp.double(), (Cout, Cin, 1, 1), dy.double())
    dbref = dy.double().sum((0, 2, 3))
    d = lambda t: t.to(DEV)
    ps, ph = (d(sc), d(sh)) if pro else (None, None)
    assert Kn.wgrad1x1_split_load_ok(d(dy), d(x))
    dw = torch.full((Cout, Cin, 1, 1), 0.25, device=DEV)
    db = torch.full((Cout,), -0.5, device=DEV)
    Kn.conv2d_wgrad1x1_split_load(d(dy), d(x), dw, db, ps, ph, accumulate=True)
    dw32, db32 = torch.zeros(Cout, Cin, 1, 1, device=DEV), torch.zeros(Cout, device=DEV)
    Kn.conv2d_wgrad(d(dy), d(x), 1, 1, dw32, db32, ps, ph, accumulate=False)
    e32, esp = _rel(dw32, dwref), _rel(dw - 0.25, dwref)
    print("wgrad1 %s: f32 %.2e split-load %.2e" % (case, e32, esp))
    assert esp <= max(2 * e32 + 1e-8, 2.0 ** -21), (esp, e32)
    assert _rel(db + 0.5, dbref) <= 1e-5


@pytest.mark.parametrize("kind", ["sol", "psa", "psa_splitk"])
def test_bn_backward_partials_from_dgrad_epilogue(kind):
    """Backward BatchNorm statistics partials written by the data-gradient
    epilogue (conv1x1_sol_kernel / conv_psa_kernel, or the split-K fallback
    pass) give the same dx, dgamma, dbeta as the statistics pass over dz."""
    from ubpl_amd import kernels as Kn
    gen = torch.Generator().manual_seed(23)
    B, Ci, Co, H = {"sol": (2, 128, 256, 32), "psa": (2, 128, 128, 32), "psa_splitk": (4, 128, 128, 8)}[kind]
    d = lambda t: t.to(DEV)
    dy = d(torch.randn(B, Ci, H, H, generator=gen))
    xbn = d(torch.randn(B, Co, H, H, generator=gen))
    w = d(torch.randn(Ci, Co, 1 if kind == "sol" else 3, 1 if kind == "sol" else 3, generator=gen) * 0.05)
    gamma = d(torch.rand(Co, generator=gen) + 0.5)
    mean, istd = d(torch.randn(Co, generator=gen) * 0.1), d(torch.rand(Co, generator=gen) + 0.5)
    coef = torch.cat([gamma * istd, d(torch.randn(Co, generator=gen)), mean])   # scale | shift | mean
    sc, sh = coef[:Co], coef[Co:2 * Co]
    part = Kn.bn_partial_buffer(Co, B * H * H, DEV)
    if kind == "sol":
        dz = Kn.conv1x1_forward_split_load(dy, Kn.conv_weight_split(w, 1, 3), None, bwd=(xbn, coef, 1, part))
    else:
        ys = Kn.split_activation(dy, 3, 1)
        dz = Kn.conv2d_forward_psa(ys, Kn.conv_weight_split(w, 1, 3), None, bwd=(xbn, coef, 1, part))
    scratch = torch.zeros(int(__import__("ubpl_amd")._lib.lib().ubpl_bn_part_doubles(B, Co)), dtype=torch.float64,
                          device=DEV)
    res = []
    for p in (part, None):
        c3 = torch.empty(3 * Co, device=DEV)
        dg, db = torch.zeros(Co, device=DEV), torch.zeros(Co, device=DEV)
        dx = Kn.bn_backward(dz, xbn, gamma, mean, istd, sc, sh, 1, scratch, c3, dg, db, out=torch.empty_like(dz),
                            part=p)
        res.append((dx, dg, db))
    for a, b in zip(*res):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("B,H", [(2, 64), (3, 32), (1, 256)])
def test_stem_s2d_vs_f64(B, H):
    """The 7x7 stride-2 stem as a 4x4 stride-1 conv over the space-to-depth
    image on the split path, within 2x the exact-f32 kernel's error."""
    from ubpl_amd import kernels as Kn
    gen = torch.Generator().manual_seed(31 + B + H)
    x = torch.rand(B, 3, H, H, generator=gen) - 0.5
    w = torch.randn(64, 3, 7, 7, generator=gen) / np.sqrt(147)
    b = torch.randn(64, generator=gen)
    yref = F.conv2d(x.double(), w.double(), b.double(), 2, 3)
    d = lambda t: t.to(DEV)
    assert Kn.stem_s2d_ok(d(x))
    y = Kn.conv2d_forward_psa(Kn.stem_s2d_split(d(x), 2), Kn.stem_weight_s2d_split(d(w)), d(b))
    y32 = Kn.conv2d_forward(d(x), d(w), d(b), 2)
    e32, esp = _rel(y32, yref), _rel(y, yref)
    print("stem s2d B=%d H=%d: f32 %.2e split %.2e" % (B, H, e32, esp))
    # K = 147 keeps the exact-f32 chain below one f32 ulp (~4e-8 relative); the
    # split path rounds once per 16-term chunk (16 chunks): a few ulps is its level
    assert esp <= max(2 * e32, 4 * 2.0 ** -24), (esp, e32)


@pytest.mark.parametrize("B,H", [(2, 256), (4, 128), (32, 256)])
def test_stem_weight_gradient_s2d_vs_f64(B, H):
    """The stem's 7x7 stride-2 weight (+ bias) gradient as the weight gradient
    of its space-to-depth 4x4 form on the split path (wgrad_stem_psa_kernel,
    then the 4x4 -> 7x7 map), from PSA operands: split(dy) with a 1-pixel border
    and the forward's phase image; within 2x the exact-f32 kernel's error vs
    float64 (B=32, 256x256: the headline step's shape)."""
    from ubpl_amd import kernels as Kn
    gen = torch.Generator().manual_seed(37 + B + H)
    x = torch.rand(B, 3, H, H, generator=gen) - 0.5
    w = torch.randn(64, 3, 7, 7, generator=gen) / np.sqrt(147)
    dy = torch.randn(B, 64, H // 2, H // 2, generator=gen)
    d = lambda t: t.to(DEV)
    sl = slice(0, min(B, 4))                        # the f64 reference over (up to) 4 images
    xr, dyr = x[sl].double(), dy[sl].double()
    wref = torch.nn.grad.conv2d_weight(xr, w.shape, dyr, stride=2, padding=3)
    bref = dyr.sum((0, 2, 3))
    xs, ys = Kn.stem_s2d_split(d(x[sl].contiguous()), 2), Kn.split_activation(d(dy[sl].contiguous()), 3, 1)
    assert Kn.wgrad_stem_psa_ok(ys, xs, d(w))
    dw, db = torch.full_like(d(w), 7.0), torch.full((64,), 7.0, device=DEV)
    Kn.conv2d_wgrad_stem_psa(ys, xs, dw, db, accumulate=False)
    dw32, db32 = torch.zeros_like(d(w)), torch.zeros(64, device=DEV)
    Kn.conv2d_wgrad(d(dy[sl].contiguous()), d(x[sl].contiguous()), 7, 2, dw32, db32, accumulate=False)
    e32, esp = _rel(dw32, wref), _rel(dw, wref)
    eb32, ebsp = _rel(db32, bref), _rel(db, bref)
    print("stem wgrad B=%d H=%d: f32 %.2e split %.2e | bias f32 %.2e split %.2e" % (B, H, e32, esp, eb32, ebsp))
    assert esp <= max(2 * e32, 4 * 2.0 ** -24), (esp, e32)
    assert ebsp <= max(2 * eb32, 4 * 2.0 ** -24), (ebsp, eb32)
    # accumulate=True adds onto what is there
    Kn.conv2d_wgrad_stem_psa(ys, xs, dw, db, accumulate=True)
    assert _rel(dw, 2 * wref) <= max(2 * e32, 4 * 2.0 ** -24) + 1e-7
    if B > 4:                                        # the full batch runs (the headline launch shape)
        xs, ys = Kn.stem_s2d_split(d(x), 2), Kn.split_activation(d(dy), 3, 1)
        Kn.conv2d_wgrad_stem_psa(ys, xs, dw, db, accumulate=False)
        Kn.conv2d_wgrad(d(dy), d(x), 7, 2, dw32, db32, accumulate=False)
        assert _rel(dw, dw32.cpu().double()) < 1e-5


@pytest.mark.parametrize("B,H", [(2, 256), (8, 128)])
def test_bf16_stem_s2d_forward_and_weight_gradient_vs_rounded_f64(B, H):
    """The "bf16" precision's stem (round 5): the 7x7 stride-2 conv as the
    space-to-depth 4x4 conv with ONE bf16 piece per operand, and its weight
    gradient from the one-piece PSA operands — against float64 of the
    bf16-rounded operands, to f32 summation error (the bar of the other
    one-piece kernels)."""
    from ubpl_amd import kernels as Kn
    gen = torch.Generator().manual_seed(53 + B + H)
    x = torch.rand(B, 3, H, H, generator=gen) - 0.5
    w = torch.randn(64, 3, 7, 7, generator=gen) / np.sqrt(147)
    b = torch.randn(64, generator=gen)
    dy = torch.randn(B, 64, H // 2, H // 2, generator=gen)
    bf = lambda t: t.to(torch.bfloat16).double()
    d = lambda t: t.to(DEV)
    yref = F.conv2d(bf(x), bf(w), b.double(), 2, 3)
    xs = Kn.stem_s2d_split(d(x), 2, 1)
    y = Kn.conv2d_forward_psa(xs, Kn.stem_weight_s2d_split(d(w), 1), d(b))
    e = _rel(y, yref)
    print("bf16 stem fwd B=%d H=%d: %.2e" % (B, H, e))
    assert e <= 2e-6, e
    wref = torch.nn.grad.conv2d_weight(bf(x), w.shape, bf(dy), stride=2, padding=3)
    ys = Kn.split_activation(d(dy), 1, 1)
    assert Kn.wgrad_stem_psa_ok(ys, xs, d(w))
    dw, db = torch.zeros_like(d(w)), torch.zeros(64, device=DEV)
    Kn.conv2d_wgrad_stem_psa(ys, xs, dw, db, accumulate=False)
    e, eb = _rel(dw, wref), _rel(db, bf(dy).sum((0, 2, 3)))
    print("bf16 stem wgrad B=%d H=%d: %.2e bias %.2e" % (B, H, e, eb))
    assert e <= 2e-6 and eb <= 2e-6, (e, eb)


# the halo kernel's shapes (conv_psah_kernel: 3x3 pad 1, 128- / 64-row tiles, whole
# rows of W = 32 / 64 / 128 per 256-pixel tile): (B, Cin, H, Cout)
HALO_CASES = [(32, 128, 64, 128), (8, 128, 128, 128), (32, 256, 32, 256), (16, 256, 64, 256),
              (32, 64, 128, 64), (32, 128, 32, 128)]


@pytest.mark.parametrize("npieces", [2, 3])
@pytest.mark.parametrize("teams", ["1", "2"])
@pytest.mark.parametrize("case", HALO_CASES)
def test_psa_halo_kernel_matches_per_tap_kernel_bit_for_bit(case, teams, npieces, _lib_dispatch):
    """conv_psah_kernel (input halo staged once per channel group) computes the
    same products in the same order as conv_psa_kernel (B staged per tap):
    forward with bias + residual and the data gradient agree bit for bit, and
    the first / last images are within the split path's bar of float64."""
    from ubpl_amd import kernels as Kn
    lib = _lib_dispatch
    lib.ubpl_set_psa_dispatch(-1, int(teams))   # one or two 4-wave teams per workgroup (W <= 64)
    B, Cin, H, Cout = case
    gen = torch.Generator().manual_seed(41 + Cin + H)
    x32 = torch.randn(B, Cin, H, H, generator=gen)
    w32 = torch.randn(Cout, Cin, 3, 3, generator=gen) / np.sqrt(Cin * 9)
    b32 = torch.randn(Cout, generator=gen)
    res32 = torch.randn(B, Cout, H, H, generator=gen)
    xs = Kn.split_activation(x32.to(DEV), npieces, 1)
    ws = Kn.conv_weight_split(w32.to(DEV), 0, npieces)
    wd = Kn.conv_weight_split(w32.to(DEV), 1, npieces)
    dys = (Kn.split_activation(torch.randn(B, Cout, H, H, generator=gen).to(DEV), npieces, 1) if Cin == Cout
           else None)
    outs = {}
    # 2: the double-buffered halo kernel required, 3: the one-buffer two-workgroup
    # variant required (an error if the plan cannot take the launch)
    for flag in ("0", "2", "3"):
        lib.ubpl_set_psa_dispatch(int(flag), int(teams))
        y = Kn.conv2d_forward_psa(xs, ws, b32.to(DEV), res=res32.to(DEV))
        dx = Kn.conv2d_forward_psa(dys, wd, None) if dys is not None else None
        torch.cuda.synchronize()
        outs[flag] = (y, dx)
    for flag in ("2", "3"):
        assert torch.equal(outs["0"][0], outs[flag][0]), flag
        if dys is not None:
            assert torch.equal(outs["0"][1], outs[flag][1]), flag
    sl = [0, B - 1]
    yref = F.conv2d(x32[sl].double(), w32.double(), b32.double(), 1, 1) + res32[sl].double()
    y_f32 = Kn.conv2d_forward(x32[sl].to(DEV), w32.to(DEV), b32.to(DEV), 1, res=res32[sl].to(DEV))
    e32, esp = _rel(y_f32, yref), _rel(outs["2"][0][sl], yref)
    print("halo %s np=%d: f32 %.2e split %.2e" % (case, npieces, e32, esp))
    assert _ok(esp, e32, npieces), (esp, e32)


@pytest.mark.parametrize("pro", [False, True])
def test_split_activation_2xfp16_with_6xbf16_image(pro):
    """ubpl_split_activation with npieces 2 and the second output: the fp16 planes
    equal the 2-piece split's and the bf16 planes the 3-piece split's, bit for bit;
    the fp16 pieces carry v * 32 to 2^-22 of v as the kernel computed it (the three
    bf16 pieces sum to it exactly)."""
    from ubpl_amd import kernels as Kn
    gen = torch.Generator().manual_seed(91)
    B, C, H = 3, 64, 16
    x = torch.randn(B, C, H, H, generator=gen).to(DEV)
    ps, ph = ((torch.rand(C, generator=gen) + 0.5).to(DEV), torch.randn(C, generator=gen).to(DEV)) if pro \
        else (None, None)
    xs2, xs3 = Kn.split_activation(x, 2, 1, ps, ph, with3=True)
    assert torch.equal(xs2.buf, Kn.split_activation(x, 2, 1, ps, ph).buf)
    assert torch.equal(xs3.buf, Kn.split_activation(x, 3, 1, ps, ph).buf)
    planes = xs2.buf.view(2, xs2.plane).cpu()
    img = (planes[0].view(torch.float16).double() + planes[1].view(torch.float16).double()) / 32.0
    img = img.view(B, C // 16, H + 2, H + 2, 16)[:, :, 1:-1, 1:-1].permute(0, 1, 4, 2, 3).reshape(B, C, H, H)
    p3 = xs3.buf.view(3, xs3.plane).cpu()
    ref = sum((p3[p].to(torch.int32) << 16).view(torch.float32).double() for p in range(3))
    ref = ref.view(B, C // 16, H + 2, H + 2, 16)[:, :, 1:-1, 1:-1].permute(0, 1, 4, 2, 3).reshape(B, C, H, H)
    if not pro:
        assert torch.equal(ref, x.double().cpu())
    assert float(((img - ref).abs() - 2.0 ** -22 * ref.abs()).max()) <= 2.0 ** -30


@pytest.mark.parametrize("teams", ["1", "2"])
@pytest.mark.parametrize("case", HALO_CASES[:2] + HALO_CASES[4:] + [(16, 128, 96, 128)])
def test_bf16_psa_halo_kernel_matches_per_tap_kernel_bit_for_bit(case, teams, _lib_dispatch):
    """The one-piece (bf16) halo kernel (one stage and barrier per channel
    group) against conv_psa_kernel's one-piece path: bit for bit."""
    from ubpl_amd import kernels as Kn
    lib = _lib_dispatch
    lib.ubpl_set_psa_dispatch(-1, int(teams))
    B, Cin, H, Cout = case
    gen = torch.Generator().manual_seed(43 + Cin + H)
    x32 = torch.randn(B, Cin, H, H, generator=gen)
    w32 = torch.randn(Cout, Cin, 3, 3, generator=gen) / np.sqrt(Cin * 9)
    b32 = torch.randn(Cout, generator=gen)
    xs = Kn.split_activation(x32.to(DEV), 1, 1)
    ws = Kn.conv_weight_split(w32.to(DEV), 0, 1)
    outs = {}
    for flag in ("0", "2"):
        lib.ubpl_set_psa_dispatch(int(flag), int(teams))
        outs[flag] = Kn.conv2d_forward_psa(xs, ws, b32.to(DEV))
        torch.cuda.synchronize()
    assert torch.equal(outs["0"], outs["2"])


@pytest.mark.parametrize("case", [(16, 128, 96, 128), (8, 256, 96, 256)])
def test_psa_halo_kernel_96_wide_planes_bit_for_bit(case, _lib_dispatch):
    """The 96-wide planes (HG8 at 384x384) on the halo kernel's 192-pixel tiles
    (one halo buffer, UBPL_PSA_HALO=3 required) against conv_psa_kernel: forward
    with bias + residual and the data gradient, bit for bit."""
    from ubpl_amd import kernels as Kn
    lib = _lib_dispatch
    B, Cin, H, Cout = case
    gen = torch.Generator().manual_seed(47 + Cin)
    x32 = torch.randn(B, Cin, H, H, generator=gen)
    w32 = torch.randn(Cout, Cin, 3, 3, generator=gen) / np.sqrt(Cin * 9)
    b32 = torch.randn(Cout, generator=gen)
    res32 = torch.randn(B, Cout, H, H, generator=gen)
    xs = Kn.split_activation(x32.to(DEV), 3, 1)
    ws = Kn.conv_weight_split(w32.to(DEV), 0, 3)
    wd = Kn.conv_weight_split(w32.to(DEV), 1, 3)
    dys = Kn.split_activation(torch.randn(B, Cout, H, H, generator=gen).to(DEV), 3, 1)
    outs = {}
    for flag in ("0", "3"):
        lib.ubpl_set_psa_dispatch(int(flag), -1)
        outs[flag] = (Kn.conv2d_forward_psa(xs, ws, b32.to(DEV), res=res32.to(DEV)), Kn.conv2d_forward_psa(dys, wd, None))
        torch.cuda.synchronize()
    assert torch.equal(outs["0"][0], outs["3"][0])
    assert torch.equal(outs["0"][1], outs["3"][1])
