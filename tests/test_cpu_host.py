"""CPU-only checks of the product's host side: the C-ABI library loads and
exports every symbol include/ubpl_hip.h declares (no compute calls), the
host logic (sampler, ramps, EMA alpha, affine inverse) matches the golden
vectors, and compute entry points fail loudly without a GPU."""
import json
import os
import re

import numpy as np
import pytest
import torch

import seeds

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GD = os.path.join(ROOT, "tests", "golden")


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "ubpl_hip.h")).read()
    return sorted(set(re.findall(r"\b(?:int|int64_t)\s+(ubpl_\w+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from ubpl_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libubpl_hip.so not built (run __graft_entry__.build())")
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)


def test_torch_ops_mirror_the_header():
    """libubpl_ops.so registers TORCH_LIBRARY(ubpl): one op per C-ABI entry,
    device pointers as Tensor? (mutable when the C pointer is), no stream
    argument (the op uses torch's current stream); host queries run on CPU."""
    from ubpl_amd import _lib
    if not os.path.exists(_lib.OPS_PATH):
        pytest.skip("libubpl_ops.so not built (run __graft_entry__.build())")
    ops = _lib.load_ops()
    txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "ubpl_hip.h")).read(), flags=re.S)
    for ret, name, args in re.findall(r"(int|int64_t)\s+(ubpl_\w+)\s*\(([^;]*?)\)\s*;", txt, flags=re.S):
        sch = _lib.op(name)._schema
        params = [a.strip() for a in args.replace("\n", " ").split(",") if a.strip()]
        c_args = [p for p in params if not p.endswith("stream")]
        assert len(sch.arguments) == len(c_args), name
        for a, p in zip(sch.arguments, c_args):
            if "*" in p:
                assert str(a.type) == "Optional[Tensor]", (name, p)
                assert (a.alias_info is not None and a.alias_info.is_write) == (not p.startswith("const")), (name, p)
            assert a.name == p.split()[-1].lstrip("*"), (name, a.name, p)
    # a host-only query through its op equals the C-ABI value
    assert ops.conv2d_forward_psa_workspace(32, 128, 128, 3, 16, 16, 3) == \
        _lib.lib().ubpl_conv2d_forward_psa_workspace(32, 128, 128, 3, 16, 16, 3)


def test_torch_ops_check_arguments_before_the_call():
    """Every device-pointer argument is checked against its header annotation
    (element type, contiguity, storage extent implied by the integer
    arguments) before the C-ABI call: a short tensor raises instead of being
    written out of bounds.  The ops are registered for
    CPU as well, so this runs without a GPU; a CPU tensor that passes every
    check is then refused as not a device tensor (no compute on the host)."""
    from ubpl_amd import _lib
    if not os.path.exists(_lib.OPS_PATH):
        pytest.skip("libubpl_ops.so not built (run __graft_entry__.build())")
    ops = _lib.load_ops()
    n = 1024
    a, b, out = torch.zeros(n), torch.zeros(n), torch.zeros(n)
    with pytest.raises(RuntimeError, match="out holds 1023 elements"):
        ops.add(a, b, n, out[1:])                           # one element short (offset view)
    with pytest.raises(RuntimeError, match="a holds 1000 elements"):
        ops.add(a[:1000], b, n, out)
    with pytest.raises(RuntimeError, match="must be f32"):
        ops.add(a.double(), b, n, out)
    with pytest.raises(RuntimeError, match="must be contiguous"):
        ops.add(torch.zeros(64, 32).t(), b, n, out)
    with pytest.raises(RuntimeError, match="expected a device tensor"):
        ops.add(a, b, n, out)                               # every check passes: refused on CPU
    # extents from expressions of several arguments: a BN apply over [B,C,HW]
    x, y, sc = torch.zeros(2 * 8 * 16), torch.zeros(2 * 8 * 16), torch.zeros(8)
    with pytest.raises(RuntimeError, match="y holds 255 elements"):
        ops.bn_apply(x, 2, 8, 16, sc, sc, 1, y[:255])
    with pytest.raises(RuntimeError, match="shift holds 7 elements"):
        ops.bn_apply(x, 2, 8, 16, sc, sc[:7], 1, y)
    # split (bf16-piece) planes: npieces planes `plane` elements apart
    B, C, H, W, pad, npieces = 1, 16, 4, 4, 1, 3
    plane = B * C * (H + 2) * (W + 2)
    dst = torch.zeros(npieces * plane, dtype=torch.int16)
    with pytest.raises(RuntimeError, match="dst holds"):
        ops.split_activation(torch.zeros(B * C * H * W), B, C, H, W, None, None, pad, npieces, dst[:-1], plane, None, 0)
    with pytest.raises(RuntimeError, match="expected a device tensor"):
        ops.split_activation(torch.zeros(B * C * H * W), B, C, H, W, None, None, pad, npieces, dst, plane, None, 0)
    # an integer output of the wrong type
    with pytest.raises(RuntimeError, match="out_cnt must be i32"):
        ops.loss_finalize(0, torch.zeros(8), None, None, None, None, 0, 0, 2, 1, 4, 0.5, torch.zeros(1),
                          torch.zeros(4, dtype=torch.int64), None, torch.zeros(8))


def test_product_fails_loudly_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ubpl_amd import hourglass, losses
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        hourglass.StackedHourglass(16, 2, "AvgPool")
    with pytest.raises(RuntimeError):
        losses.JointMSELoss(nStack=2)(torch.zeros(1, 2, 3, 4, 4), torch.zeros(1, 3, 4, 4))


def test_sampler_matches_reference_batches():
    from ubpl_amd.sampler import TwoStreamBatchSampler
    m = json.load(open(os.path.join(GD, "misc.json")))
    for name, (prim, sec, bs, sbs, seed) in seeds.sampler_cases().items():
        np.random.seed(seed)
        s = TwoStreamBatchSampler(prim, sec, bs, sbs)
        assert len(s) == m["sampler"][name]["len"]
        assert [[int(i) for i in b] for b in s] == m["sampler"][name]["batches"]


def test_sampler_shards_are_disjoint():
    from ubpl_amd.sampler import TwoStreamBatchSampler
    s = TwoStreamBatchSampler(list(range(100, 500)), list(range(100)), 32, 16)
    a, b = s.shard(0, 2), s.shard(1, 2)
    assert not set(a.primary_indices) & set(b.primary_indices)
    assert not set(a.secondary_indices) & set(b.secondary_indices)
    assert len(a) == len(b) == 200 // 16


def test_ramps_and_alpha():
    from ubpl_amd import parameters as PR
    from types import SimpleNamespace
    m = json.load(open(os.path.join(GD, "misc.json")))["ramps"]
    a = SimpleNamespace(consWeight_max=10.0, consWeight_min=0.0, consWeight_rampup=5,
                        pseudoWeight_max=1.0, pseudoWeight_min=1.0, pseudoWeight_rampup=100,
                        FDLWeight_max=1.0, FDLWeight_min=0.2, FDLWeight_rampup=30)
    for e in range(40):
        assert PR.consWeight_increase(e, a) == m["cons/%d" % e]
        assert PR.pseudoWeight_increase(e, a) == m["pseudo/%d" % e]
        assert PR.FDLWeight_decrease(e, a) == m["fdl_dec/%d" % e]
        assert PR.FDLWeight_increase(e, a) == m["fdl_inc/%d" % e]
    assert PR.ema_alpha(0, 0.999) == 0.0 and PR.ema_alpha(1, 0.999) == 0.5
    assert PR.ema_alpha(5000, 0.999) == 0.999


def test_inverse_transform_matches_oracle():
    from ubpl_amd.process import inverse_transforms
    from oracle import decode as OD
    for name, cfg in seeds.decode_cases().items():
        _, center, scale = seeds.decode_inputs(**cfg)
        t = inverse_transforms(center, scale, [cfg["R"]] * 2).numpy()
        for i in range(center.shape[0]):
            ref = OD.inverse_transform(center[i], scale[i], [cfg["R"]] * 2)[:2].reshape(-1)
            assert np.array_equal(t[i], ref)


def test_param_table_matches_reference_names():
    from ubpl_amd.hourglass import build_table
    meta = json.load(open(os.path.join(GD, "hourglass_meta.json")))
    for case, cfg in seeds.hg_cases().items():
        tab = build_table(cfg["K"], cfg["S"])
        assert [e[0] for e in tab] == meta[case]["param_names"]
        assert [list(e[1]) for e in tab] == meta[case]["param_shapes"]
    tab = build_table(16, 2)
    live = sum(int(np.prod(e[1])) for e in tab if e[3])
    dead = sum(int(np.prod(e[1])) for e in tab if not e[3])
    assert (live, dead) == (6570400, 1858688)      # grad-carrying vs unused skip params


def test_tools_weights_cpu():
    from types import SimpleNamespace
    from ubpl_amd.tools import ProjectTools
    g = np.load(os.path.join(GD, "losses.npz"))
    for case, cfg in seeds.loss_cases().items():
        isl = seeds.loss_inputs(**cfg)["islabeled"]
        a = SimpleNamespace(device="cpu", pseudoWeight=cfg["pw"])
        assert np.array_equal(ProjectTools.getSampleWeight([isl], a)[0].numpy(), g[case + "/w"])
        assert np.array_equal(ProjectTools.getSampleWeight_nega([isl], a)[0].numpy(), g[case + "/w_nega"])
        assert np.array_equal(ProjectTools.getSampleWeight_mt_cons(isl, a).numpy(), g[case + "/w_mt_cons"])


def test_checkpoint_schema_and_selection_cpu(tmp_path):
    """ubpl_amd.checkpoint on plain torch modules / AdamW (host logic only):
    projects/MT_UBPL.py:88-103 selection rule and key schema, comm.py file names."""
    import types
    import torch
    from ubpl_amd import checkpoint as CK
    args = types.SimpleNamespace(best_acc=[0.3, 0.3, 0.3], best_epoch=[1, 1, 1])
    assert CK.select_best([[0.2, 0.3], [0.9, 0.31], [0.5, 0.1]], args, 7) == [False, True, False]
    assert args.best_acc == [0.3, 0.31, 0.3] and args.best_epoch == [1, 7, 1]
    torch.manual_seed(0)
    ms = [torch.nn.Linear(3, 2) for _ in range(2)]
    es = [torch.nn.Linear(3, 2) for _ in range(2)]
    os_ = [torch.optim.AdamW(m.parameters(), lr=1e-3) for m in ms]
    for m, o in zip(ms, os_):
        m(torch.ones(1, 3)).sum().backward()
        o.step()
    ck = CK.checkpoint_state(ms, es, os_, args, 7)
    assert list(ck) == ["current_epoch", "best_acc", "best_epoch", "model1_state", "model1_ema_state",
                        "optim1_state", "model2_state", "model2_ema_state", "optim2_state"]
    path = CK.save_checkpoint(ck, False, str(tmp_path / "ckpts"))
    assert path.endswith("ckpts/checkpoint.pth.tar") and not (tmp_path / "ckpts" / "checkpoint_best.pth.tar").exists()
    ms2 = [torch.nn.Linear(3, 2) for _ in range(2)]
    es2 = [torch.nn.Linear(3, 2) for _ in range(2)]
    os2 = [torch.optim.AdamW(m.parameters(), lr=1e-3) for m in ms2]
    assert CK.load_checkpoint(path, ms2, es2, os2) == (7, [0.3, 0.31, 0.3], [1, 7, 1])
    assert torch.equal(ms2[1].weight, ms[1].weight) and torch.equal(es2[0].bias, es[0].bias)
    assert float(os2[0].state_dict()["state"][0]["step"]) == 1.0


def test_augment_geometry_matches_reference_transform():
    """f1: the keypoint map of the device augmentation is the reference's
    transform() (utils/udaap/transforms.py:119-158) on the loader's float32
    tensors (scale, angle, keypoints: utils/augment.py:18-20,150-156); the
    fixtures come from the reference run on exactly those types and include
    points planted where float64 arithmetic would truncate differently
     — this test shows the fixture sees that difference."""
    from ubpl_amd import augment as AU
    g = np.load(os.path.join(GD, "augment.npz"))
    n_f64_diff = 0
    for cname, (center, scale, rot, pts) in seeds.augment_cases().items():
        t = AU.get_transform(center, scale, [256, 256], rot=rot)
        assert np.array_equal(t, g[cname + "/t"]), cname
        got = np.array([AU.transform_point(p, t) for p in pts], np.int64)
        assert np.array_equal(got, g[cname + "/kps"]), cname
        f64, _ = seeds._f64_transform_ints(pts.numpy(), center, scale, rot)
        n_f64_diff += int((f64 != g[cname + "/kps"]).any(1).sum())
        # the integer crop corners of affine_image (utils/augment.py:108-110)
        ul, br, pad = AU.crop_box(center, scale, [256, 256], rot)
        assert np.array_equal(ul + pad, g[cname + "/ul"]) and np.array_equal(br - pad, g[cname + "/br"]), cname
    assert n_f64_diff >= 8, n_f64_diff


def test_augment_warp_matrix_is_the_crop_rotate_resize_chain():
    """f1 pixel geometry: the 2x3 matrix handed to ubpl_augment_warp equals
    the reference's chain of coordinate maps (utils/augment.py:103-137),
    composed point by point here: skimage resize's pixel centres, the pad
    strip, skimage.transform.rotate's inverse map about the padded crop's
    centre, the integer crop offset, the flip — checked on every output
    pixel centre of a grid of views."""
    from ubpl_amd import augment as AU
    import torch
    ys, xs = np.mgrid[0:256:5, 0:256:5].astype(np.float64)
    for i, (center, scale, rot, _) in enumerate(seeds.augment_cases().values()):
        for flip in (False, True):
            m = AU.warp_matrix(center, scale, [256, 256], rot, 256, flip)
            ul, br, pad = AU.crop_box(center, scale, [256, 256], rot)
            Hp, Wp = br[1] - ul[1], br[0] - ul[0]
            Hc, Wc = Hp - 2 * pad, Wp - 2 * pad
            x = (xs + 0.5) * Wc / 256 - 0.5 + pad             # resize, then un-strip the pad
            y = (ys + 0.5) * Hc / 256 - 0.5 + pad
            if pad:                                           # rotate's inverse map
                th = np.deg2rad(float(torch.as_tensor(rot)))
                cx, cy = (Wp - 1) / 2, (Hp - 1) / 2
                x, y = cx + np.cos(th) * (x - cx) - np.sin(th) * (y - cy), cy + np.sin(th) * (x - cx) + np.cos(
                    th) * (y - cy)
            x, y = x + ul[0], y + ul[1]                      # crop offset
            if flip:
                x = 255 - x
            gx = m[0, 0] * xs + m[0, 1] * ys + m[0, 2]
            gy = m[1, 0] * xs + m[1, 1] * ys + m[1, 2]
            assert np.abs(gx - x).max() < 1e-9 and np.abs(gy - y).max() < 1e-9, (i, flip)
        # angle 0 keeps no pad and no rotation: the identity view at scale 256/200
    m = AU.warp_matrix([128, 128], torch.tensor(1.28), [256, 256], torch.tensor(0.), 256)
    assert np.allclose(m, [[1, 0, 0], [0, 1, 0]], atol=0)




def test_occlusion_paste_geometry_matches_reference_paste_over():
    """f1 occlusion: paste_rect's clipping (the rectangle a paste covers and
    where it starts in the occluder) and the blend alpha*color + (1-alpha)*dst
    reproduce the reference's own paste_over (utils/udaap/utils_augment.py:
    131-163) bit for bit on the fixtures (inside, clipped at every border,
    larger than the image, fractional centres)."""
    from ubpl_amd import augment as AU
    g = np.load(os.path.join(GD, "occlusion.npz"))
    for cname, (dst, occ, center) in seeds.occlusion_cases().items():
        H, W = dst.shape[:2]
        h, w = occ.shape[:2]
        out = dst.copy()
        r = AU.paste_rect(np.asarray(center, np.float64), w, h, W, H)
        if r is not None:
            x0, y0, x1, y1, sx, sy = r
            src = occ[sy:sy + (y1 - y0), sx:sx + (x1 - x0)]
            a = src[..., 3:].astype(np.float32)
            out[y0:y1, x0:x1] = a * src[..., :3] + (1 - a) * out[y0:y1, x0:x1]
        assert np.array_equal(out, g[cname + "/out"]), cname


def test_occlusion_draws_follow_the_reference_rng_order():
    """draw_occlusion consumes np.random / random exactly as augment_occlu +
    occlude_with_objects do (aug flag, count, then per occluder: choice, scale,
    centre), so a loader seeded like the reference draws the same pastes."""
    import random
    from ubpl_amd import augment as AU
    sizes = [(40, 30), (100, 80), (16, 64)]
    np.random.seed(5)
    random.seed(5)
    got = [AU.draw_occlusion(256, 256, sizes) for _ in range(20)]
    np.random.seed(5)
    random.seed(5)
    want = []
    for _ in range(20):
        ps = []
        if np.random.uniform(0, 1) < 0.5:
            for _ in range(np.random.randint(1, 8)):
                o = random.choice(range(3))
                f = np.random.uniform(0.2, 0.8)
                w1, h1 = np.round(np.array([sizes[o][1], sizes[o][0]]) * f).astype(int)
                c = np.random.uniform([0, 0], [256, 256])
                r = AU.paste_rect(c, int(w1), int(h1), 256, 256)
                if r is not None:
                    ps.append((o, int(w1), int(h1)) + r)
        want.append(ps)
    assert got == want and sum(map(len, got)) > 5


def test_occlude_rejects_out_of_range_paste_rows():
    """kernels.occlude checks every index occlude_kernel derives from a paste
    row on the host: occluder index, source window inside the
    resized occluder, destination inside the view, bank extent."""
    import torch
    from ubpl_amd import kernels as Kn
    hw = torch.tensor([[10, 12], [20, 8]], dtype=torch.int32)
    off = torch.tensor([0, 10 * 12 * 4], dtype=torch.int64)
    nbank = 10 * 12 * 4 + 20 * 8 * 4
    # view, occluder, w1, h1, x0, y0, x1, y1, sx0 | sy0 << 16
    ok = [0, 1, 6, 10, 3, 4, 9, 14, 0]
    vf = torch.tensor([0, 1, 1], dtype=torch.int32)
    Kn._occlude_check(2, 32, 32, nbank, off, hw, torch.tensor([ok], dtype=torch.int32), vf)
    for bad in ([0, 2] + ok[2:],                       # occluder index past the bank
                ok[:6] + [40, 14, 0],                  # x1 past the view
                ok[:8] + [1],                          # source window past the resized width
                ok[:8] + [(1 << 16)]):                 # ... and height
        with pytest.raises(ValueError):
            Kn._occlude_check(2, 32, 32, nbank, off, hw, torch.tensor([bad], dtype=torch.int32), vf)
    with pytest.raises(ValueError):                    # bank shorter than the occluder
        Kn._occlude_check(2, 32, 32, nbank - 4, off, hw, torch.tensor([ok], dtype=torch.int32), vf)
    with pytest.raises(ValueError):                    # view_first not a count of the rows
        Kn._occlude_check(2, 32, 32, nbank, off, hw, torch.tensor([ok], dtype=torch.int32),
                          torch.tensor([0, 2, 2], dtype=torch.int32))


def _chain_twin(img, geo, cs, res=256):
    """augment.hip augment_rotate_kernel + augment_resize_kernel restated in
    numpy float64 (their index and weight formulas, line for line)."""
    flip, ulx, uly, Hp, Wp, Hc, Wc = geo
    co, si = cs
    H, W = img.shape[:2]
    pad = (Hp - Hc) // 2
    r, c = np.mgrid[0:Hc, 0:Wc].astype(np.float64)
    R, C = r + pad, c + pad
    cx, cy = Wp / 2 - 0.5, Hp / 2 - 0.5
    sx = co * (C - cx) - si * (R - cy) + cx
    sy = si * (C - cx) + co * (R - cy) + cy
    x0, y0, x1, y1 = np.floor(sx).astype(int), np.floor(sy).astype(int), np.ceil(sx).astype(int), np.ceil(sy).astype(int)
    dx, dy = (sx - x0)[..., None], (sy - y0)[..., None]

    def px(y, x):
        ok = (x >= 0) & (x < Wp) & (y >= 0) & (y < Hp)
        iy, ix = y + uly, x + ulx
        ix = W - 1 - ix if flip else ix
        ok &= (ix >= 0) & (ix < W) & (iy >= 0) & (iy < H)
        o = np.zeros(y.shape + (3,))
        o[ok] = img[iy[ok], ix[ok]]
        return o
    inter = (1 - dy) * ((1 - dx) * px(y0, x0) + dx * px(y0, x1)) + dy * ((1 - dx) * px(y1, x0) + dx * px(y1, x1))
    i, j = np.mgrid[0:res, 0:res].astype(np.float64)
    syy, sxx = (i + 0.5) * (Hc / res) - 0.5, (j + 0.5) * (Wc / res) - 0.5
    fy, fx = np.floor(syy).astype(int), np.floor(sxx).astype(int)
    wy, wx = (syy - fy)[..., None], (sxx - fx)[..., None]

    def mi(k, n):
        return np.where(k < 0, -k, np.where(k >= n, 2 * (n - 1) - k, k))
    Y0, Y1, X0, X1 = mi(fy, Hc), mi(fy + 1, Hc), mi(fx, Wc), mi(fx + 1, Wc)
    return (1 - wy) * ((1 - wx) * inter[Y0, X0] + wx * inter[Y0, X1]) + wy * ((1 - wx) * inter[Y1, X0] +
                                                                              wx * inter[Y1, X1])


def test_augment_chain_kernel_formulas_match_the_skimage_restatement():
    """f1 pixels: the two stage kernels' formulas (rotate about the padded
    crop's centre with floor / ceil neighbours, zero outside; resize at pixel
    centres with mirrored edges) equal oracle/augment_chain.py (scikit-image
    0.20's rotate / resize on scipy.ndimage, unpinned against skimage itself)
    to float64 rounding on the geometry cases, flipped and not; and the old
    single bilinear warp deviates from that chain on rotated views — by a mean
    of 0.04-0.06 (of a [0, 1] range) on white noise, the worst case, and
    ~1.6e-3 on the Mouse images — the gap the two-stage
    path closes."""
    from oracle import augment_chain as AC
    from ubpl_amd import augment as AU
    rs = np.random.RandomState(0)
    img = rs.uniform(0, 1, (256, 256, 3))
    gaps = []
    for name, (center, scale, rot, _) in seeds.augment_cases().items():
        ul, br, pad = AU.crop_box(center, scale, [256, 256], rot)
        a = float(torch.as_tensor(rot, dtype=torch.float32))
        for flip in (0, 1):
            geo, cs = AU.chain_geometry(center, scale, [256, 256], rot, flip)
            assert geo[1:3] == (int(ul[0]), int(ul[1])) and geo[3] - geo[5] == 2 * pad
            src = np.ascontiguousarray(img[:, ::-1]) if flip else img
            ref = AC.affine_view(src, ul, br, pad, a)
            assert np.abs(_chain_twin(img, geo, cs) - ref).max() < 1e-12, (name, flip)
        if pad:
            m = AU.warp_matrix(center, scale, [256, 256], rot, 256).reshape(-1)
            gaps.append(np.abs(AC.single_warp(img, m) - AC.affine_view(img, ul, br, pad, a)).mean())
    # white noise is the worst case for a changed resampling; measured 0.041-0.062 mean here
    assert len(gaps) >= 6 and 0.02 < float(np.mean(gaps)) < 0.1, gaps


def _gfx950_code_objects(path):
    """The gfx950 code objects of a HIP shared library: the clang offload
    bundles in its .hip_fatbin section (magic, entry count, then per entry
    offset / size / triple)."""
    import struct
    d = open(path, "rb").read()
    shoff, = struct.unpack_from("<Q", d, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", d, 0x3A)
    secs = [struct.unpack_from("<IIQQQQ", d, shoff + i * shentsize) for i in range(shnum)]
    stroff = secs[shstrndx][4]
    fb = None
    for name, _, _, _, off, size in secs:
        if d[stroff + name:d.index(b"\0", stroff + name)] == b".hip_fatbin":
            fb = d[off:off + size]
    assert fb is not None, "no .hip_fatbin section in %s" % path
    magic, pos, out = b"__CLANG_OFFLOAD_BUNDLE__", 0, []
    while (pos := fb.find(magic, pos)) >= 0:
        n, = struct.unpack_from("<Q", fb, pos + 24)
        p = pos + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", fb, p)
            triple = fb[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "gfx950" in triple:
                out.append(fb[pos + off:pos + off + size])
        pos += len(magic)
    return out


def test_device_code_has_no_packed_fp32_instructions(tmp_path):
    """The race of rounds 1-3: a packed-FP32 VALU instruction
    (v_pk_add_f32 with op_sel) produced wrong results for one 16-lane pass when
    other kernels' matrix work ran beside it from concurrent queues.  The
    library is built without the packed-FP32 feature (csrc/Makefile NOPK);
    this checks the built code objects: not one v_pk_{add,mul,fma}_f32."""
    import subprocess
    from ubpl_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libubpl_hip.so not built (run __graft_entry__.build())")
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        pytest.skip("llvm-objdump not in this image")
    cos = _gfx950_code_objects(_lib.LIB_PATH)
    assert len(cos) >= 9                                  # one per .hip translation unit
    n_kernels, bad = 0, []
    for i, co in enumerate(cos):
        f = tmp_path / ("co%d" % i)
        f.write_bytes(co)
        txt = subprocess.run([objdump, "-d", "--mcpu=gfx950", str(f)], capture_output=True, text=True,
                             check=True).stdout
        n_kernels += txt.count("s_endpgm")
        bad += re.findall(r"v_pk_(?:add|mul|fma)_f32[^\n]*", txt)[:3]
    assert n_kernels > 100
    assert not bad, bad


def test_phase_check_flags_torch_arithmetic_only():
    """train._PhaseCheck (UBPL_STREAM_CHECK): arithmetic on floating-point
    tensors is recorded; views, allocations, copies, integer counters and the
    library's own ops are not.  (CPU tensors stand in for device ones here.)"""
    from ubpl_amd import train as T
    x = torch.randn(4, 3)
    n = torch.zeros(2, dtype=torch.long)
    with T._PhaseCheck(on_device=lambda t: True) as chk:
        x.view(12).reshape(3, 4)
        torch.stack([x, x.clone()])
        torch.empty_like(x).zero_()
        x[:, 0].contiguous()
        n.add_(1)                                # BN counters: integer, allowed
    assert chk.seen == [], chk.seen
    with T._PhaseCheck(on_device=lambda t: True) as chk:
        x + 1
        torch.where(x > 0, x, x * 2)
        x.sum()
    assert {"add", "mul", "sum", "where"} <= set(chk.seen), chk.seen


def test_step_generator_collectives_in_order(monkeypatch):
    """train._drive performs the collectives a step generator yields, in order,
    and returns its value; the gradient all-reduce of the students is never
    overlapped with other networks' work any more (torch's RCCL gfx950 reduce
    kernels carry packed-FP32 adds: profiles/r05_rccl_packed_fp32.txt)."""
    from ubpl_amd import dist as D
    from ubpl_amd import train as T
    calls = []
    monkeypatch.setattr(D, "allreduce_", lambda t: calls.append(("sum", t)))
    monkeypatch.setattr(D, "allreduce_grads", lambda ms: calls.append(("grads", ms)))
    t, ms = torch.zeros(3), ["m0", "m1"]

    def gen():
        yield ("sum", t)
        yield ("grads", ms)
        return "records"
    assert T._drive(gen()) == "records"
    assert calls == [("sum", t), ("grads", ms)]
    with pytest.raises(ValueError):
        T._drive(r for r in [("bogus", None)])
    assert not hasattr(T, "_AR_OVERLAP")
    rec = open(os.path.join(os.path.dirname(__file__), "..", "profiles", "r05_rccl_packed_fp32.txt")).read()
    assert "runTreeUpDown<float, FuncSum<float>" in rec


def test_zero_pseudo_count_raises_like_the_reference():
    """projects/MT_UBPL.py:292-293 (and DualPose_UBPL.py:212-213) divide the selected
    pseudo-label count by the pseudo-label count, both Python ints, in the batch line:
    a step with none raises ZeroDivisionError.  The HIP step's records raise the same
    when they are consumed (one step late, train._LaggedRecords), whether or not the
    line is printed; with counts the rate is the reference's."""
    from types import SimpleNamespace
    from ubpl_amd import train as T
    from ubpl_amd.losses import AvgCounter
    M, K = 2, 16
    args = SimpleNamespace(pseudoScoreThr=0.95)
    cnt = lambda: [AvgCounter() for _ in range(M)]   # noqa: E731

    def mt(n_ps, verbose):
        nrec = 3 * M + 1
        host = [0.1] * nrec + [4, n_ps, 0] * M + [2] + [0.5] * K     # per model [pec_n, epc_n, n_sel], 1 FDL view
        T._mt_ubpl_records(host, 0, (1, 64, 4, 3 * M + 1, True), M, cnt(), cnt(), cnt(), AvgCounter(), args,
                           verbose)
    for verbose in (False, True):
        with pytest.raises(ZeroDivisionError):
            mt(0, verbose)
        mt(3, verbose)
    assert T._pseudo_rate(3, 6) == 0.5

    def dual(c_ps, verbose):
        nrec = 3 * M + 1
        host = [0.1] * nrec + [4, 4, 5, c_ps, 1, 2] * M + [2] + [0.5] * (2 * K)
        T._dualpose_records(host, 0, 6 * M + 1, K, True, 1, M, 4, cnt(), cnt(), cnt(), AvgCounter(), args, verbose)
    for verbose in (False, True):
        with pytest.raises(ZeroDivisionError):
            dual(0, verbose)
        dual(7, verbose)
