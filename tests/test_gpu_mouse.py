"""f2/f3 — validate() on the reference's Mouse validation split (500 real
images, 9 keypoints, PCK@0.2 with ref keypoints [1, 2]; datasources/mouse.py:
13-123, projects/MT_UBPL.py:355-408).

The teachers' heatmaps are decoded and scored on the device (D1-D4); the same
heatmaps go through the oracle's decoder and PCK (oracle/decode.py, pinned
bit-exact to the reference by test_oracle_golden), and the per-batch records
are folded with the reference's AvgCounters weights (bs per keypoint entry,
bs*k for the mean).  Accuracies are compared bit-exact, errors to 1e-6.

Needs data/mouse_100_500_0.3.npz (tools/pack_mouse.py, run by
__graft_entry__.build() in the build container; git-ignored, travels with the
tree): a GPU run without it FAILS — the only real-data PCK check must not pass
by being skipped.
"""
import os
import types

import numpy as np
import pytest
import torch

from oracle import decode as OD

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PACK = os.path.join(ROOT, "data", "mouse_100_500_0.3.npz")


def _teachers(K=9, S=2):
    from ubpl_amd.hourglass import StackedHourglass
    torch.manual_seed(1388)
    ts = []
    for _ in range(2):
        t = StackedHourglass(K, S, "AvgPool")
        for p in t.parameters():
            p.detach_()
        ts.append(t)
    return ts


def _require_pack():
    assert os.path.exists(PACK), ("Mouse pack %s missing: build it with tools/pack_mouse.py (or "
                                  "__graft_entry__.build()) where the reference tree exists" % PACK)


def test_validate_on_mouse_split_matches_oracle():
    _require_pack()
    from ubpl_amd import mouse
    from ubpl_amd import train as T
    data = mouse.MouseData.from_pack(PACK)
    semi, valid, lab, unlab, lidx, uidx, means, stds = data.getSemiData(100, 500, 0.3)
    assert (len(semi), len(valid), len(lab), len(unlab)) == (100, 500, 30, 70)
    assert sum(it["islabeled"] for it in semi) == 30 and all(semi[i]["islabeled"] == 0 for i in uidx)
    assert all(abs(m - 0.49) < 0.1 for m in means)
    dev = torch.device("cuda")
    teachers = _teachers()
    # move the running statistics off their init with train-mode forwards on training images
    x_tr = mouse.to_device_images(data.images("train")[:16], means, dev)
    with torch.no_grad():
        for t in teachers:
            t(x_tr)
    batches = mouse.valid_batches(data, 32, dev)[:3]
    args = types.SimpleNamespace(outRes=64, pck_ref=data.pck_ref, pck_thr=data.pck_thr)
    preds_arr, accs, errs = T.validate(batches, teachers, args)
    # the oracle on the same heatmaps
    n = len(teachers) + 1
    acc_c = [[OD.AvgCounter() for _ in range(10)] for _ in range(n)]
    err_c = [[OD.AvgCounter() for _ in range(10)] for _ in range(n)]
    want_preds = [[] for _ in range(n)]
    for t in teachers:
        t.eval()
    with torch.no_grad():
        for img, _, meta in batches:
            bs, k = meta["kpsMap"].shape[:2]
            pm = []
            for t in teachers:
                hm = t(img)[0][:, -1].float().cpu()
                p, _ = OD.kps_from_heatmap(hm, meta["center"], meta["scale"], [64, 64])
                pm.append(p)
            pm.append(torch.stack(pm, -1).mean(-1))
            for mi, p in enumerate(pm):
                e, a = OD.acc_pck(p, meta["kpsMap"], data.pck_ref, data.pck_thr)
                for idx in range(k + 1):
                    acc_c[mi][idx].update(a[idx].item(), bs if idx < k else bs * k)
                    err_c[mi][idx].update(e[idx].item(), bs if idx < k else bs * k)
                want_preds[mi] += p.tolist()
    for t in teachers:
        t.train()
    for mi in range(n):
        assert np.array_equal(np.array(preds_arr[mi]), np.array(want_preds[mi])), mi
        assert [c.avg for c in acc_c[mi]] == accs[mi], mi
        np.testing.assert_allclose(errs[mi], [c.avg for c in err_c[mi]], rtol=1e-6, atol=1e-6)


REF_PCK = os.path.join(ROOT, "tests", "golden", "ref_pck.json")


@pytest.mark.timeout(900)
def test_pck_tracks_the_reference_training():
    """north_star 'PCK@0.2 within ±0.1 of reference': the MT_UBPL experiment on
    the Mouse split (HG2, trainBS 4 with 2 labeled, the reference's ramps) run
    on the HIP path (tools/mouse_pck.py) against the REFERENCE's own train() /
    validate() run on CPU for the same epochs, seeds, sampler and augmentation
    draws (tools/ref_pck.py -> tests/golden/ref_pck.json): at every validated
    epoch, each teacher's PCK@0.2 and the mean-prediction PCK are within 0.1 of
    the reference's."""
    import importlib.util
    import json
    ref = json.load(open(REF_PCK))
    _require_pack()
    epochs = len(ref["epochs"])
    spec = importlib.util.spec_from_file_location("mouse_pck", os.path.join(ROOT, "tools", "mouse_pck.py"))
    mp = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mp)
    log = mp.run(mp.parser().parse_args(["--epochs", str(epochs)]), write=False)
    checked = 0
    for r_ref, r in zip(ref["epochs"], log["epochs"]):
        if "pck" not in r_ref:
            continue
        print("epoch %d  ours %s  reference %s" % (r["epoch"], r["pck"], r_ref["pck"]))
        assert r["epoch"] == r_ref["epoch"]
        for a, b in zip(r["pck"], r_ref["pck"]):
            assert abs(a - b) <= 0.1, (r["epoch"], r["pck"], r_ref["pck"])
        checked += 1
    assert checked >= 4
    # the +-0.1 window alone accepts a run that learned nothing (the reference
    # starts at 0.05): the last epoch must also reach half the reference's PCK
    last_ref, last = ref["epochs"][-1], log["epochs"][-1]
    for a, b in zip(last["pck"], last_ref["pck"]):
        assert a >= 0.5 * b, (last["epoch"], last["pck"], last_ref["pck"])
