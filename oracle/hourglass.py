"""H1-H6 — stacked hourglass forward/backward on torch CPU fp32 (oracle).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

A functional restatement of StackedHourglass (models/pose/hourglass.py:7-99)
built from Conv / Residual / Hourglass / Merge (models/base/layers.py:31-130):
parameters live in a flat name -> tensor table whose names, order, shapes
and default initialisation reproduce the reference module tree, so that
torch.manual_seed(s) gives bit-identical weights (PyTorch default init:
nn.Conv2d.reset_parameters; BatchNorm2d ones/zeros).
"""
import math

import torch
import torch.nn.functional as F


def param_table(k, nstack):
    """Ordered [(name, shape, kind, meta)] in the reference's registration order.
    kind: 'cw' conv weight, 'cb' conv bias, 'bw'/'bb' BN weight/bias."""
    tab = []

    def conv(prefix, cin, cout, ks):
        tab.append((prefix + ".weight", (cout, cin, ks, ks), "cw", None))
        tab.append((prefix + ".bias", (cout,), "cb", cin * ks * ks))

    def bn(prefix, c):
        tab.append((prefix + ".weight", (c,), "bw", None))
        tab.append((prefix + ".bias", (c,), "bb", None))

    def residual(p, cin, cout):                                   # layers.py:53-67
        h = cout // 2
        bn(p + ".bn1", cin)
        conv(p + ".conv1.conv", cin, h, 1)
        bn(p + ".bn2", h)
        conv(p + ".conv2.conv", h, h, 3)
        bn(p + ".bn3", h)
        conv(p + ".conv3.conv", h, cout, 1)
        conv(p + ".skip_layer.conv", cin, cout, 1)                 # built even when cin == cout

    def hourglass(p, n, f):                                       # layers.py:87-101
        residual(p + ".up1", f, f)
        residual(p + ".low1", f, f)
        if n > 1:
            hourglass(p + ".low2", n - 1, f)
        else:
            residual(p + ".low2", f, f)
        residual(p + ".low3", f, f)

    conv("pre.0.conv", 3, 64, 7)                                  # hourglass.py:22
    bn("pre.0.bn", 64)
    residual("pre.1", 64, 128)
    residual("pre.3", 128, 128)
    residual("pre.4", 128, 256)
    for i in range(nstack):
        hourglass("hgs.%d.0" % i, 4, 256)
    for i in range(nstack):
        residual("features.%d.0" % i, 256, 256)
        conv("features.%d.1.conv" % i, 256, 256, 1)
        bn("features.%d.1.bn" % i, 256)
    for i in range(nstack):
        conv("preds.%d.conv" % i, 256, k, 1)
    for i in range(nstack - 1):
        conv("merge_features.%d.conv.conv" % i, 256, 256, 1)
    for i in range(nstack - 1):
        conv("merge_preds.%d.conv.conv" % i, k, 256, 1)
    return tab


def bn_names(k, nstack):
    return [n[:-len(".weight")] for n, _, kind, _ in param_table(k, nstack) if kind == "bw"]


def init_params(k, nstack):
    """Default PyTorch init in registration order (consumes the global RNG the
    way the reference's constructor does)."""
    P = {}
    last_w = None
    for name, shape, kind, fan_in in param_table(k, nstack):
        t = torch.empty(shape)
        if kind == "cw":
            torch.nn.init.kaiming_uniform_(t, a=math.sqrt(5))
            last_w = t
        elif kind == "cb":
            fi, _ = torch.nn.init._calculate_fan_in_and_fan_out(last_w)
            bound = 1 / math.sqrt(fi) if fi > 0 else 0
            torch.nn.init.uniform_(t, -bound, bound)
        elif kind == "bw":
            t.fill_(1.0)
        else:
            t.zero_()
        P[name] = t
    return P


def init_buffers(k, nstack):
    B = {}
    for p in bn_names(k, nstack):
        c = None
        for name, shape, kind, _ in param_table(k, nstack):
            if name == p + ".weight":
                c = shape[0]
        B[p + ".running_mean"] = torch.zeros(c)
        B[p + ".running_var"] = torch.ones(c)
        B[p + ".num_batches_tracked"] = torch.zeros((), dtype=torch.long)
    return B


class OracleHourglass:
    """forward(x) -> preds [B,S,K,R,R] (mode 'default') or (preds, features)."""

    def __init__(self, k, nstack, mode="default", params=None):
        self.k, self.nstack, self.mode = k, nstack, mode
        self.P = init_params(k, nstack) if params is None else params
        self.buf = init_buffers(k, nstack)
        self.training = True

    def parameters(self):
        return [self.P[n] for n, _, _, _ in param_table(self.k, self.nstack)]

    def named_parameters(self):
        return [(n, self.P[n]) for n, _, _, _ in param_table(self.k, self.nstack)]

    def requires_grad_(self, flag=True):
        for t in self.P.values():
            t.requires_grad_(flag)
        return self

    # -- layers ----------------------------------------------------------
    def _conv(self, p, x, stride=1):
        w = self.P[p + ".weight"]
        return F.conv2d(x, w, self.P[p + ".bias"], stride, (w.shape[-1] - 1) // 2)

    def _bn(self, p, x):
        if self.training:
            self.buf[p + ".num_batches_tracked"] += 1
        return F.batch_norm(x, self.buf[p + ".running_mean"], self.buf[p + ".running_var"],
                            self.P[p + ".weight"], self.P[p + ".bias"], self.training, 0.1, 1e-5)

    def _residual(self, p, x):                                    # layers.py:69-84
        cin = x.shape[1]
        cout = self.P[p + ".conv3.conv.weight"].shape[0]
        res = self._conv(p + ".skip_layer.conv", x) if cin != cout else x
        o = self._conv(p + ".conv1.conv", F.relu(self._bn(p + ".bn1", x)))
        o = self._conv(p + ".conv2.conv", F.relu(self._bn(p + ".bn2", o)))
        o = self._conv(p + ".conv3.conv", F.relu(self._bn(p + ".bn3", o)))
        return o + res

    def _hourglass(self, p, n, x):                                # layers.py:104-111
        up1 = self._residual(p + ".up1", x)
        low1 = self._residual(p + ".low1", F.max_pool2d(x, 2, 2))
        low2 = self._hourglass(p + ".low2", n - 1, low1) if n > 1 else self._residual(p + ".low2", low1)
        low3 = self._residual(p + ".low3", low2)
        return up1 + F.interpolate(low3, scale_factor=2, mode="nearest")

    def __call__(self, imgs):                                     # hourglass.py:60-90
        x = F.relu(self._bn("pre.0.bn", self._conv("pre.0.conv", imgs, stride=2)))
        x = self._residual("pre.1", x)
        x = F.max_pool2d(x, 2, 2)
        x = self._residual("pre.3", x)
        x = self._residual("pre.4", x)
        hms, feats = [], []
        for i in range(self.nstack):
            hg = self._hourglass("hgs.%d.0" % i, 4, x)
            f = self._residual("features.%d.0" % i, hg)
            f = F.relu(self._bn("features.%d.1.bn" % i, self._conv("features.%d.1.conv" % i, f)))
            if self.mode != "default":
                feats.append(F.avg_pool2d(f, 2, 2) if self.mode == "AvgPool" else F.max_pool2d(f, 2, 2))
            pr = self._conv("preds.%d.conv" % i, f)
            hms.append(pr)
            if i < self.nstack - 1:
                x = x + self._conv("merge_preds.%d.conv.conv" % i, pr) + \
                    self._conv("merge_features.%d.conv.conv" % i, f)
        preds = torch.stack(hms, 1)
        if self.mode == "default":
            return preds
        return preds, torch.stack(feats, 1)

    def to(self, device):
        assert str(device) == "cpu", "the oracle runs on the CPU only"
        return self

    def train(self, flag=True):
        self.training = flag
        return self

    def eval(self):
        return self.train(False)

    def named_buffers(self):
        names = []
        for p in bn_names(self.k, self.nstack):
            names += [p + ".running_mean", p + ".running_var", p + ".num_batches_tracked"]
        return [(n, self.buf[n]) for n in names]


def oracle_factory(k, nstack, mode):
    """Model factory with PoseModel's call shape (models/pose/pose_model.py:5)."""
    return OracleHourglass(k, nstack, mode).requires_grad_(True)
