"""Stacked hourglass on the HIP kernels (H1-H6).

Drop-in for StackedHourglass / pose_model / PoseModel
(models/pose/hourglass.py:7-99, models/pose/pose_model.py:5-13,
models/__init__.py:4):

* the module tree, parameter names and order, buffer names, shapes and the
  default initialisation are the reference's (so torch.manual_seed(s) gives
  bit-identical weights, and state_dict() interchanges with reference
  checkpoints);
* every parameter is an alias into ONE flat device buffer (`flat_params`,
  grad-carrying parameters first, the never-trained skip_layer parameters of
  identity Residuals last), gradients accumulate into `flat_grads`, BN
  running statistics live in `flat_stats` — so the EMA teacher update, the
  optimizer step and the DDP all-reduce are each a single kernel / collective
  over a contiguous buffer;
* forward/backward are explicit executors over the HIP kernels (conv.hip with
  the pre-activation BN+ReLU fused into operand staging, bn.hip, pool.hip);
  autograd sees the whole network as one Function.
"""
import math
import os

import torch
from torch import nn

from . import _lib
from . import kernels as Kn

BN_EPS = 1e-5
BN_MOMENTUM = 0.1
# residual bn1 statistics from the producer's partials (conv epilogue, max-pool,
# upsample-add) instead of a pass over the input (UBPL_PRODUCER_STATS=1).  Off by
# default: partials + a finalize launch lose to the one-launch pass (-0.6 % step).
_PRODUCER_STATS = os.environ.get("UBPL_PRODUCER_STATS", "0") == "1"
# 64-channel 3x3 weight gradients on the split path (UBPL_WGRAD3_64=0: exact-f32 kernel)
_WGRAD3_64 = os.environ.get("UBPL_WGRAD3_64", "1") != "0"
# 1x1 weight gradients on the 6xbf16 split-on-load kernel (UBPL_WGRAD1_SPLIT=0: exact-f32 kernel)
_WGRAD1_SPLIT = os.environ.get("UBPL_WGRAD1_SPLIT", "1") != "0"
# BatchNorm backward statistics from the data-gradient epilogues (UBPL_BWD_EPI=1).  Off by
# default: the epilogue's x reads sit on the critical path of the big dgrad launches and
# cost more (-3 % step) than the separate streaming partials pass they replace.
_BWD_EPI = os.environ.get("UBPL_BWD_EPI", "0") == "1"
# the 7x7/s2 stem on the split path by space-to-depth (UBPL_STEM_S2D=0: exact-f32 kernel)
_STEM_S2D = os.environ.get("UBPL_STEM_S2D", "1") != "0"
# the stem's 7x7 weight gradient on the split path from the forward's space-to-depth image
# (round 5; UBPL_STEM_WGRAD=0: the exact-f32 conv_wgrad2_kernel)
_STEM_WGRAD = os.environ.get("UBPL_STEM_WGRAD", "1") != "0"
# forward BatchNorm statistics from the conv epilogues (UBPL_FWD_EPI=1).  Off by default:
# epilogue partials + a finalize launch measured 1.3 % slower than the one-launch
# statistics pass (stats_kernel) on the training step.
_FWD_EPI = os.environ.get("UBPL_FWD_EPI", "0") == "1"
# 2xfp16: the 3x3 data / weight gradients on 2xfp16 too (dy scaled by the BN backward's bound of
# it, bn.hip bwd_stats_kernel BOUND); UBPL_FP16_BWD3=0: on 6xbf16 (with the forward's 6xbf16 image
# kept for the weight gradient)
_FP16_BWD3 = os.environ.get("UBPL_FP16_BWD3", "1") != "0"
# diagnostic (tools/graph_fwd_probe.py locate): the hourglass upsample-add out of place, its
# up1 input saved, so a graph replay's first wrong activation can name up1 or the add
_UPADD_OOP = os.environ.get("UBPL_UPADD_OOP", "0") == "1"
# diagnostic (tools/fwd_race.py, forwards only, weights never updated): re-lay out the weights in a
# model's first forward only
_RELAYOUT_ONCE = os.environ.get("UBPL_RELAYOUT_ONCE", "0") == "1"
# diagnostic (tools/fwd_race.py locate): keep low3 (the add's second operand) as a saved activation
# ("1": the tensor itself, kept alive; "clone": a copy made right after it is produced)
_SAVE_LOW3 = os.environ.get("UBPL_SAVE_LOW3", "")


# ---------------------------------------------------------------------------
# Parameter table in the reference's registration order
# ---------------------------------------------------------------------------
def build_table(k, nstack):
    """[(name, shape, kind, live)] kind in {'cw','cb','bw','bb'}; live=False for the
    skip_layer of Residual(c, c) (constructed, never used: models/base/layers.py:63-67)."""
    tab = []

    def conv(p, cin, cout, ks, live=True):
        tab.append((p + ".weight", (cout, cin, ks, ks), "cw", live))
        tab.append((p + ".bias", (cout,), "cb", live))

    def bn(p, c):
        tab.append((p + ".weight", (c,), "bw", True))
        tab.append((p + ".bias", (c,), "bb", True))

    def residual(p, cin, cout):
        half = cout // 2
        bn(p + ".bn1", cin)
        conv(p + ".conv1.conv", cin, half, 1)
        bn(p + ".bn2", half)
        conv(p + ".conv2.conv", half, half, 3)
        bn(p + ".bn3", half)
        conv(p + ".conv3.conv", half, cout, 1)
        conv(p + ".skip_layer.conv", cin, cout, 1, live=cin != cout)

    def hourglass(p, n, f):
        residual(p + ".up1", f, f)
        residual(p + ".low1", f, f)
        if n > 1:
            hourglass(p + ".low2", n - 1, f)
        else:
            residual(p + ".low2", f, f)
        residual(p + ".low3", f, f)

    conv("pre.0.conv", 3, 64, 7)
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


def _default_init(tab):
    """nn.Conv2d.reset_parameters / BatchNorm2d defaults, consuming the CPU RNG in
    registration order exactly like the reference constructor."""
    vals = []
    last_w = None
    for name, shape, kind, _ in tab:
        t = torch.empty(shape)
        if kind == "cw":
            nn.init.kaiming_uniform_(t, a=math.sqrt(5))
            last_w = t
        elif kind == "cb":
            fan_in, _ = nn.init._calculate_fan_in_and_fan_out(last_w)
            bound = 1 / math.sqrt(fan_in) if fan_in > 0 else 0
            nn.init.uniform_(t, -bound, bound)
        elif kind == "bw":
            t.fill_(1.0)
        else:
            t.zero_()
        vals.append(t)
    return vals


class _Node(nn.Module):
    """Container mirroring one module of the reference tree (params/buffers only)."""

    def forward(self, *a):  # pragma: no cover - never called
        raise RuntimeError("structural node")


# ---------------------------------------------------------------------------
# The model
# ---------------------------------------------------------------------------
class StackedHourglass(nn.Module):
    """StackedHourglass(k, nStack, mode) on the HIP path.  forward(imgs) ->
    preds [B,S,K,R,R] (mode 'default') or (preds, features [B,S,256,R/2,R/2])
    for mode 'AvgPool' / 'MaxPool' (models/pose/hourglass.py:60-99).  'ConvOne'
    builds a 128-channel conv on 256-channel features in the reference and
    fails there; it is rejected here."""

    def __init__(self, k, nStack, mode="default", device=None):
        super().__init__()
        if mode not in ("default", "AvgPool", "MaxPool"):
            raise ValueError("mode %r unsupported (ConvOne is broken in the reference: hourglass.py:227)" % mode)
        _lib.require_gpu()
        device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.k, self.nStack, self.mode = k, nStack, mode
        tab = build_table(k, nStack)
        vals = _default_init(tab)          # CPU RNG, reference order
        # flat layout: live parameters first (reference order), dead ones last
        order = [i for i, e in enumerate(tab) if e[3]] + [i for i, e in enumerate(tab) if not e[3]]
        offs, o = {}, 0
        for i in order:
            n = vals[i].numel()
            offs[tab[i][0]] = (o, n, tab[i][1])
            o += (n + 3) // 4 * 4          # keep every segment 16-B aligned
        self.n_total = o
        self.n_live = max(offs[tab[i][0]][0] + offs[tab[i][0]][1] for i in order if tab[i][3])
        self.n_live = (self.n_live + 3) // 4 * 4
        host = torch.zeros(self.n_total)
        for i, e in enumerate(tab):
            s, n, _ = offs[e[0]]
            host[s:s + n] = vals[i].reshape(-1)
        self.flat_params = host.to(device)
        self.flat_grads = torch.zeros(self.n_total, device=device)
        self._offs = offs
        self._table = tab
        # BN running statistics in one flat buffer: per BN [mean(C) | var(C)]
        bns = [e[0][:-len(".weight")] for e in tab if e[2] == "bw"]
        self._bn_names = bns
        so, sidx = 0, {}
        for b in bns:
            c = offs[b + ".weight"][1]
            sidx[b] = (so, c)
            so += 2 * c
        stats = torch.zeros(so)
        for b, (s, c) in sidx.items():
            stats[s + c:s + 2 * c] = 1.0
        self.flat_stats = stats.to(device)
        self._nbt = torch.zeros(len(bns), dtype=torch.long, device=device)
        self._sidx = sidx
        self._bn_index = {b: i for i, b in enumerate(bns)}
        # module tree with aliased parameters / buffers, in reference order
        for name, shape, kind, _ in tab:
            mod, attr = self._node_for(name)
            s, n, shp = offs[name]
            mod.register_parameter(attr, nn.Parameter(self.flat_params[s:s + n].view(shp)))
            if kind == "bb":
                b = name[:-len(".bias")]
                bs, c = sidx[b]
                mod.register_buffer("running_mean", self.flat_stats[bs:bs + c])
                mod.register_buffer("running_var", self.flat_stats[bs + c:bs + 2 * c])
                mod.register_buffer("num_batches_tracked", self._nbt[self._bn_index[b]])
        self._grad_views_attached = False
        self._ws = {}
        self._grad_keep = []          # upstream gradients alive until their stream is joined
        # re-laid-out conv weights, rebuilt by one launch per forward (tap-major
        # [Cout][T][Cin] for KS > 1) and per backward (dgrad [Cin][T][Cout]):
        # tables per conv precision, see set_conv_precision / _build_weight_tables
        self._device = device
        self.set_conv_precision(None)

    # -- structure helpers ------------------------------------------------
    def _node_for(self, name):
        parts = name.split(".")
        mod = self
        for p in parts[:-1]:
            if p not in mod._modules:
                mod.add_module(p, _Node())
            mod = mod._modules[p]
        return mod, parts[-1]

    def _apply(self, fn, recurse=True):
        # Parameters alias flat device buffers: only same-device no-op moves are legal.
        probe = fn(self.flat_params)
        if probe.device != self.flat_params.device or probe.dtype != self.flat_params.dtype:
            raise RuntimeError("ubpl_amd StackedHourglass lives on its GPU in float32 (flat buffers); "
                               "moving it to %s/%s is not supported" % (probe.device, probe.dtype))
        return self

    def P(self, name):
        s, n, shp = self._offs[name]
        return self.flat_params[s:s + n].view(shp)

    def G(self, name):
        s, n, shp = self._offs[name]
        return self.flat_grads[s:s + n].view(shp)

    def stats(self, bn):
        s, c = self._sidx[bn]
        return self.flat_stats[s:s + c], self.flat_stats[s + c:s + 2 * c]

    def set_conv_precision(self, name):
        """Conv arithmetic (kernels.CONV_PRECISIONS; None = $UBPL_CONV_PRECISION or the default):
        'f32'    every conv on the exact-f32 MFMA (conv.hip);
        '6xbf16' the 3x3 convs (forward and data gradient) on split-bf16 MFMA with
                 3 bf16 pieces per operand over pre-split activations (conv_split.hip
                 PSA path, error at the f32 path's level), the 1x1 convs whose
                 planes fill the chip on the same arithmetic with the activations
                 split while they are staged, the rest f32;
        '2xfp16' the forward convs as '6xbf16' places them, on 2 fp16 pieces of the
                 power-of-two-scaled operands (3 MFMA products instead of 6, operands
                 to 2^-22); the 3x3 data and weight gradients too, their dy scaled
                 by the power of two the BN backward's bound of it picks
                 (UBPL_FP16_BWD3=0: on 6xbf16); the 1x1 gradients on 6xbf16;
        'bf16'   every conv with 16-channel contraction groups (3x3 and 1x1, forward
                 and data gradient) with ONE piece per operand = bf16 operands, f32
                 accumulation (BASELINE config 5's throughput path): 1x1 convs whose
                 plane fills the chip on the split-on-load kernel (no pre-split pass),
                 the rest on the PSA kernels; weight gradients on the PSA (3x3) and
                 split-on-load (1x1, 128-multiple channels) kernels, the other 1x1
                 weight gradients exact f32.
        The stem (7x7, stride 2, 3 input channels) runs in f32 except on the
        6xbf16 space-to-depth path."""
        self.conv_pieces = Kn.conv_precision_pieces(name)          # the forward's
        self.bwd_pieces = Kn.backward_pieces(self.conv_pieces)      # the gradients'
        # the 3x3 convs' gradients (data and weight) on the forward's 2xfp16 too
        self.bwd3_pieces = 2 if self.conv_pieces == 2 and _FP16_BWD3 else self.bwd_pieces
        self._build_weight_tables()

    def _build_weight_tables(self):
        """Split path (_wsp[mode]): the convs the precision puts there whose
        contraction runs over 16-channel groups (Cin for the forward, Cout for
        the data gradient); f32 path: _wlay[mode] = every conv that needs a
        re-layout, _wlay[("rest", mode)] = those of them not on the split path."""
        tab, offs, device = self._table, self._offs, self._device
        stem = "pre.0.conv.weight"
        self._wsp = {}
        for mode in (0, 1):
            # the pieces of a conv's table: the forward's (mode 0), its gradients' (mode 1: 3x3
            # and 1x1 may differ under 2xfp16) — one batched split launch per piece count
            pieces_of = (lambda ks: self.conv_pieces) if mode == 0 else \
                (lambda ks: self.bwd3_pieces if ks == 3 else self.bwd_pieces)
            tables = {}
            for name, shape, kind, live in tab:
                if kind != "cw" or not live or name == stem:
                    continue
                pieces = pieces_of(shape[2])
                if not pieces or shape[1 if mode == 0 else 0] % 16:
                    continue
                # 6xbf16 / 2xfp16: 3x3 (PSA path) and 1x1 (split on load; outputs of 16 channels
                # and up, the heatmap projection included)
                if pieces in (2, 3) and not (shape[2] == 3 or (shape[2] == 1 and shape[0 if mode == 0 else 1] % 16 == 0)):
                    continue
                rows, idx, o = tables.setdefault(pieces, ([], {}, [0]))
                s, n, _ = offs[name]
                T = shape[2] * shape[3]
                rows.append((s, o[0], shape[0], shape[1], T))
                idx[name] = (o[0], (shape[0], T, shape[1]) if mode == 0 else (shape[1], T, shape[0]))
                o[0] += (n + 7) // 8 * 8
            subs = []
            for pieces, (rows, idx, o) in sorted(tables.items()):
                buf = torch.empty(max(pieces, 1) * max(o[0], 8), dtype=torch.int16, device=device)
                subs.append([torch.tensor(rows, dtype=torch.int64).reshape(-1, 5).to(device), max(o[0], 8), idx, buf,
                             pieces])
            self._wsp[mode] = subs
        self._wlay = {}
        for mode in (0, 1):
            need = (lambda ks, nm: ks > 1) if mode == 0 else (lambda ks, nm: nm != stem)
            # (1x1 convs stay in "rest" too: the f32 kernel takes the small planes)
            on_split = set(nm for sub in self._wsp[mode] for nm in sub[2])
            for key, keep in ((mode, need), (("rest", mode), lambda ks, nm, f=need, sp=on_split:
                                               f(ks, nm) and (ks == 1 or nm not in sp))):
                rows, idx, o = [], {}, 0
                for name, shape, kind, live in tab:
                    if kind != "cw" or not live or not keep(shape[2], name):
                        continue
                    s, n, _ = offs[name]
                    rows.append((s, o, shape[0], shape[1], shape[2] * shape[3]))
                    T = shape[2] * shape[3]
                    idx[name] = (o, (shape[0], T, shape[1]) if mode == 0 else (shape[1], T, shape[0]))
                    o += (n + 3) // 4 * 4
                tbl = torch.tensor(rows, dtype=torch.int64).reshape(-1, 5).to(device)
                self._wlay[key] = (tbl, torch.empty(max(o, 4), device=device), idx, mode)

    def relayout_weights(self, mode):
        if self.conv_pieces:
            for tbl, plane, _, buf, pieces in self._wsp[mode]:
                Kn.conv_weights_split(self.flat_params, buf, plane, tbl, mode, pieces)
            tbl, buf, _, m = self._wlay[("rest", mode)]
            if tbl.shape[0]:
                Kn.conv_weights_relayout(self.flat_params, buf, tbl, m)
            return
        tbl, buf, _, m = self._wlay[mode]
        Kn.conv_weights_relayout(self.flat_params, buf, tbl, m)

    def W(self, mode, name):
        key = ("rest", mode) if self.conv_pieces else mode
        _, buf, idx, _ = self._wlay[key]
        o, shp = idx[name]
        return buf[o:o + shp[0] * shp[1] * shp[2]].view(shp)

    def SW(self, mode, name):
        """Split weights of a conv (None when it is not on the split path)."""
        if not self.conv_pieces:
            return None
        for _, plane, idx, buf, pieces in self._wsp[mode]:
            if name in idx:
                o, shp = idx[name]
                return Kn.SplitWeights(buf, plane, o, shp, pieces)
        return None

    def alt_grad_buffer(self):
        """Second gradient buffer for a backward pass that runs concurrently with
        another of the same network (train.py: a student's second view on its
        idle teacher's stream); merge_alt_grads adds it into flat_grads."""
        if getattr(self, "_alt_grads", None) is None:
            self._alt_grads = torch.zeros_like(self.flat_grads)
            self._alt_pending = []
        return self._alt_grads

    def merge_alt_grads(self, release=True):
        """flat_grads += the concurrent pass's gradients (on the current stream,
        after it has joined that pass's stream).  release=False keeps the
        tensors the backward streams read (upstream gradients, the concurrent
        pass's saved activations) alive: a caller merging on a side stream
        releases them with release_backward_refs() after the main stream has
        joined it — freed earlier, the caching allocator could hand their
        blocks to main while those kernels still read them."""
        if getattr(self, "_alt_pending", None):
            # (the library's add: no packed-FP32 instructions, see csrc/Makefile NOPK; this may run on a
            # side stream beside other networks' backward)
            Kn.add(self.flat_grads, self._alt_grads, out=self.flat_grads)
            self._alt_grads.zero_()
            self._alt_done = self._alt_pending
            self._alt_pending = []
        if release:
            self.release_backward_refs()

    def release_backward_refs(self):
        self._alt_done = []
        self._grad_keep = []

    def live_params(self):
        return self.flat_params[:self.n_live]

    def live_grads(self):
        return self.flat_grads[:self.n_live]

    def attach_grad_views(self):
        """Make every parameter's .grad alias flat_grads (for torch optimizers)."""
        for name, p in self.named_parameters():
            if self._offs[name][0] < self.n_live:      # dead skip_layer params keep grad None
                p.grad = self.G(name)
        self._grad_views_attached = True

    def zero_grad(self, set_to_none=True):
        self.flat_grads.zero_()
        self.attach_grad_views()

    # -- forward ----------------------------------------------------------
    def forward(self, imgs):
        _lib.require_gpu(imgs)
        if imgs.dtype != torch.float32:
            raise TypeError("imgs must be float32")
        imgs = imgs.contiguous()
        need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        if need_grad and not self.training:
            raise RuntimeError("ubpl_amd: backward through eval-mode BatchNorm is not supported")
        if need_grad:
            preds, feats = _HourglassFn.apply(imgs, self._anchor(), self)
        else:
            with torch.no_grad():
                preds, feats, _ = self._forward_impl(imgs, save=False)
        if self.mode == "default":
            return preds
        return preds, feats

    def _anchor(self):
        a = getattr(self, "_anchor_t", None)
        if a is None:
            a = torch.zeros((), device=self.flat_params.device, requires_grad=True)
            self._anchor_t = a
        return a

    def _scratch(self, B, C):
        key = ("part", B)
        if key not in self._ws:
            n = 0
            for c in (64, 128, 256, 512):
                n = max(n, int(_lib.lib().ubpl_bn_part_doubles(B, c)))
            # zeroed once: the arrival counters at its tail reset themselves
            self._ws[key] = torch.zeros(n, dtype=torch.float64, device=self.flat_params.device)
            self._ws[("coef", B)] = torch.empty(3 * 512 + 4, device=self.flat_params.device)
        return self._ws[key]

    def _forward_impl(self, imgs, save):
        B = imgs.shape[0]
        dev = imgs.device
        part = self._scratch(B, 64)
        if save:
            self._grad_keep = []     # the last step's upstream gradients (its streams joined since)
        ex = _Exec(self, B, dev, part, train=self.training, save=save)
        if _RELAYOUT_ONCE and save:
            raise RuntimeError("UBPL_RELAYOUT_ONCE is a forwards-only diagnostic: a training forward's weights "
                               "change every step, the once-laid-out copies would go stale")
        if not (_RELAYOUT_ONCE and getattr(self, "_relaid", False)):
            self.relayout_weights(0)
            self.relayout_weights(1)       # k-major 1x1 weights for conv1x1_forward_kmajor
            self._relaid = True
        if self.training:
            self._nbt.add_(1)
        else:
            ex.eval_coeffs()
        x = ex.stem(imgs)
        x = ex.residual("pre.1", x)
        x1 = x
        part = ex.stat_buffer((x1.shape[0], x1.shape[1], x1.shape[2] // 2, x1.shape[3] // 2))
        x = Kn.maxpool2x2(x1, stat_part=part)
        ex.give_part(x, part)
        ex.save("pre.2", x1)
        x = ex.residual("pre.3", x)
        x = ex.residual("pre.4", x)
        preds, feats = [], []
        for i in range(self.nStack):
            hg = ex.hourglass("hgs.%d.0" % i, 4, x)
            f0 = ex.residual("features.%d.0" % i, hg)
            f = ex.conv_bn_relu("features.%d.1" % i, f0)
            if self.mode != "default":
                feats.append(Kn.avgpool2x2(f) if self.mode == "AvgPool" else Kn.maxpool2x2(f))
            pr = ex.conv("preds.%d.conv" % i, f)
            preds.append(pr)
            if i < self.nStack - 1:
                t = ex.conv("merge_preds.%d.conv.conv" % i, pr, res=x)
                x, part = ex.conv("merge_features.%d.conv.conv" % i, f, res=t, out=t, stats=True)
                ex.give_part(x, part)
            ex.save("stack.%d" % i, (f, pr))
        P = torch.stack(preds, 1)
        Fs = torch.stack(feats, 1) if feats else None
        return P, Fs, ex

    # -- backward ---------------------------------------------------------
    def _backward_impl(self, ex, dpreds, dfeats):
        ex.backward(dpreds, dfeats)


class _HourglassFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, imgs, anchor, model):
        preds, feats, ex = model._forward_impl(imgs, save=True)
        ctx.ex = ex
        ctx.model = model
        if feats is None:
            feats = preds.new_empty(0)
        return preds, feats

    @staticmethod
    def backward(ctx, dpreds, dfeats):
        model = ctx.model
        ex = ctx.ex
        if ex.bwd_stream is not None:
            # a second view's backward on another (idle) stream, into the
            # alternate gradient buffer; the caller joins that stream and merges
            if dfeats is not None and dfeats.numel() == 0:
                dfeats = None
            s = ex.bwd_stream
            s.wait_stream(torch.cuda.current_stream(s.device))
            with torch.cuda.stream(s):
                model._backward_impl(ex, dpreds, dfeats)
            model._alt_pending.append((ex, dpreds, dfeats))   # alive until the join
            return None, None, None
        # torch optimizers may have reset .grad to None (zero_grad(set_to_none));
        # then the flat buffer is stale and is restarted from zero.
        first = next(iter(model.parameters()))
        if first.grad is None or first.grad.data_ptr() != model.flat_grads.data_ptr() + 4 * model._offs[
                model._table[0][0]][0]:
            model.flat_grads.zero_()
            model.attach_grad_views()
        if dfeats is not None and dfeats.numel() == 0:
            dfeats = None
        # the upstream gradients come from the loss backward on the main stream
        # and are read here on this network's stream; kept alive until the
        # caller has joined that stream (merge_alt_grads), or the caching
        # allocator hands their blocks back to main while these kernels still
        # read them (a race that shows once nothing paces the launches: the
        # captured step)
        model._grad_keep.append((dpreds, dfeats))
        # the saved activations stay with ctx: the reference runs backward(retain_graph=True)
        # once per student and the shared FDL term reaches both networks twice
        model._backward_impl(ctx.ex, dpreds, dfeats)
        return None, None, None


# ---------------------------------------------------------------------------
# Executor: one forward pass (+ its saved tensors) and its backward
# ---------------------------------------------------------------------------
class _Exec:
    def __init__(self, model, B, dev, part, train, save):
        self.m, self.B, self.dev, self.part, self.train, self.do_save = model, B, dev, part, train, save
        # backward on another stream into the alternate gradient buffer (train.py sets
        # model._bwd_stream around a student's second-view forward)
        self.bwd_stream = getattr(model, "_bwd_stream", None) if save else None
        self.gbuf = model.alt_grad_buffer() if self.bwd_stream is not None else model.flat_grads
        if self.bwd_stream is not None:
            key = ("alt", B)
            if key not in model._ws:
                model._ws[key] = (torch.zeros_like(part), torch.empty(3 * 512 + 4, device=dev))
            self.bpart, self.bcoef = model._ws[key]
        else:
            self.bpart, self.bcoef = part, None
        self.saved = {}
        self.saved_split = {}
        self._rp = None     # (tensor, BN partials of it) from its producer, for the next residual's bn1
        C = sum(self.m._offs[b + ".weight"][1] for b in self.m._bn_names)
        self.coef = torch.empty(4 * C, device=dev)     # per BN: scale|shift|mean|invstd
        self.cidx, o = {}, 0
        for b in self.m._bn_names:
            c = self.m._offs[b + ".weight"][1]
            self.cidx[b] = (o, c)
            o += 4 * c

    # ---- bookkeeping
    def save(self, key, val):
        if self.do_save:
            self.saved[key] = val

    def give_part(self, y, part):
        """y's producer wrote its BatchNorm partials: the residual that takes y
        next reads its bn1 statistics from them (no pass over y)."""
        self._rp = (y, part) if part is not None and _PRODUCER_STATS else None

    def take_part(self, x):
        rp, self._rp = self._rp, None
        return rp[1] if rp is not None and rp[0] is x else None

    def stat_buffer(self, x_shape):
        """Partials buffer for an elementwise producer's output (None: not on this path)."""
        B, C, H, W = x_shape
        if not self.train or not _PRODUCER_STATS or not Kn.stats_ok(H, W):
            return None
        return Kn.bn_partial_buffer(C, B * H * W, self.dev)

    def bnc(self, bn):
        o, c = self.cidx[bn]
        v = self.coef[o:o + 4 * c]
        return v[:c], v[c:2 * c], v[2 * c:3 * c], v[3 * c:]

    def eval_coeffs(self):
        for b in self.m._bn_names:
            sc, sh, _, _ = self.bnc(b)
            rm, rv = self.m.stats(b)
            Kn.bn_eval_coeffs(self.m.P(b + ".weight"), self.m.P(b + ".bias"), rm, rv, BN_EPS, sc, sh)

    def bn(self, name, x, part=None):
        """Train: batch statistics (+ running-stat update) — from the partials
        the producing conv wrote (part = (buffer, shift)) or by a pass over x;
        eval: precomputed."""
        sc, sh, mu, istd = self.bnc(name)
        if self.train:
            rm, rv = self.m.stats(name)
            g, b = self.m.P(name + ".weight"), self.m.P(name + ".bias")
            if part is not None:
                Kn.bn_stats_from_partials(part, x.shape[1], x.shape[0] * x[0, 0].numel(), g, b, BN_EPS,
                                          BN_MOMENTUM, rm, rv, mu, istd, sc, sh)
            else:
                Kn.bn_forward_stats(x, g, b, BN_EPS, BN_MOMENTUM, rm, rv, self.part, mu, istd, sc, sh)
        return sc, sh

    def conv(self, name, x, stride=1, pro=None, res=None, out=None, stats=False):
        """stats=True: also return the BatchNorm partials of the output for the
        BN that consumes it — (y, (buffer, shift)) from the conv epilogue where
        the kernel has one, (y, None) otherwise."""
        y, part = self._conv(name, x, stride, pro, res, out, stats and self.train)
        return (y, part) if stats else y

    def _conv(self, name, x, stride, pro, res, out, stats):
        w = self.m.P(name + ".weight")
        b = self.m.P(name + ".bias")
        ps, ph = (None, None) if pro is None else pro
        B, Cout = x.shape[0], w.shape[0]
        mkpart = lambda: (Kn.bn_partial_buffer(Cout, B * x.shape[2] * x.shape[3], x.device)
                          if stats and _FWD_EPI else None)
        ws = self.m.SW(0, name + ".weight") if stride == 1 else None
        if ws is not None and ws.npieces in (1, 2, 3) and ws.shape[1] == 1:
            if Kn.conv1x1_split_load_ok(x, ws, small=self.m.conv_pieces == 2):
                part = mkpart() if ws.npieces == 3 else None
                return Kn.conv1x1_forward_split_load(x, ws, b, ps, ph, res=res, out=out, stat_part=part), part
            if ws.npieces in (2, 3):
                ws = None                                # small plane: the f32 1x1 kernel (bf16: the PSA kernel)
        if ws is not None:
            if ws.npieces in (1, 2, 3):
                part = mkpart() if ws.npieces != 2 else None
                keep = self.do_save and ws.shape[1] == 9
                if ws.npieces == 2 and keep and self.m.bwd3_pieces == 3:
                    # 2xfp16 forward, 6xbf16 gradients: the conv's fp16 image and, from the same
                    # read, the 6xbf16 one its weight gradient takes
                    xs, xs3 = Kn.split_activation(x, 2, 1, ps, ph, with3=True)
                    self.saved_split[name] = xs3
                else:
                    xs = Kn.split_activation(x, ws.npieces, (ws.shape[1] == 9) * 1, ps, ph)
                    if keep:
                        self.saved_split[name] = xs      # the 3x3 weight gradient's B operand
                return Kn.conv2d_forward_psa(xs, ws, b, res=res, out=out, stat_part=part), part
            return Kn.conv2d_forward_split(x, ws, b, ps, ph, res=res, out=out), None
        if w.shape[2] == 1 and stride == 1 and Kn.conv1x1_kmajor_ok(x, w.shape[0]):
            part = mkpart()
            return Kn.conv1x1_forward_kmajor(x, self.m.W(1, name + ".weight"), b, ps, ph, res=res, out=out,
                                             stat_part=part), part
        wt = self.m.W(0, name + ".weight") if w.shape[2] > 1 else None
        return Kn.conv2d_forward(x, w, b, stride, ps, ph, res=res, out=out, w_tap=wt), None

    # ---- layers
    def stem(self, imgs):
        if self.m.conv_pieces in (1, 2, 3) and _STEM_S2D and Kn.stem_s2d_ok(imgs):
            # 7x7/s2 as a 4x4 stride-1 conv over the space-to-depth image, on the split path
            # (6xbf16, also under 2xfp16: the image is its weight gradient's operand), or on
            # bf16 operands (the "bf16" precision)
            np_ = self.m.bwd_pieces
            ws = Kn.stem_weight_s2d_split(self.m.P("pre.0.conv.weight"), np_)
            xs = Kn.stem_s2d_split(imgs, 2, np_)
            y0 = Kn.conv2d_forward_psa(xs, ws, self.m.P("pre.0.conv.bias"))
            if self.do_save and _STEM_WGRAD:
                self.saved_split["pre.0.conv"] = xs      # the weight gradient's B operand
        else:
            y0 = self.conv("pre.0.conv", imgs, stride=2)
        sc, sh = self.bn("pre.0.bn", y0)
        x0 = Kn.bn_apply(y0, sc, sh, relu=1)
        self.save("pre.0", (imgs, y0))
        return x0

    def conv_bn_relu(self, p, x):
        y, part = self.conv(p + ".conv", x, stats=True)
        sc, sh = self.bn(p + ".bn", y, part)
        f = Kn.bn_apply(y, sc, sh, relu=1)
        self.save(p, (x, y))
        return f

    def residual(self, p, x):
        """models/base/layers.py:69-84 (pre-activation bottleneck)."""
        cin = x.shape[1]
        cout = self.m._offs[p + ".conv3.conv.weight"][2][0]
        c1 = self.bn(p + ".bn1", x, self.take_part(x))
        t1, part = self.conv(p + ".conv1.conv", x, pro=c1, stats=True)
        c2 = self.bn(p + ".bn2", t1, part)
        t2, part = self.conv(p + ".conv2.conv", t1, pro=c2, stats=True)
        c3 = self.bn(p + ".bn3", t2, part)
        if cin != cout:
            r = self.conv(p + ".skip_layer.conv", x)
            out, part = self.conv(p + ".conv3.conv", t2, pro=c3, res=r, out=r, stats=True)
        else:
            out, part = self.conv(p + ".conv3.conv", t2, pro=c3, res=x, stats=True)
        self.save(p, (x, t1, t2))
        self.give_part(out, part)
        return out

    def hourglass(self, p, n, x):
        """models/base/layers.py:104-111."""
        up1 = self.residual(p + ".up1", x)
        part = self.stat_buffer((x.shape[0], x.shape[1], x.shape[2] // 2, x.shape[3] // 2))
        pl = Kn.maxpool2x2(x, stat_part=part)
        self.give_part(pl, part)
        low1 = self.residual(p + ".low1", pl)
        low2 = self.hourglass(p + ".low2", n - 1, low1) if n > 1 else self.residual(p + ".low2", low1)
        low3 = self.residual(p + ".low3", low2)
        if _SAVE_LOW3 in ("1", "clone"):                 # diagnostic: the residual's output before the add
            self.save(p + ".low3_out", low3.clone() if _SAVE_LOW3 == "clone" else low3)
        self.save(p, x)
        part = self.stat_buffer(up1.shape)
        if _UPADD_OOP:                                   # diagnostic: up1 kept, the sum in a new tensor
            self.save(p + ".up1_out", up1)
            out = Kn.upsample2x_add(up1, low3, stat_part=part)
            self.give_part(out, part)
            return out
        if _SAVE_LOW3 == "add":                          # diagnostic: both operands and the result, cloned
            self.save(p + ".add_in", (up1.clone(), low3.clone()))
        out = Kn.upsample2x_add(up1, low3, out=up1, stat_part=part)
        if _SAVE_LOW3 == "add":
            self.save(p + ".add_out", out.clone())
        self.give_part(out, part)
        return out

    # ---- backward
    def _coef(self):
        return self.bcoef if self.bcoef is not None else self.m._ws[("coef", self.B)]

    def G(self, name):
        s, n, shp = self.m._offs[name]
        return self.gbuf[s:s + n].view(shp)

    def bn_bwd(self, name, dz, x, relu, add1=None, add2=None, out=None, part=None):
        """part: the backward partials dz's producer wrote (None: a statistics pass)."""
        sc, sh, mu, istd = self.bnc(name)
        return Kn.bn_backward(dz, x, self.m.P(name + ".weight"), mu, istd, sc, sh, relu, self.bpart, self._coef(),
                              self.G(name + ".weight"), self.G(name + ".bias"), add1=add1, add2=add2, out=out,
                              part=part)

    def bn_bwd_split(self, name, dz, x, relu, part=None, pieces=None, grads=True):
        """dx as the split operand (pieces: the consumer's; 2 = 2xfp16 with its device-side
        scale); grads=False: the BN's own parameter gradients not accumulated (a second
        pass over the same dz)."""
        sc, sh, mu, istd = self.bnc(name)
        return Kn.bn_backward_split(dz, x, self.m.P(name + ".weight"), mu, istd, sc, sh, relu, self.bpart,
                                    self._coef(), self.G(name + ".weight") if grads else None,
                                    self.G(name + ".bias") if grads else None,
                                    self.m.bwd_pieces if pieces is None else pieces, 1, part=None if not grads else part)

    def wgrad(self, name, dy, x, KS, stride=1, pro=None):
        ps, ph = (None, None) if pro is None else pro
        if KS == 1 and self.m.bwd_pieces in (1, 3) and _WGRAD1_SPLIT and Kn.wgrad1x1_split_load_ok(dy, x):
            Kn.conv2d_wgrad1x1_split_load(dy, x, self.G(name + ".weight"), self.G(name + ".bias"), ps, ph,
                                          accumulate=True, npieces=self.m.bwd_pieces)
            return
        Kn.conv2d_wgrad(dy, x, KS, stride, self.G(name + ".weight"), self.G(name + ".bias"), ps, ph,
                        accumulate=True)

    def bwd_epi(self, bn, x):
        """(bwd argument, partials buffer): the data-gradient epilogue writes the
        backward statistics partials of BN `bn` (input x) — None off the path."""
        if not self.train or bn is None or not _BWD_EPI:
            return None, None
        part = Kn.bn_partial_buffer(x.shape[1], x.shape[0] * x[0, 0].numel(), x.device)
        return (x, self.bnc(bn)[0], 1, part), part

    def dgrad(self, name, dy, res=None, out=None, bnb=None):
        """bnb = (bn, x): the result is dz of BN bn (input x) — returns (dx, its
        backward partials or None); else dx."""
        ws = self.m.SW(1, name + ".weight")
        if ws is not None and ws.npieces in (1, 3) and ws.shape[1] == 1:
            if Kn.conv1x1_split_load_ok(dy, ws, small=self.m.conv_pieces == 2):
                bwd, part = self.bwd_epi(*(bnb or (None, None))) if ws.npieces == 3 else (None, None)
                y = Kn.conv1x1_forward_split_load(dy, ws, None, res=res, out=out, bwd=bwd)
                return (y, part) if bnb is not None else y
            if ws.npieces == 3:
                ws = None
        if bnb is not None:
            return self.dgrad(name, dy, res=res, out=out), None
        if ws is not None:
            if ws.npieces in (1, 3):
                ys = Kn.split_activation(dy, ws.npieces, (ws.shape[1] == 9) * 1)
                return Kn.conv2d_forward_psa(ys, ws, None, res=res, out=out)
            return Kn.conv2d_forward_split(dy, ws, None, res=res, out=out)
        w = self.m.P(name + ".weight")
        if w.shape[2] == 1 and Kn.conv1x1_kmajor_ok(dy, w.shape[1]):
            return Kn.conv1x1_forward_kmajor(dy, w, None, res=res, out=out)     # [Cout][Cin] = k-major
        return Kn.conv2d_dgrad(dy, None, res=res, out=out, wt=self.m.W(1, name + ".weight"))

    def residual_bwd(self, p, dout):
        x, t1, t2 = self.saved.get(p)
        cin = x.shape[1]
        cout = dout.shape[1]
        c1 = self.bnc(p + ".bn1")[:2]
        c2 = self.bnc(p + ".bn2")[:2]
        c3 = self.bnc(p + ".bn3")[:2]
        self.wgrad(p + ".conv3.conv", dout, t2, 1, pro=c3)
        d, part = self.dgrad(p + ".conv3.conv", dout, bnb=(p + ".bn3", t2))   # d relu(bn3(t2))
        ws = self.m.SW(1, p + ".conv2.conv.weight")
        xs = self.saved_split.get(p + ".conv2.conv")
        cb = 64 if _WGRAD3_64 else 128
        split_wgrad = (ws is not None and ws.npieces in (1, 2, 3) and xs is not None and t2.shape[1] % cb == 0
                       and xs.C % cb == 0 and t2.shape[3] % 16 == 0 and xs.npieces == ws.npieces)
        bwd2, part2 = self.bwd_epi(p + ".bn2", t1)
        if ws is not None and ws.npieces == 2:
            bwd2, part2 = None, None                                   # (no epilogue partials on 2xfp16)
        if split_wgrad:
            # d t2 only as the split operand both conv2 gradients read
            ys = self.bn_bwd_split(p + ".bn3", d, t2, relu=1, part=part, pieces=ws.npieces)
            Kn.conv2d_wgrad3_psa(ys, xs, self.G(p + ".conv2.conv.weight"), self.G(p + ".conv2.conv.bias"))
            d = Kn.conv2d_forward_psa(ys, ws, None, bwd=bwd2)         # d relu(bn2(t1))
        elif ws is not None and ws.npieces in (1, 2, 3):
            ys = None
            if ws.npieces == 2:
                # the data gradient's 2xfp16 operand with its bound-derived scale, from a second
                # statistics pass over the same dz (the BN's parameter gradients accumulate once, below)
                ys = self.bn_bwd_split(p + ".bn3", d, t2, relu=1, pieces=2, grads=False)
            d = self.bn_bwd(p + ".bn3", d, t2, relu=1, part=part)     # d t2
            self.wgrad(p + ".conv2.conv", d, t1, 3, pro=c2)
            d = Kn.conv2d_forward_psa(ys if ys is not None else Kn.split_activation(d, ws.npieces, 1), ws, None,
                                      bwd=bwd2)
        else:
            d = self.bn_bwd(p + ".bn3", d, t2, relu=1, part=part)     # d t2
            self.wgrad(p + ".conv2.conv", d, t1, 3, pro=c2)
            d = self.dgrad(p + ".conv2.conv", d)                       # d relu(bn2(t1))
            part2 = None
        d = self.bn_bwd(p + ".bn2", d, t1, relu=1, part=part2)        # d t1
        self.wgrad(p + ".conv1.conv", d, x, 1, pro=c1)
        d, part = self.dgrad(p + ".conv1.conv", d, bnb=(p + ".bn1", x))   # d relu(bn1(x))
        if cin != cout:
            self.wgrad(p + ".skip_layer.conv", dout, x, 1)
            ds = self.dgrad(p + ".skip_layer.conv", dout)
            return self.bn_bwd(p + ".bn1", d, x, relu=1, add1=ds, part=part)
        return self.bn_bwd(p + ".bn1", d, x, relu=1, add1=dout, part=part)

    def hourglass_bwd(self, p, n, dout):
        x = self.saved.get(p)
        B, C, H, W = dout.shape
        dlow3 = torch.empty((B, C, H // 2, W // 2), device=self.dev)
        Kn.upsample2x_add_backward(dout, dlow3, accumulate=False)
        dlow2 = self.residual_bwd(p + ".low3", dlow3)
        dlow1 = self.hourglass_bwd(p + ".low2", n - 1, dlow2) if n > 1 else self.residual_bwd(p + ".low2", dlow2)
        dpl = self.residual_bwd(p + ".low1", dlow1)
        dx = self.residual_bwd(p + ".up1", dout)
        Kn.maxpool2x2_backward(x, dpl, dx, accumulate=True)
        return dx

    def backward(self, dpreds, dfeats):
        m = self.m
        S = m.nStack
        # the data-gradient weights (mode 1) were laid out by the forward
        # (_forward_impl) and the weights are unchanged since: no re-layout
        # here, which would rewrite them while a concurrent pass of the same
        # network (a second view on the teacher's stream) reads them
        dpreds = dpreds.contiguous()
        if dfeats is not None:
            dfeats = dfeats.contiguous()
        dxn = None                                       # grad of the x entering stack i+1
        for i in reversed(range(S)):
            f, pr = self.saved.get("stack.%d" % i)
            dpi = dpreds[:, i].contiguous()
            if i < S - 1:
                nmf, nmp = "merge_features.%d.conv.conv" % i, "merge_preds.%d.conv.conv" % i
                self.wgrad(nmf, dxn, f, 1)
                self.wgrad(nmp, dxn, pr, 1)
                dpi = self.dgrad(nmp, dxn, res=dpi, out=dpi)
            npd = "preds.%d.conv" % i
            self.wgrad(npd, dpi, f, 1)
            df = self.dgrad(npd, dpi)
            if i < S - 1:
                df = self.dgrad(nmf, dxn, res=df, out=df)
            if dfeats is not None:
                dfi = dfeats[:, i].contiguous()
                if m.mode == "AvgPool":
                    Kn.avgpool2x2_backward(dfi, df, accumulate=True)
                else:
                    Kn.maxpool2x2_backward(f, dfi, df, accumulate=True)
            f0, yf = self.saved.get("features.%d.1" % i)
            d = self.bn_bwd("features.%d.1.bn" % i, df, yf, relu=1)
            self.wgrad("features.%d.1.conv" % i, d, f0, 1)
            d = self.dgrad("features.%d.1.conv" % i, d)
            d = self.residual_bwd("features.%d.0" % i, d)
            dx = self.hourglass_bwd("hgs.%d.0" % i, 4, d)
            if dxn is not None:
                dx = Kn.add(dx, dxn, out=dx)
            dxn = dx
        d = self.residual_bwd("pre.4", dxn)
        d = self.residual_bwd("pre.3", d)
        x1 = self.saved.get("pre.2")
        dx1 = torch.empty_like(x1)                       # (even H, W: every element written)
        Kn.maxpool2x2_backward(x1, d, dx1, accumulate=False)
        d = self.residual_bwd("pre.1", dx1)
        imgs, y0 = self.saved.get("pre.0")
        xs = self.saved_split.get("pre.0.conv")
        w0 = m.P("pre.0.conv.weight")
        if xs is not None and m.bwd_pieces in (1, 3) and d.shape[1] % 64 == 0 and d.shape[3] % 16 == 0:
            # dy of the stem only as the split operand of its weight gradient (the input
            # image takes no gradient): the space-to-depth 4x4 weight gradient, mapped to 7x7
            ys = self.bn_bwd_split("pre.0.bn", d, y0, relu=1)
            if Kn.wgrad_stem_psa_ok(ys, xs, w0):
                Kn.conv2d_wgrad_stem_psa(ys, xs, self.G("pre.0.conv.weight"), self.G("pre.0.conv.bias"))
                return
            raise RuntimeError("ubpl_amd: stem weight gradient operands %s / %s" % (
                (ys.B, ys.C, ys.H, ys.W, ys.pad), (xs.B, xs.C, xs.H, xs.W, xs.pad)))
        d = self.bn_bwd("pre.0.bn", d, y0, relu=1)
        self.wgrad("pre.0.conv", d, imgs, 7, stride=2)


def pose_model(modelType, kpsCount, mode="default", nograd=False):
    """models/pose/pose_model.py:5-13 ('HG<n>' only; LitePose is out of scope)."""
    if "HG" not in modelType:
        raise ValueError("only HG<n> models are on the HIP path (got %r)" % modelType)
    model = StackedHourglass(kpsCount, int(modelType[len("HG"):]), mode)
    if nograd:
        for p in model.parameters():
            p.detach_()
    return model


PoseModel = pose_model


def hg(k, nStack=3, mode="default", nograd=False):
    """models/pose/hourglass.py:102-107."""
    return pose_model("HG%d" % nStack, k, mode, nograd)
