"""FlatAdamW — torch.optim.AdamW semantics over a model's flat parameter
buffer, one fused HIP kernel per step (optim.hip).

The reference builds `AdamW(model.parameters(), lr=args.lr,
weight_decay=args.wd)` per student (projects/MT_UBPL.py:48).  Here the
moments are two flat buffers the size of the grad-carrying prefix; the
never-trained skip_layer parameters (which torch skips because their grad
stays None) are outside that prefix and are never touched, exactly as in the
reference.
"""
import torch

from . import kernels as Kn
from .hourglass import StackedHourglass


class FlatAdamW:
    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        if not isinstance(model, StackedHourglass):
            raise TypeError("FlatAdamW needs a ubpl_amd StackedHourglass")
        self.model = model
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        n = model.n_live
        self.exp_avg = torch.zeros(n, device=model.flat_params.device)
        self.exp_avg_sq = torch.zeros(n, device=model.flat_params.device)
        # the step count lives on the device so a captured step graph replays
        # it (ubpl_adamw_step_dev increments it); host reads sync lazily
        self._step_t = torch.zeros((), dtype=torch.int64, device=model.flat_params.device)
        self._coef = torch.zeros(4, device=model.flat_params.device)
        self.param_groups = [{"lr": lr, "betas": betas, "eps": eps, "weight_decay": weight_decay}]

    @property
    def step_count(self):
        return int(self._step_t.item())

    def zero_grad(self, set_to_none=True):
        self.model.flat_grads.zero_()
        self.model.attach_grad_views()

    def step(self):
        g = self.param_groups[0]
        Kn.adamw_step_dev_(self.model.live_params(), self.model.live_grads(), self.exp_avg, self.exp_avg_sq,
                           g["lr"], g["betas"][0], g["betas"][1], g["eps"], g["weight_decay"], self._step_t,
                           self._coef)

    def step_and_ema(self, ema_model, alpha):
        """step() then update_ema_variables(model, ema_model) with this alpha, in
        one pass over the flat buffers (bit-identical to the two calls)."""
        if not isinstance(ema_model, StackedHourglass) or ema_model.n_total != self.model.n_total:
            raise ValueError("step_and_ema: the teacher must be a StackedHourglass of the same architecture")
        g = self.param_groups[0]
        Kn.adamw_ema_step_dev_(self.model.flat_params, self.model.flat_grads, self.exp_avg, self.exp_avg_sq,
                               self.model.n_live, g["lr"], g["betas"][0], g["betas"][1], g["eps"],
                               g["weight_decay"], self._step_t, self._coef, ema_model.flat_params, alpha)

    # -- checkpoints: torch.optim.AdamW's state_dict layout -----------------
    # projects/MT_UBPL.py:97-103 stores optims[b].state_dict() in the
    # checkpoint next to the models' state_dicts (utils/base/comm.py:92-103
    # torch.save).  The state is laid out exactly as torch.optim.AdamW lays it
    # out over model.parameters() (reference order, 454 tensors for HG2): one
    # entry per parameter that has been stepped (the live ones; the dead
    # skip_layer parameters never get a gradient, so torch keeps no state for
    # them either), 'step' a CPU float tensor, group keys from torch itself.
    # Checkpoints interchange both ways with the reference's optimizers.
    def _group_template(self):
        g = self.param_groups[0]
        probe = torch.optim.AdamW([torch.zeros(1, requires_grad=True)], lr=g["lr"], betas=g["betas"], eps=g["eps"],
                                  weight_decay=g["weight_decay"])
        grp = dict(probe.state_dict()["param_groups"][0])
        grp.update({k: v for k, v in g.items()})
        return grp

    def _live_slices(self):
        m = self.model
        for i, (name, _) in enumerate(m.named_parameters()):
            s, n, shp = m._offs[name]
            yield i, s, n, shp, s < m.n_live

    def state_dict(self):
        names = list(self.model.named_parameters())
        grp = self._group_template()
        grp["params"] = list(range(len(names)))
        state = {}
        step = self.step_count
        if step > 0:
            for i, s, n, shp, live in self._live_slices():
                if live:
                    state[i] = {"step": torch.tensor(float(step)),
                                "exp_avg": self.exp_avg[s:s + n].view(shp).clone(),
                                "exp_avg_sq": self.exp_avg_sq[s:s + n].view(shp).clone()}
        return {"state": state, "param_groups": [grp]}

    def load_state_dict(self, sd):
        """Accepts torch.optim.AdamW's layout over model.parameters() (a
        reference checkpoint's optim<b>_state, or this class's state_dict)."""
        groups = sd["param_groups"]
        if len(groups) != 1:
            raise ValueError("FlatAdamW holds one parameter group, the state has %d" % len(groups))
        nparams = sum(1 for _ in self.model.parameters())
        if len(groups[0]["params"]) != nparams:
            raise ValueError("loaded state dict has a group of %d parameters, the model has %d"
                             % (len(groups[0]["params"]), nparams))
        pos = {pid: i for i, pid in enumerate(groups[0]["params"])}
        st = {pos[k]: v for k, v in sd["state"].items()}
        steps = set()
        self.exp_avg.zero_()
        self.exp_avg_sq.zero_()
        for i, s, n, shp, live in self._live_slices():
            e = st.get(i)
            if e is None:
                continue
            if not live:
                raise ValueError("state for parameter %d, which never receives a gradient here" % i)
            if tuple(e["exp_avg"].shape) != tuple(shp):
                raise ValueError("state shape %s for parameter %d of shape %s" % (tuple(e["exp_avg"].shape), i,
                                                                                  tuple(shp)))
            self.exp_avg[s:s + n].copy_(e["exp_avg"].reshape(-1))
            self.exp_avg_sq[s:s + n].copy_(e["exp_avg_sq"].reshape(-1))
            steps.add(int(float(e["step"])))
        if len(steps) > 1:
            raise ValueError("per-parameter step counts differ (%s): one flat step count cannot hold them"
                             % sorted(steps))
        self._step_t.fill_(steps.pop() if steps else 0)
        g = groups[0]
        if g.get("amsgrad") or g.get("maximize"):
            raise ValueError("FlatAdamW runs plain AdamW (amsgrad / maximize unsupported)")
        self.lr, self.betas, self.eps, self.weight_decay = g["lr"], tuple(g["betas"]), g["eps"], g["weight_decay"]
        self.param_groups[0].update(lr=g["lr"], betas=tuple(g["betas"]), eps=g["eps"], weight_decay=g["weight_decay"])
