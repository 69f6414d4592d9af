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

    def state_dict(self):
        return {"state": {"step": self.step_count, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq},
                "param_groups": [dict(self.param_groups[0])]}

    def load_state_dict(self, sd):
        self._step_t.fill_(int(sd["state"]["step"]))
        self.exp_avg.copy_(sd["state"]["exp_avg"])
        self.exp_avg_sq.copy_(sd["state"]["exp_avg_sq"])
        self.param_groups[0].update(sd["param_groups"][0])
