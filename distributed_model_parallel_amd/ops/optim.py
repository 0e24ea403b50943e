"""FlatSGD: torch.optim.SGD semantics, one HIP launch per dtype group.

Works on the flat parameter / gradient buffers of
``DistributedDataParallel(..., flat_parameters=True)``: gradients there are
already RCCL-averaged bucket views, parameters are views of a flat buffer with
the same layout, so the update of all 161 ResNet-50 tensors is a single
vectorised pass (``csrc/optim/fused_sgd.hip``).  bf16 parameter groups keep an
fp32 master copy and fp32 momentum inside the optimizer; the kernel writes the
bf16 working weights back in the same pass.

Reference parity: SGD(lr, momentum 0.9, weight_decay 1e-4) at
``model_parallel.py:105`` / ``data_parallel.py:90``.
"""
from __future__ import annotations

from typing import List, Optional

import torch

from .. import _native
from . import wgrad_stream, wt_cache



class ForeignOptimizerState(ValueError):
    """The state dict was written by another optimizer class (e.g. a
    torch.optim.SGD state from an older DataParallel run): nothing in it maps
    onto this optimizer.  ``load_checkpoint`` tolerates only this case; a
    layout mismatch of our own format stays a hard error."""

class FlatSGD(torch.optim.Optimizer):
    def __init__(self, ddp, lr: float, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, master_weights: bool = True):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        params = list(ddp._params)
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov)
        super().__init__(params, defaults)
        self.ddp = ddp
        self.master_weights = master_weights
        self._version = -1
        self._flat_state: List[dict] = []
        self._steps = 0

    # ------------------------------------------------------------------ #
    def _ensure_state(self) -> None:
        if self._version == self.ddp.layout_version:
            return
        groups = self.ddp.flat_groups()
        old = self._flat_state
        old_layout = getattr(self.ddp, "_last_old_layout", None)
        new_state = []
        for pflat, gflat in groups:
            st = {"param": pflat, "grad": gflat}
            if pflat.dtype != torch.float32 and self.master_weights:
                st["master"] = pflat.float()
            st["momentum"] = torch.zeros(pflat.numel(), dtype=torch.float32, device=pflat.device)
            new_state.append(st)
        if old and old_layout is not None:
            self._remap(old, new_state, old_layout, self.ddp.param_layout())
        self._flat_state = new_state
        self._version = self.ddp.layout_version

    @torch.no_grad()
    def _remap(self, old, new, old_layout, new_layout) -> None:
        """Carry momentum / master buffers across a bucket rebuild."""
        for p, (og, oo), (ng, no) in zip(self.ddp._params, old_layout, new_layout):
            n = p.numel()
            for key in ("momentum", "master"):
                if key in old[og] and key in new[ng]:
                    new[ng][key].narrow(0, no, n).copy_(old[og][key].narrow(0, oo, n))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._ensure_state()
        g = self.param_groups[0]
        first = self._steps == 0
        if self._flat_state and self._flat_state[0]["param"].is_cuda:
            wgrad_stream.join(self._flat_state[0]["param"].device)  # gradients from the side stream
        for st in self._flat_state:
            pflat, gflat = st["param"], st["grad"]
            master = st.get("master")
            if pflat.is_cuda:
                _native.require("FlatSGD").sgd_flat_step(
                    master, st["momentum"], gflat, pflat, float(g["lr"]), float(g["weight_decay"]),
                    float(g["momentum"]), float(g["dampening"]), bool(g["nesterov"]), 1.0, first)
            else:
                _sgd_reference(master, st["momentum"], gflat, pflat, g, first)
        self._steps += 1
        # the updated weights' W^T, one launch (ops/wt_cache.py)
        wt_cache.after_optimizer_step(p for grp in self.param_groups for p in grp["params"])
        return loss

    def zero_grad(self, set_to_none: bool = False):
        self.ddp.zero_grad()

    @torch.no_grad()
    def sync_from_params(self) -> None:
        """Re-seed the fp32 masters from the current working weights (weights
        loaded behind the optimizer's back, e.g. a checkpoint without optimizer
        state); otherwise the next step would write the stale masters back."""
        for st in self._flat_state:
            if "master" in st:
                st["master"].copy_(st["param"])

    def state_dict(self):
        self._ensure_state()
        return {"steps": self._steps, "param_groups": [{k: v for k, v in g.items() if k != "params"}
                                                       for g in self.param_groups],
                "flat_state": [{k: v for k, v in st.items() if k in ("momentum", "master")}
                               for st in self._flat_state],
                "layout": self.ddp.param_layout()}

    def load_state_dict(self, sd):
        """Restore momentum / master weights parameter by parameter.

        The saved flats follow the bucket layout of the run that wrote them
        (usually the post-rebuild autograd-ready order), while a fresh DDP
        starts in registration order -- so every parameter's slice is moved
        from ``sd['layout']`` to the current layout, never copied flat-to-flat.
        """
        if "layout" not in sd or "flat_state" not in sd:
            raise ForeignOptimizerState("FlatSGD.load_state_dict: not a FlatSGD state (e.g. a "
                                        "torch.optim.SGD state dict)")
        self._ensure_state()
        self._steps = sd["steps"]
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            g.update(sg)
        dev = self._flat_state[0]["momentum"].device if self._flat_state else None
        saved = [{k: v.to(dev) for k, v in sst.items()} for sst in sd["flat_state"]]
        old_layout = [tuple(int(v) for v in e) for e in sd["layout"]]
        if len(old_layout) != len(self.ddp._params):
            raise ValueError("FlatSGD.load_state_dict: checkpoint has %d parameters, model has %d"
                             % (len(old_layout), len(self.ddp._params)))
        self._remap(saved, self._flat_state, old_layout, self.ddp.param_layout())
        with torch.no_grad():
            for st in self._flat_state:
                if "master" in st:  # working weights follow the restored fp32 master
                    st["param"].copy_(st["master"].to(st["param"].dtype))


class MasterSGD(torch.optim.Optimizer):
    """torch.optim.SGD semantics with fp32 master weights for ANY parameter list.

    Used where there is no DDP flat layout to borrow: single-process
    DataParallel (its parameters live on ``device_ids[0]``), pipeline stages
    and plain single-GPU training.  At construction the parameters of each
    dtype/device group are moved into one flat buffer (parameters become
    views, channels-last strides preserved) and their ``.grad`` is pre-set to
    views of a flat gradient buffer, so autograd accumulates in place and the
    update is ONE ``sgd_flat_step`` launch per group, fp32 master + fp32
    momentum for bf16 groups (bf16 SGD would drop every update below one
    bf16 ulp).  Same kernel and numerics as :class:`FlatSGD` under DDP, so DP,
    pipeline and DDP train at equal precision.
    """

    def __init__(self, params, lr: float, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, master_weights: bool = True):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        params = [p for p in params if p.requires_grad]
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov)
        super().__init__(params, defaults)
        self.master_weights = master_weights
        self._steps = 0
        self._groups = []
        by_key = {}
        for p in params:
            by_key.setdefault((p.dtype, p.device), []).append(p)
        with torch.no_grad():
            for (dt, dev), ps in by_key.items():
                offs, o = [], 0
                for p in ps:
                    offs.append(o)
                    o += (p.numel() + 7) // 8 * 8  # kernel works in 8-element vectors
                pflat = torch.zeros(o, dtype=dt, device=dev)
                gflat = torch.zeros(o, dtype=dt, device=dev)
                gviews = []
                for p, off in zip(ps, offs):
                    view = pflat.as_strided(p.shape, p.stride(), off)
                    view.copy_(p.detach())
                    p.data = view
                    gv = gflat.as_strided(p.shape, p.stride(), off)
                    p.grad = gv
                    gviews.append(gv)
                st = {"params": ps, "offs": offs, "param": pflat, "grad": gflat, "gviews": gviews,
                      "momentum": torch.zeros(o, dtype=torch.float32, device=dev)}
                if dt != torch.float32 and master_weights:
                    st["master"] = pflat.float()
                self._groups.append(st)

    @torch.no_grad()
    def _adopt_grads(self, st) -> None:
        """Grads replaced behind our back (set_to_none, a stolen tensor) go back into the flat."""
        for p, gv in zip(st["params"], st["gviews"]):
            g = p.grad
            if g is gv or (g is not None and g.data_ptr() == gv.data_ptr() and g.stride() == gv.stride()):
                continue
            if g is None:
                gv.zero_()
            else:
                gv.copy_(g)
            p.grad = gv

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        g = self.param_groups[0]
        first = self._steps == 0
        if self._groups and self._groups[0]["param"].is_cuda:
            wgrad_stream.join(self._groups[0]["param"].device)  # gradients from the side stream
        for st in self._groups:
            self._adopt_grads(st)
            pflat, gflat, master = st["param"], st["grad"], st.get("master")
            if pflat.is_cuda:
                _native.require("MasterSGD").sgd_flat_step(
                    master, st["momentum"], gflat, pflat, float(g["lr"]), float(g["weight_decay"]),
                    float(g["momentum"]), float(g["dampening"]), bool(g["nesterov"]), 1.0, first)
            else:
                _sgd_reference(master, st["momentum"], gflat, pflat, g, first)
        self._steps += 1
        # the updated weights' W^T, one launch (ops/wt_cache.py)
        wt_cache.after_optimizer_step(p for grp in self.param_groups for p in grp["params"])
        return loss

    def zero_grad(self, set_to_none: bool = False):
        """One fill per group; gradients stay flat views (``set_to_none`` is ignored)."""
        for st in self._groups:
            st["grad"].zero_()
            for p, gv in zip(st["params"], st["gviews"]):
                if p.grad is not gv:
                    p.grad = gv

    @torch.no_grad()
    def sync_from_params(self) -> None:
        """Re-seed the fp32 masters from the current working weights.  The masters
        are snapshotted at construction, so weights loaded afterwards without
        optimizer state (the reference's {'net','acc','epoch'} checkpoints, a
        plain ``model.load_state_dict``) must be adopted here, or the first step
        would overwrite them with the init weights."""
        for st in self._groups:
            if "master" in st:
                st["master"].copy_(st["param"])

    def state_dict(self):
        return {"steps": self._steps,
                "param_groups": [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups],
                "numels": [[p.numel() for p in st["params"]] for st in self._groups],
                "flat_state": [{k: st[k] for k in ("momentum", "master") if k in st}
                               for st in self._groups]}

    def load_state_dict(self, sd):
        if "numels" not in sd or "flat_state" not in sd:
            raise ForeignOptimizerState("MasterSGD.load_state_dict: not a MasterSGD state (e.g. a "
                                        "torch.optim.SGD state dict)")
        if sd["numels"] != [[p.numel() for p in st["params"]] for st in self._groups]:
            raise ValueError("MasterSGD.load_state_dict: parameter layout differs from the checkpoint")
        self._steps = sd["steps"]
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            g.update(sg)
        with torch.no_grad():
            for st, sst in zip(self._groups, sd["flat_state"]):
                for k, v in sst.items():
                    if k in st:
                        st[k].copy_(v)
                if "master" in st:
                    st["param"].copy_(st["master"].to(st["param"].dtype))


def _sgd_reference(master: Optional[torch.Tensor], mom: torch.Tensor, grad: torch.Tensor,
                   param: torch.Tensor, g: dict, first: bool) -> None:
    """PyTorch implementation of the flat kernel (CPU path / test oracle)."""
    w = master if master is not None else param
    d = grad.float() + g["weight_decay"] * w.float()
    if g["momentum"] != 0:
        if first:
            mom.copy_(d)
        else:
            mom.mul_(g["momentum"]).add_(d, alpha=1 - g["dampening"])
        d = d + g["momentum"] * mom if g["nesterov"] else mom
    w.add_(d.to(w.dtype), alpha=-g["lr"])
    if master is not None:
        param.copy_(master.to(param.dtype))
