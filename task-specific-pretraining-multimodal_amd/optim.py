"""FusedAdam — torch.optim.Adam semantics on one HBM-bound HIP kernel over a flat parameter buffer.

Replaces the ``torch.optim.Adam`` that MML_Suite builds at config/optimizer_config.py:199-226
(resolver config/resolvers.py:125-156) and steps at models/avmnist.py:303: L2 weight decay folded
into the gradient, betas (0.9, 0.999), eps 1e-8, bias-corrected step size.  At construction every
parameter of a group is moved into one 16-byte-aligned flat fp32 buffer (conv weights keep their
OHWI/channels_last layout inside it) and re-pointed as a view; ``.grad`` becomes a view of a flat
gradient buffer the HIP backward writes directly.  One ``tspm_adam_step`` launch then updates the
whole group (28 B/param of HBM traffic).  The step counter lives on the device so a captured HIP
graph advances the bias correction on every replay.  ``state_dict()`` has torch.optim.Adam's
format (``step`` / ``exp_avg`` / ``exp_avg_sq`` per parameter).
"""
from __future__ import annotations

import ctypes
from typing import Any, Dict, List, Optional

import torch

from . import _lib as L

_ALIGN = 4  # floats (16 bytes)


def _layout_of(p: torch.Tensor) -> torch.memory_format:
    return torch.channels_last if p.dim() == 4 else torch.contiguous_format


def _view(flat: torch.Tensor, off: int, p: torch.Tensor) -> torch.Tensor:
    n = p.numel()
    sl = flat[off:off + n]
    if p.dim() == 4:
        o, i, h, w = p.shape
        return sl.view(o, h, w, i).permute(0, 3, 1, 2)
    return sl.view(p.shape)


class _FlatGroup:
    def __init__(self, params: List[torch.Tensor], device: torch.device):
        self.params = params
        self.offsets = []
        off = 0
        for p in params:
            self.offsets.append(off)
            off += (p.numel() + _ALIGN - 1) // _ALIGN * _ALIGN
        self.numel = off
        f32 = dict(device=device, dtype=torch.float32)
        self.param = torch.zeros(off, **f32)
        self.grad = torch.zeros(off, **f32)
        self.exp_avg = torch.zeros(off, **f32)
        self.exp_avg_sq = torch.zeros(off, **f32)
        self.hyper = torch.zeros(8, dtype=torch.float64, device=device)  # tspm_adam_hyper (64 bytes)
        self.host_hyper = torch.zeros(8, dtype=torch.float64)
        if torch.cuda.is_available():
            self.host_hyper = self.host_hyper.pin_memory()
        self.grad_views = []
        for p, o in zip(params, self.offsets):
            v = _view(self.param, o, p)
            v.copy_(p.detach())
            p.data = v
            g = _view(self.grad, o, p)
            self.grad_views.append(g)
            p.grad = g
        self.step = 0
        self.last_written = None


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 amsgrad: bool = False, *, maximize: bool = False, foreach=None, capturable: bool = False,
                 differentiable: bool = False, fused=None, grad_scale: float = 1.0):
        if amsgrad or maximize or differentiable:
            raise NotImplementedError("FusedAdam: amsgrad / maximize / differentiable are not on the AVMNIST path")
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=None)
        super().__init__(params, defaults)
        self.grad_scale = float(grad_scale)
        # device scalar multiplying every gradient in the update (the clip_grad_norm_ coefficient written
        # by tspm_grad_clip_coef; None = no clip) — set by the MOSI step (utt_fusion.py:188-190)
        self.clip_coef: Optional[torch.Tensor] = None
        self._flat: List[_FlatGroup] = []
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.requires_grad]
            if not ps:
                self._flat.append(None)
                continue
            dev = ps[0].device
            if dev.type != "cuda":
                raise L.TspmError("FusedAdam runs on the MI355X: create it after model.to('cuda')")
            if any(p.device != dev for p in ps):
                raise L.TspmError("FusedAdam: all parameters of a group must be on one device")
            fg = _FlatGroup(ps, dev)
            self._flat.append(fg)
            for p, o in zip(ps, fg.offsets):
                self.state[p] = {"step": torch.tensor(0.0), "exp_avg": _view(fg.exp_avg, o, p),
                                 "exp_avg_sq": _view(fg.exp_avg_sq, o, p)}

    # -- helpers used by the fused train step -------------------------------------------------------
    def flat_groups(self) -> List[_FlatGroup]:
        return [f for f in self._flat if f is not None]

    def _write_hyper(self, group: Dict[str, Any], fg: _FlatGroup) -> None:
        b1, b2 = group["betas"]
        vals = (float(group["lr"]), float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]),
                self.grad_scale)
        if fg.last_written == vals:
            return
        for i, v in enumerate(vals):
            fg.host_hyper[i] = v
        # only the 6 double fields: the step counter (word 6, int64) is device-owned
        fg.hyper[:6].copy_(fg.host_hyper[:6], non_blocking=True)
        fg.last_written = vals

    def sync_hyper(self) -> None:
        """Push lr/betas/eps/wd to the device (call before replaying a captured step)."""
        for group, fg in zip(self.param_groups, self._flat):
            if fg is not None:
                self._write_hyper(group, fg)

    def launch(self, stream_handle: int) -> None:
        """Enqueue step-count increment + fused update for every group (capturable)."""
        lib = L.lib()
        for fg in self.flat_groups():
            L.check(lib.tspm_adam_begin(fg.hyper.data_ptr(), stream_handle), "adam_begin")
            if self.clip_coef is not None:
                L.check(lib.tspm_adam_step_clip(fg.numel, fg.param.data_ptr(), fg.grad.data_ptr(), fg.exp_avg.data_ptr(),
                                                fg.exp_avg_sq.data_ptr(), fg.hyper.data_ptr(),
                                                self.clip_coef.data_ptr(), stream_handle), "adam_step_clip")
                continue
            L.check(lib.tspm_adam_step(fg.numel, fg.param.data_ptr(), fg.grad.data_ptr(), fg.exp_avg.data_ptr(),
                                       fg.exp_avg_sq.data_ptr(), fg.hyper.data_ptr(), stream_handle), "adam_step")

    def launch_begin(self, stream_handle: int) -> None:
        """Enqueue the device step-count increment of every group (before launch_ranges)."""
        lib = L.lib()
        for fg in self.flat_groups():
            L.check(lib.tspm_adam_begin(fg.hyper.data_ptr(), stream_handle), "adam_begin")

    def launch_ranges(self, stream_handle: int, ranges) -> None:
        """Enqueue the fused update over element ranges [a, b) of each group's flat buffers
        (``ranges[i]`` for group i; ranges start at parameter offsets, so they are 16-byte aligned).
        Adam is element-wise: any partition of the buffer gives bitwise the result of ``launch``."""
        lib = L.lib()
        for fg, rs in zip(self.flat_groups(), ranges):
            for a, b in rs:
                L.check(lib.tspm_adam_step(b - a, fg.param[a:].data_ptr(), fg.grad[a:].data_ptr(),
                                           fg.exp_avg[a:].data_ptr(), fg.exp_avg_sq[a:].data_ptr(),
                                           fg.hyper.data_ptr(), stream_handle), "adam_step(range)")

    def note_steps(self, k: int = 1) -> None:
        for fg in self.flat_groups():
            fg.step += k
            for p in fg.params:
                self.state[p]["step"].fill_(float(fg.step))

    def _regather_grads(self) -> None:
        # autograd may have replaced .grad (zero_grad(set_to_none) + AccumulateGrad): fold back
        for fg in self.flat_groups():
            for p, g in zip(fg.params, fg.grad_views):
                if p.grad is None:
                    g.zero_()
                    p.grad = g
                elif p.grad.data_ptr() != g.data_ptr():
                    g.copy_(p.grad)
                    p.grad = g

    # -- torch.optim.Optimizer API -------------------------------------------------------------------
    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._regather_grads()
        self.sync_hyper()
        self.launch(L.stream_handle())
        self.note_steps(1)
        return loss

    def zero_grad(self, set_to_none: bool = True) -> None:
        # flat gradient views stay in place (the HIP backward writes them); zero instead of None
        for fg in self.flat_groups():
            fg.grad.zero_()
            for p, g in zip(fg.params, fg.grad_views):
                p.grad = g

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        super().load_state_dict(state_dict)
        for fg in self.flat_groups():
            steps = []
            for p, o in zip(fg.params, fg.offsets):
                st = self.state[p]
                m_view, v_view = _view(fg.exp_avg, o, p), _view(fg.exp_avg_sq, o, p)
                if "exp_avg" in st:
                    m_view.copy_(st["exp_avg"])
                    v_view.copy_(st["exp_avg_sq"])
                step = float(st.get("step", torch.tensor(0.0)))
                steps.append(step)
                self.state[p] = {"step": torch.tensor(step), "exp_avg": m_view, "exp_avg_sq": v_view}
            fg.step = int(max(steps)) if steps else 0
            fg.hyper.view(torch.int64)[6:7].fill_(fg.step)
            fg.last_written = None
