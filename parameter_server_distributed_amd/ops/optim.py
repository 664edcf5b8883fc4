"""Fused parameter-server optimizer (gfx950 kernel ``csrc/kernels/optim.hip``).

One kernel pass per flat shard does: sum of K gradient sources (K = 1 after an RCCL
reduce-scatter, K = #pushes for inbox-style shards) -> scale (1/W) -> SGD / momentum / Adam /
AdamW update of the fp32 master -> bf16 working copy for the all-gather.

Reference parity: ``ParameterServerCore::aggregate_gradients`` applies ``p -= g`` with lr fixed at 1
(src/parameter_server.cpp:77-91, "can add learning rate here" at :87). ``OptimConfig(kind="sgd",
lr=1.0)`` reproduces it; the other kinds match ``torch.optim.SGD/Adam/AdamW`` (tested against them).

Per-step scalars (lr, grad scale, step count, Adam bias corrections) live in a 32-byte device
struct (``OptimDyn``) so a captured hipGraph replays with the current values.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass

import torch

from .. import native

KINDS = {"sgd": 0, "momentum": 1, "adam": 2, "adamw": 3}


@dataclass
class OptimConfig:
    kind: str = "momentum"
    lr: float = 0.1
    momentum: float = 0.9
    dampening: float = 0.0
    nesterov: bool = False
    weight_decay: float = 0.0
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-8
    maximize: bool = False

    def __post_init__(self):
        if self.kind not in KINDS:
            raise ValueError(f"unknown optimizer kind {self.kind!r}; expected one of {sorted(KINDS)}")
        if self.kind == "momentum" and self.momentum == 0.0:
            self.kind = "sgd"

    @property
    def code(self) -> int:
        return KINDS[self.kind]

    @property
    def num_states(self) -> int:
        return {"sgd": 0, "momentum": 1, "adam": 2, "adamw": 2}[self.kind]

    def to_dict(self):
        return asdict(self)


class OptimDyn:
    """Device-resident per-step scalars: ``[lr, grad_scale, bc1, bc2, step, pad x3]`` (32 B)."""

    def __init__(self, device, lr: float, grad_scale: float = 1.0):
        self.t = torch.zeros(8, dtype=torch.int32, device=device)
        self._f = self.t.view(torch.float32)
        self.set(lr=lr, grad_scale=grad_scale)

    def set(self, lr: float | None = None, grad_scale: float | None = None):
        vals = self.t.detach().cpu()
        fv = vals.view(torch.float32)
        if lr is not None:
            fv[0] = lr
        if grad_scale is not None:
            fv[1] = grad_scale
        self.t.copy_(vals)

    @property
    def step(self) -> int:
        return int(self.t[4].item())

    @property
    def lr(self) -> float:
        return float(self._f[0].item())


def fused_apply_(cfg: OptimConfig, dyn: OptimDyn, master: torch.Tensor, grads, state1=None, state2=None,
                 shadow=None, advance: bool = True) -> None:
    """In-place fused update of ``master`` from the sum of ``grads`` (list or tensor)."""
    C = native()
    if isinstance(grads, torch.Tensor):
        grads = [grads]
    if advance:
        C.optim_advance_(dyn.t, cfg.beta1, cfg.beta2)
    C.fused_apply_(master, list(grads), state1, state2, shadow, dyn.t, cfg.code, cfg.momentum, cfg.dampening,
                   cfg.nesterov, cfg.weight_decay, cfg.beta1, cfg.beta2, cfg.eps, cfg.maximize)


def advance_(cfg: OptimConfig, dyn: OptimDyn) -> None:
    native().optim_advance_(dyn.t, cfg.beta1, cfg.beta2)


def apply_no_advance_(cfg: OptimConfig, dyn: OptimDyn, master, grads, state1=None, state2=None, shadow=None):
    fused_apply_(cfg, dyn, master, grads, state1, state2, shadow, advance=False)
