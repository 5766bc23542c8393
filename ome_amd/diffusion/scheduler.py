"""Flow-matching Euler sampler of the Qwen-Image pipelines (diffusers
``FlowMatchEulerDiscreteScheduler`` with the Qwen-Image ``scheduler_config.json``: dynamic
exponential time shift from the image token count, terminal stretch, Euler steps on the velocity).

The model predicts the velocity v = noise - x0 at sigma; one Euler step moves the latents from
sigma_i to sigma_{i+1}: x <- x + (sigma_{i+1} - sigma_i) * v.  The schedule is a host-side list;
the steps themselves are one fused elementwise kernel each on the device.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch


@dataclass
class FlowMatchConfig:
    num_train_timesteps: int = 1000
    use_dynamic_shifting: bool = True
    base_image_seq_len: int = 256
    max_image_seq_len: int = 8192
    base_shift: float = 0.5
    max_shift: float = 0.9
    shift: float = 1.0
    shift_terminal: float | None = 0.02
    time_shift_type: str = "exponential"

    @classmethod
    def from_dict(cls, d: dict | None) -> "FlowMatchConfig":
        d = d or {}
        return cls(**{k: d[k] for k in cls.__dataclass_fields__ if k in d})


def calculate_shift(seq_len: int, c: FlowMatchConfig) -> float:
    """mu: linear in the image token count between (base_len, base_shift) and (max_len, max_shift)."""
    m = (c.max_shift - c.base_shift) / (c.max_image_seq_len - c.base_image_seq_len)
    return seq_len * m + (c.base_shift - m * c.base_image_seq_len)


def sigmas_for(steps: int, seq_len: int, c: FlowMatchConfig) -> np.ndarray:
    """[steps + 1] float64 sigmas (last = 0) for ``steps`` Euler steps at ``seq_len`` image tokens."""
    s = np.linspace(1.0, 1.0 / steps, steps, dtype=np.float64)
    if c.use_dynamic_shifting:
        mu = calculate_shift(seq_len, c)
        if c.time_shift_type == "exponential":
            s = math.exp(mu) / (math.exp(mu) + (1.0 / s - 1.0))
        else:   # linear
            s = mu / (mu + (1.0 / s - 1.0))
    elif c.shift != 1.0:
        s = c.shift * s / (1 + (c.shift - 1) * s)
    if c.shift_terminal:
        one_minus = 1.0 - s
        s = 1.0 - one_minus / (one_minus[-1] / (1.0 - c.shift_terminal))
    return np.concatenate([s, [0.0]])


class FlowMatchEuler:
    def __init__(self, cfg: FlowMatchConfig | None = None):
        self.cfg = cfg or FlowMatchConfig()
        self.sigmas = np.zeros(1)

    def set_timesteps(self, steps: int, seq_len: int) -> list[float]:
        """-> model timesteps (sigma * 1000) of the ``steps`` evaluations."""
        self.sigmas = sigmas_for(steps, seq_len, self.cfg)
        return [float(v) * self.cfg.num_train_timesteps for v in self.sigmas[:-1]]

    def step(self, v: torch.Tensor, i: int, x: torch.Tensor) -> torch.Tensor:
        """x at sigma_i -> x at sigma_{i+1} (fp32 accumulation, result in x's dtype)."""
        dt = float(self.sigmas[i + 1] - self.sigmas[i])
        return (x.float() + dt * v.float()).to(x.dtype)
