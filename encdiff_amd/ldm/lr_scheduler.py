"""LR multipliers mirroring ldm/lr_scheduler.py (host-side scalars per step)."""
from __future__ import annotations

import numpy as np


class LambdaWarmUpCosineScheduler:
    """lr_scheduler.py:4-35."""

    def __init__(self, warm_up_steps, lr_min, lr_max, lr_start, max_decay_steps, verbosity_interval=0):
        self.lr_warm_up_steps, self.lr_start, self.lr_min, self.lr_max = warm_up_steps, lr_start, lr_min, lr_max
        self.lr_max_decay_steps, self.last_lr, self.verbosity_interval = max_decay_steps, 0.0, verbosity_interval

    def schedule(self, n, **kwargs):
        if n < self.lr_warm_up_steps:
            lr = (self.lr_max - self.lr_start) / self.lr_warm_up_steps * n + self.lr_start
        else:
            t = min((n - self.lr_warm_up_steps) / (self.lr_max_decay_steps - self.lr_warm_up_steps), 1.0)
            lr = self.lr_min + 0.5 * (self.lr_max - self.lr_min) * (1 + np.cos(t * np.pi))
        self.last_lr = lr
        return lr

    def __call__(self, n, **kwargs):
        return self.schedule(n, **kwargs)


class LambdaWarmUpCosineScheduler2:
    """lr_scheduler.py:38-78 (list-configured cycles)."""

    def __init__(self, warm_up_steps, f_min, f_max, f_start, cycle_lengths, verbosity_interval=0):
        assert len(warm_up_steps) == len(f_min) == len(f_max) == len(f_start) == len(cycle_lengths)
        self.lr_warm_up_steps, self.f_start, self.f_min, self.f_max = warm_up_steps, f_start, f_min, f_max
        self.cycle_lengths = cycle_lengths
        self.cum_cycles = np.cumsum([0] + list(cycle_lengths))
        self.last_f, self.verbosity_interval = 0.0, verbosity_interval

    def find_in_interval(self, n):
        for i, cl in enumerate(self.cum_cycles[1:]):
            if n <= cl:
                return i
        return len(self.cycle_lengths) - 1

    def schedule(self, n, **kwargs):
        c = self.find_in_interval(n)
        n = n - self.cum_cycles[c]
        if n < self.lr_warm_up_steps[c]:
            f = (self.f_max[c] - self.f_start[c]) / self.lr_warm_up_steps[c] * n + self.f_start[c]
        else:
            t = min((n - self.lr_warm_up_steps[c]) / (self.cycle_lengths[c] - self.lr_warm_up_steps[c]), 1.0)
            f = self.f_min[c] + 0.5 * (self.f_max[c] - self.f_min[c]) * (1 + np.cos(t * np.pi))
        self.last_f = f
        return f

    def __call__(self, n, **kwargs):
        return self.schedule(n, **kwargs)


class LambdaLinearScheduler(LambdaWarmUpCosineScheduler2):
    """lr_scheduler.py:81-97: linear warm-up, then linear from f_max to f_min over the cycle."""

    def schedule(self, n, **kwargs):
        c = self.find_in_interval(n)
        n = n - self.cum_cycles[c]
        if n < self.lr_warm_up_steps[c]:
            f = (self.f_max[c] - self.f_start[c]) / self.lr_warm_up_steps[c] * n + self.f_start[c]
        else:
            f = self.f_min[c] + (self.f_max[c] - self.f_min[c]) * (self.cycle_lengths[c] - n) / self.cycle_lengths[c]
        self.last_f = f
        return f
