"""LitEma -- mirror of ldm/modules/ema.py:5-76 (buffer names, decay rule,
store/restore/copy_to).

When the tracked model lives in a parameter arena, the shadow buffers become views
of one contiguous fp32 EMA array that the fused HIP AdamW+EMA kernel updates in
the same pass as the optimizer (encdiff_adamw_ema); ``forward`` then only advances
``num_updates``/decay bookkeeping unless called stand-alone.
"""
from __future__ import annotations

import torch
from torch import nn


class LitEma(nn.Module):
    def __init__(self, model, decay=0.9999, use_num_upates=True):
        super().__init__()
        if decay < 0.0 or decay > 1.0:
            raise ValueError("Decay must be between 0 and 1")
        self.m_name2s_name = {}
        self.register_buffer("decay", torch.tensor(decay, dtype=torch.float32))
        self.register_buffer("num_updates", torch.tensor(0, dtype=torch.int) if use_num_upates
                             else torch.tensor(-1, dtype=torch.int))
        for name, p in model.named_parameters():
            if p.requires_grad:
                s_name = name.replace(".", "")
                self.m_name2s_name[name] = s_name
                self.register_buffer(s_name, p.clone().detach().data)
        self.collected_params = []
        self._arena = None
        self._prefix = ""

    # ------------------------------------------------------------ arena binding
    def bind_arena(self, arena, prefix: str = ""):
        """Re-home the shadow buffers as views of arena.ema (names keep the reference form)."""
        ema = arena.enable_ema()
        with torch.no_grad():
            for name, s_name in self.m_name2s_name.items():
                view = arena.view_in(ema, prefix + name)
                view.copy_(self._buffers[s_name].to(view.device))
                self._buffers[s_name] = view
        self._arena, self._prefix = arena, prefix

    def _host_counters(self):
        """Host mirror of (decay, num_updates): read from the buffers once (or after a
        state_dict load), then advanced on the host, so a training step never waits on the
        device for the EMA scalars.  The buffers are written back (one small H2D copy, no
        sync) at every update so state_dict() stays exact."""
        key = (self.decay.data_ptr(), self.num_updates.data_ptr(), self.num_updates._version)
        if getattr(self, "_host", None) is None or self._host[2] != key:
            self._host = [float(self.decay), int(self.num_updates), key]
        return self._host

    def next_decay(self) -> float:
        """ema.py:29-33: decay = min(decay, (1 + n) / (10 + n)) after n += 1 (returns 1 - decay)."""
        h = self._host_counters()
        decay = h[0]
        if h[1] >= 0:
            h[1] += 1
            n = h[1]
            decay = min(decay, (1 + n) / (10 + n))
            self.num_updates.fill_(n)  # device-side fill: no host sync
            h[2] = (self.decay.data_ptr(), self.num_updates.data_ptr(), self.num_updates._version)
        return float(1.0 - torch.tensor(decay, dtype=torch.float32))

    def forward(self, model):
        omd = self.next_decay()
        with torch.no_grad():
            if self._arena is not None:
                a = self._arena
                a.ema.sub_(omd * (a.ema - a.master[: a.ema_numel]))
                return
            m_param = dict(model.named_parameters())
            shadow = dict(self.named_buffers())
            for key, p in m_param.items():
                if p.requires_grad:
                    s = shadow[self.m_name2s_name[key]]
                    s.sub_(omd * (s - p))

    def copy_to(self, model):
        m_param = dict(model.named_parameters())
        shadow = dict(self.named_buffers())
        for key, p in m_param.items():
            if p.requires_grad:
                p.data.copy_(shadow[self.m_name2s_name[key]].data)
        self._dirty()

    def store(self, parameters):
        self.collected_params = [p.clone() for p in parameters]

    def restore(self, parameters):
        for c, p in zip(self.collected_params, parameters):
            p.data.copy_(c.data)
        self._dirty()

    def _dirty(self):
        """Parameter values changed behind the arena's back: bf16 weight packs are stale."""
        if self._arena is not None:
            self._arena.mark_dirty()
