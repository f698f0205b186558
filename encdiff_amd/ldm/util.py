"""Config plumbing mirroring ldm/util.py:78-93 (instantiate_from_config)."""
from __future__ import annotations

import importlib
from inspect import isfunction


def exists(x):
    return x is not None


def default(val, d):
    if exists(val):
        return val
    return d() if isfunction(d) else d


def count_params(model, verbose=False):
    total = sum(p.numel() for p in model.parameters())
    if verbose:
        print(f"{model.__class__.__name__} has {total * 1.e-6:.2f} M params.")
    return total


def get_obj_from_str(string, reload=False):
    module, cls = string.rsplit(".", 1)
    mod = importlib.import_module(module)
    if reload:
        importlib.reload(mod)
    return getattr(mod, cls)


def instantiate_from_config(config):
    """ldm/util.py:78-85: {'target': dotted.path, 'params': {...}}."""
    if "target" not in config:
        if config in ("__is_first_stage__", "__is_unconditional__"):
            return None
        raise KeyError("Expected key `target` to instantiate.")
    params = config.get("params", dict()) or {}
    return get_obj_from_str(config["target"])(**dict(params))


def mean_flat(tensor):
    return tensor.mean(dim=list(range(1, len(tensor.shape))))
