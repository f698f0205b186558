"""encdiff_amd -- MI355X-native EncDiff denoising path.

Importing this package installs an import alias so that the reference's dotted
config targets (``ldm.models.diffusion.ddpm_enc.LatentDiffusion``,
``ldm.modules.diffusionmodules.openaimodel_enc.UNetModel`` ...) resolve to the
mirror implementation in ``encdiff_amd.ldm`` -- the same module objects under
both names, so reference YAML configs load unchanged.
"""
from __future__ import annotations

import importlib
import importlib.abc
import importlib.util
import sys

__version__ = "0.1.0"

_ALIASES = {"ldm": "encdiff_amd.ldm", "main": "encdiff_amd.main", "main_val": "encdiff_amd.main"}


class _AliasFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, fullname, path, target=None):
        root = fullname.split(".", 1)[0]
        if root in _ALIASES:
            return importlib.util.spec_from_loader(fullname, self, is_package=True)
        return None

    def create_module(self, spec):
        root, _, rest = spec.name.partition(".")
        real = _ALIASES[root] + ("." + rest if rest else "")
        return importlib.import_module(real)

    def exec_module(self, module):
        pass


def install_ldm_alias():
    if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
        sys.meta_path.insert(0, _AliasFinder())


install_ldm_alias()
