"""Alias: BASELINE.json names ``ldm.models.diffusion.ddpm.LatentDiffusion``; the EncDiff
class lives in ddpm_enc (ddpm_enc.py:482).  Both import paths resolve to one class."""
from .ddpm_enc import DDPM, DiffusionWrapper, FusedArenaAdamW, LatentDiffusion, disabled_train  # noqa: F401
