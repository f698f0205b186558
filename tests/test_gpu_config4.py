"""BASELINE.json configs[4] end to end: the builder-defined CelebA 128x128 LatentDiffusion
(encdiff_amd.configs.CELEBA128: VQ-f4 latent (B, 3, 32, 32), model_channels 128, 40 concept
tokens, Encoder4 with a fifth stride-2 stage) trained by the same graph-captured HipTrainer as the
benchmark, vs the CPU oracle configured alike.  Parametrized over the attention score precision:
bf16 MFMA (the default) and fp8 (OCP e4m3) scores in the S = 1024 self-attention
(``UNetModel(attn_fp8_min_tokens=1024)``, set per test -- BASELINE names "fp8 MFMA attention"
for this config), the oracle emulating e4m3 with torch.float8_e4m3fn.  No reference config exists
for this one, so the oracle -- pinned to the reference on Shapes3D -- is
the checker ("parity unpinned" by the reference itself); tolerances as in test_gpu_trainer.py
(oracle/step_check.py TOL), every single UNet parameter gradient included."""
import pytest
import torch

pytestmark = pytest.mark.gpu

B = 8


@pytest.mark.parametrize("fp8", [False, True], ids=["bf16_scores", "fp8_scores"])
def test_celeba128_step_matches_oracle(fp8):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle.step_check import GraphStepCheck, failures, summary
    chk = GraphStepCheck(B=B, config="celeba128", seed=77, warmup=1,
                         unet_params={"attn_fp8_min_tokens": 1024 if fp8 else 0})
    st = [t for t in chk.ldm.model.diffusion_model._spec.sts if t.fp8]
    if fp8:
        assert st and all(t.h == 32 for t in st), "fp8 scores on the 32x32 (S = 1024) level only"
    else:
        assert not st, "bf16 attention scores everywhere"
    assert chk.tr.res == 128
    r = chk.check(grad_names=[], cond_names=[])
    print(("fp8" if fp8 else "bf16") + " scores: " + summary(r))
    bad = failures(r, every_param=True)
    assert not bad, (bad, summary(r))
    del chk
    torch.cuda.empty_cache()
