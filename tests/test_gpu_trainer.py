"""The benchmarked training step itself, pinned to the oracle (configs[1] and configs[3]).

bench.py times HipTrainer at configs[1] (Shapes3D, B = 128 per GPU, the whole step captured
as one HIP graph).  These tests run exactly that object -- same batch size, same graph, the
B >= 64 code paths (GroupNorm statistics from the producing GEMMs, LayerNorm in GEMM
epilogues, the measured tile / split-K plans, the fused AdamW + EMA + repack, the HIP VQ
encoder and Encoder4 trunk) -- with recipe weights, feeding each replay's image batch,
timesteps and noise through HipTrainer.enable_feed(); the CPU oracle (OracleTrainer, fp32, VQ
encode included) starts from the trainer's state after its eager warm-up steps and runs the
same inputs (oracle/step_check.py).  configs[3] (MPI3D_toy, 64x64, the same tensor shapes)
runs at 512 images per GPU: every GEMM at M = 4x the B = 128 rows, whose tile / split-K
choices come from ops.plan's heuristic rather than the measured table.

Reference: ddpm_enc.py:360-375 (training_step), :773-844 (get_input), :1040-1053 (forward),
:1183-1253 (p_losses), :1598-1639 (AdamW), ema.py:25-44 (LitEma); main_val.py:656-660 (DDP).

Tolerances (bf16 activations vs the fp32 reference): eps rel-L2 <= 3e-2 and
max-abs <= 6e-2; loss rel <= 1e-2; gradients rel-L2 <= 5e-2; AdamW / EMA parameter updates
rel-L2 <= 5e-2 (oracle/step_check.py TOL).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rig():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle.step_check import GraphStepCheck
    return GraphStepCheck(B=128)


def test_scale_factor(rig):
    from oracle.step_check import rel
    r = rel(rig.sf_hip, rig.orc.scale_factor)
    print("scale_factor", rig.sf_hip, rig.orc.scale_factor, r)
    assert r < 1e-2


@pytest.mark.parametrize("step", [0, 1])
def test_graph_step_b128_matches_oracle(rig, step):
    from oracle.step_check import failures, summary
    r = rig.check()
    print(f"step {step}: " + summary(r))
    print("listed grads: " + ", ".join(f"{k} {v:.2e}" for k, v in r["grads_listed"].items()))
    bad = failures(r)
    assert not bad, (bad, summary(r))


def test_graph_step_b512_config3_matches_oracle():
    """configs[3]: the large-batch step (512 images per GPU) vs the oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gc
    from oracle.step_check import GraphStepCheck, failures, summary
    gc.collect()
    torch.cuda.empty_cache()
    chk = GraphStepCheck(B=512, seed=512, warmup=1)
    r = chk.check()
    print(summary(r))
    bad = failures(r)
    assert not bad, (bad, summary(r))


def test_graph_step_after_ema_scope(rig):
    """after an EMA scope (whose eager sampling repacked the bf16 weights from the EMA
    shadow), the replayed training step must run on the restored training weights: the replay
    refreshes stale packs.  The shadow is set to 0.9 x the weights so stale packs would fail."""
    from oracle.step_check import failures, summary
    ldm, a = rig.ldm, rig.tr.arena
    ex = ldm.model.diffusion_model._ex
    saved_ema = a.ema.clone()
    packed = ex.pack.snapshot()
    a.ema.copy_(a.master[: a.ema.numel()] * 0.9)
    x = torch.randn(2, 3, 16, 16, device="cuda")
    with torch.no_grad(), ldm.ema_scope():
        ldm.apply_model(x, torch.tensor([5, 500], device="cuda"), torch.randn(2, 320, device="cuda"))
        assert not torch.equal(ex.pack.snapshot(), packed), "EMA scope did not repack"
    a.ema.copy_(saved_ema)
    ldm.train()
    r = rig.check()
    print("after ema_scope: " + summary(r))
    bad = failures(r)
    assert not bad, (bad, summary(r))
