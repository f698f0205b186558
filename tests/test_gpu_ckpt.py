"""main_val.py:845-862 (melk): SIGUSR1 summons a checkpoint -- HipTrainer.install_signal_handlers
raises a flag, the step in progress finishes (graph replay), its boundary writes
``ckptdir/last.ckpt`` in the Lightning layout {'state_dict', 'epoch', 'global_step',
'optimizer_states', 'lr_schedulers'} (+ the data position): the trained parameters and EMA (views
of the arenas the graph-replayed optimizer updated), loadable by ``init_from_ckpt`` into a fresh
model with no missing / unexpected keys, and a resume (HipTrainer.load_checkpoint) continues the
run bitwise as the uninterrupted trainer does."""
import os
import signal

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_sigusr1_writes_last_ckpt(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import bench
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    from encdiff_amd.trainer import HipTrainer
    torch.manual_seed(5)
    ldm, _ = bench.build_ldm()
    tr = HipTrainer(ldm, 8, graph=True, pool_size=64)
    tr.init_scale_factor()
    tr.install_signal_handlers(str(tmp_path))
    try:
        tr.step()
        tr.step()  # the graph is captured and replayed
        step_before = ldm.global_step
        assert not (tmp_path / "last.ckpt").exists()
        os.kill(os.getpid(), signal.SIGUSR1)
        tr.step()
    finally:
        signal.signal(signal.SIGUSR1, signal.SIG_DFL)
    path = tmp_path / "last.ckpt"
    assert path.exists()
    ck = torch.load(str(path), map_location="cpu", weights_only=True)
    assert set(ck) == {"state_dict", "epoch", "global_step", "optimizer_states", "lr_schedulers", "encdiff_data"}
    assert ck["global_step"] == ldm.global_step
    assert ck["optimizer_states"][0]["step"] == tr.opt.step_count and len(ck["lr_schedulers"]) == 1
    sd = ldm.state_dict()
    assert set(ck["state_dict"]) == set(sd)
    for k, v in sd.items():
        assert torch.equal(ck["state_dict"][k], v.detach().cpu()), k
    assert ck["global_step"] == step_before + 1  # written at the signalled step's boundary
    torch.manual_seed(6)
    m2 = instantiate_from_config(model_config("shapes3d"))
    missing, unexpected = m2.init_from_ckpt(str(path))
    assert not missing and not unexpected
    for k2, v in m2.state_dict().items():
        assert torch.equal(v.cpu(), ck["state_dict"][k2]), k2


def test_resume_from_last_ckpt_continues_bitwise(tmp_path):
    """A trainer resumed from save_checkpoint's file (parameters, EMA, AdamW moments and step, LR
    schedule, data position) takes the next step exactly as the uninterrupted trainer does: same
    loss, parameters and EMA bit for bit (same seed, so the same t / noise stream)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import bench
    from encdiff_amd.trainer import HipTrainer

    def make():
        torch.manual_seed(5)
        ldm, _ = bench.build_ldm()
        tr = HipTrainer(ldm, 8, graph=False, pool_size=64)
        tr.init_scale_factor()
        return ldm, tr
    ldm_a, a = make()
    for _ in range(3):
        a.step()
    path = str(tmp_path / "mid.ckpt")
    a.save_checkpoint(path)
    a.step()
    loss_a = a.loss()
    sd_a = {k: v.detach().clone() for k, v in ldm_a.state_dict().items()}  # parameters, EMA, BN buffers
    del a, ldm_a
    ldm_b, b = make()
    for _ in range(3):  # the same RNG position (t / noise are drawn on the device, step-indexed)
        b.step()
    b.arena.master.normal_()  # scramble everything the checkpoint restores
    b.arena.exp_avg.zero_()
    b.arena.exp_avg_sq.zero_()
    b.opt.step_count = 0
    b.load_checkpoint(path)
    b.step()
    assert b.loss() == loss_a
    sd_b = ldm_b.state_dict()
    assert set(sd_b) == set(sd_a)
    for k, v in sd_a.items():  # (the arena's alignment padding is not model state)
        assert torch.equal(sd_b[k], v), k
