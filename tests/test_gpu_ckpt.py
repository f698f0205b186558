"""main_val.py:845-862 (melk): SIGUSR1 summons a checkpoint -- HipTrainer.install_signal_handlers
raises a flag, the step in progress finishes (graph replay), its boundary writes
``ckptdir/last.ckpt`` in the Lightning layout {'state_dict', 'epoch', 'global_step'}: the trained
parameters and EMA (views of the arenas the graph-replayed optimizer updated), loadable by
``init_from_ckpt`` into a fresh model with no missing / unexpected keys."""
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
    assert set(ck) == {"state_dict", "epoch", "global_step"} and ck["global_step"] == ldm.global_step
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
