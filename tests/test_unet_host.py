"""CPU tests of the host side of the UNet mirror: config instantiation, module /
parameter names and shapes identical to the reference state_dict, the executor's
static schedule and the arena layout."""
import json
import os

import pytest
import torch

import encdiff_amd  # noqa: F401  (installs the ldm alias)
from oracle import encdiff_oracle as O

UNET_PARAMS = dict(image_size=16, in_channels=3, out_channels=3, model_channels=64, attention_resolutions=[1, 2, 4],
                   num_res_blocks=2, channel_mult=[1, 2, 4, 4], num_heads=8, use_scale_shift_norm=True,
                   resblock_updown=True, use_spatial_transformer=True, context_dim=16, latent_unit=20)


def test_instantiate_from_config_alias():
    from ldm.util import instantiate_from_config
    m = instantiate_from_config({"target": "ldm.modules.diffusionmodules.openaimodel_enc.UNetModel",
                                 "params": UNET_PARAMS})
    from encdiff_amd.ldm.modules.diffusionmodules.openaimodel_enc import UNetModel
    assert isinstance(m, UNetModel)


def test_unet_state_dict_matches_reference(golden_dir):
    from encdiff_amd.ldm.modules.diffusionmodules.openaimodel_enc import UNetModel
    m = UNetModel(**UNET_PARAMS)
    ref = json.load(open(os.path.join(golden_dir, "unet_state_dict_shapes.json")))
    mine = {k: list(v.shape) for k, v in m.state_dict().items()}
    assert mine == ref
    assert sum(p.numel() for p in m.parameters()) == 37469635


def test_load_reference_named_weights():
    from encdiff_amd.ldm.modules.diffusionmodules.openaimodel_enc import UNetModel
    m = UNetModel(**UNET_PARAMS)
    P = O.recipe_params(O.param_shapes(O.build_plan()))
    m.load_state_dict(P, strict=True)


def test_spec_counts_and_arena_layout():
    from encdiff_amd.unet import UNetSpec
    from encdiff_amd.arena import ParamArena
    from encdiff_amd.ldm.modules.diffusionmodules.openaimodel_enc import UNetModel
    s = UNetSpec.from_config(UNET_PARAMS)
    assert len(s.res) == 28 and len(s.sts) == 16
    assert s.film_total == 10240 and s.kv_total == 4992
    assert [t.h for t in s.sts] == [16] * 2 + [8] * 2 + [4] * 2 + [2] + [4] * 3 + [8] * 3 + [16] * 3
    m = UNetModel(**UNET_PARAMS)
    named = dict(m.named_parameters())
    arena = ParamArena(s.arena_order(named), "cpu", ema_names=list(named))
    assert arena.ema_numel >= 37469635
    # params are views of the arena, grads too
    for n, p in named.items():
        o, _ = arena.offsets[n]
        assert p.data_ptr() == arena.master.data_ptr() + 4 * o
        assert p.grad.data_ptr() == arena.grad.data_ptr() + 4 * o
    o, n = arena.span([r.prefix + "emb_layers.1.weight" for r in s.res])
    assert n == 10240 * 256


def test_unet_refuses_cpu():
    from encdiff_amd.ldm.modules.diffusionmodules.openaimodel_enc import UNetModel
    m = UNetModel(**UNET_PARAMS)
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 3, 16, 16), torch.zeros(1, dtype=torch.long), [torch.zeros(1, 320)])


@pytest.mark.parametrize("params", [UNET_PARAMS, dict(UNET_PARAMS, image_size=32, model_channels=128,
                                                        latent_unit=40)])
def test_dp_split_layout(params):
    """The data-parallel split (trainer.py / UNetExecutor.split_plan): in the arena the
    output-block + out parameters form one contiguous tail [lo, end) that excludes every
    parameter the UNet backward writes after the output blocks (batched emb / cross-K,V /
    q,k,v weights), and the norm-partial columns of those layers form a suffix."""
    from encdiff_amd.arena import NormPartials
    from encdiff_amd.ldm.modules.diffusionmodules.openaimodel_enc import UNetModel
    from encdiff_amd.unet import UNetExecutor
    m = UNetModel(**params)
    arena = m.bind_arena()
    names = [n for n, _ in m.named_parameters()]
    lo = UNetExecutor.arena_split_offset(arena, names)
    assert lo is not None and 0 < lo < arena.numel
    early = {n for n in names if UNetExecutor._early_final(n)}
    late_written = [n for n in names if ".emb_layers.1." in n or ".attn2.to_k." in n or ".attn1.to_q." in n]
    assert late_written and not early & set(late_written)
    assert all(arena.offsets[n][0] >= lo for n in early)
    assert all(arena.offsets[n][0] < lo for n in names if n not in early)
    assert {n.split(".")[0] for n in early} == {"output_blocks", "out"}
    # norm partial columns in the executor's registration order (output-block layers last)
    np_ = NormPartials(arena, 4)
    spec = m._spec
    gn = [(r.prefix + "in_layers.0.weight", r.prefix + "in_layers.0.bias") for r in spec.res]
    gn += [(r.prefix + "out_layers.0.weight", r.prefix + "out_layers.0.bias") for r in spec.res]
    gn += [(t.prefix + "norm.weight", t.prefix + "norm.bias") for t in spec.sts] + [("out.0.weight", "out.0.bias")]
    gn.sort(key=lambda p: UNetExecutor._early_final(p[0]))
    for gname, bname in gn:
        np_.add(gname, bname)
    c = np_.split_col(UNetExecutor._early_final)
    assert c is not None and 0 < c < np_.cols
    tail = [np_.index[j] for j in range(c, np_.cols)]
    head = [np_.index[j] for j in range(c)]
    assert min(tail) >= lo and max(head) < lo
    # unsorted (forward) order would not be a suffix: the plan must refuse it
    bad = NormPartials(arena, 4)
    for gname, bname in sorted(gn, key=lambda p: not UNetExecutor._early_final(p[0])):
        bad.add(gname, bname)
    assert bad.split_col(UNetExecutor._early_final) is None


def test_wg3_split_matches_kernel_rule():
    """ops.wg3_split (host plan of the 3x3 weight-gradient kernel WG3) only returns splits that
    gemm.hip wg3_check accepts: whole-image chunks (images per chunk a multiple of the images per
    32-pixel stage) whose stage count divides over the workgroup's waves; odd batches fall back."""
    from encdiff_amd import ops, _lib as L
    for B in (1, 2, 3, 4, 6, 8, 16, 32, 64, 128, 512):
        for h in (4, 8, 16, 32):
            for tile in (32, 33, 34):
                sp = ops.wg3_split(B, h, h, 64, 64, 0, 64, 64, L.OUT_F32_ACCUM, tile=tile)
                if h == 32:
                    assert sp is None
                if sp is None:
                    continue
                ni, rows = (1 if h == 16 else 2), (4 if h == 4 else 2)
                assert B % sp == 0 and (B // sp) % ni == 0
                assert ((B // sp // ni) * (h // rows)) % (8 if tile == 33 else 4) == 0
    assert ops.wg3_split(128, 16, 16, 64, 64, 0, 64, 64, L.OUT_BF16) is None  # fp32 outputs only
    assert ops.wg3_split(128, 16, 16, 48, 64, 0, 64, 64, L.OUT_F32_ACCUM) is None  # cout % 32


def test_bind_refuses_shared_per_batch_state():
    """UNetExecutor.bind keeps one buffer set per batch size; a name declared in __init__ is shared
    by all of them unless _PER_BATCH lists it.  A per-batch buffer declared in __init__ but not
    listed (the round-5 GroupNorm-partials fault: B=64 backwards wrote past a B=16 buffer) must
    fail at its first bind, and once listed it must be saved / restored across batch switches.
    The real bind() runs on CPU tensors through a stand-in _bind_new."""
    from encdiff_amd.unet import UNetExecutor

    class Ex(UNetExecutor):
        def __init__(self, per_batch):
            self._PER_BATCH = frozenset(per_batch)
            self.B = None
            self._sets = {}
            self.parts = None  # declared here, sized by B in bind (like `gn`)
            self.width = 3     # truly shared
            self._base_names = (set(self.__dict__) - self._PER_BATCH) | {"_base_names"}

        def _bind_new(self, B):
            self.act = torch.empty(B, self.width)
            self.parts = torch.empty(B, 7)

    with pytest.raises(RuntimeError, match="parts"):
        Ex(per_batch=()).bind(4)
    ex = Ex(per_batch=("parts",))
    ex.bind(4)
    p4 = ex.parts
    ex.bind(16)
    assert ex.parts.shape[0] == 16 and ex.act.shape[0] == 16
    ex.bind(4)
    assert ex.parts is p4 and ex.act.shape[0] == 4
