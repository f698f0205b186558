"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every
symbol the header declares, and the ctypes mirror of each struct has exactly the
C layout (compiled with gcc against include/encdiff_hip.h)."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "include", "encdiff_hip.h")


def header_functions():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"\bint\s+(encdiff_\w+)\s*\(", txt)))


def test_header_exports_match_library():
    import encdiff_amd._lib as L
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (encdiff_\w+)", out))
    declared = set(header_functions())
    assert declared, "no functions parsed from the header"
    assert declared <= exported, f"missing exports: {declared - exported}"
    assert set(L.EXPORTS) == declared, "ctypes prototypes out of sync with the header"


STRUCTS = {
    "EncdiffConvGeom": "ConvGeom", "EncdiffGemmArgs": "GemmArgs", "EncdiffGroupNormArgs": "GroupNormArgs",
    "EncdiffLayerNormArgs": "LayerNormArgs", "EncdiffAttnArgs": "AttnArgs", "EncdiffEwArgs": "EwArgs",
    "EncdiffSmallConvArgs": "SmallConvArgs", "EncdiffPackJob": "PackJob", "EncdiffBatchNormArgs": "BatchNormArgs",
    "EncdiffStTailArgs": "StTailArgs", "EncdiffStHeadArgs": "StHeadArgs", "EncdiffZeroJob": "ZeroJob",
    "EncdiffStepPrologueArgs": "StepPrologueArgs", "EncdiffResConvArgs": "ResConvArgs",
    "EncdiffStTailBwdArgs": "StTailBwdArgs", "EncdiffStHeadBwdArgs": "StHeadBwdArgs", "EncdiffWgradProb": "WgradProb",
}


def test_struct_layouts_match_c():
    import encdiff_amd._lib as L
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HDR}"', "int main(void){"]
    for cname, pyname in STRUCTS.items():
        lines.append(f'printf("{pyname} size %zu\\n", sizeof({cname}));')
        for fname, _ in getattr(L, pyname)._fields_:
            lines.append(f'printf("{pyname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "probe.c"), os.path.join(d, "probe")
        open(src, "w").write("\n".join(lines))
        subprocess.run(["gcc", "-std=c99", "-o", exe, src], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    for line in out.strip().splitlines():
        pyname, field, val = line.split()
        cls = getattr(L, pyname)
        if field == "size":
            assert C.sizeof(cls) == int(val), pyname
        else:
            assert getattr(cls, field).offset == int(val), f"{pyname}.{field}"


def test_product_path_has_no_oracle_or_fallback():
    """The product package never imports the oracle nor a CPU fallback."""
    pkg = os.path.join(REPO, "encdiff_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                txt = open(os.path.join(root, f)).read()
                assert "from oracle" not in txt and "import oracle" not in txt, f


def test_torch_library_ops_registered():
    """The reference-API modules call torch.ops.encdiff.* (SURVEY §8(b)); their fake kernels
    propagate shapes without a device, and the real ones refuse CPU tensors (no fallback)."""
    import torch
    from torch._subclasses.fake_tensor import FakeTensorMode
    import encdiff_amd.torch_ops  # noqa: F401
    for name in ("q_sample", "l1_loss", "ddim_step", "attention_fwd", "attention_bwd"):
        assert hasattr(torch.ops.encdiff, name), name
    with FakeTensorMode():
        x = torch.empty(4, 3, 16, 16)
        t = torch.empty(4, dtype=torch.long)
        assert torch.ops.encdiff.q_sample(x, x, t, torch.empty(1000), torch.empty(1000)).shape == x.shape
        out2, seed = torch.ops.encdiff.l1_loss(x, x, t, torch.empty(1000), 1.0)
        assert out2.shape == (2,) and seed.shape == x.shape
        q = torch.empty(2, 256, 64, dtype=torch.bfloat16)
        o, lse = torch.ops.encdiff.attention_fwd(q, q, q, 8, False)
        assert o.shape == q.shape and lse.shape == (16, 256)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        torch.ops.encdiff.q_sample(torch.zeros(1, 3, 4, 4), torch.zeros(1, 3, 4, 4), torch.zeros(1, dtype=torch.long),
                                   torch.zeros(1000), torch.zeros(1000))
