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


def test_st_wgrad_plan_layout():
    """Host logic of encdiff_st_wgrad_plan (no GPU): for a c = 64 / 128 transformer block's eight
    weight gradients at the training batch the plan covers every token in chunks, gives each problem
    a slab region of its own inside the workspace (no overlap), numbers work items and fold blocks
    contiguously, and doubles the chunk length until the slabs fit a small workspace."""
    import encdiff_amd._lib as L

    class StWg(C.Structure):  # st_bwd.hip / stwg.h StWg (plan blob, after a 64-byte header)
        _fields_ = [("dy", C.c_void_p), ("x", C.c_void_p), ("dw", C.c_void_p), ("db", C.c_void_p),
                    ("slab", C.c_void_p), ("ld_dy", C.c_long), ("ld_x", C.c_long), ("ld_dw", C.c_long)] + \
                   [(n, C.c_int) for n in ("M", "N", "K", "kc", "kb", "mb", "nb", "item0", "fold0", "kind", "bm",
                                           "bn")]
    base = 1 << 32
    for c, K in ((64, 32768), (128, 8192)):
        shapes = [(c, c, True), (3 * c, c, False), (c, c, True), (c, c, False), (c, c, True), (8 * c, c, True),
                  (c, 4 * c, True), (c, c, True)]
        arr = (L.WgradProb * len(shapes))()
        for i, (M, N, b) in enumerate(shapes):
            arr[i] = L.WgradProb(dy=base + i * (1 << 26), ld_dy=M, x=base + (1 << 30) + i * (1 << 26), ld_x=N,
                                 dw=base + (1 << 31) + i * (1 << 24), ld_dw=N,
                                 db=(base + (3 << 30) + i * 4096) if b else None, M=M, N=N, K=K)
        for ws_floats in (24 << 20, 4 << 20):
            ws = 1 << 40
            nb = C.c_long(0)
            assert L.lib.encdiff_st_wgrad_plan(arr, len(shapes), ws, ws_floats, None, 0, C.byref(nb)) == 0
            blob = (C.c_longlong * ((nb.value + 7) // 8))()
            assert L.lib.encdiff_st_wgrad_plan(arr, len(shapes), ws, ws_floats, C.addressof(blob), C.sizeof(blob),
                                               C.byref(nb)) == 0
            hdr = (C.c_int * 4).from_buffer(blob)
            magic, nprob, nitems, nfold = list(hdr)
            assert magic == 0x53545747 and nprob == len(shapes)
            probs = (StWg * nprob).from_address(C.addressof(blob) + 64)
            regions, item, fold = [], 0, 0
            for p, (M, N, b) in zip(probs, shapes):
                assert (p.M, p.N, p.K) == (M, N, K)
                assert p.kb * p.kc >= K and (p.kb - 1) * p.kc < K and p.kc % 32 == 0
                assert M % p.bm == 0 and N % p.bn == 0 and p.mb == M // p.bm and p.nb == N // p.bn
                assert p.item0 == item and p.fold0 == fold
                item += p.mb * p.nb * p.kb
                if p.kb > 1:
                    need = p.kb * M * N + (p.kb * M if b else 0)
                    lo = (p.slab - ws) // 4
                    assert lo >= 0 and lo + need <= ws_floats
                    regions.append((lo, lo + need))
                    fold += (M * N // 4 + 31) // 32 + ((M + 31) // 32 if b else 0)
            assert (item, fold) == (nitems, nfold)
            regions.sort()
            assert all(a[1] <= b[0] for a, b in zip(regions, regions[1:])), "slab regions overlap"
            if ws_floats == 4 << 20:  # the small workspace forced longer chunks
                assert max(p.kc for p in probs) > 256
