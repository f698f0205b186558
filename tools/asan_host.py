"""Host-side AddressSanitizer build of the library's C++ (argument validation, planning, launch
set-up) and a run of host-only checks against it -- SURVEY §5 "sanitizers": GPU ASan is not
available on this pool, so only the host half of every .hip file is instrumented
(`--cuda-host-only -Xarch_host -fsanitize=address`).  The build has no device code: every check
below stays on the host (planning entry points, and every launch entry's argument validation with
arguments it must refuse); a launch that got past validation would fail without a device anyway.

    python tools/asan_host.py            # build encdiff_amd/_asan/libencdiff_hip_asan.so, run the checks
    python tools/asan_host.py --checks   # (inside the preloaded child process) the checks only

Exit status 0 and no "ERROR: AddressSanitizer" in the output = clean.  tests/test_asan_host.py
runs it on CPU.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "encdiff_amd", "csrc")
OUT = os.path.join(REPO, "encdiff_amd", "_asan")
LIB = os.path.join(OUT, "libencdiff_hip_asan.so")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
FLAGS = ["-O1", "-g", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-host-only",
         "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer",
         "-I" + os.path.join(REPO, "include")]


def asan_runtime():
    c = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return c[-1] if c else None


def build():
    os.makedirs(OUT, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    hdrs = glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(REPO, "include", "encdiff_hip.h")]
    newest = max(os.path.getmtime(f) for f in srcs + hdrs)
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= newest:
        return LIB

    def one(src):
        obj = os.path.join(OUT, os.path.basename(src) + ".o")
        r = subprocess.run([HIPCC, *FLAGS, "-c", src, "-o", obj], capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(f"asan compile failed for {src}:\n{r.stderr}")
        return obj
    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(one, srcs))
    # a host-only object references its translation unit's device binary (__hip_fatbin_<cuid>), which
    # only a device compile would provide: zero-filled stand-ins let the library load on a host
    # without a GPU (no kernel is launched by the checks)
    nm = subprocess.run(["nm", "-u", *objs], capture_output=True, text=True, check=True).stdout
    syms = sorted({w for w in nm.split() if w.startswith("__hip_fatbin_")})
    stub_c, stub_o = os.path.join(OUT, "fatbin_stubs.c"), os.path.join(OUT, "fatbin_stubs.o")
    with open(stub_c, "w") as f:
        for sym in syms:
            f.write(f"__attribute__((aligned(4096))) char {sym}[4096] = {{0}};\n")
    subprocess.run(["gcc", "-c", "-fPIC", stub_c, "-o", stub_o], check=True)
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-fsanitize=address", "-shared-libsan",
                        "-o", LIB + ".tmp", *objs, stub_o], capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(f"asan link failed:\n{r.stderr}")
    os.replace(LIB + ".tmp", LIB)
    return LIB


def checks():
    """Host-only paths of the C-ABI: planning entry points over valid and invalid problem lists,
    and every launch entry point with arguments its validation must refuse."""
    import ctypes as C
    sys.path.insert(0, REPO)
    from encdiff_amd import _lib as L
    lib = L.lib
    n = 0
    assert lib.encdiff_version() > 0
    # tile choice of the fused transformer backward
    for c in (64, 128, 256):
        for rows in (256, 4096, 32768, 131072):
            for tokens in (64, 256, 1024):
                lib.encdiff_st_tail_bwd_tile(c, rows, tokens)
                n += 1
    # grouped weight-gradient plan: fake 16-B aligned device addresses (never dereferenced on the host)
    base = 1 << 32

    def probs(shapes, K):
        arr = (L.WgradProb * len(shapes))()
        for i, (M, N, b) in enumerate(shapes):
            arr[i] = L.WgradProb(dy=base + i * (1 << 26), ld_dy=M, x=base + (1 << 30) + i * (1 << 26), ld_x=N,
                                 dw=base + (1 << 31) + i * (1 << 24), ld_dw=N,
                                 db=(base + (3 << 30) + i * 4096) if b else None, M=M, N=N, K=K)
        return arr
    for c, K in ((64, 32768), (128, 8192), (256, 2048), (64, 256), (128, 131072)):
        shapes = [(c, c, True), (3 * c, c, False), (c, c, True), (c, c, False), (c, c, True), (8 * c, c, True),
                  (c, 4 * c, True), (c, c, True)]
        for ws in (0, 1 << 10, 1 << 20, 24 << 20):
            arr = probs(shapes, K)
            nb = C.c_long(0)
            rc = lib.encdiff_st_wgrad_plan(arr, len(shapes), base + (5 << 30), ws, None, 0, C.byref(nb))
            if rc == 0:
                for cap in (nb.value, nb.value - 8, 8):
                    blob = (C.c_longlong * max(1, (cap + 7) // 8))()
                    lib.encdiff_st_wgrad_plan(arr, len(shapes), base + (5 << 30), ws, C.addressof(blob), cap,
                                              C.byref(nb))
            n += 1
    bad = probs([(96, 64, True)], 512)                                   # M % 64
    assert lib.encdiff_st_wgrad_plan(bad, 1, None, 0, None, 0, C.byref(C.c_long(0))) < 0
    assert lib.encdiff_st_wgrad_plan(probs([(64, 64, True)] * 17, 512), 17, None, 0, None, 0,
                                     C.byref(C.c_long(0))) < 0          # too many problems
    assert lib.encdiff_st_wgrad_plan(None, 1, None, 0, None, 0, C.byref(C.c_long(0))) < 0
    # launch of a blob that is not a plan
    junk = (C.c_longlong * 16)()
    assert lib.encdiff_st_wgrad_launch(C.addressof(junk), C.addressof(junk), None) < 0
    # every launch entry with arguments it must refuse (NULL argument structs)
    one_arg = ["encdiff_gemm_finalize", "encdiff_groupnorm_fwd", "encdiff_groupnorm_bwd", "encdiff_layernorm_fwd",
               "encdiff_layernorm_bwd", "encdiff_attention_fwd", "encdiff_attention_bwd", "encdiff_elementwise",
               "encdiff_st_tail_fwd", "encdiff_st_head_fwd", "encdiff_st_tail_bwd", "encdiff_st_head_bwd",
               "encdiff_resconv_fwd", "encdiff_gemm", "encdiff_batchnorm_fwd", "encdiff_batchnorm_bwd",
               "encdiff_batchnorm_apply"]
    for name in one_arg:
        f = getattr(lib, name)
        rc = f(None, None)
        assert rc < 0, (name, rc)
        n += 1
    # argument structs that are zero (every pointer NULL, every size 0)
    zero = [("encdiff_groupnorm_fwd", L.GroupNormArgs), ("encdiff_groupnorm_bwd", L.GroupNormArgs),
            ("encdiff_layernorm_fwd", L.LayerNormArgs), ("encdiff_attention_fwd", L.AttnArgs),
            ("encdiff_st_tail_fwd", L.StTailArgs), ("encdiff_st_tail_bwd", L.StTailBwdArgs),
            ("encdiff_st_head_bwd", L.StHeadBwdArgs), ("encdiff_gemm", L.GemmArgs)]
    for name, T in zero:
        a = T()
        rc = getattr(lib, name)(C.byref(a), None)
        assert rc < 0, (name, rc)
        n += 1
    # the GroupNorm backward's riding fold: inconsistent plan / block count
    a = L.GroupNormArgs(fold_plan=None, fold_blocks=3)
    assert lib.encdiff_groupnorm_bwd(C.byref(a), None) < 0
    print(f"asan host checks: {n} calls, clean")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--checks", action="store_true")
    a = ap.parse_args()
    if a.checks:
        checks()
        return
    rt = asan_runtime()
    if rt is None:
        sys.exit("no libclang_rt.asan-x86_64.so under /opt/rocm/lib/llvm")
    lib = build()
    # the ASan runtime goes first; whatever the environment already preloads stays preloaded
    pre = " ".join(x for x in (rt, os.environ.get("LD_PRELOAD", "")) if x)
    env = dict(os.environ, LD_PRELOAD=pre, ENCDIFF_LIB=lib,
               ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0:alloc_dealloc_mismatch=0:"
                            "detect_odr_violation=0:halt_on_error=1")
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--checks"], env=env, capture_output=True, text=True)
    sys.stdout.write(r.stdout[-4000:])
    sys.stderr.write(r.stderr[-8000:])
    if r.returncode or "ERROR: AddressSanitizer" in r.stderr:
        sys.exit(1)


if __name__ == "__main__":
    main()
