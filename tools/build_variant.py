"""Build an A/B variant of libencdiff_hip.so with extra compile flags for some sources (the rest
reuse the default objects): encdiff_amd/_ab/libencdiff_hip_<name>.so, selected at run time with
ENCDIFF_LIB=<path> (encdiff_amd/_lib.py).

    python tools/build_variant.py NAME "gemm.hip:-DED_FRAG_PIPE=0" ["norm.hip:-DFOO=1" ...]
"""
from __future__ import annotations

import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from encdiff_amd import build as B  # noqa: E402


def main():
    name = sys.argv[1]
    extra = {}
    for spec in sys.argv[2:]:
        f, flags = spec.split(":", 1)
        extra[f] = flags.split()
    B.build()  # default objects up to date
    outd = os.path.join(B.HERE, "_ab")
    os.makedirs(outd, exist_ok=True)
    objs = []
    for s in B._sources():
        base = os.path.basename(s)
        o = os.path.join(B.OBJ, base + f".{B.ARCH}.o")
        if base in extra:
            o = os.path.join(outd, base + f".{name}.o")
            cmd = [B.HIPCC, *B.FLAGS, *B.FILE_FLAGS.get(base, []), *extra[base], "-c", s, "-o", o]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode:
                raise SystemExit(r.stderr)
        objs.append(o)
    lib = os.path.join(outd, f"libencdiff_hip_{name}.so")
    r = subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib, *objs],
                       capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr)
    print(lib)


if __name__ == "__main__":
    main()
