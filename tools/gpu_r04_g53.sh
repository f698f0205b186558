#!/bin/bash
# B=8 (sampling) entries: tune at batch 8, merge its FORWARD problems over the table, A/B DDIM B=8.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u tools/gemm_profile.py --batch 8 --pairs 0 --write-table gpurun_out/gemm_tiles_b8.json > gpurun_out/g53_tune.log 2>&1 || { tail -5 gpurun_out/g53_tune.log; exit 1; }
tail -9 gpurun_out/g53_tune.log
python - <<'PY' || exit 1
import json
old = json.load(open("encdiff_amd/gemm_tiles.json"))
new = json.load(open("gpurun_out/gemm_tiles_b8.json"))
fwd = {k: v for k, v in new.items() if k.split(",")[:2] in (["0", "0"], ["1", "0"])}  # key: a_mode,b_mode,...
ch = sum(1 for k, v in fwd.items() if k not in old or old[k][:2] != v[:2])
m = dict(old); m.update(fwd)
json.dump(m, open("gpurun_out/gemm_tiles_b8merged.json", "w"), indent=0, sort_keys=True)
print("b8 tuned", len(new), "forward", len(fwd), "changed", ch)
PY
bash tools/ddim_env_ab.sh 8 200 "ENCDIFF_GEMM_TILES=" "ENCDIFF_GEMM_TILES=$R/gpurun_out/gemm_tiles_b8merged.json" "ENCDIFF_GEMM_TILES=" "ENCDIFF_GEMM_TILES=$R/gpurun_out/gemm_tiles_b8merged.json"
