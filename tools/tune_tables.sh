#!/bin/bash
# Re-tune the GEMM (tile, split) table on the current kernels (tools/gemm_profile.py; ONLY_H=2,4,8
# restricts the sweep to implicit-im2col problems at those sizes and keeps every other entry), merge
# it over the committed table, and A/B the training step with the two tables (two runs each).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
OH=${ONLY_H:+--only-h $ONLY_H}
timeout -k 10 840 python -u tools/gemm_profile.py $OH --write-table gpurun_out/gemm_tiles_tuned.json > gpurun_out/tune.log 2>&1 || { tail -5 gpurun_out/tune.log; exit 1; }
tail -12 gpurun_out/tune.log
python - <<'PY' || exit 1
import json
old = json.load(open("encdiff_amd/gemm_tiles.json"))
new = json.load(open("gpurun_out/gemm_tiles_tuned.json"))
ch = sum(1 for k, v in new.items() if k not in old or old[k][:2] != v[:2])
m = dict(old); m.update(new)
json.dump(m, open("gpurun_out/gemm_tiles_merged.json", "w"), indent=0, sort_keys=True)
print("tuned", len(new), "changed", ch, "merged", len(m))
PY
bash tools/gpu_iter.sh "ENCDIFF_GEMM_TILES=" "ENCDIFF_GEMM_TILES=$R/gpurun_out/gemm_tiles_merged.json"
