#!/bin/bash
# Re-tune the GEMM (tile, split) table at B=128 on the current kernels, merge it over the committed
# table (sampling entries kept), and A/B the step with the two tables.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 840 python -u tools/gemm_profile.py --write-table gpurun_out/gemm_tiles_tuned.json > gpurun_out/g50_tune.log 2>&1 || { tail -5 gpurun_out/g50_tune.log; exit 1; }
tail -12 gpurun_out/g50_tune.log
python - <<'PY' || exit 1
import json
old = json.load(open("encdiff_amd/gemm_tiles.json"))
new = json.load(open("gpurun_out/gemm_tiles_tuned.json"))
ch = sum(1 for k, v in new.items() if k not in old or old[k][:2] != v[:2] or (len(old[k]) > 3) != (len(v) > 3) or (len(v) > 3 and old[k][3] != v[3]))
m = dict(old); m.update(new)
json.dump(m, open("gpurun_out/gemm_tiles_merged.json", "w"), indent=0, sort_keys=True)
print("tuned", len(new), "changed", ch, "merged", len(m))
PY
bash tools/bench_ab.sh "ENCDIFF_GEMM_TILES=" "ENCDIFF_GEMM_TILES=$R/gpurun_out/gemm_tiles_merged.json" "ENCDIFF_GEMM_TILES=" "ENCDIFF_GEMM_TILES=$R/gpurun_out/gemm_tiles_merged.json"
