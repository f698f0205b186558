#!/bin/bash
# DDIM steps/s (tools/ddim_prof.py) A/B over environment settings:  bash tools/ddim_env_ab.sh B S "A=0" "A=1 C=2" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
B=$1; S=$2; shift 2
for e in "$@"; do
  env $e timeout -k 10 200 python tools/ddim_prof.py --batch $B --steps $S > gpurun_out/ddim_env.log 2>&1 || { tail -5 gpurun_out/ddim_env.log; exit 1; }
  echo "$e: $(tail -1 gpurun_out/ddim_env.log)"
done
