#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/bench_ab.sh "ENCDIFF_TABLE_WG=0" "ENCDIFF_TABLE_WG=1" "ENCDIFF_TABLE_WG=2" "ENCDIFF_TABLE_WG=0" "ENCDIFF_TABLE_WG=1" "ENCDIFF_TABLE_WG=2"
