#!/bin/bash
# The whole -m gpu suite and smoke(), as the driver runs them at round end.  TAG=<name> (outputs gpurun_out/TAG_*)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG:-suite}_gpu_tests.txt 2>&1 || { grep -E "FAIL|Error" gpurun_out/${TAG:-suite}_gpu_tests.txt | head -20; tail -5 gpurun_out/${TAG:-suite}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG:-suite}_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG:-suite}_smoke.txt 2>&1 || { tail -20 gpurun_out/${TAG:-suite}_smoke.txt; exit 1; }
tail -3 gpurun_out/${TAG:-suite}_smoke.txt
