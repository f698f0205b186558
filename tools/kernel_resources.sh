#!/bin/bash
# Print VGPR/SGPR/spill/LDS/scratch usage of every kernel in a .hip source (device-only compile,
# the library's flags).  usage: bash tools/kernel_resources.sh encdiff_amd/csrc/norm.hip [filter] [extra flags...]
set -e
SRC=$1; FILT=${2:-.}; shift 2 || true
OUT=$(mktemp /tmp/kres.XXXXXX.co)
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=fast -mllvm -amdgpu-mfma-vgpr-form=1 -Iinclude "$@" --cuda-device-only --no-gpu-bundle-output -c "$SRC" -o "$OUT"
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$OUT" | awk '
  /\.name:/ {name=$2}
  /\.vgpr_count:/ {v=$2} /\.sgpr_count:/ {s=$2}
  /\.vgpr_spill_count:/ {vs=$2} /\.private_segment_fixed_size:/ {ps=$2}
  /\.group_segment_fixed_size:/ {lds=$2}
  /\.wavefront_size:/ {printf "%-90s vgpr=%s sgpr=%s spill=%s scratch=%s lds=%s\n", substr(name,1,90), v, s, vs, ps, lds}' | grep -E "$FILT"
rm -f "$OUT"
