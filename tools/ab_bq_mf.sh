#!/bin/bash
# Dev A/B (GPU box, repo root): config-4 biquad stage (tools/dev/bq_load.py)
# on the product library (k_biquad_lane for <= 16 sections), lib_ab
# (-DXM_BQ_PACKED_ONLY: k_biquad_pipe) and lib_ab2 (-DXM_BQ_MF: matrix-core
# products), alternating, each run under its own limit.
set -o pipefail
OUT=gpurun_out/${1:-bqmf}
mkdir -p $OUT
L=$PWD/xm-audio-utils_amd
for k in 1 2; do
  for v in lane:lib packed:lib_ab mf:lib_ab2; do
    n=${v%%:*}; d=${v##*:}
    echo "== $n $k"
    XM_AUDIO_LIB=$L/$d/libxm_audio.so timeout -k 10 120 python3 tools/dev/bq_load.py > $OUT/${n}_$k.log 2>&1 || exit $?
    grep -v amdgpu.ids $OUT/${n}_$k.log
  done
done
