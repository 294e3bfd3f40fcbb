#!/bin/bash
# Dev: k_biquad_pc ablation variants (profiling builds, results not checked), one box.
set -o pipefail
OUT=gpurun_out/${1:-bqra}; shift; mkdir -p $OUT
for v in "$@"; do
  XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/$v/libxm_audio.so timeout -k 10 200 python3 tools/dev/bq_load.py > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
  echo "== $v"; grep -v "amdgpu.ids\|SIMD of" $OUT/$v.log
done
