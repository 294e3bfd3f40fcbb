#!/bin/bash
# Dev A/B of effects-kernel variants (one box): for each lib_ab<N>/ given,
# the effects parity tests, then the config-4 biquad stage alone (bq_load.py).
#   tools/ab_bq_multi.sh 1 2 3 ...
set -o pipefail
mkdir -p gpurun_out/abbq
for n in "$@"; do
  L=$PWD/xm-audio-utils_amd/lib_ab$n/libxm_audio.so
  XM_AUDIO_LIB=$L timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "biquad or effects or fir or stream or track_eq or chain" > gpurun_out/abbq/pytest$n.log 2>&1
  rc=$?; echo "v$n $(tail -1 gpurun_out/abbq/pytest$n.log)"; [ $rc -ne 0 ] && exit $rc
  XM_AUDIO_LIB=$L timeout -k 10 200 python3 tools/dev/bq_load.py > gpurun_out/abbq/bq$n.log 2>&1 || { tail -5 gpurun_out/abbq/bq$n.log; exit 1; }
  echo "v$n $(grep pass gpurun_out/abbq/bq$n.log | tail -1)"
done
