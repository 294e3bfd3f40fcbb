#!/bin/bash
# Dev A/B of the effects kernels (one box): effects parity tests on lib_ab/,
# then the config-4 biquad stage alone and config 4 end to end for A = lib/, B = lib_ab/.
set -o pipefail
mkdir -p gpurun_out/abbq
LB=$PWD/xm-audio-utils_amd/lib_ab/libxm_audio.so
XM_AUDIO_LIB=$LB timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "biquad or effects or fir or stream or track_eq or chain or multi_track_effects" > gpurun_out/abbq/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/abbq/pytest.log; [ $rc -ne 0 ] && exit $rc
for v in A B; do
  L=$PWD/xm-audio-utils_amd/lib/libxm_audio.so; [ $v = B ] && L=$LB
  XM_AUDIO_LIB=$L timeout -k 10 200 python3 tools/dev/bq_load.py > gpurun_out/abbq/bq$v.log 2>&1 || { tail -5 gpurun_out/abbq/bq$v.log; exit 1; }
  echo "$v $(grep pass gpurun_out/abbq/bq$v.log | tail -1)"
  XM_AUDIO_LIB=$L timeout -k 10 300 python3 tools/bench_configs.py c4 --steps 2 --warmup 1 > gpurun_out/abbq/c4$v.log 2>&1 || { tail -5 gpurun_out/abbq/c4$v.log; exit 1; }
  grep '^{' gpurun_out/abbq/c4$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v c4', d['ms_per_step'], d['kernel_ms'])"
done
