#!/bin/bash
# Dev A/B of the biquad stage (one box): A = lib/ (product), B = lib_ab/.
# The config-4 biquad stage alone (tools/dev/bq_load.py) and config 4 end to
# end, alternating A B A B.
set -o pipefail
OUT=gpurun_out/${1:-abbq2}; mkdir -p $OUT
LB=$PWD/xm-audio-utils_amd/lib_ab/libxm_audio.so
for rep in 1 2; do
for v in A B; do
  L=$PWD/xm-audio-utils_amd/lib/libxm_audio.so; [ $v = B ] && L=$LB
  XM_AUDIO_LIB=$L timeout -k 10 200 python3 tools/dev/bq_load.py > $OUT/bq$v$rep.log 2>&1 || { tail -5 $OUT/bq$v$rep.log; exit 1; }
  echo "$v $(grep pass $OUT/bq$v$rep.log | tail -1)"
  XM_AUDIO_LIB=$L timeout -k 10 300 python3 tools/bench_configs.py c4 --steps 2 --warmup 1 > $OUT/c4$v$rep.log 2>&1 || { tail -5 $OUT/c4$v$rep.log; exit 1; }
  grep '^{' $OUT/c4$v$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v c4', d['ms_per_step'], d['kernel_ms'], d.get('parity_check'))"
done
done
