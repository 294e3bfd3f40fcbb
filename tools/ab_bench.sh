#!/bin/bash
# Dev A/B on one GPU box (repo root): the headline bench alternating between
# the product library (A = lib/) and a variant build (B = lib_ab/, `make ab`),
# N rounds, each run under its own limit.   tools/ab_bench.sh [rounds] [bench args]
set -o pipefail
N=${1:-3}; shift
ARGS=${@:---steps 20 --warmup 5 --no-cpu}
mkdir -p gpurun_out/ab
LA=xm-audio-utils_amd/lib/libxm_audio.so
LB=xm-audio-utils_amd/lib_ab/libxm_audio.so
for i in $(seq 1 $N); do
  for v in A B; do
    L=$LA; [ $v = B ] && L=$LB
    XM_AUDIO_LIB=$PWD/$L timeout -k 10 200 python3 -u bench.py $ARGS > gpurun_out/ab/$v$i.log 2>&1 || { tail -5 gpurun_out/ab/$v$i.log; exit 1; }
    grep '^{' gpurun_out/ab/$v$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['roofline']['frac'], d.get('parity_check'))"
  done
done
