#!/bin/bash
# Dev A/B on one GPU box (repo root): the headline bench line alternating
# between library builds (a name X means xm-audio-utils_amd/X/libxm_audio.so,
# `lib` the product), R rounds, each run under its own limit; the bench's
# parity check stays on, so every variant is also bit-checked.
#   tools/ab_libs.sh <rounds> <lib> <lib> ... [-- bench args]
set -o pipefail
R=$1; shift
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" = "--" ] && shift
ARGS=${@:---steps 20 --warmup 5 --no-cpu}
mkdir -p gpurun_out/ab
for i in $(seq 1 $R); do
  for l in "${LIBS[@]}"; do
    L=$PWD/xm-audio-utils_amd/$l/libxm_audio.so
    XM_AUDIO_LIB=$L timeout -k 10 200 python3 -u bench.py $ARGS > gpurun_out/ab/$l.$i.log 2>&1 || { tail -5 gpurun_out/ab/$l.$i.log; exit 1; }
    grep '^{' gpurun_out/ab/$l.$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$l', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d.get('parity_check'))"
  done
done
