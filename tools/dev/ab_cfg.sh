#!/bin/bash
# Dev A/B on one GPU box (repo root): config lines alternating between library
# builds (a name X means xm-audio-utils_amd/X/libxm_audio.so, `lib` the
# product), R rounds, each run under its own limit; every line bit-checked.
#   tools/dev/ab_cfg.sh <rounds> "<configs>" <lib> <lib> ...
set -o pipefail
R=$1; CFGS=$2; shift 2
mkdir -p gpurun_out/abcfg
for i in $(seq 1 $R); do
  for l in "$@"; do
    L=$PWD/xm-audio-utils_amd/$l/libxm_audio.so
    XM_AUDIO_LIB=$L timeout -k 10 400 python3 -u tools/bench_configs.py $CFGS --steps 10 --warmup 3 --no-box \
      > gpurun_out/abcfg/$l.$i.log 2>&1 || { tail -5 gpurun_out/abcfg/$l.$i.log; exit 1; }
    grep '^{' gpurun_out/abcfg/$l.$i.log | python3 -c "
import json, sys
for ln in sys.stdin:
    d = json.loads(ln)
    print('$l', '$i', d['config'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_check'))"
  done
done
