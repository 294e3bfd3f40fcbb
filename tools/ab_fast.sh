#!/bin/bash
# Dev (GPU box): A/B of headline-kernel variants, alternating separate
# processes (same box, same data); "_chk" runs add the bit-exact check.
#   tools/ab_fast.sh name:ENV=..,ENV=.. ...   (lib_vN => XM_AUDIO_LIB=xm-audio-utils_amd/lib_vN/libxm_audio.so)
set -o pipefail
mkdir -p gpurun_out/ab
run() {   # run <name> <extra bench args> <env...>
  local name=$1 extra=$2; shift 2
  env "$@" timeout -k 10 120 python3 bench.py --steps 10 --warmup 3 --no-cpu $extra > gpurun_out/ab/$name.log 2>&1 || { echo "$name FAILED"; tail -3 gpurun_out/ab/$name.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab/$name.log') if l.startswith('{')][-1]); print('$name', d['ms_per_step'], d['roofline']['frac'], d.get('parity_check_2mixes'))"
}
specs=("$@")
envs() {   # spec -> env words
  local e=${1#*:}
  [ "$e" = "$1" ] && { echo XM_NONE=0; return; }
  echo $e | tr ',' ' ' | sed "s#lib_v\([0-9]*\)#XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/lib_v\1/libxm_audio.so#g"
}
for rnd in 1 2; do
  for sp in "${specs[@]}"; do run "${sp%%:*}" "" $(envs "$sp") || exit 1; done
done
for sp in "${specs[@]}"; do run "${sp%%:*}_chk" --check $(envs "$sp") || exit 1; done
