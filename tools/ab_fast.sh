#!/bin/bash
# Dev (GPU box): A/B of headline-kernel variants, alternating separate
# processes (same box, same data), then parity (--check) of each variant and
# the instruction-cache counters of two of them.
set -o pipefail
mkdir -p gpurun_out/ab
L2=$PWD/xm-audio-utils_amd/lib_v2/libxm_audio.so
run() {   # run <name> <env...>
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 bench.py --steps 10 --warmup 3 --no-cpu $EXTRA > gpurun_out/ab/$name.log 2>&1 || { echo "$name FAILED"; tail -3 gpurun_out/ab/$name.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab/$name.log') if l.startswith('{')][-1]); print('$name', d['ms_per_step'], d['roofline']['frac'], d.get('parity_check_2mixes'))"
}
for rnd in 1 2; do
  run base XM_X=0
  run wpb8 XM_FAST_WPB=8
  run cg16 XM_AUDIO_LIB=$L2
  run cg16wpb8 XM_AUDIO_LIB=$L2 XM_FAST_WPB=8
done
EXTRA=--check
run base_chk XM_X=0
run wpb8_chk XM_FAST_WPB=8
run cg16_chk XM_AUDIO_LIB=$L2
run cg16wpb8_chk XM_AUDIO_LIB=$L2 XM_FAST_WPB=8
EXTRA=
bash tools/pmc_icache.sh ic_base || exit 1
XM_FAST_WPB=8 bash tools/pmc_icache.sh ic_wpb8 || exit 1
