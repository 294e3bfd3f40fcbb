#!/bin/bash
# Dev A/B (GPU box, repo root): the input DMA's cache policy on the mono
# lines (XM_AB_DMAPOL builds lib_ab_pol0 = nt, lib_ab_pol2 = default, against
# the product's sc1): timing (2 rounds) and one FETCH_SIZE pass per variant
set -o pipefail
OUT=gpurun_out/dmapol
mkdir -p $OUT
tools/dev/ab_cfg.sh 2 "mono1 c1s16 mono8" lib lib_ab_pol0 lib_ab_pol2 || exit 1
for l in lib lib_ab_pol0 lib_ab_pol2; do
  for c in mono1 c1s16; do
    XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/$l/libxm_audio.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/$l.$c -o run --output-format csv -- python3 tools/bench_configs.py $c --steps 2 --warmup 1 --no-check --no-box > $OUT/$l.$c.log 2>&1 || { tail -5 $OUT/$l.$c.log; exit 1; }
    python3 tools/dev/pmc_kernels.py --calls 3 $OUT/$l.$c | python3 -c "
import json,sys; d=json.load(sys.stdin); v=d['per_call'].get('k_rs147_mix',{}); print('$l', '$c', 'fetch_GB', round(v.get('fetch_GB',0),2))"
  done
done
