#!/bin/bash
# Dev A/B: config 4's time-block cut (XM_FX_CUT, block starts in 64ths) on one box
set -o pipefail
mkdir -p gpurun_out/c4cut
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in ${XM_CUTS:-"" "2,6,14,26,38,50,62"}; do
    XM_FX_CUT="$v" timeout -k 10 200 python3 -u tools/bench_configs.py c4 --steps 15 --warmup 3 --no-box > gpurun_out/c4cut/$i.log 2>&1 || { tail -5 gpurun_out/c4cut/$i.log; exit 1; }
    grep '^{' gpurun_out/c4cut/$i.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('[$v]', d['config'], d['ms_per_step'], d.get('parity_check'))"
  done
done
