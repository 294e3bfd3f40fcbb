#!/bin/bash
set -o pipefail
# Dev A/B: config 4 and the biquad stage under the placement knobs
# XM_FX_KSPLIT (biquad CUs per 32) and XM_BQ_LDS (one workgroup per CU)
mkdir -p gpurun_out/r6h
for i in 1 2; do
  for v in "" "XM_FX_KSPLIT=24" "XM_FX_KSPLIT=24 XM_BQ_LDS=90000" "XM_BQ_LDS=90000"; do
    env $v timeout -k 10 300 python3 -u tools/bench_configs.py c4 bq --steps 10 --warmup 3 --no-box > gpurun_out/r6h/c4_$i.log 2>&1 || { tail -5 gpurun_out/r6h/c4_$i.log; exit 1; }
    grep '^{' gpurun_out/r6h/c4_$i.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('[$v]', d['config'], d['ms_per_step'], d.get('parity_check'))"
  done
done
