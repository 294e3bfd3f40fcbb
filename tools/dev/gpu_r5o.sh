#!/bin/bash
# Round 5, box pass o: the whole GPU suite on the grouped direct stores (mono
# s16 and f32 1-track rows), same-box A/B of mono1 / c1s16 against lib_old
# (the kernels before the grouping), the mono1 PMC, and a WRITE_SIZE survey
# of the other config lines (write amplification of their store forms).
set -o pipefail
mkdir -p gpurun_out/r5o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5o/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/r5o/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/r5o/pytest_gpu.txt
for i in 1 2; do
  for L in lib lib_old; do
    XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/$L/libxm_audio.so timeout -k 10 300 python3 tools/bench_configs.py mono1 c1s16 --steps 30 --warmup 3 --no-box > gpurun_out/r5o/ab_$L.txt 2>&1 || { tail -5 gpurun_out/r5o/ab_$L.txt; exit 1; }
    grep '^{' gpurun_out/r5o/ab_$L.txt | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$L', d['config'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_check'))" | tee -a gpurun_out/r5o/ab.txt
  done
done
timeout -k 10 600 tools/dev/pmc_cfg.sh r5o/mono1 mono1 2 > /dev/null || exit 1
for c in s16rs oconv planar conv up mono8 r32to48 r24to48 r16to48 r44to96 r96to44 odd c3; do
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r5o/w_$c -o run --output-format csv -- python3 tools/bench_configs.py $c --steps 1 --warmup 1 --no-check --no-box > gpurun_out/r5o/w_$c.log 2>&1 || { tail -5 gpurun_out/r5o/w_$c.log; exit 1; }
  python3 tools/dev/pmc_kernels.py --calls 2 --out gpurun_out/r5o/w_$c.json gpurun_out/r5o/w_$c > /dev/null || exit 1
  echo "$c $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5o/w_$c.log | head -1) $(python3 -c "
import json
d=json.load(open('gpurun_out/r5o/w_$c.json'))
for k,v in d.items():
    if isinstance(v,dict):
        for kk,vv in v.items():
            if isinstance(vv,dict) and 'write_GB' in vv and vv['write_GB']>0.5: print(kk, round(vv['write_GB'],3), end='; ')
")" | tee -a gpurun_out/r5o/write_survey.txt
done
