#!/bin/bash
# Round 5, box pass p: address-grid segment stores for the odd-N mixes and
# sc1 whole-segment stores for the 44.1k->48k / 320/147 mixes: fused-kernel
# GPU tests, a same-box A/B against lib_old (those parts before the change)
# and WRITE_SIZE of the changed lines.
set -o pipefail
mkdir -p gpurun_out/r5p
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fast_multisp.py tests/test_gpu_fast_small.py tests/test_gpu_headline.py tests/test_gpu_fast_u2.py tests/test_gpu_streaming.py tests/test_gpu_fast_convert.py tests/test_gpu_api_edges.py tests/test_gpu_production_grids.py > gpurun_out/r5p/pytest.txt 2>&1 || { tail -30 gpurun_out/r5p/pytest.txt; exit 1; }
tail -2 gpurun_out/r5p/pytest.txt
for i in 1 2; do
  for L in lib lib_old; do
    XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/$L/libxm_audio.so timeout -k 10 300 python3 tools/bench_configs.py odd up r44to96 ptrs c2 --steps 30 --warmup 3 --no-box > gpurun_out/r5p/ab_$L.txt 2>&1 || { tail -5 gpurun_out/r5p/ab_$L.txt; exit 1; }
    grep '^{' gpurun_out/r5p/ab_$L.txt | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$L', d['config'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_check'))" | tee -a gpurun_out/r5p/ab.txt
  done
done
for c in odd up r44to96; do
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r5p/w_$c -o run --output-format csv -- python3 tools/bench_configs.py $c --steps 1 --warmup 1 --no-check --no-box > gpurun_out/r5p/w_$c.log 2>&1 || { tail -5 gpurun_out/r5p/w_$c.log; exit 1; }
  python3 tools/dev/pmc_kernels.py --calls 2 --out gpurun_out/r5p/w_$c.json gpurun_out/r5p/w_$c > /dev/null || exit 1
  echo "$c $(python3 -c "
import json
d=json.load(open('gpurun_out/r5p/w_$c.json'))
for k,v in d.items():
    if isinstance(v,dict):
        for kk,vv in v.items():
            if isinstance(vv,dict) and 'write_GB' in vv and 'k_rs' in kk: print(kk, round(vv['write_GB'],3), end='; ')
")" | tee -a gpurun_out/r5p/write.txt
done
