#!/bin/bash
# Round 5, box pass n: mono s16 grouped direct stores (DSG 4): the mono s16
# GPU tests, a same-box A/B of c1s16 against the previous kernel (lib_old),
# and WRITE_SIZE / SQ counters of the new one.
set -o pipefail
mkdir -p gpurun_out/r5n
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fast_mono16.py tests/test_gpu_fast_multisp.py tests/test_gpu_fast_small.py > gpurun_out/r5n/pytest.txt 2>&1 || { tail -30 gpurun_out/r5n/pytest.txt; exit 1; }
tail -2 gpurun_out/r5n/pytest.txt
for i in 1 2; do
  for L in lib lib_old; do
    XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/$L/libxm_audio.so timeout -k 10 200 python3 tools/bench_configs.py c1s16 --steps 50 --warmup 3 --no-box > gpurun_out/r5n/c1_$L.txt 2>&1 || { tail -5 gpurun_out/r5n/c1_$L.txt; exit 1; }
    echo "$L $(grep '^{' gpurun_out/r5n/c1_$L.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["ms_per_step"], d["roofline"]["frac"], d.get("parity_check"))')" | tee -a gpurun_out/r5n/ab.txt
  done
done
timeout -k 10 600 tools/dev/pmc_cfg.sh r5n/c1s16 c1s16 2 > /dev/null || exit 1
python3 -c "
import json
d=json.load(open('gpurun_out/r5n/c1s16/c1s16_pmc.json'))
for k,v in d.items():
    if isinstance(v,dict):
        for kk,vv in v.items():
            if isinstance(vv,dict) and 'k_rs147' in kk: print(kk, {x: vv[x] for x in ('write_GB','fetch_GB','SQ_INSTS_VALU','SQ_WAIT_INST_ANY','SQ_WAVE_CYCLES','SQ_INSTS_VMEM_WR') if x in vv})
"
