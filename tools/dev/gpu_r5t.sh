#!/bin/bash
# Round 5, box pass t: 2/1 and 3/1 mono and 2/1 stereo 1-track rows on the
# fused kernel: their GPU tests and the related suites, then the new shapes'
# lines against the generic kernel (lib_old: the previous launcher), same box.
set -o pipefail
mkdir -p gpurun_out/r5t
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fast_upsmall_rows.py tests/test_gpu_fast_small.py tests/test_gpu_fast_multisp.py tests/test_gpu_fast_u2.py tests/test_gpu_timeline.py tests/test_gpu_fast_mono.py > gpurun_out/r5t/pytest.txt 2>&1 || { tail -30 gpurun_out/r5t/pytest.txt; exit 1; }
tail -2 gpurun_out/r5t/pytest.txt
for L in lib lib_old; do
  XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/$L/libxm_audio.so timeout -k 10 400 python3 tools/bench_configs.py m24to48 m16to48 s24to48 m22to48 s22to48 --steps 10 --warmup 2 --no-box > gpurun_out/r5t/ab_$L.txt 2>&1 || { tail -5 gpurun_out/r5t/ab_$L.txt; exit 1; }
  grep '^{' gpurun_out/r5t/ab_$L.txt | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$L', d['config'], d.get('kernel'), d['ms_per_step'], d['roofline']['frac'], d.get('parity_check'))" | tee -a gpurun_out/r5t/ab.txt
done
