#!/bin/bash
# Round 5, box pass v: 147/320 stereo 1-track rows on the fused kernel: the
# 147/320 GPU tests and the timeline / parity suites, then the 1-track line
# against the generic kernel (lib_old: the previous 147/320 unit), same box.
set -o pipefail
mkdir -p gpurun_out/r5v
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fast_d2.py tests/test_gpu_timeline.py tests/test_gpu_parity.py tests/test_gpu_cpu_backend.py > gpurun_out/r5v/pytest.txt 2>&1 || { tail -30 gpurun_out/r5v/pytest.txt; exit 1; }
tail -2 gpurun_out/r5v/pytest.txt
for L in lib lib_old; do
  XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/$L/libxm_audio.so timeout -k 10 300 python3 tools/bench_configs.py s96to44 r96to44 --steps 10 --warmup 2 --no-box > gpurun_out/r5v/ab_$L.txt 2>&1 || { tail -5 gpurun_out/r5v/ab_$L.txt; exit 1; }
  grep '^{' gpurun_out/r5v/ab_$L.txt | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$L', d['config'], d.get('kernel'), d['ms_per_step'], d['roofline']['frac'], d.get('parity_check'))" | tee -a gpurun_out/r5v/ab.txt
done
