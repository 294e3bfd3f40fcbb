#!/bin/bash
# Dev (GPU box): mono tests on the product lib, then the mono lines A (lib:
# the store variant under test) / B (lib_ab: the A/B macro it was built with) with a
# WRITE_SIZE pass each.
mkdir -p gpurun_out/mpab
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fast_mono.py tests/test_gpu_fast_up.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mpab/pytest.log 2>&1 || { tail -30 gpurun_out/mpab/pytest.log; exit 1; }
tail -2 gpurun_out/mpab/pytest.log
for v in A B A B; do
  L=xm-audio-utils_amd/lib/libxm_audio.so
  [ $v = B ] && L=xm-audio-utils_amd/lib_ab/libxm_audio.so
  XM_AUDIO_LIB=$PWD/$L timeout -k 10 200 python3 -u tools/bench_configs.py mono1 mono8 > gpurun_out/mpab/$v.log 2>&1 || exit 1
  echo $v $(grep -o "\"config\": \"[a-z0-9]*\"\|\"ms_per_step\": [0-9.]*\|\"parity_check\": [a-z]*" gpurun_out/mpab/$v.log)
done
for v in A B; do
  L=xm-audio-utils_amd/lib/libxm_audio.so
  [ $v = B ] && L=xm-audio-utils_amd/lib_ab/libxm_audio.so
  XM_AUDIO_LIB=$PWD/$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/mpab/w$v -o run --output-format csv -- python3 tools/bench_configs.py mono1 --steps 2 --warmup 1 --no-check > gpurun_out/mpab/w$v.log 2>&1 || exit 1
  python3 - gpurun_out/mpab/w$v/run_counter_collection.csv <<'PY'
import csv, sys
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(sys.argv[1])) if "k_rs147" in r["Kernel_Name"]]
print("  WRITE_SIZE KiB per launch", sum(v) / len(v), "x1024 / 15.73e9 =", sum(v) / len(v) * 1024 / (8192 * 480000 * 4))
PY
done
