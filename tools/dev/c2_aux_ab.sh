#!/bin/bash
# Dev (GPU box): config-2 store cache-policy A/B (lib, lib_ab, lib_ab2) with a
# WRITE_SIZE pass each.
mkdir -p gpurun_out/c2aux
for v in A B C; do
  L=xm-audio-utils_amd/lib/libxm_audio.so
  [ $v = B ] && L=xm-audio-utils_amd/lib_ab/libxm_audio.so
  [ $v = C ] && L=xm-audio-utils_amd/lib_ab2/libxm_audio.so
  XM_AUDIO_LIB=$PWD/$L timeout -k 10 200 python3 -u tools/bench_configs.py c2 > gpurun_out/c2aux/$v.log 2>&1 || exit 1
  echo $v $(grep -o "\"ms_per_step\": [0-9.]*\|\"parity_check\": [a-z]*" gpurun_out/c2aux/$v.log)
  XM_AUDIO_LIB=$PWD/$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/c2aux/w$v -o run --output-format csv -- python3 tools/bench_configs.py c2 --steps 2 --warmup 1 --no-check > gpurun_out/c2aux/w$v.log 2>&1 || exit 1
  python3 - gpurun_out/c2aux/w$v/run_counter_collection.csv <<'PY'
import csv, sys
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(sys.argv[1])) if "k_rs147" in r["Kernel_Name"]]
print("  WRITE_SIZE KiB per launch", sum(v) / len(v), "x1024 / 14.45e9 =", sum(v) / len(v) * 1024 / 14.45e9)
PY
done
