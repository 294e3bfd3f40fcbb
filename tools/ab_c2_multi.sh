#!/bin/bash
# Dev: config-2 time and WRITE_SIZE for lib/ and each lib_ab*/ variant (one box).
set -o pipefail
mkdir -p gpurun_out/abc2m
export TMPDIR=/tmp
for L in xm-audio-utils_amd/lib xm-audio-utils_amd/lib_ab xm-audio-utils_amd/lib_ab2 xm-audio-utils_amd/lib_ab3; do
  [ -f $L/libxm_audio.so ] || continue
  v=$(basename $L)
  XM_AUDIO_LIB=$PWD/$L/libxm_audio.so timeout -k 10 200 python3 tools/bench_configs.py c2 --steps 10 --warmup 2 > gpurun_out/abc2m/$v.log 2>&1 || { tail -5 gpurun_out/abc2m/$v.log; exit 1; }
  t=$(grep '^{' gpurun_out/abc2m/$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['kernel_ms'])")
  XM_AUDIO_LIB=$PWD/$L/libxm_audio.so timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/abc2m/h$v.log 2>&1 || { tail -5 gpurun_out/abc2m/h$v.log; exit 1; }
  h=$(grep '^{' gpurun_out/abc2m/h$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['parity_check'])")
  XM_AUDIO_LIB=$PWD/$L/libxm_audio.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/abc2m/w$v -o run --output-format csv -- python3 tools/bench_configs.py c2 --steps 2 --warmup 1 > gpurun_out/abc2m/w$v.log 2>&1 || { tail -5 gpurun_out/abc2m/w$v.log; exit 1; }
  w=$(python3 - gpurun_out/abc2m/w$v/run_counter_collection.csv <<'PY'
import csv, sys, collections
per = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_rs147" in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE":
        per[r["Dispatch_Id"]] += float(r["Counter_Value"])
v = list(per.values())
print(round(sum(v) / len(v) * 1024 / 1e9, 2))
PY
)
  echo "$v: c2 ${t} ms, write ${w} GB | headline ${h}"
done
