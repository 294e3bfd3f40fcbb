#!/bin/bash
# Dev A/B for config 2 (resample-only split mode): A = lib/, B = lib_ab/;
# time (bench_configs c2) and WRITE_SIZE per variant, each step limited.
set -o pipefail
mkdir -p gpurun_out/abc2
export TMPDIR=/tmp
for v in A B; do
  L=$PWD/xm-audio-utils_amd/lib/libxm_audio.so; [ $v = B ] && L=$PWD/xm-audio-utils_amd/lib_ab/libxm_audio.so
  XM_AUDIO_LIB=$L timeout -k 10 200 python3 tools/bench_configs.py c2 --steps 10 --warmup 2 > gpurun_out/abc2/$v.log 2>&1 || { tail -5 gpurun_out/abc2/$v.log; exit 1; }
  grep '^{' gpurun_out/abc2/$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v c2', d['kernel_ms'], d['roofline']['frac'])"
  XM_AUDIO_LIB=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/abc2/w$v -o run --output-format csv -- python3 tools/bench_configs.py c2 --steps 2 --warmup 1 > gpurun_out/abc2/w$v.log 2>&1 || { tail -5 gpurun_out/abc2/w$v.log; exit 1; }
  python3 - gpurun_out/abc2/w$v/run_counter_collection.csv $v <<'PY'
import csv, sys, collections
per = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_rs147" in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE":
        per[r["Dispatch_Id"]] += float(r["Counter_Value"])
v = list(per.values())
print(sys.argv[2], "WRITE_SIZE GB per launch", round(sum(v) / len(v) * 1024 / 1e9, 2))
PY
done
