#!/bin/bash
# Dev A/B for config 2 (resample-only split mode) over several builds:
#   tools/ab_c2_multi.sh <tag> <name:libdir> ...   (libdir under xm-audio-utils_amd/)
# Two alternating timing rounds (bench_configs c2), then one WRITE_SIZE pass
# per build; every step under its own limit, stop at the first failure.
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for k in 1 2; do
  for v in "$@"; do
    n=${v%%:*}; L=$PWD/xm-audio-utils_amd/${v##*:}/libxm_audio.so
    XM_AUDIO_LIB=$L timeout -k 10 200 python3 tools/bench_configs.py c2 --steps 10 --warmup 2 > $OUT/$n$k.log 2>&1 || { tail -5 $OUT/$n$k.log; exit 1; }
    grep '^{' $OUT/$n$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['kernel_ms'], d['roofline']['frac'])"
  done
done
for v in "$@"; do
  n=${v%%:*}; L=$PWD/xm-audio-utils_amd/${v##*:}/libxm_audio.so
  XM_AUDIO_LIB=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/w$n -o run --output-format csv -- python3 tools/bench_configs.py c2 --steps 2 --warmup 1 > $OUT/w$n.log 2>&1 || { tail -5 $OUT/w$n.log; exit 1; }
  python3 - $OUT/w$n/run_counter_collection.csv $n <<'PY'
import csv, sys, collections
per = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_rs147" in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE":
        per[r["Dispatch_Id"]] += float(r["Counter_Value"])
v = list(per.values())
print(sys.argv[2], "WRITE_SIZE GB per launch", round(sum(v) / len(v) * 1024 / 1e9, 2))
PY
done
