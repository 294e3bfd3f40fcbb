#!/bin/bash
# Dev: rocprofv3 kernel-trace summary of one command.  tools/gpu_trace.sh <tag> <cmd...>
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/tr_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$TAG -o run --output-format csv -- "$@" > gpurun_out/tr_$TAG/log.txt 2>&1
rc=$?
grep '^{' gpurun_out/tr_$TAG/log.txt
python3 - "$TAG" <<'PY'
import csv, glob, sys
for f in glob.glob(f"gpurun_out/tr_{sys.argv[1]}/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:90]:90s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:9.4f}")
PY
exit $rc
