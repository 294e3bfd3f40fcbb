#!/bin/bash
# Dev (GPU box, via gpurun): run named steps in order, each under its own time
# limit, output to gpurun_out/<tag>/<name>.log; stop at the first failure.
# Replaces round 5's single-use tools/dev/gpu_r5*.sh pass scripts.
#   tools/dev/gpu_steps.sh <tag> '<name>|<seconds>|<command>' ...
# e.g.
#   tools/dev/gpu_steps.sh r6a 'hbm|300|tools/ubench/bin/hbm_ceiling' \
#       'cfg|600|python3 -u tools/bench_configs.py c2 --steps 15'
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  tail -n 40 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; exit $rc; fi
done
echo "== done: $OUT"
