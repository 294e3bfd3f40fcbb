#!/bin/bash
# Config-2 write amplification against the number of resident waves (dev; GPU
# box, repo root): the split-mode kernel at its default grid and with fewer,
# longer waves (XM_FAST_R: SPs per lane), each with its time and a WRITE_SIZE
# pass of its own.  Every step under its own limit; stop at the first failure.
#   tools/c2_occ.sh <tag> [R ...]
set -o pipefail
TAG=${1:-c2occ}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  grep -v amdgpu.ids $OUT/$name.log | tail -n 2
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; exit $rc; fi
}
for R in default "$@"; do
  if [ $R = default ]; then unset XM_FAST_R; else export XM_FAST_R=$R; fi
  step c2_$R 200 python3 tools/bench_configs.py c2 --steps 10 --warmup 2
  step write_$R 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_$R -o run --output-format csv -- python3 tools/bench_configs.py c2 --steps 2 --warmup 1
done
echo "c2_occ done: $OUT"
