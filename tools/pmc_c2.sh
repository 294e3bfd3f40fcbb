#!/bin/bash
# Config-2 (resample-only split mode) timing and HBM PMC passes (dev; GPU box,
# repo root).  FETCH_SIZE and WRITE_SIZE in separate --pmc runs, never with a
# tracing domain; each step under its own limit, stop at the first failure.
#   tools/pmc_c2.sh <tag>
set -o pipefail
TAG=${1:-c2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  grep -v amdgpu.ids $OUT/$name.log | tail -n 3
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; exit $rc; fi
}
step list 60 rocprofv3 -L
step c2 200 python3 tools/bench_configs.py c2 --steps 10 --warmup 2
step fetch 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 tools/bench_configs.py c2 --steps 2 --warmup 1
step write 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 tools/bench_configs.py c2 --steps 2 --warmup 1
step wreq 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $OUT/wreq -o run --output-format csv -- python3 tools/bench_configs.py c2 --steps 2 --warmup 1
echo "pmc_c2 done: $OUT"
