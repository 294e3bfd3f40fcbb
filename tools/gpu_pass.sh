#!/bin/bash
# GPU pass (from the repo root via gpurun): GPU tests, smoke, the driver's
# bench line, the one-process sharded bench forms, config 5, the loud
# failure of --gpus N beyond the visible devices, and optionally config
# lines.  Each GPU step has its own time
# limit; the script stops at the first failure.
#   tools/gpu_pass.sh <tag> [--no-tests] [--no-bench] [--configs "c2 c3 ..."]
set -o pipefail
TAG=${1:-r3}; shift
TESTS=1; BENCH=1; CFGS=""
while [ $# -gt 0 ]; do
  case $1 in --no-tests) TESTS=0 ;; --no-bench) BENCH=0 ;; --configs) CFGS=$2; shift ;; esac
  shift
done
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  tail -n 4 $OUT/$name.log
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; exit $rc; fi
}
if [ $TESTS = 1 ]; then
  step pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
if [ $BENCH = 1 ]; then
  step bench 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  step bench_dev00 400 python3 -u bench.py --devices 0,0 --steps 10 --warmup 3 --no-cpu
  echo "== bench --gpus 2 on a 1-GPU box (must fail loudly)"
  if timeout -k 10 120 python3 bench.py --gpus 2 --steps 1 --warmup 0 --no-cpu > $OUT/bench_gpus2.log 2>&1; then
    echo "== bench --gpus 2 did NOT fail"; exit 1
  fi
  tail -n 2 $OUT/bench_gpus2.log
  step bench_c5 400 python3 -u bench.py --config c5 --steps 5 --warmup 2
  step bench_c5_dev8 400 python3 -u bench.py --config c5 --devices 0,0,0,0,0,0,0,0 --steps 5 --warmup 2 --no-cpu
fi
if [ -n "$CFGS" ]; then
  step configs 900 python3 -u tools/bench_configs.py $CFGS
fi
echo "gpu_pass done: $OUT"
