#!/bin/bash
# One GPU-box pass (run from the repo root via gpurun): GPU parity tests,
# smoke, a checked bench line, the rocprofv3 kernel-trace summary and the two
# HBM PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs, never combined
# with a tracing domain).  Every GPU step has its own time limit and the
# script stops at the first failure.
#   tools/gpu_check.sh <tag> [--no-tests] [--no-prof]
set -o pipefail
TAG=${1:-r1}; shift
TESTS=1; PROF=1
for a in "$@"; do
  case $a in --no-tests) TESTS=0 ;; --no-prof) PROF=0 ;; esac
done
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
DRIVER="--gpus 1 --steps 20 --warmup 5"          # the driver's bench command line
PMCB="--steps 3 --warmup 1 --no-cpu --no-check"
step() {   # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  tail -n 5 $OUT/$name.log
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; exit $rc; fi
}
rocminfo 2>/dev/null | grep -m3 -E 'gfx950|Compute Unit' > $OUT/rocminfo.txt || true
nproc > $OUT/nproc.txt
python3 -c "import bench; print(bench.kernel_src_sha256())" > $OUT/kernel_src.sha256
if [ $TESTS = 1 ]; then
  step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 400 python3 -u bench.py $DRIVER
if [ $PROF = 1 ]; then
  # the same invocation under the kernel-trace profiler: its bench line and
  # its per-kernel average come from one run (profiles/<tag>_trace_bench.json)
  step trace 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $DRIVER
  step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py $PMCB
  step pmc_write 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py $PMCB
  step pmc_sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py $PMCB
fi
echo "gpu_check done: $OUT"
