#!/bin/bash
# Dev (GPU box): build and run one microbenchmark from tools/ubench.
#   tools/gpu_ub.sh <name> [seconds]
set -o pipefail
mkdir -p gpurun_out/ub /tmp/ub
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -w $UBFLAGS -o /tmp/ub/$1 tools/ubench/$1.hip || exit 1
timeout -k 10 ${2:-120} /tmp/ub/$1 > gpurun_out/ub/$1.txt 2>&1
rc=$?
cat gpurun_out/ub/$1.txt
exit $rc
