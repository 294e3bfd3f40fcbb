#!/bin/bash
# Dev (GPU box): microbenchmarks + ablation attribution of the headline kernel.
set -o pipefail
mkdir -p gpurun_out/u1 /tmp/ub
for f in mem_pattern valu_rate dep_latency; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -w -o /tmp/ub/$f tools/ubench/$f.hip || exit 1
done
timeout -k 10 120 /tmp/ub/mem_pattern > gpurun_out/u1/mem.txt 2>&1 && \
timeout -k 10 120 /tmp/ub/valu_rate > gpurun_out/u1/valu.txt 2>&1 && \
timeout -k 10 120 /tmp/ub/dep_latency > gpurun_out/u1/dep.txt 2>&1 && \
timeout -k 10 400 python3 tools/ablate.py base ctaps abl1 abl2 > gpurun_out/u1/ablate.txt 2>&1 && \
timeout -k 10 120 python3 tools/prof_fast.py > gpurun_out/u1/prof.txt 2>&1
rc=$?
cat gpurun_out/u1/*.txt
exit $rc
