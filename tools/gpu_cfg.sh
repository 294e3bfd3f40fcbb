#!/bin/bash
# Dev: secondary config benches (tools/bench_configs.py), each under its own limit.
set -o pipefail
mkdir -p gpurun_out/cfg
timeout -k 10 200 python3 tools/bench_configs.py c2 c3 > gpurun_out/cfg/c23.log 2>&1; rc=$?
cat gpurun_out/cfg/c23.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/bench_configs.py c4 --steps 1 --warmup 1 > gpurun_out/cfg/c4.log 2>&1; rc=$?
cat gpurun_out/cfg/c4.log | grep -v amdgpu.ids; exit $rc
