#!/bin/bash
# Dev: GPU parity tests (optionally filtered) then optional extra commands.
#   tools/gpu_quick.sh "<pytest -k expr or empty>" [cmd ...]
set -o pipefail
mkdir -p gpurun_out/q
K=${1:-}; shift
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${KA[@]}" > gpurun_out/q/pytest.log 2>&1
rc=$?; tail -n 15 gpurun_out/q/pytest.log; [ $rc -ne 0 ] && exit $rc
for c in "$@"; do
  echo "== $c"
  timeout -k 10 300 bash -c "$c" > gpurun_out/q/cmd.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/q/cmd.log | tail -n 20; [ $rc -ne 0 ] && exit $rc
done
exit 0
