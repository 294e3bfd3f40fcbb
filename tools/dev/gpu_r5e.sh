#!/bin/bash
# Round 5, box pass e: strong-scaling shards (bench.py --global-clips G = the
# per-GPU block of N = 4096 / G GPUs) under forced super-period runs
# (XM_FAST_SPLIT_R), against pick_split's choice.
set -o pipefail
mkdir -p gpurun_out/r5e
run() {   # run <label> <global clips> [R]
  local lab=$1 g=$2 r=$3
  XM_FAST_SPLIT_R=$r timeout -k 10 120 python3 -u bench.py --global-clips $g --steps 30 --warmup 5 --no-cpu > gpurun_out/r5e/$lab.log 2>&1 || { tail -5 gpurun_out/r5e/$lab.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r5e/$lab.log') if l.startswith('{')][-1]); print('$lab', d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('parity_check'))"
}
for it in 1 2; do
  run g512_auto 512 || exit 1
  for r in 13 14 16 20; do run g512_r$r 512 $r || exit 1; done
  run g1024_auto 1024 || exit 1
  for r in 26 28 32; do run g1024_r$r 1024 $r || exit 1; done
done
