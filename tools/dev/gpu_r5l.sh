#!/bin/bash
# Round 5, box pass l: per-wave start/end/place records of single fused-kernel
# launches (the -DXM_CLOCK_STAMPS build in lib_clk) at the strong-scaling
# blocks (64 and 128 mixes) and the headline (512); the fused-kernel GPU tests
# (with the dynamic-tail cases), then the 64/128-mix blocks with and without
# a forced tail.
set -o pipefail
mkdir -p gpurun_out/r5l
export XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/lib_clk/libxm_audio.so
for m in 64 128 512; do
  timeout -k 10 240 python3 -u tools/dev/clock_stamp.py --mixes $m --seconds 2 --steps 20 --waves 4 --label m$m >> gpurun_out/r5l/waves.jsonl 2> gpurun_out/r5l/err_$m.txt || { tail -20 gpurun_out/r5l/err_$m.txt; exit 1; }
done
unset XM_AUDIO_LIB
cut -c1-300 gpurun_out/r5l/waves.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fast_tail.py tests/test_gpu_fast_multisp.py tests/test_gpu_fast_small.py tests/test_gpu_headline.py tests/test_gpu_fast_u2.py tests/test_gpu_fast_mono16.py tests/test_gpu_fast_convert.py > gpurun_out/r5l/pytest_fast.txt 2>&1 || { tail -30 gpurun_out/r5l/pytest_fast.txt; exit 1; }
tail -2 gpurun_out/r5l/pytest_fast.txt
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5l/bench.jsonl 2>&1 || { tail -5 gpurun_out/r5l/bench.jsonl; exit 1; }
grep '^{' gpurun_out/r5l/bench.jsonl | cut -c1-200
for g in 512 1024; do
  for t in "" 15:1 25:1 25:2 35:1 50:1; do
    XM_FAST_TAIL=$t timeout -k 10 120 python3 bench.py --steps 50 --warmup 10 --global-clips $g > gpurun_out/r5l/blk.txt 2>&1 || { tail -5 gpurun_out/r5l/blk.txt; exit 1; }
    echo "clips=$g tail=$t $(grep '^{' gpurun_out/r5l/blk.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["ms_per_step"], d.get("parity_check"))')" | tee -a gpurun_out/r5l/blocks.txt
  done
done
