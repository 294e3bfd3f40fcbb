#!/bin/bash
# Dev only: the headline kernel's in-kernel clock (diagnostic build lib_clk,
# tools/dev/clock_stamp.py) next to the product bench line on the same box.
# Output: gpurun_out/clk/*.jsonl
set -o pipefail
mkdir -p gpurun_out/clk
O=gpurun_out/clk
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_a.jsonl 2> $O/bench_a.err && \
XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/lib_clk/libxm_audio.so timeout -k 10 200 python tools/dev/clock_stamp.py --label synth > $O/clock.jsonl 2> $O/clock.err && \
XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/lib_clk/libxm_audio.so timeout -k 10 200 python tools/dev/clock_stamp.py --label zero --fill zero >> $O/clock.jsonl 2>> $O/clock.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_b.jsonl 2> $O/bench_b.err
rc=$?
cat $O/clock.jsonl; cut -c1-400 $O/bench_a.jsonl $O/bench_b.jsonl
exit $rc
