#!/bin/bash
# Round 5, box pass h: is the 320/147 kernel bound by scalar-cache misses on
# its 26.9 KB coefficient table?  (XM_AB_ROW0: every group from row 0)
set -o pipefail
mkdir -p gpurun_out/r5h
for lib in lib lib_abrow0; do
  XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/$lib/libxm_audio.so timeout -k 10 300 python3 tools/bench_configs.py r44to96 up --steps 10 --warmup 3 --no-check > gpurun_out/r5h/$lib.jsonl 2>&1 || { tail -5 gpurun_out/r5h/$lib.jsonl; exit 1; }
  grep '^{' gpurun_out/r5h/$lib.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$lib', d['config'], d['ms_per_step'], d['roofline']['frac'])"
done
