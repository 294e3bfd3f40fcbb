#!/bin/bash
# Round 5, box pass m: per-XCD wave ends at the 64/128-mix blocks on another
# box (stamped part-1 build in lib_clk), SQ/HBM counters of the config-1
# shapes (c1s16, mono1), and config 2 with box identifiers.
set -o pipefail
mkdir -p gpurun_out/r5m
export XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/lib_clk/libxm_audio.so
for m in 64 128; do
  timeout -k 10 240 python3 -u tools/dev/clock_stamp.py --mixes $m --seconds 2 --steps 20 --waves 4 --label m$m >> gpurun_out/r5m/waves.jsonl 2> gpurun_out/r5m/err_$m.txt || { tail -20 gpurun_out/r5m/err_$m.txt; exit 1; }
done
unset XM_AUDIO_LIB
python3 -c "
import json
for l in open('gpurun_out/r5m/waves.jsonl'):
    d=json.loads(l)
    if 'launch' in d: print(d['label'], d['launch'], d['end_q_0_10_50_90_99_100_us'][-1], d['end_mean_per_xcc_us'])
    elif 'cu_end_corr_between_launches' in d: print(d)
"
timeout -k 10 600 tools/dev/pmc_cfg.sh r5m/c1s16 c1s16 2 || exit 1
timeout -k 10 600 tools/dev/pmc_cfg.sh r5m/mono1 mono1 2 || exit 1
timeout -k 10 300 python3 tools/bench_configs.py c2 c1s16 mono1 --steps 100 --warmup 5 > gpurun_out/r5m/configs.jsonl 2>&1 || { tail -5 gpurun_out/r5m/configs.jsonl; exit 1; }
grep '^{' gpurun_out/r5m/configs.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_check'), d.get('clocks_during'))"
