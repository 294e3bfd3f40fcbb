#!/bin/bash
# Dev (GPU box, repo root): output-store cache policies per line: time
# (tools/dev/ab_cfg.sh, R rounds alternating libraries) and WRITE_SIZE
# (tools/dev/write_survey.sh) for each library.
#   tools/dev/store_pol_ab.sh <rounds> "<lines>" <lib> ...
set -o pipefail
R=$1; LINES=$2; shift 2
tools/dev/ab_cfg.sh $R "$LINES" "$@" > gpurun_out/store_pol_ab.txt 2>&1 || exit 1
for l in "$@"; do
  XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/$l/libxm_audio.so tools/dev/write_survey.sh sp_$l $LINES || exit 1
done
