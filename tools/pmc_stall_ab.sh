#!/bin/bash
# Dev: tools/pmc_stall.sh for the product library and the ablation build
# (XM_FAST_ABLATE=1: no DMA, no copies) on one box.
set -o pipefail
bash tools/pmc_stall.sh stall_base || exit 1
XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/lib_ablate/libxm_audio.so XM_FAST_ABLATE=1 bash tools/pmc_stall.sh stall_abl1
