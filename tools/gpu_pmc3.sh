#!/bin/bash
# Dev: PMC sets for the product kernel and the two ablations (compute-only, memory-only).
set -o pipefail
bash tools/pmc_fast.sh base || exit 1
XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/lib_ablate/libxm_audio.so XM_FAST_ABLATE=1 bash tools/pmc_fast.sh abl1 || exit 1
XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/lib_ablate/libxm_audio.so XM_FAST_ABLATE=2 bash tools/pmc_fast.sh abl2 || exit 1
