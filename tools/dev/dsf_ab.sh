set -o pipefail
tools/dev/ab_cfg.sh 3 'm24to48 m16to48 m22to48' lib lib_ab_dsf16 lib_ab_dsf2 lib_ab_dsf17 > gpurun_out/dsf_ab.txt 2>&1 || exit 1
for l in lib lib_ab_dsf16 lib_ab_dsf2 lib_ab_dsf17; do
  XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/$l/libxm_audio.so tools/dev/write_survey.sh ws_$l m24to48 m16to48 m22to48 || exit 1
done
