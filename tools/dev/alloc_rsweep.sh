set -o pipefail
mkdir -p gpurun_out/rs
export REALLOCS=5
for R in 0 32 16 8 4; do
  if [ $R = 0 ]; then unset XM_FAST_SPLIT_R; else export XM_FAST_SPLIT_R=$R; fi
  timeout -k 10 200 python3 -u tools/dev/alloc_modes.py c2 quick > gpurun_out/rs/c2_R$R.log 2>&1 || exit 1
  timeout -k 10 200 python3 -u tools/dev/alloc_modes.py m24to48 quick > gpurun_out/rs/m24_R$R.log 2>&1 || exit 1
done
