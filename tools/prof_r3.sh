#!/bin/bash
# Round-3 profiling pass (GPU box, repo root): the headline's kernel trace and
# HBM passes (tools/gpu_check.sh --no-tests), config 2's write amplification
# (tools/pmc_c2.sh), and the FIR / biquad PMC passes (tools/pmc_fx.sh).
#   tools/prof_r3.sh <tag>
set -o pipefail
TAG=${1:-r3_prof}
bash tools/gpu_check.sh $TAG --no-tests || exit $?
bash tools/pmc_c2.sh ${TAG}_c2 || exit $?
bash tools/pmc_fx.sh ${TAG}_fir fir k_fir_rb > gpurun_out/${TAG}_fir.txt 2>&1 || { cat gpurun_out/${TAG}_fir.txt; exit 1; }
cat gpurun_out/${TAG}_fir.txt
bash tools/pmc_fx.sh ${TAG}_bq bq k_biquad_pc > gpurun_out/${TAG}_bq.txt 2>&1 || { cat gpurun_out/${TAG}_bq.txt; exit 1; }
cat gpurun_out/${TAG}_bq.txt
echo "prof_r3 done"
