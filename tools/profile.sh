#!/bin/bash
# Profile the headline kernel on the GPU box (run from repo root via gpurun).
#   tools/profile.sh <tag> [bench args...]
# Writes gpurun_out/prof_<tag>/: kernel-trace stats and separate PMC passes
# (never combined with tracing domains; see MI355X_MICROARCH.md §rocprofv3).
set -o pipefail
TAG=${1:-r1}; shift
ARGS=${@:---steps 5 --warmup 1 --no-cpu}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc1 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc2 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $OUT/pmc3 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc3.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_INST_CYCLES_SALU -d $OUT/pmc4 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc4.log 2>&1 || exit $?
# instruction / scalar-data cache behaviour (names as listed by rocprofv3 -L on gfx950)
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_IFETCH -d $OUT/pmc5 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc5.log 2>&1 || echo "pmc5 failed rc=$?"
echo "profile done: $OUT"
