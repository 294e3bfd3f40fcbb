#!/bin/bash
# Dev (GPU box, repo root): headline parity tests, the bench line (3 runs) and
# one SQ instruction-count pass, each step under its own limit.
#   tools/gpu_perf.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-perf}; K=${2:-"headline or resample_mix_f32 or ramp or crossfade or resample_only or ragged"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1
rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench$i.log 2>&1 || { tail -5 $OUT/bench$i.log; exit 1; }
  grep '^{' $OUT/bench$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['roofline']['frac'], d['parity_check'])"
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-check > $OUT/pmc_sq.log 2>&1 || { tail -5 $OUT/pmc_sq.log; exit 1; }
python3 - $OUT/pmc_sq/run_counter_collection.csv <<'PY'
import csv, sys, collections
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if "k_rs147" in r["Kernel_Name"]:
        per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for c, v in sorted(per.items()):
    print(f"{c:24s} {sum(v.values()) / len(v):.4g}")
PY
