#!/bin/bash
# Round-end pass (GPU box, repo root): tools/gpu_check.sh (GPU tests, smoke,
# the driver's bench line, kernel trace, FETCH/WRITE/SQ), every config line
# (box identifiers in each), the one-process sharded and config-5 forms, and
# the HBM-ceiling microbenchmark on the same box.
#   tools/dev/gpu_final.sh <tag>
set -o pipefail
TAG=${1:?tag}
bash tools/gpu_check.sh $TAG || exit 1
tools/dev/gpu_steps.sh $TAG \
  'configs|900|python3 -u tools/bench_configs.py c2 c3 c4 c5 hl c1s16 c1odd mono1 mono8 odd ptrs up s16rs conv planar oconv stream r32to48 r48to32 r96to48 r24to48 r16to48 r96to44 r44to96 r22to48 s16rs3 planar2 conv2 m22to48 s22to48 m44to96 m24to48 m16to48 s24to48 s96to44 s16r24to48 s16r16to48 s16r22to48 s44to48 s32to48 s48to32 s96to48 t2 t4 t2up t4up t2odd t4odd bq fir --steps 15 --warmup 3' \
  'dev00|300|python3 -u bench.py --devices 0,0 --steps 10 --warmup 3 --no-cpu' \
  'c5dev8|300|python3 -u bench.py --config c5 --devices 0,0,0,0,0,0,0,0 --steps 5 --warmup 2 --no-cpu' \
  'c5|300|python3 -u bench.py --config c5 --steps 5 --warmup 2' \
  'hbm|200|tools/ubench/bin/hbm_ceiling basic,tile,pst' || exit 1
grep '^{' gpurun_out/$TAG/configs.log | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    print(d['config'], d.get('kernel'), d['ms_per_step'], d['roofline']['frac'], d.get('parity_check'))"
