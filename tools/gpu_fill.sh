#!/bin/bash
# Dev: headline kernel time vs input data (power / clock sensitivity).
set -o pipefail
for f in synth zero tiny synth; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu --fill $f > gpurun_out/fill_$f.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/fill_$f.log') if l.startswith('{')][-1]); print('$f', d['ms_per_step'], d['roofline']['frac'])"
done
