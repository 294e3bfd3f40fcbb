#!/usr/bin/env python3
"""Performance attribution for the fast 147/160 kernel (dev tool, GPU box).

Runs bench.py once per variant, each in its own process, and prints ms/step:
  base        product library (lib/)
  abl<N>      lib_ablate/ build (`make ablate`), XM_FAST_ABLATE=N:
              1 no DMA/copies, 2 no taps, 4 no exchange / track sum,
              8 constant gains, 16 cycle attribution (8 waves per workgroup,
              as the product)
Ablated variants compute wrong results on purpose; only their time matters.
usage: python tools/ablate.py [variant ...]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ABL_LIB = os.path.join(ROOT, "xm-audio-utils_amd", "lib_ablate", "libxm_audio.so")
VARIANTS = {
    "base": {},
}
for n in (1, 2, 4, 8, 16):
    VARIANTS[f"abl{n}"] = {"XM_AUDIO_LIB": ABL_LIB, "XM_FAST_ABLATE": str(n)}


def variant(name):
    """name[@R]: a variant, optionally with the SPs-per-lane split forced to R"""
    base, _, r = name.partition("@")
    env = dict(VARIANTS[base])
    if r:
        env["XM_FAST_R"] = r
    return env


def main():
    names = sys.argv[1:] or list(VARIANTS)
    for name in names:
        env = dict(os.environ, **variant(name))
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "10", "--warmup", "2", "--no-cpu", "--no-check"]
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        if p.returncode or not line:
            print(f"{name:8s} FAILED rc={p.returncode}: {p.stderr[-400:]}", flush=True)
            break
        d = json.loads(line[-1])
        print(f"{name:8s} ms/step {d['ms_per_step']:8.4f}  kernel ms {d['roofline']['avg_launch_ms']:8.4f}", flush=True)


if __name__ == "__main__":
    main()
