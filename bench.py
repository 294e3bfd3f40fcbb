#!/usr/bin/env python3
"""Headline benchmark: PCM Msamples/s for 48 kHz -> 44.1 kHz polyphase
resample + 8-track gain-ramped mixdown (BASELINE.json:2).

Workload (strong scaling, SURVEY.md §8(d) "keep it fixed across 1/2/4/8
GPUs"): 4096 input clips in total = 512 mixes x 8 tracks, 10 s
stereo fp32 @ 48 kHz (480000 frames) -> 512 mixes x 441000 frames stereo
fp32 @ 44.1 kHz, split into N contiguous blocks of 512/N mixes, one per GPU.
`--weak` instead keeps 512 mixes on every GPU (labelled "weak").  Inputs are synthetic
(splitmix64 PCM) generated directly in HBM by the
library's xm_synth_pcm, outside the timed region.  One step = one
xm_audio_mixer_process_strided call over the whole per-GPU batch (every
track resampled, gained and summed; nothing cached between steps).

Unit: 1 sample = one per-channel PCM sample of an input track;
value = input samples of all ranks / wall time (max over ranks).

Multi-GPU: one process per GPU (torchrun), mixes are independent, so each
rank runs its own shard with no data-path collective; barrier + max-over-
ranks timing only.

Also reported (one JSON line on rank 0):
  roofline     — algorithmic bytes per launch (inputs read once + output
                 written once) / average kernel duration from HIP events on
                 the stream the kernel runs on, vs the 8 TB/s HBM peak;
                 traffic from the rocprofv3 PMC pass in profiles/ if present.
  cpu_baseline — the C restatement (oracle/, "port") on a bounded sample of
                 the same workload on this host's cores, and on 1 core.
  parity_check — after the timed loop every rank bit-compares the first and
                 the last mix of its block with the oracle (true = all equal).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "xm-audio-utils_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

SEED = 0x584D4155
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)

# 8 tracks: constant gains, fades, a crossfade pair, a step — every gain form
# of the contract (include/xm_audio_common.h) is exercised every step.
RAMPS = [
    dict(gain0=0.9, gain1=0.9),
    dict(gain0=0.0, gain1=0.8, ramp_start=0, ramp_len=44100),            # 1 s fade-in
    dict(gain0=0.7, gain1=0.2, ramp_start=220500, ramp_len=88200),       # 2 s duck
    dict(gain0=0.5, gain1=0.5),
    dict(mode=1, ramp_start=132300, ramp_len=88200),                     # crossfade out
    dict(gain0=0.0, gain1=1.0, ramp_start=132300, ramp_len=88200),       # crossfade in
    dict(gain0=1.0, gain1=0.0, ramp_start=396900, ramp_len=44100),       # 1 s fade-out
    dict(gain0=0.3, gain1=0.6, ramp_start=300000, ramp_len=0),           # step
]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--global-clips", type=int, default=4096,
                    help="input clips over all GPUs (strong scaling; 8 tracks per mix)")
    ap.add_argument("--weak", action="store_true", help="keep --mixes mixes on every GPU instead")
    ap.add_argument("--mixes", type=int, default=512, help="mixes per GPU with --weak")
    ap.add_argument("--tracks", type=int, default=8)
    ap.add_argument("--frames", type=int, default=480000, help="input frames per track (10 s @ 48 kHz)")
    ap.add_argument("--cpu-mixes", type=int, default=48, help="mixes in the CPU-baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target wall time of the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--fill", choices=["synth", "zero", "tiny"], default="synth",
                    help="dev only: input data (synth = the bench's synthetic PCM)")
    ap.add_argument("--no-check", action="store_true", help="skip the post-timing parity check")
    ap.add_argument("--check", action="store_true", help=argparse.SUPPRESS)   # the default now
    return ap.parse_args()


def traffic_from_profiles():
    """Latest corrected PMC traffic per launch (tools/profile_traffic.py output)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as fh:
            d = json.load(fh)
        return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, ramps):
    """The oracle's C restatement (same arithmetic) on a bounded sample of the
    workload: whole passes over --cpu-mixes mixes on every allotted core for
    about --cpu-seconds, then on one core for about a quarter of that."""
    import c_oracle as CO
    nmix = args.cpu_mixes
    x = np.empty((nmix, args.tracks, args.frames, 2), np.float32)
    for b in range(nmix):
        for t in range(args.tracks):
            x[b, t] = CO.gen_f32(SEED, b * args.tracks + t, 2, args.frames)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or 1))

    def run(xs, nth, seconds):
        passes, dt, used = 0, 0.0, 1
        while passes == 0 or (dt < seconds and passes < 200):
            t0 = time.perf_counter()
            _, used = CO.batch_resample_mix_f32(xs, ramps, 147, 160, threads=nth)
            dt += time.perf_counter() - t0
            passes += 1
        return xs.size * passes, dt, passes, used

    samples, dt, passes, used = run(x, threads, args.cpu_seconds)
    x1 = x[:2]
    s1, dt1, p1, _ = run(x1, 1, args.cpu_seconds / 4)
    del x
    return {"value": round(samples / dt / 1e6, 2), "unit": "Msamples/s", "cores": int(used), "kind": "port",
            "value_1core": round(s1 / dt1 / 1e6, 2), "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
            "sample": f"{passes} passes over {nmix} mixes x {args.tracks} tracks x {args.frames} frames x 2 ch fp32 "
                      f"({samples / 1e6:.0f} M input samples, {dt:.2f} s wall, {used} threads); 1 core: {p1} passes "
                      f"over 2 mixes ({s1 / 1e6:.0f} M samples, {dt1:.2f} s); oracle/xm_oracle.c -O3 "
                      f"-ffp-contract=off, OpenMP over mixes"}


def parity_check(x, y, idx, ramps):
    """Bit-compare mixes `idx` of this rank's output with the oracle."""
    import c_oracle as CO
    xs = x[list(idx)].cpu().numpy()
    ref, _ = CO.batch_resample_mix_f32(xs, ramps, 147, 160, threads=min(len(idx), os.cpu_count() or 1))
    got = y[list(idx)].cpu().numpy()
    return bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32)))


def main():
    args = parse()
    import xmaudio as xm
    from xmaudio import dist as xd

    rk = xd.from_env()
    world, rank = rk.world, rk.rank
    torch.cuda.set_device(rk.local)
    xd.init(rk, "nccl", torch.device("cuda", rk.local))   # RCCL; barrier + max-time only
    dev = torch.cuda.current_device()

    ntr, N = args.tracks, args.frames
    if args.weak:
        B = args.mixes
    else:
        if args.global_clips % (ntr * world):
            raise SystemExit(f"--global-clips {args.global_clips} does not split into whole mixes over {world} GPUs")
        B = args.global_clips // (ntr * world)
    ramps = RAMPS[:ntr] if ntr <= len(RAMPS) else (RAMPS * ((ntr + 7) // 8))[:ntr]
    mixer = xm.Mixer(48000, 44100, 2, "f32", mem="device", device=dev)
    mixer.set_tracks(ramps)
    F = mixer.out_frames(N)

    x = torch.empty((B, ntr, N, 2), dtype=torch.float32, device="cuda")
    y = torch.empty((B, F, 2), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream()
    # clip ids are global: rank r owns mixes [r*B, (r+1)*B) = clips [r*B*ntr, (r+1)*B*ntr)
    xm.synth(x.data_ptr(), "f32", SEED, xd.first_clip(rk, B, ntr), B * ntr, 2, N, dev, stream.cuda_stream)
    if args.fill != "synth":   # dev: power/clock sensitivity to the data (not a bench line)
        x.mul_(0.0 if args.fill == "zero" else 2.0 ** -20)
    mixer.set_stream(stream.cuda_stream)
    torch.cuda.synchronize()

    def step():
        mixer.process_strided(x.data_ptr(), N * 2, ntr * N * 2, y.data_ptr(), F * 2, B, N)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    launches_per_step = max(1, mixer.timing().n_launches)

    ev0 = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ev1 = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    xd.barrier(rk)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev0[i].record(stream)
        step()
        ev1[i].record(stream)
    torch.cuda.synchronize()
    xd.barrier(rk)
    elapsed = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in zip(ev0, ev1)]

    elapsed = xd.max_over_ranks(rk, elapsed, device="cuda")

    ok = None
    if not args.no_check:   # every rank: its first and last mix vs the oracle
        ok = parity_check(x, y, sorted({0, B - 1}), ramps)
        ok = xd.min_over_ranks(rk, ok, device="cuda")

    in_samples = B * ntr * N * 2
    ms_per_step = elapsed / args.steps * 1e3
    value = world * in_samples / (elapsed / args.steps) / 1e6
    alg_bytes = in_samples * 4 + B * F * 2 * 4
    avg_launch_ms = float(np.mean(kern_ms)) / launches_per_step
    achieved = alg_bytes / (avg_launch_ms * 1e-3) / 1e9
    traffic = traffic_from_profiles()

    if rank == 0:
        cpu = None if args.no_cpu else cpu_baseline(args, ramps)
        line = {
            "metric": "PCM Msamples/sec (48k->44.1k resample + 8-track mix), batch 4096, 1/2/4/8 GPUs",
            "value": round(value, 1), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak" if args.weak else "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "48k->44.1k polyphase resample (scipy resample_poly order) + 8-track "
                                   "gain-ramp/crossfade mixdown, stereo fp32, 10 s clips",
                       "clips_per_gpu": B * ntr, "mixes_per_gpu": B, "tracks": ntr, "frames_in": N,
                       "frames_out": F, "channels": 2, "global_clips": world * B * ntr,
                       "global_mixes": world * B,
                       "parallelism": f"dp{world} (independent mixes, no collective)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "alg_bytes_per_launch": alg_bytes, "avg_launch_ms": round(avg_launch_ms, 4),
                         "launches_per_step": launches_per_step},
            "cpu_baseline": cpu,
        }
        if ok is not None:
            line["parity_check"] = ok
            line["parity_detail"] = "bit-exact vs oracle/xm_oracle.c: first and last mix of every rank's block"
        print(json.dumps(line), flush=True)
    xd.finish(rk)


if __name__ == "__main__":
    main()
