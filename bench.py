#!/usr/bin/env python3
"""Headline benchmark: PCM Msamples/s for 48 kHz -> 44.1 kHz polyphase
resample + 8-track gain-ramped mixdown (BASELINE.json:2).

Workload (strong scaling, SURVEY.md §8(d) "keep it fixed across 1/2/4/8
GPUs"): 4096 input clips in total = 512 mixes x 8 tracks, 10 s
stereo fp32 @ 48 kHz (480000 frames) -> 512 mixes x 441000 frames stereo
fp32 @ 44.1 kHz, split into N contiguous blocks of 512/N mixes, one per GPU.
`--weak` instead keeps 512 mixes on every GPU (labelled "weak").  Inputs are synthetic
(splitmix64 PCM) generated directly in HBM by the
library's xm_synth_pcm, outside the timed region.  One step = one pass of
the C API over the whole batch (every track resampled, gained and summed;
nothing cached between steps).

Unit: 1 sample = one per-channel PCM sample of an input track;
value = input samples of all GPUs / wall time (max over ranks).

Multi-GPU, two launch forms, the same shards:
  * one process per GPU (torchrun, the driver's N > 1 form): WORLD_SIZE
    ranks, rank r owns mix block r on its LOCAL_RANK device; no data-path
    collective, barrier + max-over-ranks timing only.  --gpus must equal
    WORLD_SIZE.
  * one process, `--gpus N` without a launcher: the library's own
    multi-device handle (xm_audio_mixer_create_multi over devices 0..N-1,
    one host worker thread per device); block d is resident
    on device d and one step is one xm_audio_mixer_process_sharded call,
    which returns when every device has finished (wall time around it).
    Exits non-zero when fewer than N devices are visible.  `--devices 0,0`
    (dev) runs the same sharded path over an explicit list, repeats allowed.

--config c5 measures config 5 (BASELINE.json:11) instead: 512 mixes x 64
s16 tracks, 64/N tracks on each device, int32 partials -> one exchange
(the library's RCCL reduce-scatter over xGMI in the one-process form,
torch.distributed reduce_scatter_tensor over RCCL under torchrun) ->
saturate on the device that owns each block of mixes.

Also reported (one JSON line on rank 0):
  roofline     — algorithmic bytes per launch (inputs read once + output
                 written once) / average kernel duration from HIP events on
                 the stream the kernel runs on, vs the 8 TB/s HBM peak;
                 traffic: corrected PMC bytes per launch from the newest
                 profiles/*traffic*.json taken on the same kernel sources
                 (sha256 of KERNEL_SOURCES; an earlier rocprofv3 pass, the
                 file named in traffic_source), else null.
  cpu_baseline — the library's own host CPU backend (n_devices = 0,
                 xm-audio-utils_amd/src/cpu: the same C API call, bit-identical
                 results) on a bounded sample of the same workload, in a child
                 process on this process's allotted host cores
                 (sched_getaffinity / OMP_NUM_THREADS) and in one on 1 core.
                 The reference has no code, so this C path is
                 the "reference CPU path" of BASELINE.json:5; oracle/ stays
                 the checker.
  parity_check — after the timed loop every shard's first and last mix are
                 bit-compared with the oracle (true = all equal).
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
METRIC = "PCM Msamples/sec (48k->44.1k resample + 8-track mix), batch 4096, 1/2/4/8 GPUs"
METRIC_C5 = "PCM Msamples/sec (64-track s16 mixdown, tracks spanning devices), config 5"

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

# config 5: Q15 ramps of every form, 8 patterns x 8 (offset start frames)
_R5 = [(29491, 29491, 0, 0, 0), (0, 26214, 0, 48000, 0), (22938, 6554, 240000, 96000, 0), (16384, 16384, 0, 0, 0),
       (0, 0, 144000, 96000, 1), (0, 32768, 144000, 96000, 0), (32768, 0, 432000, 48000, 0),
       (9830, 19661, 300000, 0, 0)]
RAMPS64 = [dict(gain0_q15=q0, gain1_q15=q1, ramp_start=s + 997 * i, ramp_len=ln, mode=md)
           for i in range(8) for q0, q1, s, ln, md in _R5]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=["headline", "c5"], default="headline")
    ap.add_argument("--devices", default="",
                    help="dev: explicit device list for the one-process sharded path, e.g. 0,0")
    ap.add_argument("--global-clips", type=int, default=4096,
                    help="input clips over all GPUs (strong scaling; 8 tracks per mix)")
    ap.add_argument("--weak", action="store_true", help="keep --mixes mixes on every GPU instead")
    ap.add_argument("--mixes", type=int, default=512, help="mixes per GPU with --weak")
    ap.add_argument("--tracks", type=int, default=8)
    ap.add_argument("--frames", type=int, default=480000, help="input frames per track (10 s @ 48 kHz)")
    ap.add_argument("--mixes5", type=int, default=512, help="config 5: mixes (all devices)")
    ap.add_argument("--tracks5", type=int, default=64, help="config 5: tracks per mix (all devices)")
    ap.add_argument("--span-chunks", type=int, default=0,
                    help="config 5: exchange chunks overlapped with the partials (0: automatic, up to 4)")
    ap.add_argument("--cpu-mixes", type=int, default=48, help="mixes in the CPU-baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="target wall time of the CPU-baseline sample")
    ap.add_argument("--cpu-only", action="store_true", help=argparse.SUPPRESS)   # the baseline's child process
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--fill", choices=["synth", "zero", "tiny"], default="synth",
                    help="dev only: input data (synth = the bench's synthetic PCM)")
    ap.add_argument("--no-check", action="store_true", help="skip the post-timing parity check")
    ap.add_argument("--check", action="store_true", help=argparse.SUPPRESS)   # the default now
    return ap.parse_args(argv)


def plan(args, world: int, visible: int):
    """(mode, device list) for this invocation, or SystemExit with the reason.
    mode: "ranked" (one process per GPU under torchrun; the list is this
    rank's device) or "local" (this process drives every device in the list)."""
    if world > 1:
        if args.devices:
            raise SystemExit("bench.py: --devices is for the one-process form, not under torchrun")
        if args.gpus != world:
            raise SystemExit(f"bench.py: launched with WORLD_SIZE={world} but --gpus {args.gpus}")
        if world > visible and not rehearsal():
            raise SystemExit(f"bench.py: {world} ranks but {visible} GPU(s) visible")
        return "ranked", None
    if args.devices:
        devs = [int(d) for d in args.devices.split(",") if d.strip() != ""]
        if not devs or min(devs) < 0:
            raise SystemExit(f"bench.py: bad --devices {args.devices!r}")
        if len(set(devs)) != args.gpus:
            raise SystemExit(f"bench.py: --devices {args.devices} names {len(set(devs))} distinct GPU(s) "
                             f"but --gpus {args.gpus}")
    else:
        if args.gpus < 1:
            raise SystemExit(f"bench.py: --gpus {args.gpus}")
        devs = list(range(args.gpus))
    if max(devs) >= visible:
        raise SystemExit(f"bench.py: --gpus {args.gpus} needs device(s) {sorted(set(devs))} but {visible} "
                         f"GPU(s) are visible; run N > 1 on an N-GPU node (one process, or torchrun with "
                         f"--nproc-per-node N)")
    return "local", devs


# the sources the headline kernel is compiled from: a PMC traffic record
# counts for this run only if it was taken on these very sources
KERNEL_SOURCES = ("xm-audio-utils_amd/csrc/xm_resample_fast.hip", "xm-audio-utils_amd/csrc/xm_pk_taps.h",
                  "xm-audio-utils_amd/csrc/xm_ablate.h",
                  "xm-audio-utils_amd/csrc/xm_device.h", "xm-audio-utils_amd/csrc/xm_shim.h",
                  "xm-audio-utils_amd/tools/gen_coefs.c")


def kernel_src_sha256():
    import hashlib
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(ROOT, rel), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def traffic_from_profiles(alg_bytes=None):
    """Corrected PMC traffic per launch (tools/profile_traffic.py output) from
    the newest profiles/*traffic*.json taken on this tree's kernel sources
    (its kernel_src_sha256 equals ours), and the file it came from (a separate
    rocprofv3 pass, not this run).  None when no record matches: a number
    measured on other kernel code is not reported as this kernel's traffic;
    likewise when the record's launch moved other algorithmic bytes than this
    one (a shard of the batch at N > 1)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json")))
    if not files:
        return None, None
    try:
        mine = kernel_src_sha256()
    except OSError:
        return None, None
    for f in reversed(files):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        if d.get("kernel_src_sha256") == mine:
            rec = d.get("alg_bytes_per_launch")
            if alg_bytes is not None and rec is not None and int(rec) != int(alg_bytes):
                return None, (f"{os.path.relpath(f, ROOT)} holds a launch of {int(rec)} algorithmic bytes "
                              f"(the 1-GPU batch); this launch moves {int(alg_bytes)}")
            return d.get("hbm_bytes_per_launch"), os.path.relpath(f, ROOT)
    return None, f"none on these kernel sources (newest record: {os.path.relpath(files[-1], ROOT)})"


def practical_ceiling():
    """The measured practical HBM ceiling for the headline's byte mix (15.73 GB
    read + 1.81 GB written): the median over boxes of the best form measured by
    tools/ubench/hbm_ceiling.hip, committed in profiles/r6_hbm_ceiling.json
    (tools/dev/ceiling_table.py).  None if the record is absent."""
    f = os.path.join(ROOT, "profiles", "r6_hbm_ceiling.json")
    try:
        with open(f) as fh:
            d = json.load(fh)
        return float(d["practical"]["GBps_median"]), os.path.relpath(f, ROOT)
    except (OSError, ValueError, KeyError, TypeError):
        return None, None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def allotted_cores():
    """Host cores this process may run on (its affinity mask), capped by
    OMP_NUM_THREADS when that is set; and the machine's total."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if omp > 0:
        n = min(n, omp)
    return max(1, n), os.cpu_count() or n


def _timed_passes(fn, seconds, max_passes=200):
    passes, dt, used = 0, 0.0, 1
    while passes == 0 or (dt < seconds and passes < max_passes):
        t0 = time.perf_counter()
        used = fn()
        dt += time.perf_counter() - t0
        passes += 1
    return passes, dt, used


def _cpu_child(args, threads, mixes, seconds, config="headline"):
    """One CPU-backend measurement in a child process (the pool's thread count
    is fixed per process: XM_CPU_THREADS).  The child never touches a GPU."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-only", "--config", config, "--cpu-mixes", str(mixes),
           "--cpu-seconds", str(seconds), "--tracks", str(args.tracks), "--frames", str(args.frames),
           "--tracks5", str(args.tracks5)]
    env = dict(os.environ, XM_CPU_THREADS=str(threads))
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode or not lines:
        raise RuntimeError(f"cpu baseline child failed (rc {p.returncode}): {p.stderr[-600:]}")
    return json.loads(lines[-1])


def run_cpu_only(args):
    """--cpu-only (child): whole passes of the library's CPU backend over a
    sample of the workload, for about --cpu-seconds; prints one JSON line."""
    import xmaudio as xm
    if args.config == "c5":
        B, ntr, N = args.cpu_mixes, args.tracks5, args.frames
        x = np.empty((B, ntr, N, 2), np.int16)
        xm.synth(x.ctypes.data, "s16", SEED, 1000, B * ntr, 2, N, device="cpu")
        m = xm.Mixer(48000, 48000, 2, "s16", device="cpu")
        m.set_tracks(RAMPS64[:ntr])
    else:
        B, ntr, N = args.cpu_mixes, args.tracks, args.frames
        x = np.empty((B, ntr, N, 2), np.float32)
        xm.synth(x.ctypes.data, "f32", SEED, 0, B * ntr, 2, N, device="cpu")
        m = xm.Mixer(48000, 44100, 2, "f32", device="cpu")
        m.set_tracks(RAMPS[:ntr] if ntr <= len(RAMPS) else (RAMPS * ((ntr + 7) // 8))[:ntr])
    m.process(x)   # warm: pool threads, page faults of the output
    passes, dt, _ = _timed_passes(lambda: m.process(x), args.cpu_seconds)
    print(json.dumps({"samples": int(x.size) * passes, "seconds": dt, "passes": passes, "mixes": B,
                      "threads": int(os.environ.get("XM_CPU_THREADS", "0"))}), flush=True)


def cpu_baseline(args, ramps, config="headline"):
    """The library's CPU backend (n_devices = 0) on a bounded sample of the
    workload: whole passes over --cpu-mixes mixes on every allotted core for
    about --cpu-seconds, then over 2 mixes on one core for half of that."""
    threads, host = allotted_cores()
    mixes = args.cpu_mixes if config == "headline" else max(1, args.cpu_mixes // 12)   # c5: 64-track mixes
    a = _cpu_child(args, threads, mixes, args.cpu_seconds, config)
    one = _cpu_child(args, 1, 2, args.cpu_seconds / 2, config)
    ntr = args.tracks5 if config == "c5" else args.tracks
    what = (f"{ntr} s16 tracks (Q15 mix)" if config == "c5"
            else f"{ntr} tracks x {args.frames} frames x 2 ch fp32, 48k->44.1k + ramped mix")
    return {"value": round(a["samples"] / a["seconds"] / 1e6, 2), "unit": "Msamples/s", "cores": int(threads),
            "kind": "port", "value_1core": round(one["samples"] / one["seconds"] / 1e6, 2),
            "path": "libxm_audio's host CPU backend (XmMixerConfig.n_devices = 0; xm-audio-utils_amd/src/cpu, "
                    "-O3 -ffp-contract=off, AVX-512/AVX2 vector tap loops, pthread pool); results bit-identical "
                    "to the GPU's. The reference has no code, so this is the build's own CPU path (SURVEY.md §0)",
            "cpu_model": cpu_model(), "host_cpus": host,
            "cores_note": f"{threads} threads = this process's allotted share (sched_getaffinity / OMP_NUM_THREADS) "
                          f"of the host's {host} CPUs",
            "sample": f"{a['passes']} passes over {a['mixes']} mixes x {what} ({a['samples'] / 1e6:.0f} M input "
                      f"samples, {a['seconds']:.2f} s, {threads} threads); 1 core: {one['passes']} passes over "
                      f"{one['mixes']} mixes ({one['samples'] / 1e6:.0f} M samples, {one['seconds']:.2f} s)"}


def parity_check(x, y, idx, ramps):
    """Bit-compare mixes `idx` of a shard's output with the oracle."""
    import c_oracle as CO
    xs = x[list(idx)].cpu().numpy()
    ref, _ = CO.batch_resample_mix_f32(xs, ramps, 147, 160, threads=min(len(idx), os.cpu_count() or 1))
    got = y[list(idx)].cpu().numpy()
    return bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32)))


def headline_line(args, *, n_gpus, shards, B, ntr, N, F, value, ms_per_step, kern_ms, launches, ok, parallelism,
                  ramps, mode):
    in_samples = B * ntr * N * 2
    alg_bytes = in_samples * 4 + B * F * 2 * 4
    avg_launch_ms = float(np.mean(kern_ms)) / launches
    achieved = alg_bytes / (avg_launch_ms * 1e-3) / 1e9
    traffic, tsrc = traffic_from_profiles(alg_bytes)
    pgbs, psrc = practical_ceiling()
    cpu = None if args.no_cpu or n_gpus > 1 else cpu_baseline(args, ramps)   # rank 0 at N = 1 only
    line = {
        "metric": METRIC, "value": round(value, 1), "unit": "Msamples/s", "n_gpus": n_gpus, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "weak" if args.weak else "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "48k->44.1k polyphase resample (scipy resample_poly order) + 8-track "
                               "gain-ramp/crossfade mixdown, stereo fp32, 10 s clips",
                   "clips_per_gpu": B * ntr, "mixes_per_gpu": B, "tracks": ntr, "frames_in": N,
                   "frames_out": F, "channels": 2, "global_clips": shards * B * ntr,
                   "global_mixes": shards * B, "shards": shards, "launch": mode,
                   "parallelism": parallelism},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": tsrc,
                     "alg_bytes_per_launch": alg_bytes, "avg_launch_ms": round(avg_launch_ms, 4),
                     "launches_per_step": launches,
                     "practical": None if pgbs is None else {
                         "peak": round(pgbs, 1), "unit": "GB/s", "frac": round(achieved / pgbs, 4), "source": psrc,
                         "what": "best measured form for this byte mix (contiguous mix tiles, nt loads and stores), "
                                 "median over boxes"}},
        "cpu_baseline": cpu,
    }
    if _BOX:
        line["box"] = dict(_BOX)
    if ok is not None:
        line["parity_check"] = ok
        line["parity_detail"] = "bit-exact vs oracle/xm_oracle.c: first and last mix of every shard"
    return line


def mixes_per_shard(args, ntr, shards):
    if args.weak:
        return args.mixes
    if args.global_clips % (ntr * shards):
        raise SystemExit(f"--global-clips {args.global_clips} does not split into whole mixes over {shards} shards")
    return args.global_clips // (ntr * shards)


def rehearsal() -> bool:
    """XM_BENCH_REHEARSE=1 (dev only): the torchrun path on a box with fewer
    GPUs than ranks.  Every rank runs on GPU LOCAL_RANK % visible and the
    barrier / max-time coordination goes over gloo (RCCL refuses two ranks on
    one GPU).  Its lines carry "rehearsal": true: they check the multi-rank
    plumbing (shards, clip ids, barrier, max over ranks, rank 0's line), they
    are not bench results (the ranks share one GPU)."""
    return os.environ.get("XM_BENCH_REHEARSE") == "1"


def run_headline_ranked(args):
    """One process per GPU (or the plain one-GPU run): rank r, device LOCAL_RANK."""
    import xmaudio as xm
    from xmaudio import dist as xd

    rk = xd.from_env()
    world, rank = rk.world, rk.rank
    reh = rehearsal() and world > 1
    local = rk.local % torch.cuda.device_count() if reh else rk.local
    torch.cuda.set_device(local)
    if reh:
        xd.init(rk, "gloo")
    else:
        xd.init(rk, "nccl", torch.device("cuda", local))   # RCCL; barrier + max-time only
    dev = torch.cuda.current_device()
    cdev = "cpu" if reh else "cuda"

    ntr, N = args.tracks, args.frames
    B = mixes_per_shard(args, ntr, world)
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
    launches = max(1, mixer.timing().n_launches)

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
    elapsed = xd.max_over_ranks(rk, elapsed, device=cdev)

    ok = None
    if not args.no_check:   # every rank: its first and last mix vs the oracle
        ok = parity_check(x, y, sorted({0, B - 1}), ramps)
        ok = xd.min_over_ranks(rk, ok, device=cdev)

    if rank == 0:
        value = world * B * ntr * N * 2 / (elapsed / args.steps) / 1e6
        par = f"dp{world} (independent mixes, no collective)" + (", one process per GPU" if world > 1 else "")
        line = headline_line(args, n_gpus=world, shards=world, B=B, ntr=ntr, N=N, F=F, value=value,
                             ms_per_step=elapsed / args.steps * 1e3, kern_ms=kern_ms, launches=launches,
                             ok=ok, parallelism=par, ramps=ramps, mode="torchrun" if world > 1 else "single")
        if reh:
            line["rehearsal"] = True   # the ranks shared one GPU: plumbing check, not a bench result
        print(json.dumps(line), flush=True)
    xd.finish(rk)


def run_headline_local(args, devs):
    """One process over every device in `devs`: the library's multi-device
    handle, shard d resident on device devs[d], one process_sharded per step."""
    import xmaudio as xm

    n = len(devs)
    ntr, N = args.tracks, args.frames
    B = mixes_per_shard(args, ntr, n)
    ramps = RAMPS[:ntr] if ntr <= len(RAMPS) else (RAMPS * ((ntr + 7) // 8))[:ntr]
    mixer = xm.Mixer(48000, 44100, 2, "f32", mem="device", devices=devs)
    mixer.set_tracks(ramps)
    F = mixer.out_frames(N)
    xs, ys = [], []
    for d, dev in enumerate(devs):
        with torch.cuda.device(dev):
            x = torch.empty((B, ntr, N, 2), dtype=torch.float32, device=f"cuda:{dev}")
            y = torch.empty((B, F, 2), dtype=torch.float32, device=f"cuda:{dev}")
            xm.synth(x.data_ptr(), "f32", SEED, d * B * ntr, B * ntr, 2, N, dev,
                     torch.cuda.current_stream().cuda_stream)
            if args.fill != "synth":
                x.mul_(0.0 if args.fill == "zero" else 2.0 ** -20)
        xs.append(x)
        ys.append(y)
    for dev in set(devs):
        torch.cuda.synchronize(dev)
    ins, outs, bs = [x.data_ptr() for x in xs], [y.data_ptr() for y in ys], [B] * n

    def step():   # returns when every device has finished its block
        mixer.process_sharded(ins, N * 2, ntr * N * 2, outs, F * 2, bs, N)

    for _ in range(args.warmup):
        step()
    launches = max(1, mixer.timing().n_launches // n)
    kern_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        kern_ms.append(mixer.timing().kernel_ms)   # slowest device's HIP-event window
    elapsed = time.perf_counter() - t0

    ok = None
    if not args.no_check:
        ok = all(parity_check(x, y, sorted({0, B - 1}), ramps) for x, y in zip(xs, ys))
    value = n * B * ntr * N * 2 / (elapsed / args.steps) / 1e6
    par = (f"dp{n} (independent mixes, no collective), one process, in-library multi-device handle over "
           f"devices {devs}")
    print(json.dumps(headline_line(args, n_gpus=len(set(devs)), shards=n, B=B, ntr=ntr, N=N, F=F, value=value,
                                   ms_per_step=elapsed / args.steps * 1e3, kern_ms=kern_ms, launches=launches,
                                   ok=ok, parallelism=par, ramps=ramps, mode="one process")), flush=True)


def c5_check(xs_host_mix, ys_host_mix, ramps):
    """One finished 64-track mix vs the oracle's Q15 mix."""
    import c_oracle as CO
    ref, _ = CO.batch_mix_s16(xs_host_mix[None], ramps, threads=min(8, os.cpu_count() or 1))
    return bool(np.array_equal(ref[0], ys_host_mix))


def c5_line(args, *, n_gpus, shards, B, ntr, N, value, ms_per_step, ok, mode, parallelism):
    from xmaudio import dist as xd
    per = ntr // shards
    dev_bytes = B * per * N * 2 * 2 + (B // shards) * N * 2 * 2   # this device's tracks once + its mixes once
    achieved = dev_bytes / (ms_per_step * 1e-3) / 1e9
    xgmi = (shards - 1) * (B // shards) * N * 2 * 4 if shards > 1 else 0
    line = {
        "metric": METRIC_C5, "value": round(value, 1), "unit": "Msamples/s", "n_gpus": n_gpus,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "int32 (s16 Q15)",
        "data": "synthetic",
        "config": {"workload": f"{ntr}-track s16 Q15 gain-ramp/crossfade mixdown, {B} mixes x 10 s stereo 48 kHz, "
                               f"tracks spread over {shards} shard(s): int32 partials -> one exchange -> saturate",
                   "mixes": B, "tracks": ntr, "tracks_per_shard": per, "frames": N, "channels": 2,
                   "shards": shards, "launch": mode, "parallelism": parallelism,
                   "exchange_chunks": xd.span_chunks(args.span_chunks, B // shards) if shards > 1 else 0},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "alg_bytes_per_device_step": dev_bytes, "xgmi_bytes_per_device_step": xgmi,
                     "note": "per-device algorithmic HBM bytes over the whole step's wall time "
                             "(partial kernel + exchange + finish)"},
        "cpu_baseline": None if args.no_cpu else cpu_baseline(args, RAMPS64[:ntr], config="c5"),
    }
    if ok is not None:
        line["parity_check"] = ok
        line["parity_detail"] = "bit-exact vs oracle xo_batch_mix_s16: first and last finished mix of every shard"
    return line


def run_c5_local(args, devs):
    """Config 5 in one process: xm_audio_mixer_mix_spanning_s16 (RCCL
    reduce-scatter between distinct devices, device copies when one repeats)."""
    import xmaudio as xm

    n = len(devs)
    B, ntr, N = args.mixes5, args.tracks5, args.frames
    if ntr % n or B % n:
        raise SystemExit(f"config 5: {ntr} tracks and {B} mixes must split over {n} shards")
    per = ntr // n
    ramps = RAMPS64[:ntr]
    m = xm.Mixer(48000, 48000, 2, "s16", mem="device", devices=devs)
    m.set_tracks(ramps)
    m.set_span_chunks(args.span_chunks)
    xs, ys = [], []
    for d, dev in enumerate(devs):
        with torch.cuda.device(dev):
            x = torch.empty((B, per, N, 2), dtype=torch.int16, device=f"cuda:{dev}")
            xm.synth(x.data_ptr(), "s16", SEED, d * B * per, B * per, 2, N, dev,
                     torch.cuda.current_stream().cuda_stream)
            xs.append(x)
            ys.append(torch.empty((B // n, N, 2), dtype=torch.int16, device=f"cuda:{dev}"))
    for dev in set(devs):
        torch.cuda.synchronize(dev)
    ins, outs = [x.data_ptr() for x in xs], [y.data_ptr() for y in ys]

    def step():
        m.mix_spanning_s16(ins, N * 2, per * N * 2, outs, N * 2, B, N)

    for _ in range(args.warmup):
        step()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    elapsed = time.perf_counter() - t0
    ok = None
    if not args.no_check:
        ok = True
        nb = B // n
        for d in range(n):
            for b in sorted({0, nb - 1}):
                g = d * nb + b   # global mix: its tracks are block b of every shard
                xm_ = np.concatenate([xs[q][g].cpu().numpy() for q in range(n)])
                ok &= c5_check(xm_, ys[d][b].cpu().numpy(), ramps)
    distinct = len(set(devs)) == n
    par = (f"{n} shards, tracks of every mix split over devices {devs}; exchange: "
           + ("in-library RCCL ncclReduceScatter(int32) over xGMI, in chunks overlapped with the partials"
              if distinct else "device copies (a device repeats) + ordered int32 sum, chunk by chunk"))
    print(json.dumps(c5_line(args, n_gpus=len(set(devs)), shards=n, B=B, ntr=ntr, N=N,
                             value=B * ntr * N * 2 / (elapsed / args.steps) / 1e6,
                             ms_per_step=elapsed / args.steps * 1e3, ok=ok, mode="one process",
                             parallelism=par)), flush=True)


def run_c5_ranked(args):
    """Config 5, one process per GPU: partial -> reduce_scatter_tensor (RCCL) -> finish."""
    import xmaudio as xm
    from xmaudio import dist as xd

    rk = xd.from_env()
    if rehearsal() and rk.world > 1:
        raise SystemExit("bench.py: XM_BENCH_REHEARSE covers the headline only (config 5's exchange needs RCCL)")
    torch.cuda.set_device(rk.local)
    xd.init(rk, "nccl", torch.device("cuda", rk.local))
    dev = torch.cuda.current_device()
    B, ntr, N = args.mixes5, args.tracks5, args.frames
    if ntr % rk.world or B % rk.world:
        raise SystemExit(f"config 5: {ntr} tracks and {B} mixes must split over {rk.world} ranks")
    per = ntr // rk.world
    ramps = RAMPS64[:ntr]
    m = xm.Mixer(48000, 48000, 2, "s16", mem="device", device=dev)
    m.set_tracks(ramps[rk.rank * per:(rk.rank + 1) * per])
    s = torch.cuda.current_stream()
    m.set_stream(s.cuda_stream)
    x = torch.empty((B, per, N, 2), dtype=torch.int16, device="cuda")
    xm.synth(x.data_ptr(), "s16", SEED, rk.rank * B * per, B * per, 2, N, dev, s.cuda_stream)
    y = torch.empty((B // rk.world, N, 2), dtype=torch.int16, device="cuda")
    for _ in range(args.warmup):
        xd.mix_spanning_s16(rk, m, x, out=y, chunks=args.span_chunks)
    torch.cuda.synchronize()
    xd.barrier(rk)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        xd.mix_spanning_s16(rk, m, x, out=y, chunks=args.span_chunks)
    torch.cuda.synchronize()
    xd.barrier(rk)
    elapsed = xd.max_over_ranks(rk, time.perf_counter() - t0, device="cuda")
    ok = None
    if not args.no_check:
        # every rank's first and last owned mix: gather its 64 tracks from all ranks
        import torch.distributed as dist
        nb = B // rk.world
        ok = True
        for b in sorted({0, nb - 1}):
            mine = []
            for r in range(rk.world):
                g = r * nb + b
                part = x[g].contiguous()
                if rk.world > 1:
                    bufs = [torch.empty_like(part) for _ in range(rk.world)]
                    dist.all_gather(bufs, part)
                else:
                    bufs = [part]
                if r == rk.rank:
                    mine = [t.cpu().numpy() for t in bufs]
            ok &= c5_check(np.concatenate(mine), y[b].cpu().numpy(), ramps)
        ok = xd.min_over_ranks(rk, ok, device="cuda")
    if rk.rank == 0:
        par = (f"{rk.world} ranks, one process per GPU; exchange: torch.distributed reduce_scatter_tensor (RCCL), "
               "asynchronous, in chunks overlapped with the partials")
        print(json.dumps(c5_line(args, n_gpus=rk.world, shards=rk.world, B=B, ntr=ntr, N=N,
                                 value=B * ntr * N * 2 / (elapsed / args.steps) / 1e6,
                                 ms_per_step=elapsed / args.steps * 1e3, ok=ok, mode="torchrun",
                                 parallelism=par)), flush=True)
    xd.finish(rk)


_BOX = {}


def box_ids():
    """The GPU's HBM vendor and VBIOS (rocm-smi), read before this process
    touches the GPU (rocm-smi re-execs its interpreter, which a process whose
    GPU is initialised may not do); skipped under rocprofv3, whose preload
    initialises the GPU first.  Box classes differ in memory-side speed
    (DESIGN §5.3); the line names its box."""
    if _BOX or any(k.startswith("ROCPROF") for k in os.environ) or os.environ.get("RANK", "0") != "0":
        return _BOX   # (rank 0 prints the line)
    import subprocess
    for flag, keys in (("--showmemvendor", ("GPU memory vendor",)), ("--showvbios", ("VBIOS version",)),
                       ("--showserial", ("Serial Number",))):
        try:
            r = subprocess.run(["rocm-smi", flag, "--json"], capture_output=True, text=True, timeout=20)
            d = json.loads(r.stdout) if r.returncode == 0 and r.stdout.strip().startswith("{") else {}
            for kv in d.values():
                if isinstance(kv, dict):
                    for k in keys:
                        if k in kv:
                            _BOX[k] = kv[k]
                    break
        except Exception:   # pragma: no cover - box dependent
            pass
    return _BOX


def main(argv=None):
    args = parse(argv)
    if args.cpu_only:
        run_cpu_only(args)
        return
    box_ids()   # before any device work
    world = int(os.environ.get("WORLD_SIZE", "1"))
    mode, devs = plan(args, world, torch.cuda.device_count())
    if args.config == "c5":
        if mode == "ranked":
            run_c5_ranked(args)
        else:
            run_c5_local(args, devs)
        return
    if mode == "ranked" or (len(devs) == 1 and devs[0] == 0 and not args.devices):
        run_headline_ranked(args)
    else:
        run_headline_local(args, devs)


if __name__ == "__main__":
    main()
