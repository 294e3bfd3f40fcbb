#!/usr/bin/env python3
"""Dev only: config 4's biquad stage and the resample side by side on two
streams with disjoint CU masks (hipExtStreamCreateWithCUMask).  The biquad
workgroups each need a whole CU's LDS (158 KB), so a resample kernel that
already holds every CU delays them; with masks the resample keeps to the CUs
the biquad grid does not use.  Prints alone / together times per mask split."""
import ctypes
import sys
import time

sys.path[:0] = ["xm-audio-utils_amd", "oracle"]
import torch  # noqa: E402
import xmaudio as xm  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
NCU = torch.cuda.get_device_properties(0).multi_processor_count
print("CUs", NCU, flush=True)


def masked_stream(pred):
    words = (NCU + 31) // 32
    m = (ctypes.c_uint32 * words)()
    for i in range(NCU):
        if pred(i):
            m[i // 32] |= 1 << (i % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), m)
    assert rc == 0, rc
    return s.value


B, N, NI = 1024, 441000, 480000
x = torch.empty((B, N, 2), dtype=torch.float32, device="cuda")
xi = torch.empty((B, NI, 2), dtype=torch.float32, device="cuda")
yr = torch.empty((B, N, 2), dtype=torch.float32, device="cuda")
xm.synth(x.data_ptr(), "f32", 0x584D4155, 0, B, 2, N, 0, torch.cuda.current_stream().cuda_stream)
xm.synth(xi.data_ptr(), "f32", 0x584D4155, 7, B, 2, NI, 0, torch.cuda.current_stream().cuda_stream)
e = xm.Effects(44100, 2, mem="device")
for f0, g in ((60, 3.0), (250, -2.0), (1000, 4.0), (4000, -3.0), (12000, 2.0)):
    e.add_eq_band(0, float(f0), g, 1.0)
m = xm.Mixer(48000, 44100, 2, "f32", mem="device")
m.set_tracks([dict(gain0=1.0)])
ptrs = [x[i].data_ptr() for i in range(B)]
torch.cuda.synchronize()


def run(sb, sr, k_rs, together):
    e.set_stream(sb)
    m.set_stream(sr)
    a = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    tb, trs = torch.cuda.ExternalStream(sb), torch.cuda.ExternalStream(sr)
    t0 = time.perf_counter()
    res = {}
    if together or k_rs == 0:
        a[0].record(tb)
        e.process_ptrs(ptrs, ptrs, N)
        a[1].record(tb)
    if together or k_rs > 0:
        a[2].record(trs)
        for _ in range(k_rs):
            m.process_strided(xi.data_ptr(), NI * 2, NI * 2, yr.data_ptr(), N * 2, B, NI)
        a[3].record(trs)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    if together or k_rs == 0:
        res["bq"] = a[0].elapsed_time(a[1])
    if together or k_rs > 0:
        res["rs"] = a[2].elapsed_time(a[3])
    res["wall"] = wall
    return res


full_a, full_b = torch.cuda.Stream().cuda_stream, torch.cuda.Stream().cuda_stream
splits = [("none", full_a, full_b)]
# CU index order: i % 32 < k gives every XCD k CUs if the order is XCD-major
# (i = 32 xcd + slot); i < 8 k does if XCDs interleave (i = 8 slot + xcd)
for keep in (22, 24):
    splits.append((f"i%32<{keep}", masked_stream(lambda i, k=keep: i % 32 < k),
                   masked_stream(lambda i, k=keep: i % 32 >= k)))
    splits.append((f"i<{8 * keep}", masked_stream(lambda i, k=keep: i < 8 * k),
                   masked_stream(lambda i, k=keep: i >= 8 * k)))
for it in range(1):
    for name, sb, sr in splits:
        r1 = run(sb, sr, 0, False)
        r2 = run(sb, sr, 1, False)
        r3 = run(sb, sr, 3, True)
        print(f"run {it} [{name}]: biquad alone {r1['bq']:.2f} ms, resample alone {r2['rs']:.2f} ms; together: "
              f"biquad {r3['bq']:.2f} ms, 3 resamples {r3['rs']:.2f} ms, wall {r3['wall']:.2f} ms", flush=True)
