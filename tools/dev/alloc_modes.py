#!/usr/bin/env python3
"""Dev: are the write-heavy lines' speeds (same box, same library: m24to48
5.6 or 7.5 ms, mono1 7.5 or 8.7, profiles/r6_n_mono_ab.txt; c2 6.5 or 8.7 by
"box class") set per process, per allocation, or by the buffers' offsets?
One process (GPU box, repo root):

    python3 tools/dev/alloc_modes.py [line] [quick] [which] [flags]
        # line: m24to48 (default), mono1, m16to48, c2, hl; quick: no offsets;
        # which: new x only / new y only; flags: hipMalloc and contiguous allocations

  keep      the same buffers timed 4 times
  realloc   fresh buffers (allocator cache emptied) timed 4 times
  xoff/yoff the input / output shifted by 4 KiB .. 16 MiB inside one larger
            allocation
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "xm-audio-utils_amd"))
import xmaudio as xm  # noqa: E402

# line -> (in rate, out rate, channels, tracks per mix, mixes, frames in)
LINES = {"m24to48": (24000, 48000, 1, 1, 8192, 240000), "mono1": (44100, 48000, 1, 1, 8192, 441000),
         "m16to48": (16000, 48000, 1, 1, 8192, 160000), "c2": (48000, 44100, 2, 1, 4096, 480000),
         "hl": (48000, 44100, 2, 8, 512, 480000)}


def timed(step, s, steps=10, warmup=2):
    for _ in range(warmup):
        step()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(steps):
        step()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def main():
    line = sys.argv[1] if len(sys.argv) > 1 else "m24to48"
    fi, fo, C, T, B, N = LINES[line]
    m = xm.Mixer(fi, fo, C, "f32", mem="device")
    m.set_tracks([dict(gain0=1.0 - 0.1 * t) for t in range(T)])
    F = m.out_frames(N)
    s = torch.cuda.current_stream()
    m.set_stream(s.cuda_stream)
    PAD = 16 << 20   # bytes of slack in front of each buffer

    def alloc():
        xb = torch.empty(B * T * N * C + PAD // 4, dtype=torch.float32, device="cuda")
        yb = torch.empty(B * F * C + PAD // 4, dtype=torch.float32, device="cuda")
        xm.synth(xb.data_ptr(), "f32", 1234, 0, B * T, C, N, 0, s.cuda_stream)
        return xb, yb

    def run(xb, yb, xo=0, yo=0):
        xp, yp = xb.data_ptr() + xo, yb.data_ptr() + yo
        return timed(lambda: m.process_strided(xp, N * C, T * N * C, yp, F * C, B, N), s)

    xb, yb = alloc()
    print(line, "x at", hex(xb.data_ptr()), "y at", hex(yb.data_ptr()), flush=True)
    for i in range(4):
        print(f"keep     {i}  {run(xb, yb):.3f} ms", flush=True)
    for i in range(int(os.environ.get("REALLOCS", "4"))):
        del xb, yb
        torch.cuda.empty_cache()
        xb, yb = alloc()
        print(f"realloc  {i}  {run(xb, yb):.3f} ms  x {hex(xb.data_ptr())} y {hex(yb.data_ptr())}", flush=True)
    offs = () if "quick" in sys.argv[2:] else (4 << 10, 64 << 10, 256 << 10, 1 << 20, 2 << 20, 4 << 20, 8 << 20, 16 << 20)
    for off in offs:
        print(f"xoff {off >> 10:6d} KiB  {run(xb, yb, xo=off):.3f} ms   "
              f"yoff {off >> 10:6d} KiB  {run(xb, yb, yo=off):.3f} ms", flush=True)
    print(f"keep     end {run(xb, yb):.3f} ms", flush=True)
    if "which" in sys.argv[2:]:   # which buffer's placement matters
        for i in range(4):
            del yb
            torch.cuda.empty_cache()
            yb = torch.empty(B * F * C + PAD // 4, dtype=torch.float32, device="cuda")
            print(f"new y    {i}  {run(xb, yb):.3f} ms", flush=True)
        for i in range(4):
            del xb
            torch.cuda.empty_cache()
            xb = torch.empty(B * T * N * C + PAD // 4, dtype=torch.float32, device="cuda")
            xm.synth(xb.data_ptr(), "f32", 1234, 0, B * T, C, N, 0, s.cuda_stream)
            print(f"new x    {i}  {run(xb, yb):.3f} ms", flush=True)
    if "flags" in sys.argv[2:]:   # hipMalloc / hipExtMallocWithFlags(contiguous) outside torch's allocator
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        del xb, yb
        torch.cuda.empty_cache()
        nx, ny = (B * T * N * C) * 4, (B * F * C) * 4

        class Buf:
            def __init__(self, n, flags):
                self.p = ctypes.c_void_p()
                rc = (hip.hipMalloc(ctypes.byref(self.p), ctypes.c_size_t(n)) if flags is None else
                      hip.hipExtMallocWithFlags(ctypes.byref(self.p), ctypes.c_size_t(n), ctypes.c_uint(flags)))
                if rc:
                    raise RuntimeError(f"alloc rc {rc}")

            def data_ptr(self):
                return self.p.value

            def free(self):
                hip.hipFree(self.p)
        for name, fl in (("hipMalloc", None), ("contig", 4)):
            for i in range(4):
                try:
                    xb, yb = Buf(nx, fl), Buf(ny, fl)
                except RuntimeError as e:
                    print(f"{name:8s} {i}  {e}", flush=True)
                    break
                xm.synth(xb.data_ptr(), "f32", 1234, 0, B * T, C, N, 0, s.cuda_stream)
                print(f"{name:8s} {i}  {run(xb, yb):.3f} ms  x {hex(xb.data_ptr())} y {hex(yb.data_ptr())}", flush=True)
                torch.cuda.synchronize()
                xb.free()
                yb.free()


if __name__ == "__main__":
    main()
