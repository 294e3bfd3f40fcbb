"""CPU: the C-ABI library loads, exports every symbol include/*.h declares,
and its host-only logic (design, sizes, errors) behaves — no GPU compute.
"""
import os
import re

import numpy as np
import pytest

from conftest import ROOT, bits_equal, golden


def declared_symbols():
    names = set()
    for h in ("xm_audio_common.h", "xm_audio_mixer.h", "xm_effects.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        names |= set(re.findall(r"XM_API\s+[\w\s\*]*?\b(xm_\w+)\s*\(", src))
    return names


def test_exports_every_declared_symbol(xm):
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in sorted(syms):
        assert hasattr(xm._lib, s), f"libxm_audio.so does not export {s}"
    assert set(xm.EXPORTED) == syms


def test_no_internal_symbols_leak(xm):
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", xm.LIB_PATH], capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert exported == declared_symbols(), exported ^ declared_symbols()


def test_strerror_and_version(xm):
    assert xm.strerror(0) == "ok"
    assert "invalid" in xm.strerror(xm.XM_EINVAL)
    assert "gfx950" in xm.version()


@pytest.mark.parametrize("key", sorted(k for k in golden("tables.npz").files if k.startswith("H_")))
def test_design_bit_exact_vs_scipy(xm, key):
    L, M = map(int, key[2:].split("_"))
    z = golden("tables.npz")
    d, H = xm.design(M * 100, L * 100)
    meta = z["meta_" + key[2:]]
    assert [d.L, d.M, d.T, d.rm, d.half, d.pre] == [int(v) for v in meta]
    assert bits_equal(H, z[key])


def test_design_identity_and_bad_rates(xm):
    d, H = xm.design(48000, 48000)
    assert (d.L, d.M) == (1, 1)
    with pytest.raises(xm.XmError) as e:
        xm.design(0, 48000)
    assert e.value.code == xm.XM_EINVAL


def test_out_frames(xm):
    assert xm.out_frames(48000, 44100, 480000) == 441000
    assert xm.out_frames(44100, 48000, 441000) == 480000
    assert xm.out_frames(48000, 44100, 1) == 1
    assert xm.out_frames(48000, 44100, 161) == -(-161 * 147 // 160)


def test_gpu_handle_without_gpu_fails(xm):
    """GPU handles (the default n_devices = 1) never fall back to the CPU
    backend: with no GPU, create fails loudly.  The CPU backend is chosen
    only by n_devices = 0 / XM_DEVICE_CPU (tests/test_cpu_backend.py)."""
    if xm.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(xm.XmError) as e:
        xm.Mixer(48000, 44100, 2, "f32")
    assert e.value.code == xm.XM_EDEVICE
    with pytest.raises(xm.XmError):
        xm.Effects(48000, 2)


def test_invalid_config_rejected(xm):
    with pytest.raises(xm.XmError) as e:
        xm.Mixer(48000, 44100, 3, "f32")
    assert e.value.code == xm.XM_EINVAL
