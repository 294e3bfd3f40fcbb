"""The drop-in boundary from C: examples/xm_mix_example.c compiles against
include/*.h with plain gcc, links libxm_audio.so, and runs.  On a host without
a GPU the GPU examples must refuse loudly (XM_EDEVICE, exit 2) instead of
falling back to the CPU; on the GPU box they must complete (exit 0).  The
config-1 example asks for the CPU backend (n_devices = 0) and runs anywhere."""
import hashlib
import os
import subprocess

import pytest

from conftest import LIB_DIR, ROOT


def _build(tmp_path, name="xm_mix_example", hip=False):
    exe = tmp_path / name
    extra = ["-I", "/opt/rocm/include", "-D__HIP_PLATFORM_AMD__"] if hip else []
    libs = ["-L", "/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"] if hip else []
    cmd = ["gcc", "-std=c11", "-O2", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include")] + extra + \
          [os.path.join(ROOT, "examples", name + ".c"), "-L", LIB_DIR, "-lxm_audio",
           f"-Wl,-rpath,{LIB_DIR}"] + libs + ["-lm", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_example_builds_and_refuses_without_gpu(tmp_path):
    exe = _build(tmp_path)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    if "0 HIP device(s)" in p.stdout:
        assert p.returncode == 2, p.stderr
        assert "HIP device error" in p.stderr
    else:   # a GPU is visible here: the full run must succeed
        assert p.returncode == 0, p.stderr


@pytest.mark.gpu
def test_example_runs_on_gpu(tmp_path):
    exe = _build(tmp_path)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("mix ")]
    assert len(lines) == 2
    for ln in lines:
        assert "44100 frames" in ln
        rms = float(ln.rsplit("rms", 1)[1])
        assert 0.05 < rms < 2.0


def test_stream_example_builds_and_refuses_without_gpu(tmp_path):
    """The streaming / timeline entry points compile from plain C11 (-Werror)."""
    exe = _build(tmp_path, "xm_stream_example")
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    if "0 HIP device(s)" in p.stdout:
        assert p.returncode == 2, p.stderr
    else:
        assert p.returncode == 0, p.stderr


@pytest.mark.gpu
def test_stream_example_runs_on_gpu(tmp_path):
    exe = _build(tmp_path, "xm_stream_example")
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "bit-identical to process_batch" in p.stdout
    assert "timeline: 44100 frames" in p.stdout


def test_multi_example_builds_and_refuses_without_gpu(tmp_path):
    """The multi-device entry points (create_multi, process_strided over a
    device list, mix_spanning_s16) compile from plain C11 (-Werror)."""
    exe = _build(tmp_path, "xm_multi_example", hip=True)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    if "0 HIP device(s)" in p.stdout:
        assert p.returncode == 2, p.stderr
    else:
        assert p.returncode == 0, p.stdout + p.stderr


@pytest.mark.gpu
def test_multi_example_runs_on_gpu(tmp_path):
    exe = _build(tmp_path, "xm_multi_example", hip=True)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "bit-identical to one device" in p.stdout
    assert "config 5:" in p.stdout


def test_config1_cpu_example(tmp_path):
    """BASELINE.json:7 from plain C with no GPU: n_devices = 0 reproduces the
    committed config-1 digest (scipy-pinned)."""
    from conftest import manifest
    exe = _build(tmp_path, "xm_config1_cpu")
    out = tmp_path / "y.raw"
    p = subprocess.run([str(exe), str(out)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "441000 -> 480000 frames" in p.stdout
    assert hashlib.sha256(out.read_bytes()).hexdigest() == manifest()["config1_sha256"]
