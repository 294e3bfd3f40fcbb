"""Host-C sanitizer target (SURVEY.md §5 "Sanitizers"):
the host layer of the library (xm-audio-utils_amd/src/*.c) built with
-fsanitize=address,undefined against the CPU stand-in shim
(tests/host_asan/xm_fake_shim.c), driven through every C entry point by
tests/host_asan/run_checks.py and compared with the oracle bit for bit.
Runs on the CPU container; any ASan/UBSan report aborts the child."""
import os
import subprocess
import sys

from conftest import ROOT

HERE = os.path.join(ROOT, "tests", "host_asan")


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) else None


def test_host_layer_under_asan_ubsan():
    subprocess.run(["make", "-C", HERE, "-s"], check=True, capture_output=True, text=True)
    asan = _runtime("libasan.so")
    assert asan, "gcc's libasan runtime not found"
    env = dict(os.environ,
               LD_PRELOAD=asan,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0:exitcode=86",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:exitcode=87",
               XM_AUDIO_LIB=os.path.join(HERE, "build", "libxm_audio_asan.so"),
               XM_NO_TORCH="1", XM_FAKE_DEVICES="2", OMP_NUM_THREADS="1")
    p = subprocess.run([sys.executable, os.path.join(HERE, "run_checks.py")], env=env, capture_output=True,
                       text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-6000:]
    assert "ALL HOST CHECKS PASSED" in p.stdout
