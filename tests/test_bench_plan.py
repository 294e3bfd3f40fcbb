"""bench.py's launch plan: `--gpus N` drives N devices in
one process through the library's multi-device handle, or fails loudly; under
torchrun --gpus must equal WORLD_SIZE.  CPU-only: no device is touched."""
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _plan(argv, world=1, visible=8):
    return bench.plan(bench.parse(argv), world, visible)


def test_default_is_one_gpu():
    assert _plan([]) == ("local", [0])


def test_gpus_n_in_one_process():
    assert _plan(["--gpus", "8"]) == ("local", list(range(8)))
    assert _plan(["--gpus", "2"], visible=2) == ("local", [0, 1])


def test_gpus_beyond_visible_fails_loudly():
    with pytest.raises(SystemExit) as e:
        _plan(["--gpus", "2"], visible=1)
    assert "visible" in str(e.value)


def test_devices_list_dev_flag():
    assert _plan(["--devices", "0,0"], visible=1) == ("local", [0, 0])
    with pytest.raises(SystemExit):
        _plan(["--devices", "0,1"], visible=2)          # 2 distinct GPUs but --gpus 1
    assert _plan(["--devices", "0,1", "--gpus", "2"], visible=2) == ("local", [0, 1])


def test_torchrun_world_must_match():
    assert _plan(["--gpus", "4"], world=4)[0] == "ranked"
    with pytest.raises(SystemExit):
        _plan(["--gpus", "1"], world=4)
    with pytest.raises(SystemExit):
        _plan(["--gpus", "2", "--devices", "0,1"], world=2)


def test_torchrun_ranks_beyond_visible(monkeypatch):
    """More ranks than GPUs fails loudly, unless the dev rehearsal switch
    (ranks share one GPU, gloo coordination, lines marked "rehearsal")."""
    monkeypatch.delenv("XM_BENCH_REHEARSE", raising=False)
    with pytest.raises(SystemExit):
        _plan(["--gpus", "2"], world=2, visible=1)
    monkeypatch.setenv("XM_BENCH_REHEARSE", "1")
    assert _plan(["--gpus", "2"], world=2, visible=1)[0] == "ranked"


def test_config5_ramps_and_shards():
    assert len(bench.RAMPS64) == 64
    args = bench.parse(["--config", "c5"])
    assert args.tracks5 % 8 == 0 and args.mixes5 % 8 == 0


def test_allotted_cores_reports_affinity():
    n, host = bench.allotted_cores()
    assert 1 <= n <= host
    if hasattr(os, "sched_getaffinity") and not os.environ.get("OMP_NUM_THREADS"):
        assert n == len(os.sched_getaffinity(0))
