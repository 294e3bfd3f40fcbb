"""GPU form of tests/test_api_edges.py's effects case: process_batch in
XM_MEM_DEVICE with per-track effects, mixes (ntr + 1) tracks apart and
separately allocated outputs.  The mixer's output pointer table and the
effects path's track table must not share a device buffer (the
track table overwrote the output table, and the mixdown landed in the
inputs).  Every mix bit-exact against the C oracle."""
import pytest

from test_api_edges import _fx_irregular_case

pytestmark = pytest.mark.gpu


class _DevBuf:
    def __init__(self, a):
        import torch
        self.t = torch.from_numpy(a.copy()).to("cuda")

    def ptr(self, *idx):
        return self.t[idx].data_ptr() if idx else self.t.data_ptr()


def test_effects_irregular_strides_scattered_outputs_gpu(xm, gpu):
    import torch
    _fx_irregular_case(xm, 0, _DevBuf, lambda b: (torch.cuda.synchronize(), b.t.cpu().numpy())[1])
