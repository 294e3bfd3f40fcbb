"""Dev (GPU box): achievable HBM rate for a read+write stream of config 2's
size (15.7 GB read, 14.5 GB written): torch copy kernels and hipMemcpy D2D."""
import time
import torch

n_in = 4096 * 480000 * 2
n_out = 4096 * 441000 * 2
x = torch.empty(n_in, dtype=torch.float32, device="cuda")
x.uniform_(-1, 1)
y = torch.empty(n_out, dtype=torch.float32, device="cuda")
for name, fn, rd, wr in (
        ("copy 14.5 GB (read+write)", lambda: y.copy_(x[:n_out]), n_out * 4, n_out * 4),
        ("read 15.7 GB (sum)", lambda: x.sum(), n_in * 4, 0),
        ("write 14.5 GB (fill)", lambda: y.fill_(1.0), 0, n_out * 4)):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    print(f"{name:28s} {ms:7.3f} ms  {(rd + wr) / ms / 1e9:6.2f} TB/s", flush=True)
