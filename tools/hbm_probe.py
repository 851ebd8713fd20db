"""Achievable HBM bandwidth on this box for the access mixes of the env step:
pure streaming write (fill), read+write copy, and pure read (sum), 1 GiB each."""
import json
import torch


def t(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n / 1e3


n = 1 << 28  # 1 GiB of f32
x = torch.empty(n, device="cuda").uniform_()
y = torch.empty(n, device="cuda")
out = {"write_fill_GBps": 4 * n / t(lambda: y.fill_(1.0)) / 1e9,
       "copy_rw_GBps": 8 * n / t(lambda: y.copy_(x)) / 1e9,
       "read_sum_GBps": 4 * n / t(lambda: x.sum()) / 1e9}
print(json.dumps(out))
