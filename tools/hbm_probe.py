"""Reference HBM stream rates on this GPU (tuning aid): read-only reduction and copy of a
headline-sized buffer (32 x [1,32,16384,128] bf16 = 4 GiB)."""
import json

import torch

dev = torch.device("cuda:0")
x = torch.empty(32 * 32 * 16384 * 128, dtype=torch.bfloat16, device=dev).uniform_()
y = torch.empty_like(x)
res = {}
for name, fn, nbytes in (("sum_read", lambda: x.sum(dtype=torch.float32), x.numel() * 2),
                         ("amax_read", lambda: x.abs().amax() if False else x.amax(), x.numel() * 2),
                         ("copy_rw", lambda: y.copy_(x), x.numel() * 4)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        fn()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    res[name] = {"ms": round(ms, 4), "TB_s": round(nbytes / ms / 1e9, 3)}
print(json.dumps(res))
