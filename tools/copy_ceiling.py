"""Practical HBM copy ceiling on the box (GPU probe): device-to-device copies with torch's copy
kernel and hipMemcpyAsync at several sizes; rate = (read + write bytes) / time.  The copy-bound
calls (l2_compress kr = 0.8, decode steps) are compared against it."""
import ctypes
import json

import torch

dev = torch.device("cuda:0")
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                               ctypes.c_void_p]
HIP_D2D = 3
res = {}
for gib in (0.25, 1.0, 4.0):
    n = int(gib * 2**30) // 2
    a = torch.empty(n, dtype=torch.bfloat16, device=dev).normal_()
    b = torch.empty_like(a)
    st = torch.cuda.current_stream().cuda_stream

    def memcpy():
        assert hip.hipMemcpyAsync(b.data_ptr(), a.data_ptr(), 2 * n, HIP_D2D, st) == 0

    for name, fn in (("torch_copy", lambda: b.copy_(a)), ("hipMemcpyAsync_d2d", memcpy)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        res[f"{name}_{gib}GiB"] = {"ms": round(ms, 4), "TB_s_rd_plus_wr": round(4 * n / ms / 1e9, 3)}
    del a, b
print(json.dumps(res))
