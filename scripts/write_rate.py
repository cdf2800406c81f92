"""Achievable HBM write rate by buffer size: torch's fill_ (a vectorized
streaming store kernel) and hipMemsetAsync (torch zero_) on 256 MiB - 4 GiB,
HIP events around 20 launches each.  For the question whether the trace's
slower store rate on large frames is the frame size itself."""
import json

import torch


def rate(fn, nbytes, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    ms = a.elapsed_time(b) / reps
    return ms * 1e3, nbytes / (ms * 1e-3) / 1e12


out = {}
for mib in (256, 512, 1024, 2048, 4096):
    n = mib << 20
    x = torch.empty(n // 16, 4, dtype=torch.int32, device="cuda")
    us_f, tb_f = rate(lambda: x.fill_(7), n)
    us_z, tb_z = rate(lambda: x.zero_(), n)
    out[f"{mib}MiB"] = {"fill_us": round(us_f, 1), "fill_TBps": round(tb_f, 3),
                        "zero_us": round(us_z, 1), "zero_TBps": round(tb_z, 3)}
    print(mib, out[f"{mib}MiB"], flush=True)
    del x
    torch.cuda.empty_cache()
print(json.dumps(out))
