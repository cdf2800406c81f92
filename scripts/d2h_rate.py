import time, torch
d = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
for pin in (False, True):
    h = torch.empty(256 << 20, dtype=torch.uint8, pin_memory=pin)
    for _ in range(2): h.copy_(d); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5): h.copy_(d)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    print(f"pinned={pin}: {dt*1e3:.2f} ms  {256/1024/dt:.1f} GB/s")
