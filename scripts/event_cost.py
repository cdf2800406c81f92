"""Cost of a cross-stream hand-off: a small kernel on stream A, then a
4096^2-int4 store kernel on stream B that waits for A through an event
(hipEventDisableTiming), against the same two kernels on one stream; and
the same with stream A created at high priority.  Prints us per pair."""
import statistics
import time

import torch


def main():
    dev = torch.device("cuda:0")
    big = torch.empty(4096 * 4096 * 4, dtype=torch.int32, device=dev)
    small = torch.empty(1024, dtype=torch.int32, device=dev)
    lo, hi = torch.cuda.Stream(dev), torch.cuda.Stream(dev, priority=-1)
    a = torch.cuda.Stream(dev)
    ev = [torch.cuda.Event(enable_timing=False) for _ in range(64)]

    def one_stream(n):
        with torch.cuda.stream(a):
            for _ in range(n):
                small.fill_(1)
                big.fill_(2)

    def two_streams(n, first):
        for i in range(n):
            with torch.cuda.stream(first):
                small.fill_(1)
                ev[i % 64].record(first)
            lo.wait_event(ev[i % 64])
            with torch.cuda.stream(lo):
                big.fill_(2)

    res = {"one stream": [], "two streams": [], "two streams, A high priority": []}
    n = 40
    for _ in range(7):
        for name, fn in (("one stream", lambda: one_stream(n)),
                         ("two streams", lambda: two_streams(n, a)),
                         ("two streams, A high priority", lambda: two_streams(n, hi))):
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / n * 1e6)
    for k, v in res.items():
        print(f"{k:32s} {statistics.median(v):7.1f} us per (small, store) pair")


if __name__ == "__main__":
    main()
