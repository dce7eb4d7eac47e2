"""Practical HBM ceilings on this box: torch fill_ (write-only) and copy_ (read+write) of a
buffer the size of the C3 level-0 volume (68.7 GB), HIP events, median of 5."""
import json

import torch


def timeit(fn, reps=5):
    ts = []
    for i in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if i:
            ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    n = 64 * 16384 * 16384 // 4          # float32 elements: a quarter of the volume, 17.2 GB
    a = torch.empty(n, dtype=torch.float32, device='cuda')
    b = torch.empty(n, dtype=torch.float32, device='cuda')
    ms_fill = timeit(lambda: a.fill_(1.0))
    ms_copy = timeit(lambda: b.copy_(a))
    gb = n * 4 / 1e9
    print(json.dumps({'fill_GBps': round(gb / (ms_fill * 1e-3), 1), 'copy_GBps_rw': round(2 * gb / (ms_copy * 1e-3), 1),
                      'bytes': int(n * 4)}))


if __name__ == '__main__':
    main()
