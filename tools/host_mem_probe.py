"""Host-side read cost of the plan's pinned staging buffers (esgpu_host_alloc = hipHostMalloc) vs pageable memory:
the build step reads the gathered winner cells from pinned memory on the host."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from elasticsearch_amd import Engine, pinned_empty  # noqa: E402


def _time(f, reps=20):
    f()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        t.append(time.perf_counter() - t0)
    return sorted(t)[len(t) // 2] * 1e3


def main():
    Engine()  # HIP runtime initialised as in a plan
    out = {}
    for mb in (0.25, 1, 16):
        n = int(mb * (1 << 20)) // 8
        pin = pinned_empty(n, np.uint64)
        reg = np.empty(n, dtype=np.uint64)
        pin[:] = 1
        reg[:] = 1
        strided = lambda a: int(a[::8].sum())  # one 8-B read per 64-B line
        out[f"{mb}MB"] = {"pinned_sum_ms": _time(lambda: int(pin.sum())), "pageable_sum_ms": _time(lambda: int(reg.sum())),
                          "pinned_line_ms": _time(lambda: strided(pin)), "pageable_line_ms": _time(lambda: strided(reg)),
                          "pinned_copy_ms": _time(lambda: np.copy(pin)), "pageable_copy_ms": _time(lambda: np.copy(reg))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
