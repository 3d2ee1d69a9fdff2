"""Build-time A/B: best of R builds of 1e8 uniform periodic points (device input)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nbodyhpc_amd import hip  # noqa: E402

hip.preload()
from nbodyhpc_amd import capi, synth  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
pts = synth.uniform(n, box=1.0)
d = hip.DeviceArray.from_numpy(pts)
capi.timing_enable(True)
best = 1e9
parts = {}
first = None
for _ in range(4):
    capi.timing_reset()
    hip.synchronize()
    t0 = time.perf_counter()
    t = capi.Tree(n=n, dev_ptr=d.ptr, leafsize=64, boxsize=1.0)
    hip.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    first = ms if first is None else first
    if ms < best:
        best = ms
        parts = {k: round(capi.timing_read(k)[0], 2) for k in ("build_levels", "build_small", "build_groups")}
    t.close()
print(f"[{os.environ.get('NBKD_LIB', 'default lib')} {os.environ.get('NBKD_GROUP_BLOCKS_PER_CU', '')}] n={n:.0e} build_ms={best:.2f} first={first:.2f} {parts}")
