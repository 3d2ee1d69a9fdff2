"""Which rows differ between two settings of an experiments knob, and which
setting is exact there (the oracle):
    NBKD_LIB=.../exp/libnbkd.so python scripts/debug_ahead.py dump A.npy   (env knob set)
    python scripts/debug_ahead.py compare A.npy B.npy out.json
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

N, K, SEED = 20_000_000, 32, 20261015


def dump(path):
    from nbodyhpc_amd import capi, hip, synth
    hip.preload()
    hip.set_device(0)
    pts = synth.uniform(N, SEED)
    d = hip.DeviceArray.from_numpy(pts)
    t = capi.Tree(n=N, dev_ptr=d.ptr, leafsize=64, boxsize=1.0)
    od = hip.DeviceArray((N, K), np.float32)
    oi = hip.DeviceArray((N, K), np.uint32)
    t.query_device(d.ptr, N, K, od.ptr, oi.ptr)
    hip.synchronize()
    np.save(path, od.numpy())


def compare(a, b, out):
    from nbodyhpc_amd import synth
    from oracle.oracle import Oracle
    da, db = np.load(a, mmap_mode="r"), np.load(b, mmap_mode="r")
    rows = []
    for s in range(0, N, 1 << 20):
        e = min(N, s + (1 << 20))
        bad = np.nonzero((da[s:e].view(np.uint32) != db[s:e].view(np.uint32)).any(axis=1))[0]
        rows.extend((bad + s).tolist())
    res = {"rows_differing": len(rows), "first": rows[:20]}
    if rows:
        pts = synth.uniform(N, SEED)
        sel = np.array(rows[:2000])
        dr, ir = Oracle().tree(pts, 64, 1.0).query(pts[sel], K, workers=16)
        ea = (np.asarray(da[sel]).view(np.uint32) == dr.view(np.uint32)).all(axis=1)
        eb = (np.asarray(db[sel]).view(np.uint32) == dr.view(np.uint32)).all(axis=1)
        res.update({"a_exact": int(ea.sum()), "b_exact": int(eb.sum()), "checked": len(sel)})
        j = int(sel[0])
        res["example"] = {"row": j, "a": np.asarray(da[j]).tolist()[-4:],
                          "b": np.asarray(db[j]).tolist()[-4:], "oracle": dr[0].tolist()[-4:]}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        compare(sys.argv[2], sys.argv[3], sys.argv[4])
