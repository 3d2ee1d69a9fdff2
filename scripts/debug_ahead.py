"""Rows that differ between NBKD_COLLECT_AHEAD=0 and =1 (experiments build,
the knob is read per launch) in ONE process at 1e8, and which setting is
exact there (the C oracle):  NBKD_LIB=.../exp/libnbkd.so python scripts/debug_ahead.py out.json"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

N, K, SEED = int(float(os.environ.get("DBG_N", "1e8"))), 32, 20261015


def main(out):
    from nbodyhpc_amd import capi, hip, synth
    hip.preload()
    hip.set_device(0)
    pts = synth.uniform(N, SEED)
    d = hip.DeviceArray.from_numpy(pts)
    t = capi.Tree(n=N, dev_ptr=d.ptr, leafsize=64, boxsize=1.0)
    outs = []
    for v in ("0", "1"):
        os.environ["NBKD_COLLECT_AHEAD"] = v
        od = hip.DeviceArray((N, K), np.float32)
        oi = hip.DeviceArray((N, K), np.uint32)
        capi.stats_enable(True)
        t.query_device(d.ptr, N, K, od.ptr, oi.ptr)
        hip.synchronize()
        st = capi.stats_read_all()
        capi.stats_enable(False)
        outs.append((od, oi, {kk: st[kk] for kk in ("retry_queries", "fallback_queries",
                                                    "candidates", "node_visits")}))
    rows = []
    ch = 1 << 20
    for s in range(0, N, ch):
        e = min(N, s + ch)
        a = np.empty((e - s, K), np.float32)
        b = np.empty((e - s, K), np.float32)
        hip.memcpy(a.ctypes.data, outs[0][0].ptr + s * K * 4, a.nbytes, hip.D2H)
        hip.memcpy(b.ctypes.data, outs[1][0].ptr + s * K * 4, b.nbytes, hip.D2H)
        bad = np.nonzero((a.view(np.uint32) != b.view(np.uint32)).any(axis=1))[0]
        rows.extend((bad + s).tolist())
    res = {"n": N, "rows_differing": len(rows), "first": rows[:20],
           "stats_ahead0": outs[0][2], "stats_ahead1": outs[1][2]}
    if rows:
        from oracle.oracle import Oracle
        sel = np.array(rows[:500], np.int64)
        got = []
        for od, oi, _ in outs:
            g = np.empty((len(sel), K), np.float32)
            for j, r in enumerate(sel):
                hip.memcpy(g[j].ctypes.data, od.ptr + int(r) * K * 4, K * 4, hip.D2H)
            got.append(g)
        dr, ir = Oracle().tree(pts, 64, 1.0).query(pts[sel], K, workers=16)
        for nm, g in zip(("ahead0", "ahead1"), got):
            res[nm + "_exact"] = int((g.view(np.uint32) == dr.view(np.uint32)).all(axis=1).sum())
        res["checked"] = len(sel)
        res["example"] = {"row": int(sel[0]), "ahead0": got[0][0].tolist(),
                          "ahead1": got[1][0].tolist(), "oracle": dr[0].tolist()}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res)[:3000], flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
