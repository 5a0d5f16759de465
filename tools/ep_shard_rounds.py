"""Exchange rounds of the endpoint-owned multi-rank protocol (tests/ep_shard.py, CPU
prototype) on config 5's own node -- the sparse 4 096-endpoint, 50k-service workload
bench.py runs (synth.config5 defaults) -- at 2^20 packets: per world
size the rounds, the deliveries whose source program ran on another rank, the wall time,
and whether the merged result equals one sequential run of the per-endpoint-map
datapath (every output, every endpoint's CT4 / CT6 table, metrics, policy counters).
Prints one JSON line.  TEST INFRASTRUCTURE (the oracle is every rank's datapath)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from cilium_amd import synth
    from tests import ep_shard as E
    from tests import harness as H
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    worlds = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [2, 8]
    t0 = time.time()
    w = synth.config5(n)
    dp, maps = E.per_endpoint_dp(w)
    ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    seq_s = time.time() - t0
    deliv = int((ref.ret != E.DEFER).sum())
    res = {"packets": n, "endpoints": len(w.endpoints), "services": len(w.maps["lb4_revnat"]) + len(w.maps["lb6_revnat"]),
           "sequential_s": round(seq_s, 1), "worlds": {}}
    print(f"[{time.time() - t0:.0f}s] sequential run done", file=sys.stderr, flush=True)
    for world in worlds:
        t1 = time.time()
        results, rounds = E.simulate(w, world, w.now)
        el = time.time() - t1
        out, ct, metrics, (pk, pv) = E.merge(w, results)
        same = all((out[k] == getattr(ref, k).astype(np.int64)).all() for k in E.RankState.FIELDS)
        for e in range(len(w.endpoints)):
            for fam, (keys, vals) in zip(("ct4", "ct6"), ct[e]):
                ok, ov = maps[fam][e].dump()
                a, b = H.sorted_rows(keys, vals), H.sorted_rows(ok, ov)
                same &= a.shape == b.shape and bool((a == b).all())
        same &= bool((metrics == dp.metrics()).all())
        ok, ov = maps["policy"].dump()
        same &= bool((H.sorted_rows(pk, pv) == H.sorted_rows(ok, ov)).all())
        res["worlds"][world] = {"rounds": rounds, "cross_rank_deliveries": int(sum(r["cross"] for r in results)),
                                "wall_s": round(el, 1), "bit_exact_vs_sequential": bool(same)}
        print(f"[{time.time() - t0:.0f}s] world {world}: {rounds} rounds, exact {same}", file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
