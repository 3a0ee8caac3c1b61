"""GraphML ingestion rate: native shd_graphml_parse vs the
Python ElementTree reader (stand-in for igraph's GraphML import, which is not
installed here) on a C3-style complete tmodel graph with self-loops.

usage: python tools/bench_graphml.py [n] > profiles/<tag>_graphml.json
Host-only (no GPU); prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "shadow-1_amd")]
from shdpe.engine import parse_graphml  # noqa: E402
from shdpe.graph import Topology, read_graphml, write_graphml  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    rng = np.random.default_rng(3)
    iu, ju = np.triu_indices(n)                       # complete + self-loops
    lat = np.clip(rng.lognormal(np.log(60.0), 0.8, iu.shape[0]), 1.0, 2000.0)
    top = Topology(n=n, directed=False, src=iu.astype(np.int32), dst=ju.astype(np.int32),
                   latency=lat, loss=np.full(iu.shape[0], 0.005), vloss=np.zeros(n))
    xml = write_graphml(top).encode()
    t0 = time.perf_counter()
    nat = parse_graphml(xml, with_ids=False)
    t1 = time.perf_counter()
    py = read_graphml(xml)
    t2 = time.perf_counter()
    same = (np.array_equal(nat.src, py.src) and np.array_equal(nat.dst, py.dst) and
            np.array_equal(nat.latency.view(np.int64), py.latency.view(np.int64)) and
            np.array_equal(nat.loss.view(np.int64), py.loss.view(np.int64)))
    print(json.dumps({
        "workload": f"complete graph n={n} with self-loops (C3 style, seed 3), write_graphml text",
        "edges": int(top.m), "bytes": len(xml),
        "native_s": t1 - t0, "native_MBps": len(xml) / (t1 - t0) / 1e6,
        "native_Medges_per_s": top.m / (t1 - t0) / 1e6,
        "python_elementtree_s": t2 - t1, "speedup": (t2 - t1) / (t1 - t0),
        "identical": bool(same), "cores": 1}))


if __name__ == "__main__":
    main()
