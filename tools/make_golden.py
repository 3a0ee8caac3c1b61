"""Generate the committed golden fixtures under tests/golden/.

Run here (the build container), where /root/reference exists:
    python tools/make_golden.py
Inputs taken from the reference are DATA only:
  * resource/topology.graphml.xml.xz  (shipped topology, 183 vertices)
  * the 1-vertex <topology> CDATA graphs of src/test/**/*.xml (known-answer
    direct-path cases: latency / packetloss of the single self-loop)
Expected outputs come from the CPU oracle (oracle/pe_oracle.c) -- the
Dijkstra tie order there is "igraph-0.7.1-reconstructed" (DESIGN.md).
"""
import glob
import json
import os
import re
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "shadow-1_amd"), os.path.join(R, "oracle")]
from shdpe import generators as G  # noqa: E402
from shdpe.graph import read_graphml  # noqa: E402
from oracle import OracleGraph  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(R, "tests", "golden")


def save_rows(path, top, att, sources, extra=None):
    og = OracleGraph(top)
    res = og.rows(np.asarray(sources, np.int32), att, threads=8)
    np.savez_compressed(path, n=np.int64(top.n), directed=np.int8(top.directed),
                        src=top.src, dst=top.dst, latency=top.latency, loss=top.loss,
                        vloss=(top.vloss if top.vloss is not None else np.zeros(0)),
                        has_vloss=np.int8(top.vloss is not None),
                        attached=np.asarray(att, np.int32), sources=np.asarray(sources, np.int32),
                        lat=res["lat"], rel=res["rel"], hops=res["hops"], pred=res["pred"],
                        flags=res["flags"], **(extra or {}))
    print("wrote", path, os.path.getsize(path), "bytes")


def main():
    os.makedirs(OUT, exist_ok=True)
    # 1. shipped topology as compact arrays
    shipped = read_graphml(os.path.join(REF, "resource", "topology.graphml.xml.xz"), name="shipped")
    shipped.save_npz(os.path.join(OUT, "shipped_topology.npz"))
    print("shipped:", shipped.n, "vertices", shipped.m, "edges")

    # 2. reference test configs: 1-vertex graphs (known-answer direct path)
    cases = []
    for f in sorted(glob.glob(os.path.join(REF, "src", "test", "**", "*.xml"), recursive=True)):
        txt = open(f, encoding="utf-8", errors="replace").read()
        m = re.search(r"<topology>\s*<!\[CDATA\[(.*?)\]\]>\s*</topology>", txt, re.S)
        if not m:
            continue
        top = read_graphml(m.group(1).strip())
        cases.append(dict(file=os.path.relpath(f, REF), n=top.n, directed=bool(top.directed),
                          src=top.src.tolist(), dst=top.dst.tolist(),
                          latency=top.latency.tolist(), loss=top.loss.tolist(),
                          vloss=(None if top.vloss is None else
                                 [None if np.isnan(x) else float(x) for x in top.vloss])))
    with open(os.path.join(OUT, "ref_test_topologies.json"), "w") as fh:
        json.dump(cases, fh, indent=1)
    print("reference test topologies:", len(cases))

    # 3. oracle rows
    att = np.arange(shipped.n, dtype=np.int32)
    minus1 = G.minus_one_edge(shipped, seed=0)
    save_rows(os.path.join(OUT, "rows_shipped_minus1.npz"), minus1, att, att)
    cfgs = [
        ("rows_rand_tiefree.npz", G.random_sparse(300, 6, seed=11), 1, 4),
        ("rows_rand_quantized.npz", G.random_sparse(300, 6, seed=12, quantum=1.0), 1, 3),
        ("rows_rand_directed.npz", G.random_sparse(300, 5, seed=13, directed=True), 1, 4),
        ("rows_rand_vloss.npz", G.random_sparse(300, 5, seed=14, vloss=True), 2, 2),
    ]
    for name, top, step, sstep in cfgs:
        a = np.arange(0, top.n, step, dtype=np.int32)
        save_rows(os.path.join(OUT, name), top, a, a[::sstep])
    rg = G.rgg(2000, seed=21)
    a = np.arange(rg.n, dtype=np.int32)
    save_rows(os.path.join(OUT, "rows_rgg2000.npz"), rg, a, a[::80])
    rq = G.rgg(2000, seed=22, quantum=0.005)
    save_rows(os.path.join(OUT, "rows_rgg2000_q.npz"), rq, a, a[::80])


if __name__ == "__main__":
    main()
