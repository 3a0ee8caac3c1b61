"""Turn one workload's rocprofv3 PMC passes into profiles/traffic_<wl>.json.

usage: python tools/traffic_json.py <pmc outdir> <workload> <tag> [out.json [part-csv prefix]]

Reads the counter_collection CSVs under <outdir>/pmc_<wl>_* (one launch of
the dominant kernel per pass, bench.py --steps 1 --warmup 0), applies the
gfx950 FETCH_SIZE correction this kernel shape was calibrated for
(profiles/r02e_fetch_calibration.json: random 128-B lines read by 16-lane
groups report half their bytes) and records the kernel-source hash of the
library that was measured, so bench.py only reports `traffic` for a build
whose sources match (shdpe.engine.kernel_source_hash).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "shadow-1_amd")]

KERNELS = ("k_batch_rows", "k_sparse_rows", "k_minplus", "k_direct_rows")


def main():
    outdir, wl, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    dst = sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "profiles", f"traffic_{wl}.json")
    # per pass, only the measured step: the LAST dispatch of each path kernel
    # (bench.py runs shd_pe_tune -- both kernel variants -- before it); the
    # split batch path runs two kernels per step (k_batch_rows<.., 1> relax,
    # <.., 2> post): the last post dispatch and the relax dispatch before it
    per = defaultdict(list)          # (file, kernel family) -> [(dispatch, name, row)]
    for f in glob.glob(os.path.join(outdir, f"pmc_{wl}_*", "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            k = next((k for k in KERNELS if k in name), None)
            if k is None:
                continue
            per[(f, k)].append((int(r.get("Dispatch_Id") or 0), name, r))
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(lambda: defaultdict(set))
    parts = defaultdict(lambda: defaultdict(float))   # split batch path: relax / post separately
    for (f, k), rs in per.items():
        ids = sorted({d for d, _, _ in rs})
        last = ids[-1]
        lastName = next(nm for d, nm, _ in rs if d == last)
        keep = {last}
        if ", 2>(" in lastName:
            prev = [d for d, nm, _ in rs if d < last and ", 1>(" in nm]
            if prev:
                keep.add(max(prev))
        for d, nm, r in rs:
            if d in keep:
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k][r["Counter_Name"]].add((f, d))
                if k == "k_batch_rows" and (", 1>(" in nm or ", 2>(" in nm):
                    parts["relax" if ", 1>(" in nm else "post"][r["Counter_Name"]] += float(r["Counter_Value"])
    if not tot:
        sys.exit(f"no counters for the path kernels under {outdir}/pmc_{wl}_*")
    k = max(tot, key=lambda x: tot[x].get("FETCH_SIZE", 0.0))
    c = tot[k]
    nl = max(1, len(disp[k].get("FETCH_SIZE", ())))
    fetch = c.get("FETCH_SIZE", 0.0) * 1024      # one measured step (1 or 2 dispatches)
    write = c.get("WRITE_SIZE", 0.0) * 1024
    hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
    from shdpe.engine import kernel_source_hash
    out = {
        "kernel": k,
        "bytes_per_launch": 2 * fetch + write,
        "read_bytes": 2 * fetch,
        "fetch_size_bytes": fetch,
        "write_bytes": write,
        "l2_hit_rate": hit / (hit + miss) if hit + miss else None,
        "dispatches_per_step": nl,
        "dispatch": "the measured step only: the last launch of the pass, with the relax launch before it "
                    "when the batch path runs split (the tuning launches before them are ignored)",
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes, KB*1024, "
                  "bench.py --steps 1 --warmup 0 (one launch).  Reads = 2 x FETCH_SIZE (gfx950 "
                  "calibration for random 128-B lines, profiles/r02e_fetch_calibration.json); "
                  "writes = WRITE_SIZE.  L2-miss traffic (includes Infinity-Cache hits): an upper "
                  "bound on HBM bytes.",
        "tag": tag,
        "src_hash": kernel_source_hash(),
    }
    if k == "k_batch_rows" and parts:
        # per kernel of the split path (where the excess goes)
        out["parts"] = {}
        for pn, pc in parts.items():
            pf, pw = pc.get("FETCH_SIZE", 0.0) * 1024, pc.get("WRITE_SIZE", 0.0) * 1024
            ph, pm = pc.get("TCC_HIT_sum", 0.0), pc.get("TCC_MISS_sum", 0.0)
            out["parts"][pn] = {"bytes": 2 * pf + pw, "read_bytes": 2 * pf, "write_bytes": pw,
                                "l2_hit_rate": ph / (ph + pm) if ph + pm else None,
                                "counters": dict(pc)}
        if len(sys.argv) > 5:        # per-part counter CSVs: <prefix>_{relax,post}.csv
            for pn, pc in parts.items():
                with open(f"{sys.argv[5]}_{pn}.csv", "w") as f:
                    f.write("counter,value_per_step\n")
                    for cn in sorted(pc):
                        f.write(f"{cn},{pc[cn]:.0f}\n")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
