"""Copy a bench profile capture (gpurun_out/bench_<tag>) into profiles/.

Writes profiles/<tag>_<wl>_kernel_stats.csv (rocprofv3 --stats of the bench
command), profiles/<tag>_<wl>_pmc.json (per-dispatch PMC totals of the
dominant kernel, each counter from its own --pmc pass) and
profiles/traffic_<wl>.json (HBM bytes per launch, read by bench.py).
"""
import csv, json, os, shutil, sys, collections

tag, wl = sys.argv[1], sys.argv[2]
kern = sys.argv[3] if len(sys.argv) > 3 else "k_sparse_rows"
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(R, "gpurun_out", f"bench_{tag}")
dst = os.path.join(R, "profiles")
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "trace_kernel_stats.csv"),
            os.path.join(dst, f"{tag}_{wl}_kernel_stats.csv"))
pmc = {}
for d in sorted(os.listdir(src)):
    if not d.startswith("pmc_"):
        continue
    p = os.path.join(src, d, "pmc_counter_collection.csv")
    agg = collections.defaultdict(float); disp = collections.defaultdict(set)
    for r in csv.DictReader(open(p)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
    for k, v in agg.items():
        pmc[k] = {"total": v, "dispatches": len(disp[k]), "per_dispatch": v / len(disp[k])}
out = {"kernel": kern, "workload": wl, "tag": tag, "counters": pmc}
bench = open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1]
out["bench_line"] = json.loads(bench)
json.dump(out, open(os.path.join(dst, f"{tag}_{wl}_pmc.json"), "w"), indent=1)
if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
    fetch = pmc["FETCH_SIZE"]["per_dispatch"] * 1024
    write = pmc["WRITE_SIZE"]["per_dispatch"] * 1024
    # k_batch_rows reads [v][LB] lines with 16-lane groups: the calibrated
    # shape (random 128-B lines report exactly half).  Other kernels read
    # narrower pieces, where one request may move 64 or 128 B: FETCH_SIZE as
    # is (lower bound), 2x as the upper bound.
    lines = kern == "k_batch_rows"
    read = 2 * fetch if lines else fetch
    traffic = {"bytes_per_launch": read + write, "read_bytes": read,
               "read_bytes_upper": 2 * fetch, "fetch_size_bytes": fetch, "write_bytes": write,
               "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes, "
                         "KB*1024, bench.py --steps 1 (one launch).  "
                         + ("Reads = 2 x FETCH_SIZE: calibrated on gfx950 for this kernel's "
                            "dominant read shape (random 128-B lines read by 16-lane groups "
                            "report exactly half, like 16-B/lane streaming; "
                            "profiles/r02e_fetch_calibration.json).  " if lines else
                            "Reads = FETCH_SIZE (lower bound; 64- or 128-B requests cannot be "
                            "told apart, read_bytes_upper = 2 x).  ")
                         + "Writes = WRITE_SIZE (exact in the same calibration).  EA requests "
                           "include Infinity-Cache hits: L2-miss traffic, an upper bound on "
                           "HBM bytes.",
               "tag": tag}
    json.dump(traffic, open(os.path.join(dst, f"traffic_{wl}.json"), "w"), indent=1)
print(json.dumps({k: v["per_dispatch"] for k, v in pmc.items()}, indent=1))
