"""Per-rank compute time of one shard of the C4 table on this GPU (what
rank 0 of an N-GPU bench run does): tools/shard_time.py <workload> <N>..."""
import sys, os, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "shadow-1_amd")]
import numpy as np
from shdpe import generators as G
from shdpe.engine import Engine, DEBUG_ENV

wl = sys.argv[1]
top, att = G.make_config(wl)
for N in [int(x) for x in sys.argv[2:]]:
    dbg = DEBUG_ENV if any(k.startswith("SHDPE_") for k in os.environ) else 0
    K = int(os.environ.get("SUBK", "1"))     # row shards per GPU on concurrent streams
    eng = Engine(top, att, shard_index=0, shard_count=N, debug_flags=dbg,
                 devices=[0] * K if K > 1 else None)
    s0, cnt = eng.owned
    pos = np.arange(s0, s0 + cnt, dtype=np.int32)
    eng.tune()                               # as bench.py: per-box kernel variants
    eng.compute_positions(s0, cnt)           # warm-up (allocations)
    best = 1e9
    for _ in range(3):
        eng.reset_stats()
        t = time.perf_counter()
        eng.compute_positions(s0, cnt)
        eng.synchronize()
        best = min(best, time.perf_counter() - t)
    st = eng.stats()
    print(f"{wl} N={N} rows={cnt} ms={best*1e3:.1f} lanes={st['batchLanes']} "
          f"waves={st['batchWaves']}/{st['batchPostWaves']} coop={st.get('batchCoop', 0)} "
          f"aborts={st.get('relaxCoopAborts', 0)} exact={st['rowsExact']} "
          f"rows/s/gpu={cnt/best:.0f} -> {N*cnt/best:.0f} total "
          f"[{' '.join(k + '=' + v for k, v in os.environ.items() if k.startswith('SHDPE_') or k == 'SUBK')}]", flush=True)
    eng.close()
