# Final round-6 evidence at HEAD.  A: the driver's default bench line and
# rocprofv3 kernel stats of quick lines (C4, C5, C2, C3b); B: PMC traffic
# passes (C4, C2, C5) -> traffic_<wl>.json with HEAD's source hash, and the
# per-rank C4 shard times at N = 1 / 2 / 4 / 8.
# usage: bash tools/gpu_r06_final.sh TAG A|B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-r06f}
case ${2:-A} in
  A) STAGES="default" tools/gpu_r05.sh $T && WLS=c4,c5,c2,c3b STAGES=trace tools/gpu_r05.sh $T ;;
  B) WLS=c4,c2,c5 STAGES=pmc tools/gpu_r05.sh $T && SHARD_NS="1 2 4 8" SHARD_WL=c4 STAGES=shard tools/gpu_r05.sh $T ;;
esac
