# r04d: N=8 / N=4 shard knob sweep, then the HEAD profile set (default bench, rocprof trace, PMC traffic)
STAGES=shard SHARD_NS="4 8" SHARD_ENVS="X=0;SHDPE_BATCH_DELTA_FACTOR=1.5;SHDPE_BATCH_DELTA_FACTOR=3;SHDPE_HEAVY_DEG=32;SHDPE_HEAVY_DEG=128;SHDPE_BATCH_WPE=8;SHDPE_BATCH_LB=16 SHDPE_BATCH_DELTA_FACTOR=1.5" bash tools/gpu_r04.sh r04d || exit 1
STAGES="default trace pmc" WLS=c4 bash tools/gpu_r04.sh r04d
