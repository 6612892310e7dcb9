# Two A/B runs in one call: nt shard-row loads in k_reduce_rows (config 2 line) and in
# k_reduce_flat (config 4 shards).
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
VARIANTS="rowsnt" bash scripts/gpu_ab_order.sh
VARIANTS="flatnt" CONFIGS="4 4-perm" bash scripts/gpu_ab_cfg.sh
