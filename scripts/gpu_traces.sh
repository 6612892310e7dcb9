# Kernel traces of the config-2 line, the sparse leg and the world-1 sharded path
# (gaps between dispatches: scripts/trace_gaps.py).
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=cfg2 ARGS='--legs x --sparse-steps 0 --no-cpu --steps 200 --warmup 100' bash scripts/gpu_trace.sh
TAG=sparse ARGS='--legs x --no-cpu --steps 20 --warmup 10 --sparse-steps 40' bash scripts/gpu_trace.sh
TAG=group ARGS='--group --legs x --no-cpu --sparse-steps 0 --steps 200 --warmup 100' bash scripts/gpu_trace.sh
