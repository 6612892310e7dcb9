# Kernel trace (start / end of every dispatch) of a short config-2 line, for the
# gaps between consecutive reduces: TAG=cfg2 ARGS="..." bash scripts/gpu_trace.sh
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-cfg2}
timeout -k 10 300 rocprofv3 --kernel-trace -d "$PWD/gpurun_out/trace_$T" -o run --output-format csv -- python3 bench.py ${ARGS:---legs "" --sparse-steps 0 --no-cpu --steps 200 --warmup 100} > gpurun_out/trace_$T.log 2>&1
ls -la gpurun_out/trace_$T
