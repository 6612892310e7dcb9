# Kernel + HIP runtime trace of a config-2 line (no legs): gaps between consecutive
# reduces and where the host enqueued each one (scripts/trace_host.py).
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d "$PWD/gpurun_out/trace_host" -o run --output-format csv -- python3 bench.py --legs none --sparse-steps 0 --no-cpu --steps 200 --warmup 50 > gpurun_out/trace_host.log 2>&1
ls gpurun_out/trace_host/*/ 2>/dev/null | head; ls gpurun_out/trace_host | head
python3 scripts/trace_host.py gpurun_out/trace_host k_reduce_rows | tee gpurun_out/trace_host.txt
python3 scripts/trace_gaps.py $(find gpurun_out/trace_host -name "*kernel_trace.csv" | head -1) k_reduce_rows 2 >> gpurun_out/trace_host.txt
find gpurun_out/trace_host -name "*hip_api_trace.csv" -size +30M -delete
