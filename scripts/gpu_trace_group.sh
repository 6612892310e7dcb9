set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/trace_group -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --no-cpu --group --sparse-steps 0 > gpurun_out/trace_group.log 2>&1
ls gpurun_out/trace_group
