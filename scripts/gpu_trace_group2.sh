set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/tg -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu --sparse-steps 0 --group > gpurun_out/tg.log 2>&1
tail -3 gpurun_out/tg.log
ls gpurun_out/tg
