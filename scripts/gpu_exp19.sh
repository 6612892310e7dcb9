set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2; do
timeout -k 10 300 python bench.py --no-cpu --steps 50 --warmup 20 --sparse-steps 20 > gpurun_out/b.json 2> gpurun_out/b.err
python3 -c "import json; d=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1]); print(d['sparse'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sparse -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --sparse-steps 10 > gpurun_out/prof_sparse.log 2>&1
