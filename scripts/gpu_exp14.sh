set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python scripts/exp_variants.py 0,29,28 4 > gpurun_out/var.log 2>&1
grep variant gpurun_out/var.log
for rep in 1 2; do
timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 > gpurun_out/bench.json 2> gpurun_out/bench.err
python3 -c "import json; d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1]); print('single', d['ms_per_step'], d['value'], d['roofline']['avg_kernel_us'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 --group > gpurun_out/bench_group.json 2> gpurun_out/bench_group.err
python3 -c "import json; d=json.loads(open('gpurun_out/bench_group.json').read().strip().splitlines()[-1]); print('group', d['ms_per_step'], d['value'])"
done
