set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k config2_dense --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
DML_REDUCE_VARIANT=37 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k config2_dense --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t37.log 2>&1 || { tail -30 gpurun_out/t37.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/t.log) / v37 $(tail -1 gpurun_out/t37.log)"
for rep in 1 2; do
for v in 0 34 37; do
DML_REDUCE_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 > gpurun_out/b.json 2> gpurun_out/b.err
python3 -c "import json; d=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1]); print('v$v', d['ms_per_step'], d['value'], d['roofline']['avg_kernel_us'])"
done
done
