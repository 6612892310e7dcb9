# AdaGrad: GPU parity suite, then an interleaved A/B of the reduce shapes
# (DML_ADA_VARIANT) on config 4's per-GPU shard.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp CFG_CPU_S=0.5
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -2 gpurun_out/pytest_gpu.log
for rep in 1 2; do
for v in ${ADA_VARIANTS:-0 7 1 8}; do
DML_ADA_VARIANT=$v timeout -k 10 120 python bench.py --config 4-ada --cpu-seconds 0.5 > gpurun_out/ada.log 2>&1
echo "v=$v $(tail -1 gpurun_out/ada.log | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['roofline']['kernel_us_avg'], json.loads(l)['roofline']['achieved']) for l in sys.stdin]")"
done
done
