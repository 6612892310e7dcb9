# Sparse leaf block size A/B: default build (512 threads) vs DML_LIB_PATH=leaf256 build.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/distml_amd/libdistml_ps_leaf256.so
DML_LIB_PATH=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "array or sparse or config3" -x -q --timeout 200 --timeout-method thread > gpurun_out/leaf_tests.log 2>&1 || { tail -20 gpurun_out/leaf_tests.log; exit 1; }
tail -1 gpurun_out/leaf_tests.log
for rep in 1 2; do
for lib in default leaf256; do
if [ $lib = leaf256 ]; then export DML_LIB_PATH=$V; else unset DML_LIB_PATH; fi
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --sparse-steps 20 > gpurun_out/sp.log 2>&1
tail -1 gpurun_out/sp.log | python3 -c "import sys,json; l=json.loads(sys.stdin.read())['sparse']; print('$lib', l['ms_per_step'], l['apply_kernel_us_avg'])"
done
done
