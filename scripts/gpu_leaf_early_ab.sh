# Sparse leaf A/B: default build vs DML_SP_LEAF_EARLY=1 / =2 builds (shard loads
# issued before the LDS sort; 1 = unsorted stores, 2 = address-order stores).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in e1 e2; do
DML_LIB_PATH=$GRAFT_REPO_ROOT/distml_amd/libdistml_ps_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "array or sparse or config3" -x -q --timeout 200 --timeout-method thread > gpurun_out/leaf_tests_$v.log 2>&1 || { tail -20 gpurun_out/leaf_tests_$v.log; exit 1; }
echo $v; tail -1 gpurun_out/leaf_tests_$v.log
done
for rep in 1 2 3; do
for lib in default e1 e2; do
if [ $lib = default ]; then unset DML_LIB_PATH; else export DML_LIB_PATH=$GRAFT_REPO_ROOT/distml_amd/libdistml_ps_$lib.so; fi
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --sparse-steps 20 > gpurun_out/sp.log 2>&1
tail -1 gpurun_out/sp.log | python3 -c "import sys,json; l=json.loads(sys.stdin.read())['sparse']; print('$lib', l['ms_per_step'], l['apply_kernel_us_avg'])"
done
done
