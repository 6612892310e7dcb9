set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
for v in 30 31; do
  DML_REDUCE_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k config2_dense --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_v$v.log 2>&1 || { tail -30 gpurun_out/t_v$v.log; exit 1; }
  echo "variant $v: $(tail -1 gpurun_out/t_v$v.log)"
done
for v in 0 21 28 30 31; do
  DML_REDUCE_VARIANT=$v timeout -k 10 200 python scripts/exp_order.py 3 > gpurun_out/d_$v.log 2>&1
  python3 scripts/summ_order.py gpurun_out/d_$v.log
done
DML_STREAM_PRIO=1 timeout -k 10 200 python scripts/exp_order.py 3 > gpurun_out/d_prio.log 2>&1
python3 scripts/summ_order.py gpurun_out/d_prio.log
