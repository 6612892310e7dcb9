set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
timeout -k 10 200 python scripts/exp_order.py 5 > gpurun_out/exp_base.log 2>&1; cat gpurun_out/exp_base.log
for lds in 24576 40960 81920; do
  DML_REDUCE_LDS=$lds timeout -k 10 200 python scripts/exp_order.py 3 > gpurun_out/exp_lds$lds.log 2>&1
  echo "lds=$lds"; grep row_order gpurun_out/exp_lds$lds.log
done
for v in 11 14; do
  DML_REDUCE_VARIANT=$v timeout -k 10 200 python scripts/exp_order.py 3 > gpurun_out/exp_v$v.log 2>&1
  echo "v=$v"; grep row_order gpurun_out/exp_v$v.log
done
