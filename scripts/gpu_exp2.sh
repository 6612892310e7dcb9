set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
for v in 0 21; do
  DML_SERIAL_INDEX=1 DML_REDUCE_VARIANT=$v timeout -k 10 200 python scripts/exp_order.py 3 > gpurun_out/ser_v$v.log 2>&1
  echo "serial v=$v"; grep row_order gpurun_out/ser_v$v.log
  DML_REDUCE_VARIANT=$v timeout -k 10 200 python scripts/exp_order.py 3 > gpurun_out/ovl_v$v.log 2>&1
  echo "overlap v=$v"; grep row_order gpurun_out/ovl_v$v.log
done
