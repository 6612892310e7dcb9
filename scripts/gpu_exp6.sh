set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
for rep in 1 2; do
for sk in 0 1; do
  DML_SKIP_MEMSET=$sk timeout -k 10 200 python scripts/exp_order.py 3 > gpurun_out/sk_$sk.log 2>&1
  echo "skip_memset=$sk $(python3 scripts/summ_order.py gpurun_out/sk_$sk.log)"
done
DML_SERIAL_INDEX=1 timeout -k 10 200 python scripts/exp_order.py 3 > gpurun_out/ser.log 2>&1
echo "serial $(python3 scripts/summ_order.py gpurun_out/ser.log)"
done
