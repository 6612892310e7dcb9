set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
for iv in ${IVS:-0 2 3}; do for v in ${RVS:-0 21 28}; do
  DML_INDEX_VARIANT=$iv DML_REDUCE_VARIANT=$v timeout -k 10 200 python scripts/exp_order.py 3 > gpurun_out/x_${iv}_${v}.log 2>&1
  python3 scripts/summ_order.py gpurun_out/x_${iv}_${v}.log
done; done
