set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
for lds in 0 81920 163840; do
  DML_REDUCE_LDS=$lds timeout -k 10 200 python scripts/exp_variants.py 0,28,21 4 > gpurun_out/lds_$lds.log 2>&1
  echo "lds=$lds"; grep variant gpurun_out/lds_$lds.log
done
for lds in 65536 54000; do
  DML_REDUCE_LDS=$lds timeout -k 10 200 python scripts/exp_variants.py 28 4 > gpurun_out/lds_$lds.log 2>&1
  echo "lds=$lds"; grep variant gpurun_out/lds_$lds.log
done
