set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
for rep in 1 2; do
for lds in 0 40960 54000 65536 163840; do
  DML_REDUCE_LDS=$lds timeout -k 10 200 python scripts/exp_variants.py 28,0 3 > gpurun_out/lds_$lds.log 2>&1
  echo "lds=$lds $(grep variant gpurun_out/lds_$lds.log | tr '\n' ' ')"
done
done
