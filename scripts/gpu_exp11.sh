set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
for lds in 0 40960 53248 81920; do
  DML_REDUCE_LDS=$lds timeout -k 10 200 python scripts/exp_variants.py 0,28,20 4 > gpurun_out/lds_$lds.log 2>&1
  echo "lds=$lds"; grep variant gpurun_out/lds_$lds.log
done
