set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
timeout -k 10 200 python scripts/exp_variants.py 0 4 > gpurun_out/v0.log 2>&1; grep variant gpurun_out/v0.log
DML_REDUCE_LDS=54869 timeout -k 10 200 python scripts/exp_variants.py 31,29,20 4 > gpurun_out/v31.log 2>&1; grep variant gpurun_out/v31.log
DML_REDUCE_LDS=81920 timeout -k 10 200 python scripts/exp_variants.py 31 4 > gpurun_out/v31b.log 2>&1; grep variant gpurun_out/v31b.log
DML_REDUCE_LDS=163840 timeout -k 10 200 python scripts/exp_variants.py 31,30 4 > gpurun_out/v31c.log 2>&1; grep variant gpurun_out/v31c.log
timeout -k 10 200 python scripts/exp_variants.py 0 4 > gpurun_out/v0.log 2>&1; grep variant gpurun_out/v0.log
