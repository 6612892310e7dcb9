# FETCH_SIZE of k_reduce per variant (separate pmc passes; no tracing combined)
set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
for v in ${VARIANTS:-3 10}; do
  DML_REDUCE_VARIANT=$v timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_v$v -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --sparse-steps 0 > gpurun_out/pmc_v$v.log 2>&1
done
