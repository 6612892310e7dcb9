set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
for rpw in 2 4; do
for lds in 0 54869; do
DML_REDUCE_LDS=$lds DML_NF_RPW=$rpw timeout -k 10 600 python bench.py --config 5 --cpu-seconds 0.5 > gpurun_out/cfg.log 2>&1
echo "rpw=$rpw lds=$lds $(tail -1 gpurun_out/cfg.log | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['roofline']['kernel_us_avg'], json.loads(l)['roofline']['achieved']) for l in sys.stdin]")"
done
done
