# Config 5 per-GPU shard: shard-store policy A/B (DML_NF_SNT 0 plain, 1 nt, 2 write-through), interleaved.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp CFG_CPU_S=0.5
mkdir -p gpurun_out
for rep in 1 2; do
for v in 0 1 2; do
DML_NF_SNT=$v timeout -k 10 120 python bench.py --config 5 --cpu-seconds 0.5 > gpurun_out/c5.log 2>&1
echo "snt=$v $(tail -1 gpurun_out/c5.log | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['roofline']['kernel_us_avg'], json.loads(l)['roofline']['achieved']) for l in sys.stdin]")"
done
done
