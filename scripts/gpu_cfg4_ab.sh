# Config 4 plain-sum shard (200 cols): reduce shape A/B (DML_REDUCE_VARIANT), interleaved.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for v in 0 40 41 42 43 44; do
DML_REDUCE_VARIANT=$v timeout -k 10 120 python bench.py --config 4 --no-cpu > gpurun_out/c4.log 2>&1
echo "v=$v $(tail -1 gpurun_out/c4.log | python3 -c "import sys,json; l=json.loads(sys.stdin.read()); print(l['ms_per_step'], l['roofline']['kernel_us_avg'], l['roofline']['achieved'])")"
done
done
