# Identity-push detection A/B (DML_IDENT 1 on / 0 off), interleaved on one box.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for v in 1 0; do
DML_IDENT=$v timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 > gpurun_out/cfg2.log 2>&1
tail -1 gpurun_out/cfg2.log | python3 -c "import sys,json; l=json.loads(sys.stdin.read()); print('ident=$v config2', l['value'], l['ms_per_step'], l['roofline']['avg_kernel_us'])"
for c in 5 4-asc; do
DML_IDENT=$v timeout -k 10 200 python bench.py --config $c --no-cpu > gpurun_out/c.log 2>&1
tail -1 gpurun_out/c.log | python3 -c "import sys,json; l=json.loads(sys.stdin.read()); print('ident=$v', sys.argv[1], l['ms_per_step'], l['roofline']['kernel_us_avg'])" $c
done
done
done
