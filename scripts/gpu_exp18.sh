set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
mkdir -p gpurun_out
for rep in 1 2; do
timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 > gpurun_out/b.json 2> gpurun_out/b.err
python3 -c "import json; d=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1]); print('timed', d['ms_per_step'], d['value'], d['roofline']['avg_kernel_us'])"
timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 --no-timing > gpurun_out/b.json 2> gpurun_out/b.err
python3 -c "import json; d=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1]); print('untimed', d['ms_per_step'], d['value'])"
timeout -k 10 300 python bench.py --no-cpu --sparse-steps 0 --steps 60 > gpurun_out/b.json 2> gpurun_out/b.err
python3 -c "import json; d=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1]); print('timed60', d['ms_per_step'], d['value'], d['roofline']['avg_kernel_us'])"
done
