# End-of-round GPU call: the round script (suite, smoke, default line, world-1 sharded
# line, line profile with PMC passes), then the N = 2 legs rehearsed on one GPU (gloo).
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
bash scripts/gpu_round.sh
timeout -k 10 400 python bench.py --gpus 2 --rehearse-gloo --c4-pushes 4 --no-cpu --steps 50 --warmup 20 > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err
python -c "import json;d=json.load(open('gpurun_out/rehearse2.json'));print('rehearse N=2', d['n_gpus'], d['ms_per_step'], sorted(k for k in d if k.startswith('config')))"
