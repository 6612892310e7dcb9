# One GPU call: the -m gpu suite, smoke, the default bench line (wall time), the
# N = 2 legs rehearsed on one GPU (gloo, both ranks on cuda:0: plumbing, not a
# measurement) and the host-memory end-to-end rates (scripts/e2e.py).
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
t0=$(date +%s); timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; t1=$(date +%s)
echo "bench wall $((t1 - t0)) s"; cat gpurun_out/bench.json
timeout -k 10 400 python bench.py --gpus 2 --rehearse-gloo --c4-pushes 4 --no-cpu --steps 50 --warmup 20 > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err
cat gpurun_out/rehearse2.json
timeout -k 10 300 python scripts/e2e.py > gpurun_out/e2e.log 2>&1
cat gpurun_out/e2e.log
