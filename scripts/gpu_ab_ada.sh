# k_ada_flat write-burst A/B (new: 8-wave blocks + barrier before the write-back;
# scripts/ab/libdistml_ps_adaold.so: 4-wave blocks, no barrier), then the AdaGrad tests.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "adagrad or ada" > gpurun_out/ab_ada_tests.log 2>&1 || { tail -30 gpurun_out/ab_ada_tests.log; exit 1; }
tail -1 gpurun_out/ab_ada_tests.log
B=adaold ARGS="--legs 4a --sparse-steps 0 --no-cpu --steps 5 --warmup 2" ROUNDS=2 bash scripts/ab_bench.sh
for f in gpurun_out/ab_new_*.json gpurun_out/ab_adaold_*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); x=d['config4_ada']; print(sys.argv[1], x['ms_per_step'], x['roofline']['frac'], x['roofline']['avg_kernel_us'], x['roofline']['kernel'])" $f; done
