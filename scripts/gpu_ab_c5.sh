# Listed-row skip for sparse-row chunks (config 5): the parity tests, then A/B of the
# config-5 leg against scripts/ab/libdistml_ps_nolisted.so, 3 rounds.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_c5_tests.log 2>&1 || { tail -30 gpurun_out/ab_c5_tests.log; exit 1; }
tail -1 gpurun_out/ab_c5_tests.log
B=nolisted ARGS="--legs 5 --sparse-steps 0 --no-cpu --steps 5 --warmup 2" ROUNDS=3 bash scripts/ab_bench.sh
for f in gpurun_out/ab_new_*.json gpurun_out/ab_nolisted_*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); x=d['config5']; print(sys.argv[1], x['ms_per_step'], x['roofline']['frac'], x['roofline']['avg_kernel_us'])" $f; done
