# k_ada_ident on the box: its parity tests, then the config-4 AdaGrad leg against the
# build without it (scripts/ab/libdistml_ps_noadaident.so), 2 rounds, then the SQ passes.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  -k "adagrad_ident or adagrad_flat or (config4_model_size and adagrad)" > gpurun_out/ada_tests.log 2>&1 || { tail -30 gpurun_out/ada_tests.log; exit 1; }
tail -1 gpurun_out/ada_tests.log
B=noadaident ARGS="--legs 4a --sparse-steps 0 --no-cpu --steps 5 --warmup 2" ROUNDS=2 bash scripts/ab_bench.sh
for f in gpurun_out/ab_new_1.json gpurun_out/ab_noadaident_1.json gpurun_out/ab_new_2.json gpurun_out/ab_noadaident_2.json; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); x=d['config4_ada']; print(sys.argv[1], x['ms_per_step'], x['roofline']['frac'], x['roofline']['avg_kernel_us'], x['roofline']['kernel'])" $f
done
bash scripts/gpu_sq_legs.sh
