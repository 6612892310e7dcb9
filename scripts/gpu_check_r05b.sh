# k_flat_ident on the box: the parity tests that reach it (store + pre-reduce pieces),
# then the config-4 probe (kernel time per launch, 10 M and 1.25 M rows).
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "identity_speculation or flat_kernel_widths or config4 or sharded_speculation or prereduce or slot_reuse or shard_group" > gpurun_out/r05b_tests.log 2>&1 || { tail -40 gpurun_out/r05b_tests.log; exit 1; }
tail -3 gpurun_out/r05b_tests.log
timeout -k 10 300 python3 scripts/probe_flat.py --rows 10000000 1250000 --pushes 16 --reps 4 > gpurun_out/c4_probe_r05b.jsonl 2> gpurun_out/c4_probe_r05b.err
cat gpurun_out/c4_probe_r05b.jsonl
