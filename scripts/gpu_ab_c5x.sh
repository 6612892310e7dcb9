set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
cp distml_amd/libdistml_ps.so /tmp/ab_new.so
cp scripts/ab/libdistml_ps_c5x.so distml_amd/libdistml_ps.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "config5 or int or lda or matrix_random" > gpurun_out/c5x_tests.log 2>&1 || { cp /tmp/ab_new.so distml_amd/libdistml_ps.so; tail -20 gpurun_out/c5x_tests.log; exit 1; }
tail -1 gpurun_out/c5x_tests.log
cp /tmp/ab_new.so distml_amd/libdistml_ps.so
VARIANTS="c5x" CONFIGS="5" bash scripts/gpu_ab_cfg.sh
