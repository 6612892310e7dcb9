# Round-5 correctness checks on the box: the native group over the asynchronous RCCL
# stand-in (delayed collectives), the JNI snapshot entry points, the torch binding;
# then the same failure tests against a build WITHOUT the local-failure stream orders
# (scripts/ab/libdistml_ps_nofix.so), which must fail (the stand-in catches the race).
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_native_group.py tests/test_jni_shim.py tests/test_gpu_group.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r05a_tests.log 2>&1 || { tail -40 gpurun_out/r05a_tests.log; exit 1; }
tail -3 gpurun_out/r05a_tests.log
cp distml_amd/libdistml_ps.so /tmp/keep.so
cp scripts/ab/libdistml_ps_nofix.so distml_amd/libdistml_ps.so
if timeout -k 10 300 python -u -m pytest tests/test_native_group.py -m gpu -v -k "local_failure or begin_failure" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05a_nofix.log 2>&1; then
  echo "NOFIX: failure tests PASSED without the fix (race not caught)"
else
  echo "NOFIX: failure tests failed without the fix (race caught), rc=$?"
fi
cp /tmp/keep.so distml_amd/libdistml_ps.so
grep -E "PASSED|FAILED|assert" gpurun_out/r05a_nofix.log | head -12
