# The whole -m gpu suite and smoke() on the current sources.
export TMPDIR=/tmp; mkdir -p gpurun_out
DML_PARITY_LOG=gpurun_out/parity_rs_full.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -3 gpurun_out/gpu_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/gpu_tests.log | head
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"; echo "smoke rc=$?"
