set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench2.json 2> gpurun_out/bench2.err
cat gpurun_out/bench2.json
timeout -k 10 400 python scripts/tune.py 3 > gpurun_out/tune4.log 2>&1
cat gpurun_out/tune4.log
