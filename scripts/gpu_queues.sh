set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
A="--legs 4a --sparse-steps 0 --no-cpu --c4a-steps 3"
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py $A > gpurun_out/q8.json 2> gpurun_out/q8.err
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python bench.py $A > gpurun_out/q4.json 2> gpurun_out/q4.err
timeout -k 10 300 python bench.py --legs "" --sparse-steps 0 --no-cpu --shuffle-keep-parity > gpurun_out/par.json 2> gpurun_out/par.err
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --group --legs "" --sparse-steps 0 --no-cpu > gpurun_out/g8.json 2> gpurun_out/g8.err
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python bench.py --group --legs "" --sparse-steps 0 --no-cpu > gpurun_out/g4.json 2> gpurun_out/g4.err
timeout -k 10 300 python bench.py --legs 4a --c4a-path moments --steps 50 --warmup 10 --sparse-steps 0 --no-cpu --c4a-steps 3 > gpurun_out/mom.json 2> gpurun_out/mom.err
echo ALLDONE
