# AdaGrad-shaped stream variants (scripts/ubench_mix.hip "ada" cases) against the plain
# 4-read / 2-write stream, and the XCD-contiguous block order, 8 GiB per array.
set -e
mkdir -p gpurun_out
timeout -k 10 200 scripts/ubench_mix 8 "ada" > gpurun_out/ubench_ada.jsonl
timeout -k 10 100 scripts/ubench_mix 8 "r4w2 in place U4 nt nt" >> gpurun_out/ubench_ada.jsonl
timeout -k 10 200 scripts/ubench_mix 8 "r17w1 in place" >> gpurun_out/ubench_ada.jsonl
cat gpurun_out/ubench_ada.jsonl
