# HBM read:write mix sweep on the box (scripts/ubench_mix.hip), 2 and 8 GiB per array.
set -e
mkdir -p gpurun_out
O=gpurun_out/ubench_mix.jsonl
: > $O
timeout -k 10 120 scripts/ubench_mix 2 >> $O
timeout -k 10 300 scripts/ubench_mix 8 >> $O
cat $O
