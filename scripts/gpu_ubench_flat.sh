# Config-4 access-pattern sweep on the box (scripts/ubench_flat.hip): push-buffer
# staggering, one slab, push count, reads only. Each run its own time limit.
set -e
mkdir -p gpurun_out
O=gpurun_out/ubench_flat2.jsonl
: > $O
timeout -k 10 60 scripts/ubench_flat 1250000 16 0 0 >> $O
for ST in 256 4352 65792 1049088; do UB_ONLY=x timeout -k 10 60 scripts/ubench_flat 1250000 16 $ST 0 >> $O; done
UB_ONLY=x timeout -k 10 60 scripts/ubench_flat 1250000 16 0 1 >> $O
UB_ONLY=x timeout -k 10 60 scripts/ubench_flat 1250000 16 4352 1 >> $O
UB_ONLY=x timeout -k 10 60 scripts/ubench_flat 2500000 8 0 0 >> $O
UB_ONLY=x timeout -k 10 60 scripts/ubench_flat 625000 32 0 0 >> $O
UB_ONLY=x timeout -k 10 60 scripts/ubench_flat 5000000 4 0 0 >> $O
cat $O
