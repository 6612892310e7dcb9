# SQ counters of the config-4, config-4 AdaGrad and config-5 kernels (bench legs) and of
# the plain 4-read / 2-write stream (scripts/ubench_mix), two passes each, each pass its own
# time limit.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
O=$PWD/gpurun_out
BA="--legs 4,4a,5 --sparse-steps 0 --no-cpu --steps 3 --warmup 1 --c4-steps 1 --c4-warmup 0 --c4a-steps 1 --c4a-warmup 1 --c5-steps 2 --c5-warmup 0"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM SQ_CYCLES"
timeout -s KILL 240 rocprofv3 --pmc $P1 -d $O/sq1 -o run --output-format csv -- python3 bench.py $BA > $O/sq1.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc $P2 -d $O/sq2 -o run --output-format csv -- python3 bench.py $BA > $O/sq2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $P1 -d $O/sqm1 -o run --output-format csv -- scripts/ubench_mix 8 "r4w2 in place U4 nt nt" > $O/sqm1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $P2 -d $O/sqm2 -o run --output-format csv -- scripts/ubench_mix 8 "r4w2 in place U4 nt nt" > $O/sqm2.log 2>&1
M="k_ada_flat k_ada_ident k_flat_ident k_reduce_rows<int k_mix"
python3 scripts/pmc_reduce.py $O/sq_legs.json $O/sq1 $O/sq2 --match $M > /dev/null
python3 scripts/pmc_reduce.py $O/sq_mix.json $O/sqm1 $O/sqm2 --match $M > /dev/null
rm -rf $O/sq1 $O/sq2 $O/sqm1 $O/sqm2
cat $O/sq_legs.json $O/sq_mix.json
echo sq done
