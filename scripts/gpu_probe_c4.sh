# Config-4 kernel probe on the box: model-size sweep, stream ceilings,
# then SQ / TA counter passes over the 10 M-row case (each pass its own time limit).
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
O=$PWD/gpurun_out
timeout -k 10 300 python3 scripts/probe_flat.py --rows 10000000 2500000 1250000 --pushes 16 --reps 4 --streams > $O/c4_probe.jsonl 2> $O/c4_probe.err
cat $O/c4_probe.jsonl
timeout -k 10 60 rocprofv3 -L > $O/rocprof_L.txt 2>&1 || true
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD" ${EXTRA_PMC:-}; do
  N=$(echo $P | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/c4pmc_$N -o run --output-format csv -- python3 scripts/probe_flat.py --rows 10000000 --pushes 16 --reps 2 > $O/c4pmc_$N.log 2>&1
done
echo probe done
