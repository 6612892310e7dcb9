# Config-2 buffer placement: timing of four bucket sets (in order /
# shuffled, allocated first / after), then one TCC counter pass over the same program.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 200 python3 scripts/probe_placement.py --rounds 3 --steps 100 > gpurun_out/placement.jsonl 2> gpurun_out/placement.err
timeout -k 10 200 python3 scripts/probe_placement.py --rounds 2 --steps 100 --slab > gpurun_out/placement_slab.jsonl 2>> gpurun_out/placement.err
cat gpurun_out/placement.jsonl gpurun_out/placement_slab.jsonl | cut -c1-160
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/placement_pmc -o run --output-format csv -- python3 scripts/probe_placement.py --rounds 1 --steps 20 > gpurun_out/placement_pmc.log 2>&1
echo pmc done
