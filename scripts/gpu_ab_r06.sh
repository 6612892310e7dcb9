# Round 6 A/Bs on one box, alternating builds (scripts/ab_multi.sh): k_ada_vec shapes
# against k_ada_ident (config-4 AdaGrad leg), then the geometry pair in one process.
set -e
export TMPDIR=/tmp; mkdir -p gpurun_out
VARIANTS="base adavec1 adavec2 adavec4" ARGS="--legs 4a --sparse-steps 0 --no-cpu --steps 20 --warmup 5 --c4a-steps 4" LEG=config4_ada ROUNDS=2 bash scripts/ab_multi.sh 2>&1 | tee gpurun_out/ab_ada_vec.txt
for f in gpurun_out/abm_*_1.json gpurun_out/abm_*_2.json; do python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['config4_ada']['roofline'];print(sys.argv[1], r.get('measured_stream_floor_us'), r.get('frac_of_measured_floor'))" $f; done
