# Dense reduce geometry sweep (scripts/ubench_geom.hip): config 2's and
# config 4's geometries and their crosses, then the two alternated in one process.
set -e
mkdir -p gpurun_out
O=gpurun_out/ubench_geom.jsonl
: > $O
timeout -k 10 240 scripts/ubench_geom "" ${ROUNDS:-2} >> $O
timeout -k 10 120 scripts/ubench_geom alt 4 >> $O
python3 - <<'PY'
import json
for ln in open("gpurun_out/ubench_geom.jsonl"):
    d = json.loads(ln)
    print(f'{d["case"][:42]:42s} r{d["round"]} U{d["U_KiB_per_wave"]:2d} D{d["D"]} {d["mode"][:16]:16s} x{d["xcd"]} ws {d["write_share"]:.3f} best {d["best_us"]:9.1f} frac {d["frac_best"]:.4f} mean {d["frac_mean"]:.4f}')
PY
