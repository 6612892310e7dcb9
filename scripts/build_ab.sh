# A/B library variant: the in-tree sources rebuilt with extra -D switches into
# scripts/ab/libdistml_ps_<NAME>.so (scripts/ab_multi.sh or scripts/gpu_leaf_ab.sh swap it in on the box).
#   bash scripts/build_ab.sh name -DSOME_SWITCH=1
set -e
NAME=$1; shift
cd "$(dirname "$0")/../distml_amd/csrc"
O=build_ab/$NAME; mkdir -p $O ../../scripts/ab
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -Wall -Wno-unused-result -I../../include -I. $*"
rm -f $O/*.o
pids=""
for s in dml_kernels dml_sparse dml_store dml_group dml_split; do /opt/rocm/bin/hipcc $F -c $s.hip -o $O/$s.o & pids="$pids $!"; done
for p in $pids; do wait $p || { echo "build_ab: a compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../../scripts/ab/libdistml_ps_$NAME.so $O/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built scripts/ab/libdistml_ps_$NAME.so
