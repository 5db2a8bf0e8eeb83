#!/bin/bash
# Experiment builds of libmgcn with -D flags: scripts/build_variants.sh NAME "-DFLAG ..." ...
# -> exp/libmgcn_NAME.so (exp/ is git-ignored; MGCN_LIB=<path> selects one)
set -e
cd "$(dirname "$0")/../meta-gcn_amd/csrc"
mkdir -p ../../exp
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mcode-object-version=5 -I../../include"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  mkdir -p ../../exp/$name
  for f in graph spmm elementwise; do cp build/$f.o ../../exp/$name/; done
  /opt/rocm/bin/hipcc $FLAGS $defs -c gemm.hip -o ../../exp/$name/gemm.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../exp/libmgcn_$name.so ../../exp/$name/*.o
done
