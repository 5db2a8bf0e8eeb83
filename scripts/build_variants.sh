#!/bin/bash
# Experiment builds of libmgcn with -D flags: scripts/build_variants.sh NAME "-DFLAG ..." ...
# -> exp/libmgcn_NAME.so (exp/ is git-ignored; MGCN_LIB=<path> selects one)
# The -D flags apply to the sources listed in VARIANT_SRCS (default: gemm fused).
set -e
cd "$(dirname "$0")/../meta-gcn_amd/csrc"
mkdir -p ../../exp
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mcode-object-version=5 -I../../include"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  mkdir -p ../../exp/$name
  for f in graph spmm elementwise gemm fused; do
    case " ${VARIANT_SRCS:-gemm fused} " in
      *" $f "*) /opt/rocm/bin/hipcc $FLAGS $defs -c $f.hip -o ../../exp/$name/$f.o ;;
      *) cp build/$f.o ../../exp/$name/ ;;
    esac
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../exp/libmgcn_$name.so ../../exp/$name/*.o
done
