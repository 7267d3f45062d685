#!/bin/bash
# Timing experiments: recompile ONE translation unit with extra defines and link it with the other objects
# of the default build into magical_amd/libmagical_sim_<tag>.so (selected at run time by
# MAGICAL_AMD_EXP_LIB=<tag>; tools/gpu_ab.sh).  usage: tools/build_unit_variant.sh unit tag "-DX=1" [tag2 "defs2" ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd); P=$R/magical-1_amd; B=$P/build
unit=$1; shift
base=${unit%.hip}
while [ $# -ge 2 ]; do
  tag=$1; defs=$2; shift 2
  ( hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wno-unused-result $defs \
      -c $P/csrc/$unit -o $B/$base.$tag.o &&
    objs=$(ls $B/*.opt.o | grep -v "/$base.opt.o") &&
    hipcc --offload-arch=gfx950 -shared -fPIC -o $P/magical_amd/libmagical_sim_$tag.so $objs $B/$base.$tag.o &&
    echo "built $tag ($defs)" ) &
done
wait
