#!/bin/bash
# A/B render variants: recompile mg_raster.hip with extra defines and link it with the other objects of the
# default build into magical_amd/libmagical_sim_<tag>.so (selected at run time by MAGICAL_AMD_EXP_LIB=<tag>)
# usage: tools/build_variants.sh tag "-DX=1 -DY=2" [tag2 "defs2" ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd); P=$R/magical-1_amd; B=$P/build
while [ $# -ge 2 ]; do
  tag=$1; defs=$2; shift 2
  ( hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wno-unused-result $defs \
      -c $P/csrc/mg_raster.hip -o $B/mg_raster.$tag.o &&
    objs=$(ls $B/*.opt.o | grep -v mg_raster) &&
    hipcc --offload-arch=gfx950 -shared -fPIC -o $P/magical_amd/libmagical_sim_$tag.so $objs $B/mg_raster.$tag.o &&
    echo "built $tag ($defs)" ) &
done
wait
