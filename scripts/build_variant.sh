#!/bin/bash
# Build an A/B variant of the product library: hg_physics2.hip recompiled with extra flags, linked
# with the product objects of every other source.  Usage: build_variant.sh <name> "<flags>"
set -e
cd "$(dirname "$0")/../humanoid-gym-with-comments_amd"
make -s
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-result -fno-slp-vectorize $1 \
  -I csrc -I ../include -c ${SRC:-csrc/hg_physics2.hip} -o /tmp/hg_physics2_$name.o -Rpass-analysis=kernel-resource-usage 2>&1 \
  | grep -A10 "ILb0E" | grep -E "VGPRs|Scratch" | sed "s/.*remark: *//" | tr '\n' ' '; echo
objs=$(ls csrc/*.o | grep -v hg_physics2.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o csrc/libhgsim_rep_$name.so $objs /tmp/hg_physics2_$name.o
