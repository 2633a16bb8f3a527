#!/bin/bash
# Build an A/B variant of libegraph.so: csrc/$FILE (default frontier.hip) recompiled with extra flags (and
# optionally from another source tree, e.g. `git archive` of an older commit), linked with the
# default build's other objects -> kubernetes-aiops-evidence-graph_amd/lib/exp_<name>/libegraph.so
# Usage: scripts/build_variant.sh NAME "FLAGS" [CSRC_DIR]      (CPU container; hipcc only)
set -e
NAME=$1; FLAGS=$2; SRC=${3:-}
PKG=$(cd "$(dirname "$0")/../kubernetes-aiops-evidence-graph_amd" && pwd)
cd "$PKG"
CS=${SRC:-$PKG/csrc}
FILE=${FILE:-frontier.hip}
mkdir -p build/exp_$NAME lib/exp_$NAME
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
  -I../include -I$CS --offload-arch=gfx950 $FLAGS -c $CS/$FILE -o build/exp_$NAME/$FILE.o
OBJS=$(ls build/*.o | grep -v "/$FILE.o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o lib/exp_$NAME/libegraph.so $OBJS build/exp_$NAME/$FILE.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built lib/exp_$NAME/libegraph.so"
