#!/bin/bash
# Build experiment variants of libhftlob.so: tools/ab.sh NAME "FLAGS" [NAME "FLAGS" ...]
# -> ab/NAME/libhftlob.so (git-ignored; travels to the GPU box with the snapshot)
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  mkdir -p ab/$1
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared \
      -mllvm -structurizecfg-skip-uniform-regions=true $2 \
      -o ab/$1/libhftlob.so jaxmarl-hft_amd/csrc/hftlob.hip || exit 1
  shift 2
done
