#!/bin/bash
# Build libmgs_gpu.so (product) and the diagnostic stage-timer variant.
set -e
cd "$(dirname "$0")/../mj-grasp-sim_amd"
FLAGS="--offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared -std=c++17 -Wno-unused-value -Wno-unused-result"
hipcc $FLAGS csrc/mgs_capi.hip -o mgs/_lib/libmgs_gpu.so
if [ "$1" == "prof" ]; then hipcc $FLAGS -DMGS_PROFILE csrc/mgs_capi.hip -o mgs/_lib/libmgs_gpu_prof.so; fi
