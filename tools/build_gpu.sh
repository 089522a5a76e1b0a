#!/bin/bash
# Build libmgs_gpu.so (product), the CPU oracle, and optionally the
# diagnostic stage-timer variant (libmgs_gpu_prof.so): `tools/build_gpu.sh prof`.
set -e
cd "$(dirname "$0")/.."
if [ "$1" == "prof" ]; then
  python -c "import __graft_entry__ as g; g.build(profile_variant=True)"
else
  python -c "import __graft_entry__ as g; g.build()"
fi
