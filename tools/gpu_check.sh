#!/bin/bash
# One GPU call: parity tests, smoke, bench (N=1), kernel-trace stats of the bench.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-check}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o bench -f csv -- python3 bench.py --steps 3 --warmup 1 --cpu-budget 0 > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof_bench.err
rc=$?
tail -3 gpurun_out/${TAG}_pytest.log; cat gpurun_out/${TAG}_bench.json 2>/dev/null
exit $rc
