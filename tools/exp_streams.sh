#!/bin/bash
# bench.py at 1..4 pipelines (batches in flight) on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-streams}
mkdir -p $OUT
for s in 1 2 3 4; do
  timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --cpu-budget 0 --e2e-steps 0 --streams $s > $OUT/s$s.json 2> $OUT/s$s.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/s$s.json')); print($s, d['value'], d['ms_per_step'], d['detail']['rollout_kernel_ms'], d['detail']['pipelines_identical'], d['detail']['escalation_pass_ms'])"
done
