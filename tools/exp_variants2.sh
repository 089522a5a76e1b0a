#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-exp2}
mkdir -p $OUT
for s in 2 3; do
  MGS_LIB_MAIN=libmgs_gpu_gglobal.so timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --cpu-budget 0 --e2e-steps 0 --streams $s > $OUT/gg_s$s.json 2> $OUT/gg_s$s.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/gg_s$s.json')); print('gglobal', $s, d['value'], d['detail']['rollout_kernel_ms'], d['detail']['pipelines_identical'])"
  timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --cpu-budget 0 --e2e-steps 0 --streams $s --ncon-max 16 > $OUT/n16_s$s.json 2> $OUT/n16_s$s.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/n16_s$s.json')); print('ncon16', $s, d['value'], d['detail']['rollout_kernel_ms'], d['detail']['overflow_candidates'])"
done
