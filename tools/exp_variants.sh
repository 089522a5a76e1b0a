#!/bin/bash
# Build-variant / capacity experiments on the headline bench (one GPU call).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-exp}
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --cpu-budget 0 --e2e-steps 0"
timeout -k 10 200 $B > $OUT/base.json 2> $OUT/base.err && \
MGS_LIB_MAIN=libmgs_gpu_gglobal.so timeout -k 10 200 $B > $OUT/gglobal.json 2> $OUT/gglobal.err && \
MGS_LIB_MAIN=libmgs_gpu_gglobal.so timeout -k 10 200 $B --ncon-max 16 > $OUT/gglobal16.json 2> $OUT/gglobal16.err && \
timeout -k 10 200 $B --ncon-max 16 > $OUT/base16.json 2> $OUT/base16.err
rc=$?
for f in $OUT/*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['detail']['rollout_kernel_ms'], d['detail']['overflow_candidates'], d['detail']['escalation_kernel_ms'])"; done
exit $rc
