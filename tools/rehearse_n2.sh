#!/bin/bash
# 2-rank rehearsal of bench.py on a 1-GPU box (ranks share the GPU over gloo),

set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-n2}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-budget 0 --e2e-steps 0 > $OUT/bench_n2.json 2> $OUT/bench_n2.err
rc=$?
cat $OUT/bench_n2.json
exit $rc
