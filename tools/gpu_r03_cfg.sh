#!/bin/bash
# round-3 secondary configurations (tools/bench_configs.py): C3, C4, and C5 at
# the reference's 3000 + 3000 clutter schedule with its CPU baseline sample.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r03cfg}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python3 -u tools/bench_configs.py c5 c3 c4 --c5-steps 3000 --c5-per-object 2048 --c5-cpu-sample 1024 > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
cat $O/configs.jsonl | cut -c1-600
