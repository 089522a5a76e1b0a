#!/bin/bash
# round-3 launcher check: bench.py --gpus 2 started directly (ranks share the
# one GPU over gloo), then the N=1 bench line with the all-CPU baseline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_launch
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
(cat /sys/fs/cgroup/cpu.max; nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))") > $O/host.txt 2>&1
timeout -k 10 300 python3 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-budget 0 --e2e-steps 0 > $O/bench_n2.json 2> $O/bench_n2.err || exit 1
timeout -k 10 400 python3 bench.py --steps 20 > $O/bench_n1.json 2> $O/bench_n1.err
