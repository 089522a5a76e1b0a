#!/bin/bash
# Round-1 profiling recipe (run on the GPU box via gpurun): bench line, kernel
# trace + stats, then separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) on the
# same bench command, then the stage-timer breakdown (MGS_PROFILE build).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
B="bench.py --steps 3 --warmup 1 --cpu-budget 0"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench -f csv -- python3 $B > $OUT/trace.json 2> $OUT/trace.err && \
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc_fetch -o pmc -f csv -- python3 bench.py --steps 1 --warmup 0 --cpu-budget 0 > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err && \
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmc_write -o pmc -f csv -- python3 bench.py --steps 1 --warmup 0 --cpu-budget 0 > $OUT/pmc_write.json 2> $OUT/pmc_write.err && \
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM -d $OUT/pmc_sq -o pmc -f csv -- python3 bench.py --steps 1 --warmup 0 --cpu-budget 0 > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err && \
timeout -k 10 200 python3 tools/stage_profile.py 256 > $OUT/stages.txt 2>&1
