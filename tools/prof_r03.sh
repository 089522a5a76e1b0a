#!/bin/bash
# Round-3 profiling recipe (GPU box, via gpurun): kernel trace + stats of the
# default bench command, then separate PMC passes on a single-pipeline bench
# (one rollout launch per step, no escalation pass, so per-dispatch counters are
# per rollout launch), then the stage-timer breakdowns (MGS_PROFILE builds).
# Usage: bash tools/prof_r03.sh [tag] [nostages]
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
P="bench.py --streams 1 --steps 1 --warmup 0 --cpu-budget 0 --e2e-steps 0 --no-escalate --fused 0"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench -f csv -- python3 bench.py --cpu-budget 0 --e2e-steps 0 > $OUT/trace.json 2> $OUT/trace.err && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc_fetch -o pmc -f csv -- python3 $P > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmc_write -o pmc -f csv -- python3 $P > $OUT/pmc_write.json 2> $OUT/pmc_write.err && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM -d $OUT/pmc_sq -o pmc -f csv -- python3 $P > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_INSTS_SALU -d $OUT/pmc_valu -o pmc -f csv -- python3 $P > $OUT/pmc_valu.json 2> $OUT/pmc_valu.err || exit 1
# stage timers need the MGS_PROFILE libraries (build(profile_variant=True)); "nostages" skips them
[ "$2" = "nostages" ] && exit 0
timeout -k 10 200 python3 tools/stage_profile.py 160 > $OUT/stages.txt 2>&1 && \
timeout -k 10 300 python3 tools/stage_profile_clutter.py 300 > $OUT/stages_clutter.txt 2>&1
