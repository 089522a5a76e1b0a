#!/bin/bash
# Round-1 profiling recipe (run on the GPU box via gpurun): kernel trace + stats,
# then separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) on the same bench command.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r01 -o bench -f csv -- python3 bench.py --steps 3 --warmup 1 --cpu-budget 0 > gpurun_out/prof_r01_bench.json 2> gpurun_out/prof_r01_bench.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o pmc -f csv -- python3 bench.py --steps 1 --warmup 0 --cpu-budget 0 > gpurun_out/pmc_fetch.json 2> gpurun_out/pmc_fetch.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_write -o pmc -f csv -- python3 bench.py --steps 1 --warmup 0 --cpu-budget 0 > gpurun_out/pmc_write.json 2> gpurun_out/pmc_write.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM -d gpurun_out/pmc_sq -o pmc -f csv -- python3 bench.py --steps 1 --warmup 0 --cpu-budget 0 > gpurun_out/pmc_sq.json 2> gpurun_out/pmc_sq.err
