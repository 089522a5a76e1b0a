#!/bin/bash
# GPU suite, then an A/B of the headline bench over specialised objects and
# the stage-timer profile.  Usage: bash tools/ab1.sh tag objA objB ...
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; shift
mkdir -p gpurun_out/$T
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
bash tools/ab_special.sh "$@" || exit 1
timeout -k 10 300 python3 tools/stage_profile.py 160 > gpurun_out/$T/stages.txt 2>&1 || { tail gpurun_out/$T/stages.txt; exit 1; }
tail -4 gpurun_out/$T/stages.txt
