set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03h; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 tools/stage_profile_clutter.py 300 64 32 > $O/c5_32.txt 2>&1 || { tail $O/c5_32.txt; exit 1; }
timeout -k 10 300 python3 tools/stage_profile_clutter.py 300 2048 404 > $O/c5_404.txt 2>&1 || { tail $O/c5_404.txt; exit 1; }
head -1 $O/c5_32.txt; grep "ticks per" $O/c5_32.txt; head -1 $O/c5_404.txt; grep "ticks per" $O/c5_404.txt
