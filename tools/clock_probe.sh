#!/bin/bash
# In-kernel clock under load (MI355X_MICROARCH.md "DVFS give-back"): stage
# profiles (memtime / memrealtime spans) of the headline at 104 and ~1000
# rollouts and of the Shadow pile at 10 and 404 rollouts, and GRBM_GUI_ACTIVE
# over the product kernels of a one-pipeline bench.  Usage: bash tools/clock_probe.sh tag
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-clock}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 tools/stage_profile.py 160 > $O/c2_104.txt 2>&1 || { tail $O/c2_104.txt; exit 1; }
timeout -k 10 300 python3 tools/stage_profile.py 1600 > $O/c2_1000.txt 2>&1 || { tail $O/c2_1000.txt; exit 1; }
timeout -k 10 300 python3 tools/stage_profile_clutter.py 300 64 32 > $O/c5_10.txt 2>&1 || { tail $O/c5_10.txt; exit 1; }
timeout -k 10 300 python3 tools/stage_profile_clutter.py 300 2048 404 > $O/c5_404.txt 2>&1 || { tail $O/c5_404.txt; exit 1; }
for f in c2_104 c2_1000 c5_10 c5_404; do echo "$f $(head -1 $O/$f.txt) | $(grep 'ticks per' $O/$f.txt) | $(grep 'clock held' $O/$f.txt)"; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pmc_grbm -o pmc -f csv -- python3 bench.py --streams 1 --steps 2 --warmup 1 --cpu-budget 0 --e2e-steps 0 --no-escalate > $O/pmc_grbm.json 2> $O/pmc_grbm.err || { tail $O/pmc_grbm.err; exit 1; }
python3 - <<PY
import csv, collections
rows = list(csv.DictReader(open("$O/pmc_grbm/pmc_counter_collection.csv")))
by = collections.defaultdict(dict)
for r in rows:
    by[(r["Dispatch_Id"], r["Kernel_Name"][:40])][r["Counter_Name"]] = float(r["Counter_Value"])
tr = {r["Dispatch_Id"]: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in csv.DictReader(open("$O/pmc_grbm/pmc_kernel_trace.csv"))}
for (d, k), v in by.items():
    if "mgs" in k and d in tr and tr[d] > 1e6:
        print(k, "dur_ms %.1f" % (tr[d] / 1e6), "clock_GHz %.2f" % (v.get("GRBM_GUI_ACTIVE", 0) / 8 / tr[d]))
PY
