"""Summarise a tools/gpu.sh pmc / trace output directory into profiles/:

  profiles/<tag>_rocprof_kernel_stats.csv kernel-trace --stats of the bench command
  profiles/<tag>_pmc_{fetch,write,sq}.csv the rollout kernel's counter rows
  profiles/pmc_rollout.json               HBM bytes per launch (FETCH_SIZE x 2, the
                                          gfx950 half-count correction of
                                          MI355X_MICROARCH.md, + WRITE_SIZE; KiB) and
                                          per executed candidate-step, SQ totals
  profiles/r01_bench.json                 the bench line of the same run

    python tools/pmc_summary.py gpurun_out/r02p [tag]

Counters are averaged over the rollout dispatches of the pass (the round-2
passes run a single-pipeline bench without the escalation pass, so every
dispatch is one full rollout launch of the headline batch).
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
PROF = os.path.join(ROOT, "profiles")


def rows(path, kernels=("mgs_special_rollout", "mgs_rollout_kernel")):
    """the main rollout launches' rows (the escalation objects' *_esc kernels excluded)"""
    with open(path) as f:
        return [r for r in csv.DictReader(f)
                if any(k in r["Kernel_Name"] for k in kernels) and "_esc" not in r["Kernel_Name"]]


def _commit():
    import subprocess
    try:
        return subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                              text=True, timeout=30).stdout.strip() or None
    except (OSError, subprocess.SubprocessError):
        return None


def main_launch_stats(trace_csv, out_path):
    """per-kernel time of the traced command without the escalation objects'
    *_esc launches (one-workgroup re-runs queued behind the persistent grids:
    their trace durations are mostly dispatch wait), as
    percentages of the remaining kernel time; the *_esc rows listed apart"""
    with open(trace_csv) as f:
        rr = list(csv.DictReader(f))
    agg = {}
    for r in rr:
        k = r["Kernel_Name"].split("(")[0]
        dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        a = agg.setdefault(k, [0, 0.0, 0.0])
        a[0] += 1
        a[1] += dt
        a[2] = max(a[2], dt)
    main = {k: v for k, v in agg.items() if "_esc" not in k}
    tot = sum(v[1] for v in main.values()) or 1.0
    with open(out_path, "w") as f:
        f.write("kernel time of the traced command without the escalation re-runs (*_esc), ms\n")
        f.write("%-44s %7s %11s %10s %10s %7s\n" % ("kernel", "calls", "total", "mean", "max", "pct"))
        for k, (n, t, mx) in sorted(main.items(), key=lambda kv: -kv[1][1]):
            f.write("%-44s %7d %11.3f %10.3f %10.3f %6.1f%%\n" % (k[:44], n, t, t / n, mx, 100.0 * t / tot))
        esc = {k: v for k, v in agg.items() if "_esc" in k}
        if esc:
            f.write("\nescalation re-runs (not in the percentages: trace span includes the wait for CUs)\n")
            for k, (n, t, mx) in sorted(esc.items()):
                f.write("%-44s %7d %11.3f %10.3f %10.3f\n" % (k[:44], n, t, t / n, mx))
    print(open(out_path).read())


def main(d, tag="r03"):
    tr = os.path.join(d, "trace", "bench_kernel_stats.csv")
    if os.path.isfile(tr):
        shutil.copy(tr, os.path.join(PROF, f"{tag}_rocprof_kernel_stats.csv"))
    kt = os.path.join(d, "trace", "bench_kernel_trace.csv")
    if os.path.isfile(kt):
        main_launch_stats(kt, os.path.join(PROF, f"{tag}_rocprof_main_launches.txt"))
    out = {"source": "rocprofv3 --kernel-trace --pmc <counters> (separate passes) on `python3 bench.py --streams 1 "
                     "--steps 1 --warmup 0 --cpu-budget 0 --e2e-steps 0 --no-escalate --fused 0` (tools/gpu.sh pmc, "
                     f"{tag}); "
                     "per rollout dispatch",
           "kernel": "mgs_special_rollout (code object specialised to the headline model)",
           "measured": {"tag": tag, "commit": _commit(),
                        "date": __import__("time").strftime("%Y-%m-%d", __import__("time").gmtime())}}
    sums = {}
    for name in ("fetch", "write", "sq", "valu", "lane"):
        p = os.path.join(d, f"pmc_{name}", "pmc_counter_collection.csv")
        if not os.path.isfile(p):
            continue
        rr = rows(p)
        with open(os.path.join(PROF, f"{tag}_pmc_{name}.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rr[0].keys()))
            w.writeheader()
            w.writerows(rr)
        ndisp = len({r["Dispatch_Id"] for r in rr}) or 1
        part = {}
        for r in rr:
            part[r["Counter_Name"]] = part.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"]) / ndisp
        for k, v in part.items():       # a counter repeated in a later pass: the first pass's value
            sums.setdefault(k, v)
    with open(os.path.join(d, "pmc_fetch.json")) as f:
        steps = json.loads(f.read().strip().splitlines()[-1])["detail"]["executed_candidate_steps"]
    hbm = (2.0 * sums["FETCH_SIZE"] + sums["WRITE_SIZE"]) * 1024.0
    out.update(fetch_size_kb_raw=sums["FETCH_SIZE"], write_size_kb_raw=sums["WRITE_SIZE"],
               hbm_bytes_per_launch_corrected=hbm,
               correction="FETCH_SIZE x 2 (gfx950 half-count, MI355X_MICROARCH.md), WRITE_SIZE as reported; both KiB",
               executed_candidate_steps=steps, hbm_bytes_per_candidate_step=hbm / steps,
               sq={k: v for k, v in sums.items() if k.startswith("SQ_")})
    if "SQ_THREAD_CYCLES_VALU" in sums and sums.get("SQ_ACTIVE_INST_VALU"):
        # rocprof-compute's "VALU active threads": lanes doing work per VALU
        # instruction issued (of 64)
        out["valu_active_threads"] = sums["SQ_THREAD_CYCLES_VALU"] / sums["SQ_ACTIVE_INST_VALU"]
        out["valu_lane_utilisation"] = out["valu_active_threads"] / 64.0
    with open(os.path.join(PROF, "pmc_rollout.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:3])
