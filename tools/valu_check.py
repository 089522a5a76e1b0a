"""Recompute a bench line's roofline.valu from the committed PMC CSVs
(profiles/<tag>_pmc_sq.csv, _pmc_valu.csv: the rollout kernel's counter rows,
tools/pmc_summary.py) and compare (within 10 %).

    python tools/valu_check.py <tag> <bench.json> [--out profiles/<tag>_valu_check.txt]"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_dispatch(path):
    with open(path) as f:
        rr = list(csv.DictReader(f))
    nd = len({r["Dispatch_Id"] for r in rr}) or 1
    out = {}
    for r in rr:
        out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"]) / nd
    return out


def main():
    tag, bench = sys.argv[1], sys.argv[2]
    out_path = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    import bench as B
    sq = per_dispatch(os.path.join(ROOT, "profiles", f"{tag}_pmc_sq.csv"))
    va = per_dispatch(os.path.join(ROOT, "profiles", f"{tag}_pmc_valu.csv"))
    with open(os.path.join(ROOT, "profiles", "pmc_rollout.json")) as f:
        steps = json.load(f)["executed_candidate_steps"]
    line = json.loads(open(bench).read().strip().splitlines()[-1])
    v = line["roofline"]["valu"]
    valu = sq["SQ_INSTS_VALU"]
    f64 = sum(va.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                       "SQ_INSTS_VALU_TRANS_F64"))
    share = f64 / valu
    cyc = share * B.VALU_CYC_F64 + (1.0 - share) * B.VALU_CYC_OTHER
    peak = B.CHIP_SIMDS * B.CLOCK_HZ / cyc
    per_cs = valu / steps
    frac = per_cs * v["candidate_steps_per_s"] / peak
    txt = [f"PMC CSVs profiles/{tag}_pmc_sq.csv + _pmc_valu.csv, {steps} executed candidate-steps per dispatch",
           f"VALU wave-instructions per candidate-step {per_cs:.1f} (line: {v['valu_per_candidate_step']:.1f})",
           f"f64 share {share:.4f} (line {v['f64_share']:.4f}); mean issue cycles {cyc:.4f}; peak {peak:.4g}/s",
           f"line's candidate-steps/s {v['candidate_steps_per_s']:.4g} -> frac {frac:.4f} (line {v['frac']:.4f}, "
           f"ratio {frac / v['frac']:.4f})",
           f"bench line: {bench} value {line['value']:.1f}"]
    print("\n".join(txt))
    if out_path:
        with open(out_path, "w") as f:
            f.write("\n".join(txt) + "\n")


if __name__ == "__main__":
    main()
