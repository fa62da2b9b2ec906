#!/usr/bin/env python3
"""Per-kernel averages of the SQ counter passes of profiles/sq.sh:  python profiles/sq_summarize.py TAG
Writes profiles/<TAG>_sq.csv. Derived: VALU issue share = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (both quad-cycles
per wave, MI355X_MICROARCH.md), waits as fractions of wave cycles, instructions per wave."""
import csv
import glob
import os
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "gpurun_out")


def load(tag, p):
    acc = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for f in glob.glob(os.path.join(OUT, f"sq{p}_{tag}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:90]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k][r["Counter_Name"]] += 1
    return {k: {c: acc[k][c] / cnt[k][c] for c in acc[k]} for k in acc}


def main():
    tag = sys.argv[1]
    a, b = load(tag, 1), load(tag, 2)
    rows = []
    for k in sorted(set(a) | set(b)):
        d = dict(a.get(k, {}))
        d.update(b.get(k, {}))
        wc = d.get("SQ_WAVE_CYCLES", 0) or 1
        waves = d.get("SQ_WAVES", 0) or 1
        rows.append({"kernel": k, "waves": waves,
                     "valu_issue_share": d.get("SQ_ACTIVE_INST_VALU", 0) / wc,
                     "any_issue_share": d.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                     "wait_any_share": d.get("SQ_WAIT_ANY", 0) / wc,
                     "wait_inst_share": d.get("SQ_WAIT_INST_ANY", 0) / wc,
                     "valu_per_wave": d.get("SQ_INSTS_VALU", 0) / waves,
                     "salu_per_wave": d.get("SQ_INSTS_SALU", 0) / waves,
                     "lds_per_wave": d.get("SQ_INSTS_LDS", 0) / waves,
                     "vmem_per_wave": d.get("SQ_INSTS_VMEM", 0) / waves,
                     "branch_per_wave": d.get("SQ_INSTS_BRANCH", 0) / waves,
                     "grbm_gui_active": d.get("GRBM_GUI_ACTIVE", 0),
                     "busy_cycles": d.get("SQ_BUSY_CYCLES", 0)})
    path = os.path.join(HERE, f"{tag}_sq.csv")
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        for r in rows:
            w.writerow({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()})
    for r in rows:
        if r["waves"] > 100:
            print(f"{r['kernel'][:60]:60s} waves {r['waves']:9.0f} valu/wave {r['valu_per_wave']:9.0f} salu/wave "
                  f"{r['salu_per_wave']:8.0f} VALU-issue {r['valu_issue_share']:.2f} wait_any {r['wait_any_share']:.2f} "
                  f"wait_inst {r['wait_inst_share']:.2f}")


if __name__ == "__main__":
    main()
