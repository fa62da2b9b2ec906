#!/usr/bin/env python3
"""One step's kernel timeline from a rocprofv3 kernel trace (the last full step: preprocess to preprocess), plus the
bench line's ms/step and stage times:  python profiles/steps.py gpurun_out/prof_TAG [gpurun_out/bench_prof_TAG.json]"""
import csv
import re
import glob
import json
import sys


def timeline(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "preprocess_kernel" in r["Kernel_Name"]]
    i0, i1 = idx[-2], idx[-1]
    t0 = int(rows[i0]["Start_Timestamp"])
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        m = re.findall(r"(\w+)(?:<[^<>]*>)?\(", r["Kernel_Name"])
        name = (m[-1] if m else r["Kernel_Name"])[:44]
        print(f'{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {name:44s} grid={r["Grid_Size_X"]} lds={r["LDS_Block_Size"]} '
              f'vgpr={r["VGPR_Count"]}')


def bench(f):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print(d["value"], d["ms_per_step"], d["stages_ms"])


if __name__ == "__main__":
    timeline(sys.argv[1])
    if len(sys.argv) > 2:
        bench(sys.argv[2])
