#!/usr/bin/env python3
"""Summarise profiles/calib_fetch.sh: counter bytes / known bytes per access pattern (FETCH_SIZE and WRITE_SIZE in
KiB per dispatch, averaged over the repetitions). Writes profiles/<tag>_calib.json.

    python profiles/calib_summarize.py r02c
"""
import csv
import json
import os
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "gpurun_out")


def per_kernel(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            acc[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "calib"
    known = json.load(open(os.path.join(OUT, "calib_known.json")))
    fetch = per_kernel(os.path.join(OUT, "calib_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(OUT, "calib_write", "run_counter_collection.csv"), "WRITE_SIZE")
    res = {}
    for k, b in known.items():
        f, w = fetch.get(k, 0.0) * 1024, write.get(k, 0.0) * 1024
        res[k] = {"known_bytes": b, "fetch_bytes": f, "write_bytes": w, "fetch_over_known": f / b,
                  "write_over_known": w / b}
        print(f"{k:10s} known {b / 1e6:9.2f} MB  FETCH {f / 1e6:9.2f} MB ({f / b:6.3f}x)  WRITE {w / 1e6:9.2f} MB "
              f"({w / b:6.3f}x)")
    with open(os.path.join(HERE, f"{tag}_calib.json"), "w") as f:
        json.dump({"method": "profiles/calib_fetch.hip under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate "
                             "passes), KiB x 1024 per dispatch averaged over 3 repetitions; 2 GiB tables, hashed "
                             "indices", "patterns": res}, f, indent=1)


if __name__ == "__main__":
    main()
