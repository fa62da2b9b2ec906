#!/usr/bin/env python3
"""Summarise the rocprofv3 runs of profiles/collect.sh (CPU side, after gpurun merged gpurun_out/).

    python profiles/pmc_summarize.py r01e [sq_tag]

Writes profiles/<tag>_kernel_stats.csv (copy of the --stats summary), profiles/<tag>_pmc.csv (per-kernel FETCH_SIZE /
WRITE_SIZE averages) and profiles/pmc_latest.json, which bench.py reads for roofline.traffic.

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: rocprofv3 reports both in KiB, and on gfx950
FETCH_SIZE counts half the bytes of wide coalesced reads (MI355X_MICROARCH.md § HBM), so it is doubled.

The --stats summary averages every launch of the run: warm-ups, and the bench's per-stage pass, whose events at every
stage boundary end in system-scope releases (L2 write-back) and so slow the kernel that follows. The timed loop's
launches are the bench's live measurement, so profiles/<tag>_kernel_stats_timed.csv restates the same kernel trace
over the timed loop only (timed_window below), and pmc_latest.json's rocprof_avg_ms comes from it.
"""
import csv
import glob
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(ROOT, "gpurun_out")

# kernel-name fragment -> bench.py stage name (kernels launched once per stage)
STAGES = {
    "preprocess_kernel": "preprocess",
    "emit_kernel": "emit",
    "tile_ranges_kernel": "tile_ranges",
    "render_fwd_kernel": "render_forward",
    "render_bwd_kernel": "render_backward",
    "row_sum_kernel": "row_sums",
    "gaussian_bwd_kernel": "gaussian_backward",
}


def _col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


def per_kernel(counter_dir, counter):
    files = glob.glob(os.path.join(counter_dir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise FileNotFoundError(f"no counter_collection.csv under {counter_dir}")
    acc = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if _col(row, "Counter_Name", "Counter-Name") != counter:
                    continue
                name = _col(row, "Kernel_Name", "Kernel-Name", "KernelName")
                disp = _col(row, "Dispatch_Id", "Dispatch-Id", "Correlation_Id")
                v = float(_col(row, "Counter_Value", "Counter-Value"))
                acc.setdefault(name, {}).setdefault(disp, 0.0)
                acc[name][disp] += v  # a counter may be split over rows (per XCD/instance)
    return {k: (sum(d.values()) / len(d), len(d)) for k, d in acc.items()}


def timed_window(trace_csv, bench_json):
    """Per-kernel statistics of the bench's timed loop alone, from a rocprofv3 --kernel-trace CSV of `bench.py`.

    bench.py runs `warmup` steps, then a per-stage pass of min(steps, 10) steps, then the `steps` timed ones; every
    step launches preprocess_kernel exactly once, so the timed loop starts at the (warmup + min(steps, 10))-th
    preprocess dispatch (0-based) and runs to the end of the trace (the bench under rocprof runs with
    --no-train-step; the CPU baseline launches nothing)."""
    with open(bench_json) as f:
        bench = json.loads([ln for ln in f if ln.startswith("{")][-1])
    steps, warmup = int(bench["steps"]), int(bench["warmup"])
    skip = warmup + min(steps, 10)
    rows = []
    with open(trace_csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    pre = [t0 for t0, _, k in rows if "preprocess_kernel" in k]
    if len(pre) != skip + steps:
        raise RuntimeError(f"{trace_csv}: {len(pre)} preprocess dispatches, expected {skip} + {steps}")
    t_start = pre[skip]
    acc = {}
    for t0, t1, k in rows:
        if t0 >= t_start:
            acc.setdefault(k, []).append((t1 - t0) * 1e-6)  # ns -> ms
    out = {}
    for k, d in acc.items():
        d.sort()
        out[k] = {"calls": len(d), "avg_ms": sum(d) / len(d), "min_ms": d[0], "max_ms": d[-1],
                  "median_ms": d[len(d) // 2], "total_ms": sum(d)}
    return out, steps, (rows[-1][1] - t_start) * 1e-6


def write_timed_stats(tag, timed, steps, window_ms):
    path = os.path.join(HERE, f"{tag}_kernel_stats_timed.csv")
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "AverageNs", "MinNs", "MaxNs", "MedianNs", "TotalDurationNs", "Percentage",
                     "TimedSteps", "WindowNs"])
        tot = sum(v["total_ms"] for v in timed.values()) or 1.0
        for k, v in sorted(timed.items(), key=lambda kv: -kv[1]["total_ms"]):
            w.writerow([k, v["calls"], round(v["avg_ms"] * 1e6, 1), round(v["min_ms"] * 1e6, 1),
                        round(v["max_ms"] * 1e6, 1), round(v["median_ms"] * 1e6, 1), round(v["total_ms"] * 1e6, 1),
                        round(100.0 * v["total_ms"] / tot, 3), steps, round(window_ms * 1e6)])
    return path


def main():
    tag = sys.argv[1]
    stats = glob.glob(os.path.join(OUT, f"prof_{tag}", "**", "*kernel_stats.csv"), recursive=True)
    traces = glob.glob(os.path.join(OUT, f"prof_{tag}", "**", "*kernel_trace.csv"), recursive=True)
    rocprof_avg = {}  # stage -> rocprofv3 average duration (ms) of its kernel over the bench's timed loop
    timed_file = None
    if stats:
        shutil.copy(stats[0], os.path.join(HERE, f"{tag}_kernel_stats.csv"))
    if traces:
        timed, steps, window_ms = timed_window(traces[0], os.path.join(OUT, f"bench_prof_{tag}.json"))
        timed_file = os.path.relpath(write_timed_stats(tag, timed, steps, window_ms), ROOT)
        for name, v in timed.items():
            for frag, stage in STAGES.items():
                if frag in name:
                    rocprof_avg[stage] = (v["avg_ms"], v["calls"])
    fetch = per_kernel(os.path.join(OUT, f"pmc_fetch_{tag}"), "FETCH_SIZE")
    write = per_kernel(os.path.join(OUT, f"pmc_write_{tag}"), "WRITE_SIZE")
    with open(os.path.join(OUT, f"bench_pmc_fetch_{tag}.json")) as f:
        bench = json.loads([ln for ln in f if ln.startswith("{")][-1])
    cfg = bench["config"]["workload"].split(":")[0]
    rows, kernels = [], {}
    for name in sorted(set(fetch) | set(write)):
        fk, n = fetch.get(name, (0.0, 0))
        wk, _ = write.get(name, (0.0, 0))
        hbm = (2.0 * fk + wk) * 1024.0
        rows.append([name, n, round(fk, 1), round(wk, 1), int(hbm)])
        for frag, stage in STAGES.items():
            if frag in name:
                # lower bound: FETCH counted 1:1, as profiles/calib_fetch.hip measures for random 64-B record
                # gathers and 4-B gathers (a 64-B request each); the x2 upper bound holds for 16-B/lane streams
                kernels[stage] = {"kernel": name, "fetch_kib_raw": round(fk, 1), "write_kib": round(wk, 1),
                                  "hbm_bytes_per_launch": int(hbm), "hbm_bytes_lower": int((fk + wk) * 1024),
                                  "dispatches": n}
                if stage in rocprof_avg:
                    kernels[stage]["rocprof_avg_ms"] = round(rocprof_avg[stage][0], 5)
                    kernels[stage]["rocprof_calls"] = rocprof_avg[stage][1]
    with open(os.path.join(HERE, f"{tag}_pmc.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "dispatches", "FETCH_SIZE_KiB_avg", "WRITE_SIZE_KiB_avg", "hbm_bytes_per_launch"])
        w.writerows(rows)
    # the SQ passes of the same tree (profiles/sq.sh + sq_summarize.py -> profiles/<sq_tag>_sq.csv): each stage kernel's
    # VALU wave-instructions per launch, for bench.py's roofline.valu_issue_frac (VALU issue time against the chip's
    # 1024 SIMDs x 1.2 G wave-instructions/s)
    sq_tag = sys.argv[2] if len(sys.argv) > 2 else tag
    sq_path = os.path.join(HERE, f"{sq_tag}_sq.csv")
    sq_file = None
    if os.path.exists(sq_path):
        sq_file = os.path.relpath(sq_path, ROOT)
        with open(sq_path) as f:
            for r in csv.DictReader(f):
                for frag, stage in STAGES.items():
                    if frag in r["kernel"] and stage in kernels:
                        waves, vpw = float(r["waves"]), float(r["valu_per_wave"])
                        kernels[stage]["sq"] = {"waves": waves, "valu_per_wave": vpw,
                                                "valu_insts_per_launch": int(round(waves * vpw)),
                                                "valu_issue_share": float(r["valu_issue_share"]),
                                                "wait_inst_share": float(r["wait_inst_share"])}
    latest = {"tag": tag, "config": cfg, "P": bench["config"]["P"], "L": bench["config"]["L"], "sq_file": sq_file,
              "method": "(2*FETCH_SIZE + WRITE_SIZE) KiB * 1024, separate --pmc passes, gfx950 FETCH x2 correction",
              "kernel_stats_file": timed_file,
              "kernel_stats_all_launches_file": f"profiles/{tag}_kernel_stats.csv" if stats else None,
              "rocprof_avg_over": "the bench's timed loop only (pmc_summarize.timed_window)", "kernels": kernels}
    with open(os.path.join(HERE, "pmc_latest.json"), "w") as f:
        json.dump(latest, f, indent=1)
    print(json.dumps(latest, indent=1))


if __name__ == "__main__":
    main()
