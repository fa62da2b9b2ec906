#!/usr/bin/env python3
"""Per-kernel time per training iteration from a rocprofv3 kernel trace of profiles/train_prof.py:
    python3 profiles/train_summarize.py TRACE_CSV STEPS [OUT_CSV]
The timed iterations are the last STEPS launches of the Adam kernel's step (one per iteration): the window starts at
the first kernel after the (warmup)-th Adam launch. Prints kernels by total time per iteration, the GPU busy time and
the idle time per iteration."""
import csv
import sys


def main():
    trace, steps = sys.argv[1], int(sys.argv[2])
    out = sys.argv[3] if len(sys.argv) > 3 else None
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(trace)))
    adam = [i for i, x in enumerate(rows) if "adam_kernel" in x[2]]
    first = adam[-steps - 1] + 1  # the kernel after the last warm-up iteration's Adam
    last = adam[-1]
    win = rows[first:last + 1]
    t0, t1 = win[0][0], win[-1][1]
    acc = {}
    for a, b, k in win:
        acc.setdefault(k, []).append((b - a) * 1e-3)
    busy = sum(sum(v) for v in acc.values())
    lines = sorted(acc.items(), key=lambda kv: -sum(kv[1]))
    print(f"window {((t1 - t0) * 1e-3) / steps:.1f} us per iteration, GPU busy {busy / steps:.1f} us, "
          f"idle {((t1 - t0) * 1e-3 - busy) / steps:.1f} us, {len(win) / steps:.1f} launches per iteration")
    res = []
    for k, v in lines:
        name = k.replace("void ", "").replace("omr::(anonymous namespace)::", "")[:110]
        res.append((name, len(v) / steps, sum(v) / steps))
        print(f"{sum(v) / steps:9.1f} us/it  {len(v) / steps:4.1f} x  {name}")
    if out:
        with open(out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "launches_per_iteration", "us_per_iteration"])
            for r in res:
                w.writerow([r[0], round(r[1], 2), round(r[2], 2)])


if __name__ == "__main__":
    main()
