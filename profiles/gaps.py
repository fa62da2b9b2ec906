"""GPU idle time between kernels, from a rocprofv3 --kernel-trace CSV (host-side launch bubbles).

    python3 profiles/gaps.py gpurun_out/prof_<tag> [--last-steps N]

Finds *kernel_trace.csv under the directory, keeps the kernels of the last N steps (a step starts at each
preprocess_kernel launch), and prints the span, the busy time (union of kernel intervals), the idle share and the
largest gaps with the kernels on either side.
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last-steps", type=int, default=10)
    args = ap.parse_args()
    files = glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "preprocess_kernel" in r[2]]
    if len(starts) < args.last_steps + 1:
        raise SystemExit(f"only {len(starts)} steps in the trace")
    lo, hi = starts[-args.last_steps - 1], starts[-1]
    sel = rows[lo:hi]
    span = sel[-1][1] - sel[0][0]
    busy, cur_s, cur_e = 0, sel[0][0], sel[0][1]
    gaps = []
    for i in range(1, len(sel)):
        s, e, _ = sel[i]
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, sel[i - 1][2][:60], sel[i][2][:60]))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    steps = args.last_steps
    print(f"steps {steps}: span {span / steps / 1e3:.1f} us/step, busy {busy / steps / 1e3:.1f} us/step, "
          f"idle {(span - busy) / steps / 1e3:.1f} us/step ({100 * (span - busy) / span:.1f} %)")
    agg = {}
    for g, a, b in gaps:
        k = (a, b)
        agg[k] = agg.get(k, 0) + g
    for (a, b), g in sorted(agg.items(), key=lambda x: -x[1])[:12]:
        print(f"{g / steps / 1e3:8.2f} us/step  {a}  ->  {b}")


if __name__ == "__main__":
    main()
