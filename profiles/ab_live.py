#!/usr/bin/env python3
"""Per build of an ab3.sh run (gpurun_out/ab3/<build>_<round>.json): median MP/s and the median live launch time of the
roofline kernel (HIP events on its dispatch packet over the timed loop), per round."""
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]
runs = {}
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    name = os.path.basename(f).rsplit("_", 1)[0]
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except (ValueError, IndexError):
        continue
    runs.setdefault(name, []).append(j)
for name, js in runs.items():
    mp = [x["value"] for x in js]
    kms = [x["roofline"]["avg_launch_ms"] for x in js]
    print(f"{name:12s} kernel {js[0]['roofline']['kernel']:16s} MP/s {statistics.median(mp):8.1f} {mp}  "
          f"live ms {statistics.median(kms):.4f} {kms}  render_fwd stage {statistics.median(x['stages_ms']['render_forward'] for x in js):.4f}")
