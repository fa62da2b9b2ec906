#!/usr/bin/env python3
"""Summarise a GPU parity run's residual records (tests/helpers.record_residuals, $OMR_PARITY_RESIDUALS JSON lines)
next to what the FMA-contracted proxies of the reference need (profiles/ambiguity.json), into one JSON file.

    python profiles/parity_residuals.py gpurun_out/r04a_residuals.jsonl profiles/r04_parity_residuals.json
"""
import json
import os
import sys

KEYS = ("pixels_over_1e4", "final_T_over_1e4", "n_contrib_mismatches", "image_max_abs_err", "grad_entries_outside_strict",
        "gaussians_outside_strict", "owner_gaussians_used", "exposed_gaussians_used", "owner_bound_max_use")
PROXY_KEYS = ("pixels_over_1e-4", "grad_entries_outside_bar", "grad_gaussians_outside_bar", "grad_owner_gaussians_used")
CONFIG_OF = {"test_baseline_config_full[B]": "B", "test_baseline_config_full[C]": "C",
             "test_baseline_config_full[E_pinhole]": "E_pinhole", "test_baseline_config_full[E]": "E"}


def main(src, dst):
    here = os.path.dirname(os.path.abspath(__file__))
    try:
        amb = json.load(open(os.path.join(here, "ambiguity.json"))).get("configs", {})
    except (OSError, ValueError):
        amb = {}
    cases, seen = {}, {}
    for line in open(src):
        r = json.loads(line)
        name = r["case"].split("::")[-1]
        seen[name] = seen.get(name, 0) + 1
        if seen[name] > 1:
            name = f"{name}#{seen[name]}"
        e = {k: r[k] for k in KEYS if k in r}
        e.update(P=r.get("P"), pixels=r.get("pixels"), budget=r.get("budget"))
        if "per_tensor" in r:
            e["per_tensor"] = r["per_tensor"]
        cfg = CONFIG_OF.get(name)
        if cfg and cfg in amb:
            e["fma_proxies"] = {v: {k: x.get(k) for k in PROXY_KEYS} for v, x in amb[cfg].get("variants", {}).items()}
        cases[name] = e
    doc = {"source": src, "what": "HIP path vs the CPU oracle per GPU parity case: pixels / final_T over 1e-4, n_contrib "
           "mismatches, gradient entries and Gaussians outside the strict grad_close bar and how many owners (owner bound) "
           "and exposed Gaussians (wide bar) it took to explain them; `budget` is the asserted cap (tests/test_gpu_parity.py "
           "CONFIG_BUDGETS, helpers.default_budget); `fma_proxies` what the FMA-contracted oracle builds need at that config",
           "cases": cases}
    with open(dst, "w") as f:
        json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
