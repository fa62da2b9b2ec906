#!/usr/bin/env python3
"""The reference AS COMPILED vs the oracle (TEST INFRASTRUCTURE ONLY).

nvcc compiles the reference with its default --fmad=true (no -fmad flag in /root/reference/CMakeLists.txt:60-85),
so every mul+add pair of the preprocess, the falloff and the backward may be fused into one FMA; the oracle
(liboracle.so) is built with -ffp-contract=off and evaluates the reference expressions as written. No nvcc exists
here, so two contracted builds of the same oracle sources stand in for the reference binary: GCC and LLVM fuse
different multiplies of a sum of products (oracle/Makefile: liboracle_fma_gcc.so, liboracle_fma_clang.so). The
reference also takes atan2f / asinf from libdevice, the oracle and the HIP kernels from the shared omni_math.h; a
third build with glibc's atan2f / asinf (liboracle_libm.so) measures what a second implementation changes.

For each BASELINE config this measures what changes between the oracle and each contracted build — depth /
centre / conic / radius / rect bits, num_rendered, sorted point-list positions, pixels over 1e-4, gradient entries
outside grad_close — and checks every change against the allowance oracle/ambiguity.hpp derives from the
oracle's own forward (the sets tests/helpers.py excuses: flagged pixels within their colour bound, gradients of
the Gaussians owning a flagged decision, the wide bar for those blending behind one). Writes
profiles/ambiguity.json (bench.py reports its allowance counts as config.ambiguous).

    python oracle/contraction.py [A B C E_pinhole E] [--threads N] [--no-variants]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GRAD_NAMES = ("dmean2D", "dcolor", "dopacity", "dmean3D", "dcov3D", "dsh", "dscale", "drot")


def _bits(a):
    a = np.asarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


def point_list_check(ob, ov, allow_flip, P):
    """The contracted build's sorted point list against the oracle's, per tile: equal after dropping the rect-
    ambiguous Gaussians (G_RECT), except at positions where both Gaussians belong to an order-ambiguous run
    (G_RUN). Returns (positions that differ, positions not explained)."""
    pb, pv = ob.get("point_list"), ov.get("point_list")
    rb, rv = ob.get("ranges").reshape(-1, 2), ov.get("ranges").reshape(-1, 2)
    rect = (allow_flip & 4) != 0
    order = (allow_flip & 16) != 0
    if len(pb) == len(pv) and (rb == rv).all():
        diff = np.nonzero(pb != pv)[0]
        bad = diff[~(order[pb[diff]] & order[pv[diff]])]
        return int(len(diff)), int(len(bad))
    ndiff = nbad = 0
    for t in range(len(rb)):
        a = pb[rb[t, 0]:rb[t, 1]]
        b = pv[rv[t, 0]:rv[t, 1]]
        a, b = a[~rect[a]], b[~rect[b]]
        if len(a) != len(b):
            ndiff += abs(len(a) - len(b))
            nbad += abs(len(a) - len(b))
            continue
        d = np.nonzero(a != b)[0]
        ndiff += len(d)
        nbad += int((~(order[a[d]] & order[b[d]])).sum())
    return ndiff, nbad


def compare_variant(ob, gb, ov, gv, allow, H, W):
    """Counts of what differs between the oracle run (ob, grads gb) and a contracted build's run (ov, gv), and of
    what the allowance does not explain (every `*_unexplained` must be 0)."""
    P = ob.P
    vis = ob.get("radii") > 0
    out = {"num_rendered_delta": int(ov.num_rendered - ob.num_rendered)}
    rect = (allow["flags"] & 4) != 0
    for k in ("depths", "means2D", "conic_opacity"):
        a, b = _bits(ob.get(k)).reshape(P, -1), _bits(ov.get(k)).reshape(P, -1)
        out[f"{k}_changed"] = int((a != b).any(1)[vis].sum())
    d = np.abs(_bits(ob.get("depths")).astype(np.int64) - _bits(ov.get("depths")).astype(np.int64))
    out["depth_max_ulps"] = int(d[vis].max()) if vis.any() else 0
    radius = (allow["flags"] & 32) != 0
    for k, ok in (("radii", radius), ("tiles_touched", rect)):
        ch = ob.get(k) != ov.get(k)
        out[f"{k}_changed"] = int(ch.sum())
        out[f"{k}_unexplained"] = int((ch & ~ok).sum())
    out["point_list_positions_changed"], out["point_list_unexplained"] = point_list_check(ob, ov, allow["flags"], P)
    img_b = ob.get("out_color").reshape(3, H, W).astype(np.float64)
    img_v = ov.get("out_color").reshape(3, H, W).astype(np.float64)
    err = np.abs(img_b - img_v).max(0)
    out["pixels_over_1e-4"] = int((err > 1e-4).sum())
    out["pixels_over_1e-5"] = int((err > 1e-5).sum())
    out["image_max_abs_err"] = float(err.max())
    out["pixels_unexplained"] = int((err > 1e-4 + allow["bound"]).sum())
    over = err > 1e-4
    out["pixels_worst_fraction_of_bound"] = float(((err - 1e-4) / np.maximum(allow["bound"], 1e-30))[over].max()) \
        if over.any() else 0.0
    terr = np.abs(ob.get("final_T").reshape(H, W).astype(np.float64) - ov.get("final_T").reshape(H, W))
    out["final_T_unexplained"] = int((terr > 1e-4 + allow["t_bound"]).sum())
    if gb is not None:
        from helpers import grad_residuals

        r = grad_residuals(gv, gb, allow, P, GRAD_NAMES)
        out.update(grad_entries_outside_bar=r["entries_outside_strict"],
                   grad_gaussians_outside_bar=r["gaussians_outside_strict"],
                   grad_owner_gaussians_used=r["owner_gaussians_used"],
                   grad_exposed_gaussians_used=r["exposed_gaussians_used"],
                   grad_owner_bound_max_use=round(r["owner_bound_max_use"], 4),
                   grad_entries_unexplained=r["unexplained"])
    return out


def unexplained(cmp: dict) -> int:
    return sum(v for k, v in cmp.items() if k.endswith("_unexplained"))


VARIANTS = ("fma_gcc", "fma_clang", "libm")


def modelled_vs_measured(counts: dict, variants: dict) -> dict:
    """The allowance's modelled counts next to what each variant actually changed (every measured change must lie
    inside the modelled set: the *_unexplained counts of compare_variant are 0)."""
    out = {"modelled": {k: counts.get(k) for k in ("rect_gaussians", "radius_gaussians", "order_pairs",
                                                     "flip_gaussians", "exposed_gaussians", "allowed_pixels")}}
    for v, c in variants.items():
        out[v] = {"rects_changed": c.get("tiles_touched_changed"), "radii_changed": c.get("radii_changed"),
                  "centres_changed": c.get("means2D_changed"), "depth_keys_changed": c.get("depths_changed"),
                  "point_list_positions_changed": c.get("point_list_positions_changed"),
                  "num_rendered_delta": c.get("num_rendered_delta"), "pixels_over_1e-4": c.get("pixels_over_1e-4"),
                  "grad_gaussians_outside_bar": c.get("grad_gaussians_outside_bar"),
                  "unexplained": unexplained(c)}
    return out


def run_config(name, threads, variants=VARIANTS, backward=True):
    import _omnigs
    import oracle as O
    from helpers import reference_allowance

    scene = _omnigs.load().scene
    g, cam, dL = scene.config_scene(name)
    t0 = time.time()
    ob, L, gb = O.run_scene(g, cam, dL if backward else None, nthreads=threads)
    allow = reference_allowance(ob, dL if backward else None)
    counts = dict(allow["counts"])
    V = int((ob.get("radii") > 0).sum())
    counts.update(P=g.P, V=V, L=int(L), pixels=cam.width * cam.height,
                  exposed_gaussians=int((allow["exposed"] & ~allow["owners"]).sum()))
    res = {"allowance": counts, "variants": {}}
    for v in variants:
        ov, _, gv = O.run_scene(g, cam, dL if backward else None, nthreads=threads, variant=v)
        res["variants"][v] = compare_variant(ob, gb, ov, gv, allow, cam.height, cam.width)
        del ov, gv
    res["measured_vs_modelled"] = modelled_vs_measured(counts, res["variants"])
    res["seconds"] = round(time.time() - t0, 1)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["A", "B", "C", "E_pinhole", "E"])
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--no-variants", action="store_true", help="allowance counts only (no contracted builds)")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "ambiguity.json"))
    args = ap.parse_args()
    import oracle as O

    O.build()
    O.set_threads(args.threads)
    try:
        with open(args.out) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        doc = {}
    doc.setdefault("configs", {})
    doc["method"] = (
        "oracle/ambiguity.hpp (allowance_scan) on the oracle forward of each config's bench view, and "
        "oracle/contraction.py: the oracle vs two FMA-contracted builds of it (GCC, LLVM; the proxy of nvcc's "
        "--fmad=true reference binary) and a build with glibc's atan2f / asinf instead of omni_math.h's (libm: an "
        "independent implementation of the transcendentals, as libdevice's is for the reference). allowance: rect_gaussians = tile rect moves within the centre / "
        "atan2 / radius rounding windows; order_pairs = same-tile neighbours whose depths differ by less than their "
        "rounding windows; alpha / saturation / zero_power pixels = a blend decision inside its rounding window; "
        "order_pixels = two members of an order-ambiguous run blend; flip_gaussians own such a decision (gradients "
        "within the owner bound of ambiguity.hpp: owner_grad_bound), exposed_gaussians blend behind or in front of "
        "one (wide bar 1e-2 / 1e-3). variants: what actually changes, and what the allowance leaves unexplained "
        "(*_unexplained, all 0 expected); measured_vs_modelled puts the counts side by side")
    for name in args.configs:
        res = run_config(name, args.threads, variants=() if args.no_variants else VARIANTS)
        doc["configs"][name] = res
        print(name, json.dumps(res), flush=True)
        with open(args.out, "w") as f:
            json.dump(doc, f, indent=1)
    if "C" in doc["configs"]:
        doc["configs"]["D"] = dict(doc["configs"]["C"], note="view 0 of the config-C scene (one of D's eight views)")
    with open(args.out, "w") as f:
        json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
