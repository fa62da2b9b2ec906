#!/usr/bin/env python3
"""Training step after the backward at config C's model size (P = 1 M Gaussians, SH degree
3), HIP (csrc/optim.hip) vs the reference's formulation run by torch on the same GPU:

  adam       fused activation backward + Adam over the six groups, one launch (omr_adam_step, raster grads)
             vs autograd through cat / sigmoid / exp / normalize + torch Adam per tensor (foreach=False: the
             LibTorch 2.0.1 C++ loop the reference runs, adam.cpp), and torch's own foreach / fused Adam for scale;
  stats      addDensificationStats + max_radii2D (omr_densification_stats) vs the index_put_ formulation
             (gaussian_model.cpp:839-853, gaussian_mapper.cpp:429-434);
  densify    densifyAndPrune (omr_densify_plan + apply) vs clone / split / prune with torch cat + index
             (gaussian_model.cpp:619-837).

Algorithmic bytes: Adam 28 B per float (read p, m, v, g; write p, m, v) x 59 floats = 1652 B per Gaussian.
GPU box: python profiles/bench_optim.py [P]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, steps=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def event_ms(fn, steps=20, warmup=5):
    """Average GPU time of fn's launches (HIP events on the current stream)."""
    for _ in range(warmup):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(steps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / steps


def make_model(P, Mr, RD, requires_grad=False):
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *shape, s=1.0, m=0.0: (torch.randn(shape, device="cuda", generator=g) * s + m)  # noqa: E731
    t = [r(P, 3), r(P, 1, 3, s=0.5), r(P, Mr, 3, s=0.2), r(P, 1, s=2.0), r(P, 3, s=1.5, m=-4.0), r(P, 4)]
    t = [x.contiguous().requires_grad_(requires_grad) for x in t]
    return RD.GaussianModelParams(*t, 3, 3)


def raster_grads(P, Mr):
    g = torch.Generator(device="cuda").manual_seed(1)
    r = lambda *shape: torch.randn(shape, device="cuda", generator=g) * 1e-4  # noqa: E731
    return {"dL_dmeans3D": r(P, 3), "dL_dsh": r(P, Mr + 1, 3), "dL_dopacity": r(P, 1), "dL_dscales": r(P, 3),
            "dL_drotations": r(P, 4)}


def torch_densify(m, accum, denom, extent, max_grad=2e-4, min_opacity=0.005, percent_dense=0.01):
    """The reference's densifyAndPrune sequence in torch ops (cat / index / repeat), optimizer state included."""
    ps = [m.xyz, m.features_dc, m.features_rest, m.opacity, m.scaling, m.rotation]
    ea = [torch.zeros_like(p) for p in ps]
    es = [torch.zeros_like(p) for p in ps]
    grads = accum / denom
    grads[grads.isnan()] = 0.0

    def cat(new):
        for k in range(6):
            ea[k] = torch.cat([ea[k], torch.zeros_like(new[k])])
            es[k] = torch.cat([es[k], torch.zeros_like(new[k])])
            ps[k] = torch.cat([ps[k], new[k]])

    def prune(mask):
        keep = ~mask
        for k in range(6):
            ps[k], ea[k], es[k] = ps[k][keep], ea[k][keep], es[k][keep]

    sel = (torch.linalg.vector_norm(grads, dim=-1) >= max_grad) & \
        (torch.exp(ps[4]).max(1).values <= percent_dense * extent)
    cat([p[sel] for p in ps])
    padded = torch.zeros(ps[0].shape[0], device="cuda")
    padded[:grads.shape[0]] = grads.squeeze()
    sel = (padded >= max_grad) & (torch.exp(ps[4]).max(1).values > percent_dense * extent)
    stds = torch.exp(ps[4][sel]).repeat(2, 1)
    samples = torch.normal(torch.zeros_like(stds), stds)
    q = torch.nn.functional.normalize(ps[5][sel])
    w, x, y, z = q.unbind(-1)
    Rm = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                      2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                      2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1).view(-1, 3, 3).repeat(2, 1, 1)
    new = [torch.bmm(Rm, samples.unsqueeze(-1)).squeeze(-1) + ps[0][sel].repeat(2, 1),
           ps[1][sel].repeat(2, 1, 1), ps[2][sel].repeat(2, 1, 1), ps[3][sel].repeat(2, 1),
           torch.log(torch.exp(ps[4][sel]).repeat(2, 1) / 1.6), ps[5][sel].repeat(2, 1)]
    cat(new)
    prune(torch.cat([sel, torch.zeros(2 * int(sel.sum().item()), dtype=torch.bool, device="cuda")]))
    mask = (torch.sigmoid(ps[3]) < min_opacity).squeeze() | (torch.exp(ps[4]).max(1).values > 0.1 * extent)
    prune(mask)
    return ps[0].shape[0]


def main():
    import _omnigs

    omr = _omnigs.load()
    OPT, RD = omr.optim, omr.renderer
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    Mr = 15
    out = {"P": P, "sh_degree": 3}

    # ---- Adam -------------------------------------------------------------------------------------------------
    model = make_model(P, Mr, RD)
    opt = OPT.GaussianOptimizer(model, OPT.OptimizationParams())
    g = raster_grads(P, Mr)
    t_fused = event_ms(lambda: opt.step(raster_grads=g))
    nbytes = 28 * 59 * P
    out["adam_fused_ms"] = round(t_fused, 4)
    out["adam_fused_alg_GBps"] = round(nbytes / (t_fused * 1e-3) / 1e9, 1)
    out["adam_alg_bytes"] = nbytes
    act = {}
    try:  # + the activated tensors' writes
        out["adam_fused_activate_ms"] = round(event_ms(lambda: opt.step(raster_grads=g, act_out=act)), 4)
    except Exception as e:  # noqa: BLE001  (OMR_ADAM_SH_ROWS=0 has no activated SH output)
        out["adam_fused_activate_ms"] = f"unavailable: {e}"
    out["activate_ms"] = round(event_ms(lambda: opt.activate(act)), 4)
    out["adam_sh_rows"] = os.environ.get("OMR_ADAM_SH_ROWS", "1")
    if os.environ.get("BENCH_OPTIM_HIP_ONLY"):
        print(json.dumps(out))
        return

    ref = make_model(P, Mr, RD, requires_grad=True)
    ps = ref.parameters()
    lrs = [1.6e-4, 0.0025, 0.0025 / 20, 0.05, 0.005, 0.001]
    for name, kw in (("torch_loop", dict(foreach=False)), ("torch_foreach", dict(foreach=True)),
                     ("torch_fused", dict(fused=True))):
        try:
            topt = torch.optim.Adam([{"params": [p], "lr": lr} for p, lr in zip(ps, lrs)], eps=1e-15, **kw)
        except Exception as e:  # noqa: BLE001
            out[f"adam_{name}_ms"] = f"unavailable: {e}"
            continue

        def ref_step():
            acts = [ref.xyz * 1.0, torch.cat([ref.features_dc, ref.features_rest], 1), torch.sigmoid(ref.opacity),
                    torch.exp(ref.scaling), torch.nn.functional.normalize(ref.rotation)]
            torch.autograd.backward(acts, [g["dL_dmeans3D"], g["dL_dsh"], g["dL_dopacity"], g["dL_dscales"],
                                           g["dL_drotations"]])
            topt.step()
            topt.zero_grad(set_to_none=True)

        out[f"adam_{name}_ms"] = round(timeit(ref_step), 4)
    out["adam_speedup_vs_reference_loop"] = round(out["adam_torch_loop_ms"] / t_fused, 2)

    # ---- densification stats ----------------------------------------------------------------------------------
    gen = torch.Generator(device="cuda").manual_seed(2)
    radii = torch.randint(-2, 30, (P,), device="cuda", dtype=torch.int32, generator=gen)
    vgrad = torch.randn((P, 3), device="cuda", generator=gen) * 1e-3
    out["stats_hip_ms"] = round(event_ms(lambda: opt.add_densification_stats(vgrad, radii)), 4)
    accum, denom, mr = torch.zeros(P, 1, device="cuda"), torch.zeros(P, 1, device="cuda"), torch.zeros(P, device="cuda")

    def ref_stats():
        vis = radii > 0
        mr.index_put_((vis,), torch.max(mr[vis], radii[vis].float()))
        accum.index_put_((vis,), torch.linalg.vector_norm(vgrad[vis, :2], dim=-1, keepdim=True), accumulate=True)
        denom.index_put_((vis,), denom[vis] + 1)

    out["stats_torch_ms"] = round(timeit(ref_stats), 4)

    # ---- densifyAndPrune ----------------------------------------------------------------------------------------
    acc = (torch.rand((P, 1), device="cuda", generator=gen) * 4e-4)
    den = torch.ones((P, 1), device="cuda")

    def hip_densify():
        m = make_model(P, Mr, RD)
        o = OPT.GaussianOptimizer(m, OPT.OptimizationParams())
        o.xyz_gradient_accum.copy_(acc)
        o.denom.copy_(den)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        info = o.densify_and_prune(2e-4, 0.005, 5.0, 20, True)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3, info

    def ref_densify():
        m = make_model(P, Mr, RD)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = torch_densify(m, acc, den, 5.0)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3, n

    hip_densify(), ref_densify()  # warm up allocator / kernels
    th = sorted(hip_densify()[0] for _ in range(5))[2]
    tr = sorted(ref_densify()[0] for _ in range(5))[2]
    _, info = hip_densify()
    out["densify_hip_ms"] = round(th, 3)
    out["densify_torch_ms"] = round(tr, 3)
    out["densify_counts"] = info
    print(json.dumps(out))


if __name__ == "__main__":
    main()
