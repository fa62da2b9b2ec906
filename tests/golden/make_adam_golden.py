"""Generate tests/golden/optim/adam_*.npz with LibTorch's own C++ Adam and autograd (the reference's dependency).

The reference steps its six GaussianModel groups with torch::optim::Adam (eps 1e-15, per-group lr;
gaussian_model.cpp:485-518) after autograd has taken the loss gradient through the renderer's activations
(gaussian_model.cpp:54-77: xyz, cat(f_dc, f_rest), sigmoid(opacity), exp(scaling), normalize(rotation)).
This script compiles a small C++ program against the LibTorch in this image (2.10; the reference pins 2.0.1,
README.md:29 — adam.cpp's update is the same in both) that does exactly that for a few steps on seeded inputs
and records, per step, the raw gradients autograd produced, and at the end the parameters and Adam moments.
The fixtures pin oracle/optim_oracle.py and the HIP kernel (csrc/optim.hip) to LibTorch itself.

Run: python tests/golden/make_adam_golden.py  (≈20 s to compile; CPU only)
"""
import os
import tempfile

import numpy as np
import torch
from torch.utils.cpp_extension import load_inline

HERE = os.path.dirname(os.path.abspath(__file__))

SRC = r"""
#include <torch/torch.h>

// params: xyz, f_dc, f_rest, opacity, scaling, rotation; act_grads: per step 5 tensors (d xyz, d shs, d sigmoid(o),
// d exp(s), d normalize(q)); lrs: per step 6 floats. Returns 6 params, 6 exp_avg, 6 exp_avg_sq, steps x 6 raw grads.
std::vector<torch::Tensor> run(std::vector<torch::Tensor> init, std::vector<torch::Tensor> act_grads,
                               std::vector<double> lrs, int64_t steps)
{
    pybind11::gil_scoped_release no_gil;  // the autograd engine must not run under the GIL
    std::vector<torch::Tensor> P;
    for (auto& t : init) P.push_back(t.clone().requires_grad_(true));
    torch::optim::AdamOptions o;
    o.set_lr(0.0);
    o.eps() = 1e-15;
    torch::optim::Adam opt(std::vector<torch::Tensor>{P[0]}, o);
    for (int k = 1; k < 6; ++k) opt.add_param_group(torch::optim::OptimizerParamGroup(std::vector<torch::Tensor>{P[k]}));
    std::vector<torch::Tensor> raw;
    for (int64_t s = 0; s < steps; ++s) {
        for (int k = 0; k < 6; ++k) opt.param_groups()[k].options().set_lr(lrs[s * 6 + k]);
        auto shs = torch::cat({P[1], P[2]}, 1);
        auto op = torch::sigmoid(P[3]);
        auto sc = torch::exp(P[4]);
        auto rot = torch::nn::functional::normalize(P[5]);
        torch::autograd::backward({P[0] * 1.0, shs, op, sc, rot},
                                  {act_grads[s * 5 + 0], act_grads[s * 5 + 1], act_grads[s * 5 + 2],
                                   act_grads[s * 5 + 3], act_grads[s * 5 + 4]});
        for (int k = 0; k < 6; ++k) raw.push_back(P[k].grad().clone());
        opt.step();
        opt.zero_grad(true);
    }
    std::vector<torch::Tensor> out;
    for (int k = 0; k < 6; ++k) out.push_back(P[k].detach().clone());
    for (int k = 0; k < 6; ++k) {
        auto& st = static_cast<torch::optim::AdamParamState&>(
            *opt.state()[P[k].unsafeGetTensorImpl()]);
        out.push_back(st.exp_avg().clone());
    }
    for (int k = 0; k < 6; ++k) {
        auto& st = static_cast<torch::optim::AdamParamState&>(
            *opt.state()[P[k].unsafeGetTensorImpl()]);
        out.push_back(st.exp_avg_sq().clone());
    }
    for (auto& t : raw) out.push_back(t);
    return out;
}
"""


def make_case(P, Mr, steps, seed):
    rng = np.random.default_rng(seed)
    f = np.float32
    params = [rng.normal(0, 1, (P, 3)).astype(f), rng.normal(0, 0.5, (P, 1, 3)).astype(f),
              rng.normal(0, 0.2, (P, Mr, 3)).astype(f), rng.normal(0, 2, (P, 1)).astype(f),
              rng.normal(-3, 1, (P, 3)).astype(f), rng.normal(0, 1, (P, 4)).astype(f)]
    act = []
    for s in range(steps):
        g = [rng.normal(0, 1e-3, (P, 3)), rng.normal(0, 1e-3, (P, 1 + Mr, 3)), rng.normal(0, 1e-2, (P, 1)),
             rng.normal(0, 1e-2, (P, 3)), rng.normal(0, 1e-3, (P, 4))]
        g = [x.astype(f) for x in g]
        g[0][rng.random(P) < 0.3] = 0  # invisible Gaussians: zero gradient, Adam still moves them
        act.append(g)
    lrs = []
    for s in range(steps):
        lrs += [1.6e-4 * (0.9 ** s), 0.0025, 0.0025 / 20.0, 0.05, 0.005, 0.001]
    return params, act, lrs


def main():
    build = tempfile.mkdtemp(prefix="adam_golden_")
    mod = load_inline("omr_adam_golden", cpp_sources=[SRC], functions=["run"], build_directory=build)
    for name, P, Mr, steps, seed in (("adam_deg3_P61", 61, 15, 3, 11), ("adam_deg1_P67", 67, 3, 4, 12)):
        params, act, lrs = make_case(P, Mr, steps, seed)
        out = mod.run([torch.from_numpy(p) for p in params],
                      [torch.from_numpy(x) for g in act for x in g], lrs, steps)
        out = [t.numpy() for t in out]
        d = {"P": P, "Mr": Mr, "steps": steps, "lrs": np.array(lrs, np.float64).reshape(steps, 6)}
        for k in range(6):
            d[f"param{k}"] = params[k]
            d[f"out_param{k}"] = out[k]
            d[f"out_exp_avg{k}"] = out[6 + k]
            d[f"out_exp_avg_sq{k}"] = out[12 + k]
        for s in range(steps):
            for j in range(5):
                d[f"act_grad{s}_{j}"] = act[s][j]
            for k in range(6):
                d[f"raw_grad{s}_{k}"] = out[18 + 6 * s + k]
        os.makedirs(os.path.join(HERE, "optim"), exist_ok=True)
        np.savez_compressed(os.path.join(HERE, "optim", name + ".npz"), **d)
        print("wrote", name, {k: v.shape for k, v in list(d.items())[:8] if hasattr(v, "shape")})


if __name__ == "__main__":
    main()
