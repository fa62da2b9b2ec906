// Test program: the reference's LibTorch host, as its authors would call our drop-in.
//
// It restates what /root/reference/src/gaussian_rasterizer.cpp does on top of include/rasterize_points.h and
// links only lib/librasterize_points.so (the product's LibTorch boundary) and LibTorch:
//   - GaussianRasterizationSettings: the fields gaussian_rasterizer.h keeps (bg, view/proj matrices, campos,
//     tan fov, image size, SH degree, scale modifier, prefiltered, camera type, render_depth);
//   - RasterizerFn: a torch::autograd::Function whose forward calls RasterizeGaussiansCUDA and saves the three
//     opaque byte buffers (geomBuffer / binningBuffer / imgBuffer) + num_rendered R for the backward
//     (gaussian_rasterizer.cpp:47-98), and whose backward restores them, calls RasterizeGaussiansBackwardCUDA
//     and maps its 8 outputs onto the forward's 9 inputs (:109-169: means3D, means2D, sh, colors, opacities,
//     scales, rotations, cov3D, settings -> undefined);
//   - the exactly-one-of checks of GaussianRasterizer::forward (:190-196).
// main() reads one case from a directory of raw little-endian float32 files (written by
// tests/test_gpu_libtorch_cpp.py), runs forward, loss = sum(color * dL_dcolor), loss.backward() through LibTorch's
// autograd engine, and writes the color, radii and the leaf gradients back as raw files.
//
// Test infrastructure only: built by omnigs-fork_amd/csrc/build_torch_ext.py into tests/cpp/build/.
#include <torch/torch.h>

#include <cstdio>
#include <fstream>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "rasterize_points.h"

namespace {

struct RasterSettings {
    int64_t image_height = 0, image_width = 0;
    double tanfovx = 0, tanfovy = 0, scale_modifier = 1.0;
    torch::Tensor bg, viewmatrix, projmatrix, campos;
    int64_t sh_degree = 0, camera_type = 1;
    bool prefiltered = false, render_depth = false;
};

struct RasterizerFn : public torch::autograd::Function<RasterizerFn> {
    static torch::autograd::tensor_list forward(torch::autograd::AutogradContext* ctx, torch::Tensor means3D,
                                                torch::Tensor means2D, torch::Tensor sh, torch::Tensor colors,
                                                torch::Tensor opacities, torch::Tensor scales,
                                                torch::Tensor rotations, torch::Tensor cov3D,
                                                const RasterSettings& s) {
        (void)means2D;  // only carries dL/dmeans2D out of the backward
        auto res = RasterizeGaussiansCUDA(s.bg, means3D, colors, opacities, scales, rotations,
                                          static_cast<float>(s.scale_modifier), cov3D, s.viewmatrix, s.projmatrix,
                                          static_cast<float>(s.tanfovx), static_cast<float>(s.tanfovy),
                                          static_cast<int>(s.image_height), static_cast<int>(s.image_width), sh,
                                          static_cast<int>(s.sh_degree), s.campos, s.prefiltered,
                                          static_cast<int>(s.camera_type), s.render_depth);
        ctx->saved_data["R"] = static_cast<int64_t>(std::get<0>(res));
        ctx->saved_data["scale_modifier"] = s.scale_modifier;
        ctx->saved_data["tanfovx"] = s.tanfovx;
        ctx->saved_data["tanfovy"] = s.tanfovy;
        ctx->saved_data["sh_degree"] = s.sh_degree;
        ctx->saved_data["camera_type"] = s.camera_type;
        ctx->save_for_backward({s.bg, s.viewmatrix, s.projmatrix, s.campos, colors, means3D, scales, rotations, cov3D,
                                std::get<2>(res), sh, std::get<3>(res), std::get<4>(res), std::get<5>(res)});
        return {std::get<1>(res), std::get<2>(res)};
    }

    static torch::autograd::tensor_list backward(torch::autograd::AutogradContext* ctx,
                                                 torch::autograd::tensor_list grad_out) {
        auto v = ctx->get_saved_variables();
        const auto f = [&](const char* k) { return static_cast<float>(ctx->saved_data[k].toDouble()); };
        const auto i = [&](const char* k) { return static_cast<int>(ctx->saved_data[k].toInt()); };
        // v: 0 bg, 1 view, 2 proj, 3 campos, 4 colors, 5 means3D, 6 scales, 7 rotations, 8 cov3D, 9 radii, 10 sh,
        //    11 geomBuffer, 12 binningBuffer, 13 imgBuffer
        auto g = RasterizeGaussiansBackwardCUDA(v[0], v[5], v[9], v[4], v[6], v[7], f("scale_modifier"), v[8], v[1],
                                                v[2], f("tanfovx"), f("tanfovy"), grad_out[0].contiguous(), v[10],
                                                i("sh_degree"), v[3], v[11], i("R"), v[12], v[13], i("camera_type"));
        // outputs: 0 dmeans2D, 1 dcolors, 2 dopacity, 3 dmeans3D, 4 dcov3D, 5 dsh, 6 dscales, 7 drotations
        return {std::get<3>(g), std::get<0>(g), std::get<5>(g), std::get<1>(g), std::get<2>(g),
                std::get<6>(g), std::get<7>(g), std::get<4>(g), torch::Tensor()};
    }
};

// GaussianRasterizer::forward's argument checks (gaussian_rasterizer.cpp:190-196), then the autograd call.
torch::autograd::tensor_list rasterize(const RasterSettings& s, torch::Tensor means3D, torch::Tensor means2D,
                                       torch::Tensor opacities, torch::Tensor shs, torch::Tensor colors,
                                       torch::Tensor scales, torch::Tensor rotations, torch::Tensor cov3D) {
    const bool has_sh = shs.defined(), has_col = colors.defined();
    const bool has_sr = scales.defined() || rotations.defined(), has_cov = cov3D.defined();
    if (has_sh == has_col) throw std::runtime_error("Please provide excatly one of either SHs or precomputed colors!");
    if ((!(scales.defined() && rotations.defined()) && !has_cov) || (has_sr && has_cov))
        throw std::runtime_error(
            "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
    const auto empty = torch::empty({0}, torch::TensorOptions().device(means3D.device()));
    return RasterizerFn::apply(means3D, means2D, has_sh ? shs : empty, has_col ? colors : empty, opacities,
                               has_sr ? scales : empty, has_sr ? rotations : empty, has_cov ? cov3D : empty, s);
}

std::map<std::string, std::string> read_params(const std::string& path) {
    std::map<std::string, std::string> kv;
    std::ifstream in(path);
    if (!in) throw std::runtime_error("cannot open " + path);
    std::string k, v;
    while (in >> k >> v) kv[k] = v;
    return kv;
}

torch::Tensor read_f32(const std::string& dir, const std::string& name, std::vector<int64_t> shape) {
    int64_t n = 1;
    for (auto d : shape) n *= d;
    std::vector<float> buf(static_cast<size_t>(n));
    std::ifstream in(dir + "/" + name + ".f32", std::ios::binary);
    if (!in) throw std::runtime_error("cannot open " + dir + "/" + name + ".f32");
    in.read(reinterpret_cast<char*>(buf.data()), static_cast<std::streamsize>(n * sizeof(float)));
    if (in.gcount() != static_cast<std::streamsize>(n * sizeof(float))) throw std::runtime_error("short " + name);
    return torch::from_blob(buf.data(), shape, torch::kFloat32).clone().to(torch::kCUDA);
}

void write_raw(const std::string& dir, const std::string& name, const torch::Tensor& t) {
    auto c = t.detach().to(torch::kCPU).contiguous();
    std::ofstream out(dir + "/" + name + (c.scalar_type() == torch::kInt32 ? ".i32" : ".f32"), std::ios::binary);
    out.write(reinterpret_cast<const char*>(c.data_ptr()), static_cast<std::streamsize>(c.nbytes()));
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s <case_dir> <out_dir>\n", argv[0]);
        return 2;
    }
    const std::string dir = argv[1], out = argv[2];
    try {
        auto kv = read_params(dir + "/params.txt");
        const int64_t P = std::stoll(kv.at("P")), W = std::stoll(kv.at("W")), H = std::stoll(kv.at("H"));
        const int64_t deg = std::stoll(kv.at("sh_degree"));
        const int64_t M = std::stoll(kv.at("M"));  // SH coefficients per Gaussian in the file
        RasterSettings s;
        s.image_width = W;
        s.image_height = H;
        s.tanfovx = std::stod(kv.at("tanfovx"));
        s.tanfovy = std::stod(kv.at("tanfovy"));
        s.sh_degree = deg;
        s.camera_type = std::stoll(kv.at("camera_type"));
        s.bg = read_f32(dir, "bg", {3});
        s.viewmatrix = read_f32(dir, "viewmatrix", {4, 4});
        s.projmatrix = read_f32(dir, "projmatrix", {4, 4});
        s.campos = read_f32(dir, "campos", {3});

        auto leaf = [](torch::Tensor t) { return t.set_requires_grad(true); };
        auto means3D = leaf(read_f32(dir, "means3D", {P, 3}));
        auto means2D = leaf(torch::zeros({P, 3}, torch::TensorOptions().device(torch::kCUDA)));
        auto shs = leaf(read_f32(dir, "shs", {P, M, 3}));
        auto opac = leaf(read_f32(dir, "opacity", {P, 1}));
        auto scales = leaf(read_f32(dir, "scales", {P, 3}));
        auto rots = leaf(read_f32(dir, "rotations", {P, 4}));
        auto dL = read_f32(dir, "dL_dcolor", {3, H, W});

        auto r = rasterize(s, means3D, means2D, opac, shs, torch::Tensor(), scales, rots, torch::Tensor());
        auto loss = (r[0] * dL).sum();
        loss.backward();
        torch::cuda::synchronize();

        write_raw(out, "color", r[0]);
        write_raw(out, "radii", r[1]);
        write_raw(out, "dmean3D", means3D.grad());
        write_raw(out, "dmean2D", means2D.grad());
        write_raw(out, "dsh", shs.grad());
        write_raw(out, "dopacity", opac.grad());
        write_raw(out, "dscale", scales.grad());
        write_raw(out, "drot", rots.grad());

        // the exactly-one-of checks must throw as the reference's do
        int refused = 0;
        try {
            rasterize(s, means3D, means2D, opac, shs, r[0], scales, rots, torch::Tensor());
        } catch (const std::runtime_error&) {
            ++refused;
        }
        try {
            rasterize(s, means3D, means2D, opac, shs, torch::Tensor(), scales, torch::Tensor(), torch::Tensor());
        } catch (const std::runtime_error&) {
            ++refused;
        }
        std::printf("{\"ok\": true, \"P\": %lld, \"loss\": %.9g, \"refused\": %d}\n", static_cast<long long>(P),
                    loss.item<double>(), refused);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "reference_host_caller: %s\n", e.what());
        return 1;
    }
    return 0;
}
