// rasterize_points.cpp — the reference's LibTorch boundary (include/rasterize_points.h:29-80,
// src/rasterize_points.cu:41-319) implemented on the gfx950 C ABI (include/omnigs_raster.h).
//
// Same symbols, argument meaning, return tuples, empty-tensor-means-absent convention and error behaviour
// (c10::Error for a bad means3D shape, std::runtime_error for an invalid camera_type). The device is
// means3D.device() and the stream is that device's current HIP stream.
#include "../../include/rasterize_points.h"

#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include <stdexcept>

#include "../../include/omnigs_raster.h"

namespace {

// resizeFunctional (rasterize_points.cu:41-47) as a C callback: ctx is the torch::Tensor to resize
void* resize_cb(void* ctx, size_t n)
{
    auto* t = static_cast<torch::Tensor*>(ctx);
    t->resize_({(long long)n});
    return t->data_ptr();
}

// empty tensor -> NULL ("absent"); otherwise a contiguous float32 view kept alive by `keep`
const float* fptr(const torch::Tensor& t, std::vector<torch::Tensor>& keep)
{
    if (!t.defined() || t.numel() == 0) return nullptr;
    TORCH_CHECK(t.scalar_type() == torch::kFloat32, "rasterizer inputs must be float32");
    keep.push_back(t.contiguous());
    return keep.back().data_ptr<float>();
}

void* stream_of(const torch::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void throw_status(int rc, const char* what)
{
    if (rc == OMR_OK) return;
    const std::string msg = std::string(what) + ": " + omr_last_error();
    if (rc == OMR_ERR_CAMERA_TYPE) throw std::runtime_error("[CudaRasterizer]Invalid camera_type");
    if (rc == OMR_ERR_PREFILTERED) throw std::runtime_error(msg);
    TORCH_CHECK(false, msg);
}

}  // namespace

std::tuple<int, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor>
RasterizeGaussiansCUDA(const torch::Tensor& background, const torch::Tensor& means3D, const torch::Tensor& colors,
                       const torch::Tensor& opacity, const torch::Tensor& scales, const torch::Tensor& rotations,
                       const float scale_modifier, const torch::Tensor& cov3D_precomp, const torch::Tensor& viewmatrix,
                       const torch::Tensor& projmatrix, const float tan_fovx, const float tan_fovy,
                       const int image_height, const int image_width, const torch::Tensor& sh, const int degree,
                       const torch::Tensor& campos, const bool prefiltered, const int camera_type,
                       const bool render_depth)
{
    if (means3D.ndimension() != 2 || means3D.size(1) != 3) {
        AT_ERROR("means3D must have dimensions (num_points, 3)");
    }
    const int P = means3D.size(0);
    const int H = image_height;
    const int W = image_width;
    c10::DeviceGuard guard(means3D.device());
    auto float_opts = means3D.options().dtype(torch::kFloat32);
    // every pixel / Gaussian is written by the kernels when P > 0, so only P == 0 needs the zero fill
    torch::Tensor out_color = P == 0 ? torch::zeros({3, H, W}, float_opts) : torch::empty({3, H, W}, float_opts);
    torch::Tensor radii = torch::empty({P}, means3D.options().dtype(torch::kInt32));
    torch::TensorOptions bytes = means3D.options().dtype(torch::kByte);
    torch::Tensor geomBuffer = torch::empty({0}, bytes);
    torch::Tensor binningBuffer = torch::empty({0}, bytes);
    torch::Tensor imgBuffer = torch::empty({0}, bytes);
    int rendered = 0;
    if (P != 0) {
        int M = 0;
        if (sh.size(0) != 0) M = sh.size(1);
        std::vector<torch::Tensor> keep;
        const float* bg = fptr(background, keep);
        const float* m = fptr(means3D, keep);
        const float* shp = fptr(sh, keep);
        const float* col = fptr(colors, keep);
        const float* op = fptr(opacity, keep);
        const float* sc = fptr(scales, keep);
        const float* rot = fptr(rotations, keep);
        const float* cov = fptr(cov3D_precomp, keep);
        const float* vm = fptr(viewmatrix, keep);
        const float* pm = fptr(projmatrix, keep);
        const float* cp = fptr(campos, keep);
        int rc;
        if (camera_type == 1) {  // PINHOLE
            rc = omr_rasterizer_forward(resize_cb, &geomBuffer, resize_cb, &binningBuffer, resize_cb, &imgBuffer, P,
                                        degree, M, bg, W, H, m, shp, col, op, sc, scale_modifier, rot, cov, vm, pm,
                                        cp, tan_fovx, tan_fovy, prefiltered, out_color.data_ptr<float>(),
                                        radii.data_ptr<int>(), render_depth, stream_of(means3D), &rendered);
        } else if (camera_type == 3) {  // LONLAT
            rc = omr_lonlat_forward(resize_cb, &geomBuffer, resize_cb, &binningBuffer, resize_cb, &imgBuffer, P,
                                    degree, M, bg, W, H, m, shp, col, op, sc, scale_modifier, rot, cov, vm, cp,
                                    prefiltered, out_color.data_ptr<float>(), radii.data_ptr<int>(),
                                    stream_of(means3D), &rendered);
        } else {
            throw std::runtime_error("[CudaRasterizer]Invalid camera_type");
        }
        throw_status(rc, "RasterizeGaussiansCUDA");
    }
    return std::make_tuple(rendered, out_color, radii, geomBuffer, binningBuffer, imgBuffer);
}

std::tuple<torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor,
           torch::Tensor>
RasterizeGaussiansBackwardCUDA(const torch::Tensor& background, const torch::Tensor& means3D, const torch::Tensor& radii,
                               const torch::Tensor& colors, const torch::Tensor& scales, const torch::Tensor& rotations,
                               const float scale_modifier, const torch::Tensor& cov3D_precomp,
                               const torch::Tensor& viewmatrix, const torch::Tensor& projmatrix, const float tan_fovx,
                               const float tan_fovy, const torch::Tensor& dL_dout_color, const torch::Tensor& sh,
                               const int degree, const torch::Tensor& campos, const torch::Tensor& geomBuffer,
                               const int R, const torch::Tensor& binningBuffer, const torch::Tensor& imageBuffer,
                               const int camera_type)
{
    const int P = means3D.size(0);
    const int H = dL_dout_color.size(1);
    const int W = dL_dout_color.size(2);
    int M = 0;
    if (sh.size(0) != 0) M = sh.size(1);
    c10::DeviceGuard guard(means3D.device());
    auto o = means3D.options().dtype(torch::kFloat32);
    // the gfx950 backward writes every element, so only P == 0 needs zeros (rasterize_points.cu:200-208 zero-fill)
    auto make = [&](std::initializer_list<int64_t> s) { return P == 0 ? torch::zeros(s, o) : torch::empty(s, o); };
    torch::Tensor dL_dmeans3D = make({P, 3});
    torch::Tensor dL_dmeans2D = make({P, 3});
    torch::Tensor dL_dcolors = make({P, 3});
    torch::Tensor dL_dopacity = make({P, 1});
    torch::Tensor dL_dcov3D = make({P, 6});
    torch::Tensor dL_dsh = make({P, M, 3});
    torch::Tensor dL_dscales = make({P, 3});
    torch::Tensor dL_drotations = make({P, 4});
    if (P != 0) {
        std::vector<torch::Tensor> keep;
        const float* bg = fptr(background, keep);
        const float* m = fptr(means3D, keep);
        const float* shp = fptr(sh, keep);
        const float* col = fptr(colors, keep);
        const float* sc = fptr(scales, keep);
        const float* rot = fptr(rotations, keep);
        const float* cov = fptr(cov3D_precomp, keep);
        const float* vm = fptr(viewmatrix, keep);
        const float* cp = fptr(campos, keep);
        const float* dl = fptr(dL_dout_color, keep);
        torch::Tensor rad = radii.contiguous();
        char* gb = reinterpret_cast<char*>(geomBuffer.data_ptr());
        char* bb = reinterpret_cast<char*>(binningBuffer.data_ptr());
        char* ib = reinterpret_cast<char*>(imageBuffer.data_ptr());
        int rc;
        if (camera_type == 1) {
            const float* pm = fptr(projmatrix, keep);
            rc = omr_rasterizer_backward(P, degree, M, R, bg, W, H, m, shp, col, sc, scale_modifier, rot, cov, vm, pm,
                                         cp, tan_fovx, tan_fovy, rad.data_ptr<int>(), gb, bb, ib, dl,
                                         dL_dmeans2D.data_ptr<float>(), nullptr, dL_dopacity.data_ptr<float>(),
                                         dL_dcolors.data_ptr<float>(), dL_dmeans3D.data_ptr<float>(),
                                         dL_dcov3D.data_ptr<float>(), M ? dL_dsh.data_ptr<float>() : nullptr,
                                         dL_dscales.data_ptr<float>(), dL_drotations.data_ptr<float>(),
                                         stream_of(means3D));
        } else if (camera_type == 3) {
            rc = omr_lonlat_backward(P, degree, M, R, bg, W, H, m, shp, col, sc, scale_modifier, rot, cov, vm, cp,
                                     rad.data_ptr<int>(), gb, bb, ib, dl, dL_dmeans2D.data_ptr<float>(), nullptr,
                                     dL_dopacity.data_ptr<float>(), dL_dcolors.data_ptr<float>(),
                                     dL_dmeans3D.data_ptr<float>(), dL_dcov3D.data_ptr<float>(),
                                     M ? dL_dsh.data_ptr<float>() : nullptr, dL_dscales.data_ptr<float>(),
                                     dL_drotations.data_ptr<float>(), nullptr, nullptr, stream_of(means3D));
        } else {
            throw std::runtime_error("[CudaRasterizer]Invalid camera_type");
        }
        throw_status(rc, "RasterizeGaussiansBackwardCUDA");
    }
    return std::make_tuple(dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales,
                           dL_drotations);
}

torch::Tensor markVisible(torch::Tensor& means3D, torch::Tensor& viewmatrix, torch::Tensor& projmatrix,
                          const int camera_type)
{
    const int P = means3D.size(0);
    c10::DeviceGuard guard(means3D.device());
    torch::Tensor present = torch::full({P}, false, means3D.options().dtype(at::kBool));
    if (P != 0) {
        std::vector<torch::Tensor> keep;
        int rc;
        if (camera_type == 1) {
            rc = omr_rasterizer_mark_visible(P, fptr(means3D, keep), fptr(viewmatrix, keep), fptr(projmatrix, keep),
                                             present.data_ptr<bool>(), stream_of(means3D));
        } else if (camera_type == 3) {
            rc = omr_lonlat_mark_visible(P, present.data_ptr<bool>(), stream_of(means3D));
        } else {
            throw std::runtime_error("[CudaRasterizer]Invalid camera_type");
        }
        throw_status(rc, "markVisible");
    }
    return present;
}
