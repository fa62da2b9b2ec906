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

bool present(const torch::Tensor& t) { return t.defined() && t.numel() != 0; }

// A present input must live on the device of means3D (the kernels get raw device pointers: a host tensor or one on
// another GPU would fault there, so the mistake is reported here as a c10::Error instead) and hold `numel` elements
// when numel >= 0. The reference checks means3D's shape only (rasterize_points.cu:72-75).
void check_on(const torch::Tensor& t, const char* name, const c10::Device& dev, int64_t numel = -1)
{
    if (!present(t)) return;
    TORCH_CHECK(t.device() == dev, name, " must be on ", dev, " (the device of means3D), got ", t.device());
    TORCH_CHECK(numel < 0 || t.numel() == numel, name, " must hold ", numel, " elements, got ", t.numel(), " (shape ",
                t.sizes(), ")");
}

// empty tensor -> NULL ("absent"); otherwise a contiguous float32 view kept alive by `keep`
const float* fptr(const torch::Tensor& t, std::vector<torch::Tensor>& keep, const char* name = "rasterizer input")
{
    if (!present(t)) return nullptr;
    TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be float32, got ", t.scalar_type());
    keep.push_back(t.contiguous());
    return keep.back().data_ptr<float>();
}

// the inputs both directions share: devices and element counts of everything the kernels index by P
void check_inputs(const torch::Tensor& background, const torch::Tensor& means3D, const torch::Tensor& colors,
                  const torch::Tensor& scales, const torch::Tensor& rotations, const torch::Tensor& cov3D_precomp,
                  const torch::Tensor& viewmatrix, const torch::Tensor& projmatrix, const torch::Tensor& sh,
                  const torch::Tensor& campos, int camera_type)
{
    const int64_t P = means3D.size(0);
    TORCH_CHECK(P == 0 || means3D.is_cuda(), "means3D must be a HIP device tensor (the rasterizer has no CPU path), got ",
                means3D.device());
    const c10::Device dev = means3D.device();
    check_on(background, "background", dev, 3);
    check_on(colors, "colors", dev, 3 * P);
    check_on(scales, "scales", dev, 3 * P);
    check_on(rotations, "rotations", dev, 4 * P);
    check_on(cov3D_precomp, "cov3D_precomp", dev, 6 * P);
    check_on(viewmatrix, "viewmatrix", dev, 16);
    check_on(projmatrix, "projmatrix", dev, camera_type == 1 ? 16 : -1);
    check_on(campos, "campos", dev, 3);
    check_on(sh, "sh", dev);
    if (present(sh))
        TORCH_CHECK(sh.dim() == 3 && sh.size(0) == P && sh.size(2) == 3, "sh must be [P, M, 3] with P = ", P,
                    ", got ", sh.sizes());
    TORCH_CHECK(P == 0 || present(background), "background is required");
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
    check_inputs(background, means3D, colors, scales, rotations, cov3D_precomp, viewmatrix, projmatrix, sh, campos,
                 camera_type);
    check_on(opacity, "opacity", means3D.device(), P);
    TORCH_CHECK(H > 0 && W > 0, "image_height and image_width must be positive, got ", H, " x ", W);
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
    if (means3D.ndimension() != 2 || means3D.size(1) != 3) {
        AT_ERROR("means3D must have dimensions (num_points, 3)");
    }
    const int P = means3D.size(0);
    check_inputs(background, means3D, colors, scales, rotations, cov3D_precomp, viewmatrix, projmatrix, sh, campos,
                 camera_type);
    const c10::Device dev = means3D.device();
    // dL_dout_color is [3, H, W] of the view the forward rendered: the image buffer the backward re-reads was sized
    // for exactly that view (omr_image_bytes), and the binning buffer for R instances of it
    TORCH_CHECK(dL_dout_color.dim() == 3 && dL_dout_color.size(0) == 3 && dL_dout_color.size(1) > 0 &&
                    dL_dout_color.size(2) > 0,
                "dL_dout_color must be [3, H, W], got ", dL_dout_color.sizes());
    check_on(dL_dout_color, "dL_dout_color", dev);
    const int H = dL_dout_color.size(1);
    const int W = dL_dout_color.size(2);
    int M = 0;
    if (sh.size(0) != 0) M = sh.size(1);
    TORCH_CHECK(R >= 0, "R (num_rendered) must be >= 0, got ", R);
    if (P != 0) {
        TORCH_CHECK(radii.defined() && radii.dim() == 1 && radii.size(0) == P && radii.scalar_type() == torch::kInt32,
                    "radii must be the forward's [P] int32 tensor with P = ", P, ", got ",
                    radii.defined() ? radii.sizes() : c10::IntArrayRef{}, " ",
                    radii.defined() ? radii.scalar_type() : torch::kInt32);
        check_on(radii, "radii", dev);
        for (const auto* b : {&geomBuffer, &binningBuffer, &imageBuffer}) {
            TORCH_CHECK(b->defined() && b->scalar_type() == torch::kByte && b->dim() == 1,
                        "scratch buffers must be the forward's uint8 geomBuffer / binningBuffer / imgBuffer");
            if (b->numel() != 0) check_on(*b, "scratch buffer", dev);
        }
        TORCH_CHECK(geomBuffer.numel() > 0 && imageBuffer.numel() > 0,
                    "geomBuffer / imgBuffer are empty: pass the buffers the forward returned");
        TORCH_CHECK((size_t)imageBuffer.numel() == omr_image_bytes(W, H),
                    "dL_dout_color is [3, ", H, ", ", W, "] but imgBuffer (", imageBuffer.numel(),
                    " bytes) was sized by the forward for a different view (", omr_image_bytes(W, H),
                    " bytes for this one)");
        TORCH_CHECK(R == 0 || (size_t)binningBuffer.numel() >= omr_binning_bytes(R, W, H), "binningBuffer (",
                    binningBuffer.numel(), " bytes) is too small for R = ", R, " instances of a ", W, " x ", H,
                    " view: pass the forward's num_rendered and buffers");
    }
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
    if (means3D.ndimension() != 2 || means3D.size(1) != 3) {
        AT_ERROR("means3D must have dimensions (num_points, 3)");
    }
    const int P = means3D.size(0);
    TORCH_CHECK(P == 0 || means3D.is_cuda(), "means3D must be a HIP device tensor, got ", means3D.device());
    check_on(viewmatrix, "viewmatrix", means3D.device(), 16);
    check_on(projmatrix, "projmatrix", means3D.device(), 16);
    TORCH_CHECK(camera_type != 1 || P == 0 || (present(viewmatrix) && present(projmatrix)),
                "pinhole markVisible needs viewmatrix and projmatrix");
    c10::DeviceGuard guard(means3D.device());
    torch::Tensor visible = torch::full({P}, false, means3D.options().dtype(at::kBool));
    if (P != 0) {
        std::vector<torch::Tensor> keep;
        int rc;
        if (camera_type == 1) {
            rc = omr_rasterizer_mark_visible(P, fptr(means3D, keep), fptr(viewmatrix, keep), fptr(projmatrix, keep),
                                             visible.data_ptr<bool>(), stream_of(means3D));
        } else if (camera_type == 3) {
            rc = omr_lonlat_mark_visible(P, visible.data_ptr<bool>(), stream_of(means3D));
        } else {
            throw std::runtime_error("[CudaRasterizer]Invalid camera_type");
        }
        throw_status(rc, "markVisible");
    }
    return visible;
}
