/*
 * rasterize_points.h — LibTorch boundary of the rasterizer, symbol-for-symbol the reference's
 * include/rasterize_points.h:29-80 (raikuma/OmniGS-fork @ 2025-03-04), so that a LibTorch host
 * (src/gaussian_rasterizer.cpp, GaussianRenderer) links against librasterize_points.so unchanged.
 *
 * Implemented in omnigs-fork_amd/csrc/rasterize_points.cpp on top of the C ABI of omnigs_raster.h.
 * Differences a caller can observe (all compatible with the reference's callers):
 *   - tensors are allocated on means3D.device() and kernels run on the current HIP stream of that device
 *     (the reference hard-codes torch::kCUDA and the legacy default stream, rasterize_points.cu:87);
 *   - the scratch byte tensors have this library's private layout (only forward/backward interpret them).
 */
#pragma once
#include <torch/torch.h>

#include <cstdio>
#include <string>
#include <tuple>

std::tuple<int, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor>
RasterizeGaussiansCUDA(
    const torch::Tensor& background,
    const torch::Tensor& means3D,
    const torch::Tensor& colors,
    const torch::Tensor& opacity,
    const torch::Tensor& scales,
    const torch::Tensor& rotations,
    const float scale_modifier,
    const torch::Tensor& cov3D_precomp,
    const torch::Tensor& viewmatrix,
    const torch::Tensor& projmatrix,
    const float tan_fovx,
    const float tan_fovy,
    const int image_height,
    const int image_width,
    const torch::Tensor& sh,
    const int degree,
    const torch::Tensor& campos,
    const bool prefiltered,
    const int camera_type = 1,
    const bool render_depth = false);

std::tuple<torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor,
           torch::Tensor>
RasterizeGaussiansBackwardCUDA(
    const torch::Tensor& background,
    const torch::Tensor& means3D,
    const torch::Tensor& radii,
    const torch::Tensor& colors,
    const torch::Tensor& scales,
    const torch::Tensor& rotations,
    const float scale_modifier,
    const torch::Tensor& cov3D_precomp,
    const torch::Tensor& viewmatrix,
    const torch::Tensor& projmatrix,
    const float tan_fovx,
    const float tan_fovy,
    const torch::Tensor& dL_dout_color,
    const torch::Tensor& sh,
    const int degree,
    const torch::Tensor& campos,
    const torch::Tensor& geomBuffer,
    const int R,
    const torch::Tensor& binningBuffer,
    const torch::Tensor& imageBuffer,
    const int camera_type = 1);

torch::Tensor markVisible(
    torch::Tensor& means3D,
    torch::Tensor& viewmatrix,
    torch::Tensor& projmatrix,
    const int camera_type = 1);
