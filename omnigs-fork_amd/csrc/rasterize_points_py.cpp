// rasterize_points_py.cpp — Python binding of the LibTorch drop-in (librasterize_points.so) so that tests can
// call the exact C++ symbols a LibTorch host links against. Not on the hot path.
#include <torch/extension.h>

#include "../../include/rasterize_points.h"

PYBIND11_MODULE(_rasterize_points, m)
{
    m.doc() = "LibTorch boundary of the gfx950 rasterizer (reference include/rasterize_points.h)";
    m.def("RasterizeGaussiansCUDA", &RasterizeGaussiansCUDA, "forward (rasterize_points.h:29-50)",
          py::arg("background"), py::arg("means3D"), py::arg("colors"), py::arg("opacity"), py::arg("scales"),
          py::arg("rotations"), py::arg("scale_modifier"), py::arg("cov3D_precomp"), py::arg("viewmatrix"),
          py::arg("projmatrix"), py::arg("tan_fovx"), py::arg("tan_fovy"), py::arg("image_height"),
          py::arg("image_width"), py::arg("sh"), py::arg("degree"), py::arg("campos"), py::arg("prefiltered"),
          py::arg("camera_type") = 1, py::arg("render_depth") = false);
    m.def("RasterizeGaussiansBackwardCUDA", &RasterizeGaussiansBackwardCUDA, "backward (rasterize_points.h:52-74)",
          py::arg("background"), py::arg("means3D"), py::arg("radii"), py::arg("colors"), py::arg("scales"),
          py::arg("rotations"), py::arg("scale_modifier"), py::arg("cov3D_precomp"), py::arg("viewmatrix"),
          py::arg("projmatrix"), py::arg("tan_fovx"), py::arg("tan_fovy"), py::arg("dL_dout_color"), py::arg("sh"),
          py::arg("degree"), py::arg("campos"), py::arg("geomBuffer"), py::arg("R"), py::arg("binningBuffer"),
          py::arg("imageBuffer"), py::arg("camera_type") = 1);
    m.def("markVisible", &markVisible, "markVisible (rasterize_points.h:76-80)", py::arg("means3D"),
          py::arg("viewmatrix"), py::arg("projmatrix"), py::arg("camera_type") = 1);
}
