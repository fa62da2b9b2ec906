#!/usr/bin/env python3
"""Build the LibTorch drop-in of include/rasterize_points.h:

  lib/librasterize_points.so            RasterizeGaussiansCUDA / RasterizeGaussiansBackwardCUDA / markVisible
                                        (C++ symbols, CXX11 ABI as PyTorch-ROCm), linked to libomnigs_raster.so
  lib/_rasterize_points<ext-suffix>     pybind11 module exposing the same three functions (tests)
  tests/cpp/build/reference_host_caller  test program: the reference host's torch::autograd::Function over the
                                        drop-in (tests/test_gpu_libtorch_cpp.py); test infrastructure only

Host-only C++ (no device code: kernels live in libomnigs_raster.so), so plain g++ against the torch headers.
Skips work when outputs are newer than their inputs.
"""
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
LIB = os.path.join(PKG, "lib")


def _stale(out, deps):
    return not os.path.exists(out) or any(os.path.getmtime(d) > os.path.getmtime(out) for d in deps)


def main():
    import torch
    import torch.utils.cpp_extension as ce

    os.makedirs(LIB, exist_ok=True)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    inc = [f"-I{p}" for p in ce.include_paths()] + ["-I/opt/rocm/include", f"-I{os.path.join(ROOT, 'include')}"]
    tlib = ce.library_paths()[0]
    common = ["-O2", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1",
              "-DUSE_ROCM=1", "-Wno-deprecated-declarations"] + inc
    torch_libs = [f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch", f"-Wl,-rpath,{tlib}"]
    core = os.path.join(LIB, "librasterize_points.so")
    src = os.path.join(HERE, "rasterize_points.cpp")
    hdrs = [os.path.join(ROOT, "include", "rasterize_points.h"), os.path.join(ROOT, "include", "omnigs_raster.h")]
    if _stale(core, [src] + hdrs):
        cmd = ["g++", *common, "-shared", "-o", core, src, f"-L{LIB}", "-lomnigs_raster", "-Wl,-rpath,$ORIGIN",
               *torch_libs, "-L/opt/rocm/lib", "-lamdhip64"]
        subprocess.run(cmd, check=True)
    ext = os.path.join(LIB, "_rasterize_points" + sysconfig.get_config_var("EXT_SUFFIX"))
    bsrc = os.path.join(HERE, "rasterize_points_py.cpp")
    if _stale(ext, [bsrc, core] + hdrs):
        pyinc = f"-I{sysconfig.get_paths()['include']}"
        cmd = ["g++", *common, pyinc, "-DTORCH_EXTENSION_NAME=_rasterize_points", "-DTORCH_API_INCLUDE_EXTENSION_H",
               "-shared", "-o", ext, bsrc, f"-L{LIB}", "-lrasterize_points", "-Wl,-rpath,$ORIGIN", *torch_libs,
               "-ltorch_python"]
        subprocess.run(cmd, check=True)
    tdir = os.path.join(ROOT, "tests", "cpp")
    tsrc = os.path.join(tdir, "reference_host_caller.cpp")
    texe = os.path.join(tdir, "build", "reference_host_caller")
    if os.path.exists(tsrc) and _stale(texe, [tsrc, core] + hdrs):
        os.makedirs(os.path.dirname(texe), exist_ok=True)
        # --no-as-needed: nothing here names a torch_hip symbol, but the CUDA(HIP) device registers from it
        cmd = ["g++", *common, "-o", texe, tsrc, "-Wl,--no-as-needed", f"-L{LIB}", "-lrasterize_points",
               "-Wl,-rpath,$ORIGIN/../../../omnigs-fork_amd/lib", *torch_libs]
        subprocess.run(cmd, check=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
