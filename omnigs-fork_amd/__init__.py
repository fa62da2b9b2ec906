"""omnigs-fork_amd — MI355X-native (gfx950) omnidirectional Gaussian-splat rasterizer.

The directory name is not a Python identifier; load it as `omnigs_fork_amd` with `_omnigs.load()` at the repo root.

Layout:
  csrc/            HIP kernels for gfx950 + the C ABI (include/omnigs_raster.h) -> lib/libomnigs_raster.so
  csrc/rasterize_points.cpp  LibTorch drop-in of include/rasterize_points.h (reference symbols)
  rasterizer.py    Python mirror of the reference boundary + autograd wrapper, on the C ABI
  renderer.py      GaussianRenderer::renderLonlat / render glue (activations, settings)
  parallel.py      view-parallel data parallelism (one view per GPU, RCCL exchange of Gaussian gradients)
  losses.py        training loss (1 - lambda) L1 + lambda (1 - SSIM), fused forward+backward HIP kernel
  optim.py         Adam over the six GaussianModel groups (activation backward fused), LR schedule, densification
  trainer.py       one training iteration without autograd: render, fused loss, backward, stats, Adam
  formats.py       PLY load / save (HIP (de)interleave), distCUDA2 (exact 3-NN on gfx950), createFromPcd
  scene.py         deterministic synthetic scenes and camera poses
"""
from . import scene  # noqa: F401

__all__ = ["scene", "rasterizer"]


def __getattr__(name):
    # the HIP-backed modules import torch and the shared library lazily
    if name in ("rasterizer", "renderer", "parallel", "losses", "optim", "trainer", "formats"):
        import importlib

        mod = importlib.import_module(f"{__name__}.{name}")
        globals()[name] = mod
        return mod
    raise AttributeError(name)
