"""Loader for the `omnigs-fork_amd/` package (its directory name is not a Python identifier).

    import _omnigs
    omr = _omnigs.load()          # -> module `omnigs_fork_amd`
    omr.rasterizer.RasterizeGaussiansCUDA(...)
"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "omnigs-fork_amd")
NAME = "omnigs_fork_amd"


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(NAME, os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
