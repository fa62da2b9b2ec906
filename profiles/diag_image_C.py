"""GPU side of the config-C forward-image diagnosis: saves the HIP image, n_contrib and final_T to
gpurun_out/diag_C.npz; the oracle side and the per-pixel analysis run on the CPU (profiles/diag_image_C_cpu.py)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from helpers import hip_run, scene, to_np  # noqa: E402

g, cam, _ = scene.config_scene("C")
h = hip_run(g, cam, None)
st = h["state"]
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "diag_C.npz"), color=to_np(h["color"]),
                    n_contrib=to_np(st["n_contrib"]), final_T=to_np(st["final_T"]), L=h["L"])
print("saved", h["L"])
