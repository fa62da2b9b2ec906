"""The parity allowance against the reference AS COMPILED (no GPU).

nvcc compiles the reference with --fmad=true (its default: /root/reference/CMakeLists.txt:60-85 sets no -fmad flag),
the oracle without contraction. Two FMA-contracted builds of the oracle (oracle/Makefile: GCC and LLVM fuse
different multiplies) stand in for the reference binary. Everything they change against the oracle — sorted
point-list positions, pixels over 1e-4, gradients outside grad_close — must lie inside the allowance that
oracle/ambiguity.hpp derives from the oracle's own forward, which is exactly what the GPU parity tests excuse
(tests/helpers.py: reference_allowance, check_image, check_grads). Configs A and B in full (B: the point list
reorders under GCC's contraction; pixels over 1e-4 in both builds), a pinhole view and one with white background.
A third build with glibc's atan2f / asinf (libm) stands in for libdevice's transcendentals.
oracle/contraction.py runs the same check at every BASELINE config (profiles/ambiguity.json)."""
import numpy as np
import pytest

from helpers import check_grads, check_image, make_case, oracle_run, reference_allowance, scene

# fma_*: FMA-contracted builds (nvcc --fmad=true); libm: glibc's atan2f / asinf instead of omni_math.h's, a second
# implementation of the transcendentals the lonlat centres depend on (the reference's are libdevice's)
VARIANTS = ["fma_gcc", "fma_clang", "libm"]


@pytest.fixture(scope="module")
def contraction(oracle_mod):
    import contraction as Cn

    oracle_mod.set_threads(4)
    yield Cn
    oracle_mod.set_threads(1)


def _check(g, cam, dL, Cn, variant, bg=(0.0, 0.0, 0.0)):
    import oracle as O

    ob, _, gb = oracle_run(g, cam, dL, bg=bg, nthreads=4)
    allow = reference_allowance(ob, dL)
    ov = O.Oracle(False, variant)
    ov.forward(background=np.asarray(bg, np.float64), means3D=g.means3D, opacity=g.opacity, scales=g.scales,
               rotations=g.rotations, shs=g.shs, viewmatrix=cam.viewmatrix, projmatrix=cam.projmatrix,
               campos=cam.campos, width=cam.width, height=cam.height, sh_degree=g.sh_degree, tanfovx=cam.tanfovx,
               tanfovy=cam.tanfovy, camera_type=cam.camera_type)
    gv = ov.backward(dL, 4)
    res = Cn.compare_variant(ob, gb, ov, gv, allow, cam.height, cam.width)
    assert Cn.unexplained(res) == 0, res
    # the same bars through the comparators the GPU parity tests use
    H, W = cam.height, cam.width
    check_image(ov.get("out_color").reshape(3, H, W), ob.get("out_color").reshape(3, H, W), allow)
    check_image(ov.get("final_T").reshape(H, W), ob.get("final_T").reshape(H, W), allow, "final_T", "t_bound")
    check_grads(gv, gb, allow, g.P)
    return res, allow


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("name", ["A", "B"])
def test_contracted_reference_inside_allowance(name, variant, contraction):
    g, cam, dL = scene.config_scene(name)
    res, allow = _check(g, cam, dL, contraction, variant)
    if variant == "libm":  # only the lonlat centres (atan2 / asin) differ, and in many Gaussians
        assert res["means2D_changed"] > g.P // 10 and res["depths_changed"] == 0
    else:
        assert res["depths_changed"] > 0 and res["conic_opacity_changed"] > 0  # the builds do differ
    if name == "B":
        assert res["pixels_over_1e-4"] > 0  # and some of it shows: the allowance is exercised, not idle
        assert allow["counts"]["order_pairs"] > 0


@pytest.mark.parametrize("variant", VARIANTS)
def test_contracted_reference_inside_allowance_pinhole(variant, contraction):
    g, cam, dL = make_case(20000, 480, 270, scene.CAMERA_PINHOLE, 91, view_index=3, spread=1.5)
    _check(g, cam, dL, contraction, variant)


@pytest.mark.parametrize("variant", VARIANTS)
def test_contracted_reference_inside_allowance_white_bg(variant, contraction):
    g, cam, dL = make_case(20000, 512, 256, scene.CAMERA_LONLAT, 92, view_index=5, spread=1.5)
    _check(g, cam, dL, contraction, variant, bg=(1.0, 1.0, 1.0))


def test_allowance_flags_a_known_order_tie(oracle_mod):
    """Two Gaussians at the same depth that both blend at a pixel: the reference may blend them in either order
    (its sort key ties or differs by an ulp), so the pixel is flagged PX_ORDER and both own the decision."""
    g, cam, dL = make_case(2, 64, 32, scene.CAMERA_LONLAT, 93, spread=1.0)
    g.means3D = np.array([[0.0, 0.0, 3.0], [0.0, 0.0, 3.0]], np.float32)
    g.scales = np.full((2, 3), 0.05, np.float32)
    g.rotations = np.array([[1, 0, 0, 0], [1, 0, 0, 0]], np.float32)
    g.opacity = np.array([[0.6], [0.6]], np.float32)
    o, L, _ = oracle_run(g, cam)
    assert L > 0
    allow = reference_allowance(o)
    assert allow["counts"]["order_pixels"] > 0
    assert allow["owners"].all() and (allow["flags"] & 2).all()
