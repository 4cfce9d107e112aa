"""The reference's desktop C-ABI from C++: tests/cabi/raytrace_cabi.cpp includes
include/mobilert_amd.hpp, fills MobileRT::Config as the reference's engine tests do
(app/Unit_Testing/engine/ShaderTestEngine.cpp:8-24: 30x30, 3 threads) and calls
RayTrace(config, false) for shaders 0-4, accelerators 1-3 and both cameras, then
RayTrace(config, true) + stopRender().  Every bitmap is compared with the oracle, bit for bit.
The binary is built in-tree by __graft_entry__.build() (make -C tests/cabi)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

BIN = os.path.join(REPO, "tests", "cabi", "build", "raytrace_cabi")
CASES = {  # name: (sceneIndex, shader, accelerator, OBJ)
    "noshadows_water": (-1, 0, 3, True), "whitted_water": (-1, 1, 3, True), "pathtracer_water": (-1, 2, 3, True),
    "depthmap_water": (-1, 3, 3, True), "diffuse_water": (-1, 4, 3, True), "naive_water": (-1, 1, 1, True),
    "grid_water": (-1, 1, 2, True), "bvh_water": (-1, 1, 3, True), "orthographic_spheres": (1, 1, 3, False),
    "perspective_cornell": (0, 1, 3, False), "pathtracer_cornell": (0, 2, 3, False),
}


@pytest.fixture(scope="module")
def cabi_run(tmp_path_factory):
    from mobileraytracer_amd import scenes
    assert os.path.exists(BIN), "build it first: python -c 'import __graft_entry__ as g; g.build()'"
    out = tmp_path_factory.mktemp("cabi")
    env = dict(os.environ)
    env.pop("MOBILERT_MAX_DEPTH", None)
    p = subprocess.run([BIN, str(out), *scenes.cornell_water()], capture_output=True, text=True, timeout=180, env=env)
    return p, out


def test_raytrace_cpp_driver_runs(cabi_run):
    p, _ = cabi_run
    assert p.returncode == 0, p.stdout + p.stderr
    assert "TRIANGLES = 7086" in p.stdout and "LIGHTS = 2" in p.stdout  # C_wrapper.cpp:199-202 summary
    assert "Total Millions rays per second" in p.stdout
    assert "case async_stop: rendered and stopped" in p.stdout


@pytest.mark.parametrize("name", sorted(CASES))
def test_raytrace_cpp_bitmaps_match_oracle(oracle_mod, cabi_run, name):
    from mobileraytracer_amd import scenes
    _, out = cabi_run
    scene, shader, acc, obj = CASES[name]
    bm = np.fromfile(os.path.join(out, name + ".bin"), np.int32)
    paths = scenes.cornell_water() if obj else ("", "", "")
    o = oracle_mod.Oracle(30, 30, shader, scene, 1, 1, 6, obj=paths[0], mtl=paths[1], cam=paths[2], accelerator=acc)
    ref = np.zeros(30 * 30, np.int32)
    o.render(ref, threads=3)
    o.close()
    # 30 % 16 != 0: the reference's tile formula writes some pixels twice (DESIGN.md deviation 6)
    from test_gpu_parity import coverage
    once = coverage(30, 30) == 1
    assert np.array_equal(bm[once], ref[once]), int((bm[once] != ref[once]).sum())


def test_raytrace_async_stop_partial_frame(cabi_run):
    _, out = cabi_run
    bm = np.fromfile(os.path.join(out, "async_stop.bin"), np.int32)
    assert len(np.unique(bm)) > 1  # the samples done before stopRender() reached config.bitmap
