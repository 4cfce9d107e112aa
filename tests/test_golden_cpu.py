"""CPU: the oracle reproduces the committed golden fixtures (tests/golden/make_golden.py), the
conference stand-in file is the pinned one, and the C-ABI library loads and exports every
symbol include/*.h declares (no compute without a GPU)."""
import ctypes
import hashlib
import json
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO

GOLDEN = os.path.join(REPO, "tests", "golden")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


with open(os.path.join(GOLDEN, "golden.json")) as _f:
    GOLDEN_CASES = sorted(k for k, v in json.load(_f).items() if isinstance(v, dict))


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_oracle_matches_golden(oracle_mod, golden, name):
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    o = mg.oracle_for(mg.CASES[name])
    bm, rays = o.render(threads=min(8, os.cpu_count() or 1))
    k, i, t = o.primary_hits()
    g = golden[name]
    assert rays == g["rays"]
    assert sha(bm) == g["bitmap_sha256"]
    assert sha(np.stack([k, i, t.view(np.int32)])) == g["hits_sha256"]
    assert o.counts() == g["counts"]


def test_cornell_c1_bitmap_fixture(oracle_mod):
    bm, _ = oracle_mod.Oracle(256, 256, 1, 0).render(threads=4)
    ref = np.load(os.path.join(GOLDEN, "cornell256_whitted.npz"))["bitmap"]
    assert np.array_equal(bm, ref)
    assert len(np.unique(bm)) > 1  # ShaderTestEngine.cpp:46-48: the image is not uniform


def test_conference_standin_is_pinned(golden):
    from mobileraytracer_amd import scenes
    obj = scenes.conference()[0]
    if not scenes.is_standin(obj):
        pytest.skip("a real conference.obj was supplied")
    assert scenes.file_sha256(obj) == golden["conference_standin_obj_sha256"]


def test_conference_flat_standin_is_pinned(golden):
    """The flat-geometry stand-in (scenes.conference_flat): pinned bytes, and the counts the
    reference pins for the real Conference (scripts/test/docker/dockerfile.sh:118-119: 331,179
    triangles, 2 lights), read back through the product's own loader and BVH build (host only)."""
    import mobileraytracer_amd as m
    from mobileraytracer_amd import scenes
    obj, mtl, cam = scenes.conference_flat()
    assert scenes.file_sha256(obj) == golden["conference_flat_standin_obj_sha256"]
    cfg = m.Config(width=64, height=64, shader=1, sceneIndex=-1, objFilePath=obj, mtlFilePath=mtl, camFilePath=cam)
    _, _, cnt, order = m.triangle_bvh(cfg)
    assert len(order) == scenes.CONFERENCE_TRIANGLES
    assert cnt.sum() == scenes.CONFERENCE_TRIANGLES
    faces = light = 0
    group = None
    with open(obj) as f:
        for line in f:
            if line.startswith("usemtl "):
                group = line.split()[1]
            elif line.startswith("f "):
                faces += 1
                light += group == "light"
    assert faces - light == scenes.CONFERENCE_TRIANGLES and light == scenes.CONFERENCE_LIGHTS


def _declared_symbols():
    names = set()
    for hdr in ("mobilert_amd.h", "mobilert_amd.hpp"):
        with open(os.path.join(REPO, "include", hdr)) as f:
            src = f.read()
        names |= set(re.findall(r"\b(mrt_[a-z_]+)\s*\(", src))
        names |= set(re.findall(r'extern "C" void (\w+)\(', src))
    return names


def test_library_exports_every_declared_symbol(native_lib_path):
    out = subprocess.run(["nm", "-D", "--defined-only", native_lib_path], check=True, capture_output=True,
                         text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    declared = _declared_symbols()
    assert {"RayTrace", "stopRender", "mrt_create", "mrt_render_frame"} <= declared
    missing = declared - exported
    assert not missing, missing
    from mobileraytracer_amd import _native
    assert set(_native.EXPORTED_SYMBOLS) <= exported


def test_library_built_from_these_sources(native_lib_path):
    """The in-tree library (the one the GPU box loads) was built from the sources in the tree."""
    from mobileraytracer_amd import _native
    if os.environ.get("MOBILERT_LIB"):
        pytest.skip("another build was requested")
    assert _native.build_is_current(_native.load_library(native_lib_path)), "stale libmobilert_amd.so: run make"


def test_library_loads_without_gpu(native_lib_path):
    from mobileraytracer_amd import _native
    lib = _native.load_library(native_lib_path)
    assert lib.mrt_last_error() is not None


def test_setters_reject_null_arguments(native_lib_path):
    """mrt_set_camera / mrt_set_max_point / mrt_set_pixel_sampler return -1 with mrt_last_error set
    on a NULL renderer or vector (no GPU needed: the checks come before any device work)."""
    from mobileraytracer_amd import _native
    lib = _native.load_library(native_lib_path)
    v = (ctypes.c_float * 3)(0.0, 0.0, 1.0)
    assert lib.mrt_set_camera(None, 0, v, v, v, 45.0, 45.0) == -1
    assert b"null" in lib.mrt_last_error()
    assert lib.mrt_set_max_point(None, v) == -1
    assert lib.mrt_set_max_point(None, None) == -1
    assert lib.mrt_set_pixel_sampler(None, 0, 0.5) == -1


def test_ctypes_layouts_match_header(tmp_path):
    """The ctypes mirror of mrt_config / mrt_scene_info / mrt_frame_stats matches the C header."""
    from mobileraytracer_amd import _native
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "mobilert_amd.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu", sizeof(mrt_config), sizeof(mrt_scene_info),'
                   ' sizeof(mrt_frame_stats), offsetof(mrt_config, maxDepth));return 0;}')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    sizes = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert sizes == [ctypes.sizeof(_native.MrtConfig), ctypes.sizeof(_native.MrtSceneInfo),
                     ctypes.sizeof(_native.MrtFrameStats), _native.MrtConfig.maxDepth.offset]


def test_library_built_for_gfx950(native_lib_path):
    out = subprocess.run(["strings", native_lib_path], capture_output=True, text=True, check=True)
    assert "amdgcn-amd-amdhsa--gfx950" in out.stdout


def _bvh_walk(boxes, off, cnt):
    """Nodes in left-first depth-first order: (box bytes, numPrimitives, leaf offset)."""
    out, st = [], [0]
    while st:
        i = st.pop()
        leaf = cnt[i] > 0 or len(cnt) == 1
        out.append((boxes[i].tobytes(), int(cnt[i]), int(off[i]) if leaf else -1))
        if not leaf:
            st += [int(off[i]) + 1, int(off[i])]
    return out


@pytest.mark.parametrize("scene", ["conference", "water", "teapot", 0, 1, 2, 3])
def test_parallel_bvh_build_equals_reference_build(oracle_mod, scene):
    """The renderer's multi-threaded BVH build (f1) yields the reference build's tree: same
    boxes, leaves and primitive order as the oracle's serial restatement of BVH.hpp:161-283."""
    import mobileraytracer_amd as m
    from mobileraytracer_amd import scenes
    cfg = m.Config(width=64, height=64, sceneIndex=scene if isinstance(scene, int) else -1)
    if not isinstance(scene, int):
        cfg.objFilePath, cfg.mtlFilePath, cfg.camFilePath = {
            "conference": scenes.conference, "water": scenes.cornell_water, "teapot": scenes.teapot}[scene]()
    boxes, off, cnt, order = m.triangle_bvh(cfg)
    o = oracle_mod.Oracle(64, 64, 1, cfg.sceneIndex, obj=cfg.objFilePath, mtl=cfg.mtlFilePath, cam=cfg.camFilePath)
    oboxes, ooff, ocnt, oorder = o.triangle_bvh()
    assert _bvh_walk(boxes, off, cnt) == _bvh_walk(oboxes, ooff, ocnt)
    assert np.array_equal(order, oorder)


def test_hemisphere_trig_table_matches_oracle(oracle_mod):
    """The renderer's host table of cos / sin(two_pi * r1) (Shader.cpp:206-212) equals, bit for
    bit, the oracle's own libm evaluation of every shader-table entry; both tables equal too."""
    import mobileraytracer_amd as m
    a, b, t = m.sample_tables()
    assert np.array_equal(a, oracle_mod.table(0x4D525400)) and np.array_equal(b, oracle_mod.table(0x4D525401))
    ot = oracle_mod.hemisphere_trig().reshape(-1, 2)
    assert np.array_equal(t.view(np.int32), ot.view(np.int32))
    ph = np.float32(2 * np.pi) * a
    assert np.abs(t[:, 0] - np.cos(ph.astype(np.float64))).max() < 1e-6
