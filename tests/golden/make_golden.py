"""Regenerates the committed golden fixtures from the CPU oracle.

    python tests/golden/make_golden.py

The oracle is itself pinned by the reference's unit-test KATs (tests/test_oracle_kat.py).
Fixtures: SHA-256 of every output array + ray counts (golden.json), and the full Cornell
256x256 Whitted bitmap (cornell256_whitted.npz, config C1) so a drifting oracle is caught.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import oracle as O  # noqa: E402
from mobileraytracer_amd import scenes  # noqa: E402


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# name -> oracle kwargs; "scene" = fixture name resolved at run time
CASES = {
    "cornell256_whitted": dict(width=256, height=256, shader=1, sceneIndex=0),
    "cornell512_whitted": dict(width=512, height=512, shader=1, sceneIndex=0),
    "cornell256_pt4": dict(width=256, height=256, shader=2, sceneIndex=0, samplesPixel=4),
    "water128_whitted": dict(width=128, height=128, shader=1, sceneIndex=-1, scene="water"),
    "water128_pt4": dict(width=128, height=128, shader=2, sceneIndex=-1, samplesPixel=4, scene="water"),
    "teapot128_whitted": dict(width=128, height=128, shader=1, sceneIndex=-1, scene="teapot"),
    # the teapot's material is textured (map_Kd default.png): texel Kd, shared-Kd replay
    "teapot128_pt4": dict(width=128, height=128, shader=2, sceneIndex=-1, samplesPixel=4, scene="teapot"),
    "teapot128_diffuse": dict(width=128, height=128, shader=4, sceneIndex=-1, scene="teapot"),
    "conference96_whitted": dict(width=96, height=96, shader=1, sceneIndex=-1, scene="conference"),
    "conference96_pt4": dict(width=96, height=96, shader=2, sceneIndex=-1, samplesPixel=4, maxDepth=5,
                             scene="conference"),
    # the other built-in scenes (C_wrapper.cpp:76-99) and shaders (C_wrapper.cpp:153-193)
    "spheres128_whitted": dict(width=128, height=128, shader=1, sceneIndex=1),
    "spheres128_depthmap": dict(width=128, height=128, shader=3, sceneIndex=1),
    "cornell2_128_whitted": dict(width=128, height=128, shader=1, sceneIndex=2),
    "cornell2_128_pt4": dict(width=128, height=128, shader=2, sceneIndex=2, samplesPixel=4),
    "spheres2_128_whitted": dict(width=128, height=128, shader=1, sceneIndex=3),
    "spheres2_128_noshadows": dict(width=128, height=128, shader=0, sceneIndex=3),
    "cornell128_depthmap": dict(width=128, height=128, shader=3, sceneIndex=0),
    "cornell128_diffuse": dict(width=128, height=128, shader=4, sceneIndex=0),
    "cornell2_128_noshadows_spl2": dict(width=128, height=128, shader=5, sceneIndex=2, samplesLight=2, samplesPixel=2),
    "conference96_noshadows": dict(width=96, height=96, shader=0, sceneIndex=-1, scene="conference"),
    "conference96_diffuse": dict(width=96, height=96, shader=4, sceneIndex=-1, scene="conference"),
}


def oracle_for(case):
    kw = dict(case)
    scene = kw.pop("scene", None)
    if scene == "water":
        kw["obj"], kw["mtl"], kw["cam"] = scenes.cornell_water()
    elif scene == "teapot":
        kw["obj"], kw["mtl"], kw["cam"] = scenes.teapot()
    elif scene == "conference":
        kw["obj"], kw["mtl"], kw["cam"] = scenes.conference()
    return O.Oracle(**kw)


def main():
    out = {}
    for name, case in CASES.items():
        o = oracle_for(case)
        bm, rays = o.render(threads=os.cpu_count() or 1)
        k, i, t = o.primary_hits()
        out[name] = dict(bitmap_sha256=sha(bm), rays=rays, hits_sha256=sha(np.stack([k, i, t.view(np.int32)])),
                         counts=o.counts())
        if name == "cornell256_whitted":
            np.savez_compressed(os.path.join(HERE, "cornell256_whitted.npz"), bitmap=bm)
        o.close()
        print(name, out[name]["rays"])
    conf = scenes.conference()[0]
    out["conference_standin_obj_sha256"] = scenes.file_sha256(conf) if scenes.is_standin(conf) else None
    out["conference_flat_standin_obj_sha256"] = scenes.file_sha256(scenes.conference_flat()[0])
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
