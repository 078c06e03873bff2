#!/usr/bin/env python3
"""tools/bvh_compare.py — render one frame with two BVH builds of the same scene and compare.

  python3 tools/bvh_compare.py [--grid 500] [--width 3840] [--spp 8] [--modes sah,gpu]

The closest hit does not depend on the tree, so the frames may differ only where two primitives
are hit at exactly the same distance (hazard H9); a larger difference means a box that culls a
primitive it contains.
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-practice_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="bouncing_spheres")
    ap.add_argument("--grid", type=int, default=500)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--modes", default="sah,gpu")
    ap.add_argument("--lib", default=None)
    a = ap.parse_args()
    import rtgpu

    lib = rtgpu.Library(a.lib)
    codes = {"sah": rtgpu.RTG_BVH_SAH, "median": rtgpu.RTG_BVH_MEDIAN, "gpu": rtgpu.RTG_BVH_GPU}
    frames, info = {}, {}
    import ctypes as C
    for m0 in a.modes.split(","):
        m, _, sched = m0.partition(":")  # "gpu:4" = schedule 4 (plain grid)
        s = rtgpu.SceneLibrary().build(a.scene, grid=a.grid, image_width=a.width, aspect_ratio=16.0 / 9.0,
                                       spp=a.spp, max_depth=a.depth, bvh_mode=codes[m], rand_seed=1)
        ds = lib.scene_create(s.desc)
        H = lib.camera_resolve(s.camera).image_height
        img = np.zeros((H, a.width, 3), dtype=np.float32)
        job = rtgpu.rtg_render_desc(rtgpu.DEFAULT_SEED, 0, 1, 0, int(sched or 0) << 8, None)
        st = rtgpu.rtg_render_stats()
        lib.check("rtg_render", lib.lib.rtg_render(ds.handle, C.byref(s.camera), C.byref(job), img.ctypes.data,
                                                    C.byref(st)))
        frames[m0] = img
        info[m0] = {"segments": int(st.segments), "nodes": int(ds.info().num_nodes)}
        ds.close()
    ms = list(frames)
    base = frames[ms[0]]
    for m in ms[1:]:
        diff = np.any(frames[m] != base, axis=-1)
        info[m]["equal_pixel_frac"] = float(1.0 - diff.mean())
        info[m]["rmse"] = float(np.sqrt(np.mean((frames[m].astype(np.float64) - base) ** 2)))
        ys, xs = np.nonzero(diff)
        info[m]["first_diffs"] = [[int(y), int(x), base[y, x].tolist(), frames[m][y, x].tolist()]
                                  for y, x in list(zip(ys, xs))[:3]]
    print(json.dumps(info))


if __name__ == "__main__":
    main()
