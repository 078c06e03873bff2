#!/usr/bin/env python3
"""tests/tools/near_tie_probe.py — pixels where a build's near-tie frame (tests/tie_scene.py near_tie_scene)
differs from cpu_ref32, over camera heights, competitors and BVH builders; for choosing a test scene that
the pre-round-5 culling fails (a negative control) and the current one passes."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "raytracing-practice_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import rtgpu
    from oracle_bind import Oracle
    from tie_scene import GREEN, colour_counts, near_tie_scene

    libs = {}
    for item in sys.argv[1].split(","):
        name, path = item.split("=", 1)
        libs[name] = rtgpu.Library(path if os.path.isabs(path) else os.path.join(REPO, path))
    orc = Oracle()
    res = []
    for h in [float(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "2,20,200,1000").split(",")]:
        for comp in ("quad", "sphere"):
            for bvh in (rtgpu.RTG_BVH_SAH, rtgpu.RTG_BVH_GPU, rtgpu.RTG_BVH_MEDIAN):
                d, cam = near_tie_scene(bvh, comp, width=96, cam_height=h)
                o, osegs = orc.render_f32(d, cam, threads=16)
                row = {"h": h, "comp": comp, "bvh": bvh, "oracle_green": colour_counts(o)[GREEN]}
                for name, L in libs.items():
                    ds = L.scene_create(d)
                    g, st = ds.render_host(cam)
                    ds.close()
                    row[name] = int(np.sum(np.any(g != o, axis=-1)))
                res.append(row)
                print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
