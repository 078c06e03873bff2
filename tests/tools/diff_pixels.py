#!/usr/bin/env python3
"""tests/tools/diff_pixels.py — which of two library builds is right where their frames differ.

  python3 tests/tools/diff_pixels.py --libs new=PATH,old=PATH [--scene S --grid G --width W --height H --spp N
                               --depth D --threads T]

Renders one frame with each build (same box, same seed), lists the pixels where the two differ, renders
the rows that hold them with cpu_ref32 (the oracle, test infrastructure: this tool is a checker) and reports
for every differing pixel which build equals the oracle bit for bit. Used for the round-5 culling change
(DESIGN.md §4 "conservative culling"): a frame change must be the new build agreeing with the oracle."""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "raytracing-practice_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--scene", default="bouncing_spheres")
    ap.add_argument("--grid", type=int, default=11)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--max-rows", type=int, default=24)
    a = ap.parse_args()
    import rtgpu
    from oracle_bind import Oracle

    libs = {}
    for item in a.libs.split(","):
        name, path = item.split("=", 1)
        libs[name] = rtgpu.Library(path if os.path.isabs(path) else os.path.join(REPO, path))
    s = rtgpu.SceneLibrary().build(a.scene, grid=a.grid, image_width=a.width,
                                   aspect_ratio=(a.width / a.height) if a.height else 16.0 / 9.0,
                                   spp=a.spp, max_depth=a.depth)
    cam = s.camera
    frames, segs = {}, {}
    for name, L in libs.items():
        ds = L.scene_create(s.desc)
        frames[name], st = ds.render_host(cam)
        segs[name] = int(st.segments)
        ds.close()
    names = list(libs)
    diff = np.any(frames[names[0]] != frames[names[1]], axis=-1)
    ys, xs = np.nonzero(diff)
    rows = sorted(set(int(y) for y in ys))[: a.max_rows]
    orc = Oracle()
    verdict = []
    for y in rows:
        ref, _ = orc.render_f32(s.desc, cam, row_begin=y, row_count=1, threads=a.threads)
        for x in xs[ys == y]:
            verdict.append({"pixel": [int(x), y],
                            **{n: bool(np.array_equal(frames[n][y, x], ref[0, x])) for n in names}})
    out = {"scene": a.scene, "grid": a.grid, "width": a.width, "spp": a.spp, "depth": a.depth,
           "segments": segs, "differing_pixels": int(diff.sum()), "rows_checked": len(rows),
           "matches_oracle": {n: sum(v[n] for v in verdict) for n in names}, "pixels": verdict}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
