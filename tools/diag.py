#!/usr/bin/env python3
"""tools/diag.py — schedule diagnostics of the default kernel on one config (COUNT mode)."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-practice_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="bouncing_spheres")
    ap.add_argument("--grid", type=int, default=11)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--batches", default="48")
    ap.add_argument("--leaf", type=int, default=0)
    ap.add_argument("--schedule", type=int, default=0)
    ap.add_argument("--lib", default=None, help="librtgpu.so to load (default: the in-tree build)")
    ap.add_argument("--depth", type=int, default=50)
    a = ap.parse_args()
    import rtgpu

    lib = rtgpu.Library(os.path.join(REPO, a.lib) if a.lib else None)
    s = rtgpu.SceneLibrary().build(a.scene, grid=a.grid, image_width=a.width, aspect_ratio=16.0 / 9.0,
                                   spp=a.spp, max_depth=a.depth)
    ds = lib.scene_create(s.desc)
    ds.prepare(s.camera)  # per-camera setup the bench does too (the hot treelet of schedule 5)
    out = {}
    out["lib"] = lib.path
    for b in [int(x) for x in a.batches.split(",")]:
        import ctypes as C
        import numpy as np

        H = lib.camera_resolve(s.camera).image_height
        buf = np.zeros((H, a.width, 3), dtype=np.float32)
        job = rtgpu.rtg_render_desc(0x5EED, 0, 1, 0, rtgpu.RTG_RENDER_COUNT | (b << 16) | (a.leaf << 24)
                                    | (a.schedule << 8), None)
        st = rtgpu.rtg_render_stats()
        lib.check("rtg_render", lib.lib.rtg_render(ds.handle, C.byref(s.camera), C.byref(job),
                                                    buf.ctypes.data, C.byref(st)))
        d = list(st.diag)
        out[b] = {"kernel_ms": round(st.kernel_ms, 1), "segments": st.segments,
                  "trav_trips": d[0], "trav_lane_util": d[1] / (64 * d[0]),
                  "idle_done_frac": d[2] / (64 * d[0]), "shade_trips": d[3],
                  "shade_lane_util": d[4] / (64 * d[3]),
                  "steps_per_segment": d[1] / st.segments,
                  "box_tests_per_segment": st.box_tests / st.segments,
                  "trav_cycles_frac": d[5] / max(1, d[5] + d[6]),
                  "cycles_per_trav_trip": d[5] / max(1, d[0]),
                  "cycles_per_shade_trip": d[6] / max(1, d[3]),
                  "leaf_trip_frac": d[7] / max(1, d[0]),
                  "leaf_cycles_frac_of_trav": d[8] / max(1, d[5]),
                  "node_trip_lane_util": d[9] / (64 * max(1, d[0] - d[7])),
                  "leaf_trip_lane_util": d[10] / (64 * max(1, d[7])),
                  "node_steps_per_segment": d[9] / st.segments,
                  "leaf_steps_per_segment": d[10] / st.segments,
                  "shade_split_scatter_end": [round(d[k] / max(1, d[6]), 3) for k in (11, 12)],
                  # wave cycles of the whole loop: traversal, shading, and the restart between them
                  # (unit hand-out, camera rays of fresh samples, trav_begin + occluder test)
                  "cycle_split_trav_shade_handout_camera_begin": [
                      round(d[k] / max(1, d[5] + d[6] + d[13] + d[14] + d[15]), 3) for k in (5, 6, 13, 14, 15)]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
