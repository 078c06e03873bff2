#!/usr/bin/env python3
"""tools/ab_schedule.py — interleaved in-process A/B of render-kernel schedules on one device.

  python3 tools/ab_schedule.py [--rounds 3] [--variants 0:48,0:32,1:0] [--spp 500]

Each variant "S:B:L" = schedule S (include/rtgpu.h RTG_RENDER_SCHEDULE) with shade batch B (64ths)
and leaf batch L (lanes); 0 = library default. Renders BASELINE config 2 (book-1, 1920x1080, depth 50) and reports the
kernel time (HIP events) per variant per round plus the median Mrays/s; checks that every
variant produced the identical frame.
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="0:48,0:32,0:56,0:64,1:0")
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--grid", type=int, default=11)
    ap.add_argument("--scene", default="bouncing_spheres")
    ap.add_argument("--bvh", default="sah")
    a = ap.parse_args()
    import torch

    import rtgpu

    lib = rtgpu.Library()
    bvh = {"sah": rtgpu.RTG_BVH_SAH, "median": rtgpu.RTG_BVH_MEDIAN, "sah2": 2}[a.bvh]
    s = rtgpu.SceneLibrary().build(a.scene, grid=a.grid, image_width=a.width, aspect_ratio=16.0 / 9.0,
                                   spp=a.spp, max_depth=50, bvh_mode=bvh)
    cam = s.camera
    H = lib.camera_resolve(cam).image_height
    ds = lib.scene_create(s.desc)
    out = torch.zeros((H, a.width, 3), device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    variants = [tuple(int(x) for x in (v.split(":") + ["0", "0"])[:3]) for v in a.variants.split(",")]
    times = {v: [] for v in variants}
    frames = {}
    segs = {}
    for r in range(a.rounds):
        for v in variants:
            sched, batch, leaf = v
            flags = rtgpu.RTG_RENDER_OUT_DEVICE | (sched << 8) | (batch << 16) | (leaf << 24)
            job = rtgpu.rtg_render_desc(0x5EED, 0, 1, 0, flags, stream)
            st = rtgpu.rtg_render_stats()
            lib.check("rtg_render", lib.lib.rtg_render(ds.handle, rtgpu.C.byref(cam), rtgpu.C.byref(job),
                                                        out.data_ptr(), rtgpu.C.byref(st)))
            times[v].append(st.kernel_ms)
            segs[v] = st.segments
            if r == 0:
                frames[v] = out.cpu().numpy().copy()
    base = frames[variants[0]]
    res = {}
    for v in variants:
        med = float(np.median(times[v]))
        res[":".join(str(x) for x in v)] = {"kernel_ms": [round(t, 2) for t in times[v]], "median_ms": round(med, 2),
                                 "mrays_per_s": round(segs[v] / med / 1e3, 1),
                                 "identical_frame": bool(np.array_equal(frames[v], base))}
    print(json.dumps({"scene": a.scene, "grid": a.grid, "spp": a.spp, "width": a.width, "results": res},
                     indent=1))


if __name__ == "__main__":
    main()
