#!/usr/bin/env python3
"""tools/stack_probe.py — render with a forced traversal-stack depth (RTG_STACK) and report the
kernel time and how many waves overflowed (schedule experiment; the frame of an overflowing run
is not valid and rtg_render reports the overflow as an error)."""
import argparse
import ctypes as C
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
    ap.add_argument("--spp", type=int, default=100)
    ap.add_argument("--stacks", default="0,16,32")
    a = ap.parse_args()
    import rtgpu

    lib = rtgpu.Library()
    s = rtgpu.SceneLibrary().build(a.scene, grid=a.grid, image_width=a.width, aspect_ratio=16.0 / 9.0,
                                   spp=a.spp, max_depth=50)
    ds = lib.scene_create(s.desc)
    H = lib.camera_resolve(s.camera).image_height
    buf = np.zeros((H, a.width, 3), dtype=np.float32)
    out = {"scene": a.scene, "grid": a.grid, "stack_default": ds.info().stack_depth, "runs": {}}
    for st_depth in [int(x) for x in a.stacks.split(",")]:
        if st_depth:
            os.environ["RTG_STACK"] = str(st_depth)
        else:
            os.environ.pop("RTG_STACK", None)
        job = rtgpu.rtg_render_desc(0x5EED, 0, 1, 0, 0, None)
        st = rtgpu.rtg_render_stats()
        rc = lib.lib.rtg_render(ds.handle, C.byref(s.camera), C.byref(job), buf.ctypes.data, C.byref(st))
        out["runs"][st_depth or "default"] = {"rc": rc, "kernel_ms": round(st.kernel_ms, 2),
                                              "msg": (lib.lib.rtg_last_error() or b"").decode() if rc else ""}
    os.environ.pop("RTG_STACK", None)
    print(json.dumps(out))
    ds.close()


if __name__ == "__main__":
    main()
