#!/usr/bin/env python3
"""tools/wave_trace.py — per-wave timeline of one render (schedule analysis).

  python3 tools/wave_trace.py [--scene S] [--schedule N] [--lib path] [--spp K] ...

Runs one render with RTG_WAVE_TRACE set (librtgpu then records, per wave, s_memrealtime at start and
end and the pixels it finished) and prints the launch's occupancy profile: how many waves are still
alive at each tenth of the kernel, the start/end spread and the pixels-per-wave distribution.
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-practice_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="bouncing_spheres")
    ap.add_argument("--grid", type=int, default=11)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--schedule", type=int, default=0)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--shard-of", type=int, default=1, help="render rank 0's interleaved shard of N ranks")
    ap.add_argument("--prepare", action="store_true", help="rtg_scene_prepare the shard first (tile order)")
    a = ap.parse_args()
    import ctypes as C

    import rtgpu

    lib = rtgpu.Library(os.path.join(REPO, a.lib) if a.lib else None)
    s = rtgpu.SceneLibrary().build(a.scene, grid=a.grid, image_width=a.width, aspect_ratio=16.0 / 9.0,
                                   spp=a.spp, max_depth=a.depth)
    path = os.path.join(tempfile.gettempdir(), f"rtg_trace_{os.getpid()}.bin")
    os.environ["RTG_WAVE_TRACE"] = path  # knobs are read once, when the scene is created
    ds = lib.scene_create(s.desc)
    H = lib.camera_resolve(s.camera).image_height
    b, stride, cnt = rtgpu.shard_rows(H, 0, a.shard_of)
    if a.prepare:
        ds.prepare(s.camera, row_begin=b, row_stride=stride, row_count=cnt if a.shard_of > 1 else 0)
    buf = np.zeros((max(cnt, 1), a.width, 3), dtype=np.float32)
    job = rtgpu.rtg_render_desc(0x5EED, b, stride, cnt if a.shard_of > 1 else 0, a.schedule << 8, None)
    st = rtgpu.rtg_render_stats()
    lib.check("rtg_render", lib.lib.rtg_render(ds.handle, C.byref(s.camera), C.byref(job), buf.ctypes.data,
                                                C.byref(st)))
    del os.environ["RTG_WAVE_TRACE"]
    t = np.fromfile(path, dtype=np.uint64).reshape(-1, 4)
    os.remove(path)
    t = t[t[:, 1] > 0]
    t0, t1 = t[:, 0].astype(np.float64), t[:, 1].astype(np.float64)
    base, span = t0.min(), t1.max() - t0.min()
    tick_ns = 10.0  # s_memrealtime runs at 100 MHz
    grid = np.linspace(base, base + span, 11)
    alive = [int(np.sum((t0 <= g) & (t1 > g))) for g in grid[:-1]]
    out = {"scene": a.scene, "shard_of": a.shard_of, "schedule": a.schedule, "tile_order": int(st.tile_order),
           "kernel_ms": round(st.kernel_ms, 2), "waves": int(len(t)),
           "span_ms": round(span * tick_ns / 1e6, 2),
           "alive_at_tenths": alive,
           "start_ms_pcts": [round((np.percentile(t0, q) - base) * tick_ns / 1e6, 2) for q in (0, 50, 90, 100)],
           "end_ms_pcts": [round((np.percentile(t1, q) - base) * tick_ns / 1e6, 2) for q in (0, 10, 50, 90, 100)],
           "pixels_per_wave_pcts": [int(np.percentile(t[:, 2], q)) for q in (0, 10, 50, 90, 100)],
           "busy_frac": round(float(np.sum(t1 - t0)) / (span * max(alive)), 4)}
    print(json.dumps(out))
    ds.close()


if __name__ == "__main__":
    main()
