#!/usr/bin/env python3
"""tests/tools/full_frame_check.py — one benchmark frame at its full size AND full spp, every pixel against the
oracle (a checker: cpu_ref32 from oracle/, test infrastructure).

  python3 tests/tools/full_frame_check.py [--scene S --grid G --width W --height H --spp N --depth D]
                                    [--threads T] [--block R] [--rows-from A --rows-to B]

Renders the frame once with the library, then renders it with cpu_ref32 in blocks of R rows on T host
threads (a progress line per block), and reports the differing pixels, the RMSE and the segment counts.
The GPU tests compare the full frames at 1-2 spp and the bench lines sampled rows at full spp; this is the
whole frame at full spp (minutes of CPU time per config, so a tool run on the GPU box, not a test)."""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "raytracing-practice_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="bouncing_spheres")
    ap.add_argument("--grid", type=int, default=11)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--block", type=int, default=32)
    ap.add_argument("--rows-from", type=int, default=0)
    ap.add_argument("--rows-to", type=int, default=-1)
    ap.add_argument("--prepare", action="store_true",
                    help="rtg_scene_prepare the camera first (hot treelet, tile order), as bench.py does")
    a = ap.parse_args()
    import rtgpu
    from oracle_bind import Oracle

    lib = rtgpu.Library()
    s = rtgpu.SceneLibrary().build(a.scene, grid=a.grid, image_width=a.width,
                                   aspect_ratio=(a.width / a.height) if a.height else 16.0 / 9.0,
                                   spp=a.spp, max_depth=a.depth)
    cam = s.camera
    ds = lib.scene_create(s.desc)
    if a.prepare:
        ds.prepare(cam)
    t0 = time.time()
    gpu, st = ds.render_host(cam)
    tile_order = int(st.tile_order)
    ds.close()
    H = gpu.shape[0]
    tie_rule = None
    if s.desc.tie_rank:  # the same frame with list-order ranks: the pixels the bvh_node tie order decides
        d_list = rtgpu.rtg_scene_desc.from_buffer_copy(s.desc)
        d_list.tie_rank = None
        ds = lib.scene_create(d_list)
        g_list, st_list = ds.render_host(cam)
        ds.close()
        dl = np.any(gpu != g_list, axis=-1)
        yl, xl = np.nonzero(dl)
        tie_rule = {"pixels_differing_from_list_order": int(dl.sum()),
                    "segments_list_order": int(st_list.segments),
                    "where": [[int(x), int(y)] for y, x in zip(yl[:64], xl[:64])]}
    r1 = H if a.rows_to < 0 else min(H, a.rows_to)
    print(f"gpu frame {gpu.shape} in {time.time() - t0:.1f} s, segments {st.segments}", flush=True)
    orc = Oracle()
    ref = np.zeros_like(gpu[a.rows_from:r1])
    segs = 0
    t0 = time.time()
    for y in range(a.rows_from, r1, a.block):
        n = min(a.block, r1 - y)
        part, sg = orc.render_f32(s.desc, cam, row_begin=y, row_count=n, threads=a.threads)
        ref[y - a.rows_from:y - a.rows_from + n] = part
        segs += sg
        print(f"oracle rows {y}..{y + n - 1} of {H}: {time.time() - t0:.0f} s", flush=True)
    g = gpu[a.rows_from:r1]
    diff = np.any(g != ref, axis=-1)
    ys, xs = np.nonzero(diff)
    out = {"scene": a.scene, "grid": a.grid, "width": a.width, "height": H, "spp": a.spp, "depth": a.depth,
           "rows": [a.rows_from, r1], "pixels": int(diff.size), "differing_pixels": int(diff.sum()),
           "identical_frac": float(1.0 - diff.mean()),
           "rmse": float(np.sqrt(np.mean((g.astype(np.float64) - ref) ** 2))),
           "max_abs": float(np.max(np.abs(g.astype(np.float64) - ref))) if g.size else 0.0,
           "oracle_segments": int(segs),
           "gpu_segments_whole_frame": int(st.segments), "gpu_tile_order": tile_order,
           "oracle_seconds": round(time.time() - t0, 1), "threads": a.threads,
           "differing": [[int(x), int(y) + a.rows_from] for y, x in zip(ys[:64], xs[:64])]}
    if tie_rule is not None:
        out["tie_rule"] = tie_rule
    if a.rows_from == 0 and r1 == H:
        out["segments_equal"] = int(segs) == int(st.segments)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
