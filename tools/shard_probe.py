#!/usr/bin/env python3
"""tools/shard_probe.py — the per-rank work of an N-GPU frame, measured on one GPU.

Renders the interleaved row shards of N = 1, 2, 4, 8 ranks one after another on one device (the
same shards bench.py gives each rank) and reports, per N, the kernel time of every shard (HIP
events) and the host wall time of a render_device call; max-over-shards approximates the N-GPU
frame time, so N * max / full-frame time is the strong-scaling efficiency of the kernel schedule
(without the RCCL gather, which bench.py adds).

  python3 tools/shard_probe.py [--config 2] [--reps 2] [--ns 1,2,4,8]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-practice_amd", "python"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--lib", default="", help="librtgpu.so to load (default: the in-tree build)")
    ap.add_argument("--prepare", action="store_true",
                    help="rtg_scene_prepare each shard before its renders (hot treelet, tile order), as bench.py does")
    ap.add_argument("--layout", default="strided", choices=["strided", "contig"],
                    help="contig: rank r renders one block of ceil(H/N) rows (coherence probe; unbalanced)")
    a = ap.parse_args()
    import torch

    import rtgpu
    from bench import CONFIGS

    c = CONFIGS[a.config]
    lib = rtgpu.Library(a.lib or None)
    s = rtgpu.SceneLibrary().build(c["scene"], grid=c["grid"], image_width=c["width"],
                                   aspect_ratio=c["width"] / c["height"], spp=c["spp"],
                                   max_depth=c["depth"], rand_seed=1)
    cam = s.camera
    H, W = lib.camera_resolve(cam).image_height, c["width"]
    ds = lib.scene_create(s.desc)
    stream = torch.cuda.current_stream().cuda_stream
    res = {"config": a.config, "lib": a.lib or "default", "layout": a.layout, "height": H, "width": W, "per_n": {}}
    full_ms = None
    ns = [int(x) for x in a.ns.split(",")]
    for n in ([1] if 1 not in ns else []) + sorted(ns, key=lambda x: x != 1):  # N = 1 first: the baseline
        out = torch.zeros((rtgpu.padded_rows(H, n), W, 3), device="cuda")
        kern, wall = [], []
        for r in range(n):
            b, stride, cnt = rtgpu.shard_rows(H, r, n)
            if a.layout == "contig":
                rows = rtgpu.padded_rows(H, n)
                b, stride, cnt = r * rows, 1, max(0, min(rows, H - r * rows))
            if cnt <= 0:  # a rank past the image's last row renders nothing (its shard stays padding)
                kern.append(0.0)
                wall.append(0.0)
                continue
            if a.prepare:
                ds.prepare(cam, row_begin=b, row_stride=stride, row_count=cnt)
            best_k, best_w = 1e30, 1e30
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                st = ds.render_device(cam, out.data_ptr(), stream, row_begin=b, row_stride=stride, row_count=cnt)
                torch.cuda.synchronize()
                best_w = min(best_w, (time.perf_counter() - t0) * 1e3)
                best_k = min(best_k, st.kernel_ms)
            kern.append(round(best_k, 3))
            wall.append(round(best_w, 3))
        if n == 1:  # the efficiency baseline is the one-rank frame, whatever order --ns lists
            full_ms = max(wall)
        res["per_n"][n] = {"kernel_ms": kern, "sum_kernel_ms": round(sum(kern), 3), "wall_ms": wall,
                           "max_wall_ms": max(wall),
                           "efficiency_vs_n1": (round(full_ms / (n * max(wall)), 4) if full_ms else None)}
        print(json.dumps({n: res["per_n"][n]}), file=sys.stderr, flush=True)
    ds.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
