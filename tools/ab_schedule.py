#!/usr/bin/env python3
"""tools/ab_schedule.py — interleaved in-process A/B of render kernels on one device.

  python3 tools/ab_schedule.py [--rounds 3] [--variants 0:48,0:32,1:0] [--spp 500]
                               [--libs new=raytracing-practice_amd/lib/librtgpu.so,base=...]

Each variant "S:B:L" = schedule S (include/rtgpu.h RTG_RENDER_SCHEDULE) with shade batch B (64ths)
and leaf batch L (lanes); 0 = library default. A variant may be prefixed "name@" to pick one of
the --libs builds (default: the first) and suffixed "#ct:ml" to build its BVH with SAH traversal
cost ct and max leaf size ml (RTG_SAH_TUNE), "#@K" / "#ct:ml@K" to render with K samples per chunk
(RTG_CHUNK_SAMPLES; the frame then differs from the rtg-f32 spec, for schedule experiments only). Renders BASELINE config 2 (book-1, 1920x1080, depth 50)
and reports the kernel time (HIP events) per variant per round plus the median Mrays/s; checks
every variant's frame against the first one (identical, or the fraction of equal pixels).
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
    ap.add_argument("--variants", default="0:0:0")
    ap.add_argument("--libs", default="")
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--grid", type=int, default=11)
    ap.add_argument("--scene", default="bouncing_spheres")
    ap.add_argument("--bvh", default="sah")
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--count", action="store_true", help="also report box / prim tests per segment per variant")
    ap.add_argument("--height", type=int, default=0, help="0: 16:9 of --width")
    ap.add_argument("--prepare", action="store_true",
                    help="rtg_scene_prepare each scene for the camera before the rounds (hot treelet, tile order)")
    a = ap.parse_args()
    import torch

    import rtgpu

    libs = {}
    for item in filter(None, a.libs.split(",")):
        name, path = item.split("=", 1)
        libs[name] = rtgpu.Library(os.path.join(REPO, path) if not os.path.isabs(path) else path)
    if not libs:
        libs["lib"] = rtgpu.Library()
    first = next(iter(libs))
    bvh = {"sah": rtgpu.RTG_BVH_SAH, "median": rtgpu.RTG_BVH_MEDIAN, "sah2": 2, "gpu": 3}[a.bvh]
    s = rtgpu.SceneLibrary().build(a.scene, grid=a.grid, image_width=a.width,
                                   aspect_ratio=(a.width / a.height) if a.height else 16.0 / 9.0,
                                   spp=a.spp, max_depth=a.depth, bvh_mode=bvh)
    cam = s.camera
    H = libs[first].camera_resolve(cam).image_height
    scenes = {}

    def scene_for(name, tune, env=""):
        tune = tune.split("%", 1)[0]
        if (name, tune, env) not in scenes:
            if tune.split("@", 1)[0]:
                os.environ["RTG_SAH_TUNE"] = tune.split("@", 1)[0]
            else:
                os.environ.pop("RTG_SAH_TUNE", None)
            scenes[(name, tune, env)] = libs[name].scene_create(s.desc)
            os.environ.pop("RTG_SAH_TUNE", None)
            if a.prepare:
                scenes[(name, tune, env)].prepare(cam)
        return scenes[(name, tune, env)]
    out = torch.zeros((H, a.width, 3), device="cuda")
    stream = torch.cuda.current_stream().cuda_stream

    variants = []
    envs = {}
    for v in a.variants.split(","):
        # "...!K=V;K2=V2": environment variables set around this variant's renders (library A/B knobs)
        v, env = (v.split("!", 1) if "!" in v else (v, ""))
        head, tune = (v.split("#", 1) if "#" in v else (v, ""))
        name, spec = (head.split("@", 1) if "@" in head else (first, head))
        nums = tuple(int(x) for x in (spec.split(":") + ["0", "0"])[:3])
        variants.append((name, nums, tune, env))
        # ";" or "^" between variables ("^" survives a shell command line unquoted)
        envs[variants[-1]] = dict(kv.split("=", 1) for kv in env.replace("^", ";").split(";") if kv)
    times = {v: [] for v in variants}
    frames, segs, counts = {}, {}, {}
    for r in range(a.rounds):
        for v in variants:
            name, (sched, batch, leaf), tune, env = v
            for k, val in envs[v].items():
                os.environ[k] = val
            L, ds = libs[name], scene_for(name, tune, env)
            if "%" in tune:  # "...%v": RTG_COMBINE=v
                os.environ["RTG_COMBINE"] = tune.split("%", 1)[1]
                tune = tune.split("%", 1)[0]
            else:
                os.environ.pop("RTG_COMBINE", None)
            if "@" in tune:  # "#ct:ml@K" or "#@K": samples-per-chunk override (RTG_CHUNK_SAMPLES)
                os.environ["RTG_CHUNK_SAMPLES"] = tune.split("@", 1)[1]
            else:
                os.environ.pop("RTG_CHUNK_SAMPLES", None)
            flags = rtgpu.RTG_RENDER_OUT_DEVICE | (sched << 8) | (batch << 16) | (leaf << 24)
            job = rtgpu.rtg_render_desc(0x5EED, 0, 1, 0, flags, stream)
            st = rtgpu.rtg_render_stats()
            L.check("rtg_render", L.lib.rtg_render(ds.handle, rtgpu.C.byref(cam), rtgpu.C.byref(job),
                                                    out.data_ptr(), rtgpu.C.byref(st)))
            for k in envs[v]:
                os.environ.pop(k, None)
            times[v].append(st.kernel_ms)
            segs[v] = st.segments
            if r == 0:
                frames[v] = out.cpu().numpy().copy()
                if a.count:  # box / primitive tests per segment of this variant (counting kernel)
                    job = rtgpu.rtg_render_desc(0x5EED, 0, 1, 0, flags | rtgpu.RTG_RENDER_COUNT, stream)
                    cst = rtgpu.rtg_render_stats()
                    for k2, val in envs[v].items():
                        os.environ[k2] = val
                    L.check("rtg_render", L.lib.rtg_render(ds.handle, rtgpu.C.byref(cam), rtgpu.C.byref(job),
                                                            out.data_ptr(), rtgpu.C.byref(cst)))
                    for k2 in envs[v]:
                        os.environ.pop(k2, None)
                    counts[v] = (cst.box_tests / max(cst.segments, 1), cst.prim_tests / max(cst.segments, 1),
                                 getattr(cst, "stack_spills", 0) / max(cst.segments, 1))
    base = frames[variants[0]]
    res = {}
    for v in variants:
        med = float(np.median(times[v]))
        key = f"{v[0]}@" + ":".join(str(x) for x in v[1]) + (f"#{v[2]}" if v[2] else "") + (f"!{v[3]}" if v[3] else "")
        res[key] = {"kernel_ms": [round(t, 2) for t in times[v]], "median_ms": round(med, 2),
                    "mrays_per_s": round(segs[v] / med / 1e3, 1), "segments": int(segs[v]),
                    "identical_frame": bool(np.array_equal(frames[v], base)),
                    "equal_pixel_frac": float(np.mean(np.all(frames[v] == base, axis=-1)))}
        if v in counts:
            res[key]["box_tests_per_segment"] = round(counts[v][0], 3)
            res[key]["prim_tests_per_segment"] = round(counts[v][1], 3)
            res[key]["stack_spills_per_segment"] = round(counts[v][2], 4)
    for ds in scenes.values():
        ds.close()
    print(json.dumps({"scene": a.scene, "grid": a.grid, "spp": a.spp, "width": a.width, "depth": a.depth,
                      "results": res}, indent=1))


if __name__ == "__main__":
    main()
