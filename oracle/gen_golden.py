"""oracle/gen_golden.py — TEST INFRASTRUCTURE: regenerates tests/golden/ from the reference.

Run in the build container (needs /root/reference and the harness built by oracle/Makefile):
    make -C oracle && python oracle/gen_golden.py

Writes
  tests/golden/reference_golden.json  unit KATs, RNG streams, the book-1 scene, bvh_node traversal
                                      logs — all produced by the reference's own code (ref_harness)
  tests/golden/hybrid_<scene>.npz     fp64 framebuffers (pixel_samples_scale * pixel_color) of the
                                      "ref-hybrid" render (reference geometry/BVH/RNG/perlin code +
                                      restated camera/material loop) and their segment counts
  tests/golden/moments_<scene>.npz    G5: per-pixel mean and per-sample variance of the ref-hybrid
                                      estimator at thousands of samples per pixel (many srand
                                      streams), the statistical golden of the GPU frames
  tests/golden/reference_scene_g500.json  G1': bouncing_spheres at grid half-width 500 (BASELINE
                                      config 5, 1,000,001 records): per-material counts and the
                                      sha256 of the reference's (N, 13) float64 record array
  tests/golden/ties.json              exact-t tie winners of the reference's own hittable_list and
                                      bvh_node over the tie world (scenes.hpp tie_world), 101 rays
  tests/golden/earthmap.ppm           earthmap.jpg decoded to 8-bit sRGB (PIL), the input the image
                                      loader expects in place of stb_image (parity unpinned at the
                                      JPEG decoder: stb vs libjpeg may differ by 1 LSB)
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ORACLE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(ORACLE)
GOLDEN = os.path.join(REPO, "tests", "golden")
HARNESS = os.path.join(ORACLE, "_ref", "ref_harness")
REF_IMAGE = "/root/reference/images/earthmap.jpg"

# (scene, W, H, spp, depth, render seed): small enough to keep fixtures at tens of KB
HYBRID_RENDERS = [
    ("book1", 96, 54, 8, 10, 1),
    ("cornell", 40, 40, 8, 20, 3),
    ("cornell_translate", 40, 40, 8, 100, 9),  # the reference's translate class (hittable.hpp:74-117)
    ("simple_light", 64, 36, 8, 20, 5),
    ("perlin", 64, 36, 4, 10, 7),
    ("earth", 64, 36, 4, 10, 11),  # image_texture on the committed texels (texture.hpp:91-122)
    ("earth_perlin", 64, 36, 4, 20, 13),  # BASELINE config 3's scene
    ("checkered", 64, 36, 8, 20, 17),  # checkered_spheres (main.cpp:104-138)
    ("quads", 40, 40, 8, 50, 19),  # quads (main.cpp:210-251)
]

# G5: (scene, W, H, spp per process, processes, depth). book1 = BASELINE config-1
# geometry (400 wide, 16/9 double aspect -> 225 rows) at config 2's depth 50; cornell at config 4's
# depth 100; cornell_translate = its boxes and a sphere placed by the reference's translate class
# (hittable.hpp:74-117); book1_g500 = config 5's 1M-sphere field on a small frame.
MOMENTS = [
    ("book1", 400, 225, 512, 8, 50),
    ("cornell", 120, 120, 512, 8, 100),
    ("cornell_translate", 96, 96, 512, 8, 100),
    ("simple_light", 192, 108, 512, 8, 50),
    ("perlin", 160, 90, 256, 8, 50),
    ("book1_g500", 96, 54, 256, 8, 50),
    ("earth_perlin", 192, 108, 512, 8, 50),  # BASELINE config 3's scene: image + noise textures
    ("earth", 128, 72, 512, 8, 50),
    ("checkered", 128, 72, 512, 8, 20),  # the reference's own depth (main.cpp:122)
    ("quads", 96, 96, 512, 8, 50),
]
MOMENTS_SEED0 = 90001


def gen_moments(only=None) -> None:
    for scene, W, H, spp, procs, depth in MOMENTS:
        if only and scene not in only:
            continue
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "m.bin")
            out = subprocess.run([HARNESS, "moments", scene, str(W), str(H), str(spp), str(depth),
                                  str(procs), str(MOMENTS_SEED0), path],
                                 check=True, capture_output=True, text=True).stdout.split("\n")
            segs = sum(int(x) for x in out if x.strip().isdigit())
            meta = json.loads([x for x in out if x.startswith("{")][0])
            m = np.fromfile(path, dtype=np.float64).reshape(meta["height"], meta["width"], 6)
        n = meta["samples_per_pixel"]
        mean = m[..., :3] / n
        var = np.maximum(m[..., 3:] / n - mean * mean, 0.0) * (n / (n - 1.0))
        np.savez_compressed(os.path.join(GOLDEN, f"moments_{scene}.npz"), mean=mean.astype(np.float32),
                            var=var.astype(np.float32), n=n, W=W, H=meta["height"], depth=depth,
                            segments=segs, seed0=MOMENTS_SEED0, procs=procs)
        print(f"moments_{scene}: {mean.shape} n={n} segments/sample={segs / (n * W * meta['height']):.4f}")


def gen_ties() -> None:
    out = subprocess.run([HARNESS, "ties"], check=True, capture_output=True, text=True).stdout
    data = json.loads(out)
    with open(os.path.join(GOLDEN, "ties.json"), "w") as f:
        json.dump(data, f, separators=(",", ":"))
    diff = sum(a != b for a, b in zip(data["list"]["winner"], data["bvh"]["winner"]))
    print(f"ties.json: {len(data['rays'])} rays, list vs bvh_node winners differ on {diff}")


def gen_scene_records() -> None:
    rec = {}
    for grid in (11, 500):
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "r.bin")
            meta = json.loads(subprocess.run([HARNESS, "records", str(grid), path], check=True,
                                             capture_output=True, text=True).stdout)
            a = np.fromfile(path, dtype="<f8").reshape(-1, 13)
        meta["sha256"] = hashlib.sha256(a.tobytes()).hexdigest()
        meta["first"] = a[:4].tolist()
        meta["last"] = a[-4:].tolist()
        rec[str(grid)] = meta
        print(f"records grid {grid}: {meta['records']} sha256 {meta['sha256'][:16]}")
    with open(os.path.join(GOLDEN, "reference_scene_g500.json"), "w") as f:
        json.dump(rec, f, indent=1)


def main() -> int:
    if not os.path.exists(HARNESS):
        print("ref_harness not built (make -C oracle)", file=sys.stderr)
        return 1
    os.makedirs(GOLDEN, exist_ok=True)
    out = subprocess.run([HARNESS, "golden"], check=True, capture_output=True, text=True).stdout
    data = json.loads(out)
    with open(os.path.join(GOLDEN, "reference_golden.json"), "w") as f:
        json.dump(data, f, separators=(",", ":"))
    print("reference_golden.json:", {k: len(v) if isinstance(v, list) else "…" for k, v in data.items()})

    gen_hybrid()
    gen_ties()
    gen_scene_records()
    gen_moments()

    if os.path.exists(REF_IMAGE):
        from PIL import Image

        img = np.asarray(Image.open(REF_IMAGE).convert("RGB"), dtype=np.uint8)
        h, w, _ = img.shape
        with open(os.path.join(GOLDEN, "earthmap.ppm"), "wb") as f:
            f.write(f"P6\n{w} {h}\n255\n".encode())
            f.write(img.tobytes())
        print("earthmap.ppm:", img.shape)
    return 0


def gen_hybrid(only=None) -> None:
    for scene, W, H, spp, depth, seed in HYBRID_RENDERS:
        if only and scene not in only:
            continue
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "fb.bin")
            meta = json.loads(subprocess.run(
                [HARNESS, "render", scene, str(W), str(H), str(spp), str(depth), str(seed), path],
                check=True, capture_output=True, text=True).stdout)
            fb = np.fromfile(path, dtype=np.float64).reshape(meta["height"], meta["width"], 3)
        np.savez_compressed(os.path.join(GOLDEN, f"hybrid_{scene}.npz"), fb=fb,
                            W=W, H=H, spp=spp, depth=depth, seed=seed,
                            segments=meta["segments"])
        print(f"hybrid_{scene}: {fb.shape} segments={meta['segments']}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "moments":  # regenerate only the G5 fixtures
        gen_moments(sys.argv[2:] or None)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "hybrid":
        gen_hybrid(sys.argv[2:] or None)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "ties":
        gen_ties()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "records":
        gen_scene_records()
        sys.exit(0)
    sys.exit(main())
