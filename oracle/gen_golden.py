"""oracle/gen_golden.py — TEST INFRASTRUCTURE: regenerates tests/golden/ from the reference.

Run in the build container (needs /root/reference and the harness built by oracle/Makefile):
    make -C oracle && python oracle/gen_golden.py

Writes
  tests/golden/reference_golden.json  unit KATs, RNG streams, the book-1 scene, bvh_node traversal
                                      logs — all produced by the reference's own code (ref_harness)
  tests/golden/hybrid_<scene>.npz     fp64 framebuffers (pixel_samples_scale * pixel_color) of the
                                      "ref-hybrid" render (reference geometry/BVH/RNG/perlin code +
                                      restated camera/material loop) and their segment counts
  tests/golden/earthmap.ppm           earthmap.jpg decoded to 8-bit sRGB (PIL), the input the image
                                      loader expects in place of stb_image (parity unpinned at the
                                      JPEG decoder: stb vs libjpeg may differ by 1 LSB)
"""
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
    ("simple_light", 64, 36, 8, 20, 5),
    ("perlin", 64, 36, 4, 10, 7),
]


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

    for scene, W, H, spp, depth, seed in HYBRID_RENDERS:
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

    if os.path.exists(REF_IMAGE):
        from PIL import Image

        img = np.asarray(Image.open(REF_IMAGE).convert("RGB"), dtype=np.uint8)
        h, w, _ = img.shape
        with open(os.path.join(GOLDEN, "earthmap.ppm"), "wb") as f:
            f.write(f"P6\n{w} {h}\n255\n".encode())
            f.write(img.tobytes())
        print("earthmap.ppm:", img.shape)
    return 0


if __name__ == "__main__":
    sys.exit(main())
