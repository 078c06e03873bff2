"""Helpers for the statistical golden (G5) and the 1M-sphere scene pin (G1'), shared by the CPU
and GPU tests. Test infrastructure only.

G5 fixtures (tests/golden/moments_<scene>.npz, written by oracle/gen_golden.py from the ref-hybrid
harness) hold, per pixel, the mean and the per-sample variance of the reference's estimator
(ray_color over get_ray, camera.hpp:55-62 / 180-232, glibc rand() streams) at thousands of
samples. A frame of the same camera rendered with any other random numbers must agree with that
mean within its Monte-Carlo error: `block_z` turns the difference into z-scores of 8x8 pixel
blocks per channel.
"""
import os

import numpy as np

import rtgpu
from conftest import GOLDEN

# fixture scene -> (librtscenes scene, bouncing_spheres grid)
MOMENT_SCENES = {"book1": ("bouncing_spheres", 0), "cornell": ("cornell_box", 0),
                 "cornell_translate": ("cornell_translate", 0),
                 "simple_light": ("simple_light", 0), "perlin": ("perlin_sphere", 0),
                 "book1_g500": ("bouncing_spheres", 500), "earth_perlin": ("earth_perlin", 0),
                 "earth": ("earth", 0), "checkered": ("checkered_spheres", 0), "quads": ("quads", 0)}

# numpy views of the C-ABI records (include/rtgpu.h)
PRIM_DT = np.dtype([("kind", "<i4"), ("material", "<i4"), ("p0", "<f8", 3), ("p1", "<f8", 3),
                    ("p2", "<f8", 3), ("radius", "<f8")])
MAT_DT = np.dtype([("type", "<i4"), ("texture", "<i4"), ("albedo", "<f8", 3), ("fuzz", "<f8"),
                   ("ri", "<f8")])
TEX_DT = np.dtype([("type", "<i4"), ("even", "<i4"), ("odd", "<i4"), ("image", "<i4"), ("perlin", "<i4"),
                   ("pad", "<i4"), ("scale", "<f8"), ("color", "<f8", 3)])


def load_moments(scene):
    z = np.load(os.path.join(GOLDEN, f"moments_{scene}.npz"))
    return {k: z[k] for k in z.files}


def moments_camera(scene, spp):
    """The harness camera of a G5 fixture (oracle/ref_harness.cpp setup_cam, main.cpp's cameras)."""
    from test_oracle_parity import hybrid_camera

    m = load_moments(scene)
    W, H, depth = int(m["W"]), int(m["H"]), int(m["depth"])
    return hybrid_camera("book1" if scene == "book1_g500" else scene, W, H, spp, depth), m


def block_z(frame, mean, var, n_frame, n_ref, b=8, floor=1e-5):
    """z-scores of the per-channel means of b x b pixel blocks of (frame - mean), whether each
    block carries Monte-Carlo variance at all, and the z of the whole frame per channel. The
    variance of a pixel difference is var * (1/n_frame + 1/n_ref) (the two estimates are
    independent); `floor` (absolute, per block mean) covers fp32 rounding of the frame where the
    estimator has no variance (sky seen through no geometry: every sample is the background)."""
    H, W, _ = mean.shape
    hb, wb = H // b, W // b
    d = frame.astype(np.float64) - mean.astype(np.float64)
    v = var.astype(np.float64) * (1.0 / n_frame + 1.0 / n_ref)

    def blocks(x):
        return x[:hb * b, :wb * b].reshape(hb, b, wb, b, 3).sum(axis=(1, 3))

    bd = blocks(d) / (b * b)
    mc = blocks(v) / (b * b) ** 2
    z = bd / np.sqrt(mc + floor ** 2)
    noisy = mc > 4 * floor ** 2
    gz = d.reshape(-1, 3).mean(axis=0) / np.sqrt(v.reshape(-1, 3).sum(axis=0) / (H * W) ** 2 + floor ** 2)
    return z, noisy, gz


def assert_statistical_parity(frame, m, n_frame, z_max=4.0, frac=0.999, global_sigma=3.0):
    """|z| < z_max on >= frac of the 8x8 blocks (per channel); over the blocks with Monte-Carlo
    variance, the mean of z^2 consistent with 1 (chi-square: a wrong variance or a small bias
    everywhere shows here first; the three channels of a block are strongly correlated, so the
    band counts blocks, not block-channels); the global mean of every channel within global_sigma
    standard errors. z_max covers the skew of block means at low sample counts (rare bright or
    dark paths): 4 at GPU sample counts, 5 for the CPU oracle's few samples per pixel.
    At least two blocks may exceed z_max whatever the frame size: at 16 spp a light-lit scene's
    block means are heavy-tailed, and across 40 seeds of the 120x120 Cornell frame (675
    block-channels each) 9 block-channels exceeded 5 sigma with the round-1 PCG32 draws (4 with a
    multiply-with-carry generator tried in round 2), so a "none of 675" rule (0.999 of 675) failed
    about one seed in ten whatever the generator."""
    z, noisy, gz = block_z(frame, m["mean"], m["var"], n_frame, int(m["n"]))
    ok = float(np.mean(np.abs(z) < z_max))
    outliers = int(np.sum(np.abs(z) >= z_max))
    zn = z[noisy]
    chi = float(np.mean(zn * zn))
    band = 6.0 * np.sqrt(2.0 * 3.0 / zn.size)  # 6 sigma of the chi-square mean, zn.size / 3 blocks
    assert outliers <= max(2, int((1.0 - frac) * z.size)), (ok, outliers, float(np.abs(z).max()))
    assert abs(chi - 1.0) < band + 0.05, (chi, band)  # +0.05: non-gaussian tails of bright paths
    assert np.all(np.abs(gz) < global_sigma), gz.tolist()
    return {"blocks": int(z.size), "noisy": int(zn.size), "frac_ok": ok, "mean_z2": chi,
            "max_abs_z": float(np.abs(z).max()), "global_z": gz.tolist()}


def scene_records(desc):
    """The mirror's bouncing_spheres scene as the reference harness's (N, 13) record array:
    c1[3] c2[3] r mat albedo[3] fuzz ri, mat 0 = checker ground, 1 lambertian, 2 metal,
    3 dielectric (oracle/ref_harness.cpp records_mode)."""
    import ctypes as C

    n = int(desc.num_prims)
    prims = np.frombuffer((C.c_char * (n * PRIM_DT.itemsize)).from_address(
        C.addressof(desc.prims.contents)), dtype=PRIM_DT)
    mats = np.frombuffer((C.c_char * (desc.num_materials * MAT_DT.itemsize)).from_address(
        C.addressof(desc.materials.contents)), dtype=MAT_DT)
    texs = np.frombuffer((C.c_char * (desc.num_textures * TEX_DT.itemsize)).from_address(
        C.addressof(desc.textures.contents)), dtype=TEX_DT)
    assert np.all(prims["kind"] == rtgpu.RTG_PRIM_SPHERE)
    m = mats[prims["material"]]
    t = texs[m["texture"]]
    out = np.zeros((n, 13), dtype="<f8")
    out[:, 0:3] = prims["p0"]
    out[:, 3:6] = prims["p1"]
    out[:, 6] = prims["radius"]
    lam = m["type"] == rtgpu.RTG_MAT_LAMBERTIAN
    checker = lam & (t["type"] == rtgpu.RTG_TEX_CHECKER)
    solid = lam & (t["type"] == rtgpu.RTG_TEX_SOLID)
    metal = m["type"] == rtgpu.RTG_MAT_METAL
    diel = m["type"] == rtgpu.RTG_MAT_DIELECTRIC
    assert np.all(checker | solid | metal | diel)
    out[:, 7] = np.select([checker, solid, metal, diel], [0, 1, 2, 3])
    out[solid, 8:11] = t["color"][solid]
    out[metal, 8:11] = m["albedo"][metal]
    out[metal, 11] = m["fuzz"][metal]
    out[diel, 12] = m["ri"][diel]
    return out
