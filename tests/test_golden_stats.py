"""CPU side of the reference pins that need no GPU:

* G1' — the 1M-sphere scene of BASELINE config 5 (bouncing_spheres with the grid loop bounds
  generalised to [-500, 500), main.cpp:24-26) built by the C++ mirror equals the reference's
  record for record (sha256 of the (N, 13) record array from oracle/ref_harness records 500).
* G5 — the oracle's fp32 spec (cpu_ref32, counter RNG, direct sampling) agrees with the reference
  estimator's per-pixel mean (tests/golden/moments_*.npz, thousands of samples per pixel from
  glibc rand() streams) within the Monte-Carlo error. The same check runs on the GPU frames in
  test_gpu.py::test_statistical_parity_vs_reference.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from golden_stats import MOMENT_SCENES, assert_statistical_parity, load_moments, moments_camera, scene_records


@pytest.mark.parametrize("grid", [11, 500])
def test_bouncing_spheres_grid_matches_reference(scenes, grid):
    with open(os.path.join(GOLDEN, "reference_scene_g500.json")) as f:
        ref = json.load(f)[str(grid)]
    s = scenes.build("bouncing_spheres", grid=grid, rand_seed=1)
    rec = scene_records(s.desc)
    assert rec.shape[0] == ref["records"]
    mat = rec[:, 7].astype(int)
    counts = {k: int(np.sum(mat == v)) for k, v in (("ground", 0), ("lambertian", 1), ("metal", 2),
                                                   ("dielectric", 3))}
    assert counts == {k: ref[k] for k in counts}
    assert rec[:4].tolist() == ref["first"] and rec[-4:].tolist() == ref["last"]
    assert hashlib.sha256(rec.astype("<f8").tobytes()).hexdigest() == ref["sha256"]
    if grid == 500:  # 799,468 lambertian / 150,434 metal / 50,095 dielectric small spheres
        assert rec.shape[0] == 1_000_001
        assert (counts["lambertian"] - 1, counts["metal"] - 1, counts["dielectric"] - 1) == (799468, 150434, 50095)


@pytest.mark.parametrize("scene,spp", [("book1", 8), ("cornell", 16), ("cornell_translate", 16), ("simple_light", 8), ("perlin", 8),
                                       ("book1_g500", 4), ("earth_perlin", 8), ("earth", 8), ("checkered", 8),
                                       ("quads", 8)])
def test_cpu_ref32_statistical_parity_vs_reference(scenes, oracle, scene, spp):
    name, grid = MOMENT_SCENES[scene]
    s = scenes.build(name, grid=grid, rand_seed=1)
    cam, m = moments_camera(scene, spp)
    f32, segs = oracle.render_f32(s.desc, cam, seed=0xC0FFEE)
    assert f32.shape == m["mean"].shape
    assert_statistical_parity(f32, m, spp, z_max=5.0)
    # mean path length (segments per sample) of the spec vs the reference estimator
    H, W = f32.shape[:2]
    ref_len = float(m["segments"]) / (int(m["n"]) * H * W)
    assert abs(segs / (spp * H * W) - ref_len) / ref_len < 0.02, (segs / (spp * H * W), ref_len)


def test_moment_fixtures_are_consistent():
    """The fixtures describe what gen_golden.py says they do (many samples, non-negative variance)."""
    for scene in MOMENT_SCENES:
        m = load_moments(scene)
        assert int(m["n"]) >= 2048
        assert m["mean"].shape == (int(m["H"]), int(m["W"]), 3)
        assert np.all(m["var"] >= 0) and np.all(np.isfinite(m["mean"]))
