"""bench.py's per-pixel check of the benchmark frame (the metric's "per-pixel RMSE vs CPU ref"):
row selection and the comparison against cpu_ref32, on CPU with oracle rows standing in for the
GPU's (no GPU needed)."""
import numpy as np

import bench  # noqa: E402 (repo root is on sys.path via conftest)
import rtgpu


def test_parity_rows_spread_over_the_frame():
    for H, n in ((1080, 36), (2160, 12), (800, 128), (10, 64), (7, 1), (1080, 1)):
        first, step, cnt = bench.parity_rows(H, n)
        rows = [first + k * step for k in range(cnt)]
        assert cnt == min(n, H) and step >= 1
        assert rows[0] >= 0 and rows[-1] <= H - 1
        assert len(set(rows)) == cnt


def test_cpu_parity_against_the_oracle(scenes, oracle):
    s = scenes.build("bouncing_spheres", rand_seed=1, image_width=64, aspect_ratio=16.0 / 9.0, spp=4,
                     max_depth=10)
    cam = s.camera
    H = oracle.camera_resolve(cam).image_height
    seed = 0x5EED + 7
    frame, _ = oracle.render_f32(s.desc, cam, seed=seed)
    first, step, n = bench.parity_rows(H, 9)
    rows = frame[first::step][:n]
    rep = bench.cpu_parity(s.desc, cam, rows, first, step, seed, threads=4)
    assert rep["pass"] and rep["rmse"] == 0.0 and rep["identical_frac"] == 1.0, rep
    assert rep["rows"] == n and rep["pixels"] == n * frame.shape[1]
    # another seed's frame is a different Monte-Carlo estimate: the check must see it
    other, _ = oracle.render_f32(s.desc, cam, seed=rtgpu.DEFAULT_SEED)
    bad = bench.cpu_parity(s.desc, cam, other[first::step][:n], first, step, seed, threads=3)
    assert bad["identical_frac"] < 0.5 and bad["rmse"] > 0.0
    # a uniformly shifted frame fails the tolerance
    off = bench.cpu_parity(s.desc, cam, rows + np.float32(0.01), first, step, seed, threads=2)
    assert not off["pass"]
