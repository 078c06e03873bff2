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


def _args(gpus):
    import types
    return types.SimpleNamespace(gpus=gpus)


def test_self_launch_starts_n_ranks(monkeypatch):
    """`bench.py --gpus N` without a launcher starts torch.distributed.run with N ranks as a child
    process (never an exec) and returns its exit code; one GPU or an existing launcher: no launch."""
    import subprocess
    import sys

    seen = {}

    class Done:
        returncode = 7

    def fake_run(cmd, env=None, **kw):
        seen["cmd"], seen["env"] = cmd, env
        return Done()

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv(bench.LAUNCH_GUARD, raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "3"])
    assert bench.self_launch(_args(8)) == 7
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5].endswith("bench.py")
    assert seen["env"][bench.LAUNCH_GUARD] == "1"
    seen.clear()
    assert bench.self_launch(_args(1)) is None and not seen
    monkeypatch.setenv("WORLD_SIZE", "8")
    assert bench.self_launch(_args(8)) is None and not seen


def test_world_size_mismatch_exits_nonzero():
    """Under a launcher whose WORLD_SIZE differs from --gpus the line would describe another job:
    bench.py exits non-zero before touching torch or a GPU."""
    import os
    import subprocess
    import sys

    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "8"], env=env, capture_output=True, text=True,
                       timeout=60)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
