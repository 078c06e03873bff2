"""Multi-rank frame assembly on CPU (gloo, world_size 2 and 3, including ranks past the last row).

Every rank takes its shard from the library's own layout (rtg_shard_layout: rows r, r+N, ...,
padded to ceil(H/N) rows — the arithmetic rtg_render_frame and rtg_gather_rows use), fills it with a
code that names the global pixel it holds, and the frame is assembled on rank 0 both ways bench.py
can do it: (a) the RCCL-gather layout (N padded blocks, one per rank, gathered into one staging
buffer) de-interleaved by rtg_deinterleave_rows_host, the host twin of the root's de-interleave
kernel (same index function); (b) rtgpu.gather_frame (torch.distributed.gather, bench.py's default
N>1 gather). Both must give every pixel its own code, fp32 and RGB8 rows alike. The GPU side of the
same layout (the de-interleave kernel, the world-of-one RCCL gather, rtg_render_frame over two
devices where a node has them) is in test_gpu.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pixel_codes(rows, W):
    """fp32 code of each pixel (image row, column, channel) of the given image rows."""
    r = np.asarray(rows, dtype=np.float32)[:, None, None]
    c = np.arange(W, dtype=np.float32)[None, :, None]
    ch = np.arange(3, dtype=np.float32)[None, None, :]
    return r * 4096.0 + c * 4.0 + ch


def _worker(rank, world, port, H, W, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import rtgpu

        lib = rtgpu.Library()
        b, stride, n, padded = lib.shard_layout(H, world, rank)
        assert (b, stride, n) == rtgpu.shard_rows(H, rank, world) and padded == rtgpu.padded_rows(H, world)
        shard = torch.full((padded, W, 3), -1.0, dtype=torch.float32)  # padding rows stay -1
        if n:
            shard[:n] = torch.from_numpy(_pixel_codes([b + k * stride for k in range(n)], W))
        # (a) the RCCL layout: N padded blocks gathered into one staging buffer, host de-interleave
        blocks = [torch.empty_like(shard) for _ in range(world)] if rank == 0 else None
        dist.gather(shard, gather_list=blocks, dst=0)
        # (b) bench.py's default torch.distributed gather + torch de-interleave
        frame_t = rtgpu.gather_frame(shard, H)
        # RGB8 rows (write_color bytes, 3 B per pixel: rows of W*3 bytes, not a multiple of 16)
        bytes8 = torch.from_numpy(rtgpu.write_color_bytes(shard.numpy() / 8192.0))
        blocks8 = [torch.empty_like(bytes8) for _ in range(world)] if rank == 0 else None
        dist.gather(bytes8, gather_list=blocks8, dst=0)
        if rank == 0:
            stage = torch.cat(blocks).numpy()
            np.save(result_path, lib.deinterleave_rows_host(stage, world, H))
            np.save(result_path + ".torch.npy", frame_t.numpy())
            np.save(result_path + ".rgb8.npy", lib.deinterleave_rows_host(torch.cat(blocks8).numpy(), world, H))
        else:
            assert frame_t is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H", [(2, 225), (3, 224), (3, 2)])
def test_gloo_frame_assembly_uses_the_library_layout(tmp_path, world, H):
    W = 40
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(world, _free_port(), H, W, out), nprocs=world, join=True)
    want = _pixel_codes(range(H), W)
    frame = np.load(out)
    assert frame.shape == (H, W, 3) and np.array_equal(frame, want)
    assert np.array_equal(np.load(out + ".torch.npy"), want)
    import rtgpu

    assert np.array_equal(np.load(out + ".rgb8.npy"), rtgpu.write_color_bytes(want / 8192.0))


def test_shard_layout_matches_python_and_covers_the_image(lib):
    """rtg_shard_layout (C) = rtgpu.shard_rows / padded_rows (Python, bench.py), and the shards of
    every rank cover each image row exactly once, for image heights below, at and above N."""
    import rtgpu

    for H in (1, 2, 7, 225, 1080, 2160):
        for world in (1, 2, 3, 4, 8, 16):
            rows = []
            for r in range(world):
                b, stride, n, padded = lib.shard_layout(H, world, r)
                assert (b, stride, n) == rtgpu.shard_rows(H, r, world)
                assert padded == rtgpu.padded_rows(H, world) and n <= padded
                rows += [b + k * stride for k in range(n)]
            assert sorted(rows) == list(range(H))


def test_host_deinterleave_matches_numpy(lib):
    """The host twin of the de-interleave kernel against rtgpu.deinterleave (numpy) on byte rows of
    every width class (16-B multiples and not) and ranks past the last row."""
    import rtgpu

    rng = np.random.default_rng(3)
    for H, world, W in ((1080, 8, 16), (7, 3, 5), (2, 5, 3), (13, 4, 1)):
        padded = rtgpu.padded_rows(H, world)
        blocks = rng.integers(0, 255, size=(world, padded, W, 3), dtype=np.uint8)
        want = rtgpu.deinterleave(list(blocks), H)
        got = lib.deinterleave_rows_host(blocks.reshape(world * padded, W, 3), world, H)
        assert np.array_equal(got, want)


def test_bad_layout_arguments_are_rejected(lib):
    import rtgpu

    for args in ((0, 2, 0), (10, 0, 0), (10, 2, 2), (10, 2, -1)):
        with pytest.raises(rtgpu.RtgError):
            lib.shard_layout(*args)


def _frame_gather_worker(rank, world, port, H, W, result_path):
    """bench.py's timed N > 1 gather (rtgpu.FrameGather): buffers allocated once at set-up; a step —
    gather into the staging blocks, the library's de-interleave — allocates no tensor (torch's
    allocating factories are made to raise around the calls) and returns the same frame tensor."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import rtgpu

        lib = rtgpu.Library()
        b, stride, n, padded = lib.shard_layout(H, world, rank)
        shard = torch.full((padded, W, 3), -1.0, dtype=torch.float32)
        fg = rtgpu.FrameGather(lib, shard, H)

        def boom(*a, **k):
            raise AssertionError("tensor allocated inside a timed gather step")

        names = ("empty", "zeros", "empty_like", "zeros_like", "cat", "stack")
        saved = {k: getattr(torch, k) for k in names}
        saved_new = torch.Tensor.new_empty
        frames = []
        for step in range(3):
            if n:  # this step's pixel codes, offset per step
                shard[:n] = torch.from_numpy(_pixel_codes([b + k * stride for k in range(n)], W) + step)
            for k in names:
                setattr(torch, k, boom)
            torch.Tensor.new_empty = boom
            try:
                f = fg(shard)
            finally:
                for k, v in saved.items():
                    setattr(torch, k, v)
                torch.Tensor.new_empty = saved_new
            if rank == 0:
                assert f is not None and (not frames or f.data_ptr() == frames[0][0])
                frames.append((f.data_ptr(), f.numpy().copy()))
            else:
                assert f is None
        if rank == 0:
            np.save(result_path, np.stack([fr for _, fr in frames]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H", [(2, 225), (3, 7)])
def test_frame_gather_allocates_nothing_per_step(tmp_path, world, H):
    W = 24
    out = str(tmp_path / "frames.npy")
    mp.spawn(_frame_gather_worker, args=(world, _free_port(), H, W, out), nprocs=world, join=True)
    frames = np.load(out)
    for step in range(3):
        assert np.array_equal(frames[step], _pixel_codes(range(H), W) + step)
