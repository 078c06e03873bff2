"""Multi-rank path on CPU (gloo, world_size 2 and 3): each rank renders its interleaved shard,
rtgpu.gather_frame collects and de-interleaves on rank 0, and the frame must equal a single-rank
render bit for bit — the RNG is keyed by the global pixel id, so tiling cannot change a pixel.
The per-rank renderer here is the fp32 oracle (the GPU kernel is exercised by test_gpu.py)."""
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


def _worker(rank, world, port, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import rtgpu
        from oracle_bind import Oracle

        s = rtgpu.SceneLibrary().build("bouncing_spheres", rand_seed=1)
        cam = rtgpu.rtg_camera_desc.from_buffer_copy(s.camera)
        cam.image_width, cam.samples_per_pixel, cam.max_depth = 40, 2, 10
        H = rtgpu.Library().camera_resolve(cam).image_height
        b, stride, n = rtgpu.shard_rows(H, rank, world)
        rows = rtgpu.padded_rows(H, world)
        shard = torch.zeros((rows, 40, 3), dtype=torch.float32)
        if n:
            img, _ = Oracle().render_f32(s.desc, cam, row_begin=b, row_stride=stride, row_count=n)
            shard[:n] = torch.from_numpy(img)
        frame = rtgpu.gather_frame(shard, H)
        # the RGB8 variant: write_color bytes gathered, 4x fewer bytes
        bytes8 = torch.from_numpy(np.stack([rtgpu.write_color_bytes(r) for r in shard.numpy()]))
        frame8 = rtgpu.gather_frame(bytes8, H)
        if rank == 0:
            np.save(result_path, frame.numpy())
            np.save(result_path + ".rgb8.npy", frame8.numpy())
        else:
            assert frame is None and frame8 is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_render_equals_single(tmp_path, world, scenes, oracle, lib):
    import rtgpu

    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    frame = np.load(out)
    s = scenes.build("bouncing_spheres", rand_seed=1)
    cam = rtgpu.rtg_camera_desc.from_buffer_copy(s.camera)
    cam.image_width, cam.samples_per_pixel, cam.max_depth = 40, 2, 10
    full, _ = oracle.render_f32(s.desc, cam)
    assert frame.shape == full.shape
    assert np.array_equal(frame, full)
    frame8 = np.load(out + ".rgb8.npy")
    assert frame8.dtype == np.uint8 and np.array_equal(frame8, rtgpu.write_color_bytes(full))


def test_shard_rows_cover_the_image():
    import rtgpu

    for H in (1, 7, 225, 1080, 2160):
        for world in (1, 2, 3, 4, 8, 16):
            rows = []
            for r in range(world):
                b, stride, n = rtgpu.shard_rows(H, r, world)
                rows += [b + k * stride for k in range(n)]
                assert n <= rtgpu.padded_rows(H, world)
            assert sorted(rows) == list(range(H))
