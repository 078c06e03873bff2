#!/usr/bin/env python3
"""tools/comm_probe.py — N-rank check of the C-ABI RCCL path (rtg_comm_create_rank + rtg_gather_rows)
under torch.distributed.run: every rank renders its interleaved shard of a small book-1 frame,
rank 0 gathers + de-interleaves and compares with a single-device render of the whole frame.

  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/comm_probe.py [--same-device]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-practice_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--same-device", action="store_true", help="every rank on device 0 (one-GPU box)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist

    import rtgpu

    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    dev = 0 if a.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = rtgpu.Library()
    s = rtgpu.SceneLibrary().build("bouncing_spheres", rand_seed=1)
    c = rtgpu.rtg_camera_desc.from_buffer_copy(s.camera)
    c.image_width, c.samples_per_pixel, c.max_depth = 96, 4, 20
    ds = lib.scene_create(s.desc, device=dev)
    H, W = lib.camera_resolve(c).image_height, 96
    uid = [lib.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    comm = lib.comm_rank(uid[0], world, rank, dev)
    b, stride, n = rtgpu.shard_rows(H, rank, world)
    shard = torch.zeros((rtgpu.padded_rows(H, world), W, 3), device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    if n > 0:
        ds.render_device(c, shard.data_ptr(), stream, seed=3, row_begin=b, row_stride=stride, row_count=n)
    frame = torch.zeros((H, W, 3), device="cuda") if rank == 0 else None
    comm.gather_rows([shard.data_ptr()], H, W * 12, 0, frame.data_ptr() if frame is not None else 0, [stream])
    torch.cuda.synchronize()
    if rank == 0:
        full, _ = ds.render_host(c, seed=3)
        ok = bool(np.array_equal(frame.cpu().numpy(), full))
        print(json.dumps({"world": world, "same_device": a.same_device, "identical": ok}), flush=True)
    comm.close()
    ds.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
