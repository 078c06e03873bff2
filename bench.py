#!/usr/bin/env python3
"""bench.py — Mrays/s of the per-pixel sample loop (camera::render -> ray_color -> bvh/sphere hit
-> material::scatter) on the book-1 random-sphere scene, BASELINE config 2: 1920x1080, 500 spp,
depth 50, on the MI355X kernels of librtgpu.so.

  python bench.py [--gpus N] [--steps K] [--warmup W]     (N > 1: starts its own N ranks, below)
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Without a launcher, `--gpus N` (N > 1) starts `torch.distributed.run --nproc-per-node N` itself as a
child process before touching torch or a GPU, and exits with its code; under a launcher, a WORLD_SIZE
that differs from --gpus is an error.

A step renders one full frame: rank r renders rows r, r+N, ... (interleaved tiling) into a
device buffer and the frame is gathered on rank 0 over RCCL (torch.distributed "nccl" by default, or
the C-ABI's rtg_gather_rows with --gather-impl rtg). The scene is built and uploaded before timing
(reported separately as setup_ms). value = ray segments traced by all ranks / max-over-ranks wall
time of the K timed steps. Prints ONE JSON line on rank 0.

Every line carries the per-pixel check of the benchmark frame itself (`parity`: rows of the last timed
frame — at N > 1 the frame gathered on rank 0 — against the oracle's fp32 spec on the same seeds).
N > 1 lines also carry `ranks` (each rank's rows, segments, kernel and gather times, all-gathered
after timing) and `rtg_gather_check`: after the timed loop, the same shards gathered through the C-ABI's
own RCCL gather (rtg_comm_create_rank, ranks_seen from ncclCommCount) once per timed step, each call
timed on the render stream (the product gather's time beside the timed torch gather's, and the library's
allocations across the calls), the frame compared byte for byte with the timed one, under a watchdog, so a
fault in that path cannot lose the line.
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "raytracing-practice_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))

METRIC = "Mrays/sec at 1920×1080, 500 spp, depth 50; per-pixel RMSE vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# ds_read_b128 / b64 aggregate with every CU streaming at ~2.4 GHz (MI355X_MICROARCH.md §LDS: 256 B/clk/CU)
LDS_PEAK_GBS = 150000.0
SIMDS = 1024  # 256 CUs x 4
BYTES_PER_BOX, BYTES_PER_PRIM, BYTES_PER_HIT = 32, 32, 16  # SURVEY.md §8d algorithmic bytes


# BASELINE.json configs (config 1 is the reference's own CPU plumbing run, not a GPU bench line)
CONFIGS = {
    2: dict(scene="bouncing_spheres", grid=11, width=1920, height=1080, spp=500, depth=50),
    3: dict(scene="earth_perlin", grid=0, width=1920, height=1080, spp=500, depth=50),
    4: dict(scene="cornell_box", grid=0, width=800, height=800, spp=2000, depth=100),
    5: dict(scene="bouncing_spheres", grid=500, width=3840, height=2160, spp=1000, depth=50),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS),
                    help="BASELINE.json config preset (2 = the headline metric); flags below override it")
    ap.add_argument("--scene", default=None)
    ap.add_argument("--grid", type=int, default=None, help="bouncing_spheres grid half-width (500 = 1M spheres)")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--depth", type=int, default=None)
    ap.add_argument("--bvh", choices=["sah", "median", "gpu"], default="sah")
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--gather", choices=["f32", "rgb8"], default="f32",
                    help="gather the linear fp32 frame (default) or the write_color bytes (4x fewer)")
    ap.add_argument("--gather-impl", choices=["rtg", "torch"], default="torch",
                    help="N>1 timed gather: torch.distributed.gather into blocks allocated once + the library's "
                         "de-interleave kernel (rtgpu.FrameGather; default until the C-ABI path has run on a "
                         "multi-GPU node) or the C-ABI's RCCL gather + de-interleave kernel (rtg_gather_rows)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="N>1 process group: nccl (= RCCL, one rank per GPU) or gloo (rehearsal of the N>1 flow "
                         "with several ranks on one GPU; the frame is gathered through host memory)")
    ap.add_argument("--no-rtg-check", action="store_true",
                    help="N>1: skip the untimed rtg_gather_rows cross-check of the last frame")
    ap.add_argument("--check-timeout", type=float, default=180.0,
                    help="N>1: seconds the rtg_gather_rows cross-check may take before the line is printed "
                         "without it")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="wall time the all-cores CPU sample is sized for (the 1-core sample adds ~3-5 s)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core of the host (cgroup quota bound)")
    ap.add_argument("--parity-seconds", type=float, default=4.0,
                    help="CPU wall time the per-pixel check of the benchmark frame (rows vs cpu_ref32) is "
                         "sized for; 0 = off")
    a = ap.parse_args()
    for k, v in CONFIGS[a.config].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    return a


def host_cpus():
    """(cores this process may run on, CPU model, online CPUs, cgroup CPU quota or None). The cores
    used are the affinity set, bounded by a cgroup CPU quota when one is set (more workers than the
    quota would only time-share the same cores)."""
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    cores = avail if quota is None else max(1, min(avail, int(quota)))
    return cores, model, os.cpu_count(), quota


# scenes the ref-hybrid harness builds from the reference's own geometry code
HARNESS_SCENE = {("bouncing_spheres", 11): "book1", ("cornell_box", 0): "cornell",
                 ("bouncing_spheres", 500): "book1_g500", ("earth_perlin", 0): "earth_perlin"}


def _cpu_run(args, scene_desc, cam, procs, spp, row_step):
    """One timed CPU render of the workload's frame (rows 0, row_step, ... dealt over procs
    workers, spp samples per pixel): (seconds, segments, kind, what)."""
    W, H, depth = args.width, args.height, args.depth
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    hscene = HARNESS_SCENE.get((args.scene, args.grid))
    if hscene and os.access(harness, os.X_OK):
        try:
            out = subprocess.run([harness, "bench", hscene, str(W), str(H), str(spp), str(depth), str(procs),
                                  str(row_step)], check=True, capture_output=True, text=True, timeout=900).stdout
            r = json.loads(out)
            return r["seconds"], r["segments"], "reference", "ref-hybrid build"
        except (subprocess.SubprocessError, OSError, ValueError, KeyError) as e:
            print(f"[bench] ref_harness failed ({e}); timing the fp64 port instead", file=sys.stderr)
    import rtgpu
    from oracle_bind import Oracle

    c = rtgpu.rtg_camera_desc.from_buffer_copy(cam)
    c.samples_per_pixel = spp
    sec, segs = Oracle().bench_f64(scene_desc, c, procs, H, row_step=row_step)
    return sec, segs, "port", "cpu_ref64"


def parity_rows(H, n):
    """n rows spread evenly over the frame as (first, step, count): a regular stride, so each CPU
    worker renders its share with one oracle call (one world build) as rows first + k*step."""
    n = max(1, min(n, H))
    step = H // n
    return (H - 1 - step * (n - 1)) // 2, step, n


def cpu_parity(scene_desc, cam, gpu_rows, first, step, seed, threads):
    """The metric's second half ("per-pixel RMSE vs CPU ref", north_star: < 1e-3 with matched
    per-pixel seeds): rows first + k*step of the benchmark frame the GPU rendered with `seed`
    (gpu_rows, host copy, linear fp32) against the oracle's fp32 spec (cpu_ref32) on the same seeds,
    dealt over `threads` CPU threads (ctypes releases the GIL). A checker of the cpu_baseline leg:
    nothing of the timed region comes from here."""
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np
    from oracle_bind import Oracle

    n = gpu_rows.shape[0]
    threads = max(1, min(threads, n))
    orc = Oracle()
    t0 = time.perf_counter()

    def part(t):  # worker t: rows k = t, t + threads, ...
        cnt = len(range(t, n, threads))
        return t, orc.render_f32(scene_desc, cam, seed=seed, row_begin=first + t * step,
                                 row_stride=step * threads, row_count=cnt)[0]

    ref = np.zeros_like(gpu_rows, dtype=np.float32)
    with ThreadPoolExecutor(threads) as ex:
        for t, rows in ex.map(part, range(threads)):
            ref[t::threads] = rows
    sec = time.perf_counter() - t0
    g = gpu_rows.astype(np.float64)
    err = g - ref.astype(np.float64)
    rmse = float(np.sqrt(np.mean(err ** 2)))
    return {"vs": "cpu_ref32 (oracle/cpu_ref.c, the fp32 spec of DESIGN.md section 4), same per-pixel seeds",
            "rows": n, "row_first": first, "row_step": step, "pixels": int(n * gpu_rows.shape[1]),
            "seed": seed, "rmse": rmse, "max_abs": float(np.max(np.abs(err))),
            "identical_frac": round(float(np.mean(np.all(gpu_rows == ref, axis=-1))), 6),
            "tolerance": 1e-3, "pass": bool(rmse < 1e-3 and np.all(np.isfinite(g))),
            "cpu_threads": threads, "seconds": round(sec, 3)}


def cpu_baseline(args, scene_desc, cam):
    """The reference timed on this host's cores: oracle/_ref/ref_harness (reference
    geometry, BVH, RNG and vector code compiled from /root/reference; camera/material loop
    restated, DESIGN.md 'ref-hybrid') if it was built, else the oracle's fp64 port (cpu_ref64).
    First one core on a row sample (~4 s, also the calibration), then every core of the host
    (bounded by the cgroup quota) for ~cpu_seconds on the whole frame. The rate is spp-invariant."""
    cores, model, online, quota = host_cpus()
    threads = args.cpu_threads or cores
    W, H = args.width, args.height
    # 1 core: every row_step-th row (~68 rows), spp grown until the sample takes >= 2.5 s
    step1, spp1 = max(1, H // 68), 1
    while True:
        sec1, segs1, kind, what = _cpu_run(args, scene_desc, cam, 1, spp1, step1)
        if sec1 >= 2.5 or spp1 >= 64:
            break
        spp1 = min(64, max(spp1 + 1, int(spp1 * 3.0 / max(sec1, 1e-3))))
    rate1 = segs1 / sec1
    rows1 = len(range(0, H, step1))
    rps = segs1 / (W * rows1 * spp1)  # segments per sample
    # all cores: the whole frame, spp sized for ~cpu_seconds of wall time at threads x rate1
    spp_all = max(1, int(round(args.cpu_seconds * rate1 * threads / (W * H * rps))))
    sec, segs, kind, what = _cpu_run(args, scene_desc, cam, threads, spp_all, 1)
    return {"value": round(segs / sec / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": kind,
            "sample": f"{args.scene} {W}x{H}, {spp_all} spp, depth {args.depth}, rows dealt over {threads} "
                      f"worker processes ({what})",
            "seconds": round(sec, 3), "segments": segs,
            "cpu_model": model, "host_cpus_online": online, "cgroup_cpu_quota": quota,
            "one_core": {"value": round(rate1 / 1e6, 3), "unit": "Mrays/s", "seconds": round(sec1, 3),
                         "segments": segs1,
                         "sample": f"{rows1} rows (every {step1}th), {spp1} spp, 1 process ({what})"}}


def _pmc_record(name, workload):
    """The record of `workload` in profiles/<name> (a {"records": [...]} file written by
    tools/pmc_report.py from rocprofv3 PMC passes of the same command; an older single-record file is
    read as one record), or None when that workload was not measured."""
    try:
        with open(os.path.join(REPO, "profiles", name)) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        return None
    for rec in doc.get("records", [doc]):
        if rec.get("workload") == workload:
            return rec
    return None


def pmc_traffic(workload):
    """HBM bytes per render launch (FETCH_SIZE x2 + WRITE_SIZE, separate passes, MI355X_MICROARCH.md
    §HBM), or None."""
    rec = _pmc_record("pmc_traffic.json", workload)
    return rec.get("hbm_bytes_per_launch") if rec else None


def pmc_binding(workload, kernel_s, plan):
    """The binding resource of the render kernel for this workload: VALU issue fraction, lane
    utilisation, wave-cycle split, LDS bank conflicts (profiles/pmc_binding.json), with the register
    count replaced by the compiled kernel's own (rtg_render_plan) and, where the counters could only
    see a different launch than the timed one (the dual launch: counter collection serialises its two
    dispatches), the issue fraction re-derived for the timed launch from the counted instructions."""
    rec = _pmc_record("pmc_binding.json", workload)
    if rec is None:
        return None
    rec = dict(rec)
    rec.pop("vgpr", None)  # rocprofv3's VGPR_Count is an allocation-granule field, not the count
    rec["vgprs"] = plan.get("vgprs")
    rec["timed_launch"] = {k: plan.get(k) for k in ("schedule", "workgroups", "waves_per_workgroup", "dual",
                                                     "dual_workgroups", "waves_per_simd", "vgprs", "dual_vgprs")}
    insts, clk = rec.get("sq_insts_valu_per_launch"), rec.get("effective_clock_ghz")
    if insts and clk and kernel_s > 0:
        issue = 2.0 * insts / (SIMDS * kernel_s * clk * 1e9)
        rec["valu_issue_frac_timed"] = round(issue, 4)
        if rec.get("valu_lane_utilization"):
            rec["useful_valu_frac_timed"] = round(issue * rec["valu_lane_utilization"], 4)
    return rec


class _Watchdog:
    """Runs fn() in this thread; if it has not returned after `seconds`, on_timeout() runs on a timer
    thread (it prints the line and ends the process: a hang in an optional check must not lose it)."""

    def __init__(self, seconds, on_timeout):
        import threading

        self.t = threading.Timer(seconds, on_timeout)
        self.t.daemon = True

    def __enter__(self):
        self.t.start()
        return self

    def __exit__(self, *exc):
        self.t.cancel()
        return False


LAUNCH_GUARD = "RTG_BENCH_LAUNCHED"  # set in the ranks bench.py starts itself (no second launch)


def self_launch(args):
    """`--gpus N` (N > 1) without a launcher: start the N ranks here, one process per GPU, as
    `python -m torch.distributed.run --nproc-per-node N bench.py ...` in a fresh child process, and
    return its exit code (rank 0's one JSON line goes straight to this process's stdout). Runs before
    torch is imported or any GPU is touched, and never execs: the driver's plain
    `bench.py --gpus 8` then measures eight ranks, not one. Returns None when no launch is needed."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    if os.environ.get(LAUNCH_GUARD):
        sys.exit(f"[bench] --gpus {args.gpus}: a rank started by bench.py has no WORLD_SIZE")
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, **{LAUNCH_GUARD: "1", "MASTER_ADDR": "127.0.0.1"})
    print(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def main():
    args = parse()
    rc = self_launch(args)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        # a launcher with a different rank count: the line would describe another job than asked for
        sys.exit(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: run with --gpus {world}, or without "
                 f"a launcher (bench.py starts its own ranks)")
    import numpy as np
    import torch
    import torch.distributed as dist

    import rtgpu
    gloo = args.dist_backend == "gloo"
    if gloo:
        if args.gather_impl == "rtg":
            sys.exit("--dist-backend gloo gathers through host memory: use --gather-impl torch")
        local = local % max(1, torch.cuda.device_count())  # several ranks may share one GPU
    elif local >= torch.cuda.device_count():
        # one rank per GPU over RCCL: a rank without its own device cannot join (RCCL refuses two ranks
        # on one GPU); --dist-backend gloo rehearses the flow with shared GPUs
        sys.exit(f"[bench] rank {rank}: LOCAL_RANK {local} but {torch.cuda.device_count()} visible GPU(s); "
                 f"--gpus {args.gpus} needs that many GPUs on the node (or --dist-backend gloo)")
    torch.cuda.set_device(local)
    if world > 1:
        if gloo:  # rehearsal of the N > 1 flow with several ranks on one GPU (tests/test_gpu.py)
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world,
                                    device_id=torch.device("cuda", local))

    lib = rtgpu.Library()
    scenes = rtgpu.SceneLibrary()
    bvh = {"sah": rtgpu.RTG_BVH_SAH, "median": rtgpu.RTG_BVH_MEDIAN, "gpu": rtgpu.RTG_BVH_GPU}[args.bvh]
    t0 = time.perf_counter()
    s = scenes.build(args.scene, grid=args.grid, image_width=args.width,
                     aspect_ratio=args.width / args.height, spp=args.spp, max_depth=args.depth,
                     bvh_mode=bvh, rand_seed=1)
    cam = s.camera
    t_scene = time.perf_counter() - t0
    params = lib.camera_resolve(cam)
    H, W = params.image_height, params.image_width
    t1 = time.perf_counter()
    ds = lib.scene_create(s.desc, device=local)
    t_create = time.perf_counter() - t1
    info = ds.info()
    b, stride, n, padded = lib.shard_layout(H, world, rank)
    # per-camera setup before the first frame (rtg_scene_prepare): the hot treelet of scenes that
    # render with the treelet schedule (config 5: a probe render and the node array renumbered)
    t2 = time.perf_counter()
    if n > 0:
        ds.prepare(cam, row_begin=b, row_stride=stride, row_count=n)
    t_prepare = time.perf_counter() - t2
    plan = ds.plan(cam, row_begin=b, row_stride=stride, row_count=n).as_dict() if n > 0 else {}
    shard = torch.zeros((padded, W, 3), dtype=torch.float32, device="cuda")
    shard8 = torch.zeros(shard.shape, dtype=torch.uint8, device="cuda") if args.gather == "rgb8" else None
    stream = torch.cuda.current_stream().cuda_stream
    comm, frame = None, None
    if world > 1 and args.gather_impl == "rtg":
        # one RCCL communicator of the C-ABI (rtg_comm_create_rank), its id shared over torch.distributed
        uid = [lib.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = lib.comm_rank(uid[0], world, rank, local)
        if rank == 0:
            frame = torch.zeros((H, W, 3), dtype=(torch.uint8 if shard8 is not None else torch.float32),
                                device="cuda")
    ev_g0, ev_g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    gathered = [None]  # the last gathered frame (rank 0, N > 1)
    # --gather-impl torch: every buffer of the timed gather allocated here, once (rtgpu.FrameGather: the
    # staging blocks and the frame on rank 0, the de-interleave by the library's own kernel); gloo
    # rehearsals stage the shard through one pinned host buffer
    fgather, host_src = None, None
    if world > 1 and comm is None:
        gsrc = shard8 if shard8 is not None else shard
        if gloo:
            host_src = torch.empty(gsrc.shape, dtype=gsrc.dtype, pin_memory=True)
        fgather = rtgpu.FrameGather(lib, host_src if gloo else gsrc, H, dst=0, device=local)

    def step(i, evs=None):
        # a rank past the image's last row renders nothing (its shard stays zero padding)
        st = (ds.render_device(cam, shard.data_ptr(), stream, seed=args.seed + i, row_begin=b,
                               row_stride=stride, row_count=n) if n > 0 else rtgpu.rtg_render_stats())
        if shard8 is not None:  # write_color on the device (rtg_resolve_rgb8), gather the bytes
            ds.resolve_rgb8(shard.data_ptr(), shard8.data_ptr(), shard.shape[0] * W, stream)
        if world > 1:
            src = shard8 if shard8 is not None else shard
            g0, g1 = evs if evs is not None else (ev_g0, ev_g1)
            g0.record()
            if comm is not None:  # ncclGather to rank 0 + the de-interleave kernel there (rtg_gather_rows)
                comm.gather_rows([src.data_ptr()], H, W * 3 * src.element_size(), 0,
                                 frame.data_ptr() if frame is not None else 0, [stream])
                gathered[0] = frame
            elif gloo:
                host_src.copy_(src)
                gathered[0] = fgather(host_src)
            else:
                gathered[0] = fgather(src, stream)
            g1.record()
        return st

    for i in range(args.warmup):
        step(i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    segs, kernel_ms, st = 0, [], None
    # one event pair per timed step around the gather, on the render stream (torch's current stream)
    gev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)] if world > 1 else [None] * args.steps
    for i in range(args.steps):
        st = step(args.warmup + i, gev[i])
        segs += st.segments
        kernel_ms.append(st.kernel_ms)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    gather_ms = [a.elapsed_time(b_) for a, b_ in gev] if world > 1 else []
    # host copy of the last timed frame (seed args.seed + warmup + steps - 1), for the per-pixel check
    want_parity = not args.no_cpu_baseline and args.parity_seconds > 0
    last_frame = None
    if want_parity:
        if world == 1:
            last_frame = shard[:H].cpu().numpy()
        elif rank == 0 and gathered[0] is not None:
            last_frame = gathered[0].cpu().numpy()

    tot = torch.tensor([float(segs)], dtype=torch.float64, device="cpu" if gloo else "cuda")
    tmax = torch.tensor([dt], dtype=torch.float64, device="cpu" if gloo else "cuda")
    if world > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    total_segs, wall = float(tot.item()), float(tmax.item())

    # algorithmic bytes of one launch (counting variant of the same kernel, same seed, untimed)
    cst = (ds.render_device(cam, shard.data_ptr(), stream, seed=args.seed + args.warmup, row_begin=b,
                            row_stride=stride, row_count=n, count=True) if n > 0 else rtgpu.rtg_render_stats())
    algo_bytes = (BYTES_PER_BOX * cst.box_tests + BYTES_PER_PRIM * cst.prim_tests
                  + BYTES_PER_HIT * cst.hits)
    avg_kernel_s = max(sum(kernel_ms) / len(kernel_ms) / 1e3, 1e-9)
    achieved = algo_bytes / avg_kernel_s / 1e9
    workload = (f"{args.scene}(grid={args.grid}) {W}x{H} {args.spp}spp depth{args.depth} bvh={args.bvh} "
                f"chunk={rtgpu.chunk_samples(args.spp)}")
    traffic = pmc_traffic(workload) if world == 1 else None
    setup_ms = {"scene_build_ms": round(t_scene * 1e3, 1), "scene_create_ms": round(t_create * 1e3, 1),
                "host_compile_ms": round(info.build_ms, 1), "bvh_ms": round(info.bvh_ms, 1),
                "collapse_ms": round(info.collapse_ms, 1), "flatten_ms": round(info.flatten_ms, 1),
                "upload_ms": round(info.upload_ms, 1), "prepare_ms": round(t_prepare * 1e3, 1)}
    my = {"rank": rank, "device": local, "rows": n, "row_begin": b, "row_stride": stride,
          "segments": int(segs), "kernel_ms": round(sum(kernel_ms) / len(kernel_ms), 3),
          "kernel_ms_max": round(max(kernel_ms), 3),
          "gather_ms": round(sum(gather_ms) / len(gather_ms), 3) if gather_ms else None,
          "gather_ms_max": round(max(gather_ms), 3) if gather_ms else None,
          "wall_s": round(dt, 4), "setup_ms": round((t_scene + t_create + t_prepare) * 1e3, 1),
          "vgprs": plan.get("vgprs"), "schedule": plan.get("schedule")}
    ranks = [my]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, my)

    line = None
    if rank == 0:
        samples = W * H * args.spp * args.steps
        lds = {"achieved": round(achieved, 2), "peak": LDS_PEAK_GBS, "unit": "GB/s",
               "frac": round(achieved / LDS_PEAK_GBS, 4),
               "note": "the same algorithmic bytes against the ds_read_b128 aggregate (MI355X_MICROARCH.md "
                       "§LDS): the scene is LDS-resident for configs 2-4 (config 5: the top of the tree)"}
        binding = pmc_binding(workload, avg_kernel_s, plan) if world == 1 else None
        line = {
            "metric": METRIC,
            "value": round(total_segs / wall / 1e6, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic (the reference's scene regenerated from glibc rand seed 1"
                     + (", earthmap texels from tests/golden" if args.scene.startswith("earth") else "") + ")"),
            "config": {"workload": workload, "baseline_config": args.config, "scene": args.scene,
                       "grid": args.grid, "width": W,
                       "height": H, "spp": args.spp, "depth": args.depth, "bvh": args.bvh,
                       "parallelism": (f"rows interleaved over {world} GPUs, one RCCL gather ({args.gather}, "
                                       f"{'rtg_gather_rows' if args.gather_impl == 'rtg' else 'torch.distributed'}) "
                                       f"of the frame to rank 0 per step" if world > 1 else
                                       "1 GPU, whole frame (no gather)")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "traffic_gbs": (round(traffic / avg_kernel_s / 1e9, 2) if traffic else None),
                         "lds": lds,
                         "useful_valu_frac": (binding or {}).get("useful_valu_frac_timed",
                                                                 (binding or {}).get("useful_valu_frac")),
                         "note": ("frac > 1: the algorithmic bytes are served on chip (LDS-resident scene, "
                                  "or L2/MALL for scenes too large for LDS), so the HBM fraction is not the "
                                  "bound; `lds.frac` prices the same bytes against the LDS read aggregate and "
                                  "`useful_valu_frac` is the fraction of the chip's fp32 lane-issue slots doing "
                                  "path-tracing work in the timed launch (binding: VALU issue x lane "
                                  "utilisation, DESIGN.md section 6); traffic = PMC-measured HBM bytes per "
                                  "launch (null when not measured for this workload)"),
                         "binding": binding,
                         "kernel_ms": round(avg_kernel_s * 1e3, 3),
                         "algorithmic_bytes_per_launch": int(algo_bytes),
                         "per_segment": {"box_tests": round(cst.box_tests / max(cst.segments, 1), 3),
                                         "prim_tests": round(cst.prim_tests / max(cst.segments, 1), 3),
                                         "hit_frac": round(cst.hits / max(cst.segments, 1), 4),
                                         # pushes into the global spill area (4-B store + 4-B load each)
                                         "stack_spills": round(cst.stack_spills / max(cst.segments, 1), 4)}},
            "launch": plan,
            "msamples_per_s": round(samples / wall / 1e6, 3),
            "rays_per_sample": round(total_segs / samples, 4),
            "setup_ms": round((t_scene + t_create + t_prepare) * 1e3, 1),
            "setup": setup_ms,
            # rtg_scene_prepare's cost-ordered tile hand-out (DESIGN.md §3 "tile order"): whether the timed
            # frames used it (rank 0's last step) and its probe's host + device time within setup.prepare_ms
            "tile_order": ({"used": bool(st.tile_order), "tune_ms": round(st.tile_order_tune_us / 1e3, 2)}
                           if st is not None else None),
            "scene_build_ms": round(t_scene * 1e3, 1),
            "bvh": {"nodes": info.num_nodes, "depth": info.bvh_depth, "build_ms": round(info.build_ms, 1),
                    "upload_ms": round(info.upload_ms, 1)},
            "cpu_baseline": None,
        }
        if world > 1:
            line["ranks"] = ranks
            line["gather_ms"] = [r["gather_ms"] for r in ranks]
            line["kernel_ms_per_rank"] = [r["kernel_ms"] for r in ranks]
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args, s.desc, cam)
            cb = line["cpu_baseline"]
            line["speedup_vs_cpu"] = round(line["value"] / cb["value"], 1) if cb["value"] else None
            line["speedup_vs_cpu_one_core"] = (round(line["value"] / cb["one_core"]["value"], 1)
                                               if cb["one_core"]["value"] else None)
            # the same ratio against every CPU the host has online, extrapolated linearly from the
            # one-core rate (the box's cgroup grants only cb["cores"] of them): an upper bound on what
            # the whole host could do, next to the measured ratios
            online = cb.get("host_cpus_online") or 0
            if cb["one_core"]["value"] and online:
                lin = cb["one_core"]["value"] * online
                line["speedup_vs_cpu_all_host_cores_linear"] = {
                    "cores": online, "cpu_value": round(lin, 1), "speedup": round(line["value"] / lin, 1)}
        if last_frame is not None:
            cores = host_cpus()[0]
            cb = line["cpu_baseline"]
            # rows sized for ~parity_seconds on the cores at the measured one-core rate (the fp32 spec
            # runs at about the reference's speed; 2.5 Mrays/s per core assumed
            # where no CPU baseline was timed, i.e. N > 1), 2..128 rows
            rate1 = cb["one_core"]["value"] if cb else 2.5
            per_row = W * args.spp * max(line["rays_per_sample"], 1.0)
            nrows = int(args.parity_seconds * cores * rate1 * 1e6 / per_row)
            first, pstep, nrows = parity_rows(H, max(2, min(128, nrows)))
            rows = last_frame[first::pstep][:nrows]
            seed_last = args.seed + args.warmup + args.steps - 1
            if last_frame.dtype == np.uint8:  # --gather rgb8: write_color bytes against the oracle's
                line["parity"] = cpu_parity_rgb8(s.desc, cam, rows, first, pstep, seed_last, cores)
            else:
                line["parity"] = cpu_parity(s.desc, cam, rows, first, pstep, seed_last, cores)
            if world > 1:
                line["parity"]["frame"] = f"gathered on rank 0 from {world} ranks"

    if world > 1 and not args.no_rtg_check and not gloo:
        # the C-ABI's RCCL gather, outside the timed region, on the last frame's shards, once per timed step:
        # its per-call time beside the timed torch gather's, and byte-compared with the timed frame
        def give_up():
            if rank == 0:
                line["rtg_gather_check"] = {"status": f"timeout after {args.check_timeout:.0f} s"}
                print(json.dumps(line), flush=True)
            os._exit(0)

        with _Watchdog(args.check_timeout, give_up):
            line_check = rtg_gather_check(lib, dist, torch, world, rank, local, H, W,
                                          shard8 if shard8 is not None else shard,
                                          gathered[0] if rank == 0 else None, stream, args.steps)
        if rank == 0:
            line["rtg_gather_check"] = line_check
    if rank == 0:
        print(json.dumps(line), flush=True)
    if comm is not None:
        torch.cuda.synchronize()
        comm.close()
    ds.close()
    if world > 1:
        dist.destroy_process_group()


def rtg_gather_check(lib, dist, torch, world, rank, local, H, W, src, timed_frame, stream, calls):
    """The C-ABI's own gather (rtg_gather_rows through rtg_comm_create_rank; the id broadcast over
    torch.distributed) of this rank's last shard into a fresh frame on rank 0, once per timed step
    (`calls`), each call timed with an event pair on the render stream like the timed torch gather:
    the product gather's time beside torch's, and the library's allocation count across the calls (0
    after the first: the communicator keeps its staging buffer). The frame is compared byte for byte
    with the one the timed loop gathered. Returns the check record on rank 0."""
    t0 = time.perf_counter()
    uid = [lib.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    comm = lib.comm_rank(uid[0], world, rank, local)
    try:
        ranks_seen = comm.size()[0]
        out = torch.zeros((H, W, 3), dtype=src.dtype, device="cuda") if rank == 0 else None
        torch.cuda.synchronize()
        calls = max(1, calls)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(calls)]
        allocs = []
        for e0, e1 in ev:
            e0.record()
            comm.gather_rows([src.data_ptr()], H, W * 3 * src.element_size(), 0,
                             out.data_ptr() if out is not None else 0, [stream])
            e1.record()
            allocs.append(lib.allocation_count()[0])
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in ev]
        rec = None
        if rank == 0:
            same = bool(torch.equal(out, timed_frame)) if timed_frame is not None else None
            later = ms[1:] or ms
            rec = {"status": "ok", "impl": "rtg_gather_rows (ncclGather + de-interleave kernel)",
                   "ranks_seen": ranks_seen, "identical_to_timed_frame": same, "calls": calls,
                   "gather_ms_first": round(ms[0], 3),
                   "gather_ms": round(sum(later) / len(later), 3), "gather_ms_max": round(max(later), 3),
                   "allocations_after_first_call": allocs[-1] - allocs[0],
                   "seconds_incl_comm_init": round(time.perf_counter() - t0, 3)}
        dist.barrier()
        return rec
    finally:
        comm.close()


def cpu_parity_rgb8(scene_desc, cam, rows8, first, step, seed, threads):
    """--gather rgb8: the gathered write_color bytes against write_color of the oracle's rows."""
    import numpy as np

    import rtgpu

    from oracle_bind import Oracle

    orc = Oracle()
    ref = np.concatenate([orc.render_f32(scene_desc, cam, seed=seed, row_begin=first + k * step, row_stride=step,
                                         row_count=1)[0] for k in range(rows8.shape[0])])
    ref8 = rtgpu.write_color_bytes(ref)
    diff = np.abs(rows8.astype(np.int32) - ref8.astype(np.int32))
    return {"vs": "write_color(cpu_ref32) bytes", "rows": int(rows8.shape[0]), "row_first": first, "row_step": step,
            "identical_frac": round(float(np.mean(diff == 0)), 6), "max_abs_lsb": int(diff.max()),
            "pass": bool(diff.max() <= 1)}


if __name__ == "__main__":
    main()
