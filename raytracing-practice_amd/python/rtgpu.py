"""rtgpu.py — Python binding of the MI355X path tracer's C-ABI (include/rtgpu.h) via ctypes.

Layers it exposes:
  * the structs of include/rtgpu.h (rtg_primitive, rtg_scene_desc, rtg_camera_desc, ...)
  * :class:`Library` — librtgpu.so (device scene + render kernels); raises RtgError on failure,
    never falls back to a CPU path
  * :class:`SceneLibrary` — librtscenes.so, the reference's scenes built with the C++ API mirror
  * :func:`shard_rows` / :func:`deinterleave` — the interleaved-row tiling used across GPUs

Reference mapping: camera::render (src/core/camera.hpp:29-72) is rtg_render over all rows;
the per-GPU shard of rows r, r+N, r+2N, ... is the multi-GPU split of SURVEY.md §8e.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_DIR = os.path.join(PKG_DIR, "lib")

RTG_ABI_VERSION = 7
RTG_OK = 0
RTG_E_INVALID, RTG_E_HIP, RTG_E_NODEVICE, RTG_E_NOMEM, RTG_E_UNSUPPORTED = -1, -2, -3, -4, -5
RTG_PRIM_SPHERE, RTG_PRIM_QUAD = 1, 2
RTG_MAT_LAMBERTIAN, RTG_MAT_METAL, RTG_MAT_DIELECTRIC, RTG_MAT_DIFFUSE_LIGHT = 1, 2, 3, 4
RTG_TEX_SOLID, RTG_TEX_CHECKER, RTG_TEX_IMAGE, RTG_TEX_NOISE = 1, 2, 3, 4
RTG_BVH_MEDIAN, RTG_BVH_SAH, RTG_BVH_GPU = 0, 1, 3
RTG_RENDER_OUT_DEVICE, RTG_RENDER_ASYNC, RTG_RENDER_COUNT = 0x1, 0x2, 0x4


def RTG_RENDER_SCHEDULE(n: int) -> int:  # diagnostic kernel-schedule selector (include/rtgpu.h)
    return (n & 0xFF) << 8


def RTG_RENDER_SHADE_BATCH(n: int) -> int:
    return (n & 0xFF) << 16


def RTG_RENDER_LEAF_BATCH(n: int) -> int:
    return (n & 0x7F) << 24
DEFAULT_SEED = 0x5EED

D3 = C.c_double * 3


class rtg_primitive(C.Structure):
    _fields_ = [("kind", C.c_int32), ("material", C.c_int32), ("p0", D3), ("p1", D3), ("p2", D3),
                ("radius", C.c_double)]


class rtg_material(C.Structure):
    _fields_ = [("type", C.c_int32), ("texture", C.c_int32), ("albedo", D3), ("fuzz", C.c_double),
                ("refraction_index", C.c_double)]


class rtg_texture(C.Structure):
    _fields_ = [("type", C.c_int32), ("even", C.c_int32), ("odd", C.c_int32), ("image", C.c_int32),
                ("perlin", C.c_int32), ("pad_", C.c_int32), ("scale", C.c_double), ("color", D3)]


class rtg_image(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("rgb", C.POINTER(C.c_uint8))]


class rtg_perlin(C.Structure):
    _fields_ = [("randvec", (C.c_double * 3) * 256), ("perm_x", C.c_int32 * 256),
                ("perm_y", C.c_int32 * 256), ("perm_z", C.c_int32 * 256)]


class rtg_scene_desc(C.Structure):
    _fields_ = [("abi_version", C.c_uint32), ("bvh_mode", C.c_int32),
                ("prims", C.POINTER(rtg_primitive)), ("num_prims", C.c_int64),
                ("materials", C.POINTER(rtg_material)), ("num_materials", C.c_int32),
                ("num_textures", C.c_int32), ("textures", C.POINTER(rtg_texture)),
                ("images", C.POINTER(rtg_image)), ("num_images", C.c_int32),
                ("num_perlins", C.c_int32), ("perlins", C.POINTER(rtg_perlin)),
                ("tie_rank", C.POINTER(C.c_int64))]  # ABI 7: the reference's test order (NULL: list order)


class rtg_camera_desc(C.Structure):
    _fields_ = [("aspect_ratio", C.c_double), ("image_width", C.c_int32),
                ("samples_per_pixel", C.c_int32), ("max_depth", C.c_int32), ("pad_", C.c_int32),
                ("background", D3), ("vfov", C.c_double), ("lookfrom", D3), ("lookat", D3),
                ("vup", D3), ("defocus_angle", C.c_double), ("focus_dist", C.c_double)]


class rtg_camera_params(C.Structure):
    _fields_ = [("image_width", C.c_int32), ("image_height", C.c_int32),
                ("pixel_samples_scale", C.c_double), ("center", D3), ("pixel00_loc", D3),
                ("pixel_delta_u", D3), ("pixel_delta_v", D3), ("u", D3), ("v", D3), ("w", D3),
                ("defocus_disk_u", D3), ("defocus_disk_v", D3)]


class rtg_render_desc(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("row_begin", C.c_int32), ("row_stride", C.c_int32),
                ("row_count", C.c_int32), ("flags", C.c_int32), ("stream", C.c_void_p),
                ("partial", C.c_void_p), ("chunk_begin", C.c_int32), ("chunk_count", C.c_int32)]


class rtg_render_stats(C.Structure):
    _fields_ = [("segments", C.c_uint64), ("samples", C.c_uint64), ("box_tests", C.c_uint64),
                ("prim_tests", C.c_uint64), ("hits", C.c_uint64), ("kernel_ms", C.c_double),
                ("diag", C.c_uint64 * 16), ("stack_spills", C.c_uint64), ("tile_order", C.c_uint32),
                ("tile_order_tune_us", C.c_uint32), ("reserved_", C.c_uint64 * 2)]


class rtg_scene_info(C.Structure):
    _fields_ = [("device", C.c_int32), ("bvh_mode", C.c_int32), ("num_prims", C.c_int64),
                ("num_nodes", C.c_int64), ("bvh_depth", C.c_int32), ("stack_depth", C.c_int32),
                ("device_bytes", C.c_int64), ("build_ms", C.c_double), ("upload_ms", C.c_double),
                ("bvh_ms", C.c_double), ("collapse_ms", C.c_double), ("flatten_ms", C.c_double)]


class rtg_launch_plan(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "schedule", "workgroups", "waves_per_workgroup", "lds_bytes", "vgprs", "sgprs", "scratch_bytes",
        "waves_per_simd", "dual", "dual_workgroups", "dual_lds_bytes", "dual_vgprs", "stack_entry_bytes",
        "lds_stack_entries", "spill_entries", "treelet_nodes", "shade_batch", "leaf_batch", "chunk_samples",
        "chunks")] + [("partial_bytes", C.c_int64), ("num_cus", C.c_int32), ("tile_slots", C.c_int32),
                      ("treelet_hot", C.c_int32), ("treelet_tune_us", C.c_int32),
                      ("treelet_visit_permille", C.c_int32), ("ray_queue", C.c_int32),
                      ("node_width", C.c_int32), ("origin_bound", C.c_int32)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_ if n != "reserved_"}


class rtg_bvh_node_host(C.Structure):
    _fields_ = [("lo", (C.c_double * 3) * 2), ("hi", (C.c_double * 3) * 2),
                ("child", C.c_int32 * 2), ("count", C.c_int32 * 2)]


class rts_params(C.Structure):
    _fields_ = [("grid", C.c_int32), ("image_width", C.c_int32), ("aspect_ratio", C.c_double),
                ("samples_per_pixel", C.c_int32), ("max_depth", C.c_int32),
                ("bvh_mode", C.c_int32), ("rand_seed", C.c_uint32)]


# exported symbols of librtgpu.so (must match include/rtgpu.h)
RTG_SYMBOLS = ("rtg_abi_version", "rtg_last_error", "rtg_device_count", "rtg_camera_resolve",
               "rtg_scene_create", "rtg_scene_get_info", "rtg_scene_destroy", "rtg_render",
               "rtg_render_wait", "rtg_resolve_rgb8", "rtg_bvh_build_host", "rtg_comm_create_local",
               "rtg_comm_unique_id", "rtg_comm_create_rank", "rtg_comm_size", "rtg_comm_destroy",
               "rtg_gather_rows", "rtg_deinterleave_rows", "rtg_render_frame", "rtg_render_plan",
               "rtg_shard_layout", "rtg_deinterleave_rows_host", "rtg_scene_prepare",
               "rtg_hot_treelet_order_host", "rtg_bvh_node_order",
               "rtg_allocation_count")
RTG_COMM_ID_BYTES = 128


class RtgError(RuntimeError):
    def __init__(self, call: str, status: int, message: str):
        super().__init__(f"{call} failed ({status}): {message}")
        self.status = status


def _P(t):
    return C.POINTER(t)


def chunk_samples(spp: int) -> int:
    """rtgpu.h rtg_chunk_samples: samples per accumulation chunk of the rtg-f32 spec."""
    n = max(1, (spp + 15) // 16)  # RTG_CHUNK_MAX
    return (spp + n - 1) // n if spp > 0 else 1


def num_chunks(spp: int) -> int:
    """rtgpu.h rtg_num_chunks: accumulation chunks of a pixel (progressive-rendering units)."""
    k = chunk_samples(spp)
    return (spp + k - 1) // k if spp > 0 else 1


def _one_hip_runtime():
    """Load torch (when installed) before librtgpu.so, so the process holds ONE HIP runtime.

    torch's wheel bundles its own libamdhip64; librtgpu.so links the system one under the same
    soname. Loaded first, torch's copy also serves librtgpu.so and device pointers, streams and
    events pass between the two freely. Loaded the other way round, the system runtime initialises the
    device first and torch's later initialisation fails ("No HIP GPUs are available", MI355X box,
    torch 2.10+rocm7.0 beside ROCm 7.2)."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


class Library:
    """librtgpu.so. Loading it requires the built library (make -C raytracing-practice_amd)."""

    def __init__(self, path: Optional[str] = None):
        # RTGPU_LIB: an alternative build of the library (same-box A/B runs, tools/); default the in-tree one
        path = path or os.environ.get("RTGPU_LIB") or os.path.join(LIB_DIR, "librtgpu.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} not built (run __graft_entry__.build())")
        self.path = path
        _one_hip_runtime()
        L = self.lib = C.CDLL(path)
        L.rtg_abi_version.restype = C.c_uint32
        L.rtg_last_error.restype = C.c_char_p
        L.rtg_device_count.argtypes = [_P(C.c_int32)]
        L.rtg_camera_resolve.argtypes = [_P(rtg_camera_desc), _P(rtg_camera_params)]
        L.rtg_scene_create.argtypes = [_P(rtg_scene_desc), C.c_int32, _P(C.c_void_p)]
        L.rtg_scene_get_info.argtypes = [C.c_void_p, _P(rtg_scene_info)]
        L.rtg_scene_destroy.argtypes = [C.c_void_p]
        L.rtg_scene_destroy.restype = None
        L.rtg_render.argtypes = [C.c_void_p, _P(rtg_camera_desc), _P(rtg_render_desc), C.c_void_p,
                                 _P(rtg_render_stats)]
        L.rtg_render_wait.argtypes = [C.c_void_p, _P(rtg_render_stats)]
        L.rtg_resolve_rgb8.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
        L.rtg_bvh_build_host.argtypes = [_P(rtg_scene_desc), _P(rtg_bvh_node_host), C.c_int64,
                                         _P(C.c_int64), C.c_int64, _P(C.c_int64), _P(C.c_int64),
                                         _P(C.c_int32)]
        L.rtg_comm_create_local.argtypes = [_P(C.c_int32), C.c_int32, _P(C.c_void_p)]
        L.rtg_comm_unique_id.argtypes = [C.c_void_p]
        L.rtg_comm_create_rank.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, _P(C.c_void_p)]
        L.rtg_comm_size.argtypes = [C.c_void_p, _P(C.c_int32), _P(C.c_int32)]
        L.rtg_comm_destroy.argtypes = [C.c_void_p]
        L.rtg_comm_destroy.restype = None
        L.rtg_gather_rows.argtypes = [C.c_void_p, _P(C.c_void_p), C.c_int32, C.c_int64, C.c_int32, C.c_void_p,
                                      _P(C.c_void_p)]
        L.rtg_deinterleave_rows.argtypes = [C.c_int32, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int64,
                                            C.c_void_p]
        L.rtg_render_frame.argtypes = [C.c_void_p, _P(C.c_void_p), _P(rtg_camera_desc), C.c_uint64, C.c_int32,
                                       C.c_void_p, _P(rtg_render_stats)]
        L.rtg_render_plan.argtypes = [C.c_void_p, _P(rtg_camera_desc), _P(rtg_render_desc), _P(rtg_launch_plan)]
        L.rtg_scene_prepare.argtypes = [C.c_void_p, _P(rtg_camera_desc), _P(rtg_render_desc)]
        L.rtg_hot_treelet_order_host.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.rtg_shard_layout.argtypes = [C.c_int32, C.c_int32, C.c_int32] + [_P(C.c_int32)] * 4
        L.rtg_deinterleave_rows_host.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int64]
        L.rtg_bvh_node_order.argtypes = [C.c_void_p, C.c_int64, C.c_void_p]
        L.rtg_allocation_count.argtypes = [_P(C.c_uint64), _P(C.c_uint64)]
        for name in ("rtg_device_count", "rtg_camera_resolve", "rtg_scene_create",
                     "rtg_scene_get_info", "rtg_render", "rtg_render_wait", "rtg_resolve_rgb8",
                     "rtg_bvh_build_host", "rtg_comm_create_local", "rtg_comm_unique_id",
                     "rtg_comm_create_rank", "rtg_comm_size", "rtg_gather_rows", "rtg_deinterleave_rows",
                     "rtg_render_frame", "rtg_render_plan", "rtg_shard_layout", "rtg_deinterleave_rows_host",
                     "rtg_bvh_node_order", "rtg_allocation_count"):
            getattr(L, name).restype = C.c_int32
        if L.rtg_abi_version() != RTG_ABI_VERSION:
            raise RuntimeError("librtgpu ABI version mismatch")

    def check(self, call: str, status: int) -> None:
        if status != RTG_OK:
            raise RtgError(call, status, (self.lib.rtg_last_error() or b"").decode())

    def device_count(self) -> int:
        n = C.c_int32(0)
        st = self.lib.rtg_device_count(C.byref(n))
        return n.value if st == RTG_OK else 0

    def camera_resolve(self, cam: rtg_camera_desc) -> rtg_camera_params:
        out = rtg_camera_params()
        self.check("rtg_camera_resolve", self.lib.rtg_camera_resolve(C.byref(cam), C.byref(out)))
        return out

    def bvh_build_host(self, desc: rtg_scene_desc):
        """Topology of the BVH the library builds for `desc` (host only, no GPU)."""
        nn, nr, depth = C.c_int64(0), C.c_int64(0), C.c_int32(0)
        self.check("rtg_bvh_build_host", self.lib.rtg_bvh_build_host(
            C.byref(desc), None, 0, None, 0, C.byref(nn), C.byref(nr), C.byref(depth)))
        nodes = (rtg_bvh_node_host * max(nn.value, 1))()
        refs = (C.c_int64 * max(nr.value, 1))()
        self.check("rtg_bvh_build_host", self.lib.rtg_bvh_build_host(
            C.byref(desc), nodes, nn.value, refs, nr.value, C.byref(nn), C.byref(nr), C.byref(depth)))
        return list(nodes)[:nn.value], list(refs)[:nr.value], depth.value

    def bvh_node_order(self, boxes):
        """rtg_bvh_node_order: list indices in bvh_node(objects, 0, n)'s leaf order, for n object boxes
        given as an (n, 6) array {lo.xyz, hi.xyz} in list order (bvh_node.hpp:25-77; host only)."""
        import numpy as np

        b = np.ascontiguousarray(boxes, dtype=np.float64).reshape(-1, 6)
        out = np.empty(len(b), dtype=np.int64)
        self.check("rtg_bvh_node_order", self.lib.rtg_bvh_node_order(b.ctypes.data, len(b), out.ctypes.data))
        return out

    def allocation_count(self):
        """rtg_allocation_count: (allocations, bytes) the library made in this process so far."""
        n, b = C.c_uint64(0), C.c_uint64(0)
        self.check("rtg_allocation_count", self.lib.rtg_allocation_count(C.byref(n), C.byref(b)))
        return n.value, b.value

    def scene_create(self, desc: rtg_scene_desc, device: int = 0) -> "DeviceScene":
        h = C.c_void_p()
        self.check("rtg_scene_create", self.lib.rtg_scene_create(C.byref(desc), device, C.byref(h)))
        return DeviceScene(self, h)

    # ---- multi-GPU frames (rtgpu.h: rtg_comm_*, rtg_gather_rows, rtg_render_frame) ----
    def comm_local(self, devices: Sequence[int]) -> "Comm":
        """One process driving `devices` (ranks 0..N-1), ncclCommInitAll."""
        arr = (C.c_int32 * len(devices))(*devices)
        h = C.c_void_p()
        self.check("rtg_comm_create_local", self.lib.rtg_comm_create_local(arr, len(devices), C.byref(h)))
        return Comm(self, h)

    def comm_unique_id(self) -> bytes:
        buf = (C.c_uint8 * RTG_COMM_ID_BYTES)()
        self.check("rtg_comm_unique_id", self.lib.rtg_comm_unique_id(buf))
        return bytes(buf)

    def comm_rank(self, uid: bytes, nranks: int, rank: int, device: int) -> "Comm":
        """One rank of a one-process-per-GPU communicator (uid from comm_unique_id on rank 0)."""
        buf = (C.c_uint8 * RTG_COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        self.check("rtg_comm_create_rank", self.lib.rtg_comm_create_rank(buf, nranks, rank, device, C.byref(h)))
        return Comm(self, h)

    def shard_layout(self, height: int, nranks: int, rank: int):
        """rtg_shard_layout: (row_begin, row_stride, row_count, padded_rows) of rank's interleaved shard
        (host only; the arithmetic rtg_render_frame / rtg_gather_rows use)."""
        v = [C.c_int32(0) for _ in range(4)]
        self.check("rtg_shard_layout", self.lib.rtg_shard_layout(height, nranks, rank, *[C.byref(x) for x in v]))
        return tuple(x.value for x in v)

    def hot_treelet_order_host(self, nodes, visits):
        """rtg_hot_treelet_order_host: a copy of `nodes` ((n, 28) int32 device-format 4-wide records)
        renumbered as rtg_scene_prepare does (root first, then by descending visits)."""
        import numpy as np

        out = np.ascontiguousarray(nodes, dtype=np.int32).copy()
        v = np.ascontiguousarray(visits, dtype=np.uint32)
        assert out.ndim == 2 and out.shape[1] == 28 and v.shape == (out.shape[0],)
        self.check("rtg_hot_treelet_order_host", self.lib.rtg_hot_treelet_order_host(
            out.ctypes.data, v.ctypes.data, out.shape[0]))
        return out

    def deinterleave_rows_host(self, gathered, nranks: int, height: int):
        """rtg_deinterleave_rows_host on a host array of nranks blocks of padded rows (row = last axes):
        returns the (height, ...) image in row order (same index function as the device kernel)."""
        import numpy as np

        g = np.ascontiguousarray(gathered)
        padded = (height + nranks - 1) // nranks
        rows = g.reshape(nranks * padded, -1)
        out = np.empty((height,) + g.shape[1:], dtype=g.dtype)
        self.check("rtg_deinterleave_rows_host", self.lib.rtg_deinterleave_rows_host(
            g.ctypes.data, out.ctypes.data, nranks, height, rows.shape[1] * g.itemsize))
        return out

    def deinterleave_rows(self, device: int, gathered_ptr: int, out_ptr: int, nranks: int, height: int,
                          row_bytes: int, stream_ptr: Optional[int] = None) -> None:
        self.check("rtg_deinterleave_rows", self.lib.rtg_deinterleave_rows(
            device, C.c_void_p(gathered_ptr), C.c_void_p(out_ptr), nranks, height, row_bytes,
            C.c_void_p(stream_ptr) if stream_ptr else None))


class Comm:
    """rtg_comm*: RCCL communicator over the GPUs a frame is tiled across."""

    def __init__(self, lib: Library, handle: C.c_void_p):
        self.L = lib
        self.handle = handle

    def size(self):
        n, nl = C.c_int32(0), C.c_int32(0)
        self.L.check("rtg_comm_size", self.L.lib.rtg_comm_size(self.handle, C.byref(n), C.byref(nl)))
        return n.value, nl.value

    def gather_rows(self, shard_ptrs: Sequence[int], height: int, row_bytes: int, root: int, out_ptr: int,
                    stream_ptrs: Optional[Sequence[int]] = None) -> None:
        """Enqueue the RCCL gather of this process's shards (device pointers, one per local rank)
        and the de-interleave into out_ptr on the root (asynchronous on the given streams)."""
        n = len(shard_ptrs)
        sh = (C.c_void_p * n)(*shard_ptrs)
        st = (C.c_void_p * n)(*(stream_ptrs or [0] * n))
        self.L.check("rtg_gather_rows", self.L.lib.rtg_gather_rows(self.handle, sh, height, row_bytes, root,
                                                                    C.c_void_p(out_ptr), st))

    def render_frame(self, scenes: Sequence["DeviceScene"], cam: rtg_camera_desc, seed: int = DEFAULT_SEED,
                     root: int = 0):
        """Whole frame over the communicator's local GPUs (rtg_render_frame): (H, W, 3) on the root."""
        import numpy as np

        p = self.L.camera_resolve(cam)
        out = np.zeros((p.image_height, p.image_width, 3), dtype=np.float32)
        arr = (C.c_void_p * len(scenes))(*[s.handle.value if isinstance(s.handle, C.c_void_p) else s.handle
                                           for s in scenes])
        stats = rtg_render_stats()
        self.L.check("rtg_render_frame", self.L.lib.rtg_render_frame(self.handle, arr, C.byref(cam), seed, root,
                                                                      out.ctypes.data, C.byref(stats)))
        return out, stats

    def close(self) -> None:
        if self.handle:
            self.L.lib.rtg_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceScene:
    """A scene resident in HBM on one device (rtg_scene*)."""

    def __init__(self, lib: Library, handle: C.c_void_p):
        self.L = lib
        self.handle = handle

    def info(self) -> rtg_scene_info:
        out = rtg_scene_info()
        self.L.check("rtg_scene_get_info", self.L.lib.rtg_scene_get_info(self.handle, C.byref(out)))
        return out

    def close(self) -> None:
        if self.handle:
            self.L.lib.rtg_scene_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def plan(self, cam: rtg_camera_desc, row_begin: int = 0, row_stride: int = 1, row_count: int = 0,
             flags: int = RTG_RENDER_OUT_DEVICE) -> rtg_launch_plan:
        """rtg_render_plan: the launch plan (schedule, workgroups, LDS, the kernel's own VGPR count)
        a render of these rows would use, without rendering."""
        job = rtg_render_desc(DEFAULT_SEED, row_begin, row_stride, row_count, flags, None)
        out = rtg_launch_plan()
        self.L.check("rtg_render_plan", self.L.lib.rtg_render_plan(self.handle, C.byref(cam), C.byref(job),
                                                                    C.byref(out)))
        return out

    def prepare(self, cam: rtg_camera_desc, row_begin: int = 0, row_stride: int = 1, row_count: int = 0,
                stream=None):
        """rtg_scene_prepare: the setup the first render of this camera would do (the hot treelet of
        scenes that render with the treelet schedule; a no-op otherwise)."""
        job = rtg_render_desc(DEFAULT_SEED, row_begin, row_stride, row_count, RTG_RENDER_OUT_DEVICE, stream)
        self.L.check("rtg_scene_prepare", self.L.lib.rtg_scene_prepare(self.handle, C.byref(cam), C.byref(job)))

    def render_host(self, cam: rtg_camera_desc, seed: int = DEFAULT_SEED, row_begin: int = 0,
                    row_stride: int = 1, row_count: int = 0, count: bool = False):
        """Render into a new numpy array (rows, W, 3) float32; returns (array, stats)."""
        import numpy as np

        params = self.L.camera_resolve(cam)
        H, W = params.image_height, params.image_width
        rows = row_count if row_count > 0 else (H - 1 - row_begin) // row_stride + 1
        out = np.zeros((rows, W, 3), dtype=np.float32)
        job = rtg_render_desc(seed, row_begin, row_stride, rows, RTG_RENDER_COUNT if count else 0, None)
        st = rtg_render_stats()
        self.L.check("rtg_render", self.L.lib.rtg_render(self.handle, C.byref(cam), C.byref(job),
                                                          out.ctypes.data, C.byref(st)))
        return out, st

    def render_device(self, cam: rtg_camera_desc, out_ptr: int, stream_ptr: Optional[int],
                      seed: int = DEFAULT_SEED, row_begin: int = 0, row_stride: int = 1,
                      row_count: int = 0, asynchronous: bool = False,
                      count: bool = False) -> rtg_render_stats:
        """Render into device memory at out_ptr on `stream_ptr` (hipStream_t) ."""
        flags = RTG_RENDER_OUT_DEVICE | (RTG_RENDER_ASYNC if asynchronous else 0)
        flags |= RTG_RENDER_COUNT if count else 0
        job = rtg_render_desc(seed, row_begin, row_stride, row_count, flags,
                              C.c_void_p(stream_ptr) if stream_ptr else None)
        st = rtg_render_stats()
        self.L.check("rtg_render", self.L.lib.rtg_render(self.handle, C.byref(cam), C.byref(job),
                                                          C.c_void_p(out_ptr), C.byref(st)))
        return st

    def render_chunks(self, cam: rtg_camera_desc, partial_ptr: int, chunk_begin: int, chunk_count: int,
                      out_ptr: int = 0, stream_ptr: Optional[int] = None, seed: int = DEFAULT_SEED,
                      row_begin: int = 0, row_stride: int = 1, row_count: int = 0) -> rtg_render_stats:
        """Progressive rendering (rtgpu.h rtg_render_desc.partial): render sample chunks
        [chunk_begin, chunk_begin + chunk_count) into the device partial-sum buffer at partial_ptr
        (num_chunks(spp) x rows x W x 3 float32) and, when out_ptr is given, write the running mean
        of chunks [0, chunk_begin + chunk_count) there (device memory)."""
        flags = RTG_RENDER_OUT_DEVICE
        job = rtg_render_desc(seed, row_begin, row_stride, row_count, flags,
                              C.c_void_p(stream_ptr) if stream_ptr else None,
                              C.c_void_p(partial_ptr), chunk_begin, chunk_count)
        st = rtg_render_stats()
        self.L.check("rtg_render", self.L.lib.rtg_render(self.handle, C.byref(cam), C.byref(job),
                                                          C.c_void_p(out_ptr) if out_ptr else None,
                                                          C.byref(st)))
        return st

    def wait(self) -> rtg_render_stats:
        st = rtg_render_stats()
        self.L.check("rtg_render_wait", self.L.lib.rtg_render_wait(self.handle, C.byref(st)))
        return st

    def resolve_rgb8(self, in_ptr: int, out_ptr: int, n_pixels: int, stream_ptr: Optional[int]) -> None:
        self.L.check("rtg_resolve_rgb8", self.L.lib.rtg_resolve_rgb8(
            self.handle, C.c_void_p(in_ptr), C.c_void_p(out_ptr), n_pixels,
            C.c_void_p(stream_ptr) if stream_ptr else None))


class BuiltScene:
    """A scene from librtscenes.so: owns the flattened desc and the reference camera."""

    def __init__(self, slib: "SceneLibrary", handle: C.c_void_p):
        self.S = slib
        self.handle = handle
        self.desc: rtg_scene_desc = slib.lib.rts_scene_desc(handle).contents
        self.camera: rtg_camera_desc = rtg_camera_desc.from_buffer_copy(
            slib.lib.rts_scene_camera(handle).contents)

    def close(self) -> None:
        if self.handle:
            self.S.lib.rts_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SceneLibrary:
    """librtscenes.so — bouncing_spheres, checkered_spheres, earth, perlin_sphere, quads,
    simple_light, cornell_box (main.cpp:12-346) and earth_perlin (benchmark config 3)."""

    def __init__(self, path: Optional[str] = None):
        path = path or os.path.join(LIB_DIR, "librtscenes.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} not built (run __graft_entry__.build())")
        _one_hip_runtime()
        L = self.lib = C.CDLL(path)
        L.rts_build.argtypes = [C.c_char_p, _P(rts_params), _P(C.c_void_p)]
        L.rts_build.restype = C.c_int32
        L.rts_scene_desc.argtypes = [C.c_void_p]
        L.rts_scene_desc.restype = _P(rtg_scene_desc)
        L.rts_scene_camera.argtypes = [C.c_void_p]
        L.rts_scene_camera.restype = _P(rtg_camera_desc)
        L.rts_free.argtypes = [C.c_void_p]
        L.rts_free.restype = None
        L.rts_last_error.restype = C.c_char_p

    def build(self, name: str, grid: int = 0, image_width: int = 0, aspect_ratio: float = 0.0,
              spp: int = 0, max_depth: int = -1, bvh_mode: int = RTG_BVH_SAH,
              rand_seed: int = 1, image_dir: Optional[str] = None) -> BuiltScene:
        if image_dir is None:
            image_dir = os.path.join(REPO_DIR, "tests", "golden")
        os.environ.setdefault("RTW_IMAGES", image_dir)
        p = rts_params(grid, image_width, aspect_ratio, spp, max_depth, bvh_mode, rand_seed)
        h = C.c_void_p()
        st = self.lib.rts_build(name.encode(), C.byref(p), C.byref(h))
        if st != RTG_OK:
            raise RtgError("rts_build", st, (self.lib.rts_last_error() or b"").decode())
        return BuiltScene(self, h)


# ---------------------------------------------------------------------------------------------
# Interleaved-row tiling across GPUs: rank r of N renders rows r, r+N, ...

def shard_rows(height: int, rank: int, world: int):
    """(row_begin, row_stride, row_count) of `rank`'s interleaved shard; ranks past the image get 0 rows."""
    if rank >= height:
        return rank, world, 0
    return rank, world, (height - 1 - rank) // world + 1


def padded_rows(height: int, world: int) -> int:
    """Rows per shard after padding every shard to the same length (for a fixed-size gather)."""
    return (height + world - 1) // world


def deinterleave(shards: Sequence, height: int):
    """Assemble the image from per-rank shards (each (rows_padded, W, 3)); works for numpy and torch."""
    world = len(shards)
    first = shards[0]
    W = first.shape[1]
    try:
        import torch

        if isinstance(first, torch.Tensor):
            out = torch.empty((height, W, 3), dtype=first.dtype, device=first.device)
            for r, s in enumerate(shards):
                _, _, n = shard_rows(height, r, world)
                if n:
                    out[r::world][:n] = s[:n]
            return out
    except ImportError:  # pragma: no cover
        pass
    import numpy as np

    out = np.empty((height, W, 3), dtype=first.dtype)
    for r, s in enumerate(shards):
        _, _, n = shard_rows(height, r, world)
        if n:
            out[r::world][:n] = s[:n]
    return out


def camera(**kw) -> rtg_camera_desc:
    """rtg_camera_desc with the reference's defaults (camera.hpp:13-25) overridden by kw."""
    c = rtg_camera_desc()
    c.aspect_ratio, c.image_width, c.samples_per_pixel, c.max_depth = 1.0, 100, 10, 10
    c.vfov, c.defocus_angle, c.focus_dist = 90.0, 0.0, 10.0
    c.lookfrom, c.lookat, c.vup = D3(0, 0, 0), D3(0, 0, -1), D3(0, 1, 0)
    c.background = D3(0, 0, 0)
    for k, v in kw.items():
        if k in ("background", "lookfrom", "lookat", "vup"):
            v = D3(*v)
        setattr(c, k, v)
    return c


def write_color_bytes(rgb):
    """write_color (color.hpp:26-58) on a float array (..., 3): sqrt gamma (in double, as the
    reference's linear_to_gamma), clamp to [0, 0.999], int(256 * x) -> uint8. Host twin of
    rtg_resolve_rgb8 for CPU-side shards."""
    import numpy as np

    x = np.asarray(rgb, dtype=np.float64)
    x = np.where(x > 0.0, np.sqrt(np.maximum(x, 0.0)), 0.0)
    x = np.clip(x, 0.0, np.float64(np.float32(0.999)))
    return (256.0 * x).astype(np.int32).astype(np.uint8)


def gather_frame(shard, height: int, dst: int = 0):
    """Collect every rank's interleaved shard on `dst` and de-interleave.

    `shard` is this rank's torch tensor of shape (padded_rows(height, N), W, 3) — rows past its
    real row count are padding. One collective: torch.distributed.gather (RCCL's ncclGather
    pattern under the "nccl" backend, a point-to-point send from each peer to dst over xGMI;
    gloo on CPU for the tests). Returns the (height, W, 3) frame on dst and None elsewhere.
    """
    import torch.distributed as dist

    world = dist.get_world_size()
    rank = dist.get_rank()
    if world == 1:
        _, _, n = shard_rows(height, 0, 1)
        return shard[:n]
    if rank == dst:
        parts = [shard.new_empty(shard.shape) for _ in range(world)]
        dist.gather(shard, gather_list=parts, dst=dst)
        return deinterleave(parts, height)
    dist.gather(shard, dst=dst)
    return None


class FrameGather:
    """The N > 1 frame gather of bench.py's timed loop, with every buffer allocated once.

    Rank `dst` owns a staging tensor of N padded shard blocks (the rtg_gather_rows layout) and the
    (height, W, C) frame; each call gathers every rank's shard into the blocks (torch.distributed.gather:
    the RCCL gather under "nccl", gloo on CPU) and de-interleaves them with the library's own kernel
    (rtg_deinterleave_rows on the shard's stream; its host twin rtg_deinterleave_rows_host for CPU
    tensors), so a timed step allocates nothing. Returns the frame on dst (the same tensor every call) and
    None elsewhere. The shard must keep its shape between calls."""

    def __init__(self, lib: Library, shard, height: int, dst: int = 0, device: int = 0):
        import torch.distributed as dist

        self.lib, self.height, self.dst, self.device = lib, height, dst, device
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        self.shape = tuple(shard.shape)
        self.row_bytes = int(shard[0].numel() * shard.element_size())
        self.stage = self.parts = self.frame = None
        if self.rank == dst:
            self.stage = shard.new_empty((self.world,) + self.shape)
            self.parts = list(self.stage.unbind(0))  # views into the staging blocks
            self.frame = shard.new_empty((height,) + self.shape[1:])

    def __call__(self, shard, stream_ptr: Optional[int] = None):
        import torch.distributed as dist

        assert tuple(shard.shape) == self.shape, "the shard changed shape after FrameGather was set up"
        if self.world == 1:
            return shard[: self.height]
        if self.rank != self.dst:
            dist.gather(shard, dst=self.dst)
            return None
        dist.gather(shard, gather_list=self.parts, dst=self.dst)
        return self.deinterleave(stream_ptr)

    def deinterleave(self, stream_ptr: Optional[int] = None):
        """The staging blocks -> the frame: the library's kernel for device tensors (on stream_ptr), its
        host twin for CPU tensors (test_gpu checks the two agree)."""
        if self.stage.is_cuda:
            self.lib.deinterleave_rows(self.device, self.stage.data_ptr(), self.frame.data_ptr(), self.world,
                                       self.height, self.row_bytes, stream_ptr)
        else:
            self.lib.check("rtg_deinterleave_rows_host", self.lib.lib.rtg_deinterleave_rows_host(
                C.c_void_p(self.stage.data_ptr()), C.c_void_p(self.frame.data_ptr()), self.world,
                self.height, self.row_bytes))
        return self.frame
