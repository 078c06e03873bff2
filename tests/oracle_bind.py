"""ctypes binding of oracle/lib/liboracle.so — TEST INFRASTRUCTURE ONLY (see oracle/cpu_ref.c).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker; never by
the product path (raytracing-practice_amd/)."""
import ctypes as C
import os

import numpy as np

import rtgpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_LIB = os.path.join(REPO, "oracle", "lib", "liboracle.so")
P = C.POINTER
D3P = P(C.c_double)


class Oracle:
    def __init__(self, path: str = ORACLE_LIB):
        L = self.lib = C.CDLL(path)
        L.orc_camera_resolve.argtypes = [P(rtgpu.rtg_camera_desc), P(rtgpu.rtg_camera_params)]
        L.orc_render_f32.argtypes = [P(rtgpu.rtg_scene_desc), P(rtgpu.rtg_camera_desc), C.c_uint64,
                                     C.c_int, C.c_int, C.c_int, C.c_void_p, P(C.c_uint64)]
        L.orc_render_f32_mt.argtypes = [P(rtgpu.rtg_scene_desc), P(rtgpu.rtg_camera_desc), C.c_uint64,
                                        C.c_int, C.c_int, C.c_int, C.c_void_p, P(C.c_uint64), C.c_int]
        L.orc_render_f64.argtypes = [P(rtgpu.rtg_scene_desc), P(rtgpu.rtg_camera_desc), C.c_uint,
                                     C.c_int, C.c_int, C.c_void_p, P(C.c_uint64)]
        L.orc_bench_f64.argtypes = [P(rtgpu.rtg_scene_desc), P(rtgpu.rtg_camera_desc), C.c_int,
                                    C.c_int, C.c_int, C.c_uint, P(C.c_double), P(C.c_uint64)]
        L.orc_glibc_random_double.argtypes = [C.c_uint, C.c_int]
        L.orc_glibc_random_double.restype = C.c_double
        L.orc_rng_state.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32]
        L.orc_rng_state.restype = C.c_uint64
        L.orc_rng_uniform.argtypes = [P(C.c_uint64)]
        L.orc_rng_uniform.restype = C.c_float
        L.orc_kat_random_unit_vector.argtypes = [C.c_uint, D3P, D3P]
        L.orc_kat_random_in_unit_disk.argtypes = [C.c_uint, D3P, D3P]
        L.orc_kat_sphere_hit.argtypes = [P(rtgpu.rtg_primitive), D3P, D3P, C.c_double, C.c_double,
                                         C.c_double, D3P]
        L.orc_kat_quad_hit.argtypes = [P(rtgpu.rtg_primitive), D3P, D3P, C.c_double, C.c_double,
                                       D3P, D3P]
        L.orc_kat_aabb_hit.argtypes = [D3P, D3P, D3P, D3P, C.c_double, C.c_double, D3P, P(C.c_int)]
        L.orc_kat_reflect_refract.argtypes = [D3P, D3P, C.c_double, D3P, D3P]
        L.orc_write_color.argtypes = [D3P, P(C.c_int)]
        L.orc_perlin_noise64.argtypes = [P(rtgpu.rtg_perlin), D3P]
        L.orc_perlin_noise64.restype = C.c_double
        L.orc_perlin_turb64.argtypes = [P(rtgpu.rtg_perlin), D3P]
        L.orc_perlin_turb64.restype = C.c_double
        L.orc_bvh_replay.argtypes = [P(rtgpu.rtg_scene_desc), D3P, D3P, C.c_double, P(C.c_int64),
                                     C.c_int64, D3P]
        L.orc_bvh_replay.restype = C.c_int64
        L.orc_closest_hit32.argtypes = [P(rtgpu.rtg_scene_desc), C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p, C.c_void_p]
        L.orc_closest_hit32.restype = None
        L.orc_sincos_turn.argtypes = [C.c_float, P(C.c_float), P(C.c_float)]
        for name, nargs in (("orc_sin_spec", 1), ("orc_atan2_spec", 2), ("orc_acos_spec", 1)):
            getattr(L, name).argtypes = [C.c_float] * nargs
            getattr(L, name).restype = C.c_float
        L.orc_f32_unit_vector.argtypes = [C.c_uint64, P(C.c_float)]
        L.orc_sphere_t32.argtypes = [P(C.c_float), P(C.c_float), P(C.c_float), C.c_float, C.c_float,
                                     C.c_float]
        L.orc_sphere_t32.restype = C.c_float

    def sin_spec(self, x):
        return self.lib.orc_sin_spec(x)

    def atan2_spec(self, y, x):
        return self.lib.orc_atan2_spec(y, x)

    def acos_spec(self, v):
        return self.lib.orc_acos_spec(v)

    def sincos_turn(self, u):
        sn, cs = C.c_float(), C.c_float()
        self.lib.orc_sincos_turn(u, C.byref(sn), C.byref(cs))
        return sn.value, cs.value

    def unit_vector(self, state):
        out = (C.c_float * 3)()
        self.lib.orc_f32_unit_vector(state, out)
        return tuple(out)

    @staticmethod
    def _d(v):
        return (C.c_double * len(v))(*v)

    def camera_resolve(self, cam):
        out = rtgpu.rtg_camera_params()
        self.lib.orc_camera_resolve(C.byref(cam), C.byref(out))
        return out

    def render_f32(self, desc, cam, seed=rtgpu.DEFAULT_SEED, row_begin=0, row_stride=1, row_count=0, threads=1):
        """cpu_ref32 rows (threads > 1: one shared world, rows dealt over that many threads; the frame
        does not depend on it)."""
        p = self.camera_resolve(cam)
        rows = row_count if row_count > 0 else (p.image_height - 1 - row_begin) // row_stride + 1
        out = np.zeros((rows, p.image_width, 3), dtype=np.float32)
        segs = C.c_uint64(0)
        self.lib.orc_render_f32_mt(C.byref(desc), C.byref(cam), seed, row_begin, row_stride, rows,
                                   out.ctypes.data, C.byref(segs), threads)
        return out, segs.value

    def render_f64(self, desc, cam, seed=1, row_begin=0, row_count=0):
        p = self.camera_resolve(cam)
        rows = row_count if row_count > 0 else p.image_height - row_begin
        out = np.zeros((rows, p.image_width, 3), dtype=np.float64)
        segs = C.c_uint64(0)
        self.lib.orc_render_f64(C.byref(desc), C.byref(cam), seed, row_begin, rows,
                                out.ctypes.data, C.byref(segs))
        return out, segs.value

    def bench_f64(self, desc, cam, threads, rows, base_seed=1000, row_step=1):
        sec, segs = C.c_double(0), C.c_uint64(0)
        self.lib.orc_bench_f64(C.byref(desc), C.byref(cam), threads, rows, row_step, base_seed,
                               C.byref(sec), C.byref(segs))
        return sec.value, segs.value

    def glibc_random_double(self, seed, k):
        return self.lib.orc_glibc_random_double(seed, k)

    def rng_uniforms(self, seed, pixel, sample, n):
        st = C.c_uint64(self.lib.orc_rng_state(seed, pixel, sample))
        return [self.lib.orc_rng_uniform(C.byref(st)) for _ in range(n)]

    def random_unit_vector(self, seed):
        v, nxt = (C.c_double * 3)(), (C.c_double * 1)()
        self.lib.orc_kat_random_unit_vector(seed, v, nxt)
        return list(v), nxt[0]

    def random_in_unit_disk(self, seed):
        v, nxt = (C.c_double * 3)(), (C.c_double * 1)()
        self.lib.orc_kat_random_in_unit_disk(seed, v, nxt)
        return list(v), nxt[0]

    def sphere_hit(self, prim, o, d, time, tmin, tmax):
        rec = (C.c_double * 10)()
        h = self.lib.orc_kat_sphere_hit(C.byref(prim), self._d(o), self._d(d), time, tmin, tmax, rec)
        return bool(h), list(rec)

    def sphere_t32(self, rec8, o, d, time=0.0, tmin=0.001, tmax=float("inf")):
        f3 = C.c_float * 3
        return float(self.lib.orc_sphere_t32((C.c_float * 8)(*rec8), f3(*o), f3(*d), time, tmin, tmax))

    def quad_hit(self, prim, o, d, tmin, tmax):
        rec, bbox = (C.c_double * 10)(), (C.c_double * 6)()
        h = self.lib.orc_kat_quad_hit(C.byref(prim), self._d(o), self._d(d), tmin, tmax, rec, bbox)
        return bool(h), list(rec), list(bbox)

    def aabb_hit(self, a, b, o, d, tmin, tmax):
        box, axis = (C.c_double * 6)(), C.c_int(0)
        h = self.lib.orc_kat_aabb_hit(self._d(a), self._d(b), self._d(o), self._d(d), tmin, tmax,
                                      box, C.byref(axis))
        return bool(h), list(box), axis.value

    def reflect_refract(self, v, n, eta):
        r, t = (C.c_double * 3)(), (C.c_double * 3)()
        self.lib.orc_kat_reflect_refract(self._d(v), self._d(n), eta, r, t)
        return list(r), list(t)

    def write_color(self, rgb):
        out = (C.c_int * 3)()
        self.lib.orc_write_color(self._d(rgb), out)
        return list(out)

    def perlin_noise(self, perlin, p):
        return self.lib.orc_perlin_noise64(C.byref(perlin), self._d(p))

    def perlin_turb(self, perlin, p):
        return self.lib.orc_perlin_turb64(C.byref(perlin), self._d(p))

    def closest_hit32(self, desc, o, d, time):
        """cpu_ref32's closest hit of n camera-like segments (fp32 rays): (winner index or -1, t)."""
        import numpy as np

        o = np.ascontiguousarray(o, dtype=np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, dtype=np.float32).reshape(-1, 3)
        tm = np.ascontiguousarray(np.broadcast_to(np.asarray(time, np.float32), (len(o),)))
        best = np.empty(len(o), np.int64)
        t = np.empty(len(o), np.float32)
        self.lib.orc_closest_hit32(C.byref(desc), len(o), o.ctypes.data, d.ctypes.data, tm.ctypes.data,
                                   best.ctypes.data, t.ctypes.data)
        return best, t

    def bvh_replay(self, desc, o, d, time, cap=4096):
        log, t = (C.c_int64 * cap)(), (C.c_double * 1)()
        n = self.lib.orc_bvh_replay(C.byref(desc), self._d(o), self._d(d), time, log, cap, t)
        return list(log)[:n], t[0]


def sphere_prim(c1, c2, r, mat=0):
    p = rtgpu.rtg_primitive()
    p.kind, p.material = rtgpu.RTG_PRIM_SPHERE, mat
    p.p0, p.p1, p.radius = rtgpu.D3(*c1), rtgpu.D3(*c2), r
    return p


def quad_prim(Q, u, v, mat=0):
    p = rtgpu.rtg_primitive()
    p.kind, p.material = rtgpu.RTG_PRIM_QUAD, mat
    p.p0, p.p1, p.p2 = rtgpu.D3(*Q), rtgpu.D3(*u), rtgpu.D3(*v)
    return p
