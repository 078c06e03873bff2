"""A scene built for exact-t ties (DESIGN.md §4 "tie rule"): three identical quads with different
emitted colours, so every camera ray that reaches them hits all three at bit-identical t, beside a
sphere. The reference tests its list in order (hittable_list.hpp:40-64) and quad::hit accepts t ==
closest_so_far (interval::contains, quad.hpp:62), so its image shows the LAST quad's colour."""
import ctypes as C

import rtgpu

RED, GREEN, BLUE, WHITE = (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0), (1.0, 1.0, 1.0)


def tie_scene(bvh_mode=rtgpu.RTG_BVH_SAH, width=48):
    cols = [RED, BLUE, GREEN, WHITE]
    tex = [rtgpu.rtg_texture(type=rtgpu.RTG_TEX_SOLID, color=rtgpu.D3(*c)) for c in cols]
    mat = [rtgpu.rtg_material(type=rtgpu.RTG_MAT_DIFFUSE_LIGHT, texture=k) for k in range(4)]

    def quad(m):
        return rtgpu.rtg_primitive(kind=rtgpu.RTG_PRIM_QUAD, material=m, p0=rtgpu.D3(-3.0, -1.5, 0.0),
                                   p1=rtgpu.D3(2.5, 0.0, 0.0), p2=rtgpu.D3(0.0, 3.0, 0.0))

    def sphere(m):
        return rtgpu.rtg_primitive(kind=rtgpu.RTG_PRIM_SPHERE, material=m, p0=rtgpu.D3(1.6, 0.0, 0.0),
                                   p1=rtgpu.D3(1.6, 0.0, 0.0), radius=1.0)

    # list order: quad (white), quad (red), sphere (blue), quad (green)
    prims = [quad(3), quad(0), sphere(1), quad(2)]
    P = (rtgpu.rtg_primitive * 4)(*prims)
    M = (rtgpu.rtg_material * 4)(*mat)
    T = (rtgpu.rtg_texture * 4)(*tex)
    d = rtgpu.rtg_scene_desc(abi_version=rtgpu.RTG_ABI_VERSION, bvh_mode=bvh_mode,
                             prims=C.cast(P, C.POINTER(rtgpu.rtg_primitive)), num_prims=4,
                             materials=C.cast(M, C.POINTER(rtgpu.rtg_material)), num_materials=4,
                             textures=C.cast(T, C.POINTER(rtgpu.rtg_texture)), num_textures=4)
    d._keep = (P, M, T)
    cam = rtgpu.camera(image_width=width, aspect_ratio=2.0, samples_per_pixel=4, max_depth=4,
                       background=(0.0, 0.0, 0.0), lookfrom=(0, 0, 5), lookat=(0, 0, 0), vfov=60.0)
    return d, cam


def colour_counts(frame):
    """Pixels whose every sample saw one primitive colour: {colour: count}."""
    out = {}
    for c in (RED, GREEN, BLUE, WHITE):
        out[c] = int(((frame == C_arr(c)).all(axis=-1)).sum())
    return out


def C_arr(c):
    import numpy as np

    return np.array(c, dtype=np.float32)


def make_desc(prims, mats, texs, bvh_mode):
    P = (rtgpu.rtg_primitive * len(prims))(*prims)
    M = (rtgpu.rtg_material * len(mats))(*mats)
    T = (rtgpu.rtg_texture * len(texs))(*texs)
    d = rtgpu.rtg_scene_desc(abi_version=rtgpu.RTG_ABI_VERSION, bvh_mode=bvh_mode,
                             prims=C.cast(P, C.POINTER(rtgpu.rtg_primitive)), num_prims=len(prims),
                             materials=C.cast(M, C.POINTER(rtgpu.rtg_material)), num_materials=len(mats),
                             textures=C.cast(T, C.POINTER(rtgpu.rtg_texture)), num_textures=len(texs))
    d._keep = (P, M, T)
    return d


def _sphere(m, c, r):
    return rtgpu.rtg_primitive(kind=rtgpu.RTG_PRIM_SPHERE, material=m, p0=rtgpu.D3(*c), p1=rtgpu.D3(*c),
                               radius=r)


def _lights(cols):
    tex = [rtgpu.rtg_texture(type=rtgpu.RTG_TEX_SOLID, color=rtgpu.D3(*c)) for c in cols]
    mat = [rtgpu.rtg_material(type=rtgpu.RTG_MAT_DIFFUSE_LIGHT, texture=k) for k in range(len(cols))]
    return mat, tex


def duplicate_sphere_scene(bvh_mode=rtgpu.RTG_BVH_SAH, width=64, dedup=False):
    """Sphere-sphere exact-t ties (DESIGN.md §4 "tie rule", round 5): a 4x4 grid of groups of three
    identical spheres (emitting red, green, blue), every ray that reaches a group hits its three spheres at
    bit-identical t. The list holds every group's first member, then every second, then every third, with
    the colours rotated per group; sphere::hit never replaces an equal-t hit (interval::surrounds,
    sphere.hpp:70), so the reference's list walk (hittable_list.hpp:40-64) shows each group's FIRST
    member. dedup=True: the same scene with only those first members (the expected image)."""
    cols = [RED, GREEN, BLUE]
    mat, tex = _lights(cols)
    groups = [(-4.5 + 3.0 * (g % 4), -4.5 + 3.0 * (g // 4)) for g in range(16)]
    prims = []
    for member in range(1 if dedup else 3):
        for g, (x, y) in enumerate(groups):
            prims.append(_sphere((g + member) % 3, (x, y, 0.0), 1.2))
    cam = rtgpu.camera(image_width=width, aspect_ratio=1.0, samples_per_pixel=4, max_depth=3,
                       background=(0.0, 0.0, 0.0), lookfrom=(0.3, 0.2, 20.0), lookat=(0, 0, 0), vfov=36.0)
    return make_desc(prims, mat, tex, bvh_mode), cam


# near-tie height: the competitor's surface at Y0, the small spheres' tops a fraction of an fp32 ulp above it
NEAR_TIE_Y0 = 1000.0


def near_tie_scene(bvh_mode=rtgpu.RTG_BVH_SAH, competitor="quad", width=64, cam_height=2.0):
    """Near ties for the BVH culling margin (DESIGN.md §4 "conservative culling"): a
    3x3 field of small spheres (centre y = 999.5, radius 0.5 + j 2^-21, j = 1..3) whose tops poke 1/64 ..
    3/64 of an fp32 ulp above a competitor surface at y = 1000 (a large quad, or a sphere of radius 1000
    below it), far from the world origin. A ray from just above an apex hits the small sphere at its box's
    top face a little before the competitor, which is tested first (its box is entered first, or it is the
    scene-spanning occluder); the fp32 slab test's rounding, about 2^-24 |o| / |d|, is ~60x that gap here,
    so a culling bound without the host padding and the tbest margin culls the box that holds the closest
    hit. The camera sits above the centre apex, zoomed in on it."""
    import numpy as np

    mat, tex = _lights([RED, GREEN, BLUE, WHITE])
    y0 = NEAR_TIE_Y0
    prims = []
    if competitor == "quad":
        prims.append(rtgpu.rtg_primitive(kind=rtgpu.RTG_PRIM_QUAD, material=3, p0=rtgpu.D3(-8.0, y0, -8.0),
                                         p1=rtgpu.D3(16.0, 0.0, 0.0), p2=rtgpu.D3(0.0, 0.0, 16.0)))
    else:
        prims.append(_sphere(3, (0.0, y0 - 1000.0, 0.0), 1000.0))
    for g in range(9):
        x, z = -4.0 + 4.0 * (g % 3), -4.0 + 4.0 * (g // 3)
        prims.append(_sphere(g % 3, (x, y0 - 0.5, z), 0.5 + (1 + g % 3) * 2.0 ** -21))
    half = 1.5e-3  # the apex discs poking above y0 have radii 0.7e-3 .. 1.2e-3
    cam = rtgpu.camera(image_width=width, aspect_ratio=1.0, samples_per_pixel=4, max_depth=3,
                       background=(0.0, 0.0, 0.0), lookfrom=(0.0, y0 + cam_height, 0.0),
                       lookat=(0.0, y0, 0.0), vup=(0.0, 0.0, 1.0),
                       vfov=float(np.degrees(2 * np.arctan(half / cam_height))), focus_dist=cam_height)
    return make_desc(prims, mat, tex, bvh_mode), cam


def _quad(m, Q, u, v):
    return rtgpu.rtg_primitive(kind=rtgpu.RTG_PRIM_QUAD, material=m, p0=rtgpu.D3(*Q), p1=rtgpu.D3(*u),
                               p2=rtgpu.D3(*v))


def _box_quads(m, lo, hi, R=None, pivot=(0.0, 0.0, 0.0)):
    """The six faces of a box as quads sharing their edges (as the reference's box(), quad.hpp), optionally
    rotated by the 3x3 matrix R about `pivot`."""
    import numpy as np

    lo, hi = np.asarray(lo, float), np.asarray(hi, float)
    dx, dy, dz = np.array([hi[0] - lo[0], 0, 0]), np.array([0, hi[1] - lo[1], 0]), np.array([0, 0, hi[2] - lo[2]])
    faces = [(lo, dy, dz), (lo + dx, dy, dz), (lo, dx, dz), (lo + dy, dx, dz), (lo, dx, dy), (lo + dz, dx, dy)]
    out = []
    for Q, u, v in faces:
        if R is not None:
            p = np.asarray(pivot, float)
            Q, u, v = R @ (Q - p) + p, R @ u, R @ v
        out.append(_quad(m, tuple(float(x) for x in Q), tuple(float(x) for x in u), tuple(float(x) for x in v)))
    return out


def quad_edge_scene(bvh_mode=rtgpu.RTG_BVH_SAH, width=64, offset=0.0, spp=8, seed=7):
    """Quads meeting at shared edges (DESIGN.md §4 "conservative culling", round 5): an open room of
    axis-aligned walls, axis-aligned blocks standing on its floor and against a wall, blocks rotated about
    skew axes (no flat axis: every plane padded by 2^-18 (|v| + M)), quads flat in z but rotated within
    their plane (u, v not along the axes: treated as general quads), small spheres resting on block tops
    and a ceiling light, the whole scene translated by `offset` along every axis (|v| + M large against the
    room's size). Rays leave faces at every angle and graze their neighbours' edges, which is where the
    per-axis culling boxes and the widened exits have to hold."""
    import numpy as np

    rng = np.random.default_rng(seed)
    tex = [rtgpu.rtg_texture(type=rtgpu.RTG_TEX_SOLID, color=rtgpu.D3(*c))
           for c in ((0.73, 0.73, 0.73), (0.65, 0.05, 0.05), (0.12, 0.45, 0.15), (15.0, 15.0, 15.0))]
    mat = [rtgpu.rtg_material(type=rtgpu.RTG_MAT_LAMBERTIAN, texture=k) for k in range(3)]
    mat.append(rtgpu.rtg_material(type=rtgpu.RTG_MAT_DIFFUSE_LIGHT, texture=3))
    o = np.array([offset, offset, offset])
    S = 20.0
    t = lambda *p: tuple(float(x) for x in np.asarray(p, float) + o)
    prims = [_quad(2, t(S, 0, 0), (0, S, 0), (0, 0, S)), _quad(1, t(0, 0, 0), (0, S, 0), (0, 0, S)),
             _quad(0, t(0, 0, 0), (S, 0, 0), (0, 0, S)), _quad(0, t(S, S, S), (-S, 0, 0), (0, 0, -S)),
             _quad(0, t(0, 0, S), (S, 0, 0), (0, S, 0)), _quad(3, t(17, S - 0.01, 17), (-14, 0, 0), (0, 0, -14))]
    prims += _box_quads(0, t(3, 0, 3), t(9, 6, 9))      # on the floor
    prims += _box_quads(1, t(12, 0, 14), t(S, 10, S))   # in the back corner, flush with two walls
    for k in range(3):  # rotated about skew axes
        axis = rng.normal(size=3)
        axis /= np.linalg.norm(axis)
        a = rng.uniform(0.3, 1.2)
        K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
        R = np.eye(3) + np.sin(a) * K + (1 - np.cos(a)) * (K @ K)
        c = np.array([4.0 + 6.0 * k, 12.0, 6.0 + 3.0 * k])
        prims += _box_quads(k % 3, t(*(c - 1.5)), t(*(c + 1.5)), R, pivot=t(*c))
    for k in range(3):  # flat in z, rotated within the plane
        a = rng.uniform(0.2, 1.3)
        u = (3.0 * np.cos(a), 3.0 * np.sin(a), 0.0)
        v = (-2.0 * np.sin(a), 2.0 * np.cos(a), 0.0)
        prims.append(_quad(k % 3, t(5.0 + 4.0 * k, 3.0 + 2.0 * k, 12.0), u, v))
    prims += [_sphere(1, t(6, 7, 6), 1.0), _sphere(2, t(16, 11.5, 17), 1.5)]
    cam = rtgpu.camera(image_width=width, aspect_ratio=1.0, samples_per_pixel=spp, max_depth=8,
                       background=(0.0, 0.0, 0.0), lookfrom=t(10, 10, -18), lookat=t(10, 9, 10), vfov=55.0)
    return make_desc(prims, mat, tex, bvh_mode), cam
