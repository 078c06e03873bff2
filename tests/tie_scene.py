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
