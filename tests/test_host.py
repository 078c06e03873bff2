"""Host-side logic of the product (no GPU needed): the C-ABI surface, camera::initialize, the
scene generator of the C++ API mirror, the image loader, Perlin tables and the BVH builder —
each checked against the reference's golden vectors or the oracle."""
import ctypes as C
import math
import os
import re
import subprocess

import numpy as np
import pytest

import rtgpu
from conftest import GOLDEN, REPO

REFERENCE_SRC = "/root/reference/src"


def test_cabi_exports_every_declared_symbol(lib):
    with open(os.path.join(REPO, "include", "rtgpu.h")) as f:
        header = f.read()
    declared = set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(rtg_\w+)\s*\(", header, re.M))
    inline = set(re.findall(r"^static inline \w+ (rtg_\w+)\s*\(", header, re.M))  # header-only rules
    declared -= inline
    assert declared == set(rtgpu.RTG_SYMBOLS)
    for name in declared:
        assert hasattr(lib.lib, name), name  # dlsym succeeds
    assert lib.lib.rtg_abi_version() == rtgpu.RTG_ABI_VERSION


def test_numerics_check_library_loads():
    """The test library that checks the kernels' div_rn / sqrt_rn against hipcc's IEEE operations
    (tests/native/numerics_check.hip, run on the GPU by test_gpu.py) is built and exports its entry."""
    so = C.CDLL(os.path.join(REPO, "tests", "native", "libnumcheck.so"))
    assert hasattr(so, "rtg_numerics_check")


def test_chunk_rule():
    """rtg_chunk_samples (rtgpu.h): one chunk up to 16 spp, chunks of <= 16 samples above."""
    def k(spp):
        n = max(1, (spp + 15) // 16)
        return (spp + n - 1) // n if spp > 0 else 1
    assert [k(s) for s in (1, 10, 16, 17, 64, 500, 1000, 2000)] == [1, 10, 16, 9, 16, 16, 16, 16]
    assert [rtgpu.chunk_samples(s) for s in (1, 10, 16, 17, 64, 500, 1000, 2000)] == \
        [k(s) for s in (1, 10, 16, 17, 64, 500, 1000, 2000)]
    assert rtgpu.num_chunks(500) == 32 and rtgpu.num_chunks(16) == 1


def test_scenes_lib_exports(scenes):
    for name in ("rts_build", "rts_scene_desc", "rts_scene_camera", "rts_free", "rts_last_error"):
        assert hasattr(scenes.lib, name)


CAMERAS = {
    "book1_cfg1": dict(aspect_ratio=16.0 / 9.0, image_width=400, samples_per_pixel=10, max_depth=10,
                       vfov=20.0, lookfrom=(13, 2, 3), lookat=(0, 0, 0), defocus_angle=0.6,
                       focus_dist=10.0),
    "book1_cfg2": dict(aspect_ratio=16.0 / 9.0, image_width=1920, samples_per_pixel=500, max_depth=50,
                       vfov=20.0, lookfrom=(13, 2, 3), lookat=(0, 0, 0), defocus_angle=0.6,
                       focus_dist=10.0),
    "reference_float_aspect": dict(aspect_ratio=float(np.float32(16.0) / np.float32(9.0)),
                                   image_width=1920, samples_per_pixel=7),
    "cornell": dict(aspect_ratio=1.0, image_width=800, samples_per_pixel=2000, max_depth=100,
                    vfov=40.0, lookfrom=(278, 278, -800), lookat=(278, 278, 0)),
    "tiny": dict(aspect_ratio=4.0, image_width=3, samples_per_pixel=3),
}


@pytest.mark.parametrize("name", sorted(CAMERAS))
def test_camera_initialize_matches_oracle(lib, oracle, name):
    cam = rtgpu.camera(**CAMERAS[name])
    a, b = lib.camera_resolve(cam), oracle.camera_resolve(cam)
    assert bytes(a) == bytes(b)  # bitwise: both restate camera.hpp:76-136 in fp64


def test_image_height_truncation(lib):
    # H4: 16.0f/9.0f (float) gives 1079 rows at 1920; 16.0/9.0 (double) gives 1080
    assert lib.camera_resolve(rtgpu.camera(**CAMERAS["reference_float_aspect"])).image_height == 1079
    assert lib.camera_resolve(rtgpu.camera(**CAMERAS["book1_cfg2"])).image_height == 1080
    assert lib.camera_resolve(rtgpu.camera(**CAMERAS["book1_cfg1"])).image_height == 225
    # pixel_samples_scale is float(1.0f / spp) (H7)
    p = lib.camera_resolve(rtgpu.camera(**CAMERAS["reference_float_aspect"]))
    assert p.pixel_samples_scale == float(np.float32(1.0) / np.float32(7))


def test_book1_scene_matches_reference(scenes, golden):
    """bouncing_spheres built by the C++ mirror (explicit GCC draw order) == the reference's."""
    s = scenes.build("bouncing_spheres", rand_seed=1)
    d = s.desc
    ref = golden["book1"]["spheres"]
    assert d.num_prims == len(ref) == 484
    for i, r in enumerate(ref):
        p = d.prims[i]
        assert p.kind == rtgpu.RTG_PRIM_SPHERE
        assert list(p.p0) == r["c1"] and list(p.p1) == r["c2"] and p.radius == r["r"], i
        m = d.materials[p.material]
        if r["mat"] == 0:
            t = d.textures[m.texture]
            assert m.type == rtgpu.RTG_MAT_LAMBERTIAN and t.type == rtgpu.RTG_TEX_CHECKER
            assert t.scale == float(np.float32(0.32))
            assert list(d.textures[t.even].color) == [float(np.float32(x)) for x in (0.2, 0.3, 0.1)]
        elif r["mat"] == 1:
            t = d.textures[m.texture]
            assert m.type == rtgpu.RTG_MAT_LAMBERTIAN and t.type == rtgpu.RTG_TEX_SOLID
            assert list(t.color) == r["albedo"], i
        elif r["mat"] == 2:
            assert m.type == rtgpu.RTG_MAT_METAL
            assert list(m.albedo) == r["albedo"] and m.fuzz == r["fuzz"], i
        else:
            assert m.type == rtgpu.RTG_MAT_DIELECTRIC and m.refraction_index == r["ri"]


def test_perlin_tables_match_reference(scenes, oracle, golden):
    """perlin() tables drawn from the seed-1 stream by the mirror reproduce the reference's
    noise_perlin / turb (perlin.hpp:12-158) at 200 points, bit for bit."""
    s = scenes.build("perlin_sphere", rand_seed=1)
    assert s.desc.num_perlins == 1
    pl = s.desc.perlins[0]
    for rec in golden["perlin_seed1"]["points"]:
        assert oracle.perlin_noise(pl, rec["p"]) == rec["noise"]
        assert oracle.perlin_turb(pl, rec["p"]) == rec["turb7"]
    for k in range(256):
        assert sorted(pl.perm_x) == list(range(256))


def _stb_texel_lut():
    # stbi__ldr_to_hdr: (float)(pow(b / 255.0f, 2.2f) * 1.0f), then float_to_byte (rtw_stb_image.hpp:137-150)
    lut = np.zeros(256, dtype=np.uint8)
    for b in range(256):
        f = np.float32(math.pow(float(np.float32(b) / np.float32(255.0)), float(np.float32(2.2))) * 1.0)
        lut[b] = 0 if f <= 0 else (255 if f >= 1 else int(np.float32(256.0) * f))
    return lut


def test_image_loader_conversion(scenes):
    s = scenes.build("earth", rand_seed=1)
    assert s.desc.num_images == 1
    im = s.desc.images[0]
    assert (im.width, im.height) == (1024, 512)
    got = np.ctypeslib.as_array(im.rgb, shape=(512 * 1024 * 3,))
    with open(os.path.join(GOLDEN, "earthmap.ppm"), "rb") as f:
        raw = f.read()
    srgb = np.frombuffer(raw[-512 * 1024 * 3:], dtype=np.uint8)
    assert np.array_equal(got, _stb_texel_lut()[srgb])


def _slab(box_lo, box_hi, o, d, tmin, tmax):
    """aabb::hit (aabb.hpp:61-112) in Python doubles."""
    for a in range(3):
        adinv = (1.0 / d[a]) if d[a] != 0 else math.copysign(math.inf, d[a])
        t0 = (box_lo[a] - o[a]) * adinv
        t1 = (box_hi[a] - o[a]) * adinv
        if t0 < t1:
            tmin = t0 if t0 > tmin else tmin
            tmax = t1 if t1 < tmax else tmax
        else:
            tmin = t1 if t1 > tmin else tmin
            tmax = t0 if t0 < tmax else tmax
        if tmax <= tmin:
            return False
    return True


def test_median_bvh_topology_matches_bvh_node(lib, scenes, oracle, golden):
    """RTG_BVH_MEDIAN reproduces bvh_node's tree (bvh_node.hpp:25-77): replaying the reference's
    unordered traversal (left, then right with t_max = rec.t) over the library's tree visits the
    primitives in exactly the order the reference's bvh_node::hit did, for all 160 golden rays."""
    s = scenes.build("bouncing_spheres", rand_seed=1, bvh_mode=rtgpu.RTG_BVH_MEDIAN)
    nodes, refs, depth = lib.bvh_build_host(s.desc)
    assert len(nodes) == 511 and len(refs) == 484  # 484 objects -> 511 nodes
    EMPTY = -2 ** 31

    def child(n, side):
        return n.child[side], list(n.lo[side]), list(n.hi[side])

    root = nodes[0]
    root_lo = [min(root.lo[0][k], root.lo[1][k]) for k in range(3)]
    root_hi = [max(root.hi[0][k], root.hi[1][k]) for k in range(3)]
    assert root_lo + root_hi == golden["book1_bvh"]["root_box"]

    def visit(code, lo, hi, ray, tmin, tmax, log):
        if code < 0:  # object: sphere::hit, no box test (bvh_node.hpp:89-90)
            pid = refs[-(code + 1)]
            log.append(pid)
            h, rec = oracle.sphere_hit(s.desc.prims[pid], ray["o"], ray["d"], ray["time"], tmin, tmax)
            return h, rec[0]
        if not _slab(lo, hi, ray["o"], ray["d"], tmin, tmax):
            return False, None
        n = nodes[code]
        left = child(n, 0)
        right = child(n, 1) if n.child[1] != EMPTY else left  # 1-object node: left = right (H8)
        hl, tl = visit(*left, ray, tmin, tmax, log)
        hr, tr = visit(*right, ray, tmin, tl if hl else tmax, log)
        return hl or hr, (tr if hr else tl)

    for ray in golden["book1_bvh"]["rays"]:
        log = []
        h, t = visit(0, root_lo, root_hi, ray, 0.001, math.inf, log)
        assert log == ray["order"]
        assert h == bool(ray["hit"]) and (not h or t == ray["t"])


@pytest.mark.parametrize("name,grid", [("bouncing_spheres", 11), ("bouncing_spheres", 40), ("tie_world", 0)])
def test_tie_ranks_are_the_median_tree_leaf_order(lib, scenes, name, grid):
    """The C++ mirror's bvh_node hands the order its hit() tests objects in as tie ranks (ABI 7,
    rtg_scene_desc.tie_rank, from rtg_bvh_node_order): for a world of primitives wrapped in one bvh_node that
    is the leaf order of the reference's median tree, which RTG_BVH_MEDIAN rebuilds node for node (pinned
    above), so the primitives sorted by rank are that build's leaf references exactly. Book-1's root sorts
    483 equal y-minima (std::sort's placement of equal keys matters); tie_world has compound children."""
    s = scenes.build(name, grid=grid)
    r = np.ctypeslib.as_array(s.desc.tie_rank, shape=(s.desc.num_prims,))
    assert sorted(r.tolist()) == list(range(s.desc.num_prims))
    if name == "tie_world":  # children of two quads: ranks keep each child's two primitives adjacent
        assert int(r[29]) == int(r[28]) + 1 and int(r[31]) == int(r[30]) + 1
        return
    m = scenes.build(name, grid=grid, bvh_mode=rtgpu.RTG_BVH_MEDIAN)
    _, refs, _ = lib.bvh_build_host(m.desc)
    assert np.argsort(r).tolist() == list(refs)


def test_bvh_node_order_matches_sort_semantics(lib):
    """rtg_bvh_node_order on hand-made boxes: spans of one and two are not sorted (bvh_node.hpp:53-62),
    three or more are sorted by box minimum on the longest axis of their box and split at the median."""
    def box(x, y=0.0, z=0.0, w=1.0):
        return [x, y, z, x + w, y + w, z + w]
    assert lib.bvh_node_order([box(5), box(1)]).tolist() == [0, 1]          # two: left, right as listed
    assert lib.bvh_node_order([box(5), box(1), box(3)]).tolist() == [1, 2, 0]  # three: sorted on x
    # longest axis y: sorted by y-min whatever the x order
    assert lib.bvh_node_order([box(0, 9, w=0.5), box(1, 0, w=0.5), box(2, 4, w=0.5)]).tolist() == [1, 2, 0]
    assert lib.bvh_node_order([]).tolist() == []


def test_tie_rank_must_be_a_permutation(lib, scenes):
    """rtg_scene_create validates tie_rank before any device work (RTG_E_INVALID anywhere); an ABI-6
    descriptor (no tie_rank field) is still accepted and read as list order (here: no device ->
    RTG_E_NODEVICE, i.e. it got past validation)."""
    import ctypes as C

    s = scenes.build("tie_world", grid=0)
    d = rtgpu.rtg_scene_desc.from_buffer_copy(s.desc)
    bad = (C.c_int64 * d.num_prims)(*([0] * d.num_prims))
    d.tie_rank = C.cast(bad, C.POINTER(C.c_int64))
    with pytest.raises(rtgpu.RtgError) as e:
        lib.scene_create(d)
    assert e.value.status == rtgpu.RTG_E_INVALID and "permutation" in str(e.value)
    if lib.device_count() == 0:
        d.abi_version = 6  # bytes past the ABI-6 layout (the bad ranks) are not read
        with pytest.raises(rtgpu.RtgError) as e:
            lib.scene_create(d)
        assert e.value.status == rtgpu.RTG_E_NODEVICE


@pytest.mark.parametrize("name", ["bouncing_spheres", "cornell_box", "simple_light"])
def test_sah_bvh_is_complete(lib, scenes, name):
    s = scenes.build(name, rand_seed=1, bvh_mode=rtgpu.RTG_BVH_SAH)
    nodes, refs, depth = lib.bvh_build_host(s.desc)
    assert sorted(refs) == list(range(s.desc.num_prims))  # every primitive exactly once
    EMPTY = -2 ** 31
    seen_nodes = {0}
    for n in nodes:
        for side in range(2):
            c = n.child[side]
            if c == EMPTY:
                continue
            assert n.lo[side][0] <= n.hi[side][0]
            if c >= 0:
                seen_nodes.add(c)
                cn = nodes[c]
                for s2 in range(2):  # child boxes nest in the parent's box for that child
                    if cn.child[s2] != EMPTY:
                        for k in range(3):
                            assert n.lo[side][k] <= cn.lo[s2][k] and cn.hi[s2][k] <= n.hi[side][k]
            else:
                assert 1 <= n.count[side] <= 4
    assert seen_nodes == set(range(len(nodes)))
    assert depth <= 64


def test_invalid_scene_reports_invalid(lib):
    prim = rtgpu.rtg_primitive(kind=rtgpu.RTG_PRIM_SPHERE, material=3, radius=1.0)
    desc = rtgpu.rtg_scene_desc(abi_version=rtgpu.RTG_ABI_VERSION, bvh_mode=rtgpu.RTG_BVH_SAH,
                                prims=C.pointer(prim), num_prims=1)
    with pytest.raises(rtgpu.RtgError) as e:
        lib.scene_create(desc)
    assert e.value.status == -1 and "material" in str(e.value)
    desc.abi_version = 99
    with pytest.raises(rtgpu.RtgError):
        lib.scene_create(desc)


def test_no_cpu_fallback_without_device(lib, scenes):
    if lib.device_count() > 0:
        pytest.skip("a device is present; the no-device path is exercised on CPU-only hosts")
    s = scenes.build("cornell_box", rand_seed=1)
    with pytest.raises(rtgpu.RtgError) as e:
        lib.scene_create(s.desc)
    assert e.value.status == -3  # RTG_E_NODEVICE: the render path fails loudly


@pytest.mark.skipif(not os.path.isdir(REFERENCE_SRC), reason="reference tree not present")
def test_reference_main_compiles_against_mirror(tmp_path):
    """Drop-in check: the reference's unmodified main.cpp builds against the C++ API mirror and
    links to librtgpu.so (it is fed on stdin so its own headers are not found first)."""
    inc = [f"-I{REPO}/raytracing-practice_amd/include", f"-I{REPO}/include"]
    with open(os.path.join(REFERENCE_SRC, "main.cpp"), "rb") as src:
        subprocess.run(["g++", "-std=c++17", "-Wno-unused-parameter", *inc, "-x", "c++", "-c", "-",
                        "-o", str(tmp_path / "main.o")], stdin=src, check=True, cwd=tmp_path)
    subprocess.run(["g++", str(tmp_path / "main.o"), f"-L{REPO}/raytracing-practice_amd/lib",
                    "-lrtgpu", "-o", str(tmp_path / "raytracer")], check=True)


def test_parallel_ppm_body_matches_write_color(tmp_path):
    """camera::write_ppm_body (threads format the P3 text) writes exactly the bytes of the
    reference's per-pixel write_color stream (color.hpp:26-58)."""
    src = tmp_path / "ppm.cpp"
    src.write_text(r'''
#include <cstdio>
#include <random>
#include <sstream>
#include "core/camera.hpp"
int main() {
  std::mt19937 g(7);
  std::uniform_real_distribution<float> u(-0.1f, 1.4f);
  std::vector<float> rgb(3 * 50000);
  for (float& x : rgb) x = u(g);
  rgb[0] = 0.0f; rgb[1] = 0.998001f; rgb[2] = 1e-9f;
  std::ostringstream a, b;
  camera::write_ppm_body(a, rgb);
  for (size_t k = 0; k < rgb.size(); k += 3) write_color(b, color(rgb[k], rgb[k + 1], rgb[k + 2]));
  std::printf("%d %zu\n", a.str() == b.str() ? 1 : 0, a.str().size());
  return a.str() == b.str() ? 0 : 1;
}
''')
    inc = [f"-I{REPO}/raytracing-practice_amd/include", f"-I{REPO}/include"]
    subprocess.run(["g++", "-std=c++17", "-O1", *inc, str(src), "-pthread", "-o", str(tmp_path / "ppm")],
                   check=True)
    r = subprocess.run([str(tmp_path / "ppm")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout


def test_write_color_bytes_matches_oracle(oracle):
    """rtgpu.write_color_bytes (the host twin of rtg_resolve_rgb8, used for RGB8 gathers) equals
    the oracle's write_color, itself pinned to the reference (test_oracle_golden)."""
    rng = np.random.default_rng(3)
    vals = np.concatenate([rng.uniform(-0.2, 1.3, 3000), [0.0, 0.998001, 0.99800104, 1e-12, 1.0]])
    vals = vals.astype(np.float32)
    got = rtgpu.write_color_bytes(vals.reshape(-1, 1).repeat(3, axis=1))[:, 0]
    want = [oracle.write_color([float(v)] * 3)[0] for v in vals]
    assert np.array_equal(got.astype(int), np.array(want))


def test_parallel_sah_build_is_the_single_thread_tree(lib, scenes, monkeypatch):
    """The host SAH builder runs its top-level loops and large subtrees on several threads (config 5's
    setup, DESIGN.md §3 "BVH"): bins merge by exact min / max and counts, the partitions stay
    sequential and subtrees are spliced in depth-first order, so the tree (nodes, boxes, leaf refs)
    must be the single-thread build's, bit for bit. 90k spheres: subtrees above 32k primitives spawn,
    loops above 64k run data-parallel."""
    import ctypes as C

    s = scenes.build("bouncing_spheres", grid=150, rand_seed=1)
    d = rtgpu.rtg_scene_desc.from_buffer_copy(s.desc)
    d.bvh_mode = rtgpu.RTG_BVH_SAH
    trees = {}
    for t in ("1", "8"):
        monkeypatch.setenv("RTG_BUILD_THREADS", t)
        nn, nr, depth = C.c_int64(0), C.c_int64(0), C.c_int32(0)
        lib.check("rtg_bvh_build_host", lib.lib.rtg_bvh_build_host(
            C.byref(d), None, 0, None, 0, C.byref(nn), C.byref(nr), C.byref(depth)))
        nodes = (rtgpu.rtg_bvh_node_host * nn.value)()
        refs = (C.c_int64 * nr.value)()
        lib.check("rtg_bvh_build_host", lib.lib.rtg_bvh_build_host(
            C.byref(d), nodes, nn.value, refs, nr.value, C.byref(nn), C.byref(nr), C.byref(depth)))
        trees[t] = (bytes(nodes), bytes(refs), depth.value)
    assert nn.value > 40000 and trees["1"] == trees["8"]


def test_hot_treelet_order_keeps_the_tree(lib):
    """rtg_hot_treelet_order_host, the host twin of rtg_scene_prepare's renumbering (DESIGN.md §3 "hot
    treelet"): the root stays node 0, the others follow by descending visits (ties in their previous
    order), inner child codes (byte offsets) are remapped, leaf and empty codes kept — so walking the
    tree from the root reaches the same node records in the same slot order."""
    rng = np.random.default_rng(7)
    n = 300
    nodes = np.zeros((n, 28), dtype=np.int32)
    nodes[:, :24] = rng.integers(-2**20, 2**20, size=(n, 24))  # plane payload: just carried along
    nodes[:, 24:] = np.iinfo(np.int32).min                      # empty slots
    nxt = 1
    for k in range(n):  # a random 4-wide tree in depth-first-ish order, leaves as negative codes
        for c in range(rng.integers(1, 5)):
            if k < nxt < n and rng.random() < 0.8:  # children after their parent: no cycles
                nodes[k, 24 + c] = nxt * 112
                nxt += 1
            else:
                nodes[k, 24 + c] = ~((int(rng.integers(0, 4096)) << 3) | int(rng.integers(0, 4)))
    assert nxt == n
    visits = rng.integers(0, 50, size=n).astype(np.uint32)
    visits[0] = 7  # the root keeps index 0 whatever its count
    out = lib.hot_treelet_order_host(nodes, visits)
    order = sorted(range(1, n), key=lambda k: -int(visits[k]))  # Python's sort is stable
    assert (out[0, :24] == nodes[0, :24]).all()
    for new, old in enumerate([0] + order):
        assert (out[new, :24] == nodes[old, :24]).all()

    def walk(a, k, acc):
        acc.append(tuple(a[k, :24]))
        for c in range(4):
            code = int(a[k, 24 + c])
            if code >= 0:
                assert code % 112 == 0
                walk(a, code // 112, acc)
            else:
                acc.append(code)
        return acc

    import sys
    sys.setrecursionlimit(10000)
    assert walk(out, 0, []) == walk(nodes, 0, [])
    bad = nodes.copy()
    bad[5, 24] = n * 112  # a code past the array is rejected, nothing renumbered
    with pytest.raises(rtgpu.RtgError):
        lib.hot_treelet_order_host(bad, visits)


def test_ctypes_structs_match_the_header(tmp_path):
    """Every ctypes mirror of an include/rtgpu.h struct (python/rtgpu.py) has the C compiler's size and
    field offsets: a field added to the header (e.g. round 4's plan words ray_queue / node_width) but
    not to the binding would otherwise shift every later field silently."""
    structs = sorted(n for n in dir(rtgpu) if n.startswith("rtg_") and isinstance(getattr(rtgpu, n), type)
                     and issubclass(getattr(rtgpu, n), C.Structure))
    assert "rtg_launch_plan" in structs and "rtg_render_desc" in structs
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "rtgpu.h"', "int main(void) {"]
    expect = []
    for n in structs:
        cls = getattr(rtgpu, n)
        lines.append(f'printf("{n} %zu\\n", sizeof({n}));')
        expect.append(f"{n} {C.sizeof(cls)}")
        for f in cls._fields_:
            lines.append(f'printf("{n}.{f[0]} %zu\\n", offsetof({n}, {f[0]}));')
            expect.append(f"{n}.{f[0]} {getattr(cls, f[0]).offset}")
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    assert [g for g in got if g] == expect
