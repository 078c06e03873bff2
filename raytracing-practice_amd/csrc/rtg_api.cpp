// rtg_api.cpp — the extern "C" boundary of librtgpu.so (include/rtgpu.h).
//
// Host responsibilities: validate the flat scene, run camera::initialize in fp64
// (camera.hpp:76-136), build + flatten the BVH (rtg_bvh.cpp), upload the scene once, and launch
// the gfx950 render kernel (rtg_kernels.hip) on the caller's stream. No CPU fallback exists:
// without a usable device every entry point that renders returns RTG_E_NODEVICE / RTG_E_HIP.
#include <algorithm>
#include <atomic>
#include <array>
#include <functional>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <thread>
#include <vector>

#include "rtg_internal.hpp"

namespace rtg {
hipError_t launch_combine(const float* partial, float* out, int64_t n_pixels, int chunks, float scale,
                          hipStream_t stream);
hipError_t launch_repad(float* nodes, int64_t num_nodes, int width, float delta, hipStream_t stream);
KernelChoice choose_kernel(const DevScene& S, const DevJob& J, int stack, bool count, int variant);
hipError_t launch_render(const KernelChoice& k, const DevScene& S, const DevCamera& C, const DevJob& J,
                         int lds_bytes, int grid_blocks, hipStream_t stream);
KernelResources kernel_resources(const void* fn);
int lds_layout(const DevScene& S, int stack, int waves, int esz, DevJob* J);
int lds_layout_treelet(DevScene* S, int stack, int waves, DevJob* J);
bool dual_fits_registers(bool count, bool ring, bool verbose);
hipError_t launch_resolve(const float* in, uint8_t* out, int64_t n_pixels, hipStream_t stream);
}  // namespace rtg

using namespace rtg;

namespace {
constexpr int kMaxStackNeed = 4096;     // traversal stack entries per lane (LDS part + global spill)
constexpr int kPlainWgsPerCu = 5;        // schedule 4 grid: resident workgroups per CU (waves pull work)
constexpr int kDefaultShadeBatch = 48;  // of 64 live lanes: measured best on book-1
constexpr int kTexShadeBatch = 56;      // ... and on scenes with image / noise textures
constexpr int kCacheShadeBatch = 40;    // ... and where nodes come through the caches (config 5)
constexpr int kDefaultLeafBatch = 12;   // lanes waiting at a leaf before a leaf trip
// Scenes with a handful of BVH nodes once waited for 48 lanes (Cornell -15 % with the SAH cost 0.7
// tree, profiles/r01_leafbatch); with the cost 0.5 tree and the ground occluder 12 is as good or
// better there too (Cornell 13.97 -> 13.56 ms at 800x450x300, earth_perlin 17.40 vs 17.43 ms); with
// the cheaper round-2 trip (kTravDone) 16 is best again: Cornell -1.2 %, earth_perlin +0.3 %
constexpr int kSmallBvhNodes = 16;
constexpr int kSmallBvhLeafBatch = 16;
constexpr int kLdsWaves = 16;           // persistent LDS workgroup size (rtg_kernels.hip)
constexpr int kSmallSceneWgs = 5;       // 4-wave persistent workgroups per CU for small scenes
// full-frame partials above this: the tile ring. 32 GiB of the MI355X's 288 GB: config 5's 6.3 GB of partials
// (4K, 63 chunks) stay full-frame since round 5 — its render loop is 2.0 % faster without the ring's
// bookkeeping and its HBM writes drop from 16.3 GB (ring slots + the ring kernel's scratch) to the
// partials' 6.3 GB (profiles/r05_dd, r05_final); the ring remains for frames whose partials would not fit
constexpr int64_t kRingAutoBytes = int64_t(32) << 30;
constexpr int kNumCounters = 28;        // see DevJob::counters ([8..23] diagnostics, [24..25] tile ring, [26] stack spills)
// gfx950 allocates a workgroup's LDS in 1280-byte granules (160 KB = 128 of them): measured with the
// dual launch, whose two workgroups stop sharing a CU exactly when the rounded sizes pass 160 KB
constexpr int kLdsGranule = 1280;
constexpr int kLdsPerCu = 160 * 1024;
int lds_alloc(int bytes) { return (bytes + kLdsGranule - 1) / kLdsGranule * kLdsGranule; }
}

namespace {

thread_local std::string g_last_error;

rtg_status fail(rtg_status code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

rtg_status hip_fail(hipError_t e, const char* what) {
  return fail(e == hipErrorOutOfMemory ? RTG_E_NOMEM : RTG_E_HIP,
              std::string(what) + ": " + hipGetErrorString(e));
}

#define RTG_HIP(call, what)                   \
  do {                                        \
    hipError_t e_ = (call);                   \
    if (e_ != hipSuccess) return hip_fail(e_, what); \
  } while (0)

// A render that returns an error after enqueuing work waits for its stream first, so the scene's scratch
// (below) is idle again whatever the caller does next.
struct SyncOnError {
  hipStream_t stream = nullptr;
  bool committed = false;
  ~SyncOnError() {
    if (!committed && stream) (void)hipStreamSynchronize(stream);  // error path: the first error is reported
  }
};

// ---- fp64 vector helpers with the reference's operator semantics (vec3.hpp:100-155) ----
struct D3 {
  double x, y, z;
};
D3 d3(const double v[3]) { return D3{v[0], v[1], v[2]}; }
D3 operator+(D3 a, D3 b) { return D3{a.x + b.x, a.y + b.y, a.z + b.z}; }
D3 operator-(D3 a, D3 b) { return D3{a.x - b.x, a.y - b.y, a.z - b.z}; }
D3 operator-(D3 a) { return D3{-a.x, -a.y, -a.z}; }
D3 operator*(double t, D3 a) { return D3{t * a.x, t * a.y, t * a.z}; }
D3 operator/(D3 a, double t) { return (1 / t) * a; }
double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
D3 cross(D3 a, D3 b) {
  return D3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
D3 unit_vector(D3 v) { return v / std::sqrt(dot(v, v)); }
void put(double o[3], D3 v) {
  o[0] = v.x;
  o[1] = v.y;
  o[2] = v.z;
}

float round_down(double x) {
  float f = static_cast<float>(x);
  if (static_cast<double>(f) > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
  return f;
}
float round_up(double x) {
  float f = static_cast<float>(x);
  if (static_cast<double>(f) < x) f = std::nextafter(f, std::numeric_limits<float>::infinity());
  return f;
}
float ibits_to_float(int32_t i) {
  float f;
  std::memcpy(&f, &i, 4);
  return f;
}

uint64_t mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xbf58476d1ce4e5b9ull;
  z ^= z >> 27;
  z *= 0x94d049bb133111ebull;
  z ^= z >> 31;
  return z;
}

// Host loops over large scenes (config 5: 1M primitives, 400k nodes) in contiguous chunks on up to 16
// threads (the GPU box's cgroup quota); fn(begin, end, t). Small ranges run inline.
template <class F>
void host_par_for(int64_t n, F&& fn) {
  int T = static_cast<int>(std::thread::hardware_concurrency());
  T = std::min(16, std::max(1, T));
  if (n < 65536) T = 1;
  if (T == 1) {
    fn(int64_t(0), n, 0);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back([&, t]() { fn(n * t / T, n * (t + 1) / T, t); });
  fn(int64_t(0), n / T, 0);
  for (auto& x : th) x.join();
}
int host_threads(int64_t n) {
  const int T = std::min(16, std::max(1, static_cast<int>(std::thread::hardware_concurrency())));
  return n < 65536 ? 1 : T;
}

// Culling margin (DESIGN.md §4 "conservative culling"). Every BVH box the kernels test is the union of its
// primitives' culling boxes, each the reference's box with every plane v moved outward by an eta that depends
// on the primitive and the axis, then rounded outward to fp32. M is the largest |coordinate| of the primitive
// boxes, so of every hit point a later segment starts from; every origin with |o| <= 2M is covered
// (ensure_origin_bound widens the device boxes for a camera farther out). The kernels' slab test
// fma(plane, rcp(d), -o rcp(d)) computes a plane's distance t within 3 2^-24 |t| + 2^-24 |o / d| (v_rcp_f32:
// 1 ulp; the rounded -o rcp(d); the fma); children are culled against fmaf(tbest, 1 + 2^-19, 2^-19) with the
// exit floor at 0.0009, and kernels that test quads compare the entry with min(exit, tbest) (1 + 2^-19)
// instead (kCullWiden: the relative margin taken on the exit distance too).
// - spheres, every axis: eta = 2^-21 (|v| + M) >= 3 2^-24 |v - o| + 2^-24 |o| for |o| <= 2M: no computed entry
//   (exit) distance is past the unpadded box's true one; the rest covers the discriminant letting a ray
//   graze a face.
// - axis-aligned quads (quad_flat_axis; quad_t's root t_c is then within 2 2^-24 of the true crossing t*,
//   and the hit point it accepts lies past the edge through Q by at most 2^-24 |p| (the sign of p - Q is
//   exact) and past the far edge by at most 4 2^-24 |u| + 2^-24 |p|): on the flat axis k eta = 2^-23 (|v| + M)
//   (1 + 2^-16) >= 2^-24 |o| (1 + 2^-20) + the rounding of Q_k; on an in-plane axis a, with U_a the quad's
//   extent along it, eta = 2^-24 (6 U_a + 3 |v| + 2M) (1 + 2^-10) >= 4 2^-24 U_a (alpha or beta, and p - Q) +
//   2^-24 (|Q_a| + U_a) (the record's rounded corners) + 2^-24 |p| (p ~ v) + 2^-24 |o| (|o| <= 2M), so a quad's
//   box reaches past its neighbours' planes by less than the exit floor for most rays leaving them (Cornell's
//   blocks: a ray leaving a face enters the block's node when that reach exceeds 0.0009 of its exit
//   distance). What grows with the distance
//   (the slab's and quad_t's relative errors, <= 5 2^-24 of t) is taken by kCullWiden, so the computed entry
//   distance never exceeds the computed exit of a box holding an accepted hit, nor the cull bound. A flat box
//   stays thin: a ray leaving the quad at a shallow angle leaves it before the exit floor.
// - other quads, every axis: eta = 2^-18 (|v| + M): their float normal and plane distance are rounded, so
//   the accepted points leave the corners' box by a few 2^-24 (|v| + M) plus 2^-24 of the distance
//   (<= |v| + 2M), all taken in the pad.
// The flat axis of an axis-aligned quad (u and v each along one coordinate axis, so the record's normal is
// exactly +-e_k, its plane distance +-Q_k, and alpha / beta each depend on one coordinate of the hit point),
// or -1.
int quad_flat_axis(const rtg_primitive& p) {
  auto axis_of = [](const double v[3]) {
    const int nz = (v[0] != 0.0) + (v[1] != 0.0) + (v[2] != 0.0);
    return nz != 1 ? -1 : v[0] != 0.0 ? 0 : v[1] != 0.0 ? 1 : 2;
  };
  const int i = axis_of(p.p1), j = axis_of(p.p2);
  if (i < 0 || j < 0 || i == j) return -1;
  const int k = 3 - i - j;
  const D3 n = unit_vector(cross(d3(p.p1), d3(p.p2)));  // as the quad record's normal (compile_scene)
  const double c[3] = {n.x, n.y, n.z};
  return std::fabs(c[k]) == 1.0 && c[i] == 0.0 && c[j] == 0.0 ? k : -1;
}
void culling_box(const rtg_primitive& p, double m, double lo[3], double hi[3]) {
  prim_bbox(p, lo, hi);
  const int flat = p.kind == RTG_PRIM_QUAD ? quad_flat_axis(p) : -1;
  if (flat >= 0) lo[flat] = hi[flat] = p.p0[flat];  // the reference's 0.0001 minimum extent is not needed here
  for (int a = 0; a < 3; ++a) {
    if (p.kind == RTG_PRIM_QUAD && flat >= 0 && a != flat) {  // in-plane: 2^-24 (6 |U_a| + 3 |v| + 2M)
      const double ua = std::fabs(p.p1[a]) + std::fabs(p.p2[a]), k = 0x1p-24 * (1.0 + 0x1p-10);
      lo[a] -= k * (6.0 * ua + 3.0 * std::fabs(lo[a]) + 2.0 * m);
      hi[a] += k * (6.0 * ua + 3.0 * std::fabs(hi[a]) + 2.0 * m);
      continue;
    }
    const double c = p.kind == RTG_PRIM_SPHERE ? 0x1p-21 : flat < 0 ? 0x1p-18 : 0x1p-23 * (1.0 + 0x1p-16);
    lo[a] -= c * (std::fabs(lo[a]) + m);
    hi[a] += c * (std::fabs(hi[a]) + m);
  }
}
// Replace the child boxes of a built tree (binary or W-wide; leaves -(1 + first ref), count) by the unions of
// their primitives' culling boxes. The tree itself (built from the reference's boxes) is unchanged.
template <class Node, int W>
void refit_culling_boxes(std::vector<Node>& nodes, const std::vector<int64_t>& refs, const rtg_scene_desc* d,
                         double m) {
  if (nodes.empty()) return;
  std::vector<std::array<double, 6>> pb(refs.size());
  host_par_for(static_cast<int64_t>(refs.size()), [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e; ++i) culling_box(d->prims[refs[i]], m, pb[i].data(), pb[i].data() + 3);
  });
  struct Refit {
    std::vector<Node>& nodes;
    const std::vector<std::array<double, 6>>& pb;
    void node(int32_t k, double lo[3], double hi[3]) {  // refits node k, returns the union of its children
      Node& n = nodes[k];
      for (int a = 0; a < 3; ++a) lo[a] = HUGE_VAL, hi[a] = -HUGE_VAL;
      for (int c = 0; c < W; ++c) {
        if (n.child[c] == kEmptyChild) continue;
        double cl[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, ch[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
        if (n.child[c] >= 0) {
          node(n.child[c], cl, ch);
        } else {
          const int64_t first = -(static_cast<int64_t>(n.child[c]) + 1);
          for (int64_t r = first; r < first + n.count[c]; ++r)
            for (int a = 0; a < 3; ++a) cl[a] = std::min(cl[a], pb[r][a]), ch[a] = std::max(ch[a], pb[r][3 + a]);
        }
        for (int a = 0; a < 3; ++a) {
          n.lo[c][a] = cl[a], n.hi[c][a] = ch[a];
          lo[a] = std::min(lo[a], cl[a]), hi[a] = std::max(hi[a], ch[a]);
        }
      }
    }
  } rf{nodes, pb};
  double lo[3], hi[3];
  rf.node(0, lo, hi);
}

bool texture_uses_uv(const rtg_scene_desc* d, int32_t tex, int depth) {
  if (depth > 16 || tex < 0 || tex >= d->num_textures) return false;
  const rtg_texture& t = d->textures[tex];
  if (t.type == RTG_TEX_IMAGE) return true;
  if (t.type == RTG_TEX_CHECKER)
    return texture_uses_uv(d, t.even, depth + 1) || texture_uses_uv(d, t.odd, depth + 1);
  return false;
}

bool validate_texture(const rtg_scene_desc* d, int32_t tex, int depth, std::string* err) {
  if (tex < 0 || tex >= d->num_textures) {
    *err = "texture index out of range";
    return false;
  }
  if (depth >= 16) {
    *err = "checker textures nested deeper than 16 (or cyclic)";
    return false;
  }
  const rtg_texture& t = d->textures[tex];
  switch (t.type) {
    case RTG_TEX_SOLID:
      return true;
    case RTG_TEX_CHECKER:
      return validate_texture(d, t.even, depth + 1, err) && validate_texture(d, t.odd, depth + 1, err);
    case RTG_TEX_IMAGE:
      if (t.image >= d->num_images) {
        *err = "image index out of range";
        return false;
      }
      return true;
    case RTG_TEX_NOISE:
      if (t.perlin < 0 || t.perlin >= d->num_perlins) {
        *err = "perlin index out of range";
        return false;
      }
      return true;
    default:
      *err = "unknown texture type";
      return false;
  }
}

}  // namespace

namespace rtg {

rtg_status set_last_error(rtg_status code, const std::string& msg) { return fail(code, msg); }

Knobs read_knobs() {
  Knobs k;
  auto num = [](const char* name, int lo, int hi, int* out) {
    const char* e = std::getenv(name);
    if (!e || !*e) return false;
    char* end = nullptr;
    const long v = std::strtol(e, &end, 10);
    if (*end != '\0' || v < lo || v > hi) {
      std::fprintf(stderr, "[rtg] ignoring %s=%s (expected %d..%d)\n", name, e, lo, hi);
      return false;
    }
    *out = static_cast<int>(v);
    return true;
  };
  k.verbose = std::getenv("RTG_VERBOSE") != nullptr;
  num("RTG_TILE_LW", 0, 6, &k.tile_lw);
  num("RTG_CHUNK_SAMPLES", 1, 63, &k.chunk_samples);  // <= 63: the kernels pack a unit's samples left in 6 bits
  num("RTG_STACK_LDS_ENTRIES", 1, 32, &k.stack_lds_entries);
  int w = 0;
  if (num("RTG_LDS_WAVES", 4, 16, &w) && (w == 4 || w == 16)) k.lds_waves = w;
  num("RTG_DUAL", 0, 1, &k.dual);
  int ts = 0;  // tile-ring slots: 0 or a power of two (tests shrink the ring to force slot waits)
  if (num("RTG_TILE_SLOTS", 0, 65536, &ts) && (ts & (ts - 1)) == 0) k.tile_slots = ts;
  num("RTG_TREELET_STACK", 4, 16, &k.treelet_stack);
  num("RTG_TREELET_HOT", 0, 1, &k.treelet_hot);
  num("RTG_TILE_ORDER", 0, 1, &k.tile_order);
  num("RTG_TILE_ORDER_SPP", 1, 64, &k.tile_order_spp);
  if (const char* e = std::getenv("RTG_WAVE_TRACE")) k.wave_trace = e;
  return k;
}

void resolve_camera(const rtg_camera_desc* cam, rtg_camera_params* o) {
  // camera::initialize (camera.hpp:76-136), fp64 with the reference's float-literal quirks.
  const double pi = 3.1415926535897932385;
  const int W = cam->image_width;
  int H = static_cast<int>(W / cam->aspect_ratio);
  H = (H < 1) ? 1 : H;
  o->image_width = W;
  o->image_height = H;
  o->pixel_samples_scale = static_cast<double>(1.0f / cam->samples_per_pixel);
  const double theta = cam->vfov * pi / 180.0f;
  const double h = std::tan(theta / 2);
  const double viewport_height = 2 * h * cam->focus_dist;
  const double viewport_width = viewport_height * (static_cast<double>(W) / H);
  const D3 center = d3(cam->lookfrom);
  const D3 w = unit_vector(d3(cam->lookfrom) - d3(cam->lookat));
  const D3 u = unit_vector(cross(d3(cam->vup), w));
  const D3 v = cross(w, u);
  const D3 viewport_u = viewport_width * u;
  const D3 viewport_v = viewport_height * -v;
  const D3 du = viewport_u / W;
  const D3 dv = viewport_v / H;
  const D3 upper_left = center - (cam->focus_dist * w) - viewport_u / 2 - viewport_v / 2;
  const D3 p00 = upper_left + 0.5 * (du + dv);
  const double defocus_radius = cam->focus_dist * std::tan(cam->defocus_angle * pi / 180.0f / 2.0f);
  put(o->center, center);
  put(o->pixel00_loc, p00);
  put(o->pixel_delta_u, du);
  put(o->pixel_delta_v, dv);
  put(o->u, u);
  put(o->v, v);
  put(o->w, w);
  put(o->defocus_disk_u, defocus_radius * u);
  put(o->defocus_disk_v, defocus_radius * v);
}

// W-wide nodes, 28 W bytes: lo.x[W], lo.y[W], lo.z[W], hi.x[W], hi.y[W], hi.z[W], code[W]; inner child
// codes are byte offsets of the child node, leaf codes ~((first << 3) | (count - 1)), empty slots
// kEmptyChild with the inverted box (+inf, -inf). Boxes rounded outward to fp32.
template <int W>
bool emit_wide(const BvhW<W>& t, HostScene* out, std::string* err) {
  constexpr int64_t kBytes = node_bytes(W), kWords = 7 * W;
  if (t.nodes.size() > static_cast<size_t>(INT32_MAX / kBytes)) {
    *err = "BVH too large for 32-bit node offsets";
    return false;
  }
  out->nodes.resize(t.nodes.size() * kWords);
  const int64_t nn = static_cast<int64_t>(t.nodes.size());
  std::vector<int> bad(host_threads(nn), 0);  // 1: a node without children, 2: a leaf not encodable
  host_par_for(nn, [&](int64_t b, int64_t e, int th) {
    for (int64_t k = b; k < e && !bad[th]; ++k) {
      const BuildNodeW<W>& n = t.nodes[k];
      float* f = &out->nodes[k * kWords];
      if (n.child[0] == kEmptyChild) {
        bad[th] = 1;
        break;
      }
      for (int c = 0; c < W; ++c) {
        int32_t code = kEmptyChild;
        const bool empty = n.child[c] == kEmptyChild;
        if (!empty) {
          if (n.child[c] >= 0) {
            code = static_cast<int32_t>(n.child[c] * kBytes);  // inner children: byte offset of the node
          } else {
            const int64_t first = -(static_cast<int64_t>(n.child[c]) + 1);
            if (n.count[c] < 1 || n.count[c] > 8 || first >= (int64_t(1) << 28)) {
              bad[th] = 2;
              break;
            }
            code = ~static_cast<int32_t>((first << 3) | (n.count[c] - 1));
          }
        }
        for (int a = 0; a < 3; ++a) {
          f[a * W + c] = empty ? std::numeric_limits<float>::infinity() : round_down(n.lo[c][a]);
          f[3 * W + a * W + c] = empty ? -std::numeric_limits<float>::infinity() : round_up(n.hi[c][a]);
        }
        f[6 * W + c] = ibits_to_float(code);
      }
    }
  });
  for (const int b : bad) {
    if (b == 1) {
      *err = "wide BVH node without children";
      return false;
    }
    if (b == 2) {
      *err = "BVH leaf not encodable";
      return false;
    }
  }
  return true;
}

bool compile_scene(const rtg_scene_desc* d, HostScene* out, std::string* err) {
  // phase timings of the host compile (RTG_VERBOSE): config 5's 1M spheres make these the setup cost
  const bool verbose = std::getenv("RTG_VERBOSE") != nullptr;
  auto tp = std::chrono::steady_clock::now();
  auto phase = [&](const char* what) {
    const auto now = std::chrono::steady_clock::now();
    const double ms = std::chrono::duration<double, std::milli>(now - tp).count();
    if (verbose) std::fprintf(stderr, "[rtg] compile %-10s %8.1f ms\n", what, ms);
    if (std::strcmp(what, "bvh") == 0) out->bvh_ms += ms;
    if (std::strcmp(what, "collapse") == 0 || std::strcmp(what, "bfs") == 0) out->collapse_ms += ms;
    tp = now;
  };
  if (d->num_prims < 0 || (d->num_prims > 0 && !d->prims) || d->num_materials < 0 ||
      (d->num_materials > 0 && !d->materials) || d->num_textures < 0 ||
      (d->num_textures > 0 && !d->textures) || d->num_images < 0 ||
      (d->num_images > 0 && !d->images) || d->num_perlins < 0 ||
      (d->num_perlins > 0 && !d->perlins)) {
    *err = "malformed scene descriptor (negative count or null array)";
    return false;
  }
  for (int32_t m = 0; m < d->num_materials; ++m) {
    const rtg_material& mt = d->materials[m];
    if (mt.type == RTG_MAT_LAMBERTIAN || mt.type == RTG_MAT_DIFFUSE_LIGHT) {
      if (!validate_texture(d, mt.texture, 0, err)) return false;
    } else if (mt.type != RTG_MAT_METAL && mt.type != RTG_MAT_DIELECTRIC) {
      *err = "unknown material type";
      return false;
    }
  }
  for (int64_t i = 0; i < d->num_prims; ++i) {
    const rtg_primitive& p = d->prims[i];
    if (p.kind != RTG_PRIM_SPHERE && p.kind != RTG_PRIM_QUAD) {
      *err = "unknown primitive kind at index " + std::to_string(i);
      return false;
    }
    if (p.material < 0 || p.material >= d->num_materials) {
      *err = "primitive material index out of range at index " + std::to_string(i);
      return false;
    }
  }
  // tie ranks (ABI 7): a permutation of the primitive indices, or none (list order)
  if (d->tie_rank) {
    if (d->num_prims > INT32_MAX) {
      *err = "tie_rank needs fewer than 2^31 primitives";
      return false;
    }
    std::vector<uint8_t> seen(static_cast<size_t>(d->num_prims), 0);
    for (int64_t i = 0; i < d->num_prims; ++i) {
      const int64_t r = d->tie_rank[i];
      if (r < 0 || r >= d->num_prims || seen[r]) {
        *err = "tie_rank is not a permutation of the primitive indices (index " + std::to_string(i) + ")";
        return false;
      }
      seen[r] = 1;
    }
  }
  auto tie_rank = [d](int64_t i) -> int64_t { return d->tie_rank ? d->tie_rank[i] : i; };
  // M of the culling margin (culling_box): the largest |coordinate| of any primitive box, i.e. of any hit
  // point a later segment starts from; rtg_render widens the boxes when a camera lies farther out
  {
    const int T = host_threads(d->num_prims);
    std::vector<double> part(T, 0.0);
    host_par_for(d->num_prims, [&](int64_t b, int64_t e, int t) {
      double m = 0.0;
      for (int64_t i = b; i < e; ++i) {
        double lo[3], hi[3];
        prim_bbox(d->prims[i], lo, hi);
        for (int a = 0; a < 3; ++a) m = std::max({m, std::fabs(lo[a]), std::fabs(hi[a])});
        if (!std::isfinite(lo[0] + lo[1] + lo[2] + hi[0] + hi[1] + hi[2])) m = HUGE_VAL;
      }
      part[t] = m;
    });
    out->origin_bound = 0.0;
    for (const double m : part) out->origin_bound = std::max(out->origin_bound, m);
    if (!(out->origin_bound < 1e30)) {
      *err = "primitive coordinates are not finite (or above 1e30)";
      return false;
    }
  }

  // internal mode 2 = SAH kept binary (diagnostic A/B of the node width)
  rtg_scene_desc bd = *d;
  const bool binary_sah = d->bvh_mode == 2;
  if (binary_sah) bd.bvh_mode = RTG_BVH_SAH;
  const bool gpu_bvh = d->bvh_mode == RTG_BVH_GPU;
  Bvh bvh;
  // 4-wide trees (host SAH or device-built): a sphere whose box covers at least half of the scene
  // box's surface area (a ground sphere) is kept out of the tree; every ray tests it before
  // traversing, so the leaf trips it would cost are gone and the traversal starts with its hit as
  // the closest so far
  int64_t occ = -1;
  if ((d->bvh_mode == RTG_BVH_SAH || gpu_bvh) && d->num_prims > 1 && !std::getenv("RTG_NO_OCCLUDER")) {
    double slo[3] = {1e300, 1e300, 1e300}, shi[3] = {-1e300, -1e300, -1e300};
    std::vector<double> area(d->num_prims);
    {
      const int T = host_threads(d->num_prims);
      std::vector<std::array<double, 6>> part(T, {1e300, 1e300, 1e300, -1e300, -1e300, -1e300});
      host_par_for(d->num_prims, [&](int64_t b, int64_t e, int t) {
        std::array<double, 6>& m = part[t];
        for (int64_t i = b; i < e; ++i) {
          double lo[3], hi[3];
          prim_bbox(d->prims[i], lo, hi);
          for (int a = 0; a < 3; ++a) {
            m[a] = std::min(m[a], lo[a]);
            m[3 + a] = std::max(m[3 + a], hi[a]);
          }
          const double ex = hi[0] - lo[0], ey = hi[1] - lo[1], ez = hi[2] - lo[2];
          area[i] = ex * ey + ey * ez + ez * ex;
        }
      });
      for (const auto& m : part)
        for (int a = 0; a < 3; ++a) {
          slo[a] = std::min(slo[a], m[a]);
          shi[a] = std::max(shi[a], m[3 + a]);
        }
    }
    const double ex = shi[0] - slo[0], ey = shi[1] - slo[1], ez = shi[2] - slo[2];
    const double scene_area = ex * ey + ey * ez + ez * ex;
    for (int64_t i = 0; i < d->num_prims; ++i)
      if (d->prims[i].kind == RTG_PRIM_SPHERE && area[i] >= 0.5 * scene_area && (occ < 0 || area[i] > area[occ]))
        occ = i;
  }
  out->occluder_prim = occ;
  if (gpu_bvh) {  // primitives in input order; the device builds the tree (rtg_gpubvh.hip)
    if (d->num_prims > (int64_t(1) << 28) || d->num_prims > INT32_MAX / 112) {
      *err = "too many primitives for the device BVH builder";
      return false;
    }
    bvh.refs.reserve(d->num_prims);
    for (int64_t i = 0; i < d->num_prims; ++i)
      if (i != occ) bvh.refs.push_back(i);
  } else {
    std::vector<rtg_primitive> rest;
    if (occ >= 0) {
      rest.reserve(d->num_prims - 1);
      for (int64_t i = 0; i < d->num_prims; ++i)
        if (i != occ) rest.push_back(d->prims[i]);
      bd.prims = rest.data();
      bd.num_prims = d->num_prims - 1;
    }
    phase("validate");
    if (!build_bvh(&bd, &bvh, err)) return false;
    phase("bvh");
    if (occ >= 0)  // refs back to input indices
      for (auto& r : bvh.refs) r = r >= occ ? r + 1 : r;
  }
  out->num_prims = d->num_prims;
  out->num_nodes = static_cast<int64_t>(bvh.nodes.size());
  out->depth = bvh.depth;
  out->stack_need = bvh.depth;
  out->node_width = 2;
  Bvh4 bvh4;
  if (gpu_bvh) {
    out->gpu_bvh = true;
    out->node_width = 4;
    out->node_capacity = std::max<int64_t>(1, static_cast<int64_t>(bvh.refs.size()));
    out->num_nodes = 0;
    out->depth = 0;
    out->stack_need = 0;
  } else if (d->bvh_mode == RTG_BVH_SAH && !bvh.nodes.empty()) {
    // 4-wide collapse: SAH-optimal (dynamic program, leaves <= 4) by default: Cornell 800x800 2000 spp
    // -2.7 % against the greedy collapse (box tests 12.7 -> 9.4 per segment), book-1 and the 1M-sphere
    // field unchanged (profiles/r03_e). A wide-node visit is priced as half a primitive test since round
    // 5: with one primitive per leaf trip a quad test costs a trip of its own, and Cornell's tree at 0.5
    // (single-quad leaves: box tests 9.48 -> 10.59, quad tests 1.61 -> 1.22 per segment) is 8 % faster
    // than at 1.0; book-1 and the 1M field within 0.3 % (profiles/r05_s ... r05_u). RTG_COLLAPSE="greedy"
    // keeps round 2's greedy collapse, "sah:c_node:max_leaf" other constants (A/B)
    CollapseParams cp;
    cp.sah = true;
    cp.c_node = 0.5;
    if (const char* e = std::getenv("RTG_COLLAPSE")) {
      double cn = 0.5;
      int ml = 4;
      if (std::strncmp(e, "greedy", 6) == 0) {
        cp.sah = false;
      } else if (std::strncmp(e, "sah", 3) == 0) {
        if (std::sscanf(e, "sah:%lf:%d", &cn, &ml) >= 1 && cn > 0.0) cp.c_node = cn;
        cp.max_leaf = std::min(8, std::max(1, ml));
      }
    }
    collapse_bvh4(bvh, &bvh4, cp);
    phase("collapse");
    reorder_top_bfs(&bvh4, kTreeletBfsNodes);
    phase("bfs");
    out->num_nodes = static_cast<int64_t>(bvh4.nodes.size());
    out->depth = bvh4.depth;
    out->stack_need = bvh4.max_pushes;
    out->node_width = 4;
  }
  if (std::getenv("RTG_VERBOSE"))
    std::fprintf(stderr, "[rtg] bvh: %lld primitives, %zu binary nodes -> %lld nodes of width %d, depth %d, stack %d\n",
                 static_cast<long long>(d->num_prims), bvh.nodes.size(), static_cast<long long>(out->num_nodes),
                 out->node_width, out->depth, out->stack_need);

  // primitives, laid out in first-reference order for locality
  std::vector<int32_t> slot(d->num_prims, -1);
  int32_t nsph = 0, nquad = 0;
  out->refs.resize(bvh.refs.size());
  for (size_t r = 0; r < bvh.refs.size(); ++r) {
    const int64_t pid = bvh.refs[r];
    const rtg_primitive& p = d->prims[pid];
    if (slot[pid] < 0) {
      if (p.kind == RTG_PRIM_SPHERE) {
        slot[pid] = nsph++;
        const float rec[8] = {static_cast<float>(p.p0[0]),
                              static_cast<float>(p.p0[1]),
                              static_cast<float>(p.p0[2]),
                              static_cast<float>(p.radius),
                              static_cast<float>(p.p1[0] - p.p0[0]),
                              static_cast<float>(p.p1[1] - p.p0[1]),
                              static_cast<float>(p.p1[2] - p.p0[2]),
                              ibits_to_float(p.material)};
        out->spheres.insert(out->spheres.end(), rec, rec + 8);
      } else {
        slot[pid] = nquad++;
        // quad ctor (quad.hpp:12-27) in fp64, then rounded; the v row's 4th word holds the quad's tie
        // rank (its position in the reference's test order, read with the inside test's loads)
        const D3 Q = d3(p.p0), u = d3(p.p1), v = d3(p.p2);
        const D3 n = cross(u, v);
        const D3 normal = unit_vector(n);
        const double D = dot(normal, Q);
        const D3 w = n / dot(n, n);
        const float rec[20] = {static_cast<float>(Q.x),      static_cast<float>(Q.y),
                               static_cast<float>(Q.z),      static_cast<float>(D),
                               static_cast<float>(u.x),      static_cast<float>(u.y),
                               static_cast<float>(u.z),      ibits_to_float(p.material),
                               static_cast<float>(v.x),      static_cast<float>(v.y),
                               static_cast<float>(v.z),      ibits_to_float(static_cast<int32_t>(tie_rank(pid))),
                               static_cast<float>(w.x),      static_cast<float>(w.y),
                               static_cast<float>(w.z),      0.0f,
                               static_cast<float>(normal.x), static_cast<float>(normal.y),
                               static_cast<float>(normal.z), 0.0f};
        out->quads.insert(out->quads.end(), rec, rec + 20);
      }
    }
    out->refs[r] = (p.kind == RTG_PRIM_QUAD) ? (slot[pid] | kQuadRefBit) : slot[pid];
  }
  if (out->occluder_prim >= 0) {  // after every referenced sphere, so the refs stay the identity
    const rtg_primitive& p = d->prims[out->occluder_prim];
    slot[out->occluder_prim] = nsph;
    out->occluder = nsph++;
    const float rec[8] = {static_cast<float>(p.p0[0]),          static_cast<float>(p.p0[1]),
                          static_cast<float>(p.p0[2]),          static_cast<float>(p.radius),
                          static_cast<float>(p.p1[0] - p.p0[0]), static_cast<float>(p.p1[1] - p.p0[1]),
                          static_cast<float>(p.p1[2] - p.p0[2]), ibits_to_float(p.material)};
    out->spheres.insert(out->spheres.end(), rec, rec + 8);
  }

  // the exact-t tie rule's order: tie rank per sphere slot, then per quad slot
  out->tie_rank.assign(static_cast<size_t>(nsph) + nquad, -1);
  for (int64_t i = 0; i < d->num_prims; ++i)
    if (slot[i] >= 0)
      out->tie_rank[(d->prims[i].kind == RTG_PRIM_QUAD ? nsph : 0) + slot[i]] = static_cast<int32_t>(tie_rank(i));
  phase("prims");
  // culling boxes (the margin above) in place of the reference's, then rounded outward
  if (out->node_width == 4) refit_culling_boxes<BuildNode4, 4>(bvh4.nodes, bvh.refs, d, out->origin_bound);
  if (out->node_width == 2) refit_culling_boxes<BuildNode, 2>(bvh.nodes, bvh.refs, d, out->origin_bound);
  // leaf code = ~((first << 3) | (count - 1))
  if (out->node_width == 4 && !emit_wide(bvh4, out, err)) return false;
  // child-pair nodes: 64 B
  if (out->node_width == 2) out->nodes.resize(bvh.nodes.size() * 16);
  for (size_t k = 0; out->node_width == 2 && k < bvh.nodes.size(); ++k) {
    const BuildNode& n = bvh.nodes[k];
    float lo[2][3], hi[2][3];
    int32_t code[2];
    if (n.child[0] == kEmptyChild) {  // the kernel only guards the right slot
      *err = "BVH node with an empty left child";
      return false;
    }
    for (int s = 0; s < 2; ++s) {
      if (n.child[s] == kEmptyChild) {
        for (int a = 0; a < 3; ++a) {
          lo[s][a] = std::numeric_limits<float>::infinity();
          hi[s][a] = -std::numeric_limits<float>::infinity();
        }
        code[s] = kEmptyChild;
        continue;
      }
      for (int a = 0; a < 3; ++a) {
        lo[s][a] = round_down(n.lo[s][a]);
        hi[s][a] = round_up(n.hi[s][a]);
      }
      if (n.child[s] >= 0) {
        code[s] = n.child[s];
      } else {
        const int64_t first = -(static_cast<int64_t>(n.child[s]) + 1);
        const int32_t count = n.count[s];
        if (count < 1 || count > 8 || first >= (int64_t(1) << 28)) {
          *err = "BVH leaf not encodable";
          return false;
        }
        code[s] = ~static_cast<int32_t>((first << 3) | (count - 1));
      }
    }
    float* f = &out->nodes[k * 16];
    f[0] = lo[0][0];
    f[1] = lo[0][1];
    f[2] = lo[0][2];
    f[3] = hi[0][0];
    f[4] = hi[0][1];
    f[5] = hi[0][2];
    f[6] = lo[1][0];
    f[7] = lo[1][1];
    f[8] = lo[1][2];
    f[9] = hi[1][0];
    f[10] = hi[1][1];
    f[11] = hi[1][2];
    f[12] = ibits_to_float(code[0]);
    f[13] = ibits_to_float(code[1]);
    f[14] = 0.0f;
    f[15] = 0.0f;
  }

  phase("nodes");
  // materials {type, texture, fuzz, eta}, {albedo.xyz, uses_uv}. A lambertian or diffuse_light whose
  // texture is a solid_color carries the colour itself (texture -1, albedo = the colour: the value
  // solid_color::value returns, texture.hpp:34-44), and only the textures some material still
  // references (checkers and their children, images, noise) are kept, renumbered: book-1's 388
  // per-sphere solid textures (12.4 KB of LDS) disappear and its shading skips a dependent fetch.
  auto is_textured = [&](const rtg_material& mt) {
    return mt.type == RTG_MAT_LAMBERTIAN || mt.type == RTG_MAT_DIFFUSE_LIGHT;
  };
  std::vector<int32_t> tex_map(static_cast<size_t>(d->num_textures), -1);
  std::vector<int32_t> tex_order;
  std::function<void(int32_t)> keep = [&](int32_t t) {
    if (t < 0 || t >= d->num_textures || tex_map[t] >= 0) return;
    tex_map[t] = static_cast<int32_t>(tex_order.size());
    tex_order.push_back(t);
    if (d->textures[t].type == RTG_TEX_CHECKER) {
      keep(d->textures[t].even);
      keep(d->textures[t].odd);
    }
  };
  for (int32_t m = 0; m < d->num_materials; ++m)
    if (is_textured(d->materials[m]) && d->textures[d->materials[m].texture].type != RTG_TEX_SOLID)
      keep(d->materials[m].texture);
  for (int32_t m = 0; m < d->num_materials; ++m) {
    const rtg_material& mt = d->materials[m];
    const double fuzz = mt.fuzz < 1.0f ? mt.fuzz : 1.0f;  // metal ctor clamp (material.hpp:83)
    const bool uv = is_textured(mt) && texture_uses_uv(d, mt.texture, 0);
    const bool inline_solid = is_textured(mt) && d->textures[mt.texture].type == RTG_TEX_SOLID;
    const double* alb = inline_solid ? d->textures[mt.texture].color : mt.albedo;
    const float rec[8] = {ibits_to_float(mt.type),
                          ibits_to_float(inline_solid ? -1 : (is_textured(mt) ? tex_map[mt.texture] : -1)),
                          static_cast<float>(fuzz),
                          static_cast<float>(mt.refraction_index),
                          static_cast<float>(alb[0]),
                          static_cast<float>(alb[1]),
                          static_cast<float>(alb[2]),
                          ibits_to_float(uv ? 1 : 0)};
    out->materials.insert(out->materials.end(), rec, rec + 8);
  }
  // textures {type, even, odd, scale'}, {color.xyz, image|perlin}
  uint64_t texel_off = 0;
  for (int32_t im = 0; im < d->num_images; ++im) {
    const rtg_image& img = d->images[im];
    const bool ok = img.rgb != nullptr && img.width > 0 && img.height > 0;
    const int32_t hdr[4] = {ok ? img.width : 0, ok ? img.height : 0,
                            static_cast<int32_t>(texel_off & 0xffffffffu),
                            static_cast<int32_t>(texel_off >> 32)};
    out->image_hdr.insert(out->image_hdr.end(), hdr, hdr + 4);
    if (ok) {
      const uint64_t bytes = static_cast<uint64_t>(img.width) * img.height * 3;
      out->texels.insert(out->texels.end(), img.rgb, img.rgb + bytes);
      texel_off += bytes;
      while (texel_off % 16) {
        out->texels.push_back(0);
        ++texel_off;
      }
    }
  }
  for (const int32_t t : tex_order) {
    const rtg_texture& tx = d->textures[t];
    float scale = 0.0f;
    int32_t aux = -1;
    if (tx.type == RTG_TEX_CHECKER) scale = static_cast<float>(1.0f / tx.scale);  // texture.hpp:50-51
    if (tx.type == RTG_TEX_NOISE) {
      scale = static_cast<float>(tx.scale);
      aux = tx.perlin;
    }
    if (tx.type == RTG_TEX_IMAGE) aux = (tx.image >= 0 && tx.image < d->num_images) ? tx.image : -1;
    const bool checker = tx.type == RTG_TEX_CHECKER;
    const float rec[8] = {ibits_to_float(tx.type),
                          ibits_to_float(checker ? tex_map[tx.even] : tx.even),
                          ibits_to_float(checker ? tex_map[tx.odd] : tx.odd),
                          scale,
                          static_cast<float>(tx.color[0]),
                          static_cast<float>(tx.color[1]),
                          static_cast<float>(tx.color[2]),
                          ibits_to_float(aux)};
    out->textures.insert(out->textures.end(), rec, rec + 8);
  }
  for (int32_t pt = 0; pt < d->num_perlins; ++pt) {
    const rtg_perlin& pl = d->perlins[pt];
    for (int i = 0; i < 256; ++i) {
      const float v[4] = {static_cast<float>(pl.randvec[i][0]), static_cast<float>(pl.randvec[i][1]),
                          static_cast<float>(pl.randvec[i][2]), 0.0f};
      out->perlin_vec.insert(out->perlin_vec.end(), v, v + 4);
    }
    for (int i = 0; i < 256; ++i) {
      if (pl.perm_x[i] < 0 || pl.perm_x[i] > 255 || pl.perm_y[i] < 0 || pl.perm_y[i] > 255 ||
          pl.perm_z[i] < 0 || pl.perm_z[i] > 255) {
        *err = "perlin permutation entry out of [0, 255]";
        return false;
      }
    }
    // the packed words of rtg_internal.hpp (kPerlinPermWords): a noise octave reads both corner entries
    // of every axis with three LDS instructions, and two XORs per word give two corners' gradient offsets
    auto off = [](int32_t v) { return static_cast<uint32_t>(v) << 4; };
    for (int i = 0; i < 256; ++i) out->perlin_perm.push_back(off(pl.perm_x[i]) | off(pl.perm_x[(i + 1) & 255]) << 16);
    for (const int32_t* perm : {pl.perm_y, pl.perm_z})
      for (int i = 0; i < 256; ++i) {
        out->perlin_perm.push_back(off(perm[i]) * 0x10001u);
        out->perlin_perm.push_back(off(perm[(i + 1) & 255]) * 0x10001u);
      }
  }
  phase("materials");
  return true;
}

// Every device / pinned-host allocation of the library goes through these, so rtg_allocation_count can
// show that steady-state frames allocate nothing.
std::atomic<uint64_t> g_allocs{0}, g_alloc_bytes{0};
hipError_t dev_alloc(void** p, size_t bytes) {
  const hipError_t e = hipMalloc(p, bytes);
  if (e == hipSuccess) {
    g_allocs.fetch_add(1, std::memory_order_relaxed);
    g_alloc_bytes.fetch_add(bytes, std::memory_order_relaxed);
  }
  return e;
}
hipError_t dev_alloc_async(void** p, size_t bytes, hipStream_t st) {
  const hipError_t e = hipMallocAsync(p, bytes, st);
  if (e == hipSuccess) {
    g_allocs.fetch_add(1, std::memory_order_relaxed);
    g_alloc_bytes.fetch_add(bytes, std::memory_order_relaxed);
  }
  return e;
}
hipError_t host_alloc(void** p, size_t bytes) {
  const hipError_t e = hipHostMalloc(p, bytes, hipHostMallocDefault);
  if (e == hipSuccess) {
    g_allocs.fetch_add(1, std::memory_order_relaxed);
    g_alloc_bytes.fetch_add(bytes, std::memory_order_relaxed);
  }
  return e;
}

}  // namespace rtg

// Grow-only device scratch of a scene's renders (stack spill, wave trace, tile ring or chunk partial sums).
// Renders of one scene never overlap — rtg_render refuses while one is pending, collect_stats waits for
// its stream, a failed render waits for it (SyncOnError) — so a buffer is idle whenever a render starts,
// and frames allocate nothing once the buffers reached their sizes (config 2: 0.8 GB of partials, config
// 5: 6.3 GB, kept with the scene; 288 GB of HBM).
struct ScratchBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct rtg_scene {
  int device = 0;
  int num_cus = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t aux_stream = nullptr;  // second persistent launch (dual workgroup shapes)
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  void* dmem = nullptr;  // one allocation for all scene arrays
  size_t dbytes = 0;
  unsigned long long* counters = nullptr;  // device [8]
  unsigned long long* host_counters = nullptr;  // pinned [8]
  DevScene dev{};
  rtg_scene_info info{};
  int stack_need = 0;  // structural maximum of traversal stack entries of the BVH
  Knobs knobs;         // environment knobs, read once when the scene was created
  // host-output renders land in this pinned staging buffer first (DMA to pinned memory completes
  // with the stream; an async copy straight into pageable user memory was seen to return from
  // the stream sync before all of its bytes had arrived), then a host memcpy to the caller
  void* host_stage = nullptr;
  size_t host_stage_bytes = 0;
  float* dev_out = nullptr;  // device frame of host-output renders (kept between renders)
  size_t dev_out_bytes = 0;
  ScratchBuf scr_spill, scr_trace, scr_partial;  // render scratch (ScratchBuf)
  float* pending_host_out = nullptr;
  size_t pending_host_bytes = 0;
  // hot treelet (schedule 5): the node array is renumbered so the nodes a probe render of this
  // camera visited most come first, i.e. into the LDS prefix (tune_treelet); key of that camera
  uint64_t treelet_key = 0;
  uint32_t* probe_visits = nullptr;  // set only while the probe render runs
  double treelet_tune_ms = 0.0;
  std::vector<uint64_t> treelet_cum;  // probe visits of the first k nodes after the renumbering, k = 0..n
  // host copy of the device node array in its current order (scenes on the treelet schedule): the hot
  // treelet renumbers this copy and uploads it, so a tuning downloads only the visit counts
  std::vector<int32_t> host_nodes;
  // M of the culling margin the device node boxes are padded for (HostScene::origin_bound); raised,
  // with the boxes, when a camera lies farther out (ensure_origin_bound)
  double origin_bound = 0.0;
  // cost-ordered tile hand-out (tune_tile_order): the tile handed out at each position for the camera and
  // shard of order_key (order_tiles entries, device; grow-only), the probe's most expensive tile first
  uint64_t order_key = 0;
  int32_t* order_dev = nullptr;
  int64_t order_tiles = 0, order_cap = 0;
  double order_tune_ms = 0.0;
  uint32_t* probe_tile_cost = nullptr;  // set only while the tile-cost probe runs
  // deferred (async) render state
  bool pending = false;
  hipStream_t pending_stream = nullptr;
  uint64_t pending_samples = 0;
  bool pending_tile_order = false;
};

extern "C" {

uint32_t rtg_abi_version(void) { return RTG_ABI_VERSION; }

const char* rtg_last_error(void) { return g_last_error.c_str(); }

rtg_status rtg_device_count(int32_t* count) {
  if (!count) return fail(RTG_E_INVALID, "count is NULL");
  int n = 0;
  const hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return fail(RTG_E_NODEVICE, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  }
  *count = n;
  return RTG_OK;
}

rtg_status rtg_camera_resolve(const rtg_camera_desc* cam, rtg_camera_params* out) {
  if (!cam || !out) return fail(RTG_E_INVALID, "null argument");
  if (cam->image_width <= 0 || cam->samples_per_pixel <= 0)
    return fail(RTG_E_INVALID, "image_width and samples_per_pixel must be positive");
  resolve_camera(cam, out);
  return RTG_OK;
}

rtg_status rtg_bvh_build_host(const rtg_scene_desc* desc, rtg_bvh_node_host* nodes_out,
                              int64_t max_nodes, int64_t* refs_out, int64_t max_refs,
                              int64_t* num_nodes, int64_t* num_refs, int32_t* depth) {
  if (!desc) return fail(RTG_E_INVALID, "desc is NULL");
  if (desc->num_prims < 0 || (desc->num_prims > 0 && !desc->prims))
    return fail(RTG_E_INVALID, "malformed primitive array");
  Bvh bvh;
  std::string err;
  if (!build_bvh(desc, &bvh, &err)) return fail(RTG_E_INVALID, err);
  if (num_nodes) *num_nodes = static_cast<int64_t>(bvh.nodes.size());
  if (num_refs) *num_refs = static_cast<int64_t>(bvh.refs.size());
  if (depth) *depth = bvh.depth;
  if (nodes_out) {
    const int64_t n = std::min<int64_t>(max_nodes, bvh.nodes.size());
    for (int64_t k = 0; k < n; ++k) {
      const BuildNode& b = bvh.nodes[k];
      rtg_bvh_node_host& h = nodes_out[k];
      std::memcpy(h.lo, b.lo, sizeof(h.lo));
      std::memcpy(h.hi, b.hi, sizeof(h.hi));
      h.child[0] = b.child[0];
      h.child[1] = b.child[1];
      h.count[0] = b.count[0];
      h.count[1] = b.count[1];
    }
  }
  if (refs_out) {
    const int64_t n = std::min<int64_t>(max_refs, bvh.refs.size());
    for (int64_t k = 0; k < n; ++k) refs_out[k] = bvh.refs[k];
  }
  return RTG_OK;
}

rtg_status rtg_allocation_count(uint64_t* count, uint64_t* bytes) {
  if (count) *count = g_allocs.load(std::memory_order_relaxed);
  if (bytes) *bytes = g_alloc_bytes.load(std::memory_order_relaxed);
  return RTG_OK;
}

rtg_status rtg_bvh_node_order(const double* boxes, int64_t n, int64_t* order) {
  if (n < 0 || (n > 0 && (!boxes || !order))) return fail(RTG_E_INVALID, "null array or negative count");
  try {
    bvh_node_order(boxes, n, order);
  } catch (const std::bad_alloc&) {
    return fail(RTG_E_NOMEM, "rtg_bvh_node_order: out of host memory");
  }
  return RTG_OK;
}

rtg_status rtg_scene_create(const rtg_scene_desc* desc_in, int32_t device, rtg_scene** out) {
  if (!desc_in || !out) return fail(RTG_E_INVALID, "null argument");
  *out = nullptr;
  if (desc_in->abi_version != RTG_ABI_VERSION && desc_in->abi_version != 6)
    return fail(RTG_E_INVALID, "abi_version mismatch (expected " +
                                   std::to_string(RTG_ABI_VERSION) + " or 6)");
  // an ABI-6 descriptor ends before tie_rank: read only its own bytes
  rtg_scene_desc desc_v{};
  std::memcpy(&desc_v, desc_in,
              desc_in->abi_version == 6 ? offsetof(rtg_scene_desc, tie_rank) : sizeof(rtg_scene_desc));
  const rtg_scene_desc* desc = &desc_v;
  // validate + compile first (host only), so malformed scenes report RTG_E_INVALID anywhere
  const auto t0 = std::chrono::steady_clock::now();
  HostScene hs;
  std::string err;
  if (!compile_scene(desc, &hs, &err)) return fail(RTG_E_INVALID, err);
  if (hs.stack_need > kMaxStackNeed)
    return fail(RTG_E_UNSUPPORTED, "BVH needs " + std::to_string(hs.stack_need) + " stack entries (limit " +
                                       std::to_string(kMaxStackNeed) + ")");
  const auto t1 = std::chrono::steady_clock::now();

  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(RTG_E_NODEVICE, "no HIP device available (librtgpu has no CPU fallback)");
  if (device < 0 || device >= ndev) return fail(RTG_E_INVALID, "device index out of range");
  RTG_HIP(hipSetDevice(device), "hipSetDevice");
  hipDeviceProp_t prop;
  RTG_HIP(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(RTG_E_NODEVICE, std::string("device is ") + prop.gcnArchName +
                                    ", this build targets gfx950 only");

  // one device allocation, 256-B aligned sub-buffers
  struct Part {
    const void* src;
    size_t bytes;
    size_t off;
  };
  Part parts[9] = {
      {hs.gpu_bvh ? nullptr : hs.nodes.data(),
       hs.gpu_bvh ? static_cast<size_t>(hs.node_capacity) * 112 : hs.nodes.size() * 4, 0},       {hs.refs.data(), hs.refs.size() * 4, 0},
      {hs.spheres.data(), hs.spheres.size() * 4, 0},   {hs.quads.data(), hs.quads.size() * 4, 0},
      {hs.materials.data(), hs.materials.size() * 4, 0}, {hs.textures.data(), hs.textures.size() * 4, 0},
      {hs.image_hdr.data(), hs.image_hdr.size() * 4, 0}, {hs.texels.data(), hs.texels.size(), 0},
      {hs.perlin_vec.data(), hs.perlin_vec.size() * 4, 0}};
  size_t total = 0;
  for (Part& p : parts) {
    p.off = total;
    total += (p.bytes + 255) & ~size_t(255);
  }
  const size_t perm_off = total;
  total += (hs.perlin_perm.size() * 4 + 255) & ~size_t(255);
  const size_t rank_off = total;
  total += (hs.tie_rank.size() * 4 + 255) & ~size_t(255);
  total = std::max<size_t>(total, 256);

  rtg_scene* s = new (std::nothrow) rtg_scene();
  if (!s) return fail(RTG_E_NOMEM, "host allocation failed");
  s->device = device;
  s->knobs = read_knobs();
  auto cleanup = [&](rtg_status st) {
    rtg_scene_destroy(s);
    return st;
  };
  hipError_t e = dev_alloc(&s->dmem, total);
  if (e != hipSuccess) return cleanup(hip_fail(e, "hipMalloc(scene)"));
  s->dbytes = total;
  if ((e = hipStreamCreateWithFlags(&s->own_stream, hipStreamNonBlocking)) != hipSuccess)
    return cleanup(hip_fail(e, "hipStreamCreate"));
  if ((e = hipEventCreate(&s->ev0)) != hipSuccess || (e = hipEventCreate(&s->ev1)) != hipSuccess)
    return cleanup(hip_fail(e, "hipEventCreate"));
  if ((e = dev_alloc(reinterpret_cast<void**>(&s->counters), kNumCounters * sizeof(unsigned long long))) != hipSuccess)
    return cleanup(hip_fail(e, "hipMalloc(counters)"));
  if ((e = host_alloc(reinterpret_cast<void**>(&s->host_counters), kNumCounters * sizeof(unsigned long long))) != hipSuccess)
    return cleanup(hip_fail(e, "hipHostMalloc(counters)"));
  char* base = static_cast<char*>(s->dmem);
  {
    // every array into one pinned staging image of the allocation (host copies on up to 16 threads),
    // then one DMA: pageable sources went through the runtime's own small staging buffers (config 5:
    // ~100 ms for 90 MB); without pinned memory the arrays are copied from where they are
    struct Src {
      const void* p;
      size_t bytes, off;
    };
    std::vector<Src> srcs;
    for (const Part& p : parts)
      if (p.bytes != 0 && p.src) srcs.push_back({p.src, p.bytes, p.off});
    if (!hs.perlin_perm.empty()) srcs.push_back({hs.perlin_perm.data(), hs.perlin_perm.size() * 4, perm_off});
    if (!hs.tie_rank.empty()) srcs.push_back({hs.tie_rank.data(), hs.tie_rank.size() * 4, rank_off});
    size_t end = 0;
    for (const Src& x : srcs) end = std::max(end, x.off + x.bytes);
    void* stage = nullptr;
    if (end > 0 && host_alloc(&stage, end) == hipSuccess) {
      char* st = static_cast<char*>(stage);
      host_par_for(static_cast<int64_t>(srcs.size()), [&](int64_t b, int64_t e2, int) {
        for (int64_t k = b; k < e2; ++k) std::memcpy(st + srcs[k].off, srcs[k].p, srcs[k].bytes);
      });
      e = hipMemcpyAsync(base, stage, end, hipMemcpyHostToDevice, s->own_stream);
      if (e == hipSuccess) e = hipStreamSynchronize(s->own_stream);
      (void)hipHostFree(stage);
      if (e != hipSuccess) return cleanup(hip_fail(e, "hipMemcpy(scene)"));
    } else {
      for (const Src& x : srcs)
        if ((e = hipMemcpyAsync(base + x.off, x.p, x.bytes, hipMemcpyHostToDevice, s->own_stream)) != hipSuccess)
          return cleanup(hip_fail(e, "hipMemcpy(scene)"));
      if ((e = hipStreamSynchronize(s->own_stream)) != hipSuccess)
        return cleanup(hip_fail(e, "hipStreamSynchronize(upload)"));
    }
  }
  const auto t2 = std::chrono::steady_clock::now();
  double gpu_build_ms = 0.0;
  const int64_t nrefs = static_cast<int64_t>(hs.refs.size());
  if (hs.gpu_bvh && nrefs > 0) {  // RTG_BVH_GPU: build the nodes and leaf-ordered refs here
    int32_t* refs_dev = reinterpret_cast<int32_t*>(base + parts[1].off);
    int32_t* sorted = nullptr;
    if ((e = dev_alloc_async(reinterpret_cast<void**>(&sorted), nrefs * 4, s->own_stream)) != hipSuccess)
      return cleanup(hip_fail(e, "hipMalloc(bvh refs)"));
    GpuBvhResult r{};
    e = gpu_build_bvh4(reinterpret_cast<const float4*>(base + parts[2].off),
                       reinterpret_cast<const float4*>(base + parts[3].off), refs_dev, nrefs,
                       round_up(hs.origin_bound), reinterpret_cast<float*>(base + parts[0].off),
                       hs.node_capacity, sorted, &r, s->own_stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(refs_dev, sorted, nrefs * 4, hipMemcpyDeviceToDevice, s->own_stream);
    const hipError_t ef = hipFreeAsync(sorted, s->own_stream);
    if (e == hipSuccess) e = ef;
    if (e == hipSuccess) e = hipStreamSynchronize(s->own_stream);
    if (e != hipSuccess) return cleanup(hip_fail(e, "device BVH build"));
    hs.num_nodes = r.num_nodes;
    hs.depth = r.depth;
    hs.stack_need = r.stack_need;
    // the device tree's bound is only known now; the 4-wide LDS node step has no overflow check
    // outside the COUNT diagnostics, so this host-side bound is the guard (as for host builds)
    if (hs.stack_need > kMaxStackNeed)
      return cleanup(fail(RTG_E_UNSUPPORTED, "device BVH needs " + std::to_string(hs.stack_need) +
                                                 " stack entries (limit " + std::to_string(kMaxStackNeed) + ")"));
    gpu_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t2).count();
  }

  s->dev.nodes = reinterpret_cast<const float4*>(base + parts[0].off);
  s->dev.refs = reinterpret_cast<const int32_t*>(base + parts[1].off);
  s->dev.spheres = reinterpret_cast<const float4*>(base + parts[2].off);
  s->dev.quads = reinterpret_cast<const float4*>(base + parts[3].off);
  s->dev.materials = reinterpret_cast<const float4*>(base + parts[4].off);
  s->dev.textures = reinterpret_cast<const float4*>(base + parts[5].off);
  s->dev.images = reinterpret_cast<const int4*>(base + parts[6].off);
  s->dev.texels = reinterpret_cast<const uint8_t*>(base + parts[7].off);
  s->dev.perlin_vec = reinterpret_cast<const float4*>(base + parts[8].off);
  s->dev.perlin_perm = reinterpret_cast<const uint32_t*>(base + perm_off);
  s->dev.tie_rank = reinterpret_cast<const int32_t*>(base + rank_off);
  s->dev.num_nodes = hs.num_nodes;
  s->dev.root_code = 0;
  s->dev.occluder = hs.occluder;
  s->dev.sphere_f4 = 2;
  s->dev.treelet_bytes = 0;  // set per render by the treelet schedule
  s->dev.treelet_lds = 0;
  s->dev.node_limit = static_cast<int32_t>(
      std::min<int64_t>(hs.num_nodes * node_bytes(4), INT32_MAX));
  s->dev.num_refs = static_cast<int64_t>(hs.refs.size());
  s->dev.num_spheres = static_cast<int64_t>(hs.spheres.size() / 8);
  s->dev.num_quads = static_cast<int64_t>(hs.quads.size() / 20);
  s->dev.node_width = hs.node_width;
  s->dev.num_materials = static_cast<int32_t>(hs.materials.size() / 8);
  s->dev.num_textures = static_cast<int32_t>(hs.textures.size() / 8);
  s->dev.ref_mode = 0;
  {
    bool ident_s = !hs.refs.empty(), ident_q = !hs.refs.empty();
    for (size_t r = 0; r < hs.refs.size() && (ident_s || ident_q); ++r) {
      ident_s = ident_s && hs.refs[r] == static_cast<int32_t>(r);
      ident_q = ident_q && hs.refs[r] == (static_cast<int32_t>(r) | kQuadRefBit);
    }
    s->dev.ref_mode = ident_s ? 1 : (ident_q ? 2 : 0);
    if (hs.gpu_bvh) s->dev.ref_mode = 0;  // the device build permuted the refs
  }
  s->dev.tex_full = 0;
  for (int32_t t = 0; t < desc->num_textures; ++t)
    if (desc->textures[t].type == RTG_TEX_IMAGE || desc->textures[t].type == RTG_TEX_NOISE) s->dev.tex_full = 1;
  s->dev.diffuse_only = 1;
  for (int32_t m = 0; m < desc->num_materials; ++m)
    if (desc->materials[m].type == RTG_MAT_METAL || desc->materials[m].type == RTG_MAT_DIELECTRIC)
      s->dev.diffuse_only = 0;
  s->dev.num_perlins = static_cast<int32_t>(hs.perlin_perm.size() / kPerlinPermWords);
  s->num_cus = prop.multiProcessorCount;
  // trees too large for any LDS schedule render on the treelet schedule: keep their node array on the
  // host for the hot-treelet renumbering (device-built trees are downloaded once, on the first tuning)
  if (!hs.gpu_bvh && hs.node_width >= 4 && hs.num_nodes * node_bytes(hs.node_width) > kLdsPerCu)
    s->host_nodes.assign(reinterpret_cast<const int32_t*>(hs.nodes.data()),
                         reinterpret_cast<const int32_t*>(hs.nodes.data()) + hs.nodes.size());

  s->origin_bound = hs.origin_bound;
  s->info.device = device;
  s->info.bvh_mode = desc->bvh_mode;
  s->info.num_prims = hs.num_prims;
  s->info.num_nodes = hs.num_nodes;
  s->info.bvh_depth = hs.depth;
  s->info.stack_depth = hs.stack_need;
  s->stack_need = hs.stack_need;
  s->info.device_bytes = static_cast<int64_t>(total);
  s->info.build_ms = std::chrono::duration<double, std::milli>(t1 - t0).count() + gpu_build_ms;
  s->info.upload_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
  s->info.bvh_ms = hs.bvh_ms + gpu_build_ms;
  s->info.collapse_ms = hs.collapse_ms;
  s->info.flatten_ms = std::chrono::duration<double, std::milli>(t1 - t0).count() - hs.bvh_ms - hs.collapse_ms;
  *out = s;
  return RTG_OK;
}

rtg_status rtg_scene_get_info(const rtg_scene* scene, rtg_scene_info* out) {
  if (!scene || !out) return fail(RTG_E_INVALID, "null argument");
  *out = scene->info;
  return RTG_OK;
}

void rtg_scene_destroy(rtg_scene* s) {
  if (!s) return;
  // teardown: errors cannot be reported from a void destructor, they are deliberately dropped
  (void)hipSetDevice(s->device);
  if (s->pending && s->pending_stream) (void)hipStreamSynchronize(s->pending_stream);
  if (s->dmem) (void)hipFree(s->dmem);
  if (s->counters) (void)hipFree(s->counters);
  if (s->host_counters) (void)hipHostFree(s->host_counters);
  if (s->host_stage) (void)hipHostFree(s->host_stage);
  if (s->dev_out) (void)hipFree(s->dev_out);
  if (s->order_dev) (void)hipFree(s->order_dev);
  for (ScratchBuf* b : {&s->scr_spill, &s->scr_trace, &s->scr_partial})
    if (b->p) (void)hipFree(b->p);
  if (s->ev0) (void)hipEventDestroy(s->ev0);
  if (s->ev1) (void)hipEventDestroy(s->ev1);
  if (s->own_stream) (void)hipStreamDestroy(s->own_stream);
  if (s->aux_stream) (void)hipStreamDestroy(s->aux_stream);
  if (s->ev_fork) (void)hipEventDestroy(s->ev_fork);
  if (s->ev_join) (void)hipEventDestroy(s->ev_join);
  delete s;
}

static rtg_status collect_stats(rtg_scene* s, rtg_render_stats* stats) {
  RTG_HIP(hipEventSynchronize(s->ev1), "render kernel");
  float ms = 0.0f;
  RTG_HIP(hipEventElapsedTime(&ms, s->ev0, s->ev1), "hipEventElapsedTime");
  RTG_HIP(hipStreamSynchronize(s->pending_stream), "render stream");
  if (s->pending_host_out) {
    std::memcpy(s->pending_host_out, s->host_stage, s->pending_host_bytes);
    s->pending_host_out = nullptr;
  }
  const unsigned long long* c = s->host_counters;
  s->pending = false;
  if (stats) {
    stats->segments = c[0];
    stats->box_tests = c[1];
    stats->prim_tests = c[2];
    stats->hits = c[3];
    stats->samples = s->pending_samples;
    stats->kernel_ms = ms;
    for (int k = 0; k < 16; ++k) stats->diag[k] = c[8 + k];
    stats->stack_spills = c[26];
    stats->tile_order = s->pending_tile_order ? 1u : 0u;
    stats->tile_order_tune_us = static_cast<uint32_t>(std::min(s->order_tune_ms * 1e3, 4e9));
  }
  // stats stay filled for diagnosis; the frame is not valid in either case
  if (c[4] != 0)
    return fail(RTG_E_UNSUPPORTED, "BVH traversal stack overflow in " + std::to_string(c[4]) + " waves");
  if (c[5] != 0) return fail(RTG_E_INVALID, "corrupt BVH child code met during traversal");
  if (c[24] != 0)
    return fail(RTG_E_HIP, "tile-ring slot waits timed out (frame incomplete) in " + std::to_string(c[24]) + " waves");
  if (c[7] != 0)
    return fail(RTG_E_UNSUPPORTED, "the LDS layout (16-bit stack codes, or perlin rows below 64 KiB) does not "
                                   "hold in " + std::to_string(c[7]) + " workgroups (nothing rendered)");
  return RTG_OK;
}

}  // extern "C"

namespace {

// Everything one render decides before it launches (rtg_render executes it, rtg_render_plan
// reports it): the schedule, the kernels, the LDS layout, the job parameters and the scratch.
struct Plan {
  rtg_camera_params cp{};
  int W = 0, H = 0, rows = 0;
  bool dev_out = false, async = false, progressive = false, count = false;
  DevCamera dc{};
  DevJob dj{};
  DevJob j4{};  // the dual launch's job (lds4 > 0)
  DevScene dscene{};
  int variant = 0;
  int lds_bytes = -1, lds4 = -1, lds_wgs = 1;
  int stack_depth = 0, grid_blocks = 1, grid_waves = 0;
  bool default_sched = false, chunked = false, skip_kernel = false;
  int ring_slots = 0;  // chunked: tile slots of the partial-sum ring (0: full-frame partials + combine_kernel)
  size_t ring_bytes = 0;
  int sum_chunks = 1;
  float out_scale = 1.0f;
  size_t out_bytes = 0;
  KernelChoice kmain, kaux;
};

uint64_t treelet_key(const rtg_camera_desc* c, const rtg_render_desc* j);

// The camera and shard tiles a tile order was tuned for: the treelet key (camera, width, first row, row
// stride) and the plan's tile layout (rows, tile width, tiles), so a row_count of 0 and the shard's row
// count name the same order.
uint64_t order_key(const rtg_camera_desc* c, const rtg_render_desc* j, const DevJob& dj) {
  uint64_t h = treelet_key(c, j);
  for (const int64_t v : {int64_t(dj.row_count), int64_t(dj.tile_lw), int64_t(dj.tiles_x), int64_t(dj.num_tiles)})
    h = (h ^ static_cast<uint64_t>(v)) * 1099511628211ull;
  return h | 1;  // never 0 (0: not tuned)
}

rtg_status plan_render(const rtg_scene* s, const rtg_camera_desc* cam, const rtg_render_desc* job, Plan* P) {
  if (!s || !cam || !job) return fail(RTG_E_INVALID, "null argument");
  const Knobs& K = s->knobs;
  P->progressive = job->partial != nullptr;
  if (cam->image_width <= 0 || cam->samples_per_pixel <= 0)
    return fail(RTG_E_INVALID, "image_width and samples_per_pixel must be positive");
  if (job->row_stride <= 0 || job->row_begin < 0) return fail(RTG_E_INVALID, "bad row range");
  P->dev_out = (job->flags & RTG_RENDER_OUT_DEVICE) != 0;
  P->async = (job->flags & RTG_RENDER_ASYNC) != 0;
  P->count = (job->flags & RTG_RENDER_COUNT) != 0;
  if (P->async && !P->dev_out) return fail(RTG_E_INVALID, "RTG_RENDER_ASYNC requires RTG_RENDER_OUT_DEVICE");

  resolve_camera(cam, &P->cp);
  const int W = P->W = P->cp.image_width, H = P->H = P->cp.image_height;
  if (job->row_begin >= H) return fail(RTG_E_INVALID, "row_begin beyond image height");
  const int reachable = (H - 1 - job->row_begin) / job->row_stride + 1;
  const int rows = P->rows = job->row_count <= 0 ? reachable : job->row_count;
  if (rows > reachable) return fail(RTG_E_INVALID, "row_count reaches past the image");
  if (static_cast<int64_t>(W) * H >= (int64_t(1) << 32))
    return fail(RTG_E_INVALID, "image larger than 2^32 pixels");
  if (W > 65535 || rows > 65535)  // the kernels pack a lane's pixel as 16-bit column / row
    return fail(RTG_E_INVALID, "image width or shard rows above 65535");
  P->out_bytes = static_cast<size_t>(rows) * W * 3 * sizeof(float);

  DevCamera& dc = P->dc;
  const rtg_camera_params& cp = P->cp;
  for (int k = 0; k < 3; ++k) {
    dc.center[k] = static_cast<float>(cp.center[k]);
    dc.pixel00[k] = static_cast<float>(cp.pixel00_loc[k]);
    dc.du[k] = static_cast<float>(cp.pixel_delta_u[k]);
    dc.dv[k] = static_cast<float>(cp.pixel_delta_v[k]);
    dc.defu[k] = static_cast<float>(cp.defocus_disk_u[k]);
    dc.defv[k] = static_cast<float>(cp.defocus_disk_v[k]);
    dc.background[k] = static_cast<float>(cam->background[k]);
  }
  dc.scale = static_cast<float>(cp.pixel_samples_scale);
  dc.width = W;
  dc.height = H;
  dc.spp = cam->samples_per_pixel;
  dc.max_depth = cam->max_depth;
  dc.defocus = cam->defocus_angle <= 0.0f ? 0 : 1;  // camera.hpp:155

  DevJob& dj = P->dj;
  dj = DevJob{};
  dj.seed_mix = mix64(job->seed);
  dj.row_begin = job->row_begin;
  dj.row_stride = job->row_stride;
  dj.row_count = rows;
  const int batch = (job->flags >> 16) & 0xff;
  // scenes with image / noise textures shade at a higher cost per lane: fuller shading batches
  // (earth_perlin: 56 -2.2 % against 48; book-1 and Cornell keep 48, profiles/r02_ab)
  dj.shade_batch = batch > 64 ? 64 : batch;  // 0: the schedule's default, set below
  const int leaf_batch = (job->flags >> 24) & 0x7f;
  const int default_leaf_batch = s->dev.num_nodes <= kSmallBvhNodes ? kSmallBvhLeafBatch : kDefaultLeafBatch;
  dj.leaf_batch = leaf_batch == 0 ? default_leaf_batch : (leaf_batch > 64 ? 64 : leaf_batch);
  // tile shape: 8x8 pixels of a contiguous image; wider and flatter tiles for row-interleaved shards,
  // whose consecutive shard rows lie row_stride image rows apart (keeps a wave's rays coherent)
  dj.tile_lw = K.tile_lw >= 0 ? K.tile_lw : (job->row_stride <= 1 ? 3 : 4);
  {
    const int tw = 1 << dj.tile_lw, th = 64 / tw;
    dj.tiles_x = (W + tw - 1) / tw;
    dj.num_tiles = dj.tiles_x * ((rows + th - 1) / th);
  }
  // the kernels pack a lane's sample index in 26 bits (render_stream's `su`)
  if (cam->samples_per_pixel >= (1 << 26)) return fail(RTG_E_UNSUPPORTED, "samples_per_pixel must be below 2^26");
  dj.chunk_samples = rtg_chunk_samples(cam->samples_per_pixel);
  // RTG_CHUNK_SAMPLES overrides K for schedule experiments (the frame then differs from the spec)
  if (K.chunk_samples > 0) dj.chunk_samples = K.chunk_samples;
  const int total_chunks =
      cam->samples_per_pixel > 0 ? (cam->samples_per_pixel + dj.chunk_samples - 1) / dj.chunk_samples : 1;
  dj.chunks = total_chunks;
  dj.chunk_begin = 0;
  dj.partial = nullptr;
  P->sum_chunks = total_chunks;  // chunks the output mean covers
  P->out_scale = dc.scale;
  if (P->progressive) {
    if (job->chunk_begin < 0 || job->chunk_begin >= total_chunks)
      return fail(RTG_E_INVALID, "chunk_begin outside [0, rtg_num_chunks(spp))");
    dj.chunk_begin = job->chunk_begin;
    dj.chunks = job->chunk_count <= 0 ? total_chunks - job->chunk_begin
                                      : std::min(job->chunk_count, total_chunks - job->chunk_begin);
    dj.partial = job->partial;
    P->sum_chunks = dj.chunk_begin + dj.chunks;
    const int samples_done = std::min(cam->samples_per_pixel, P->sum_chunks * dj.chunk_samples);
    // the final mean uses pixel_samples_scale itself (H7), so a finished progressive render is
    // bit-identical to a one-shot one
    P->out_scale = P->sum_chunks == total_chunks ? dc.scale : 1.0f / static_cast<float>(samples_done);
  }

  // one-shot chunked frames of the default schedules sum each tile's chunks through the tile ring
  // (RING kernels; the counting kernels keep the full-frame partials, same frame)
  // By default only where the full-frame partial buffers would be very large (kRingAutoBytes): the ring
  // costs the render loop time (config 5 +2.0 %, config 2 +7.5 %, config 4 +17 %: DESIGN.md §9), the
  // full-frame buffers cost memory. RTG_TILE_SLOTS=0 / >0 forces it off / on.
  const int64_t full_partial_bytes = int64_t(rows) * W * 12 * dj.chunks;
  // ... and at most half of the device memory free to this scene (the partials it already holds count as
  // free: they are reused), so a smaller or busier device takes the ring instead of failing
  int64_t ring_auto = kRingAutoBytes;
  if (K.tile_slots < 0 && full_partial_bytes > (int64_t(1) << 30)) {
    size_t free_b = 0, total_b = 0;
    if (hipSetDevice(s->device) == hipSuccess && hipMemGetInfo(&free_b, &total_b) == hipSuccess)
      ring_auto = std::min<int64_t>(ring_auto, static_cast<int64_t>((free_b + s->scr_partial.bytes) / 2));
  }
  const bool ring_on = K.tile_slots > 0 || (K.tile_slots < 0 && full_partial_bytes > ring_auto);
  // the ring kernels index the frame with 32-bit byte offsets (ring_combine's buffer descriptor: the
  // shard's frame below 2 GiB) and pack a tile into 25 bits of the per-wave batch table (tile << 7):
  // larger shards keep the full-frame partials, whose indexing is 64-bit
  const bool ring_fits = int64_t(rows) * W * 12 < (int64_t(1) << 31) && dj.num_tiles < (1 << 25);
  const bool want_ring = !P->progressive && dj.chunks > 1 && dj.chunks <= (1 << 20) && dc.max_depth > 0 &&
                         !P->count && ring_on && ring_fits;
  dj.ring_log2 = want_ring ? 0 : -1;  // provisional: the LDS layouts reserve the per-wave batch tables
  // schedule: explicit (diagnostic flags) or the persistent LDS kernel when the geometry fits
  int variant = (job->flags >> 8) & 0xff;
  // traversal stack: 16 LDS entries for the persistent kernel, 16 or 32 for the plain grid (the
  // most its occupancy allows), deeper BVHs spill the rest to a global per-wave area
  const int need = std::max(1, s->stack_need);
  int treelet_entries = kLdsStack;  // LDS stack entries per lane of the treelet schedule
  DevScene& dscene = P->dscene;
  dscene = s->dev;         // this render's view (the treelet schedule sets its LDS part)
  dscene.node_visits = P->count ? s->probe_visits : nullptr;  // the hot-treelet probe only
  dj.lds_sphere_f4 = 3;    // 48-B sphere records in LDS (bank spread)
  // persistent LDS schedule, by scene size (DESIGN.md §3 "occupancy"): five 4-wave workgroups per CU
  // when five copies of scene + stacks fit one CU's LDS (5 waves per SIMD at <= 96 VGPRs; Cornell
  // -9.3 %); else one 16-wave workgroup (4 waves per SIMD, the most one workgroup holds) plus, when a
  // second copy fits beside it, a 4-wave workgroup from a second persistent launch (dual, below); else
  // the 16-wave workgroup alone. RTG_LDS_WAVES=16 keeps the single workgroup, RTG_DUAL=0 no dual.
  // stack entries of the persistent LDS schedule: 16-bit for 4-wide trees whose leaf codes fit 16 bits
  // (first primitive < 4096) and whose node array ends below 32 KB of LDS (inner codes are absolute LDS
  // addresses) and whose stack needs no spill (kernel LdsStack16), else 32-bit
  const bool lds_entries_knob = K.stack_lds_entries > 0;
  const bool stk16 = dscene.node_width == 4 && dscene.num_refs <= 4096 && dscene.num_nodes * 112 <= 32768 &&
                     need <= kLdsStack && !lds_entries_knob && !dscene.tex_full;
  dj.stack_esz = stk16 ? 2 : 4;
  dj.lds_waves = kLdsWaves;
  int lds_bytes = lds_layout(dscene, kLdsStack, kLdsWaves, dj.stack_esz, &dj);
  int lds_wgs = 1;  // persistent workgroups per CU
  {
    DevJob t = dj;
    const int b4 = lds_layout(dscene, kLdsStack, 4, dj.stack_esz, &t);
    if ((K.lds_waves == 0 || K.lds_waves == 4) && dscene.node_width == 4 && need <= kLdsStack &&
        !lds_entries_knob && b4 > 0 && lds_alloc(b4) * kSmallSceneWgs <= kLdsPerCu && (stk16 || dscene.tex_full)) {
      dj = t;
      dj.lds_waves = 4;
      lds_bytes = b4;
      lds_wgs = kSmallSceneWgs;
    }
  }
  // dual: the 16-wave workgroup's kernel (<= 104 VGPRs, tex_full off) leaves 96 registers per SIMD
  // lane (4 x 104 + 96 = 512) for one wave of the 4-wave kernel (<= 96 VGPRs); LDS must hold both
  // copies, with 32-B sphere records if the padded 48-B ones do not fit (book-1: 90 + 66 KB)
  DevJob j4{};
  int lds4 = -1;
  if (dj.lds_waves == kLdsWaves && stk16 && !dscene.tex_full && K.dual != 0 && K.lds_waves != 16 &&
      dual_fits_registers(P->count, want_ring, K.verbose)) {
    for (const int f4 : {3, 2}) {
      DevJob a = dj, b = dj;
      a.lds_sphere_f4 = b.lds_sphere_f4 = f4;
      const int b16 = lds_layout(dscene, kLdsStack, kLdsWaves, 2, &a);
      const int bb4 = lds_layout(dscene, kLdsStack, 4, 2, &b);
      if (b16 > 0 && bb4 > 0 && lds_alloc(b16) + lds_alloc(bb4) <= kLdsPerCu) {
        dj = a;
        lds_bytes = b16;
        j4 = b;
        j4.lds_waves = 4;
        lds4 = bb4;
        break;
      }
    }
  }
  // default: the whole scene in LDS (3); else the top of a 4-wide tree in LDS (5, config 5's 1M
  // spheres: -1.3 % against 4, profiles/r02_ab), else the plain grid (4)
  if (variant == 0) variant = lds_bytes > 0 ? 3 : (dscene.node_width >= 4 ? 5 : 4);
  if (variant == 5) {  // persistent workgroups with the top of the tree in LDS (4- or 8-wide trees)
    if (dscene.node_width < 4) return fail(RTG_E_INVALID, "schedule 5 needs a wide BVH (RTG_BVH_SAH)");
    dj.stack_esz = 4;
    dj.lds_waves = kLdsWaves;
    // LDS stack entries: trees that spill anyway may keep fewer of them in LDS and more treelet nodes
    treelet_entries = need > kLdsStack && !lds_entries_knob ? K.treelet_stack : kLdsStack;
    lds_bytes = lds_layout_treelet(&dscene, treelet_entries, kLdsWaves, &dj);
    if (lds_bytes < 0) return fail(RTG_E_INVALID, "schedule 5: no LDS room for the treelet");
  }
  if (variant == 4) variant = 0;  // plain-grid ballot schedule
  // shading batch: a trip costs more where node rows come through the caches (config 5: 40 -2.0 %
  // against 48, profiles/r02_ab), shading more with image / noise textures (earth_perlin: 56 -2.2 %)
  if (dj.shade_batch == 0)
    dj.shade_batch = (variant == 5 || variant == 0) ? kCacheShadeBatch
                                                    : (s->dev.tex_full ? kTexShadeBatch : kDefaultShadeBatch);
  if (variant == 3 && lds_bytes < 0) return fail(RTG_E_INVALID, "scene does not fit the LDS schedule");
  // schedules 1 and 2 (round 1's per-segment kernels) were retired in round 5
  // (tools/experiments/legacy_schedules.patch)
  if (variant == 1 || variant == 2) return fail(RTG_E_UNSUPPORTED, "schedules 1 and 2 were retired (round 5)");
  if (variant < 0 || variant > 5) return fail(RTG_E_INVALID, "unknown render schedule");
  int stack_depth = 0;
  int grid_blocks = 1, grid_waves = 0;
  if (variant == 3 || variant == 5) {
    stack_depth = kLdsStack;
    grid_blocks = std::max(1, std::min(s->num_cus * (variant == 3 ? lds_wgs : 1), dj.num_tiles));
    grid_waves = grid_blocks * (variant == 3 ? dj.lds_waves : kLdsWaves);
  } else if (variant == 0) {
    stack_depth = need <= 16 ? 16 : 32;
    grid_blocks = std::max(1, std::min(s->num_cus * kPlainWgsPerCu, (dj.num_tiles + 3) / 4));
    grid_waves = grid_blocks * 4;
  }
  dj.lds_stack = stack_depth;
  // RTG_STACK_LDS_ENTRIES (tests): keep fewer entries in LDS so the global spill path is exercised
  if (lds_entries_knob) dj.lds_stack = std::min(stack_depth, K.stack_lds_entries);
  if (variant == 5) dj.lds_stack = std::min(dj.lds_stack, treelet_entries);
  P->default_sched = variant == 3 || variant == 0 || variant == 5;  // the ballot-batched stream
  dj.spill_depth = P->default_sched ? std::max(0, need - dj.lds_stack) : 0;
  if (P->progressive && !P->default_sched)
    return fail(RTG_E_INVALID, "progressive rendering needs the default schedules");
  P->chunked = !P->progressive && dj.chunks > 1 && P->default_sched && dc.max_depth > 0;
  dj.ring_log2 = -1;
  dj.ring_words = nullptr;
  if (P->chunked && want_ring) {
    // per-tile combine: R tile slots of chunks x 64 float4 partials. R * chunks is
    // ~2^17 batches, about 8x the span between the oldest unfinished tile and the newest handed out
    // (a slot that is still in use only delays a batch); a ring of at least the shard's tiles never waits
    int lg = 0;
    if (K.tile_slots > 0) {
      while ((1 << lg) < K.tile_slots) ++lg;
    } else {
      while ((static_cast<int64_t>(2) << lg) * dj.chunks <= (int64_t(1) << 17)) ++lg;
    }
    while (lg > 0 && (1 << (lg - 1)) >= dj.num_tiles) --lg;  // no more slots than tiles
    // a unit's ring index (< 2^28, packed beside its entry) and the ring's byte size (< 2^31, one
    // buffer descriptor) bound the ring
    while (lg > 0 && (static_cast<int64_t>(dj.chunks) << (lg + 10)) >= (int64_t(1) << 31)) --lg;
    dj.ring_log2 = lg;
    P->ring_slots = 1 << lg;
    P->ring_bytes = (static_cast<size_t>(dj.chunks) << (lg + 10)) + (size_t(8) << lg);
  }
  // the tile hand-out order rtg_scene_prepare tuned for this camera and shard (none for the ring kernels, whose
  // slot hand-off needs tile-major order); the tile-cost probe's counters in its own (counting) render
  dj.tile_order = variant == 3 && dj.ring_log2 < 0 && s->order_dev && s->order_tiles == dj.num_tiles &&
                          s->order_key == order_key(cam, job, dj)
                      ? s->order_dev
                      : nullptr;
  dj.tile_cost = P->count ? s->probe_tile_cost : nullptr;
  // max_depth <= 0: every pixel is black and nothing is traced (camera.hpp:183-186): no kernel; the frame
  // (one-shot) or the chunk sums (progressive) are zeroed by rtg_render
  P->skip_kernel = dc.max_depth <= 0;
  if (P->skip_kernel || variant != 3) lds4 = -1;
  if (lds4 > 0) {  // the dual launch's job: the same frame, counters and buffers as dj
    const int32_t l4[] = {j4.lds_nodes, j4.lds_refs, j4.lds_spheres, j4.lds_quads, j4.lds_materials,
                          j4.lds_textures, j4.lds_perlin_vec, j4.lds_perlin_perm, j4.lds_stacks, j4.lds_ring};
    j4 = dj;
    j4.lds_waves = 4;
    j4.lds_nodes = l4[0], j4.lds_refs = l4[1], j4.lds_spheres = l4[2], j4.lds_quads = l4[3];
    j4.lds_materials = l4[4], j4.lds_textures = l4[5], j4.lds_perlin_vec = l4[6], j4.lds_perlin_perm = l4[7];
    j4.lds_stacks = l4[8];
    j4.lds_ring = l4[9];
    j4.trace = nullptr;  // the per-wave timeline covers the main launch's waves only
  }
  P->j4 = j4;
  P->variant = variant;
  P->lds_bytes = lds_bytes;
  P->lds4 = lds4;
  P->lds_wgs = lds_wgs;
  P->stack_depth = stack_depth;
  P->grid_blocks = grid_blocks;
  P->grid_waves = grid_waves;
  P->kmain = choose_kernel(dscene, dj, stack_depth, P->count, variant);
  if (!P->skip_kernel && !P->kmain.fn) return fail(RTG_E_INVALID, "no render kernel fits this plan");
  if (lds4 > 0) {
    P->kaux = choose_kernel(dscene, P->j4, stack_depth, P->count, variant);
    if (!P->kaux.fn) return fail(RTG_E_INVALID, "no render kernel fits the dual launch");
  }
  return RTG_OK;
}

// The camera (and shard rows) a hot treelet was tuned for.
uint64_t treelet_key(const rtg_camera_desc* c, const rtg_render_desc* j) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t k = 0; k < n; ++k) h = (h ^ b[k]) * 1099511628211ull;
  };
  const double d[] = {c->aspect_ratio, c->vfov, c->lookfrom[0], c->lookfrom[1], c->lookfrom[2], c->lookat[0],
                      c->lookat[1],    c->lookat[2], c->vup[0],   c->vup[1],    c->vup[2],    c->defocus_angle,
                      c->focus_dist};
  const int32_t i[] = {c->image_width, c->max_depth, j->row_begin, j->row_stride};
  mix(d, sizeof(d));
  mix(i, sizeof(i));
  return h | 1;  // never 0 (0: not tuned)
}

bool wants_treelet_tune(const rtg_scene* s, const rtg_camera_desc* cam, const rtg_render_desc* job, const Plan& P) {
  return P.variant == 5 && !P.count && s->knobs.treelet_hot && s->dev.node_width >= 4 &&
         treelet_key(cam, job) != s->treelet_key;
}

// Hot treelet (schedule 5, scenes whose tree does not fit LDS): the persistent workgroups keep the
// first treelet_bytes of the node array in LDS, so which nodes come first decides which visits are
// ds_reads. A probe render of this camera (1 sample per pixel on ~2^19 pixels: every k-th row of the shard, the
// counting kernel with one counter per node) counts the visits of every node; the node array is then
// renumbered on the host, the root first, the others by visits (ties and unvisited nodes in their
// previous order), and uploaded again. Traversal order and the frame are unchanged (same tree, same
// child slots); only where a node is read from changes. Runs on the first render of a camera.
rtg_status tune_treelet(rtg_scene* s, const rtg_camera_desc* cam, const rtg_render_desc* job, uint64_t key) {
  const auto t0 = std::chrono::steady_clock::now();
  const int64_t n = s->dev.num_nodes;
  s->treelet_key = key;  // tuned or not, a failed probe is not retried for this camera
  if (n <= 1 || n > (int64_t(1) << 24)) return RTG_OK;
  rtg_camera_desc c2 = *cam;
  c2.samples_per_pixel = 1;
  rtg_render_desc j2 = *job;
  j2.flags = RTG_RENDER_COUNT | RTG_RENDER_OUT_DEVICE | (5 << 8);
  {  // about 2^19 probe pixels: every k-th row of the shard (1080p: every 3rd, 4K: every 15th)
    rtg_camera_params full;
    resolve_camera(cam, &full);
    const int64_t shard_rows = (full.image_height - 1 - job->row_begin) / job->row_stride + 1;
    const int64_t k = std::max<int64_t>(1, std::min<int64_t>(64, (shard_rows * full.image_width) >> 19));
    j2.row_stride = job->row_stride * static_cast<int32_t>(k);
  }
  j2.row_count = 0;
  j2.partial = nullptr;
  j2.chunk_begin = j2.chunk_count = 0;
  j2.stream = nullptr;
  rtg_camera_params cp;
  resolve_camera(&c2, &cp);
  const int64_t rows = (cp.image_height - 1 - j2.row_begin) / j2.row_stride + 1;
  uint32_t* visits = nullptr;
  float* out = nullptr;
  RTG_HIP(dev_alloc(reinterpret_cast<void**>(&visits), n * 4), "hipMalloc(node visits)");
  hipError_t e = dev_alloc(reinterpret_cast<void**>(&out), rows * cp.image_width * 12);
  // the probe runs on the scene's own (non-blocking) stream: every copy here is ordered on it
  hipStream_t os = s->own_stream;
  if (e == hipSuccess) e = hipMemsetAsync(visits, 0, n * 4, os);
  rtg_status st = e == hipSuccess ? RTG_OK : hip_fail(e, "hot treelet probe buffers");
  if (st == RTG_OK) {
    s->probe_visits = visits;
    rtg_render_stats ps{};
    st = rtg_render(s, &c2, &j2, out, &ps);
    s->probe_visits = nullptr;
  }
  std::vector<uint32_t> cnt;
  std::vector<int32_t> rec;
  const int width = s->dev.node_width;
  const int64_t nb = node_bytes(width);
  const bool have_host = static_cast<int64_t>(s->host_nodes.size()) == n * nb / 4;
  if (st == RTG_OK) {
    cnt.resize(n);
    if (!have_host) rec.resize(n * nb / 4);  // device-built trees: the node array comes from the device
    e = hipMemcpyAsync(cnt.data(), visits, n * 4, hipMemcpyDeviceToHost, os);
    if (e == hipSuccess && !have_host) e = hipMemcpyAsync(rec.data(), s->dev.nodes, n * nb, hipMemcpyDeviceToHost, os);
    if (e == hipSuccess) e = hipStreamSynchronize(os);
    if (e != hipSuccess) st = hip_fail(e, "hot treelet download");
  }
  (void)hipFree(out);
  (void)hipFree(visits);
  if (st != RTG_OK) return st;
  if (have_host) rec.swap(s->host_nodes);
  std::vector<int32_t> order;
  if (!hot_order_nodes(rec.data(), width, cnt.data(), n, &order)) {
    s->host_nodes.clear();  // rec may be the host copy: it no longer claims to match the device array
    return fail(RTG_E_INVALID, "hot treelet: a BVH inner code outside the node array (corrupt tree)");
  }
  void* stage = nullptr;  // the renumbered array through pinned memory (one DMA), else from the vector
  if (host_alloc(&stage, n * nb) == hipSuccess) {
    std::memcpy(stage, rec.data(), n * nb);
    e = hipMemcpyAsync(const_cast<float4*>(s->dev.nodes), stage, n * nb, hipMemcpyHostToDevice, os);
  } else {
    stage = nullptr;
    e = hipMemcpyAsync(const_cast<float4*>(s->dev.nodes), rec.data(), n * nb, hipMemcpyHostToDevice, os);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(os);
  if (stage) (void)hipHostFree(stage);
  if (e != hipSuccess) {
    s->host_nodes.clear();  // the device array may be half written: no host copy claims to match it
    return hip_fail(e, "hot treelet upload");
  }
  s->host_nodes.swap(rec);  // the host copy follows the device order
  s->treelet_tune_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  s->treelet_cum.assign(n + 1, 0);
  for (int64_t k = 0; k < n; ++k) s->treelet_cum[k + 1] = s->treelet_cum[k] + cnt[order[k]];
  if (s->knobs.verbose) {
    const uint64_t total = s->treelet_cum[n], top = s->treelet_cum[std::min<int64_t>(n, 877)];
    std::fprintf(stderr, "[rtg] hot treelet: %.1f ms, probe %lld rows, %llu node visits, first 877 nodes %.1f %%\n",
                 s->treelet_tune_ms, static_cast<long long>(rows), static_cast<unsigned long long>(total),
                 total ? 100.0 * top / total : 0.0);
  }
  return RTG_OK;
}

// Cost-ordered tile hand-out (round 6; DESIGN.md §3 "tile order"). Units are handed out tile-major, so a tile
// of expensive pixels (the earth's contact with the ground in config 3, glass in book-1) may start late and
// run past the rest of the launch: the wave timeline of an 8-GPU shard of config 3 ends 2 ms after its median
// wave. A probe render of this camera and shard (the counting kernel at up to 4 samples per pixel by default,
// RTG_TILE_ORDER_SPP, one counter
// per tile: the segments its units traced) ranks the tiles; renders of that camera and shard then hand out
// the tiles in descending cost (ties in tile order), so the expensive units start first and the launch ends
// on cheap ones. Which wave renders a unit, and when, changes; what each unit sums does not: frames and
// segment counts are identical. For the LDS-resident schedule (3) only: the treelet schedule reads nodes and
// primitives through L1/L2, where tile-major order keeps the waves of a CU on neighbouring pixels — ordered by
// cost, config 5 rendered 3 % slower at N = 1 and 11 % slower per 8-GPU shard (profiles/r06_q). Nor for the
// ring kernels (their slot hand-off needs tile-major order).
bool wants_tile_order(const rtg_scene* s, const rtg_camera_desc* cam, const rtg_render_desc* job, const Plan& P) {
  return s->knobs.tile_order && !P.count && P.variant == 3 && !P.skip_kernel && P.dj.ring_log2 < 0 &&
         P.dj.num_tiles > 1 && order_key(cam, job, P.dj) != s->order_key;
}

rtg_status tune_tile_order(rtg_scene* s, const rtg_camera_desc* cam, const rtg_render_desc* job, const Plan& P) {
  const auto t0 = std::chrono::steady_clock::now();
  const int64_t n = P.dj.num_tiles;
  const uint64_t key = order_key(cam, job, P.dj);
  s->order_key = 0;  // the previous order no longer holds while this one is built
  rtg_camera_desc c2 = *cam;
  c2.samples_per_pixel = std::min(cam->samples_per_pixel, s->knobs.tile_order_spp);
  rtg_render_desc j2 = *job;
  j2.flags = RTG_RENDER_COUNT | RTG_RENDER_OUT_DEVICE | (job->flags & (0xff << 8));  // the render's schedule
  j2.row_count = P.rows;
  j2.partial = nullptr;
  j2.chunk_begin = j2.chunk_count = 0;
  j2.stream = nullptr;
  uint32_t* cost = nullptr;
  float* out = nullptr;
  RTG_HIP(dev_alloc(reinterpret_cast<void**>(&cost), n * 4), "hipMalloc(tile costs)");
  hipError_t e = dev_alloc(reinterpret_cast<void**>(&out), int64_t(P.rows) * P.W * 12);
  hipStream_t os = s->own_stream;  // the probe runs on the scene's own stream: every copy here is ordered on it
  if (e == hipSuccess) e = hipMemsetAsync(cost, 0, n * 4, os);
  rtg_status st = e == hipSuccess ? RTG_OK : hip_fail(e, "tile-cost probe buffers");
  if (st == RTG_OK) {
    s->probe_tile_cost = cost;
    rtg_render_stats ps{};
    st = rtg_render(s, &c2, &j2, out, &ps);
    s->probe_tile_cost = nullptr;
  }
  std::vector<uint32_t> cnt;
  if (st == RTG_OK) {
    cnt.resize(n);
    e = hipMemcpyAsync(cnt.data(), cost, n * 4, hipMemcpyDeviceToHost, os);
    if (e == hipSuccess) e = hipStreamSynchronize(os);
    if (e != hipSuccess) st = hip_fail(e, "tile-cost download");
  }
  (void)hipFree(out);
  (void)hipFree(cost);
  if (st != RTG_OK) return st;
  std::vector<int32_t> order(n);
  for (int64_t k = 0; k < n; ++k) order[k] = static_cast<int32_t>(k);
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return cnt[a] > cnt[b]; });
  if (s->order_cap < n) {
    if (s->order_dev) RTG_HIP(hipFree(s->order_dev), "hipFree(tile order)");  // device-synchronous
    s->order_dev = nullptr;
    s->order_cap = 0;
    RTG_HIP(dev_alloc(reinterpret_cast<void**>(&s->order_dev), n * 4), "hipMalloc(tile order)");
    s->order_cap = n;
  }
  RTG_HIP(hipMemcpyAsync(s->order_dev, order.data(), n * 4, hipMemcpyHostToDevice, os), "tile order upload");
  RTG_HIP(hipStreamSynchronize(os), "tile order upload");
  s->order_tiles = n;
  s->order_key = key;
  s->order_tune_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (s->knobs.verbose) {
    uint64_t total = 0;
    for (const uint32_t c : cnt) total += c;
    std::fprintf(stderr, "[rtg] tile order: %.1f ms, %lld tiles, probe %d spp, %llu segments, costliest tile %u\n",
                 s->order_tune_ms, static_cast<long long>(n), c2.samples_per_pixel,
                 static_cast<unsigned long long>(total), n ? cnt[order[0]] : 0u);
  }
  return RTG_OK;
}

// The culling margin covers ray origins with |coordinate| <= 2 s->origin_bound (culling_box: M = the
// primitive boxes' reach when the scene was created). A camera whose lens reaches farther out widens every
// node box on the device first (repad_nodes_kernel, on the render's stream; 1/16 headroom so a camera moving
// about does not repad every frame) by 2^-20 per unit of M added: the most any margin's origin terms grow (a
// quad's in-plane axes, 7 2^-24 |o|). Boxes only grow: frames are unchanged, the bound holds again.
rtg_status ensure_origin_bound(rtg_scene* s, const rtg_camera_desc* cam, hipStream_t stream) {
  if (s->dev.num_nodes <= 0) return RTG_OK;
  rtg_camera_params cp;
  resolve_camera(cam, &cp);
  double mc = 0.0;
  for (int a = 0; a < 3; ++a)
    mc = std::max(mc, std::fabs(cp.center[a]) + std::fabs(cp.defocus_disk_u[a]) + std::fabs(cp.defocus_disk_v[a]));
  if (mc <= 2.0 * s->origin_bound) return RTG_OK;
  if (!(mc < 1e30)) return fail(RTG_E_INVALID, "camera position not finite (or above 1e30)");
  const double target = 0.5 * mc * (1.0 + 1.0 / 16.0);
  const float delta = round_up(0x1p-20 * (target - s->origin_bound));
  RTG_HIP(launch_repad(reinterpret_cast<float*>(const_cast<float4*>(s->dev.nodes)), s->dev.num_nodes,
                       s->dev.node_width, delta, stream),
          "repad kernel launch");
  // synchronous: work on another stream (rtg_scene_prepare's probe and node download with a
  // NULL stream, a later render elsewhere) must see the repadded boxes; a camera moving outward is rare
  RTG_HIP(hipStreamSynchronize(stream), "repad kernel");
  s->origin_bound = target;
  s->host_nodes.clear();  // the hot treelet downloads the repadded array when it next tunes
  if (s->knobs.verbose) std::fprintf(stderr, "[rtg] culling margin widened for origins up to %.6g\n", target);
  return RTG_OK;
}

}  // namespace

extern "C" {

rtg_status rtg_render_plan(rtg_scene* s, const rtg_camera_desc* cam, const rtg_render_desc* job,
                           rtg_launch_plan* out) {
  if (!out) return fail(RTG_E_INVALID, "null argument");
  Plan P;
  const rtg_status st = plan_render(s, cam, job, &P);
  if (st != RTG_OK) return st;
  *out = rtg_launch_plan{};
  out->schedule = P.variant;
  out->workgroups = P.grid_blocks;
  out->waves_per_workgroup = P.kmain.block / 64;
  out->lds_bytes = P.kmain.dynamic_lds ? P.lds_bytes : 0;
  const KernelResources r = kernel_resources(P.kmain.fn);
  out->vgprs = r.vgprs;
  out->scratch_bytes = r.scratch;
  out->dual = P.lds4 > 0 ? 1 : 0;
  int waves_cu = 0;  // resident waves per CU of the persistent schedules
  if (P.variant == 3) waves_cu = P.lds_wgs * P.dj.lds_waves;
  if (P.variant == 5) waves_cu = kLdsWaves;
  if (out->dual) {
    out->dual_workgroups = s->num_cus;
    out->dual_lds_bytes = P.lds4;
    out->dual_vgprs = kernel_resources(P.kaux.fn).vgprs;
    waves_cu += 4;
  }
  out->waves_per_simd = waves_cu / 4;
  out->stack_entry_bytes = P.dj.stack_esz;
  out->lds_stack_entries = P.dj.lds_stack;
  out->spill_entries = P.dj.spill_depth;
  out->treelet_nodes = P.variant == 5 ? P.dscene.treelet_bytes / node_bytes(P.dscene.node_width) : 0;
  out->shade_batch = P.dj.shade_batch;
  out->leaf_batch = P.dj.leaf_batch;
  out->chunk_samples = P.dj.chunk_samples;
  out->chunks = P.dj.chunks;
  out->partial_bytes = !P.chunked ? 0 : P.ring_slots ? static_cast<int64_t>(P.ring_bytes)
                                                     : static_cast<int64_t>(P.out_bytes) * P.dj.chunks;
  out->tile_slots = P.ring_slots;
  out->num_cus = s->num_cus;
  out->ray_queue = 0;  // retired in round 5 (tools/experiments/ray_queue.patch)
  out->origin_bound = static_cast<int32_t>(std::min(std::ceil(s->origin_bound), 2147483647.0));
  out->node_width = P.dscene.node_width;
  if (P.variant == 5) {
    out->treelet_hot = s->treelet_key == treelet_key(cam, job) ? 1 : 0;
    out->treelet_tune_us = static_cast<int32_t>(std::min(s->treelet_tune_ms * 1e3, 2e9));
    const int64_t tn = P.dscene.treelet_bytes / node_bytes(P.dscene.node_width);
    if (out->treelet_hot && !s->treelet_cum.empty() && s->treelet_cum.back() > 0)
      out->treelet_visit_permille = static_cast<int32_t>(
          1000 * s->treelet_cum[std::min<int64_t>(tn, static_cast<int64_t>(s->treelet_cum.size()) - 1)] /
          s->treelet_cum.back());
  }
  return RTG_OK;
}

rtg_status rtg_scene_prepare(rtg_scene* s, const rtg_camera_desc* cam, const rtg_render_desc* job) {
  if (!s || !cam || !job) return fail(RTG_E_INVALID, "null argument");
  if (s->pending) return fail(RTG_E_INVALID, "a previous async render was not waited for");
  Plan P;
  rtg_status pst = plan_render(s, cam, job, &P);
  if (pst != RTG_OK) return pst;
  const bool treelet = wants_treelet_tune(s, cam, job, P), order = wants_tile_order(s, cam, job, P);
  if (!treelet && !order) return RTG_OK;
  RTG_HIP(hipSetDevice(s->device), "hipSetDevice");
  // renders still in flight on the caller's stream read the node array and the tile order this rewrites
  if (job->stream) RTG_HIP(hipStreamSynchronize(static_cast<hipStream_t>(job->stream)), "stream sync");
  if (treelet) {
    pst = tune_treelet(s, cam, job, treelet_key(cam, job));
    if (pst != RTG_OK) return pst;
  }
  // the tile order's probe runs on the renumbered node array (same frames; its costs are the render's)
  return order ? tune_tile_order(s, cam, job, P) : RTG_OK;
}

rtg_status rtg_hot_treelet_order_host(int32_t* nodes, const uint32_t* visits, int64_t num_nodes) {
  if (num_nodes < 0 || (num_nodes > 0 && (!nodes || !visits))) return fail(RTG_E_INVALID, "null argument");
  if (num_nodes > (int64_t(1) << 24)) return fail(RTG_E_INVALID, "num_nodes above 2^24");
  for (int64_t k = 0; k < num_nodes; ++k)  // every inner code must name a node of the array
    for (int c = 0; c < 4; ++c) {
      const int32_t code = nodes[k * 28 + 24 + c];
      if (code >= 0 && (code % 112 != 0 || code / 112 >= num_nodes))
        return fail(RTG_E_INVALID, "inner child code outside the node array");
    }
  std::vector<int32_t> order;
  if (!hot_order_nodes4(nodes, visits, num_nodes, &order)) return fail(RTG_E_INVALID, "corrupt node array");
  return RTG_OK;
}

rtg_status rtg_render(rtg_scene* s, const rtg_camera_desc* cam, const rtg_render_desc* job,
                      float* out_rgb, rtg_render_stats* stats) {
  if (!s || !cam || !job) return fail(RTG_E_INVALID, "null argument");
  if (!out_rgb && !job->partial) return fail(RTG_E_INVALID, "null output buffer");
  if (s->pending) return fail(RTG_E_INVALID, "a previous async render was not waited for");
  Plan P;
  rtg_status pst = plan_render(s, cam, job, &P);
  if (pst != RTG_OK) return pst;
  const Knobs& K = s->knobs;
  // the scene's first render on the treelet schedule tunes its hot treelet implicitly (probe, renumber,
  // plan again); a later camera or shard re-tunes only through rtg_scene_prepare, so a moving camera does
  // not pay a probe render and a node re-upload inside every frame's rtg_render
  if (s->treelet_key == 0 && wants_treelet_tune(s, cam, job, P)) {
    // the hot treelet only: the tile order's probe is rtg_scene_prepare's (no second probe inside a render)
    RTG_HIP(hipSetDevice(s->device), "hipSetDevice");
    if (job->stream) RTG_HIP(hipStreamSynchronize(static_cast<hipStream_t>(job->stream)), "stream sync");
    pst = tune_treelet(s, cam, job, treelet_key(cam, job));
    if (pst != RTG_OK) return pst;
    P = Plan{};
    pst = plan_render(s, cam, job, &P);
    if (pst != RTG_OK) return pst;
  } else if (K.verbose && P.variant == 5 && !P.count && s->treelet_key != 0 && treelet_key(cam, job) != s->treelet_key) {
    // a moved camera keeps the first camera's hot treelet until rtg_scene_prepare re-tunes it
    std::fprintf(stderr, "[rtg] treelet render with the node order tuned for another camera or shard "
                         "(rtg_scene_prepare re-tunes it; plan.treelet_hot = 0)\n");
  }
  const int W = P.W, rows = P.rows;
  DevJob& dj = P.dj;
  DevJob& j4 = P.j4;

  RTG_HIP(hipSetDevice(s->device), "hipSetDevice");
  hipStream_t stream = job->stream ? static_cast<hipStream_t>(job->stream) : s->own_stream;
  pst = ensure_origin_bound(s, cam, stream);
  if (pst != RTG_OK) return pst;
  const size_t out_bytes = P.out_bytes;
  float* dout = out_rgb;
  if (!P.dev_out && out_rgb) {  // a scene-owned device frame (not the stream-ordered pool)
    if (s->dev_out_bytes < out_bytes) {
      RTG_HIP(hipStreamSynchronize(stream), "stream sync");
      if (s->dev_out) RTG_HIP(hipFree(s->dev_out), "hipFree(out)");
      s->dev_out = nullptr;
      s->dev_out_bytes = 0;
      RTG_HIP(dev_alloc(reinterpret_cast<void**>(&s->dev_out), out_bytes), "hipMalloc(out)");
      s->dev_out_bytes = out_bytes;
    }
    dout = s->dev_out;
  }
  dj.out = dout;
  SyncOnError sync_on_error;
  sync_on_error.stream = stream;
  auto grow = [](ScratchBuf& b, size_t need, const char* what) -> rtg_status {
    if (b.p && b.bytes >= need) return RTG_OK;
    if (b.p) RTG_HIP(hipFree(b.p), "hipFree(scratch)");  // device-synchronous: nothing still reads it
    b.p = nullptr;
    b.bytes = 0;
    RTG_HIP(dev_alloc(&b.p, std::max<size_t>(need, 256)), what);
    b.bytes = need;
    return RTG_OK;
  };
  dj.spill = nullptr;
  if (dj.spill_depth > 0) {
    pst = grow(s->scr_spill, static_cast<size_t>(P.grid_waves) * 64 * dj.spill_depth * sizeof(int32_t),
               "hipMalloc(stack spill)");
    if (pst != RTG_OK) return pst;
    dj.spill = static_cast<int32_t*>(s->scr_spill.p);
  }
  dj.counters = s->counters;
  RTG_HIP(hipMemsetAsync(s->counters, 0, kNumCounters * sizeof(unsigned long long), stream), "hipMemsetAsync");
  // optional per-wave timeline for schedule analysis (tools/wave_trace.py)
  const bool trace = !K.wave_trace.empty();
  int64_t trace_slots = 0;
  if (trace) {
    trace_slots = int64_t(P.grid_waves);
    if ((pst = grow(s->scr_trace, trace_slots * 32, "hipMalloc(trace)")) != RTG_OK) return pst;
    dj.trace = static_cast<unsigned long long*>(s->scr_trace.p);
    RTG_HIP(hipMemsetAsync(dj.trace, 0, trace_slots * 32, stream), "hipMemset(trace)");
  }
  if (P.chunked && P.ring_slots) {  // [slot words: gen R, ticket R][ring of tile slots]
    if ((pst = grow(s->scr_partial, P.ring_bytes, "hipMalloc(tile ring)")) != RTG_OK) return pst;
    unsigned char* base = static_cast<unsigned char*>(s->scr_partial.p);
    const size_t words = size_t(8) * P.ring_slots;  // a multiple of 16 B at the allocation's start
    RTG_HIP(hipMemsetAsync(base, 0, words, stream), "hipMemsetAsync(tile ring words)");
    dj.ring_words = reinterpret_cast<uint32_t*>(base);
    dj.partial = reinterpret_cast<float*>(base + words);
  } else if (P.chunked) {
    if ((pst = grow(s->scr_partial, out_bytes * dj.chunks, "hipMalloc(partial sums)")) != RTG_OK) return pst;
    dj.partial = static_cast<float*>(s->scr_partial.p);
  }
  if (P.skip_kernel && P.progressive)
    RTG_HIP(hipMemsetAsync(dj.partial + static_cast<size_t>(dj.chunk_begin) * rows * W * 3, 0,
                           out_bytes * dj.chunks, stream),
            "hipMemsetAsync(partial sums)");
  if (P.skip_kernel && !P.progressive && dout) RTG_HIP(hipMemsetAsync(dout, 0, out_bytes, stream), "hipMemsetAsync(out)");
  RTG_HIP(hipEventRecord(s->ev0, stream), "hipEventRecord");
  const int lds4 = P.lds4;
  if (K.verbose)
    std::fprintf(stderr, "[rtg] schedule %d: %d workgroups of %d waves, %d B LDS, stack %d x %d B, dual %s (%d B)\n",
                 P.variant, P.grid_blocks, P.kmain.block / 64, P.lds_bytes, P.stack_depth, dj.stack_esz,
                 lds4 > 0 ? "on" : "off", lds4);
  if (lds4 > 0) {
    j4.out = dj.out;
    j4.counters = dj.counters;
    j4.spill = dj.spill;
    j4.partial = dj.partial;
    j4.ring_words = dj.ring_words;
    // the aux launch must sit in a hardware queue of its own, or it only starts after the main launch
    // has drained (HIP shares its GPU_MAX_HW_QUEUES = 4 queues round-robin among a process's streams:
    // with RCCL or a second library's streams the two launches serialised, +10 %); high-priority
    // streams are served from a separate queue pool
    if (!s->aux_stream) {
      int least = 0, greatest = 0;
      RTG_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
      RTG_HIP(hipStreamCreateWithPriority(&s->aux_stream, hipStreamNonBlocking, greatest), "hipStreamCreate");
    }
    if (!s->ev_fork) RTG_HIP(hipEventCreateWithFlags(&s->ev_fork, hipEventDisableTiming), "hipEventCreate");
    if (!s->ev_join) RTG_HIP(hipEventCreateWithFlags(&s->ev_join, hipEventDisableTiming), "hipEventCreate");
    RTG_HIP(hipEventRecord(s->ev_fork, stream), "hipEventRecord");
    RTG_HIP(hipStreamWaitEvent(s->aux_stream, s->ev_fork, 0), "hipStreamWaitEvent");
  }
  if (!P.skip_kernel)
    RTG_HIP(launch_render(P.kmain, P.dscene, P.dc, dj, P.lds_bytes, P.grid_blocks, stream), "render kernel launch");
  if (lds4 > 0) {
    RTG_HIP(launch_render(P.kaux, P.dscene, P.dc, j4, lds4, s->num_cus, s->aux_stream), "render kernel launch (aux)");
    RTG_HIP(hipEventRecord(s->ev_join, s->aux_stream), "hipEventRecord");
    RTG_HIP(hipStreamWaitEvent(stream, s->ev_join, 0), "hipStreamWaitEvent");
  }
  if ((P.chunked && !P.ring_slots && !(P.skip_kernel && !P.progressive)) || (P.progressive && dout))
    RTG_HIP(launch_combine(dj.partial, dout, static_cast<int64_t>(rows) * W, P.sum_chunks, P.out_scale, stream),
            "combine kernel launch");
  RTG_HIP(hipEventRecord(s->ev1, stream), "hipEventRecord");
  if (trace) {
    std::vector<unsigned long long> tr(static_cast<size_t>(trace_slots) * 4);
    RTG_HIP(hipMemcpyAsync(tr.data(), dj.trace, trace_slots * 32, hipMemcpyDeviceToHost, stream), "trace copy");
    RTG_HIP(hipStreamSynchronize(stream), "trace sync");
    if (FILE* f = std::fopen(K.wave_trace.c_str(), "wb")) {
      std::fwrite(tr.data(), 8, tr.size(), f);
      std::fclose(f);
    }
  }
  RTG_HIP(hipMemcpyAsync(s->host_counters, s->counters, kNumCounters * sizeof(unsigned long long),
                         hipMemcpyDeviceToHost, stream),
          "hipMemcpyAsync(counters)");
  if (!P.dev_out && out_rgb) {
    if (s->host_stage_bytes < out_bytes) {
      if (s->host_stage) RTG_HIP(hipHostFree(s->host_stage), "hipHostFree(stage)");
      s->host_stage = nullptr;
      s->host_stage_bytes = 0;
      RTG_HIP(host_alloc(&s->host_stage, out_bytes), "hipHostMalloc(stage)");
      s->host_stage_bytes = out_bytes;
    }
    RTG_HIP(hipMemcpyAsync(s->host_stage, dout, out_bytes, hipMemcpyDeviceToHost, stream), "hipMemcpy(out)");
    s->pending_host_out = out_rgb;
    s->pending_host_bytes = out_bytes;
  }
  sync_on_error.committed = true;
  s->pending = true;
  s->pending_stream = stream;
  {
    const int spp = cam->samples_per_pixel;
    const int s0 = std::min(spp, dj.chunk_begin * dj.chunk_samples);
    const int s1 = P.progressive ? std::min(spp, (dj.chunk_begin + dj.chunks) * dj.chunk_samples) : spp;
    s->pending_samples = static_cast<uint64_t>(rows) * W * static_cast<uint64_t>(s1 - s0);
  }
  s->pending_tile_order = dj.tile_order != nullptr;
  if (P.async) return RTG_OK;
  return collect_stats(s, stats);
}

rtg_status rtg_render_wait(rtg_scene* s, rtg_render_stats* stats) {
  if (!s) return fail(RTG_E_INVALID, "null scene");
  if (!s->pending) return fail(RTG_E_INVALID, "no render pending");
  RTG_HIP(hipSetDevice(s->device), "hipSetDevice");
  return collect_stats(s, stats);
}

rtg_status rtg_resolve_rgb8(rtg_scene* s, const float* in_rgb, uint8_t* out_rgb8, int64_t n_pixels,
                            void* stream) {
  if (!s || !in_rgb || !out_rgb8) return fail(RTG_E_INVALID, "null argument");
  RTG_HIP(hipSetDevice(s->device), "hipSetDevice");
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : s->own_stream;
  RTG_HIP(launch_resolve(in_rgb, out_rgb8, n_pixels, st), "resolve kernel launch");
  if (!stream) RTG_HIP(hipStreamSynchronize(st), "resolve kernel");
  return RTG_OK;
}

}  // extern "C"
