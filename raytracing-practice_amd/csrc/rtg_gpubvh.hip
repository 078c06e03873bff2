// rtg_gpubvh.hip — device BVH construction (RTG_BVH_GPU): SURVEY.md §8f row 1, the GPU replacement
// of the host build of bvh_node::bvh_node (src/accelerator/bvh_node.hpp:25-77) for large scenes.
//
// Pipeline (all on the scene's stream, one host sync per 4-wide level at the end):
//   1. prim_bounds_kernel   primitive AABBs (fp32, padded outward) and the centroid bounds
//   2. morton_kernel        30-bit Morton codes of the centroids in those bounds
//   3. rocprim radix sort   (code, primitive) pairs
//   4. karras_kernel        binary radix tree over the sorted codes (Karras 2012), ties broken
//                           by primitive order, so the tree is deterministic
//   5. bounds_up_kernel     bottom-up node boxes: the second child to finish a node computes it
//                           (agent-scope acquire/release atomics: per-XCD L2s are not coherent)
//   6. collapse_kernel      level-synchronous top-down collapse into the library's 4-wide SoA
//                           nodes (open the largest-area child until 4 slots; subtrees of <= 4
//                           primitives become leaves), codes and stack bound as the host path
// The result uses exactly the node / leaf / ref encoding of the host builder (rtg_api.cpp), so the
// render kernels do not know which builder made the tree. LBVH trees are built in milliseconds
// but cost more traversal steps than the binned SAH; RTG_BVH_SAH stays the default.
#include <cstring>  // rocprim/iterator/texture_cache_iterator.hpp needs ::memset

#include <rocprim/device/device_radix_sort.hpp>

#include <cstdint>

#include "rtg_internal.hpp"

namespace rtg {
namespace {

constexpr int kLeafMax = 1;  // one primitive per leaf (−16 % on the 1M scene)
constexpr float kInfF = __builtin_huge_valf();

struct Box6 {
  float lo[3], hi[3];
};

// The culling margin of the host builder (rtg_api.cpp culling_box; DESIGN.md §4 "conservative culling"):
// each plane moves outward by c (|v| + M), c = 2^-21 for spheres, 2^-23 (1 + 2^-16) on an axis-aligned quad's
// flat axis and 2^-24 (6 U + 3 |v| + 2M) on its in-plane axes (U its extent there), 2^-18 on every axis of
// other quads; here the M terms come from the host
// (pads, rounded up) and the |v| terms are doubled, so that the box's own fp32 arithmetic (centre +- r, the
// corner sums, the minimum extent, this subtraction: a few 2^-24 |v|) is covered as well
struct CullPads {
  float sphere, quad, flat, inplane;  // 2^-21 M, 2^-18 M, 2^-23 M (1 + 2^-16), 2^-23 M; rounded up
};
__device__ __forceinline__ float pad_by(float v, float rel, float abs_pad) { return fabsf(v) * rel + abs_pad; }

// Box of one primitive record (the fp32 records the render kernels intersect), unpadded; thin axes other
// than an axis-aligned quad's flat one get the reference's 0.0001 minimum extent (aabb::pad_to_minimums,
// aabb.hpp:135-154).
__device__ Box6 prim_box(const float4* spheres, const float4* quads, int32_t ref, int* flat) {
  Box6 b;
  *flat = -1;
  if (ref & kQuadRefBit) {
    const float4* q = quads + static_cast<int64_t>(ref & ~kQuadRefBit) * 5;
    const float4 Q = q[0], u = q[1], v = q[2], n = q[4];
    const float px[4] = {Q.x, Q.x + u.x, Q.x + v.x, Q.x + u.x + v.x};
    const float py[4] = {Q.y, Q.y + u.y, Q.y + v.y, Q.y + u.y + v.y};
    const float pz[4] = {Q.z, Q.z + u.z, Q.z + v.z, Q.z + u.z + v.z};
    b.lo[0] = fminf(fminf(px[0], px[1]), fminf(px[2], px[3]));
    b.lo[1] = fminf(fminf(py[0], py[1]), fminf(py[2], py[3]));
    b.lo[2] = fminf(fminf(pz[0], pz[1]), fminf(pz[2], pz[3]));
    b.hi[0] = fmaxf(fmaxf(px[0], px[1]), fmaxf(px[2], px[3]));
    b.hi[1] = fmaxf(fmaxf(py[0], py[1]), fmaxf(py[2], py[3]));
    b.hi[2] = fmaxf(fmaxf(pz[0], pz[1]), fmaxf(pz[2], pz[3]));
    // flat axis (rtg_api.cpp quad_flat_axis): u and v each along one coordinate axis, normal exactly +-e_k
    const int nu = (u.x != 0.0f) + (u.y != 0.0f) + (u.z != 0.0f), nv = (v.x != 0.0f) + (v.y != 0.0f) + (v.z != 0.0f);
    const int iu = u.x != 0.0f ? 0 : u.y != 0.0f ? 1 : 2, iv = v.x != 0.0f ? 0 : v.y != 0.0f ? 1 : 2;
    if (nu == 1 && nv == 1 && iu != iv) {
      const int k = 3 - iu - iv;
      const float nn[3] = {n.x, n.y, n.z};
      if (fabsf(nn[k]) == 1.0f && nn[iu] == 0.0f && nn[iv] == 0.0f) *flat = k;
    }
  } else {
    const float4 s0 = spheres[static_cast<int64_t>(ref) * 2];
    const float4 s1 = spheres[static_cast<int64_t>(ref) * 2 + 1];
    const float r = fabsf(s0.w);
    const float c0[3] = {s0.x, s0.y, s0.z};
    const float c1[3] = {s0.x + s1.x, s0.y + s1.y, s0.z + s1.z};
    for (int k = 0; k < 3; ++k) {
      b.lo[k] = fminf(c0[k], c1[k]) - r;
      b.hi[k] = fmaxf(c0[k], c1[k]) + r;
    }
  }
  for (int k = 0; k < 3; ++k) {
    if (b.hi[k] - b.lo[k] < 0.0001f && k != *flat) {  // a flat axis gets its own pad (prim_bounds_kernel)
      b.lo[k] -= 0.00005f;
      b.hi[k] += 0.00005f;
    }
  }
  return b;
}

// order-preserving float <-> uint for atomic min/max of the centroid bounds
__device__ __forceinline__ uint32_t f2o(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float o2f(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__global__ void prim_bounds_kernel(const float4* spheres, const float4* quads, const int32_t* refs, int64_t n,
                                   CullPads pads, Box6* boxes, uint32_t* cbounds) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  float c[3] = {0.0f, 0.0f, 0.0f};
  const bool ok = i < n;
  if (ok) {
    const int32_t ref = refs[i];
    int flat;
    Box6 b = prim_box(spheres, quads, ref, &flat);
    const bool quad = (ref & kQuadRefBit) != 0;
    float qu[3] = {0.0f, 0.0f, 0.0f}, qv[3] = {0.0f, 0.0f, 0.0f};
    if (quad) {
      const float4* q = quads + static_cast<int64_t>(ref & ~kQuadRefBit) * 5;
      const float4 u = q[1], v = q[2];
      qu[0] = u.x, qu[1] = u.y, qu[2] = u.z, qv[0] = v.x, qv[1] = v.y, qv[2] = v.z;
    }
    for (int k = 0; k < 3; ++k) {  // centroid of the unpadded box: Morton codes independent of the margin
      c[k] = 0.5f * (b.lo[k] + b.hi[k]);
      // in-plane axis of an axis-aligned quad: 2^-24 (6 U_k + 3 |v| + 2M) as on the host, here 8 and 8 2^-24
      const bool inplane = quad && flat >= 0 && k != flat;
      const float rel = !quad || inplane ? 0x1p-20f : k == flat ? 0x1p-22f : 0x1p-17f;
      const float ab = !quad ? pads.sphere
                       : inplane ? fmaf(fabsf(qu[k]) + fabsf(qv[k]), 0x1p-21f, pads.inplane)
                       : k == flat ? pads.flat : pads.quad;
      b.lo[k] -= pad_by(b.lo[k], rel, ab);
      b.hi[k] += pad_by(b.hi[k], rel, ab);
    }
    boxes[i] = b;
  }
  for (int k = 0; k < 3; ++k) {
    uint32_t mn = ok ? f2o(c[k]) : 0xffffffffu, mx = ok ? f2o(c[k]) : 0u;
    for (int off = 32; off > 0; off >>= 1) {
      mn = min(mn, static_cast<uint32_t>(__shfl_xor(static_cast<int>(mn), off, 64)));
      mx = max(mx, static_cast<uint32_t>(__shfl_xor(static_cast<int>(mx), off, 64)));
    }
    if ((threadIdx.x & 63) == 0) {
      atomicMin(&cbounds[k], mn);
      atomicMax(&cbounds[3 + k], mx);
    }
  }
}

__device__ __forceinline__ uint32_t spread10(uint32_t v) {  // 10 bits -> every third bit
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000ffu;
  v = (v | (v << 8)) & 0x0300f00fu;
  v = (v | (v << 4)) & 0x030c30c3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

__global__ void morton_kernel(const Box6* boxes, int64_t n, const uint32_t* cbounds, uint32_t* codes,
                              uint32_t* ids) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Box6 b = boxes[i];
  // one scale for all three axes (the centroid bounds' largest extent): per-axis scales give a
  // thin axis — the 0.8-unit height of a 1000-unit sphere field — a third of the Morton bits, and
  // every split on it leaves two children that each span the whole field (3.4x the box tests)
  float ext = 0.0f;
  for (int k = 0; k < 3; ++k) ext = fmaxf(ext, o2f(cbounds[3 + k]) - o2f(cbounds[k]));
  uint32_t q[3];
  for (int k = 0; k < 3; ++k) {
    const float lo = o2f(cbounds[k]);
    const float c = 0.5f * (b.lo[k] + b.hi[k]);
    const float t = ext > 0.0f ? (c - lo) / ext : 0.5f;
    q[k] = static_cast<uint32_t>(fminf(fmaxf(t * 1024.0f, 0.0f), 1023.0f));
  }
  codes[i] = (spread10(q[0]) << 2) | (spread10(q[1]) << 1) | spread10(q[2]);
  ids[i] = static_cast<uint32_t>(i);
}

// common-prefix length of sorted keys i and j (Karras 2012), -1 outside [0, n)
__device__ __forceinline__ int delta(const uint32_t* codes, int64_t n, int64_t i, int64_t j) {
  if (j < 0 || j >= n) return -1;
  const uint32_t a = codes[i], b = codes[j];
  if (a != b) return __clz(a ^ b);
  return 32 + __clz(static_cast<uint32_t>(i ^ j));  // equal codes: primitive order decides
}

// binary radix tree: internal nodes 0..n-2 (0 is the root); child codes >= 0 internal, < 0 leaf ~j
__global__ void karras_kernel(const uint32_t* codes, int64_t n, int32_t* left, int32_t* right, int32_t* first,
                              int32_t* last, int32_t* iparent, int32_t* lparent) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n - 1) return;
  const int d = (delta(codes, n, i, i + 1) - delta(codes, n, i, i - 1)) >= 0 ? 1 : -1;
  const int dmin = delta(codes, n, i, i - d);
  int64_t lmax = 2;
  while (delta(codes, n, i, i + lmax * d) > dmin) lmax *= 2;
  int64_t l = 0;
  for (int64_t t = lmax / 2; t >= 1; t /= 2)
    if (delta(codes, n, i, i + (l + t) * d) > dmin) l += t;
  const int64_t j = i + l * d;
  const int dnode = delta(codes, n, i, j);
  int64_t s = 0;
  int64_t div = 2;
  int64_t t;
  do {
    t = (l + div - 1) / div;
    if (delta(codes, n, i, i + (s + t) * d) > dnode) s += t;
    div *= 2;
  } while (t > 1);
  const int64_t gamma = i + s * d + (d < 0 ? -1 : 0);
  const int64_t lo = i < j ? i : j, hi = i < j ? j : i;
  const int32_t lc = lo == gamma ? ~static_cast<int32_t>(gamma) : static_cast<int32_t>(gamma);
  const int32_t rc = hi == gamma + 1 ? ~static_cast<int32_t>(gamma + 1) : static_cast<int32_t>(gamma + 1);
  left[i] = lc;
  right[i] = rc;
  first[i] = static_cast<int32_t>(lo);
  last[i] = static_cast<int32_t>(hi);
  if (lc >= 0) iparent[lc] = static_cast<int32_t>(i); else lparent[~lc] = static_cast<int32_t>(i);
  if (rc >= 0) iparent[rc] = static_cast<int32_t>(i); else lparent[~rc] = static_cast<int32_t>(i);
  if (i == 0) iparent[0] = -1;
}

__device__ __forceinline__ Box6 load_box(const Box6* p) {
  Box6 b;
  const uint32_t* u = reinterpret_cast<const uint32_t*>(p);
  uint32_t v[6];
  for (int k = 0; k < 6; ++k) v[k] = __hip_atomic_load(u + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int k = 0; k < 3; ++k) {
    b.lo[k] = __uint_as_float(v[k]);
    b.hi[k] = __uint_as_float(v[3 + k]);
  }
  return b;
}
__device__ __forceinline__ void store_box(Box6* p, const Box6& b) {
  uint32_t* u = reinterpret_cast<uint32_t*>(p);
  for (int k = 0; k < 3; ++k) {
    __hip_atomic_store(u + k, __float_as_uint(b.lo[k]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(u + 3 + k, __float_as_uint(b.hi[k]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// leaves in sorted order: lbox[j] = box of sorted primitive j; internal boxes bottom-up
__global__ void bounds_up_kernel(const Box6* boxes, const uint32_t* ids, int64_t n, const int32_t* left,
                                 const int32_t* right, const int32_t* iparent, const int32_t* lparent,
                                 Box6* lbox, Box6* ibox, uint32_t* flags) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= n) return;
  store_box(&lbox[j], boxes[ids[j]]);
  if (n == 1) return;
  int32_t p = lparent[j];
  while (p >= 0) {
    // release our child's box, acquire the sibling's: the second arrival builds the parent
    const uint32_t old = __hip_atomic_fetch_add(&flags[p], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == 0) return;
    const int32_t l = left[p], r = right[p];
    const Box6 a = l >= 0 ? load_box(&ibox[l]) : load_box(&lbox[~l]);
    const Box6 b = r >= 0 ? load_box(&ibox[r]) : load_box(&lbox[~r]);
    Box6 u;
    for (int k = 0; k < 3; ++k) {
      u.lo[k] = fminf(a.lo[k], b.lo[k]);
      u.hi[k] = fmaxf(a.hi[k], b.hi[k]);
    }
    store_box(&ibox[p], u);
    __atomic_thread_fence(__ATOMIC_RELEASE);
    p = iparent[p];
  }
}

struct Slot {
  int32_t b;      // binary child code (>= 0 internal, < 0 leaf ~j)
  int32_t first;  // sorted range
  int32_t count;
};

__device__ __forceinline__ float half_area(const Box6& b) {
  const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
  return dx * dy + dy * dz + dz * dx;
}

struct CollapseIO {
  const int32_t *left, *right, *first, *last;
  const Box6 *lbox, *ibox;
  const int32_t* in_q;  // pairs (binary internal node, output node)
  int32_t n_in;
  const int32_t* in_push;
  int32_t* out_q;
  int32_t* out_push;
  uint32_t* counters;  // [0] output queue length, [1] node count, [2] max pushes
  float* nodes;        // 28 floats per node
  int64_t max_nodes;
};

__device__ __forceinline__ Slot make_slot(const CollapseIO& io, int32_t code) {
  Slot s;
  s.b = code;
  if (code < 0) {
    s.first = ~code;
    s.count = 1;
  } else {
    s.first = io.first[code];
    s.count = io.last[code] - io.first[code] + 1;
  }
  return s;
}

__global__ void collapse_kernel(CollapseIO io) {
  const int e = static_cast<int>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= io.n_in) return;
  const int32_t bnode = io.in_q[2 * e];
  const int32_t onode = io.in_q[2 * e + 1];
  const int32_t pushes = io.in_push[e];
  Slot slot[4];
  int ns = 0;
  if (bnode < 0) {  // the whole scene is one leaf
    slot[ns++] = make_slot(io, bnode);
  } else {
    slot[ns++] = make_slot(io, io.left[bnode]);
    slot[ns++] = make_slot(io, io.right[bnode]);
  }
  while (ns < 4) {  // open the largest-area child that is too big for a leaf
    int best = -1;
    float best_area = -1.0f;
    for (int k = 0; k < ns; ++k) {
      if (slot[k].b < 0 || slot[k].count <= kLeafMax) continue;
      const float a = half_area(io.ibox[slot[k].b]);
      if (a > best_area) {
        best_area = a;
        best = k;
      }
    }
    if (best < 0) break;
    const int32_t b = slot[best].b;
    slot[best] = make_slot(io, io.left[b]);
    slot[ns++] = make_slot(io, io.right[b]);
  }
  const int32_t here = pushes + ns - 1;
  atomicMax(&io.counters[2], static_cast<uint32_t>(here));
  float* f = io.nodes + static_cast<int64_t>(onode) * 28;
  for (int k = 0; k < 4; ++k) {
    int32_t code = kEmptyChild;
    Box6 bx;
    for (int a = 0; a < 3; ++a) {
      bx.lo[a] = kInfF;
      bx.hi[a] = -kInfF;
    }
    if (k < ns) {
      const Slot& s = slot[k];
      bx = s.b >= 0 ? io.ibox[s.b] : io.lbox[~s.b];
      if (s.b >= 0 && s.count > kLeafMax) {
        const int32_t child = static_cast<int32_t>(atomicAdd(&io.counters[1], 1u));
        const int32_t q = static_cast<int32_t>(atomicAdd(&io.counters[0], 1u));
        io.out_q[2 * q] = s.b;
        io.out_q[2 * q + 1] = child;
        io.out_push[q] = here;
        code = child * 112;  // inner children: byte offset of the node (as the host path)
      } else {
        code = ~((s.first << 3) | (s.count - 1));
      }
    }
    for (int a = 0; a < 3; ++a) {
      f[a * 4 + k] = bx.lo[a];
      f[12 + a * 4 + k] = bx.hi[a];
    }
    f[24 + k] = __int_as_float(code);
  }
}

__global__ void gather_refs_kernel(const int32_t* refs_in, const uint32_t* ids, int64_t n, int32_t* refs_out) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j < n) refs_out[j] = refs_in[ids[j]];
}

unsigned blocks_for(int64_t n) { return static_cast<unsigned>((n + 255) / 256); }

}  // namespace

#define GB_CHECK(x)                  \
  do {                               \
    hipError_t e_ = (x);             \
    if (e_ != hipSuccess) return e_; \
  } while (0)

// Builds the 4-wide BVH of n primitive refs (refs_in: input order) on the device. Writes up to
// max_nodes nodes (28 floats each) to `nodes` and the leaf-ordered refs to `refs_out` (n entries).
hipError_t gpu_build_bvh4(const float4* spheres, const float4* quads, const int32_t* refs_in, int64_t n,
                          float m, float* nodes, int64_t max_nodes, int32_t* refs_out, GpuBvhResult* res,
                          hipStream_t st) {
  *res = GpuBvhResult{};
  if (n <= 0) return hipSuccess;
  if (n > (int64_t(1) << 28) || max_nodes < 1) return hipErrorInvalidValue;
  const int64_t ni = n > 1 ? n - 1 : 1;
  // scratch: one allocation
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  const size_t o_boxes = take(n * sizeof(Box6)), o_lbox = take(n * sizeof(Box6)), o_ibox = take(ni * sizeof(Box6));
  const size_t o_codes = take(n * 4), o_codes2 = take(n * 4), o_ids = take(n * 4), o_ids2 = take(n * 4);
  const size_t o_left = take(ni * 4), o_right = take(ni * 4), o_first = take(ni * 4), o_last = take(ni * 4);
  const size_t o_ipar = take(ni * 4), o_lpar = take(n * 4), o_flags = take(ni * 4);
  const size_t o_q0 = take(max_nodes * 8), o_q1 = take(max_nodes * 8), o_p0 = take(max_nodes * 4),
               o_p1 = take(max_nodes * 4);
  const size_t o_cnt = take(64), o_cb = take(64);
  size_t sort_bytes = 0;
  GB_CHECK(rocprim::radix_sort_pairs(nullptr, sort_bytes, static_cast<uint32_t*>(nullptr),
                                     static_cast<uint32_t*>(nullptr), static_cast<uint32_t*>(nullptr),
                                     static_cast<uint32_t*>(nullptr), static_cast<size_t>(n), 0, 30, st));
  const size_t o_sort = take(sort_bytes);
  char* base = nullptr;
  GB_CHECK(hipMallocAsync(reinterpret_cast<void**>(&base), off, st));
  auto P = [&](size_t o) { return base + o; };
  Box6* boxes = reinterpret_cast<Box6*>(P(o_boxes));
  Box6* lbox = reinterpret_cast<Box6*>(P(o_lbox));
  Box6* ibox = reinterpret_cast<Box6*>(P(o_ibox));
  uint32_t* codes = reinterpret_cast<uint32_t*>(P(o_codes));
  uint32_t* codes2 = reinterpret_cast<uint32_t*>(P(o_codes2));
  uint32_t* ids = reinterpret_cast<uint32_t*>(P(o_ids));
  uint32_t* ids2 = reinterpret_cast<uint32_t*>(P(o_ids2));
  int32_t* left = reinterpret_cast<int32_t*>(P(o_left));
  int32_t* right = reinterpret_cast<int32_t*>(P(o_right));
  int32_t* first = reinterpret_cast<int32_t*>(P(o_first));
  int32_t* last = reinterpret_cast<int32_t*>(P(o_last));
  int32_t* ipar = reinterpret_cast<int32_t*>(P(o_ipar));
  int32_t* lpar = reinterpret_cast<int32_t*>(P(o_lpar));
  uint32_t* flags = reinterpret_cast<uint32_t*>(P(o_flags));
  int32_t* q[2] = {reinterpret_cast<int32_t*>(P(o_q0)), reinterpret_cast<int32_t*>(P(o_q1))};
  int32_t* pq[2] = {reinterpret_cast<int32_t*>(P(o_p0)), reinterpret_cast<int32_t*>(P(o_p1))};
  uint32_t* cnt = reinterpret_cast<uint32_t*>(P(o_cnt));
  uint32_t* cb = reinterpret_cast<uint32_t*>(P(o_cb));

  hipError_t err = hipSuccess;
  do {
    const uint32_t cb_init[6] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u};
    if ((err = hipMemcpyAsync(cb, cb_init, sizeof(cb_init), hipMemcpyHostToDevice, st)) != hipSuccess) break;
    // M terms of the culling pads (m: M rounded up; power-of-two scalings are exact, the flat factor is
    // rounded up by one ulp)
    const CullPads pads{m * 0x1p-21f, m * 0x1p-18f, __builtin_nextafterf(m * 0x1p-23f * (1.0f + 0x1p-16f), __builtin_inff()),
                        m * 0x1p-23f};
    hipLaunchKernelGGL(prim_bounds_kernel, dim3(blocks_for(n)), dim3(256), 0, st, spheres, quads, refs_in, n,
                       pads, boxes, cb);
    hipLaunchKernelGGL(morton_kernel, dim3(blocks_for(n)), dim3(256), 0, st, boxes, n, cb, codes, ids);
    if ((err = rocprim::radix_sort_pairs(P(o_sort), sort_bytes, codes, codes2, ids, ids2, static_cast<size_t>(n), 0,
                                         30, st)) != hipSuccess)
      break;
    if ((err = hipMemsetAsync(flags, 0, ni * 4, st)) != hipSuccess) break;
    if (n > 1)
      hipLaunchKernelGGL(karras_kernel, dim3(blocks_for(n - 1)), dim3(256), 0, st, codes2, n, left, right, first,
                         last, ipar, lpar);
    hipLaunchKernelGGL(bounds_up_kernel, dim3(blocks_for(n)), dim3(256), 0, st, boxes, ids2, n, left, right, ipar,
                       lpar, lbox, ibox, flags);
    hipLaunchKernelGGL(gather_refs_kernel, dim3(blocks_for(n)), dim3(256), 0, st, refs_in, ids2, n, refs_out);
    if ((err = hipGetLastError()) != hipSuccess) break;
    // collapse, one level per launch: queue entries (binary node, output node)
    const int32_t root[2] = {n > 1 ? 0 : ~0, 0};
    const int32_t zero = 0;
    if ((err = hipMemcpyAsync(q[0], root, sizeof(root), hipMemcpyHostToDevice, st)) != hipSuccess) break;
    if ((err = hipMemcpyAsync(pq[0], &zero, 4, hipMemcpyHostToDevice, st)) != hipSuccess) break;
    const uint32_t cnt_init[4] = {0u, 1u, 0u, 0u};
    if ((err = hipMemcpyAsync(cnt, cnt_init, sizeof(cnt_init), hipMemcpyHostToDevice, st)) != hipSuccess) break;
    int32_t n_in = 1;
    int depth = 0;
    uint32_t hc[4] = {0, 1, 0, 0};
    while (n_in > 0) {
      ++depth;
      CollapseIO io{left, right, first, last, lbox, ibox, q[(depth - 1) & 1], n_in, pq[(depth - 1) & 1],
                    q[depth & 1], pq[depth & 1], cnt, nodes, max_nodes};
      hipLaunchKernelGGL(collapse_kernel, dim3(blocks_for(n_in)), dim3(256), 0, st, io);
      if ((err = hipMemcpyAsync(hc, cnt, sizeof(hc), hipMemcpyDeviceToHost, st)) != hipSuccess) break;
      if ((err = hipStreamSynchronize(st)) != hipSuccess) break;
      if (static_cast<int64_t>(hc[1]) > max_nodes) {
        err = hipErrorInvalidValue;
        break;
      }
      n_in = static_cast<int32_t>(hc[0]);
      const uint32_t z = 0;
      if ((err = hipMemcpyAsync(cnt, &z, 4, hipMemcpyHostToDevice, st)) != hipSuccess) break;
    }
    if (err != hipSuccess) break;
    res->num_nodes = hc[1];
    res->depth = depth;
    res->stack_need = static_cast<int32_t>(hc[2]);
  } while (false);
  const hipError_t e2 = hipFreeAsync(base, st);
  if (err == hipSuccess) err = e2;
  if (err == hipSuccess) err = hipStreamSynchronize(st);
  return err;
}

}  // namespace rtg
