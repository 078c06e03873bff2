// rtg_internal.hpp — layouts shared by the host scene compiler (rtg_api.cpp, rtg_bvh.cpp) and the
// gfx950 kernels (rtg_kernels.hip). Not part of the public C-ABI (include/rtgpu.h).
//
// Device scene layout in HBM (all 16-B aligned, read-only during a render):
//   nodes    : float4[4*num_nodes]   64-B child-pair BVH node (both child boxes + child codes)
//   refs     : int32[num_refs]       leaf primitive references (bit 30 = quad)
//   spheres  : float4[2*num_spheres] {c0.xyz, r}, {dc.xyz, material}
//   quads    : float4[5*num_quads]   {Q.xyz, D}, {u.xyz, material}, {v.xyz, -}, {w.xyz, -}, {n.xyz, -}
//   materials: float4[2*num_mats]    {type, texture, fuzz, eta}, {albedo.xyz, -}
//   textures : float4[2*num_tex]     {type, even, odd, scale}, {color.xyz, image|perlin}
//   images   : int4[num_images]      {width, height, byte offset lo, byte offset hi} + uint8 texels
//   perlin   : per table float4 randvec[256]; permutation words (kPerlinPermWords per table, below)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "rtgpu.h"

namespace rtg {

constexpr int32_t kEmptyChild = INT32_MIN;  // child slot with an inverted box; never visited
constexpr int32_t kQuadRefBit = 1 << 30;
// A perlin table's permutations as the noise lookup reads them (perlin.hpp:95-158): 16-bit lanes, each a
// gradient index times 16 (its byte offset among the 16-B gradient rows); X[i] = (p_x[i], p_x[i+1]) in one
// word, Y[j] = {(p_y[j], p_y[j]), (p_y[j+1], p_y[j+1])} and Z[k] = {(p_z[k], p_z[k]), (p_z[k+1], p_z[k+1])}
// in two (indices + 1 mod 256), so X[i] ^ Y[j][dj] ^ Z[k][dk] holds the offsets of corners (0, dj, dk) and
// (1, dj, dk). Words: X 256, then Y 2 x 256, then Z 2 x 256
constexpr int32_t kPerlinPermWords = 1280;

// A float view of the scene, ready for upload. Produced on the host from rtg_scene_desc.
struct HostScene {
  std::vector<float> nodes;      // 16 floats per node
  std::vector<int32_t> refs;
  std::vector<float> spheres;    // 8 floats per sphere
  std::vector<float> quads;      // 20 floats per quad
  std::vector<float> materials;  // 8 floats per material
  std::vector<float> textures;   // 8 floats per texture
  std::vector<int32_t> image_hdr;  // 4 ints per image
  std::vector<uint8_t> texels;
  std::vector<float> perlin_vec;   // 4 floats * 256 per table
  std::vector<uint32_t> perlin_perm;  // kPerlinPermWords per table
  // exact-t tie rule: the input (list-order) index of every sphere slot, then of every
  // quad slot; read by the kernels only when a primitive's root equals the closest hit so far
  std::vector<int32_t> tie_rank;
  int64_t num_nodes = 0;
  int32_t depth = 0;
  int32_t stack_need = 0;  // traversal stack entries needed (<= depth for BVH2)
  int32_t node_width = 2;  // 2: child-pair 64-B nodes, 4: 4-wide 112-B nodes
  int64_t num_prims = 0;
  bool gpu_bvh = false;       // RTG_BVH_GPU: nodes are built on the device after the upload
  int64_t occluder_prim = -1;  // input primitive kept out of the BVH (a sphere; -1: none)
  int32_t occluder = -1;       // its sphere index (stored after the BVH-referenced spheres)
  int64_t node_capacity = 0;  // gpu_bvh: 4-wide nodes to reserve
  // M of the culling margin: the node boxes are padded for ray origins with |coordinate| <= M
  // (rtg_api.cpp pad_down; DESIGN.md §4 "conservative culling")
  double origin_bound = 0.0;
  double bvh_ms = 0.0, collapse_ms = 0.0;  // host build phases (rtg_scene_info)
};

// Double-precision BVH produced by the builders (child-pair form, pre-order DFS).
struct BuildNode {
  double lo[2][3];
  double hi[2][3];
  int32_t child[2];
  int32_t count[2];
};

struct Bvh {
  std::vector<BuildNode> nodes;
  std::vector<int64_t> refs;  // primitive indices (into desc->prims)
  int32_t depth = 0;
};

// W-wide node collapsed from the binary tree (2..W children; unused slots kEmptyChild), W = 4 or 8.
template <int W>
struct BuildNodeW {
  double lo[W][3];
  double hi[W][3];
  int32_t child[W];  // >= 0 node index, < 0 leaf -(1 + first ref), kEmptyChild unused
  int32_t count[W];
};
using BuildNode4 = BuildNodeW<4>;

template <int W>
struct BvhW {
  std::vector<BuildNodeW<W>> nodes;
  int32_t depth = 0;       // nodes on the longest root-to-leaf path
  int32_t max_pushes = 0;  // most stack entries an ordered traversal (one per sibling) can hold at once
};
using Bvh4 = BvhW<4>;

// Collapse a binary child-pair BVH into a W-wide one: greedy (open the largest-area inner child until
// W slots are filled; leaves unchanged) or SAH-optimal (dynamic program over the binary tree; may
// merge small subtrees into leaves of up to max_leaf primitives, whose refs are contiguous).
struct CollapseParams {
  bool sah = false;
  double c_node = 1.0;  // cost of a wide-node visit relative to one primitive test
  int max_leaf = 4;     // <= 8 (the leaf code's count field)
};
template <int W>
void collapse_bvh(const Bvh& bin, BvhW<W>* out, const CollapseParams& prm = CollapseParams{});
inline void collapse_bvh4(const Bvh& bin, Bvh4* out, const CollapseParams& prm = CollapseParams{}) {
  collapse_bvh<4>(bin, out, prm);
}

// Renumber a W-wide tree so its first `top` nodes are the top of the tree in breadth-first order
// (the root stays node 0; the rest keep their depth-first order). Scenes too large for LDS keep
// that prefix in LDS (the treelet schedule), so the nodes every ray visits are ds_reads.
constexpr int64_t kTreeletBfsNodes = 4096;
template <int W>
void reorder_top_bfs(BvhW<W>* t, int64_t top);
// Hot treelet (rtg_scene_prepare): renumber n device-format W-wide nodes (28 W bytes = 7 W int32 each:
// six plane rows, then the code row; inner child = byte offset of its node) so the root stays first
// and the others follow by descending visits (stable); inner codes remapped, leaf and empty codes
// unchanged. order_out[k] = the old index of new node k. Returns false, renumbering nothing, when an inner
// code does not name a node of the array.
bool hot_order_nodes(int32_t* rec, int width, const uint32_t* visits, int64_t n, std::vector<int32_t>* order_out);
inline bool hot_order_nodes4(int32_t* rec, const uint32_t* visits, int64_t n, std::vector<int32_t>* order_out) {
  return hot_order_nodes(rec, 4, visits, n, order_out);
}
// Device bytes of one node of a W-wide tree (W = 4: 112, W = 8: 224).
constexpr int node_bytes(int width) { return 28 * width; }

// aabb of one primitive exactly as the reference computes it (aabb.hpp:30-48,135-154;
// sphere.hpp:16-44; quad.hpp:30-38).
void prim_bbox(const rtg_primitive& p, double lo[3], double hi[3]);

bool build_bvh(const rtg_scene_desc* desc, Bvh* out, std::string* err);
// rtg_bvh_node_order: the leaf order of bvh_node(objects, 0, n) over n boxes {lo.xyz, hi.xyz} (rtg_bvh.cpp)
void bvh_node_order(const double* boxes6, int64_t n, int64_t* order);
bool compile_scene(const rtg_scene_desc* desc, HostScene* out, std::string* err);
void resolve_camera(const rtg_camera_desc* cam, rtg_camera_params* out);
// Counted allocations (rtg_allocation_count; rtg_api.cpp): every device / pinned-host buffer of the library
hipError_t dev_alloc(void** p, size_t bytes);
hipError_t dev_alloc_async(void** p, size_t bytes, hipStream_t st);
hipError_t host_alloc(void** p, size_t bytes);
// rtg_last_error() text of the calling thread; returns `code` (rtg_api.cpp)
rtg_status set_last_error(rtg_status code, const std::string& msg);

// Kernel-side camera / job parameters (passed by value to the kernels).
struct DevCamera {
  float center[3];
  float pixel00[3];
  float du[3];
  float dv[3];
  float defu[3];
  float defv[3];
  float background[3];
  float scale;  // pixel_samples_scale
  int32_t width;
  int32_t height;
  int32_t spp;
  int32_t max_depth;
  int32_t defocus;  // defocus_angle > 0
};

struct DevScene {
  const float4* nodes;
  const int32_t* refs;
  const float4* spheres;
  const float4* quads;
  const float4* materials;
  const float4* textures;
  const int4* images;
  const uint8_t* texels;
  const float4* perlin_vec;
  const uint32_t* perlin_perm;
  int64_t num_nodes;
  int64_t num_refs;
  int64_t num_spheres;
  int64_t num_quads;
  int32_t node_width;  // 2 or 4 (see HostScene)
  int32_t num_materials;
  int32_t num_textures;
  // leaf reference mode: 0 = look up refs[]; 1 = refs[r] == r, all spheres; 2 = refs[r] == r | quad
  // (single-kind scenes store primitives in reference order, so the indirection is the identity)
  int32_t ref_mode;
  int32_t tex_full;  // 1 when some texture is an image or noise texture (kernel variant selector)
  int32_t diffuse_only;  // 1 when no material is metal or dielectric (kernel variant selector)
  int32_t num_perlins;  // perlin tables (256 gradients + kPerlinPermWords permutation words each)
  // 4-wide trees: inner-node codes are byte offsets from `nodes`, the root's is root_code (0 in
  // HBM; the persistent kernel rebases its LDS copy so codes are absolute LDS addresses) and every
  // valid one is below node_limit (root_code + num_nodes * 112)
  int32_t root_code;
  int32_t node_limit;
  // a sphere whose box spans most of the scene (book-1's ground) is kept out of the BVH and tested
  // by every ray before its traversal, in the shading phase (sphere index, -1: none)
  int32_t occluder;
  // treelet schedule: inner-node codes below this byte offset are read from the LDS copy of the
  // first nodes (the breadth-first top of the tree), the others from HBM / caches
  int32_t treelet_bytes;
  uint32_t treelet_lds;  // LDS byte address of that copy (set inside the kernel)
  int32_t sphere_f4;     // float4s per sphere record: 2 in HBM, DevJob::lds_sphere_f4 in the LDS copy
  // counting renders of the cache-read schedules: per-node visit counters (node index = code / 112),
  // the probe behind the hot treelet (rtg_api.cpp tune_treelet); null otherwise
  uint32_t* node_visits;
  // input (reference list-order) index of each sphere slot [0, num_spheres), then of each quad slot
  // [num_spheres, num_spheres + num_quads): the exact-t tie rule of the rtg-f32 spec
  const int32_t* tie_rank;
};

// A render kernel picked for a plan (rtg_kernels.hip choose_kernel); fn == nullptr: none fits.
struct KernelChoice {
  const void* fn = nullptr;
  int block = 0;             // threads per workgroup
  bool dynamic_lds = false;  // persistent kernels: the plan's LDS bytes are dynamic shared memory
};
struct KernelResources {
  bool ok = false;
  int vgprs = 0;
  int scratch = 0;  // private bytes per lane
};

struct GpuBvhResult {  // rtg_gpubvh.hip
  int64_t num_nodes;
  int32_t depth;
  int32_t stack_need;
};
// m: M of the culling margin (HostScene::origin_bound, rounded up; rtg_api.cpp culling_box)
hipError_t gpu_build_bvh4(const float4* spheres, const float4* quads, const int32_t* refs_in, int64_t n,
                          float m, float* nodes, int64_t max_nodes, int32_t* refs_out, GpuBvhResult* res,
                          hipStream_t st);

constexpr int kLdsStack = 16;  // LDS stack entries per lane of the persistent kernel

// Interleaved row shards of the multi-GPU frame (rtg_shard_layout, rtg_render_frame, rtg_gather_rows):
// rank r of N renders image rows r, r+N, ...; every shard is padded to P = ceil(H/N) rows.
struct ShardLayout {
  int32_t row_begin, row_stride, row_count, padded_rows;
};
inline ShardLayout shard_layout(int32_t height, int32_t nranks, int32_t rank) {
  ShardLayout L;
  L.row_begin = rank;
  L.row_stride = nranks;
  L.row_count = rank < height ? (height - 1 - rank) / nranks + 1 : 0;
  L.padded_rows = (height + nranks - 1) / nranks;
  return L;
}
// De-interleave: image row `row` comes from row (row / N) of rank (row % N)'s block, i.e. row
// (row % N) * P + row / N of the gathered staging buffer (shared by the kernel and its host twin).
__host__ __device__ inline int64_t gathered_row(int64_t row, int32_t nranks, int32_t padded) {
  return (row % nranks) * padded + row / nranks;
}

// Tuning / probe knobs of the library, read from the environment once per scene (rtg_scene_create)
// and clamped there, never per render (a stray variable then cannot change a render mid-run).
struct Knobs {
  bool verbose = false;         // RTG_VERBOSE: print the BVH and each render's launch plan
  int tile_lw = -1;             // RTG_TILE_LW 0..6: log2 tile width (-1: by shard stride)
  int chunk_samples = 0;        // RTG_CHUNK_SAMPLES >= 1 (schedule experiments; frames leave the spec)
  int stack_lds_entries = 0;    // RTG_STACK_LDS_ENTRIES 1..32 (tests: exercise the global spill)
  int lds_waves = 0;            // RTG_LDS_WAVES 4 | 16 (0: by scene size)
  int dual = -1;                // RTG_DUAL 0 | 1 (-1: where it fits)
  int tile_slots = -1;          // RTG_TILE_SLOTS 0 (full-frame partials) | 1..65536 (-1: by chunks)
  int treelet_stack = 16;       // RTG_TREELET_STACK 4..16: LDS stack entries of the treelet schedule
                                // (fewer: more treelet nodes, more spill traffic; spilling trees only)
  int treelet_hot = 1;          // RTG_TREELET_HOT 0 | 1: treelet of the most-visited nodes for the
                                // camera (a probe render counts node visits), 0: breadth-first top
  int tile_order = 1;           // RTG_TILE_ORDER 0 | 1: rtg_scene_prepare orders the tile hand-out by a
                                // probe render's per-tile cost (1), or leaves it tile-major (0)
  int tile_order_spp = 4;       // RTG_TILE_ORDER_SPP 1..64: samples per pixel of that probe (at most the render's)
  std::string wave_trace;      // RTG_WAVE_TRACE=<file>: per-wave timeline (tools/wave_trace.py)
};
Knobs read_knobs();

struct DevJob {
  uint64_t seed_mix;
  int32_t row_begin;
  int32_t row_stride;
  int32_t row_count;
  int32_t shade_batch;  // schedule 0: shade once ceil(alive * shade_batch / 64) lanes are ready
  float* out;
  // [0] segments, [1] box tests, [2] prim tests, [3] hits, [4] stack overflow, [5] bad BVH code,
  // [6] persistent kernels' tile counter, [7] workgroups that could not run the 16-bit LDS stack
  // layout (codes past 16 bits: RTG_E_UNSUPPORTED, nothing rendered), [8..23] schedule diagnostics,
  // [24] tile-ring waits that timed out (RTG_E_INTERNAL: frame incomplete), [25] batches that found
  // their ring slot still owned by an earlier tile (waits; diagnostic), [26] COUNT: traversal-stack pushes
  // into the global spill area
  unsigned long long* counters;
  int32_t leaf_batch;  // default schedules: run a leaf trip once this many lanes wait at a leaf
  int32_t tiles_x;    // 64-pixel tiles per shard row of tiles
  int32_t num_tiles;  // 64-pixel tiles in the shard (one wave's batch: a tile and a sample chunk)
  int32_t tile_lw;    // log2 tile width: 3 = 8x8 shard pixels, 4 = 16x4, 5 = 32x2 (row-strided shards)
  int32_t chunks;         // sample chunks rendered by this launch (work units = pixel x chunk)
  int32_t chunk_begin;    // first of them (progressive rendering; 0 for a one-shot frame)
  // chunks > 1, one-shot frame: log2 of the tile slots of the partial-sum ring (the chunks of a
  // tile are summed by the wave whose batch of that tile finishes last; DESIGN.md §4 "per-tile
  // combine"); -1: progressive rendering or one chunk (partial, if any, is the full-frame layout)
  int32_t ring_log2;
  int32_t chunk_samples;  // K: samples per chunk (the last chunk may be shorter)
  // ring_log2 >= 0: [slot][chunk][64 tile pixels] float4 partial sums (rgb, pad), written sc1;
  // else chunks > 1: [chunk][row][column][3] partial sums; else null
  float* partial;
  // ring_log2 >= 0: [0, R) slot generation (the tile that may write slot s next is gen * R + s),
  // [R, 2R) slot ticket (batches finished in the slot, all generations); zeroed before every launch
  uint32_t* ring_words;
  int32_t* spill;         // traversal-stack entries beyond the LDS part: [wave][depth][lane]
  int32_t spill_depth;    // entries per lane in `spill` (0: the LDS stack suffices)
  int32_t lds_stack;      // stack entries kept in LDS (the kernel's STACK; tests may lower it)
  // optional per-wave timeline (RTG_WAVE_TRACE, tools/wave_trace.py): 4 x u64 per wave =
  // {s_memrealtime at start, at end, pixels finished, block << 8 | wave}; null when off
  unsigned long long* trace;
  // persistent LDS kernel: byte offsets of the scene copies in dynamic LDS
  int32_t lds_nodes, lds_refs, lds_spheres, lds_quads, lds_materials, lds_textures;
  int32_t lds_perlin_vec, lds_perlin_perm;  // noise tables (full-texture kernels only)
  int32_t lds_sphere_f4;                     // float4s per sphere record in the LDS copy (2 or 3)
  int32_t lds_waves;                         // persistent LDS kernel: waves per workgroup
  int32_t stack_esz;                         // persistent kernels: bytes per LDS stack entry (2 or 4)
  int32_t lds_stacks;                        // persistent kernels: byte offset of the traversal stacks in LDS
  int32_t lds_ring;                          // RING kernels: byte offset of the per-wave batch tables (64 B each)
  // cost-ordered hand-out (rtg_scene_prepare): the tile handed out at each position, num_tiles entries, the
  // probe's most expensive tile first; null: tile-major (always null for RING kernels)
  const int32_t* tile_order;
  // the tile-cost probe (COUNT kernels only): segments traced per tile, num_tiles counters; else null
  uint32_t* tile_cost;
};

}  // namespace rtg
