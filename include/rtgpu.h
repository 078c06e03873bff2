/*
 * rtgpu.h — C-ABI of the MI355X path-tracing library (librtgpu.so).
 *
 * This is the device boundary for the reference's per-pixel sample loop
 *   camera::render -> ray_color -> bvh_node::hit / sphere::hit -> material::scatter
 * (reference: src/core/camera.hpp:29-72, 180-232; src/accelerator/bvh_node.hpp:80-94;
 *  src/hittable/sphere.hpp:47-93; src/core/material.hpp:51-206).
 *
 * The reference has no FFI: its "operator API" is the C++ virtual surface
 * (hittable::hit, material::scatter, texture::value, camera::render). The C++ mirror of that
 * surface (raytracing-practice_amd/include/) flattens a world into an rtg_scene_desc and
 * calls the entry points below. Every signature uses plain pointers and sizes; nothing
 * throws across the boundary; every call returns an rtg_status (0 = OK, negative = error)
 * and rtg_last_error() describes the last failure on the calling thread.
 *
 * Threading: calls are blocking unless RTG_RENDER_ASYNC is set; one host thread (or process)
 * per GPU; a scene handle is bound to the device it was created on and must not be used
 * from two threads at once. The render RNG is stateless (counter-based), so calls are
 * reentrant and results do not depend on tiling or scheduling.
 */
#ifndef RTGPU_H
#define RTGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTG_ABI_VERSION 7

typedef int32_t rtg_status;
#define RTG_OK 0
#define RTG_E_INVALID (-1)     /* bad argument / malformed scene */
#define RTG_E_HIP (-2)         /* HIP runtime error (message in rtg_last_error) */
#define RTG_E_NODEVICE (-3)    /* no usable gfx950 device */
#define RTG_E_NOMEM (-4)       /* host or device allocation failed */
#define RTG_E_UNSUPPORTED (-5) /* feature not supported (e.g. BVH deeper than the kernel stack) */

/* ---- primitives: replaces sphere (sphere.hpp:16-23, 32-44) and quad (quad.hpp:12-27) ---- */
#define RTG_PRIM_SPHERE 1
#define RTG_PRIM_QUAD 2

typedef struct rtg_primitive {
  int32_t kind;     /* RTG_PRIM_SPHERE | RTG_PRIM_QUAD */
  int32_t material; /* index into rtg_scene_desc.materials */
  double p0[3];     /* sphere: centre at time 0 (ray center.orig) | quad: Q */
  double p1[3];     /* sphere: centre at time 1 (static: == p0)   | quad: u */
  double p2[3];     /* sphere: unused                             | quad: v */
  double radius;    /* sphere radius (sign kept, as the reference allows) */
} rtg_primitive;

/* ---- materials: replaces material.hpp:42-75, 80-111, 122-207, 223-240 ---- */
#define RTG_MAT_LAMBERTIAN 1
#define RTG_MAT_METAL 2
#define RTG_MAT_DIELECTRIC 3
#define RTG_MAT_DIFFUSE_LIGHT 4

typedef struct rtg_material {
  int32_t type;            /* RTG_MAT_* */
  int32_t texture;         /* lambertian / diffuse_light: index into textures */
  double albedo[3];        /* metal albedo */
  double fuzz;             /* metal fuzz, already clamped to <= 1 (material.hpp:83) */
  double refraction_index; /* dielectric */
} rtg_material;

/* ---- textures: replaces texture.hpp:25-41, 47-85, 91-122, 127-156 ---- */
#define RTG_TEX_SOLID 1
#define RTG_TEX_CHECKER 2
#define RTG_TEX_IMAGE 3
#define RTG_TEX_NOISE 4

typedef struct rtg_texture {
  int32_t type;    /* RTG_TEX_* */
  int32_t even;    /* checker: texture index of even cells */
  int32_t odd;     /* checker: texture index of odd cells */
  int32_t image;   /* image: index into images */
  int32_t perlin;  /* noise: index into perlins */
  int32_t pad_;
  double scale;    /* checker: constructor scale (inv_scale = 1.0f/scale, texture.hpp:50-51); noise: scale */
  double color[3]; /* solid albedo */
} rtg_texture;

/* RGB8 image after rtw_image::convert_to_bytes (rtw_stb_image.hpp:137-169); rgb == NULL or
 * height <= 0 means "could not load" and the texture returns cyan (texture.hpp:100-103). */
typedef struct rtg_image {
  int32_t width;
  int32_t height;
  const uint8_t* rgb; /* width*height*3 bytes, row 0 = top */
} rtg_image;

/* Perlin tables as drawn by perlin::perlin() (perlin.hpp:12-31). */
typedef struct rtg_perlin {
  double randvec[256][3];
  int32_t perm_x[256];
  int32_t perm_y[256];
  int32_t perm_z[256];
} rtg_perlin;

/* BVH construction modes (the library always builds its own device BVH). */
#define RTG_BVH_MEDIAN 0 /* bvh_node.hpp:25-77: longest axis, std::sort by bbox.min, median */
#define RTG_BVH_SAH 1    /* binned SAH, leaves of <= 4 primitives, collapsed to 4-wide nodes */
#define RTG_BVH_GPU 3    /* built on the device: Morton-code LBVH (Karras) collapsed to 4-wide nodes;
                            milliseconds for 1M primitives, more traversal steps than SAH */

typedef struct rtg_scene_desc {
  uint32_t abi_version; /* RTG_ABI_VERSION (6 is still accepted: it has no tie_rank, read as NULL) */
  int32_t bvh_mode;     /* RTG_BVH_* */
  const rtg_primitive* prims;
  int64_t num_prims; /* object order == hittable_list order */
  const rtg_material* materials;
  int32_t num_materials;
  int32_t num_textures;
  const rtg_texture* textures;
  const rtg_image* images;
  int32_t num_images;
  int32_t num_perlins;
  const rtg_perlin* perlins;
  /* ABI 7. Exact-t ties (H9): the reference's closest-hit walk keeps the first sphere and the last quad
   * hit at the smallest t (interval::surrounds, sphere.hpp:70; interval::contains, quad.hpp:62) in the
   * order it tests objects: a hittable_list in list order (hittable_list.hpp:40-64), a bvh_node left
   * then right (bvh_node.hpp:89-90), i.e. its children in the median tree's leaf order, not the list's.
   * tie_rank[i] = primitive i's position in that order, a permutation of 0..num_prims-1 (the C++
   * mirror's bvh_node fills it from rtg_bvh_node_order); NULL = the primitive order itself. */
  const int64_t* tie_rank;
} rtg_scene_desc;

/* ---- camera: the reference's public fields (camera.hpp:13-25) ---- */
typedef struct rtg_camera_desc {
  double aspect_ratio;
  int32_t image_width;
  int32_t samples_per_pixel;
  int32_t max_depth;
  int32_t pad_;
  double background[3];
  double vfov;
  double lookfrom[3];
  double lookat[3];
  double vup[3];
  double defocus_angle;
  double focus_dist;
} rtg_camera_desc;

/* camera::initialize() results (camera.hpp:76-136), computed in fp64 exactly as the reference. */
typedef struct rtg_camera_params {
  int32_t image_width;
  int32_t image_height;
  double pixel_samples_scale; /* float(1.0f / spp) (H7) */
  double center[3];
  double pixel00_loc[3];
  double pixel_delta_u[3];
  double pixel_delta_v[3];
  double u[3], v[3], w[3];
  double defocus_disk_u[3];
  double defocus_disk_v[3];
} rtg_camera_params;

/* ---- one render call ---- */
#define RTG_RENDER_OUT_DEVICE 0x1 /* out_rgb is a device pointer on the scene's device */
#define RTG_RENDER_ASYNC 0x2      /* do not synchronize (requires OUT_DEVICE); stats filled later */
#define RTG_RENDER_COUNT 0x4      /* also count box / primitive tests (slower, diagnostic) */
/* Diagnostic schedule selection (A/B of kernel variants; 0 = the default everywhere):
 * bits 8-15 schedule (0 default = 3 when the scene geometry fits in LDS, else 5 for 4-wide trees,
 * else 4; 3 persistent workgroups with LDS-resident geometry (five 4-wave workgroups per
 * CU for small scenes, else a 16-wave one plus, where it fits, a second launch of one 4-wave
 * workgroup per CU: 5 waves per SIMD); 4 ballot-batched on
 * a plain grid, scene through the caches; 5 the persistent workgroups with the breadth-first top
 * of a 4-wide tree in LDS and the rest through the caches; round 1's per-segment schedules 1 and 2
 * were retired in round 5 and return RTG_E_UNSUPPORTED),
 * bits 16-23 shade batch of schedule 0 in 64ths of the live lanes (0 = library default). */
#define RTG_RENDER_SCHEDULE(n) (((n) & 0xff) << 8)
#define RTG_RENDER_SHADE_BATCH(n) (((n) & 0xff) << 16)
#define RTG_RENDER_LEAF_BATCH(n) (((n) & 0x7f) << 24) /* bits 24-30: leaf batch in lanes (0 = default) */

/* rtg-f32 per-pixel accumulation (DESIGN.md §4 "sample chunks"): a pixel's samples are summed in
 * chunks of K = rtg_chunk_samples(spp) consecutive samples, each chunk in sample order starting from
 * zero, and the chunk sums are then added in chunk order; the pixel is pixel_samples_scale * that.
 * spp <= 16 gives one chunk, i.e. the reference's single running sum (camera.hpp:55-62). Chunks are
 * the device's unit of work, so one expensive pixel never holds a wavefront for all its samples, and
 * the last units of a frame (or of a 1/8 shard of one) end close together (ABI 4: 16, was 64). */
#define RTG_CHUNK_MAX 16
static inline int rtg_chunk_samples(int spp) {
  int n = (spp + RTG_CHUNK_MAX - 1) / RTG_CHUNK_MAX;
  if (n < 1) n = 1;
  return spp > 0 ? (spp + n - 1) / n : 1;
}

static inline int rtg_num_chunks(int spp) {
  int k = rtg_chunk_samples(spp);
  return spp > 0 ? (spp + k - 1) / k : 1;
}

typedef struct rtg_render_desc {
  uint64_t seed;      /* run seed of the counter RNG */
  int32_t row_begin;  /* first image row of this shard */
  int32_t row_stride; /* rows row_begin + k*row_stride, k < row_count (interleaved tiling) */
  int32_t row_count;  /* <= 0: every row reachable from row_begin with row_stride */
  int32_t flags;      /* RTG_RENDER_* */
  void* stream;       /* hipStream_t to launch on; NULL = the library's own stream */
  /* Progressive / checkpointable rendering. NULL partial: one-shot render (fields below unused).
   * Otherwise `partial` is a DEVICE buffer of rtg_num_chunks(spp) x rows x width x 3 floats holding
   * per-chunk partial sums (layout [chunk][row][column][rgb]); only chunks [chunk_begin,
   * chunk_begin + chunk_count) are rendered into it (chunk_count <= 0: through the last chunk),
   * the rest of the buffer is left alone, and out_rgb (may be NULL) receives the mean over the
   * samples of chunks [0, chunk_begin + chunk_count). Once every chunk has been rendered the
   * mean is bit-identical to a one-shot render; saving the buffer is a checkpoint. */
  float* partial;
  int32_t chunk_begin;
  int32_t chunk_count;
} rtg_render_desc;

typedef struct rtg_render_stats {
  uint64_t segments;   /* ray segments traced == world.hit() calls (camera.hpp:192) */
  uint64_t samples;    /* camera samples == rows*width*spp */
  uint64_t box_tests;  /* RTG_RENDER_COUNT only: child AABB tests */
  uint64_t prim_tests; /* RTG_RENDER_COUNT only: sphere/quad tests */
  uint64_t hits;       /* RTG_RENDER_COUNT only: segments that hit something */
  double kernel_ms;    /* device time of the render kernel (HIP events on the launch stream) */
  /* RTG_RENDER_COUNT only, wave-level schedule diagnostics (default schedule):
   * [0] traversal trips, [1] lanes stepping summed over trips, [2] lanes idle because their
   * pixel is finished summed over trips, [3] shading trips, [4] lanes shading summed over trips,
   * [5] / [6] shader-clock cycles spent in the traversal / shading phases (s_memtime, all waves),
   * [7] traversal trips that were leaf trips, [8] shader-clock cycles of the leaf trips,
   * [9] lanes that ran a node step summed over node trips, [10] lanes that ran a leaf step summed
   * over leaf trips; cycles of the shading phase split into [11] miss / material scatter,
   * [12] path end (sample restart or chunk store); cycles between shading and the next traversal:
   * [13] unit hand-out, [14] camera rays of fresh samples, [15] traversal setup (trav_begin and
   * the scene-spanning occluder test) */
  uint64_t diag[16];
  /* ABI 6: RTG_RENDER_COUNT only: traversal-stack pushes that went to the global spill area (entries past
   * the stack's LDS part; deep trees such as config 5's), each a 4-B store and, at the pop, a 4-B load */
  uint64_t stack_spills;
  /* round 6, layout-compatible (the first of ABI 6's reserved words): 1 when this render handed its tiles out in
   * the cost order rtg_scene_prepare tuned for its camera and shard (0: tile-major), and the host + probe time
   * of the scene's last tile-order tuning in microseconds */
  uint32_t tile_order;
  uint32_t tile_order_tune_us;
  uint64_t reserved_[2];
} rtg_render_stats;

typedef struct rtg_scene rtg_scene; /* opaque; owns the device copy of the scene */

typedef struct rtg_scene_info {
  int32_t device;
  int32_t bvh_mode;
  int64_t num_prims;
  int64_t num_nodes;
  int32_t bvh_depth;   /* longest root-to-leaf path in nodes */
  int32_t stack_depth; /* traversal stack entries the selected kernel provides */
  int64_t device_bytes;
  double build_ms; /* host BVH build + flatten */
  double upload_ms;
  /* phases of build_ms (ABI 5): binned-SAH build of the binary tree, its 4-wide collapse (+ the
   * breadth-first renumbering of the tree's top), and the rest (validation, primitive / node /
   * material / texture records) */
  double bvh_ms;
  double collapse_ms;
  double flatten_ms;
} rtg_scene_info;

/* Library identity. */
uint32_t rtg_abi_version(void);
const char* rtg_last_error(void);
rtg_status rtg_device_count(int32_t* count);

/* camera::initialize() on the host (camera.hpp:76-136). */
rtg_status rtg_camera_resolve(const rtg_camera_desc* cam, rtg_camera_params* out);

/* Scene lifetime. Host arrays are read during the call only; the scene owns device memory. */
rtg_status rtg_scene_create(const rtg_scene_desc* desc, int32_t device, rtg_scene** out);
rtg_status rtg_scene_get_info(const rtg_scene* scene, rtg_scene_info* out);
void rtg_scene_destroy(rtg_scene* scene);

/* Render rows of the image. out_rgb receives row_count*image_width*3 floats: the linear,
 * pre-gamma per-pixel mean  pixel_samples_scale * sum_s ray_color(...)  that the reference hands
 * to write_color (camera.hpp:65), rows in shard order. */
rtg_status rtg_render(rtg_scene* scene, const rtg_camera_desc* cam, const rtg_render_desc* job,
                      float* out_rgb, rtg_render_stats* stats);

/* Block until an RTG_RENDER_ASYNC render on `scene` finished; fills the deferred stats. */
rtg_status rtg_render_wait(rtg_scene* scene, rtg_render_stats* stats);

/* The launch plan rtg_render would use for (scene, cam, job), without rendering (ABI 5): which
 * kernel schedule, how many persistent workgroups of how many waves, the LDS each one requests,
 * and the compiled kernel's own resources (hipFuncGetAttributes of the code object that would run:
 * the real VGPR count, not a profiler's allocation granule). The bench record reports it beside the
 * roofline so the counted occupancy and the kernel that was timed are named by the library itself. */
typedef struct rtg_launch_plan {
  int32_t schedule;          /* 3 LDS-resident scene, 5 LDS treelet, 0 plain grid */
  int32_t workgroups;        /* main launch */
  int32_t waves_per_workgroup;
  int32_t lds_bytes;         /* dynamic LDS per workgroup of the main launch */
  int32_t vgprs;             /* VGPRs per lane of the main launch's kernel */
  int32_t sgprs;             /* SGPRs per wave (0 when the runtime does not report it) */
  int32_t scratch_bytes;     /* private (spill) bytes per lane */
  int32_t waves_per_simd;    /* resident waves per SIMD of the whole plan (main + dual) */
  int32_t dual;              /* 1: a second persistent launch of 4-wave workgroups shares the CUs */
  int32_t dual_workgroups;
  int32_t dual_lds_bytes;
  int32_t dual_vgprs;
  int32_t stack_entry_bytes; /* 2 or 4 */
  int32_t lds_stack_entries; /* traversal stack entries per lane in LDS (the rest spill to HBM) */
  int32_t spill_entries;     /* per lane, in the global spill area */
  int32_t treelet_nodes;     /* schedule 5: 4-wide nodes of the tree's top kept in LDS */
  int32_t shade_batch;       /* in 64ths of the live lanes */
  int32_t leaf_batch;        /* lanes */
  int32_t chunk_samples;     /* K of rtg_chunk_samples */
  int32_t chunks;
  int64_t partial_bytes;     /* device scratch of the chunk partial sums this render allocates */
  int32_t num_cus;
  int32_t tile_slots;        /* > 0: chunks are summed per tile through a ring of this many tile
                                slots (partial_bytes = ring + slot words); 0: full-frame partials */
  int32_t treelet_hot;       /* schedule 5: 1 when the node array is ordered for this camera (the
                                most-visited nodes are the treelet; rtg_scene_prepare), 0: not yet */
  int32_t treelet_tune_us;   /* host + probe time of the scene's last hot-treelet tuning */
  int32_t treelet_visit_permille; /* treelet_hot: of the probe's node visits, the share (per mille)
                                     that the treelet_nodes in LDS take */
  /* round 4, layout-compatible (two of ABI 5's reserved words): */
  int32_t ray_queue;         /* always 0 since round 5 (the RTG_RAY_QUEUE prototype was retired to
                                tools/experiments/ray_queue.patch); the word keeps the layout */
  int32_t node_width;        /* BVH node width the kernels traverse: 2 (RTG_BVH_MEDIAN) or 4 */
  /* round 5, layout-compatible (ABI 5's last reserved word): M of the conservative culling margin, rounded
     up: the node boxes are padded for ray origins with |coordinate| <= 2M; a render whose
     camera reaches farther raises it (and the padding) first */
  int32_t origin_bound;
} rtg_launch_plan;

rtg_status rtg_render_plan(rtg_scene* scene, const rtg_camera_desc* cam, const rtg_render_desc* job,
                           rtg_launch_plan* out);

/* Optional setup before the first render of a camera (and shard rows) on a scene (ABI 5 addition; the tile
 * order since round 6, layout-compatible).
 * Tile order (every default schedule, RTG_TILE_ORDER=1 default): a probe render of the camera and shard
 * (counting kernel, up to 4 samples per pixel, one counter per 64-pixel tile) measures each tile's traced
 * segments, and later renders of that camera and shard hand their tiles out most expensive first, so a
 * launch ends on cheap units instead of one late expensive tile (an 8-GPU shard's tail). Frames and
 * segment counts are unchanged: only which wave renders a unit, and when, changes. rtg_render_stats.tile_order
 * says whether a render used it; renders of other cameras or shards (and the tile-ring kernels) keep the
 * tile-major order.
 * Scenes whose BVH does not fit LDS render with the treelet schedule, which keeps a prefix of the
 * 4-wide node array in each workgroup's LDS; here a probe render (1 sample per pixel on about 2^19
 * pixels, every k-th row of the shard; counting kernel) counts every node's visits for this camera and the node array
 * is renumbered so the most-visited nodes form that prefix (the "hot treelet"; the root stays first).
 * Traversal order and frames are unchanged: only where a node is read from changes. rtg_render does
 * the same on the scene's first treelet render only (later cameras keep the tuned order until this is
 * called for them: a moving camera pays no probe and node re-upload inside its frames); calling this
 * first keeps the probe (~0.13 s for 1M spheres at 4K) out of that render. A no-op for every other
 * schedule and with RTG_TREELET_HOT=0.
 * Not concurrent with renders of the same scene (it rewrites the scene's node array and tile order). No reference
 * counterpart: the reference's bvh_node keeps its nodes in host memory (bvh_node.hpp:25-77). */
rtg_status rtg_scene_prepare(rtg_scene* scene, const rtg_camera_desc* cam, const rtg_render_desc* job);

/* Host twin of the hot treelet's renumbering (tests; no device): num_nodes 4-wide nodes in the device
 * record format (112 B each: 24 plane floats, then 4 int32 child codes; inner child = byte offset of
 * its node, leaf < 0, empty INT32_MIN), renumbered in place so node 0 stays first and the others
 * follow by descending visits[old index] (ties keep their order), inner codes remapped. */
rtg_status rtg_hot_treelet_order_host(int32_t* nodes, const uint32_t* visits, int64_t num_nodes);

/* write_color (color.hpp:26-58) on the device: gamma 2, clamp [0, 0.999], int(256*x).
 * in_rgb / out_rgb8 are device pointers on the scene's device; n_pixels pixels. */
rtg_status rtg_resolve_rgb8(rtg_scene* scene, const float* in_rgb, uint8_t* out_rgb8,
                            int64_t n_pixels, void* stream);

/* ---- multi-GPU frames: row-interleaved shards, one RCCL gather over xGMI ----
 * Replaces the reference's single-device pixel loop of camera::render (camera.hpp:29-72) when the
 * image is tiled over several GPUs: rank r renders rows r, r+N, r+2N, ... (any N gives the same
 * image: the RNG is keyed by the global pixel), every shard is padded to ceil(H/N) rows, and the
 * root receives them with one ncclGather, then de-interleaves them on its device.
 * A communicator spans N ranks; a process holds one of them (one process per GPU, ids shared out
 * of band) or all of them (one process driving every local GPU, ncclCommInitAll). */
typedef struct rtg_comm rtg_comm;
#define RTG_COMM_ID_BYTES 128

/* One process, `ndev` local devices: ranks 0..ndev-1 are devices[0..ndev-1]. */
rtg_status rtg_comm_create_local(const int32_t* devices, int32_t ndev, rtg_comm** out);
/* One process per device: rank 0 calls rtg_comm_unique_id and hands the bytes to every rank. */
rtg_status rtg_comm_unique_id(uint8_t id[RTG_COMM_ID_BYTES]);
rtg_status rtg_comm_create_rank(const uint8_t id[RTG_COMM_ID_BYTES], int32_t nranks, int32_t rank,
                                int32_t device, rtg_comm** out);
/* nranks: ranks of the communicator as RCCL counts them (ncclCommCount); nlocal: ranks this
 * process drives. */
rtg_status rtg_comm_size(const rtg_comm* comm, int32_t* nranks, int32_t* nlocal);
void rtg_comm_destroy(rtg_comm* comm);

/* Host-only: the interleaved shard of `rank` in an image of `height` rows tiled over `nranks`
 * (the arithmetic rtg_render_frame and rtg_gather_rows use): rows row_begin + k*row_stride,
 * k < row_count (0 for a rank past the last row), every shard padded to padded_rows =
 * ceil(height/nranks) rows, so rank r's block starts at byte r*padded_rows*row_bytes of the root's
 * staging buffer. Any output pointer may be NULL. */
rtg_status rtg_shard_layout(int32_t height, int32_t nranks, int32_t rank, int32_t* row_begin,
                            int32_t* row_stride, int32_t* row_count, int32_t* padded_rows);

/* Gather the interleaved shards of a `height`-row image of `row_bytes`-byte rows onto rank
 * `root`. shards[i] (device memory of the i-th local rank) holds ceil(height/nranks) rows:
 * image rows rank, rank+nranks, ... then padding. out: device memory on root's device, height
 * rows in image order (ignored by processes without the root). streams[i] (hipStream_t, may be
 * NULL = the communicator's own) orders the gather after the render that filled shards[i].
 * Asynchronous: returns once enqueued (every local rank's part, one RCCL group). The root's staging
 * buffer belongs to the communicator, grown on demand and kept (ABI 7: steady-state gathers allocate
 * nothing); a gather on another stream than the previous one first waits for that one's
 * de-interleave, so gathers in flight on two streams take turns at it. Calls that use a communicator
 * from several host threads at once are not supported (RCCL groups are per thread). */
rtg_status rtg_gather_rows(rtg_comm* comm, const void* const* shards, int32_t height, int64_t row_bytes,
                           int32_t root, void* out, void* const* streams);

/* Host twin of the de-interleave step (same index function as the device kernel): `gathered`
 * holds nranks blocks of ceil(height/nranks) rows in host memory; `out` receives height rows in
 * image order. For CPU-side gathers (gloo) and for testing the layout without a GPU. */
rtg_status rtg_deinterleave_rows_host(const void* gathered, void* out, int32_t nranks, int32_t height,
                                      int64_t row_bytes);

/* The de-interleave step of rtg_gather_rows on its own: `gathered` holds nranks blocks of
 * ceil(height/nranks) rows (block r = rank r's shard); writes image row r + k*nranks from row k of
 * block r. Device memory on `device`; asynchronous on `stream`. */
rtg_status rtg_deinterleave_rows(int32_t device, const void* gathered, void* out, int32_t nranks,
                                 int32_t height, int64_t row_bytes, void* stream);

/* A whole multi-GPU frame for the C++ mirror's camera (camera.devices): scenes[i] is the scene on
 * the i-th local rank's device; each renders its interleaved rows into device memory, the frame is
 * gathered to `root` over RCCL and copied to out_rgb (host, H*W*3 floats, on the root's process).
 * stats: segments / samples summed over the local ranks, kernel_ms the slowest rank's. */
rtg_status rtg_render_frame(rtg_comm* comm, rtg_scene* const* scenes, const rtg_camera_desc* cam,
                            uint64_t seed, int32_t root, float* out_rgb, rtg_render_stats* stats);

/* Host-only: build the BVH the scene would use and report its topology (no GPU needed).
 * nodes_out (optional, capacity max_nodes) receives per node: {left, right} child codes
 * (>= 0 node index, < 0 leaf = -(1 + first_ref), leaf prim refs in refs_out) in DFS order
 * plus the node's child boxes; returns counts in *num_nodes / *num_refs / *depth. */
typedef struct rtg_bvh_node_host {
  double lo[2][3]; /* child boxes (left, right) */
  double hi[2][3];
  int32_t child[2]; /* >= 0: node index; < 0: leaf -(1+first ref); INT32_MIN: empty */
  int32_t count[2]; /* primitives in a leaf child */
} rtg_bvh_node_host;

rtg_status rtg_bvh_build_host(const rtg_scene_desc* desc, rtg_bvh_node_host* nodes_out,
                              int64_t max_nodes, int64_t* refs_out, int64_t max_refs,
                              int64_t* num_nodes, int64_t* num_refs, int32_t* depth);

/* ABI 7: device and pinned-host allocations librtgpu made in this process so far (count, bytes). Scene
 * creation allocates; a render, rtg_gather_rows and rtg_render_frame allocate only while their
 * grow-only buffers (the scene's render scratch and output, the communicator's shards, frame and
 * staging) reach a frame's sizes, nothing per frame after that. Either pointer may be NULL. */
rtg_status rtg_allocation_count(uint64_t* count, uint64_t* bytes);

/* Host-only (ABI 7): the order in which bvh_node(objects, 0, n) (bvh_node.hpp:25-77) leaves `objects`
 * — its leaves left to right, the order bvh_node::hit (bvh_node.hpp:80-94) tests them in. boxes holds
 * each object's bounding_box() as {lo.x, lo.y, lo.z, hi.x, hi.y, hi.z} (n x 6 doubles, list order);
 * order receives n list indices. The reference's own steps: range box, aabb::longest_axis, std::sort
 * by box min on that axis (libstdc++'s, so objects with equal keys land where the reference's land),
 * median split, no sort for spans of 1 or 2. Replaces nothing on the device path: the C++ mirror's
 * bvh_node uses it to fill rtg_scene_desc.tie_rank. */
rtg_status rtg_bvh_node_order(const double* boxes, int64_t n, int64_t* order);

#ifdef __cplusplus
}
#endif
#endif /* RTGPU_H */
