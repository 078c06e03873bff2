/*
 * oracle/cpu_ref.c — TEST INFRASTRUCTURE ONLY. A CPU restatement of the reference's per-pixel
 * sample loop, used exclusively by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * as the checker / the timed CPU baseline. It is never linked into, called by, or a fallback of
 * the product library (raytracing-practice_amd/lib/librtgpu.so).
 *
 * Two renderers, both written from the reference's algorithm (file:line cited per function):
 *
 *  orc_render_f64  ("cpu_ref64")  fp64, recursive ray_color, reference BVH traversal (unordered,
 *                  left then right), the reference's sphere/quad formulas, and the reference's RNG:
 *                  glibc random() (= rand(), rtweekend.hpp:23-27) consumed sequentially in
 *                  scanline -> pixel -> sample -> bounce order, with GCC's right-to-left argument
 *                  evaluation order (hazard H2). Pinned against the reference compiled from
 *                  /root/reference (oracle/ref_harness.cpp): identical framebuffer doubles.
 *
 *  orc_render_f32  ("cpu_ref32")  the fp32 spec the GPU implements (DESIGN.md "rtg-f32"):
 *                  counter RNG keyed by (seed, pixel, sample), iterative throughput form (H12),
 *                  robust sphere / quad roots, the plane offset and a large sphere's (|r| >= 16)
 *                  |oc|^2 - r^2 formed in f64. This is
 *                  the per-pixel parity target of the HIP kernels (same seeds => same pixels).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, so expressions round as written).
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/rtgpu.h"

#define ORC_PI 3.1415926535897932385

/* ------------------------------------------------------------------------------------------ */
/* fp64 vec3 (vec3.hpp:8-226)                                                                  */
typedef struct {
  double x, y, z;
} d3;
static inline d3 D3(double x, double y, double z) {
  d3 r = {x, y, z};
  return r;
}
static inline d3 dadd(d3 a, d3 b) { return D3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline d3 dsub(d3 a, d3 b) { return D3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline d3 dmul(d3 a, d3 b) { return D3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline d3 dscl(double t, d3 a) { return D3(t * a.x, t * a.y, t * a.z); }
static inline d3 ddiv(d3 a, double t) { return dscl(1 / t, a); } /* operator/ = (1/t)*v */
static inline d3 dneg(d3 a) { return D3(-a.x, -a.y, -a.z); }
static inline double ddot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline d3 dcross(d3 a, d3 b) {
  return D3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline double dlen(d3 a) { return sqrt(ddot(a, a)); }
static inline d3 dunit(d3 a) { return ddiv(a, dlen(a)); }
static inline d3 dv(const double v[3]) { return D3(v[0], v[1], v[2]); }

/* ------------------------------------------------------------------------------------------ */
/* camera::initialize (camera.hpp:76-136)                                                      */
int orc_camera_resolve(const rtg_camera_desc* c, rtg_camera_params* o) {
  int W = c->image_width;
  int H = (int)(W / c->aspect_ratio);
  if (H < 1) H = 1;
  o->image_width = W;
  o->image_height = H;
  o->pixel_samples_scale = (double)(1.0f / c->samples_per_pixel);
  double theta = c->vfov * ORC_PI / 180.0f; /* degrees_to_radians, rtweekend.hpp:17-20 */
  double h = tan(theta / 2);
  double vh = 2 * h * c->focus_dist;
  double vw = vh * ((double)W / H);
  d3 center = dv(c->lookfrom);
  d3 w = dunit(dsub(dv(c->lookfrom), dv(c->lookat)));
  d3 u = dunit(dcross(dv(c->vup), w));
  d3 v = dcross(w, u);
  d3 vu = dscl(vw, u);
  d3 vv = dscl(vh, dneg(v));
  d3 du = ddiv(vu, W);
  d3 dvv = ddiv(vv, H);
  d3 ul = dsub(dsub(dsub(center, dscl(c->focus_dist, w)), ddiv(vu, 2)), ddiv(vv, 2));
  d3 p00 = dadd(ul, dscl(0.5, dadd(du, dvv)));
  double rad = c->focus_dist * tan(c->defocus_angle * ORC_PI / 180.0f / 2.0f);
  d3 du_ = dscl(rad, u), dv_ = dscl(rad, v);
  memcpy(o->center, &center, 24);
  memcpy(o->pixel00_loc, &p00, 24);
  memcpy(o->pixel_delta_u, &du, 24);
  memcpy(o->pixel_delta_v, &dvv, 24);
  memcpy(o->u, &u, 24);
  memcpy(o->v, &v, 24);
  memcpy(o->w, &w, 24);
  memcpy(o->defocus_disk_u, &du_, 24);
  memcpy(o->defocus_disk_v, &dv_, 24);
  return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* aabb and the reference BVH (aabb.hpp, bvh_node.hpp:25-94)                                   */
typedef struct {
  double lo[3], hi[3];
} obox;

static void pad_box(obox* b) { /* aabb::pad_to_minimums, aabb.hpp:135-154 */
  for (int a = 0; a < 3; ++a) {
    if (b->hi[a] - b->lo[a] < 0.0001) {
      double pad = 0.0001 / 2.0f;
      b->lo[a] -= pad;
      b->hi[a] += pad;
    }
  }
}
static obox box_pts(d3 a, d3 b) { /* aabb(point, point), aabb.hpp:30-39 */
  obox r;
  double A[3] = {a.x, a.y, a.z}, B[3] = {b.x, b.y, b.z};
  for (int k = 0; k < 3; ++k) {
    r.lo[k] = A[k] <= B[k] ? A[k] : B[k];
    r.hi[k] = A[k] <= B[k] ? B[k] : A[k];
  }
  pad_box(&r);
  return r;
}
static obox box_join(obox a, obox b) { /* aabb(box0, box1), aabb.hpp:42-48 */
  obox r;
  for (int k = 0; k < 3; ++k) {
    r.lo[k] = a.lo[k] <= b.lo[k] ? a.lo[k] : b.lo[k];
    r.hi[k] = a.hi[k] >= b.hi[k] ? a.hi[k] : b.hi[k];
  }
  return r;
}
static obox box_empty(void) {
  obox r;
  for (int k = 0; k < 3; ++k) {
    r.lo[k] = INFINITY;
    r.hi[k] = -INFINITY;
  }
  return r;
}
static obox prim_box(const rtg_primitive* p) {
  if (p->kind == RTG_PRIM_SPHERE) { /* sphere.hpp:16-44 */
    d3 rv = D3(p->radius, p->radius, p->radius);
    d3 c0 = dv(p->p0), c1 = dv(p->p1);
    if (c0.x == c1.x && c0.y == c1.y && c0.z == c1.z) return box_pts(dsub(c0, rv), dadd(c0, rv));
    d3 dir = dsub(c1, c0);
    d3 a0 = dadd(c0, dscl(0.0, dir)), a1 = dadd(c0, dscl(1.0, dir));
    return box_join(box_pts(dsub(a0, rv), dadd(a0, rv)), box_pts(dsub(a1, rv), dadd(a1, rv)));
  }
  d3 Q = dv(p->p0), u = dv(p->p1), v = dv(p->p2); /* quad.hpp:30-38 */
  return box_join(box_pts(Q, dadd(dadd(Q, u), v)), box_pts(dadd(Q, u), dadd(Q, v)));
}

/* node child code: >= 0 node, < 0 primitive -(1+id) */
typedef struct {
  obox box;
  int32_t left, right;
} onode;
typedef struct {
  onode* nodes;
  int64_t n;
  int64_t cap;
} obvh;

typedef struct {
  const obox* boxes;
  int axis;
} sort_ctx;
static __thread sort_ctx g_sort;
static int cmp_min(const void* a, const void* b) {
  double ka = g_sort.boxes[*(const int64_t*)a].lo[g_sort.axis];
  double kb = g_sort.boxes[*(const int64_t*)b].lo[g_sort.axis];
  return (ka < kb) ? -1 : (kb < ka ? 1 : 0);
}
static int longest(obox b) { /* aabb::longest_axis, aabb.hpp:116-127 */
  double sx = b.hi[0] - b.lo[0], sy = b.hi[1] - b.lo[1], sz = b.hi[2] - b.lo[2];
  if (sx > sy) return sx > sz ? 0 : 2;
  return sy > sz ? 1 : 2;
}
static int32_t build_median(obvh* t, const obox* boxes, int64_t* ids, int64_t start, int64_t end) {
  if (t->n == t->cap) {
    t->cap = t->cap ? t->cap * 2 : 64;
    t->nodes = (onode*)realloc(t->nodes, sizeof(onode) * t->cap);
  }
  int32_t me = (int32_t)t->n++;
  obox b = box_empty();
  for (int64_t i = start; i < end; ++i) b = box_join(b, boxes[ids[i]]);
  int axis = longest(b);
  int64_t span = end - start;
  int32_t l, r;
  if (span == 1) {
    l = r = (int32_t)(-1 - ids[start]); /* left = right = object (H8, tested twice) */
  } else if (span == 2) {
    l = (int32_t)(-1 - ids[start]);
    r = (int32_t)(-1 - ids[start + 1]);
  } else {
    g_sort.boxes = boxes;
    g_sort.axis = axis;
    qsort(ids + start, (size_t)span, sizeof(int64_t), cmp_min);
    int64_t mid = start + span / 2;
    l = build_median(t, boxes, ids, start, mid);
    r = build_median(t, boxes, ids, mid, end);
  }
  t->nodes[me].box = b;
  t->nodes[me].left = l;
  t->nodes[me].right = r;
  return me;
}
static void bvh_build(obvh* t, const rtg_scene_desc* s) {
  memset(t, 0, sizeof(*t));
  if (s->num_prims <= 0) return;
  obox* boxes = (obox*)malloc(sizeof(obox) * s->num_prims);
  int64_t* ids = (int64_t*)malloc(sizeof(int64_t) * s->num_prims);
  for (int64_t i = 0; i < s->num_prims; ++i) {
    boxes[i] = prim_box(&s->prims[i]);
    ids[i] = i;
  }
  build_median(t, boxes, ids, 0, s->num_prims);
  free(boxes);
  free(ids);
}

/* aabb::hit (aabb.hpp:61-112) on a double ray */
static inline int box_hit(const obox* b, const double o[3], const double d[3], double tmin,
                          double tmax) {
  for (int a = 0; a < 3; ++a) {
    const double adinv = 1.0f / d[a];
    double t0 = (b->lo[a] - o[a]) * adinv;
    double t1 = (b->hi[a] - o[a]) * adinv;
    if (t0 < t1) {
      if (t0 > tmin) tmin = t0;
      if (t1 < tmax) tmax = t1;
    } else {
      if (t1 > tmin) tmin = t1;
      if (t0 < tmax) tmax = t0;
    }
    if (tmax <= tmin) return 0;
  }
  return 1;
}

/* ------------------------------------------------------------------------------------------ */
/* glibc random() stream: rand() == random() (TYPE_3 additive feedback); srand == srandom.     */
typedef struct {
  struct random_data rd;
  char state[128];
} glibc_rng;
static void grng_seed(glibc_rng* g, unsigned seed) {
  memset(g, 0, sizeof(*g));
  initstate_r(seed, g->state, sizeof(g->state), &g->rd);
}
static inline double grand(glibc_rng* g) { /* random_double(), rtweekend.hpp:23-27 */
  int32_t r;
  random_r(&g->rd, &r);
  return (double)((float)r / (2147483647 + 1.0f));
}
static inline double grand_mm(glibc_rng* g, double mn, double mx) { /* rtweekend.hpp:29-33 */
  return mn + (mx - mn) * grand(g);
}

/* exported for KATs: k-th random_double() of the stream seeded with `seed` */
double orc_glibc_random_double(unsigned seed, int k) {
  glibc_rng g;
  grng_seed(&g, seed);
  double v = 0;
  for (int i = 0; i <= k; ++i) v = grand(&g);
  return v;
}

/* random_unit_vector (vec3.hpp:172-184): vec3::random(-1,1) evaluated z, y, x under GCC (H2) */
static d3 f64_random_unit_vector(glibc_rng* g) {
  while (1) {
    double z = grand_mm(g, -1, 1);
    double y = grand_mm(g, -1, 1);
    double x = grand_mm(g, -1, 1);
    d3 p = D3(x, y, z);
    double lensq = ddot(p, p);
    if (1e-160 < lensq && lensq <= 1) return ddiv(p, sqrt(lensq));
  }
}

/* ------------------------------------------------------------------------------------------ */
/* fp64 world (reference formulas)                                                             */
typedef struct {
  d3 p, normal;
  double t, u, v;
  int front;
  int32_t mat;
} hrec64;

typedef struct {
  const rtg_scene_desc* s;
  obvh bvh;
  /* quad derived data, quad ctor (quad.hpp:12-27) */
  d3* qn;
  double* qD;
  d3* qw;
} world64;

static int sphere_hit64(const rtg_primitive* p, const d3 o, const d3 d, double time, double tmin,
                        double tmax, hrec64* rec) { /* sphere.hpp:47-93 */
  d3 c0 = dv(p->p0), dir = dsub(dv(p->p1), c0);
  d3 C = dadd(c0, dscl(time, dir));
  d3 oc = dsub(o, C);
  double a = ddot(d, d);
  double hb = ddot(oc, d);
  double c = ddot(oc, oc) - p->radius * p->radius;
  double disc = hb * hb - a * c;
  if (disc < 0) return 0;
  double sq = sqrt(disc);
  double root = (-hb - sq) / a;
  if (!(tmin < root && root < tmax)) {
    root = (-hb + sq) / a;
    if (!(tmin < root && root < tmax)) return 0;
  }
  rec->t = root;
  rec->p = dadd(o, dscl(root, d));
  d3 out = ddiv(dsub(rec->p, C), p->radius);
  rec->front = ddot(d, out) < 0;
  rec->normal = rec->front ? out : dneg(out);
  double theta = acos(-out.y); /* get_sphere_uv, sphere.hpp:100-111 */
  double phi = atan2(-out.z, out.x) + ORC_PI;
  rec->u = phi / (2.0f * ORC_PI);
  rec->v = theta / ORC_PI;
  rec->mat = p->material;
  return 1;
}

static int quad_hit64(const world64* w, int64_t id, const d3 o, const d3 d, double tmin, double tmax,
                      hrec64* rec) { /* quad.hpp:44-114 */
  const rtg_primitive* p = &w->s->prims[id];
  d3 n = w->qn[id];
  double denom = ddot(n, d);
  if (fabs(denom) < 1e-8) return 0;
  double t = (w->qD[id] - ddot(n, o)) / denom;
  if (!(tmin <= t && t <= tmax)) return 0;
  d3 P = dadd(o, dscl(t, d));
  d3 hp = dsub(P, dv(p->p0));
  double alpha = ddot(w->qw[id], dcross(hp, dv(p->p2)));
  double beta = ddot(w->qw[id], dcross(dv(p->p1), hp));
  if (!(0.0f <= alpha && alpha <= 1.0f) || !(0.0f <= beta && beta <= 1.0f)) return 0;
  rec->u = alpha;
  rec->v = beta;
  rec->t = t;
  rec->p = P;
  rec->mat = p->material;
  rec->front = ddot(d, n) < 0;
  rec->normal = rec->front ? n : dneg(n);
  return 1;
}

static int prim_hit64(const world64* w, int64_t id, d3 o, d3 d, double time, double tmin,
                      double tmax, hrec64* rec) {
  if (w->s->prims[id].kind == RTG_PRIM_SPHERE)
    return sphere_hit64(&w->s->prims[id], o, d, time, tmin, tmax, rec);
  return quad_hit64(w, id, o, d, tmin, tmax, rec);
}

/* bvh_node::hit (bvh_node.hpp:80-94): own box, then left, then right with t_max = rec.t */
static int node_hit64(const world64* w, int32_t code, d3 o, d3 d, const double O[3],
                      const double Dd[3], double time, double tmin, double tmax, hrec64* rec) {
  if (code < 0) return prim_hit64(w, -1 - (int64_t)code, o, d, time, tmin, tmax, rec);
  const onode* n = &w->bvh.nodes[code];
  if (!box_hit(&n->box, O, Dd, tmin, tmax)) return 0;
  int hl = node_hit64(w, n->left, o, d, O, Dd, time, tmin, tmax, rec);
  int hr = node_hit64(w, n->right, o, d, O, Dd, time, tmin, hl ? rec->t : tmax, rec);
  return hl || hr;
}

static int world_hit64(const world64* w, d3 o, d3 d, double time, hrec64* rec) {
  if (w->bvh.n == 0) return 0;
  const double O[3] = {o.x, o.y, o.z}, Dd[3] = {d.x, d.y, d.z};
  hrec64 tmp;
  int hit = node_hit64(w, 0, o, d, O, Dd, time, 0.001, INFINITY, &tmp); /* camera.hpp:192 */
  if (hit) *rec = tmp;
  return hit;
}

static double perlin_turb_scalar64(const rtg_perlin* pl, d3 p);

static d3 tex_value64(const rtg_scene_desc* s, int32_t t, double u, double v, d3 p) {
  for (int guard = 0; guard < 16; ++guard) {
    const rtg_texture* tx = &s->textures[t];
    if (tx->type == RTG_TEX_SOLID) return dv(tx->color);
    if (tx->type == RTG_TEX_CHECKER) { /* texture.hpp:57-79 */
      double inv = 1.0f / tx->scale;
      int xi = (int)floor(inv * p.x), yi = (int)floor(inv * p.y), zi = (int)floor(inv * p.z);
      t = ((xi + yi + zi) % 2 == 0) ? tx->even : tx->odd;
      continue;
    }
    if (tx->type == RTG_TEX_IMAGE) { /* texture.hpp:97-118, rtw_stb_image.hpp:104-134 */
      const rtg_image* im = (tx->image >= 0 && tx->image < s->num_images) ? &s->images[tx->image] : 0;
      if (!im || !im->rgb || im->height <= 0) return D3(0, 1, 1);
      u = u < 0 ? 0 : (u > 1 ? 1 : u);
      v = 1.0f - (v < 0 ? 0 : (v > 1 ? 1 : v));
      int i = (int)(u * im->width), j = (int)(v * im->height);
      i = i < 0 ? 0 : (i < im->width ? i : im->width - 1);
      j = j < 0 ? 0 : (j < im->height ? j : im->height - 1);
      const uint8_t* px = im->rgb + ((int64_t)j * im->width + i) * 3;
      float cs = 1.0f / 255.0f;
      return D3(cs * px[0], cs * px[1], cs * px[2]);
    }
    if (tx->type == RTG_TEX_NOISE) { /* noise_texture::value, texture.hpp:133-151 */
      double sv = 1.0f + sin(tx->scale * p.z + 10.0f * perlin_turb_scalar64(&s->perlins[tx->perlin], p));
      return dscl(sv, D3(0.5f, 0.5f, 0.5f));
    }
    break;
  }
  return D3(1, 0, 1);
}

/* perlin::noise_perlin + perlin_interp (perlin.hpp:95-132, 219-255): double math, float accum */
static double perlin_noise64(const rtg_perlin* pl, d3 p) {
  double u = p.x - floor(p.x), v = p.y - floor(p.y), w = p.z - floor(p.z);
  int i = (int)floor(p.x), j = (int)floor(p.y), k = (int)floor(p.z);
  double uu = u * u * (3 - 2 * u), vv = v * v * (3 - 2 * v), ww = w * w * (3 - 2 * w);
  float accum = 0.0f;
  for (int di = 0; di < 2; di++)
    for (int dj = 0; dj < 2; dj++)
      for (int dk = 0; dk < 2; dk++) {
        int idx = pl->perm_x[(i + di) & 255] ^ pl->perm_y[(j + dj) & 255] ^ pl->perm_z[(k + dk) & 255];
        d3 c = dv(pl->randvec[idx]);
        d3 wv = D3(u - di, v - dj, w - dk);
        accum += (di * uu + (1 - di) * (1 - uu)) * (dj * vv + (1 - dj) * (1 - vv)) *
                 (dk * ww + (1 - dk) * (1 - ww)) * ddot(c, wv);
      }
  return accum;
}
static double perlin_turb_scalar64(const rtg_perlin* pl, d3 p) { /* perlin.hpp:135-158 */
  float accum = 0.0f;
  d3 tp = p;
  float weight = 1.0f;
  for (int i = 0; i < 7; i++) {
    accum += weight * perlin_noise64(pl, tp);
    weight *= 0.5f;
    tp = dscl(2.0f, tp);
  }
  return fabsf(accum);
}
double orc_perlin_noise64(const rtg_perlin* pl, const double p[3]) { return perlin_noise64(pl, dv(p)); }
double orc_perlin_turb64(const rtg_perlin* pl, const double p[3]) {
  return perlin_turb_scalar64(pl, dv(p));
}
typedef struct {
  const world64* w;
  const rtg_camera_desc* cam;
  rtg_camera_params cp;
  d3 bg;
  glibc_rng* g;
  uint64_t segments;
} ctx64;

static d3 texture64(ctx64* c, int32_t tex, const hrec64* rec) {
  return tex_value64(c->w->s, tex, rec->u, rec->v, rec->p);
}

/* camera::ray_color (camera.hpp:180-232), recursive */
static d3 ray_color64(ctx64* c, d3 o, d3 d, double time, int depth) {
  if (depth <= 0) return D3(0, 0, 0);
  hrec64 rec;
  c->segments++;
  if (!world_hit64(c->w, o, d, time, &rec)) return c->bg;
  const rtg_material* m = &c->w->s->materials[rec.mat];
  d3 emit = D3(0, 0, 0);
  if (m->type == RTG_MAT_DIFFUSE_LIGHT) {
    emit = texture64(c, m->texture, &rec);
    return emit;
  }
  d3 att, dir;
  if (m->type == RTG_MAT_LAMBERTIAN) { /* material.hpp:51-71 */
    dir = dadd(rec.normal, f64_random_unit_vector(c->g));
    const double s = 1e-8; /* near_zero, vec3.hpp:70-77 (H5) */
    if (fabs(dir.x) < s && fabs((double)(dir.y < s)) && fabs(dir.z) < s) dir = rec.normal;
    att = texture64(c, m->texture, &rec);
  } else if (m->type == RTG_MAT_METAL) { /* material.hpp:86-106 */
    double fuzz = m->fuzz < 1.0f ? m->fuzz : 1.0f;
    d3 refl = dsub(d, dscl(2.0f * ddot(d, rec.normal), rec.normal));
    d3 r = f64_random_unit_vector(c->g);
    dir = dadd(dunit(refl), dscl(fuzz, r));
    att = dv(m->albedo);
    if (!(ddot(dir, rec.normal) > 0)) return emit;
  } else if (m->type == RTG_MAT_DIELECTRIC) { /* material.hpp:128-206 */
    att = D3(1.0f, 1.0f, 1.0f);
    double ri = rec.front ? (1.0f / m->refraction_index) : m->refraction_index;
    d3 ud = dunit(d);
    double ct = fmin(ddot(dneg(ud), rec.normal), 1.0f);
    double st = sqrt(1.0f - ct * ct);
    int cannot = ri * st > 1.0f;
    int reflect = cannot;
    if (!cannot) {
      double r0 = (1.0f - ri) / (1.0f + ri);
      r0 = r0 * r0;
      double refl = r0 + (1.0f - r0) * pow((1.0f - ct), 5);
      reflect = refl > grand(c->g);
    }
    if (reflect) {
      dir = dsub(ud, dscl(2.0f * ddot(ud, rec.normal), rec.normal));
    } else { /* refract, vec3.hpp:216-226 */
      double c2 = fmin(ddot(dneg(ud), rec.normal), 1.0f);
      d3 perp = dscl(ri, dadd(ud, dscl(c2, rec.normal)));
      d3 par = dscl(-sqrt(fabs(1.0f - ddot(perp, perp))), rec.normal);
      dir = dadd(perp, par);
    }
  } else {
    return emit;
  }
  d3 next = ray_color64(c, rec.p, dir, time, depth - 1);
  return dadd(emit, dmul(att, next));
}

static void world64_init(world64* w, const rtg_scene_desc* s) {
  memset(w, 0, sizeof(*w));
  w->s = s;
  bvh_build(&w->bvh, s);
  int64_t n = s->num_prims > 0 ? s->num_prims : 1;
  w->qn = (d3*)calloc(n, sizeof(d3));
  w->qD = (double*)calloc(n, sizeof(double));
  w->qw = (d3*)calloc(n, sizeof(d3));
  for (int64_t i = 0; i < s->num_prims; ++i) {
    const rtg_primitive* p = &s->prims[i];
    if (p->kind != RTG_PRIM_QUAD) continue;
    d3 nn = dcross(dv(p->p1), dv(p->p2));
    w->qn[i] = dunit(nn);
    w->qD[i] = ddot(w->qn[i], dv(p->p0));
    w->qw[i] = ddiv(nn, ddot(nn, nn));
  }
}
static void world64_free(world64* w) {
  free(w->bvh.nodes);
  free(w->qn);
  free(w->qD);
  free(w->qw);
}

/* camera::render loop for rows [row_begin, row_begin+row_count) with one sequential stream */
static void render64_rows(ctx64* c, int row_begin, int row_count, double* out) {
  const rtg_camera_params* cp = &c->cp;
  d3 p00 = dv(cp->pixel00_loc), du = dv(cp->pixel_delta_u), dvv = dv(cp->pixel_delta_v);
  d3 center = dv(cp->center), ddu = dv(cp->defocus_disk_u), ddv = dv(cp->defocus_disk_v);
  for (int jj = 0; jj < row_count; ++jj) {
    int j = row_begin + jj;
    for (int i = 0; i < cp->image_width; ++i) {
      d3 pix = D3(0, 0, 0);
      for (int s = 0; s < c->cam->samples_per_pixel; ++s) {
        /* get_ray (camera.hpp:139-177); sample_square draws y then x under GCC (H2) */
        double oy = grand(c->g) - 0.5f;
        double ox = grand(c->g) - 0.5f;
        d3 ps = dadd(dadd(p00, dscl(i + ox, du)), dscl(j + oy, dvv));
        d3 origin = center;
        if (!(c->cam->defocus_angle <= 0.0f)) {
          double px, py;
          while (1) { /* random_in_unit_disk, vec3.hpp:158-169: y then x */
            py = grand_mm(c->g, -1.0f, 1.0f);
            px = grand_mm(c->g, -1.0f, 1.0f);
            if (px * px + py * py + 0.0 * 0.0 < 1.0f) break;
          }
          origin = dadd(dadd(center, dscl(px, ddu)), dscl(py, ddv));
        }
        d3 dir = dsub(ps, origin);
        double time = grand(c->g);
        pix = dadd(pix, ray_color64(c, origin, dir, time, c->cam->max_depth));
      }
      double* o = out + ((int64_t)jj * cp->image_width + i) * 3;
      o[0] = cp->pixel_samples_scale * pix.x;
      o[1] = cp->pixel_samples_scale * pix.y;
      o[2] = cp->pixel_samples_scale * pix.z;
    }
  }
}

/* Reference render (cpu_ref64). seed: glibc srandom seed (1 == the reference's unseeded rand()).
 * out: row_count * W * 3 doubles = pixel_samples_scale * pixel_color (input of write_color). */
int orc_render_f64(const rtg_scene_desc* s, const rtg_camera_desc* cam, unsigned seed, int row_begin,
                   int row_count, double* out, uint64_t* segments) {
  world64 w;
  world64_init(&w, s);
  glibc_rng g;
  grng_seed(&g, seed);
  ctx64 c;
  memset(&c, 0, sizeof(c));
  c.w = &w;
  c.cam = cam;
  orc_camera_resolve(cam, &c.cp);
  c.bg = dv(cam->background);
  c.g = &g;
  if (row_count <= 0) row_count = c.cp.image_height - row_begin;
  render64_rows(&c, row_begin, row_count, out);
  if (segments) *segments = c.segments;
  world64_free(&w);
  return 0;
}

/* Multi-threaded timing of cpu_ref64: `threads` workers, each renders rows of the image with its
 * own glibc stream (seed = base_seed + worker), rows dealt round-robin; returns wall seconds and
 * segments. Rate is spp-invariant, so callers pick spp/rows to bound the run time. */
typedef struct {
  const world64* w;
  const rtg_camera_desc* cam;
  unsigned seed;
  int worker, workers, rows, row_step;
  uint64_t segments;
} bench_arg;
static void* bench_worker(void* p) {
  bench_arg* a = (bench_arg*)p;
  glibc_rng g;
  grng_seed(&g, a->seed);
  ctx64 c;
  memset(&c, 0, sizeof(c));
  c.w = a->w;
  c.cam = a->cam;
  orc_camera_resolve(a->cam, &c.cp);
  c.bg = dv(a->cam->background);
  c.g = &g;
  double* row = (double*)malloc(sizeof(double) * 3 * c.cp.image_width);
  for (int j = a->worker * a->row_step; j < a->rows; j += a->workers * a->row_step) render64_rows(&c, j, 1, row);
  free(row);
  a->segments = c.segments;
  return 0;
}
int orc_bench_f64(const rtg_scene_desc* s, const rtg_camera_desc* cam, int threads, int rows, int row_step,
                  unsigned base_seed, double* seconds, uint64_t* segments) {
  if (row_step < 1) row_step = 1;
  world64 w;
  world64_init(&w, s);
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  bench_arg* args = (bench_arg*)calloc(threads, sizeof(bench_arg));
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int k = 0; k < threads; ++k) {
    args[k].w = &w;
    args[k].cam = cam;
    args[k].seed = base_seed + (unsigned)k;
    args[k].worker = k;
    args[k].workers = threads;
    args[k].rows = rows;
    args[k].row_step = row_step;
    pthread_create(&th[k], 0, bench_worker, &args[k]);
  }
  uint64_t total = 0;
  for (int k = 0; k < threads; ++k) {
    pthread_join(th[k], 0);
    total += args[k].segments;
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
  *segments = total;
  free(th);
  free(args);
  world64_free(&w);
  return 0;
}

/* ========================================================================================== */
/* fp32 spec ("rtg-f32"): the per-pixel parity target of the GPU kernels.           */
typedef struct {
  float x, y, z;
} f3;
static inline f3 F3(float x, float y, float z) {
  f3 r = {x, y, z};
  return r;
}
static inline f3 fv_add(f3 a, f3 b) { return F3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline f3 fv_sub(f3 a, f3 b) { return F3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline f3 fmul3(f3 a, f3 b) { return F3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline f3 fscl(float t, f3 a) { return F3(t * a.x, t * a.y, t * a.z); }
static inline f3 fneg(f3 a) { return F3(-a.x, -a.y, -a.z); }
/* fused multiply-adds of the spec (round 2): the same fmaf chains, in the same order,
   as rtg_kernels.hip dot / cross / madd / vfma */
static inline float fdot(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static inline f3 fcross(f3 a, f3 b) {
  return F3(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
static inline f3 fmadd3(float t, f3 a, f3 b) { return F3(fmaf(t, a.x, b.x), fmaf(t, a.y, b.y), fmaf(t, a.z, b.z)); }
static inline f3 fvfma(f3 a, f3 b, f3 c) { return F3(fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y), fmaf(a.z, b.z, c.z)); }
static inline f3 funit(f3 a) { return fscl(1.0f / sqrtf(fdot(a, a)), a); }
static inline f3 fd(const double v[3]) { return F3((float)v[0], (float)v[1], (float)v[2]); }

/* counter RNG (DESIGN.md §4 RNG): state = mix64(((pixel << 32) | sample) ^ mix64(seed)); each draw
   advances the 64-bit LCG (PCG's constants) and takes the top 24 bits of the new state */
static inline uint64_t mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xbf58476d1ce4e5b9ull;
  z ^= z >> 27;
  z *= 0x94d049bb133111ebull;
  z ^= z >> 31;
  return z;
}
static inline float U(uint64_t* s) {
  *s = *s * 6364136223846793005ull + 1442695040888963407ull;
  return (float)(uint32_t)(*s >> 40) * 5.9604644775390625e-8f;
}

/* exported for KATs */
uint64_t orc_rng_state(uint64_t seed, uint32_t pixel, uint32_t sample) {
  return mix64((((uint64_t)pixel << 32) | sample) ^ mix64(seed));
}
float orc_rng_uniform(uint64_t* state) { return U(state); }

/* sin and cos of 2*pi*u, u in [0,1) (DESIGN.md rtg-f32 "direct sampling"): quadrant reduction and
   Taylor polynomials on [-pi/4, pi/4), plain fp32 multiply / fmaf only (no libm), so the GPU kernel
   (rtg_kernels.hip sincos_turn) reproduces every bit. Used instead of the reference's rejection
   loops (vec3.hpp:158-184), which make a wavefront wait for its unluckiest lane. */
static void sincos_turn(float u, float* sn, float* cs) {
  float t = 4.0f * u;
  float q = floorf(t);
  float x = (t - q - 0.5f) * 1.57079637f;
  float x2 = x * x;
  float ps = fmaf(x2, fmaf(x2, fmaf(x2, 2.75573188e-6f, -1.98412701e-4f), 8.33333377e-3f), -1.66666672e-1f);
  float sx = fmaf(x * x2, ps, x);
  float pc = fmaf(x2, fmaf(x2, fmaf(x2, fmaf(x2, -2.75573188e-7f, 2.48015876e-5f), -1.38888892e-3f), 4.16666679e-2f),
                  -0.5f);
  float cx = fmaf(x2, pc, 1.0f);
  float a = (sx + cx) * 0.707106769f; /* sin(pi/4 + x) */
  float b = (cx - sx) * 0.707106769f; /* cos(pi/4 + x) */
  int qi = (int)q;
  float c0 = (qi & 1) ? a : b, s0 = (qi & 1) ? b : a;
  *cs = (qi == 1 || qi == 2) ? -c0 : c0;
  *sn = (qi >= 2) ? -s0 : s0;
}

/* The textures' transcendentals in the rtg-f32 spec (round 3; rtg_kernels.hip sin_spec / atan2_spec /
   acos_spec, same operations in the same order): glibc's sinf / acosf / atan2f and the GPU's ocml
   differ in the last ulp. sin: Cody-Waite reduction by pi/2 in three fmaf steps, Cephes' sinf / cosf
   polynomials on [-pi/4, pi/4]; atan2: ratio of the smaller to the larger magnitude, shifted by pi/4
   above tan(pi/8), Cephes' atanf polynomial, then the octant; acos v = atan2(sqrt(1 - v^2), v). */
static float sin_spec(float x) {
  float k = rintf(x * 0x1.45f306p-1f);
  float r = fmaf(-k, 0x1.921fb6p+0f, x);
  r = fmaf(-k, -0x1.777a5cp-25f, r);
  r = fmaf(-k, -0x1.ee59dap-50f, r);
  float z = r * r;
  float sr = fmaf(fmaf(fmaf(-0x1.9943f2p-13f, z, 0x1.11073cp-7f), z, -0x1.555546p-3f) * z, r, r);
  float cr = fmaf(fmaf(fmaf(0x1.99eb9cp-16f, z, -0x1.6c0c34p-10f), z, 0x1.55554ap-5f), z * z, fmaf(-0.5f, z, 1.0f));
  /* quadrant k mod 4 in float, exact for integer-valued k, NaN / inf -> 0: no out-of-range float -> int
     conversion; accuracy is claimed for |x| < 8192 */
  float m = k - 4.0f * floorf(0.25f * k);
  int q = (m >= 0.0f && m < 4.0f) ? (int)m : 0;
  float v = (q & 1) ? cr : sr;
  return (q & 2) ? -v : v;
}
static float atan2_spec(float y, float x) {
  float ax = fabsf(x), ay = fabsf(y);
  float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
  float a = mn > 0x1p-100f ? mn / mx : 0.0f;
  int big = a > 0x1.a8279ap-2f;
  float t = big ? (a - 1.0f) / (a + 1.0f) : a;
  float z = t * t;
  float r = fmaf(fmaf(fmaf(fmaf(0x1.49e1a2p-4f, z, -0x1.1c370ap-3f), z, 0x1.9924bep-3f), z, -0x1.555454p-2f) * z, t, t);
  if (big) r = r + 0x1.921fb6p-1f;
  if (ay > ax) r = 0x1.921fb6p+0f - r;
  if (x < 0.0f) r = 0x1.921fb6p+1f - r;
  return copysignf(r, y);
}
static float acos_spec(float v) { return atan2_spec(sqrtf(fmaxf(0.0f, fmaf(-v, v, 1.0f))), v); }
/* exported for the accuracy check against libm (tests/test_oracle_parity.py) */
float orc_sin_spec(float x) { return sin_spec(x); }
float orc_atan2_spec(float y, float x) { return atan2_spec(y, x); }
float orc_acos_spec(float v) { return acos_spec(v); }

/* random_unit_vector (vec3.hpp:172-184), direct: z = 1 - 2U, then the azimuth from a second U */
static f3 f32_random_unit_vector(uint64_t* s) {
  float z = 1.0f - 2.0f * U(s);
  float r = sqrtf(fmaxf(0.0f, fmaf(-z, z, 1.0f)));
  float sn, cs;
  sincos_turn(U(s), &sn, &cs);
  return F3(r * cs, r * sn, z);
}

/* random_in_unit_disk (vec3.hpp:158-169), direct: radius sqrt(U), then the angle from a second U */
static void f32_random_in_unit_disk(uint64_t* s, float* px, float* py) {
  float r = sqrtf(U(s));
  float sn, cs;
  sincos_turn(U(s), &sn, &cs);
  *px = r * cs;
  *py = r * sn;
}

/* exported for the sampling checks (tests/test_oracle_parity.py) */
void orc_sincos_turn(float u, float* sn, float* cs) { sincos_turn(u, sn, cs); }
void orc_f32_unit_vector(uint64_t state, float out[3]) {
  f3 v = f32_random_unit_vector(&state);
  out[0] = v.x;
  out[1] = v.y;
  out[2] = v.z;
}

typedef struct {
  const rtg_scene_desc* s;
  obvh bvh;
  /* float records */
  float* sph; /* 8 per prim: c0, r, dc, - */
  float* qd;  /* 16 per prim: Q, D, u, v, w, n */
  float* mat; /* 8 per material: fuzz, eta, albedo */
  float* tex; /* per texture: scale', color */
  float* pvec; /* perlin randvec float */
} world32;

static void world32_init(world32* w, const rtg_scene_desc* s) {
  memset(w, 0, sizeof(*w));
  w->s = s;
  bvh_build(&w->bvh, s);
  int64_t n = s->num_prims > 0 ? s->num_prims : 1;
  w->sph = (float*)calloc(n * 8, sizeof(float));
  w->qd = (float*)calloc(n * 16, sizeof(float));
  for (int64_t i = 0; i < s->num_prims; ++i) {
    const rtg_primitive* p = &s->prims[i];
    if (p->kind == RTG_PRIM_SPHERE) {
      float* r = w->sph + i * 8;
      r[0] = (float)p->p0[0];
      r[1] = (float)p->p0[1];
      r[2] = (float)p->p0[2];
      r[3] = (float)p->radius;
      r[4] = (float)(p->p1[0] - p->p0[0]);
      r[5] = (float)(p->p1[1] - p->p0[1]);
      r[6] = (float)(p->p1[2] - p->p0[2]);
    } else {
      d3 nn = dcross(dv(p->p1), dv(p->p2));
      d3 nrm = dunit(nn);
      double D = ddot(nrm, dv(p->p0));
      d3 ww = ddiv(nn, ddot(nn, nn));
      float* r = w->qd + i * 16;
      r[0] = (float)p->p0[0];
      r[1] = (float)p->p0[1];
      r[2] = (float)p->p0[2];
      r[3] = (float)D;
      r[4] = (float)p->p1[0];
      r[5] = (float)p->p1[1];
      r[6] = (float)p->p1[2];
      r[7] = (float)p->p2[0];
      r[8] = (float)p->p2[1];
      r[9] = (float)p->p2[2];
      r[10] = (float)ww.x;
      r[11] = (float)ww.y;
      r[12] = (float)ww.z;
      r[13] = (float)nrm.x;
      r[14] = (float)nrm.y;
      r[15] = (float)nrm.z;
    }
  }
  int nm = s->num_materials > 0 ? s->num_materials : 1;
  w->mat = (float*)calloc(nm * 8, sizeof(float));
  for (int m = 0; m < s->num_materials; ++m) {
    const rtg_material* mt = &s->materials[m];
    float* r = w->mat + m * 8;
    r[0] = (float)(mt->fuzz < 1.0f ? mt->fuzz : 1.0f);
    r[1] = (float)mt->refraction_index;
    r[2] = (float)mt->albedo[0];
    r[3] = (float)mt->albedo[1];
    r[4] = (float)mt->albedo[2];
  }
  int nt = s->num_textures > 0 ? s->num_textures : 1;
  w->tex = (float*)calloc(nt * 4, sizeof(float));
  for (int t = 0; t < s->num_textures; ++t) {
    const rtg_texture* tx = &s->textures[t];
    float* r = w->tex + t * 4;
    r[0] = tx->type == RTG_TEX_CHECKER ? (float)(1.0f / tx->scale) : (float)tx->scale;
    r[1] = (float)tx->color[0];
    r[2] = (float)tx->color[1];
    r[3] = (float)tx->color[2];
  }
  int np = s->num_perlins > 0 ? s->num_perlins : 1;
  w->pvec = (float*)calloc(np * 768, sizeof(float));
  for (int k = 0; k < s->num_perlins; ++k)
    for (int i = 0; i < 256; ++i)
      for (int a = 0; a < 3; ++a) w->pvec[k * 768 + i * 3 + a] = (float)s->perlins[k].randvec[i][a];
}
/* The spec's closest hit is over every primitive by the fp32 tests (with the tie rule); the BVH only
   prunes. The reference's exact f64 boxes can prune a hit the fp32 tests accept: a point the fp32 quad
   test puts inside an edge, or a ray the fp32 sphere discriminant lets graze a box face. So cpu_ref32 tests
   its (f64) boxes padded by 2^-18 (|plane| + M), M the largest |coordinate| of the scene and the camera:
   far beyond both the fp32 tests' acceptance error and the kernels' own margin (DESIGN.md §4
   "conservative culling"), so neither side's culling decides a pixel. cpu_ref64 keeps the reference's
   boxes as they are. */
static void world32_pad(world32* w, double cam_bound) {
  if (w->bvh.n <= 0) return;
  double m = cam_bound;
  for (int a = 0; a < 3; ++a) m = fmax(m, fmax(fabs(w->bvh.nodes[0].box.lo[a]), fabs(w->bvh.nodes[0].box.hi[a])));
  for (int64_t k = 0; k < w->bvh.n; ++k)
    for (int a = 0; a < 3; ++a) {
      obox* b = &w->bvh.nodes[k].box;
      b->lo[a] -= 0x1p-18 * (fabs(b->lo[a]) + m);
      b->hi[a] += 0x1p-18 * (fabs(b->hi[a]) + m);
    }
}
static void world32_free(world32* w) {
  free(w->bvh.nodes);
  free(w->sph);
  free(w->qd);
  free(w->mat);
  free(w->tex);
  free(w->pvec);
}

/* sphere::hit, fp32 robust form: c = |oc|^2 - r^2 in f64 for |r| >= 16, fp32 below;
   returns root or -1. `origin`: the ray starts on this sphere (its previous segment hit it), so
   the root at t ~ 0 is the ray's own origin and only the far root counts, and only for a ray
   entering the sphere (h < 0) — DESIGN.md §4 "origin rule". In fp32 the origin lies ~ulp(|p|)
   off the surface, and a grazing ray's own root c/q can exceed tmin = 0.001: a chrome sphere's
   reflection then re-hits the sphere from inside and stays trapped until max_depth. */
static float sphere_t32(const float* s, f3 o, f3 d, float time, float tmin, float tmax, int origin) {
  f3 C = fmadd3(time, F3(s[4], s[5], s[6]), F3(s[0], s[1], s[2]));
  f3 oc = fv_sub(o, C);
  float a = fdot(d, d), inv_a = 1.0f / a; /* per ray on the GPU (Trav::a, inv_a) */
  float hb = fdot(oc, d);
  float c, disc;
  if (fabsf(s[3]) < 16.0f) {
    /* disc = a (r^2 - |oc - (h/a) d|^2), 1/a rounded first */
    c = fmaf(-s[3], s[3], fdot(oc, oc));
    float sh = hb * inv_a;
    f3 f = fmadd3(-sh, d, oc);
    disc = a * fmaf(s[3], s[3], -fdot(f, f));
  } else {
    double ox = (double)o.x - (double)C.x, oy = (double)o.y - (double)C.y,
           oz = (double)o.z - (double)C.z, r = (double)s[3];
    c = (float)((ox * ox + oy * oy + oz * oz) - r * r);
    disc = fmaf(hb, hb, -(a * c));
  }
  if (disc < 0.0f) return -1.0f;
  float sq = sqrtf(disc);
  float q = -(hb + copysignf(sq, hb));
  /* |q| < 2^-100 (a ray tangent at its own origin) counts as a miss: the rtg-f32 spec's guard that
     keeps the device's division (div_rn, no special-case steps) in range */
  if (fabsf(q) < 0x1p-100f || a == 0.0f) return -1.0f;
  float t0 = q * inv_a, t1 = c / q; /* far root by the reciprocal, near root divided */
  float lo = fminf(t0, t1), hi = fmaxf(t0, t1);
  /* roots in (tmin, tmax]: strictly above tmin (interval::surrounds, sphere.hpp:70); a root equal to
     tmax is returned for the exact-t tie rule (sphere_wins_tie32) to decide, round 5 */
  if (origin) return (hb < 0.0f && tmin < hi && hi <= tmax) ? hi : -1.0f;
  if (tmin < lo && lo <= tmax) return lo;
  if (tmin < hi && hi <= tmax) return hi;
  return -1.0f;
}
/* quad::hit, fp32: returns t or -1 */
static float quad_t32(const float* q, f3 o, f3 d, float tmin, float tmax) {
  f3 n = F3(q[13], q[14], q[15]);
  float denom = fdot(n, d);
  if (fabsf(denom) < 1e-8f) return -1.0f;
  double dn = (double)n.x * o.x + (double)n.y * o.y + (double)n.z * o.z;
  float t = (float)((double)q[3] - dn) / denom;
  if (!(tmin <= t && t <= tmax)) return -1.0f;
  f3 p = fmadd3(t, d, o);
  f3 hp = fv_sub(p, F3(q[0], q[1], q[2]));
  f3 w = F3(q[10], q[11], q[12]);
  float alpha = fdot(w, fcross(hp, F3(q[7], q[8], q[9])));
  float beta = fdot(w, fcross(F3(q[4], q[5], q[6]), hp));
  if (!(0.0f <= alpha && alpha <= 1.0f) || !(0.0f <= beta && beta <= 1.0f)) return -1.0f;
  return t;
}

/* Exact-t tie rule of the rtg-f32 spec (rtg_kernels.hip quad_wins_tie / sphere_wins_tie):
   the reference tests its list in order (hittable_list.hpp:40-64), quads accept t == closest
   (interval::contains, quad.hpp:62), spheres do not (interval::surrounds, sphere.hpp:70). So among the
   primitives at the smallest t the last quad of the list wins if there is one, else the first sphere,
   whatever order they are tested in: at equal t a quad replaces a sphere and an earlier quad, a sphere
   replaces a later sphere (round 5) and no quad. "Order" is the order the reference tests objects in:
   a hittable_list's list order, a bvh_node's children left then right (bvh_node.hpp:89-90), i.e. the
   median tree's leaf order — the descriptor's tie_rank (ABI 7) when present, else the input order. */
static inline int64_t tie_rank32(const world32* w, int64_t id) {
  return w->s->abi_version >= 7 && w->s->tie_rank ? w->s->tie_rank[id] : id;
}
static int quad_wins_tie32(const world32* w, int64_t id, int64_t best) {
  if (w->s->prims[best].kind != RTG_PRIM_QUAD) return 1;
  return tie_rank32(w, id) > tie_rank32(w, best);
}
static int sphere_wins_tie32(const world32* w, int64_t id, int64_t best) {
  return best >= 0 && w->s->prims[best].kind == RTG_PRIM_SPHERE && tie_rank32(w, id) < tie_rank32(w, best);
}

/* closest hit: reference BVH order; boxes tested in f64 (pure culling), primitives in fp32 */
/* `origin`: the primitive the ray starts on (-1 for camera rays). A quad is planar, so a ray
   leaving it can never hit it again: it is skipped (DESIGN.md §4 "origin rule"). */
static void node_hit32(const world32* w, int32_t code, f3 o, f3 d, const double O[3],
                       const double Dd[3], float time, int64_t origin, float* tbest, int64_t* best) {
  if (code < 0) {
    int64_t id = -1 - (int64_t)code;
    float t = w->s->prims[id].kind == RTG_PRIM_SPHERE
                  ? sphere_t32(w->sph + id * 8, o, d, time, 0.001f, *tbest, id == origin)
                  : (id == origin ? -1.0f : quad_t32(w->qd + id * 16, o, d, 0.001f, *tbest));
    int take = t > 0.0f;
    if (take && t == *tbest)
      take = w->s->prims[id].kind == RTG_PRIM_QUAD ? quad_wins_tie32(w, id, *best) : sphere_wins_tie32(w, id, *best);
    if (take) {
      *tbest = t;
      *best = id;
    }
    return;
  }
  const onode* n = &w->bvh.nodes[code];
  if (!box_hit(&n->box, O, Dd, 0.0009, (double)*tbest * (1 + 1e-6) + 1e-6)) return;
  node_hit32(w, n->left, o, d, O, Dd, time, origin, tbest, best);
  if (n->right != n->left) node_hit32(w, n->right, o, d, O, Dd, time, origin, tbest, best);
}

static float perlin_noise32(const float* vec, const rtg_perlin* pl, f3 p) {
  float fx = floorf(p.x), fy = floorf(p.y), fz = floorf(p.z);
  float u = p.x - fx, v = p.y - fy, w = p.z - fz;
  int i = (int)fx, j = (int)fy, k = (int)fz;
  float uu = u * u * (3.0f - 2.0f * u), vv = v * v * (3.0f - 2.0f * v), ww = w * w * (3.0f - 2.0f * w);
  float accum = 0.0f;
  for (int di = 0; di < 2; ++di)
    for (int dj = 0; dj < 2; ++dj)
      for (int dk = 0; dk < 2; ++dk) {
        int idx = pl->perm_x[(i + di) & 255] ^ pl->perm_y[(j + dj) & 255] ^ pl->perm_z[(k + dk) & 255];
        f3 c = F3(vec[idx * 3], vec[idx * 3 + 1], vec[idx * 3 + 2]);
        f3 wv = F3(u - di, v - dj, w - dk);
        float fu = di ? uu : (1.0f - uu), fv = dj ? vv : (1.0f - vv), fw = dk ? ww : (1.0f - ww);
        accum = fmaf(fu * fv * fw, fdot(c, wv), accum);
      }
  return accum;
}

static f3 tex_value32(const world32* w, int32_t t, float u, float v, f3 p) {
  const rtg_scene_desc* s = w->s;
  for (int guard = 0; guard < 16; ++guard) {
    const rtg_texture* tx = &s->textures[t];
    const float* tf = w->tex + t * 4;
    if (tx->type == RTG_TEX_SOLID) return F3(tf[1], tf[2], tf[3]);
    if (tx->type == RTG_TEX_CHECKER) {
      int xi = (int)floorf(tf[0] * p.x), yi = (int)floorf(tf[0] * p.y), zi = (int)floorf(tf[0] * p.z);
      t = ((xi + yi + zi) % 2 == 0) ? tx->even : tx->odd;
      continue;
    }
    if (tx->type == RTG_TEX_IMAGE) {
      const rtg_image* im = (tx->image >= 0 && tx->image < s->num_images) ? &s->images[tx->image] : 0;
      if (!im || !im->rgb || im->height <= 0 || im->width <= 0) return F3(0.0f, 1.0f, 1.0f);
      float uc = fminf(fmaxf(u, 0.0f), 1.0f);
      float vc = 1.0f - fminf(fmaxf(v, 0.0f), 1.0f);
      int i = (int)(uc * (float)im->width), j = (int)(vc * (float)im->height);
      i = i < 0 ? 0 : (i < im->width ? i : im->width - 1);
      j = j < 0 ? 0 : (j < im->height ? j : im->height - 1);
      const uint8_t* px = im->rgb + ((int64_t)j * im->width + i) * 3;
      float cs = 1.0f / 255.0f;
      return F3(cs * px[0], cs * px[1], cs * px[2]);
    }
    if (tx->type == RTG_TEX_NOISE) {
      const rtg_perlin* pl = &s->perlins[tx->perlin];
      const float* vec = w->pvec + tx->perlin * 768;
      float accum = 0.0f, weight = 1.0f;
      f3 tp = p;
      for (int o = 0; o < 7; ++o) {
        accum = fmaf(weight, perlin_noise32(vec, pl, tp), accum);
        weight *= 0.5f;
        tp = fscl(2.0f, tp);
      }
      float tb = fabsf(accum);
      float sv = 0.5f * (1.0f + sin_spec(fmaf(tf[0], p.z, 10.0f * tb)));
      return F3(sv, sv, sv);
    }
    break;
  }
  return F3(1.0f, 0.0f, 1.0f);
}

static int tex_uses_uv(const rtg_scene_desc* s, int32_t t, int depth) {
  if (depth > 16 || t < 0 || t >= s->num_textures) return 0;
  const rtg_texture* tx = &s->textures[t];
  if (tx->type == RTG_TEX_IMAGE) return 1;
  if (tx->type == RTG_TEX_CHECKER) return tex_uses_uv(s, tx->even, depth + 1) || tex_uses_uv(s, tx->odd, depth + 1);
  return 0;
}

/* One camera sample (get_ray + iterative ray_color) in the fp32 spec. */
static f3 sample32(const world32* w, const rtg_camera_desc* cam, const float* cf, uint64_t seed,
                   uint32_t pixel_id, uint32_t sample, int i, int j, uint64_t* segs) {
  uint64_t st = orc_rng_state(seed, pixel_id, sample);
  f3 p00 = F3(cf[0], cf[1], cf[2]), du = F3(cf[3], cf[4], cf[5]), dvv = F3(cf[6], cf[7], cf[8]);
  f3 center = F3(cf[9], cf[10], cf[11]);
  float ox = U(&st) - 0.5f;
  float oy = U(&st) - 0.5f;
  f3 ps = fmadd3((float)j + oy, dvv, fmadd3((float)i + ox, du, p00));
  f3 o = center;
  if (!(cam->defocus_angle <= 0.0f)) {
    float px, py;
    f32_random_in_unit_disk(&st, &px, &py);
    o = fmadd3(py, F3(cf[15], cf[16], cf[17]), fmadd3(px, F3(cf[12], cf[13], cf[14]), center));
  }
  f3 d = fv_sub(ps, o);
  float time = U(&st);
  f3 T = F3(1.0f, 1.0f, 1.0f), L = F3(0.0f, 0.0f, 0.0f);
  f3 bg = F3(cf[18], cf[19], cf[20]);
  int64_t origin = -1; /* the primitive the current segment starts on */
  for (int depth = cam->max_depth; depth > 0; --depth) {
    float tbest = INFINITY;
    int64_t best = -1;
    (*segs)++;
    if (w->bvh.n > 0) {
      const double O[3] = {o.x, o.y, o.z}, Dd[3] = {d.x, d.y, d.z};
      node_hit32(w, 0, o, d, O, Dd, time, origin, &tbest, &best);
    }
    if (best < 0) {
      L = fvfma(T, bg, L);
      break;
    }
    const rtg_primitive* pr = &w->s->prims[best];
    f3 p = fmadd3(tbest, d, o), outward;
    float u = 0.0f, v = 0.0f;
    int sphere = pr->kind == RTG_PRIM_SPHERE;
    if (sphere) {
      const float* s = w->sph + best * 8;
      f3 C = fmadd3(time, F3(s[4], s[5], s[6]), F3(s[0], s[1], s[2]));
      outward = fscl(1.0f / s[3], fv_sub(p, C));
    } else {
      const float* q = w->qd + best * 16;
      f3 hp = fv_sub(p, F3(q[0], q[1], q[2]));
      f3 ww = F3(q[10], q[11], q[12]);
      u = fdot(ww, fcross(hp, F3(q[7], q[8], q[9])));
      v = fdot(ww, fcross(F3(q[4], q[5], q[6]), hp));
      outward = F3(q[13], q[14], q[15]);
    }
    int front = fdot(d, outward) < 0.0f;
    f3 n = front ? outward : fneg(outward);
    const rtg_material* m = &w->s->materials[pr->material];
    const float* mf = w->mat + pr->material * 8;
    int needs_uv = sphere && (m->type == RTG_MAT_LAMBERTIAN || m->type == RTG_MAT_DIFFUSE_LIGHT) &&
                   tex_uses_uv(w->s, m->texture, 0);
    if (needs_uv) {
      float theta = acos_spec(-outward.y);
      float phi = atan2_spec(-outward.z, outward.x) + 3.14159265358979323846f;
      u = phi / (2.0f * 3.14159265358979323846f);
      v = theta / 3.14159265358979323846f;
    }
    f3 att, dir;
    if (m->type == RTG_MAT_DIFFUSE_LIGHT) {
      L = fvfma(T, tex_value32(w, m->texture, u, v, p), L);
      break;
    } else if (m->type == RTG_MAT_LAMBERTIAN) {
      dir = fv_add(n, f32_random_unit_vector(&st));
      if (fabsf(dir.x) < 1e-8f && dir.y < 1e-8f && fabsf(dir.z) < 1e-8f) dir = n;
      att = tex_value32(w, m->texture, u, v, p);
    } else if (m->type == RTG_MAT_METAL) {
      f3 refl = fmadd3(-(2.0f * fdot(d, n)), n, d);
      f3 r = f32_random_unit_vector(&st);
      dir = fmadd3(mf[0], r, funit(refl));
      att = F3(mf[2], mf[3], mf[4]);
      if (!(fdot(dir, n) > 0.0f)) break;
    } else if (m->type == RTG_MAT_DIELECTRIC) {
      att = F3(1.0f, 1.0f, 1.0f);
      float ri = front ? (1.0f / mf[1]) : mf[1];
      f3 ud = funit(d);
      float ct = fminf(fdot(fneg(ud), n), 1.0f);
      float stt = sqrtf(fmaf(-ct, ct, 1.0f));
      int cannot = ri * stt > 1.0f;
      int reflect = cannot;
      if (!cannot) {
        float r0 = (1.0f - ri) / (1.0f + ri);
        r0 = r0 * r0;
        float x = 1.0f - ct;
        float refl = fmaf(1.0f - r0, x * x * x * x * x, r0);
        reflect = refl > U(&st);
      }
      if (reflect) {
        dir = fmadd3(-(2.0f * fdot(ud, n)), n, ud);
      } else {
        float c2 = fminf(fdot(fneg(ud), n), 1.0f);
        f3 perp = fscl(ri, fmadd3(c2, n, ud));
        dir = fmadd3(-sqrtf(fabsf(1.0f - fdot(perp, perp))), n, perp);
      }
    } else {
      break;
    }
    T = fmul3(T, att);
    o = p;
    d = dir;
    origin = best;
  }
  return L;
}

/* cpu_ref32 render: rows row_begin + k*row_stride, k < row_count; out = scale * sum (fp32). */
/* rows r = r0, r0 + rstep, ... < row_count of the shard (image row row_begin + r * row_stride) */
typedef struct {
  const world32* w;
  const rtg_camera_desc* cam;
  const float* cf;
  const rtg_camera_params* cp;
  uint64_t seed;
  int row_begin, row_stride, row_count, r0, rstep;
  float* out;
  uint64_t segs;
} rows32_arg;

static void* render_rows32(void* p) {
  rows32_arg* a = (rows32_arg*)p;
  const rtg_camera_params* cp = a->cp;
  const rtg_camera_desc* cam = a->cam;
  const float scale = (float)cp->pixel_samples_scale;
  uint64_t segs = 0;
  for (int r = a->r0; r < a->row_count; r += a->rstep) {
    int j = a->row_begin + r * a->row_stride;
    for (int i = 0; i < cp->image_width; ++i) {
      uint32_t pid = (uint32_t)j * (uint32_t)cp->image_width + (uint32_t)i;
      /* rtg-f32 accumulation (rtgpu.h rtg_chunk_samples): chunks of K samples summed from zero in
         sample order, chunk sums added in chunk order; one chunk == the reference's running sum */
      f3 acc = F3(0.0f, 0.0f, 0.0f);
      if (cam->max_depth > 0) {
        int spp = cam->samples_per_pixel, K = rtg_chunk_samples(spp);
        for (int c0 = 0; c0 < spp; c0 += K) {
          f3 part = F3(0.0f, 0.0f, 0.0f);
          for (int smp = c0; smp < spp && smp < c0 + K; ++smp)
            part = fv_add(part, sample32(a->w, cam, a->cf, a->seed, pid, (uint32_t)smp, i, j, &segs));
          acc = c0 == 0 ? part : fv_add(acc, part);
        }
      }
      float* o = a->out + ((int64_t)r * cp->image_width + i) * 3;
      o[0] = scale * acc.x;
      o[1] = scale * acc.y;
      o[2] = scale * acc.z;
    }
  }
  a->segs = segs;
  return 0;
}

/* cpu_ref32 over rows row_begin + k * row_stride, k < row_count, on `threads` threads sharing one world
   (rows dealt round-robin; every pixel's arithmetic is the single-threaded one, so the frame does not
   depend on the thread count). threads <= 1: the caller's thread only. */
int orc_render_f32_mt(const rtg_scene_desc* s, const rtg_camera_desc* cam, uint64_t seed, int row_begin,
                      int row_stride, int row_count, float* out, uint64_t* segments, int threads) {
  rtg_camera_params cp;
  orc_camera_resolve(cam, &cp);
  if (row_stride < 1) row_stride = 1;
  if (row_count <= 0) row_count = (cp.image_height - 1 - row_begin) / row_stride + 1;
  float cf[21];
  for (int k = 0; k < 3; ++k) {
    cf[k] = (float)cp.pixel00_loc[k];
    cf[3 + k] = (float)cp.pixel_delta_u[k];
    cf[6 + k] = (float)cp.pixel_delta_v[k];
    cf[9 + k] = (float)cp.center[k];
    cf[12 + k] = (float)cp.defocus_disk_u[k];
    cf[15 + k] = (float)cp.defocus_disk_v[k];
    cf[18 + k] = (float)cam->background[k];
  }
  world32 w;
  world32_init(&w, s);
  double cam_bound = 0.0;
  for (int a = 0; a < 3; ++a)
    cam_bound = fmax(cam_bound, fabs(cp.center[a]) + fabs(cp.defocus_disk_u[a]) + fabs(cp.defocus_disk_v[a]));
  world32_pad(&w, cam_bound);
  if (threads < 1) threads = 1;
  if (threads > row_count) threads = row_count > 0 ? row_count : 1;
  rows32_arg* args = (rows32_arg*)calloc(threads, sizeof(rows32_arg));
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  int* started = (int*)calloc(threads, sizeof(int));
  for (int k = 0; k < threads; ++k) {
    rows32_arg a = {&w, cam, cf, &cp, seed, row_begin, row_stride, row_count, k, threads, out, 0};
    args[k] = a;
    if (k > 0) started[k] = pthread_create(&th[k], 0, render_rows32, &args[k]) == 0;
  }
  render_rows32(&args[0]);
  uint64_t segs = args[0].segs;
  for (int k = 1; k < threads; ++k) {
    if (started[k]) pthread_join(th[k], 0);
    else render_rows32(&args[k]); /* no thread (e.g. a cgroup thread limit): its rows on this one */
    segs += args[k].segs;
  }
  free(started);
  if (segments) *segments = segs;
  free(th);
  free(args);
  world32_free(&w);
  return 0;
}

int orc_render_f32(const rtg_scene_desc* s, const rtg_camera_desc* cam, uint64_t seed, int row_begin,
                   int row_stride, int row_count, float* out, uint64_t* segments) {
  return orc_render_f32_mt(s, cam, seed, row_begin, row_stride, row_count, out, segments, 1);
}

/* write_color (color.hpp:14-58) on a double pixel: the reference's byte triple */
void orc_write_color(const double rgb[3], int out[3]) {
  for (int k = 0; k < 3; ++k) {
    double x = rgb[k];
    x = x > 0.0f ? sqrt(x) : 0.0f;
    double lo = 0.000f, hi = 0.999f;
    x = x < lo ? lo : (x > hi ? hi : x);
    out[k] = (int)(256 * x);
  }
}

/* ------------------------------------------------------------------------------------------ */
/* KAT entry points (tests/test_oracle_golden.py): the fp64 pieces above, one call each.       */
void orc_kat_random_unit_vector(unsigned seed, double out[3], double* next) {
  glibc_rng g;
  grng_seed(&g, seed);
  d3 v = f64_random_unit_vector(&g);
  out[0] = v.x;
  out[1] = v.y;
  out[2] = v.z;
  *next = grand(&g);
}
void orc_kat_random_in_unit_disk(unsigned seed, double out[3], double* next) {
  glibc_rng g;
  grng_seed(&g, seed);
  double px, py;
  while (1) {
    py = grand_mm(&g, -1.0f, 1.0f);
    px = grand_mm(&g, -1.0f, 1.0f);
    if (px * px + py * py + 0.0 * 0.0 < 1.0f) break;
  }
  out[0] = px;
  out[1] = py;
  out[2] = 0.0f;
  *next = grand(&g);
}
/* sphere::hit: rec = {t, p[3], normal[3], front, u, v} */
int orc_kat_sphere_hit(const rtg_primitive* p, const double o[3], const double d[3], double time,
                       double tmin, double tmax, double rec[10]) {
  hrec64 r;
  int h = sphere_hit64(p, dv(o), dv(d), time, tmin, tmax, &r);
  if (h) {
    rec[0] = r.t;
    rec[1] = r.p.x, rec[2] = r.p.y, rec[3] = r.p.z;
    rec[4] = r.normal.x, rec[5] = r.normal.y, rec[6] = r.normal.z;
    rec[7] = r.front;
    rec[8] = r.u;
    rec[9] = r.v;
  }
  return h;
}
/* the rtg-f32 sphere test (sphere_t32) on one record {center, r, motion, material}: t or -1, a root
   inside (tmin, tmax) as sphere::hit accepts it (a root equal to tmax, which the tie rule sees, is a miss) */
float orc_sphere_t32(const float s[8], const float o[3], const float d[3], float time, float tmin,
                     float tmax) {
  const float t = sphere_t32(s, F3(o[0], o[1], o[2]), F3(d[0], d[1], d[2]), time, tmin, tmax, 0);
  return t == tmax ? -1.0f : t;
}
int orc_kat_quad_hit(const rtg_primitive* p, const double o[3], const double d[3], double tmin,
                     double tmax, double rec[10], double bbox[6]) {
  rtg_scene_desc s;
  memset(&s, 0, sizeof(s));
  s.prims = p;
  s.num_prims = 1;
  world64 w;
  memset(&w, 0, sizeof(w));
  w.s = &s;
  d3 qn[1], qw[1];
  double qD[1];
  d3 nn = dcross(dv(p->p1), dv(p->p2));
  qn[0] = dunit(nn);
  qD[0] = ddot(qn[0], dv(p->p0));
  qw[0] = ddiv(nn, ddot(nn, nn));
  w.qn = qn;
  w.qD = qD;
  w.qw = qw;
  obox b = prim_box(p);
  for (int k = 0; k < 3; ++k) {
    bbox[k] = b.lo[k];
    bbox[3 + k] = b.hi[k];
  }
  hrec64 r;
  int h = quad_hit64(&w, 0, dv(o), dv(d), tmin, tmax, &r);
  if (h) {
    rec[0] = r.t;
    rec[1] = r.p.x, rec[2] = r.p.y, rec[3] = r.p.z;
    rec[4] = r.normal.x, rec[5] = r.normal.y, rec[6] = r.normal.z;
    rec[7] = r.front;
    rec[8] = r.u;
    rec[9] = r.v;
  }
  return h;
}
/* aabb(a, b) then aabb::hit; box[6] receives the padded box, *axis the longest axis */
int orc_kat_aabb_hit(const double a[3], const double b[3], const double o[3], const double d[3],
                     double tmin, double tmax, double box[6], int* axis) {
  obox bx = box_pts(dv(a), dv(b));
  for (int k = 0; k < 3; ++k) {
    box[k] = bx.lo[k];
    box[3 + k] = bx.hi[k];
  }
  *axis = longest(bx);
  return box_hit(&bx, o, d, tmin, tmax);
}
void orc_kat_reflect_refract(const double v[3], const double n[3], double eta, double refl[3],
                             double refr[3]) {
  d3 V = dv(v), N = dv(n);
  d3 r = dsub(V, dscl(2.0f * ddot(V, N), N));
  double c = fmin(ddot(dneg(V), N), 1.0f);
  d3 perp = dscl(eta, dadd(V, dscl(c, N)));
  d3 par = dscl(-sqrt(fabs(1.0f - ddot(perp, perp))), N);
  d3 t = dadd(perp, par);
  memcpy(refl, &r, 24);
  memcpy(refr, &t, 24);
}
/* bvh traversal replay: the sequence of primitive ids whose hit() the reference traversal calls
 * for one ray over the oracle's own median tree (bvh_node.hpp:25-94); returns the count. */
typedef struct {
  int64_t* log;
  int64_t n, cap;
} hitlog;
static int node_hit_logged(const world64* w, int32_t code, d3 o, d3 d, const double O[3],
                           const double Dd[3], double time, double tmin, double tmax, hrec64* rec,
                           hitlog* lg) {
  if (code < 0) {
    int64_t id = -1 - (int64_t)code;
    if (lg->n < lg->cap) lg->log[lg->n] = id;
    lg->n++;
    return prim_hit64(w, id, o, d, time, tmin, tmax, rec);
  }
  const onode* n = &w->bvh.nodes[code];
  if (!box_hit(&n->box, O, Dd, tmin, tmax)) return 0;
  int hl = node_hit_logged(w, n->left, o, d, O, Dd, time, tmin, tmax, rec, lg);
  int hr = node_hit_logged(w, n->right, o, d, O, Dd, time, tmin, hl ? rec->t : tmax, rec, lg);
  return hl || hr;
}
int64_t orc_bvh_replay(const rtg_scene_desc* s, const double o[3], const double d[3], double time,
                       int64_t* log, int64_t cap, double* t_hit) {
  world64 w;
  world64_init(&w, s);
  hitlog lg = {log, 0, cap};
  hrec64 rec;
  const double O[3] = {o[0], o[1], o[2]}, Dd[3] = {d[0], d[1], d[2]};
  int h = w.bvh.n ? node_hit_logged(&w, 0, dv(o), dv(d), O, Dd, time, 0.001, INFINITY, &rec, &lg) : 0;
  *t_hit = h ? rec.t : -1.0;
  world64_free(&w);
  return lg.n;
}

/* cpu_ref32's closest hit for n rays (o, d, time as fp32, the camera segment's form: tmin 0.001, no
 * origin primitive): best[k] = the winning primitive (input index, -1 on a miss), t[k] its fp32 t. The
 * exact-t tie rule decides equal t by the descriptor's tie_rank (tests/test_oracle_golden.py pins it
 * against the winners of the reference's own compiled hittable_list / bvh_node / sphere / quad). */
void orc_closest_hit32(const rtg_scene_desc* s, int64_t n, const float* o, const float* d, const float* time,
                       int64_t* best, float* t) {
  world32 w;
  world32_init(&w, s);
  double bound = 0.0;
  for (int64_t k = 0; k < n; ++k)
    for (int a = 0; a < 3; ++a) bound = fmax(bound, fabs((double)o[k * 3 + a]));
  world32_pad(&w, bound);
  for (int64_t k = 0; k < n; ++k) {
    f3 O3 = F3(o[k * 3], o[k * 3 + 1], o[k * 3 + 2]), D3v = F3(d[k * 3], d[k * 3 + 1], d[k * 3 + 2]);
    float tb = INFINITY;
    int64_t b = -1;
    if (w.bvh.n > 0) {
      const double O[3] = {O3.x, O3.y, O3.z}, Dd[3] = {D3v.x, D3v.y, D3v.z};
      node_hit32(&w, 0, O3, D3v, O, Dd, time[k], -1, &tb, &b);
    }
    best[k] = b;
    t[k] = b >= 0 ? tb : -1.0f;
  }
  world32_free(&w);
}
