// rtg_kernels.hip — gfx950 kernels of the per-pixel sample loop.
//
// Replaces (reference file:line):
//   camera::render 29-72, get_ray 139-177, ray_color 180-232      (src/core/camera.hpp)
//   hittable_list::hit 40-64 + bvh_node::hit 80-94 + aabb::hit 61-112
//   sphere::hit 47-93 / get_sphere_uv 100-111, quad::hit 44-114
//   material::scatter / emitted (src/core/material.hpp:51-240)
//   texture::value (src/core/texture.hpp:34-151), perlin::turb (src/core/perlin.hpp:95-158,219-255)
//   write_color (src/common/color.hpp:14-58)
//
// Execution model: one lane owns one pixel of the shard and walks its samples in order
// s = 0..spp-1, so the per-pixel sum is accumulated in exactly the order the reference uses
// (camera.hpp:55-62). Paths are regenerated in place: when a lane's path ends it immediately
// starts its next sample, so every lane of a wave traces one segment per loop trip until the
// lane has finished all of its samples (no per-bounce wave drain). A 64-lane wave covers an
// 8x8 pixel tile; a 256-thread workgroup covers 16x16. Each lane's BVH stack lives in LDS
// laid out [depth][lane] (bank-conflict-free for ds_read_b32/ds_write_b32).
//
// Numerics: the fp32 spec in DESIGN.md ("rtg-f32"); compiled with -ffp-contract=off so every
// expression rounds as written and matches the CPU restatement in oracle/cpu_ref.c. Fused ops are
// explicit fmaf calls (dot / cross / madd / vfma and the forms marked in the code), placed exactly
// as in the oracle; the slab tests' packed FMAs only cull (boxes are rounded outward on the host).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "rtg_internal.hpp"
#include "rtg_numerics.hpp"


namespace rtg {
namespace {

constexpr float kTMin = 0.001f;  // interval(0.001, infinity), camera.hpp:192
// Conservative culling. Box tests only prune: a child is skipped when
// its entry distance is past fmaf(tbest, kCullRel, kCullAbs) or its exit before kCullTMin, a margin at
// least the oracle's (oracle/cpu_ref.c node_hit32: tbest (1 + 1e-6) + 1e-6, floor 0.0009), while the
// primitive tests keep the exact tbest and tmin. With the boxes padded on the host for the slab test's
// rounding (rtg_api.cpp pad_down), a box holding the closest hit is never culled by fp32 error.
constexpr float kCullTMin = 0.0009f;
constexpr float kCullRel = 1.0f + 0x1p-19f;
constexpr float kCullAbs = 0x1p-19f;
__device__ __forceinline__ float cull_bound(float tbest) { return fmaf(tbest, kCullRel, kCullAbs); }
// Kernels that test quads compare a child's entry distance with min(exit, tbest) * kCullWiden instead: the
// slab test's relative error (3 2^-24 of t per plane) and quad_t's (2 2^-24) are then taken in t, so the boxes
// need padding only for the errors that do not grow with the distance (rtg_api.cpp culling_box), and the
// factor is the cull bound's relative margin as well (its absolute 2^-19 is covered by the pads there). One
// v_pk_mul_f32 per child pair replaces cull_bound. Sphere-only kernels keep cull_bound and the plain exit
// (their boxes carry the distance terms).
constexpr float kCullWiden = 1.0f + 0x1p-19f;
constexpr float kPi = 3.14159265358979323846f;
constexpr int kMaxTexNesting = 16;

struct V3 {
  float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 mul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ V3 scl(float t, V3 a) { return v3(t * a.x, t * a.y, t * a.z); }
__device__ __forceinline__ V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
// Fused multiply-adds of the rtg-f32 spec (round 2): dot products, cross products,
// `b + t a` and the other forms below are single-rounding fmaf chains in exactly this order, here
// and in oracle/cpu_ref.c (fmaf is correctly rounded on both sides, so the bits still agree).
__device__ __forceinline__ float dot(V3 a, V3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return v3(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
__device__ __forceinline__ V3 madd(float t, V3 a, V3 b) {  // b + t a
  return v3(fmaf(t, a.x, b.x), fmaf(t, a.y, b.y), fmaf(t, a.z, b.z));
}
__device__ __forceinline__ V3 vfma(V3 a, V3 b, V3 c) {  // a * b + c per component
  return v3(fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y), fmaf(a.z, b.z, c.z));
}
// div_rn / sqrt_rn: rtg_numerics.hpp (shared with the numerics check, tests/native)
__device__ __forceinline__ V3 unit(V3 a) {  // unit_vector: v / v.length() == (1/len) * v
  const float len = sqrt_rn(dot(a, a));
  return scl(div_rn(1.0f, len), a);
}
__device__ __forceinline__ V3 xyz(float4 f) { return v3(f.x, f.y, f.z); }
__device__ __forceinline__ int ibits(float f) { return __float_as_int(f); }

// ---------------------------------------------------------------------------------------
// Counter RNG: a 64-bit LCG (PCG's multiplier and increment) seeded per
// (pixel, sample) by a splitmix64 finaliser; a draw is the top 24 bits of the advanced state.
// Replaces the global glibc rand() stream (rtweekend.hpp:23-39, hazard H1). Round 1 drew PCG32
// XSH-RR outputs; the top bits of the 64-bit state are as good for 24-bit uniforms (G5 tests)
// at 7 VALU per draw instead of ~14.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xbf58476d1ce4e5b9ull;
  z ^= z >> 27;
  z *= 0x94d049bb133111ebull;
  z ^= z >> 31;
  return z;
}
// One draw's 24 bits as an exact float integer in [0, 2^24): uniform() = draw24() * 2^-24. Callers that
// scale U by a power of two or add a constant fold the scaling into one exact product (and the constant
// into an fmaf, whose one rounding is the spec's rounding of the sum): bit-identical, fewer VALU ops.
__device__ __forceinline__ float draw24(uint64_t& s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  // bits 63..40, converted by an explicit v_cvt_f32_u32: the compiler widens a plain
  // (float)(uint32_t)(s >> 40) back into a 64-bit integer-to-float expansion (+6 VALU per draw)
  const uint32_t top = static_cast<uint32_t>(s >> 32) >> 8;
  float f;
  asm("v_cvt_f32_u32 %0, %1" : "=v"(f) : "v"(top));
  return f;
}
__device__ __forceinline__ float uniform(uint64_t& s) {  // random_double(), [0,1), 24 bits
  return draw24(s) * 5.9604644775390625e-8f;
}

// sin and cos of 2*pi*u, u in [0,1): quadrant reduction and Taylor polynomials on [-pi/4, pi/4),
// plain fp32 multiply / fmaf only, so oracle/cpu_ref.c (sincos_turn) reproduces every bit. Takes
// t = 4u (for a draw: draw24 * 2^-22, the spec's 4 * (draw24 * 2^-24) exactly)
__device__ __forceinline__ void sincos_turn4(float t, float& sn, float& cs) {
  const float q = floorf(t);
  const float x = (t - q - 0.5f) * 1.57079637f;
  const float x2 = x * x;
  // Horner steps as fmaf (rtg-f32 round 2)
  const float ps = fmaf(x2, fmaf(x2, fmaf(x2, 2.75573188e-6f, -1.98412701e-4f), 8.33333377e-3f), -1.66666672e-1f);
  const float sx = fmaf(x * x2, ps, x);
  const float pc = fmaf(x2, fmaf(x2, fmaf(x2, fmaf(x2, -2.75573188e-7f, 2.48015876e-5f), -1.38888892e-3f),
                                 4.16666679e-2f), -0.5f);
  const float cx = fmaf(x2, pc, 1.0f);
  const float a = (sx + cx) * 0.707106769f;  // sin(pi/4 + x)
  const float b = (cx - sx) * 0.707106769f;  // cos(pi/4 + x)
  const int qi = static_cast<int>(q);
  const float c0 = (qi & 1) ? a : b, s0 = (qi & 1) ? b : a;
  cs = (qi == 1 || qi == 2) ? -c0 : c0;
  sn = (qi >= 2) ? -s0 : s0;
}

// The textures' transcendentals in the rtg-f32 spec (round 3). libm's sinf / acosf / atan2f (ocml
// here, glibc in the oracle) differ in the last ulp, which left ~26 % of config 3's pixels off the
// oracle by ~1e-6. These are fixed sequences of fp32 operations (fmaf, correctly rounded division and
// square root, rint), restated in oracle/cpu_ref.c, so the GPU and the oracle agree to the bit.
// sin: Cody-Waite reduction by pi/2 in three fmaf steps, then Cephes' sinf / cosf polynomials on
// [-pi/4, pi/4] (about 1 ulp for |x| < 8192; the noise texture's argument is scale * z + 10 * turb).
__device__ __forceinline__ float sin_spec(float x) {
  const float k = rintf(x * 0x1.45f306p-1f);  // nearest multiple of pi/2
  float r = fmaf(-k, 0x1.921fb6p+0f, x);
  r = fmaf(-k, -0x1.777a5cp-25f, r);
  r = fmaf(-k, -0x1.ee59dap-50f, r);
  const float z = r * r;
  const float sr = fmaf(fmaf(fmaf(-0x1.9943f2p-13f, z, 0x1.11073cp-7f), z, -0x1.555546p-3f) * z, r, r);
  const float cr = fmaf(fmaf(fmaf(0x1.99eb9cp-16f, z, -0x1.6c0c34p-10f), z, 0x1.55554ap-5f), z * z,
                        fmaf(-0.5f, z, 1.0f));
  // the quadrant k mod 4 in float (exact for every integer-valued k; NaN / inf fall to 0), so no
  // float -> int conversion sees an out-of-range value here or in the oracle. The spec's
  // accuracy claim is |x| < 8192 (three-step reduction); larger arguments stay bit-identical between
  // kernel and oracle but drift from libm's sin.
  const float m = k - 4.0f * floorf(0.25f * k);
  const int q = (m >= 0.0f && m < 4.0f) ? static_cast<int>(m) : 0;
  const float v = (q & 1) ? cr : sr;
  return (q & 2) ? -v : v;
}
// atan2: the ratio of the smaller to the larger magnitude, above tan(pi/8) shifted by pi/4, Cephes'
// atanf polynomial, then the octant; the sign follows y (atan2(+-0, x >= +0) = +-0, x < 0: +-pi)
__device__ __forceinline__ float atan2_spec(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
  const float a = mn > 0x1p-100f ? div_rn(mn, mx) : 0.0f;  // div_rn's exact range (and atan ~ 0 below)
  const bool big = a > 0x1.a8279ap-2f;  // tan(pi/8)
  const float t = big ? div_rn(a - 1.0f, a + 1.0f) : a;
  const float z = t * t;
  float r = fmaf(fmaf(fmaf(fmaf(0x1.49e1a2p-4f, z, -0x1.1c370ap-3f), z, 0x1.9924bep-3f), z, -0x1.555454p-2f) * z,
                 t, t);
  if (big) r = r + 0x1.921fb6p-1f;      // + pi/4
  if (ay > ax) r = 0x1.921fb6p+0f - r;  // pi/2 - r
  if (x < 0.0f) r = 0x1.921fb6p+1f - r; // pi - r
  return copysignf(r, y);
}
// acos v = atan2(sqrt(1 - v^2), v), v in [-1, 1]
__device__ __forceinline__ float acos_spec(float v) {
  return atan2_spec(sqrtf(fmaxf(0.0f, fmaf(-v, v, 1.0f))), v);
}

// random_unit_vector (vec3.hpp:172-184) by direct sampling (DESIGN.md rtg-f32): z = 1 - 2U, then
// the azimuth from a second U. The reference's rejection loop would make every wave wait for its
// unluckiest lane (~5 tries for 30 lanes at acceptance pi/6); this costs two draws, always.
__device__ __forceinline__ V3 random_unit_vector(uint64_t& s) {
  const float z = fmaf(-0x1p-23f, draw24(s), 1.0f);  // 1 - 2U: 2U = draw24 * 2^-23 exactly
  const float r = sqrt_rn(fmaxf(0.0f, fmaf(-z, z, 1.0f)));
  float sn, cs;
  sincos_turn4(draw24(s) * 0x1p-22f, sn, cs);
  return v3(r * cs, r * sn, z);
}

// ---------------------------------------------------------------------------------------
// Geometry
// sphere::hit (sphere.hpp:47-93) with the fp32-robust root form of DESIGN.md: c = |oc|^2 - r^2
// is formed in f64 for spheres of radius >= kSphereF64Radius (a ground sphere, where fp32
// cancellation would put self-hits above tmin), in fp32 below it, where the discriminant is
// taken from the centre-to-line distance; the near root is c/q. Returns the root or -1.
// `origin`: the ray starts on this sphere (its previous segment hit it): only the far root of a
// ray entering the sphere counts (DESIGN.md §4 "origin rule"; fp32 puts the origin ~ulp(|p|) off
// the surface, and a grazing ray's own root could pass tmin and trap a reflection inside).
constexpr float kSphereF64Radius = 16.0f;
// a = d.d and inv_a = 1/a (correctly rounded) are per ray (Trav): the far root is q * inv_a and
// only the near root c / q is a division.
template <bool INCL = false>
__device__ __forceinline__ float sphere_t(float4 s0, float4 s1, V3 o, V3 d, float a, float inv_a, float time,
                                          float tmin, float tmax, bool origin) {
  const V3 C = madd(time, xyz(s1), xyz(s0));
  const V3 oc = sub(o, C);
  const float hb = dot(oc, d);
  float c, disc;
  if (fabsf(s0.w) < kSphereF64Radius) {
    c = fmaf(-s0.w, s0.w, dot(oc, oc));
    // disc = a (r^2 - |f|^2), f = oc - (h/a) d the centre-to-line offset: no h^2 - a c
    // cancellation, so a grazing ray far from a small sphere is classified to ~r^2 2^-22, not
    // ~h^2 2^-24 (a false hit outside the sphere's box, which box culling precision then decides)
    const float s = hb * inv_a;
    const V3 f = madd(-s, d, oc);
    disc = a * fmaf(s0.w, s0.w, -dot(f, f));
  } else {
    const double ox = static_cast<double>(o.x) - static_cast<double>(C.x);
    const double oy = static_cast<double>(o.y) - static_cast<double>(C.y);
    const double oz = static_cast<double>(o.z) - static_cast<double>(C.z);
    const double r = static_cast<double>(s0.w);
    // r * r of a float r is exact in f64, so the fma's one rounding is the subtraction's
    c = static_cast<float>(fma(-r, r, ox * ox + oy * oy + oz * oz));
    disc = fmaf(hb, hb, -(a * c));
  }
  if (disc < 0.0f) return -1.0f;
  const float sq = sqrtf(disc);
  const float q = -(hb + copysignf(sq, hb));
  // |q| < 2^-100 (a ray tangent at its own origin, q would otherwise have no lower bound) counts as a
  // miss in the rtg-f32 spec (oracle/cpu_ref.c the same): div_rn is exact for every divisor left, and
  // the guard is the compare the q == 0 test already made (div_rn_wide, which scaled tiny
  // divisors instead, cost earth_perlin 4-6 % in register allocation, profiles/r03_c/ab_div_*)
  if (fabsf(q) < 0x1p-100f || a == 0.0f) return -1.0f;
  const float t0 = q * inv_a;
  const float t1 = div_rn(c, q);
  const float lo = fminf(t0, t1);
  const float hi = fmaxf(t0, t1);
  // roots inside (tmin, tmax), interval::surrounds (sphere.hpp:70); INCL: (tmin, tmax], so that the leaf test
  // sees a root equal to the closest hit and applies the exact-t tie rule (DESIGN.md §4 "tie rule")
  if (origin) return (hb < 0.0f && tmin < hi && (INCL ? hi <= tmax : hi < tmax)) ? hi : -1.0f;
  if (tmin < lo && (INCL ? lo <= tmax : lo < tmax)) return lo;
  if (tmin < hi && (INCL ? hi <= tmax : hi < tmax)) return hi;
  return -1.0f;
}

// Scene classes a kernel is compiled for (PRIMS): bits 0-1 the primitives its leaf test and shading
// handle — any (the scene's ref_mode decides at run time), spheres only, quads only — and bit 2 set when
// no material is metal or dielectric. The small-scene / dual-launch LDS kernels are built per class so
// a scene's kernel carries no code for what the scene lacks (default_kernel).
constexpr int kPrimsAny = 0, kPrimsSpheres = 1, kPrimsQuads = 2, kPrimsKind = 3, kPrimsDiffuse = 4;

// quad::hit (quad.hpp:44-114); plane distance D - n.O formed in f64.
// `rank`: the quad's list index (its record's v.w, DESIGN.md §4 "tie rule"), set with a hit. `brank`: the
// closest hit's rank (-1: a sphere or none); a root equal to tmax is a miss unless this quad comes later
// in the list than that hit (exact-t tie rule; compared on the hit path only). brank = -2: no tie check
// (the cache-read schedules settle ties after the call)
__device__ __forceinline__ float quad_t(const float4* q, V3 o, V3 d, float tmin, float tmax, int32_t brank,
                                        int32_t& rank) {
  const float4 q0 = q[0], q4 = q[4];
  const V3 n = xyz(q4);
  const float denom = dot(n, d);
  if (fabsf(denom) < 1e-8f) return -1.0f;
  // products of two floats are exact in f64, so the fma chain rounds exactly where mul + add would
  const double dn = fma(static_cast<double>(n.z), static_cast<double>(o.z),
                        fma(static_cast<double>(n.y), static_cast<double>(o.y),
                            static_cast<double>(n.x) * static_cast<double>(o.x)));
  const float num = static_cast<float>(static_cast<double>(q0.w) - dn);
  const float t = div_rn(num, denom);
  if (!(tmin <= t && t <= tmax)) return -1.0f;
  const V3 p = madd(t, d, o);
  const V3 hp = sub(p, xyz(q0));
  const float4 q2 = q[2];
  const V3 u = xyz(q[1]), v = xyz(q2), w = xyz(q[3]);
  const float alpha = dot(w, cross(hp, v));
  const float beta = dot(w, cross(u, hp));
  if (!(0.0f <= alpha && alpha <= 1.0f) || !(0.0f <= beta && beta <= 1.0f)) return -1.0f;
  rank = ibits(q2.w);
  if (t == tmax && rank <= brank) return -1.0f;
  return t;
}

// Exact-t ties (rtg-f32 spec, DESIGN.md §4 "tie rule"). The reference tests the world's objects in
// list order (hittable_list.hpp:40-64) against a shrinking interval: quad::hit accepts t ==
// closest_so_far (interval::contains, quad.hpp:62, interval.hpp:29), sphere::hit does not
// (interval::surrounds, sphere.hpp:70, interval.hpp:32). So among the primitives at the smallest t it
// keeps the last quad of the list if there is one, else the first sphere, whatever order they are tested
// in. The kernels test in BVH order: quad_t returns roots up to tmax, and a quad root equal to the closest
// hit replaces it only if that hit is a sphere or an earlier quad of the list (S.tie_rank: each slot's list
// index, read only on a tie; the check is one compare and a wave-uniform branch); the leaf tests take sphere
// roots up to tmax too (sphere_t<true>), and a sphere root equal to the closest hit replaces it only if that
// hit is a sphere later in the list, again with the ranks read only on a tie (tie_ranks_late). The sphere
// half (round 5) decides 14 pixels of the 10 M of configs 2 and 5 at full spp at no net cost (earlier forms
// that carried ranks through the loop cost 2-8 %: tools/experiments/sphere_tie_rule.patch).
__device__ __forceinline__ uint64_t ballot_tie(bool p) { return __builtin_amdgcn_ballot_w64(p); }
// S.tie_rank for the sphere tie rule, read from the kernel arguments at the (rare) tie itself: every kernel
// that runs leaf_step (render_kernel, render_kernel_lds) takes its DevScene as the first argument. A volatile
// load there keeps the pointer out of the SGPRs live across the trip loop; with S.tie_rank instead the
// compiler held it from the kernel's start and spilled other scalars to VGPR lanes (config 2 +0.7 %,
// config 3 +4.5 %, config 5 +1.2 %, frames identical)
__device__ __forceinline__ const int32_t* tie_ranks_late() {
  const volatile DevScene* ks = (const volatile DevScene*)(__builtin_amdgcn_kernarg_segment_ptr());
  return ks->tie_rank;
}
// The counting (COUNT) kernels check that assumption at every tie: a kernel whose first argument
// is not its DevScene reads another pointer there, reported as a corrupt render (rtg_render: RTG_E_INVALID);
// they then use S.tie_rank itself
template <bool COUNT>
__device__ __forceinline__ const int32_t* tie_ranks_at_tie(const DevScene& S, bool& corrupt) {
  const int32_t* r = tie_ranks_late();
  if (COUNT && r != S.tie_rank) {
    corrupt = true;
    return S.tie_rank;
  }
  return r;
}
// DevJob::tile_order read from the kernel arguments where a batch is handed out, as tie_ranks_late reads the
// tie ranks: J.tile_order itself was held in SGPRs from the kernel's start and pushed other scalars into VGPR
// lanes (config 2 +1 % with the order off). Every kernel that runs render_stream takes (DevScene, DevCamera,
// DevJob) by value, so DevJob sits at the offset below in the kernel-argument segment (arguments in order, each
// at its own alignment); the COUNT kernels compare the two pointers and report a mismatch as corrupt.
constexpr size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
constexpr size_t kDevJobKernarg =
    align_up(align_up(sizeof(DevScene), alignof(DevCamera)) + sizeof(DevCamera), alignof(DevJob));
template <bool COUNT>
__device__ __forceinline__ const int32_t* tile_order_late(const DevJob& J, bool& corrupt) {
  const char* ka = (const char*)(__builtin_amdgcn_kernarg_segment_ptr());
  const uint64_t v = reinterpret_cast<uint64_t>(
      *reinterpret_cast<const int32_t* const volatile*>(ka + kDevJobKernarg + offsetof(DevJob, tile_order)));
  // the load is a vector load: its (uniform) value back into SGPRs, so the null test is a scalar branch
  const int32_t* r = reinterpret_cast<const int32_t*>(
      (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v >> 32)))) << 32) |
      static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v & 0xffffffffu))));
  if (COUNT && r != J.tile_order) {
    corrupt = true;
    return J.tile_order;
  }
  return r;
}
// Cache-read schedules (Trav::mat holds the hit's material): the closest hit's rank is re-read from the
// list ranks, only on a tie (wave-uniform branch).
__device__ __forceinline__ bool quad_wins_tie(const DevScene& S, int32_t qrank, int32_t best) {
  if (!(best & kQuadRefBit)) return true;
  return qrank > S.tie_rank[S.num_spheres + (best & ~kQuadRefBit)];
}

template <bool COUNT>
struct Counts {
  uint32_t box = 0, prim = 0;
  uint32_t spill = 0;  // stack pushes into the global spill area (counters[26])
};

// Per-lane traversal state of the child-pair BVH (replaces hittable_list::hit -> bvh_node::hit
// -> aabb::hit, hittable_list.hpp:40-64, bvh_node.hpp:80-94, aabb.hpp:61-112). Ordered
// traversal: the nearer child first, the farther one pushed on the lane's LDS stack.
struct Trav {
  float ix, iy, iz;  // 1/d (approximate: culling only)
  float a, inv_a;    // d.d and its correctly rounded reciprocal (sphere_t)
  float ox, oy, oz;  // -o/d, for the fused slab test
  int32_t sx, sy, sz;  // 4-wide nodes: byte offset (0 or 48) of each axis' near-plane row
  float tbest;    // closest hit so far (the shrinking interval.max of the reference)
  int32_t best;   // primitive ref of the closest hit, -1 = none
  int32_t todo;   // inner node (>= 0: index, or byte offset in 4-wide trees) or leaf code (< 0)
  int32_t sp;     // stack depth
  int32_t origin; // primitive ref the ray starts on (-1: camera ray), DESIGN.md §4 "origin rule"
  int32_t mat;    // material of the closest hit: the cache-read schedules' shading then fetches the
                  // material beside the primitive instead of after it (one memory round trip less);
                  // in the LDS schedule instead the closest hit's tie rank (a quad's list index, -1
                  // for a sphere or none: the exact-t tie rule)
};

// todo of a finished traversal. "Traversal active" is this integer compare, not a bool of its own:
// a bool carried around the trip loop becomes a lane mask that every ballot copies into a VGPR and
// compares back (2 VALU per ballot); a compare of todo feeds s_bcnt1 / the exec mask directly.
constexpr int32_t kTravDone = INT32_MAX;
__device__ __forceinline__ bool trav_active(const Trav& t) { return t.todo != kTravDone; }
__device__ __forceinline__ bool at_inner(const Trav& t) {  // 0 <= todo < kTravDone
  return static_cast<uint32_t>(t.todo) < static_cast<uint32_t>(kTravDone);
}

template <int WIDE = 4>
__device__ __forceinline__ void trav_begin(Trav& t, const DevScene& S, V3 o, V3 d, int32_t origin) {
  t.ix = __builtin_amdgcn_rcpf(d.x);
  t.iy = __builtin_amdgcn_rcpf(d.y);
  t.iz = __builtin_amdgcn_rcpf(d.z);
  // byte offset of the far-plane rows (hi.x after lo.x, ...) in 4-wide nodes
  constexpr int32_t kHalf = 48;
  t.sx = (static_cast<uint32_t>(ibits(t.ix)) >> 31) * kHalf;
  t.sy = (static_cast<uint32_t>(ibits(t.iy)) >> 31) * kHalf;
  t.sz = (static_cast<uint32_t>(ibits(t.iz)) >> 31) * kHalf;
  t.a = dot(d, d);
  t.inv_a = div_rn(1.0f, t.a);
  t.ox = -o.x * t.ix;
  t.oy = -o.y * t.iy;
  t.oz = -o.z * t.iz;
  t.tbest = __builtin_inff();
  t.best = -1;
  t.mat = -1;  // no hit: tie rank -1 (LDS schedule; the cache-read schedules overwrite it on a hit)
  t.todo = S.num_nodes > 0 ? S.root_code : kTravDone;
  t.sp = 0;
  t.origin = origin;
}

// Per-lane traversal stacks, laid out [depth][lane] (bank-conflict-free ds_read/write_b32).
// LdsStack: all N entries in LDS. SpillStack: the first N entries in LDS, deeper ones (deep BVHs
// only, e.g. the 1M-sphere scene's 36-entry bound) in a global per-wave area of the same layout,
// so the LDS part stays small enough for full occupancy and no tree is too deep.
template <int N>
struct LdsStack {
  int32_t* lds;
  __device__ __forceinline__ bool spills(int32_t) const { return false; }
  __device__ __forceinline__ int32_t capacity() const { return N; }
  __device__ __forceinline__ void store(int32_t sp, int32_t v) const { lds[sp * 64] = v; }
  __device__ __forceinline__ int32_t load(int32_t sp) const { return lds[sp * 64]; }
};
// LdsStack16: 16-bit entries for the LDS schedule of 4-wide trees whose codes fit an int16: the node
// array sits at LDS address 0, so inner-node codes (absolute LDS byte addresses) stay below 32768
// for trees of <= 292 nodes, and leaf codes ~((first << 3) | (count - 1)) need first < 4096 (the host
// checks both, the kernel re-checks the node range): half the LDS of 32-bit entries, which is what
// lets a second persistent launch share the CU with book-1 (DESIGN.md §3 "occupancy").
template <int N>
struct LdsStack16 {
  int16_t* lds;
  __device__ __forceinline__ bool spills(int32_t) const { return false; }
  __device__ __forceinline__ int32_t capacity() const { return N; }
  __device__ __forceinline__ void store(int32_t sp, int32_t v) const { lds[sp * 64] = static_cast<int16_t>(v); }
  __device__ __forceinline__ int32_t load(int32_t sp) const { return lds[sp * 64]; }
};
template <int N>
struct SpillStack {
  int32_t* lds;
  int32_t* spill;  // this lane's global area, entries n.. at spill[(sp - n) * 64]
  int32_t n;       // entries kept in LDS (<= N; J.lds_stack, lowered only by tests)
  int32_t cap;     // n + spill depth
  __device__ __forceinline__ bool spills(int32_t sp) const { return sp >= n; }
  __device__ __forceinline__ int32_t capacity() const { return cap; }
  __device__ __forceinline__ void store(int32_t sp, int32_t v) const {
    if (__builtin_expect(sp < n, 1))
      lds[sp * 64] = v;
    else
      spill[(sp - n) * 64] = v;
  }
  __device__ __forceinline__ int32_t load(int32_t sp) const {
    int32_t v;
    if (__builtin_expect(sp < n, 1))
      v = lds[sp * 64];
    else
      v = spill[(sp - n) * 64];
    return v;
  }
};

template <class Stk>
__device__ __forceinline__ void trav_pop(Trav& t, const Stk& stk) {
  if (t.sp == 0) {
    t.todo = kTravDone;
    return;
  }
  --t.sp;
  t.todo = stk.load(t.sp);
}

// Visit one inner node (t.todo >= 0): test both child boxes, continue with the nearer hit child
// and push the farther one, or pop when neither is hit.
template <class Stk, bool COUNT>
__device__ __forceinline__ void node_step(Trav& t, const DevScene& S, const Stk& stk, Counts<COUNT>& cnt,
                                          bool& overflow, bool& corrupt) {
  if (t.todo >= S.num_nodes) {  // corrupt child code: report, never read out of bounds
    corrupt = true;
    t.todo = kTravDone;
    return;
  }
  const float4* n = S.nodes + static_cast<int64_t>(t.todo) * 4;
  const float4 a = n[0], b = n[1], c = n[2];
  const int4 ch = *reinterpret_cast<const int4*>(n + 3);
  if (COUNT) cnt.box += 2;
  const V3 inv = v3(t.ix, t.iy, t.iz), oi = v3(t.ox, t.oy, t.oz);
  // left box lo=(a.x,a.y,a.z) hi=(a.w,b.x,b.y); right lo=(b.z,b.w,c.x) hi=(c.y,c.z,c.w)
  const float l0x = fmaf(a.x, inv.x, oi.x), l1x = fmaf(a.w, inv.x, oi.x);
  const float l0y = fmaf(a.y, inv.y, oi.y), l1y = fmaf(b.x, inv.y, oi.y);
  const float l0z = fmaf(a.z, inv.z, oi.z), l1z = fmaf(b.y, inv.z, oi.z);
  const float r0x = fmaf(b.z, inv.x, oi.x), r1x = fmaf(c.y, inv.x, oi.x);
  const float r0y = fmaf(b.w, inv.y, oi.y), r1y = fmaf(c.z, inv.y, oi.y);
  const float r0z = fmaf(c.x, inv.z, oi.z), r1z = fmaf(c.w, inv.z, oi.z);
  const float tc = cull_bound(t.tbest);
  const float ln = fmaxf(fmaxf(fminf(l0x, l1x), fminf(l0y, l1y)), fmaxf(fminf(l0z, l1z), kCullTMin));
  const float lf = fminf(fminf(fminf(fmaxf(l0x, l1x), fmaxf(l0y, l1y)), fmaxf(l0z, l1z)) * kCullWiden, tc);
  const float rn = fmaxf(fmaxf(fminf(r0x, r1x), fminf(r0y, r1y)), fmaxf(fminf(r0z, r1z), kCullTMin));
  const float rf = fminf(fminf(fminf(fmaxf(r0x, r1x), fmaxf(r0y, r1y)), fmaxf(r0z, r1z)) * kCullWiden, tc);
  // An empty slot (right child only; the host guarantees the left one is never empty) has an
  // inverted box, which the symmetric min/max slab form would report as all of space: test
  // the child code explicitly.
  const bool hl = ln <= lf;
  const bool hr = rn <= rf && ch.y != kEmptyChild;
  if (hl && hr) {
    const bool lfirst = ln <= rn;
    if (COUNT) cnt.spill += stk.spills(t.sp) ? 1u : 0u;
    if (t.sp < stk.capacity()) {
      stk.store(t.sp, lfirst ? ch.y : ch.x);
      ++t.sp;
    } else {
      overflow = true;
    }
    t.todo = lfirst ? ch.x : ch.y;
  } else if (hl || hr) {
    t.todo = hl ? ch.x : ch.y;
  } else {
    trav_pop(t, stk);
  }
}

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float nf4 __attribute__((ext_vector_type(4)));
// LDS loads from 32-bit LDS byte addresses (no generic-pointer base arithmetic)
__device__ __forceinline__ nf4 lds_ld4(uint32_t a) {
  return *reinterpret_cast<__attribute__((address_space(3))) const nf4*>(static_cast<uintptr_t>(a));
}
__device__ __forceinline__ int32_t lds_ld1(uint32_t a) {
  return *reinterpret_cast<__attribute__((address_space(3))) const int32_t*>(static_cast<uintptr_t>(a));
}
__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// Entry distance of one child (tn) or a miss: the slab test with the near/far planes already
// chosen by the ray's direction signs, so no min/max between a slab's two planes is needed.
// tc: the cull bound of the closest hit so far (cull_bound)
__device__ __forceinline__ uint32_t child_key(float tnx, float tny, float tnz, float tfx, float tfy, float tfz,
                                              float tc, uint32_t slot) {
  const float tn = fmaxf(fmaxf(fmaxf(tnx, tny), tnz), kCullTMin);
  const float tf = fminf(fminf(fminf(tfx, tfy), tfz), tc);
  // tn >= kCullTMin > 0, so its bits order like the float; the low 4 bits carry the slot (x4)
  return tn <= tf ? ((static_cast<uint32_t>(ibits(tn)) & ~15u) | slot) : ~0u;
}
// the same with the bound already formed (quad kernels: min(exit, tbest) * kCullWiden)
__device__ __forceinline__ uint32_t child_key_exit(float tnx, float tny, float tnz, float tf, uint32_t slot) {
  const float tn = fmaxf(fmaxf(fmaxf(tnx, tny), tnz), kCullTMin);
  return tn <= tf ? ((static_cast<uint32_t>(ibits(tn)) & ~15u) | slot) : ~0u;
}

__device__ __forceinline__ void psort(uint32_t& ka, int32_t& ca, uint32_t& kb, int32_t& cb) {
  const bool sw = kb < ka;
  const uint32_t k = sw ? kb : ka;
  const int32_t c = sw ? cb : ca;
  kb = sw ? ka : kb;
  cb = sw ? ca : cb;
  ka = k;
  ca = c;
}

__device__ __forceinline__ void usort(uint32_t& a, uint32_t& b) {
  const uint32_t lo = min(a, b);
  b = max(a, b);
  a = lo;
}

// Visit one 4-wide node (SoA rows lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, code; 16 B each). Per ray
// the near plane of each axis is fixed by the sign of 1/d (Trav::sx/sy/sz pick the row), so each
// child costs 6 fma (packed two children per v_pk_fma_f32) + max3/max + min3/min. The four hit
// children are sorted as integer keys (entry distance with the slot in the low bits) by a
// 5-comparator min/max network; the nearest becomes the next node, the others are pushed
// far-to-near. Empty slots hold the inverted box (+inf, -inf): whatever the signs, at least one
// axis has a finite 1/d, for which the near plane gives tn = +inf and the far one tf = -inf, so an
// empty slot can never be entered (rays with all three components zero do not exist).
// Node geometry of a schedule: where node rows are read from.
enum Geom : int {
  kGeomLds = 0,      // whole scene in LDS; inner codes are absolute LDS addresses, codes read after the sort
  kGeomGlobal = 1,   // scene through the caches; codes travel with their keys through the sort network
  kGeomTreelet = 2,  // nodes below S.treelet_bytes from their LDS copy, the rest through the caches
};

// WIDEN (kernels that test quads): exit distances widened by kCullWiden (DESIGN.md §4 "conservative culling").
template <class Stk, bool COUNT, int GEOM, bool WIDEN = true>
__device__ __forceinline__ void node_step4(Trav& t, const DevScene& S, const Stk& stk, Counts<COUNT>& cnt,
                                           bool& overflow, bool& corrupt) {
  constexpr bool PAIRS = GEOM != kGeomLds;
  // 4-wide inner-node codes are byte offsets into the node array (node index * 112)
  // corrupt codes: checked wherever a bad code could fault (nodes through the vector-memory path)
  // and in the COUNT diagnostics; an LDS read outside the allocation cannot fault, and the host
  // validated the tree it copied there, so the hot LDS schedule skips the compare-and-branch
  if ((GEOM != kGeomLds || COUNT) && t.todo >= S.node_limit) {
    corrupt = true;
    t.todo = kTravDone;
    return;
  }
  // the probe of the hot treelet counts every visit of a node held in HBM (rtg_api.cpp tune_treelet)
  if (COUNT && GEOM != kGeomLds && S.node_visits) atomicAdd(S.node_visits + t.todo / 112, 1u);
  const char* nb = reinterpret_cast<const char*>(S.nodes) + t.todo;
  const int32_t sx = t.sx, sy = t.sy, sz = t.sz;
  const uint32_t na = static_cast<uint32_t>(t.todo);  // LDS scenes: the node's LDS address
  nf4 nx, ny, nz, fx, fy, fz;
  int4 cc;
  if constexpr (GEOM == kGeomLds) {
    nx = lds_ld4(na + sx), ny = lds_ld4(na + 16 + sy), nz = lds_ld4(na + 32 + sz);
    fx = lds_ld4(na + 48 - sx), fy = lds_ld4(na + 64 - sy), fz = lds_ld4(na + 80 - sz);
  } else {
    if (GEOM == kGeomTreelet && t.todo < S.treelet_bytes) {  // the top of the tree: a ds_read
      const uint32_t la = S.treelet_lds + na;
      nx = lds_ld4(la + sx), ny = lds_ld4(la + 16 + sy), nz = lds_ld4(la + 32 + sz);
      fx = lds_ld4(la + 48 - sx), fy = lds_ld4(la + 64 - sy), fz = lds_ld4(la + 80 - sz);
      const nf4 c4 = lds_ld4(la + 96);
      cc = *reinterpret_cast<const int4*>(&c4);
    } else {
      auto row = [&](int32_t off) -> nf4 { return *reinterpret_cast<const nf4*>(nb + off); };
      nx = row(sx), ny = row(16 + sy), nz = row(32 + sz);
      fx = row(48 - sx), fy = row(64 - sy), fz = row(80 - sz);
      cc = *reinterpret_cast<const int4*>(nb + 96);
    }
  }
  if (COUNT) cnt.box += 4;
  const f2 ix = {t.ix, t.ix}, iy = {t.iy, t.iy}, iz = {t.iz, t.iz};
  const f2 ox = {t.ox, t.ox}, oy = {t.oy, t.oy}, oz = {t.oz, t.oz};
  const f2 nx01 = pk_fma(f2{nx.x, nx.y}, ix, ox), nx23 = pk_fma(f2{nx.z, nx.w}, ix, ox);
  const f2 ny01 = pk_fma(f2{ny.x, ny.y}, iy, oy), ny23 = pk_fma(f2{ny.z, ny.w}, iy, oy);
  const f2 nz01 = pk_fma(f2{nz.x, nz.y}, iz, oz), nz23 = pk_fma(f2{nz.z, nz.w}, iz, oz);
  const f2 fx01 = pk_fma(f2{fx.x, fx.y}, ix, ox), fx23 = pk_fma(f2{fx.z, fx.w}, ix, ox);
  const f2 fy01 = pk_fma(f2{fy.x, fy.y}, iy, oy), fy23 = pk_fma(f2{fy.z, fy.w}, iy, oy);
  const f2 fz01 = pk_fma(f2{fz.x, fz.y}, iz, oz), fz23 = pk_fma(f2{fz.z, fz.w}, iz, oz);
  uint32_t k0, k1, k2, k3;
  if constexpr (WIDEN) {  // min(exit, tbest) * kCullWiden: one v_pk_mul_f32 per child pair, no cull_bound
    const float tb = t.tbest;
    const f2 tf01 = f2{fminf(fminf(fminf(fx01.x, fy01.x), fz01.x), tb), fminf(fminf(fminf(fx01.y, fy01.y), fz01.y), tb)} *
                    f2{kCullWiden, kCullWiden};
    const f2 tf23 = f2{fminf(fminf(fminf(fx23.x, fy23.x), fz23.x), tb), fminf(fminf(fminf(fx23.y, fy23.y), fz23.y), tb)} *
                    f2{kCullWiden, kCullWiden};
    k0 = child_key_exit(nx01.x, ny01.x, nz01.x, tf01.x, 0);
    k1 = child_key_exit(nx01.y, ny01.y, nz01.y, tf01.y, 4);
    k2 = child_key_exit(nx23.x, ny23.x, nz23.x, tf23.x, 8);
    k3 = child_key_exit(nx23.y, ny23.y, nz23.y, tf23.y, 12);
  } else {
    const float tc = cull_bound(t.tbest);
    k0 = child_key(nx01.x, ny01.x, nz01.x, fx01.x, fy01.x, fz01.x, tc, 0);
    k1 = child_key(nx01.y, ny01.y, nz01.y, fx01.y, fy01.y, fz01.y, tc, 4);
    k2 = child_key(nx23.x, ny23.x, nz23.x, fx23.x, fy23.x, fz23.x, tc, 8);
    k3 = child_key(nx23.y, ny23.y, nz23.y, fx23.y, fy23.y, fz23.y, tc, 12);
  }
  if constexpr (PAIRS) {
    // scene in global memory: the codes travel with their keys through the network, so no second
    // memory round trip sits between the sort and the next node load (-3.6 % on config 5; with
    // the scene in LDS the extra selects cost more than the LDS latency they save)
    int32_t c0 = cc.x, c1 = cc.y, c2 = cc.z, c3 = cc.w;
    psort(k0, c0, k1, c1);
    psort(k2, c2, k3, c3);
    psort(k0, c0, k2, c2);
    psort(k1, c1, k3, c3);
    psort(k1, c1, k2, c2);
    if (k0 == ~0u) {
      trav_pop(t, stk);
      return;
    }
    const int npush = (k1 != ~0u) + (k2 != ~0u) + (k3 != ~0u);
    if (COUNT)
      for (int j = 0; j < npush; ++j) cnt.spill += stk.spills(t.sp + j) ? 1u : 0u;
    if (t.sp + npush > stk.capacity()) {
      overflow = true;
    } else {
      if (k3 != ~0u) stk.store(t.sp++, c3);
      if (k2 != ~0u) stk.store(t.sp++, c2);
      if (k1 != ~0u) stk.store(t.sp++, c1);
    }
    t.todo = c0;
  } else {
    usort(k0, k1);
    usort(k2, k3);
    usort(k0, k2);
    usort(k1, k3);
    usort(k1, k2);
    if (k0 == ~0u) {
      trav_pop(t, stk);
      return;
    }
    // node addresses are 16-byte aligned (112-byte nodes from an aligned base), so the code of
    // slot (k & 12) / 4 is at (node | (k & 12)) + 96: one v_and_or per code
    auto code_of = [&](uint32_t k) { return lds_ld1((na | (k & 12u)) + 96u); };
    // the host sizes every stack from the tree's structural bound (sum of siblings along a path,
    // Bvh4::max_pushes), so pushes cannot overflow; the check runs in the COUNT diagnostics only
    const int npush = (k1 != ~0u) + (k2 != ~0u) + (k3 != ~0u);
    if (COUNT)
      for (int j = 0; j < npush; ++j) cnt.spill += stk.spills(t.sp + j) ? 1u : 0u;
    if (COUNT && t.sp + npush > stk.capacity()) {
      overflow = true;
    } else {
      if (k3 != ~0u) stk.store(t.sp++, code_of(k3));
      if (k2 != ~0u) stk.store(t.sp++, code_of(k2));
      if (k1 != ~0u) stk.store(t.sp++, code_of(k1));
    }
    t.todo = code_of(k0);
  }
}

// Test the primitives of a leaf (t.todo < 0). ONE: only the first, and the lane stays at the rest of the leaf
// (first + 1, count - 1) for its next leaf trip, or pops after the last: one primitive per lane per trip
// keeps the leaf trip's lanes in step (a loop over each lane's own count runs as long as the wave's largest
// leaf): config 2 -0.5 %, config 5 -0.4 %, Cornell +0.3 %, frames identical. The tile-ring kernels of the
// cache-read schedules loop over the leaf and pop (config 5 with the ring: one per trip +1.4 %; DESIGN.md §8
// round 5). Either way a lane tests its primitives in the same order, so ties resolve the same way. CHECK:
// validate the leaf code (off in the LDS schedule outside the COUNT diagnostics, as for node codes).
template <class Stk, bool COUNT, bool CHECK = true, bool MAT = false, int WIDE = 4, int GEOM = kGeomLds,
          int PRIMS = kPrimsAny, bool ONE = true>
__device__ __forceinline__ void leaf_step(Trav& t, const DevScene& S, V3 o, V3 d, float time,
                                          const Stk& stk, Counts<COUNT>& cnt, bool& corrupt) {
  auto pop = [&]() { trav_pop(t, stk); };
  const int32_t code = ~t.todo;
  const int32_t first = code >> 3;
  const int32_t count = (code & 7) + 1;
  if ((CHECK || COUNT) && static_cast<int64_t>(first) + count > S.num_refs) {
    corrupt = true;
    t.todo = kTravDone;
    return;
  }
  if ((PRIMS & kPrimsKind) == kPrimsSpheres || ((PRIMS & kPrimsKind) == kPrimsAny && S.ref_mode == 1)) {  // sphere-only scene, primitives stored in reference order
    for (int k = 0; k < (ONE ? 1 : count); ++k) {
      const float4* sp4 = S.spheres + static_cast<int64_t>(first + k) * S.sphere_f4;
      if (COUNT) cnt.prim += 1;
      const float th = sphere_t<true>(sp4[0], sp4[1], o, d, t.a, t.inv_a, time, kTMin, t.tbest, first + k == t.origin);
      // exact-t tie (rare; a wave-uniform branch): the sphere earlier in the list wins, as the reference's list
      // walk keeps the first sphere at a t (interval::surrounds); the ranks are read only then (tie_ranks_late)
      bool take = th > 0.0f && th < t.tbest;
      if (ballot_tie(th == t.tbest) != 0 && th == t.tbest) {
        const int32_t* rk = tie_ranks_at_tie<COUNT>(S, corrupt);
        take = rk[first + k] < rk[t.best];
      }
      if (take) {
        t.tbest = th;
        t.best = first + k;
        t.mat = MAT ? ibits(sp4[1].w) : -1;
      }
    }
    if (ONE && count > 1)
      t.todo = ~(((first + 1) << 3) | (count - 2));
    else
      pop();
    return;
  }
  for (int k = 0; k < (ONE ? 1 : count); ++k) {
    const int32_t ref = S.ref_mode == 0 ? S.refs[first + k] : ((first + k) | kQuadRefBit);
    float th;
    if (COUNT) cnt.prim += 1;
    int32_t m = 0, qrank = -1;
    bool take;
    if ((PRIMS & kPrimsKind) == kPrimsQuads || (ref & kQuadRefBit)) {  // planar: a ray leaving a quad never hits it again
      const float4* q = S.quads + static_cast<int64_t>(ref & ~kQuadRefBit) * 5;
      // exact-t tie rule: a quad root equal to the closest hit replaces it only if that
      // is a sphere or an earlier quad of the list. LDS schedule: t.mat holds the closest hit's rank and
      // quad_t rejects a losing tie on its hit path; cache-read schedules (t.mat = material): the rank
      // is re-read, only on a tie
      th = ref == t.origin ? -1.0f : quad_t(q, o, d, kTMin, t.tbest, MAT ? -2 : t.mat, qrank);
      if (MAT && th > 0.0f) m = ibits(q[1].w);
      take = th > 0.0f;
      if constexpr (MAT) {
        if (ballot_tie(th == t.tbest) != 0 && th == t.tbest) take = quad_wins_tie(S, qrank, t.best);
      }
    } else {
      const float4* sp4 = S.spheres + static_cast<int64_t>(ref) * S.sphere_f4;
      th = sphere_t<true>(sp4[0], sp4[1], o, d, t.a, t.inv_a, time, kTMin, t.tbest, ref == t.origin);
      if (MAT) m = ibits(sp4[1].w);
      take = th > 0.0f && th < t.tbest;
      // exact-t tie: a sphere replaces only an equal-t sphere later in the list (never a quad)
      if (ballot_tie(th == t.tbest) != 0 && th == t.tbest) {
        const int32_t* rk = tie_ranks_at_tie<COUNT>(S, corrupt);
        take = !(t.best & kQuadRefBit) && rk[ref] < rk[t.best];
      }
    }
    if (take) {  // th > tmin >= 0.001 on a hit
      t.tbest = th;
      t.best = ref;
      t.mat = MAT ? m : qrank;
    }
  }
  if (ONE && count > 1)
    t.todo = ~(((first + 1) << 3) | (count - 2));
  else
    pop();
}

// ---------------------------------------------------------------------------------------
// Textures (texture.hpp:34-151, perlin.hpp:95-158, 219-255)
// LDS: the gradient rows and permutation words are the workgroup's LDS copy, whose Z words carry the
// rows' LDS address (render_lds_scene), so a corner's offset is its row's LDS address; else offsets are
// relative to `vec` (global memory)
template <bool LDS>
__device__ float perlin_noise(const float4* vec, const uint32_t* perm, V3 p) {
  const float fx = floorf(p.x), fy = floorf(p.y), fz = floorf(p.z);
  const float u = p.x - fx, v = p.y - fy, w = p.z - fz;
  const int i = static_cast<int>(fx), j = static_cast<int>(fy), k = static_cast<int>(fz);
  // Hermite weights u u (3 - 2 u) (perlin.hpp:226-228): 2 u is exact, so the one-rounding fmaf(-2, u, 3)
  // is bit for bit the spec's 3 - 2 u (cpu_ref32), one VALU op fewer per axis
  const float uu = u * u * fmaf(-2.0f, u, 3.0f);
  const float vv = v * v * fmaf(-2.0f, v, 3.0f);
  const float ww = w * w * fmaf(-2.0f, w, 3.0f);
  // both corner entries of each axis in one read (the words of rtg_internal.hpp kPerlinPermWords), all
  // three issued before any is used (round 2: one LDS round trip per octave; config 3 shades 7 octaves
  // per ground hit); X ^ Y[dj] ^ Z[dk] holds the gradient offsets of corners (0, dj, dk) and (1, dj, dk)
  const uint32_t px = perm[i & 255];
  const uint2 py = reinterpret_cast<const uint2*>(perm + 256)[j & 255];
  const uint2 pz = reinterpret_cast<const uint2*>(perm + 768)[k & 255];
  auto grad = [&](uint32_t off) -> V3 {
    if constexpr (LDS) {
      typedef float nf3 __attribute__((ext_vector_type(3)));
      const nf3 g = *reinterpret_cast<__attribute__((address_space(3))) const nf3*>(static_cast<uintptr_t>(off));
      return v3(g.x, g.y, g.z);
    } else {
      return xyz(*reinterpret_cast<const float4*>(reinterpret_cast<const unsigned char*>(vec) + off));
    }
  };
  float accum = 0.0f;
  // the corner gradients in pairs (di, dj fixed; dk = 0, 1), each pair fetched (xyz only) before it
  // is used and the sum in the reference's corner order: fetching all eight float4s at once (round 2)
  // saved LDS round trips but made the textured kernel spill its path state to scratch at 5 waves
  // per SIMD (config 3: 97 GB of scratch write traffic per frame, TA 69 % busy, profiles/r03_c)
#pragma unroll
  for (int di = 0; di < 2; ++di) {
#pragma unroll
    for (int dj = 0; dj < 2; ++dj) {
      const uint32_t pxy = px ^ (dj ? py.y : py.x);
      const uint32_t ph = di ? pxy >> 16 : pxy;
      const uint32_t o0 = (ph ^ pz.x) & 0xffffu;
      const uint32_t o1 = (ph ^ pz.y) & 0xffffu;
      const V3 g0 = grad(o0), g1 = grad(o1);
#pragma unroll
      for (int dk = 0; dk < 2; ++dk) {
        const V3 c = dk ? g1 : g0;
        const V3 wv = v3(u - di, v - dj, w - dk);
        const float fu = di ? uu : (1.0f - uu);
        const float fv = dj ? vv : (1.0f - vv);
        const float fw = dk ? ww : (1.0f - ww);
        accum = fmaf(fu * fv * fw, dot(c, wv), accum);
      }
      // one pair of gradient rows in flight at a time: the scheduler otherwise issues six of the eight
      // reads at once and the textured kernel spills 16 B/lane (round 6)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  return accum;
}

template <bool LDS>
__device__ float perlin_turb(const float4* vec, const uint32_t* perm, V3 p) {
  float accum = 0.0f, weight = 1.0f;
  V3 tp = p;
  for (int i = 0; i < 7; ++i) {  // not unrolled: 2 octaves at once ±0, all 7 spill 576 B/lane (7x slower)
    accum = fmaf(weight, perlin_noise<LDS>(vec, perm, tp), accum);
    weight *= 0.5f;
    tp = scl(2.0f, tp);
  }
  return fabsf(accum);
}

// FULL = false compiles solid and checker textures only (scenes without image / noise textures):
// the perlin and image paths cost ~12 vector registers the common scenes would otherwise spill.
// LDS_TAB: the perlin tables are the workgroup's LDS copy (perlin_noise)
template <bool FULL, bool LDS_TAB = false>
__device__ V3 texture_value(const DevScene& S, int32_t tex, float u, float v, V3 p) {
  // a checker resolves to another texture: one trip per nesting level (solid under checker: 2);
  // not unrolled (16 unrolled copies cost ~70 scalar branch instructions per shade)
#pragma unroll 1
  for (int guard = 0; guard < kMaxTexNesting; ++guard) {
    const float4 t0 = S.textures[tex * 2];
    const float4 t1 = S.textures[tex * 2 + 1];
    const int type = ibits(t0.x);
    if (type == RTG_TEX_SOLID) return xyz(t1);
    if (type == RTG_TEX_CHECKER) {
      const float inv_scale = t0.w;
      const int xi = static_cast<int>(floorf(inv_scale * p.x));
      const int yi = static_cast<int>(floorf(inv_scale * p.y));
      const int zi = static_cast<int>(floorf(inv_scale * p.z));
      const bool even = ((xi + yi + zi) % 2) == 0;
      tex = even ? ibits(t0.y) : ibits(t0.z);
      continue;
    }
    if (FULL && type == RTG_TEX_IMAGE) {
      const int img = ibits(t1.w);
      if (img < 0) return v3(0.0f, 1.0f, 1.0f);
      const int4 h = S.images[img];
      if (h.y <= 0) return v3(0.0f, 1.0f, 1.0f);
      // the empty asm keeps v's flip here: hoisted out of the nesting loop (it is loop-invariant), 1 - v
      // outlived the loop in scratch (config 3's textured kernel, round 6)
      float vin = v;
      __asm__ volatile("" : "+v"(vin));
      const float uc = fminf(fmaxf(u, 0.0f), 1.0f);
      const float vc = 1.0f - fminf(fmaxf(vin, 0.0f), 1.0f);
      int i = static_cast<int>(uc * static_cast<float>(h.x));
      int j = static_cast<int>(vc * static_cast<float>(h.y));
      i = i < 0 ? 0 : (i < h.x ? i : h.x - 1);
      j = j < 0 ? 0 : (j < h.y ? j : h.y - 1);
      const uint64_t off = (static_cast<uint64_t>(static_cast<uint32_t>(h.w)) << 32) |
                           static_cast<uint32_t>(h.z);
      const uint8_t* px = S.texels + off + (static_cast<int64_t>(j) * h.x + i) * 3;
      const float cs = 1.0f / 255.0f;
      return v3(cs * px[0], cs * px[1], cs * px[2]);
    }
    if (FULL && type == RTG_TEX_NOISE) {
      const int pt = ibits(t1.w);
      const float4* vec = S.perlin_vec + pt * 256;
      const uint32_t* perm = S.perlin_perm + pt * kPerlinPermWords;
      const float t = perlin_turb<LDS_TAB>(vec, perm, p);
      const float s = 0.5f * (1.0f + sin_spec(fmaf(t0.w, p.z, 10.0f * t)));
      return v3(s, s, s);
    }
    break;
  }
  return v3(1.0f, 0.0f, 1.0f);
}

// ---------------------------------------------------------------------------------------
struct PathState {
  V3 o, d;
  float time;
  V3 T, L;
  int depth;
  int32_t origin;  // primitive ref the current segment starts on (-1: camera ray)
  uint64_t rng;
};

// get_ray (camera.hpp:139-177): jitter x then y, lens disk (rejection), time.
__device__ __forceinline__ void start_sample(PathState& ps, const DevCamera& C, uint64_t seed_mix,
                                             uint32_t pixel_id, uint32_t sample, int i, int j) {
  ps.rng = mix64(((static_cast<uint64_t>(pixel_id) << 32) | sample) ^ seed_mix);
  const float ox = fmaf(draw24(ps.rng), 0x1p-24f, -0.5f);  // U - 0.5 (U exact: one rounding either way)
  const float oy = fmaf(draw24(ps.rng), 0x1p-24f, -0.5f);
  const float fi = static_cast<float>(i) + ox;
  const float fj = static_cast<float>(j) + oy;
  const V3 p00 = v3(C.pixel00[0], C.pixel00[1], C.pixel00[2]);
  const V3 du = v3(C.du[0], C.du[1], C.du[2]);
  const V3 dv = v3(C.dv[0], C.dv[1], C.dv[2]);
  const V3 sample_pt = madd(fj, dv, madd(fi, du, p00));
  V3 origin = v3(C.center[0], C.center[1], C.center[2]);
  if (C.defocus) {
    // random_in_unit_disk (vec3.hpp:158-169), direct: radius sqrt(U), angle from a second U
    const float r = sqrt_rn(uniform(ps.rng));
    float sn, cs;
    sincos_turn4(draw24(ps.rng) * 0x1p-22f, sn, cs);
    const float px = r * cs, py = r * sn;
    origin = madd(py, v3(C.defv[0], C.defv[1], C.defv[2]), madd(px, v3(C.defu[0], C.defu[1], C.defu[2]), origin));
  }
  ps.o = origin;
  ps.d = sub(sample_pt, origin);
  ps.time = uniform(ps.rng);
  ps.T = v3(1.0f, 1.0f, 1.0f);
  ps.L = v3(0.0f, 0.0f, 0.0f);
  ps.depth = C.max_depth;
  ps.origin = -1;
}

// Shades the closest hit `ref` at distance t; returns false when the path ends
// (ray_color's emission-only return, camera.hpp:213-216, or a miss handled by the caller).
// MAT: `mat` is the hit's material (Trav::mat), so its record is fetched beside the primitive's
// (the cache-read schedules: two independent loads instead of a dependent pair)
// PRIMS: the scene class (kPrimsAny ...): sphere-only kernels shade spheres only, quad-only ones quads
// only (chosen only without a sphere occluder), diffuse-only ones have no metal / dielectric code
// LDS_TAB: the perlin tables are in LDS (the whole-scene LDS schedule's textured kernels)
template <bool FULL, bool MAT = false, int PRIMS = kPrimsAny, bool LDS_TAB = false>
__device__ bool shade(const DevScene& S, PathState& ps, int32_t ref, float t, int32_t mat_hit = 0) {
  V3 p, outward;
  float u = 0.0f, v = 0.0f;
  int mat;
  const bool sphere = (PRIMS & kPrimsKind) == kPrimsSpheres ||
                      ((PRIMS & kPrimsKind) == kPrimsAny && !(ref & kQuadRefBit));
  if (sphere) {
    const float4* s = S.spheres + static_cast<int64_t>(ref) * S.sphere_f4;
    const float4 s0 = s[0], s1 = s[1];
    const V3 C = madd(ps.time, xyz(s1), xyz(s0));
    p = madd(t, ps.d, ps.o);
    outward = scl(div_rn(1.0f, s0.w), sub(p, C));
    mat = MAT ? mat_hit : ibits(s1.w);
  } else {
    const float4* q = S.quads + static_cast<int64_t>(ref & ~kQuadRefBit) * 5;
    const float4 q0 = q[0];
    p = madd(t, ps.d, ps.o);
    const V3 hp = sub(p, xyz(q0));
    const V3 w = xyz(q[3]);
    u = dot(w, cross(hp, xyz(q[2])));
    v = dot(w, cross(xyz(q[1]), hp));
    outward = xyz(q[4]);
    mat = MAT ? mat_hit : ibits(q[1].w);
  }
  const bool front = dot(ps.d, outward) < 0.0f;  // set_face_normal, hittable.hpp:29-35
  const V3 n = front ? outward : neg(outward);
  const float4 m0 = S.materials[mat * 2];
  const float4 m1 = S.materials[mat * 2 + 1];
  const int type = ibits(m0.x);
  const int tex = ibits(m0.y);
  const bool needs_uv = sphere && ibits(m1.w) != 0;  // texture (transitively) is an image

  // texture coordinates on spheres are only consumed by image textures
  auto sphere_uv = [&]() {
    const float theta = acos_spec(-outward.y);
    const float phi = atan2_spec(-outward.z, outward.x) + kPi;
    u = div_rn(phi, 2.0f * kPi);
    v = div_rn(theta, kPi);
  };

  if (type == RTG_MAT_DIFFUSE_LIGHT) {
    if (needs_uv) sphere_uv();
    const V3 e = tex < 0 ? xyz(m1) : texture_value<FULL, LDS_TAB>(S, tex, u, v, p);  // < 0: solid colour inline
    ps.L = vfma(ps.T, e, ps.L);
    return false;
  }
  V3 dir, att;
  constexpr bool kDiffuse = (PRIMS & kPrimsDiffuse) != 0;
  if (type == RTG_MAT_LAMBERTIAN || (!kDiffuse && type == RTG_MAT_METAL)) {
    // the albedo first (it draws no random numbers): with the direction drawn first, one of its uniforms
    // stayed live across the texture evaluation and went to scratch in the textured kernel (round 6)
    if (kDiffuse || type == RTG_MAT_LAMBERTIAN) {
      if (needs_uv) sphere_uv();
      att = tex < 0 ? xyz(m1) : texture_value<FULL, LDS_TAB>(S, tex, u, v, p);
    }
    // both scatter around a random unit vector: one sampling code path for the lanes of either
    const V3 r = random_unit_vector(ps.rng);
    if (kDiffuse || type == RTG_MAT_LAMBERTIAN) {
      dir = add(n, r);
      // near_zero with the reference's fabs(e[1] < s) quirk (vec3.hpp:70-77, H5)
      const float s = 1e-8f;
      if (fabsf(dir.x) < s && dir.y < s && fabsf(dir.z) < s) dir = n;
    } else {
      const V3 in = ps.d;
      const V3 refl = madd(-(2.0f * dot(in, n)), n, in);
      dir = madd(m0.z, r, unit(refl));
      att = xyz(m1);
      if (!(dot(dir, n) > 0.0f)) return false;  // absorbed: color_from_emission == 0
    }
  } else if (!kDiffuse && type == RTG_MAT_DIELECTRIC) {
    att = v3(1.0f, 1.0f, 1.0f);
    const float eta = m0.w;
    const float ri = front ? div_rn(1.0f, eta) : eta;
    const V3 ud = unit(ps.d);
    const float cos_t = fminf(dot(neg(ud), n), 1.0f);
    const float sin_t = sqrt_rn(fmaf(-cos_t, cos_t, 1.0f));
    const bool cannot = ri * sin_t > 1.0f;
    bool reflect = cannot;
    if (!cannot) {
      float r0 = div_rn(1.0f - ri, 1.0f + ri);
      r0 = r0 * r0;
      const float x = 1.0f - cos_t;
      const float refl = fmaf(1.0f - r0, x * x * x * x * x, r0);
      reflect = refl > uniform(ps.rng);
    }
    if (reflect) {
      dir = madd(-(2.0f * dot(ud, n)), n, ud);
    } else {
      const float ct = fminf(dot(neg(ud), n), 1.0f);
      const V3 perp = scl(ri, madd(ct, n, ud));
      dir = madd(-sqrt_rn(fabsf(1.0f - dot(perp, perp))), n, perp);
    }
  } else {
    return false;  // base material: scatter() == false, emitted() == 0
  }
  ps.T = mul(ps.T, att);
  ps.o = p;
  ps.d = dir;
  ps.origin = ref;
  return true;
}

// Wave ballot of a lane predicate straight from its condition mask (HIP's __ballot takes an int,
// which makes the compiler materialise the predicate in a VGPR and compare it again).
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

// The lane id recomputed where a kernel ends (flush_stats, trace_wave): an asm mbcnt the compiler cannot merge
// with the one at the kernel's start, so the lane id is not held (or spilled, config 3) across the render loop
__device__ __forceinline__ int lane_now() {
  int l;
  __asm__ volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// Per-wave accumulators that outlive one tile.
template <bool COUNT>
struct WaveStats {
  uint32_t segs = 0, hits = 0, pixels = 0;
  Counts<COUNT> cnt;
  bool overflow = false, corrupt = false;
  uint64_t diag[16] = {};  // wave-uniform schedule diagnostics (COUNT only, rtg_render_stats::diag)
};

__device__ __forceinline__ void trace_wave(const DevJob& J, uint64_t t0, uint32_t pixels, int lane,
                                           int slot, int tag) {
  if (J.trace == nullptr) return;
  const uint32_t wp = wave_sum(pixels);
  if (lane == 0) {
    unsigned long long* r = J.trace + static_cast<int64_t>(slot) * 4;
    r[0] = t0;
    r[1] = __builtin_amdgcn_s_memrealtime();
    r[2] = wp;
    r[3] = static_cast<unsigned long long>(tag);
  }
}

template <bool COUNT>
__device__ __forceinline__ void flush_stats(const DevJob& J, WaveStats<COUNT>& w, int lane) {
  const uint32_t wsegs = wave_sum(w.segs);
  if (COUNT) {
    const uint32_t wbox = wave_sum(w.cnt.box);
    const uint32_t wprim = wave_sum(w.cnt.prim);
    const uint32_t whits = wave_sum(w.hits);
    const uint32_t wspill = wave_sum(w.cnt.spill);
    if (lane == 0) {
      atomicAdd(&J.counters[1], static_cast<unsigned long long>(wbox));
      atomicAdd(&J.counters[2], static_cast<unsigned long long>(wprim));
      atomicAdd(&J.counters[3], static_cast<unsigned long long>(whits));
      atomicAdd(&J.counters[26], static_cast<unsigned long long>(wspill));
      for (int k = 0; k < 16; ++k) atomicAdd(&J.counters[8 + k], static_cast<unsigned long long>(w.diag[k]));
    }
  }
  if (lane == 0) atomicAdd(&J.counters[0], static_cast<unsigned long long>(wsegs));
  if (__any(w.overflow) && lane == 0) atomicAdd(&J.counters[4], 1ull);
  if (__any(w.corrupt) && lane == 0) atomicAdd(&J.counters[5], 1ull);
}

// A lane's pixel, packed: column in the low 16 bits, shard-local row in the high 16 bits.
__device__ __forceinline__ int px_i(uint32_t px) { return static_cast<int>(px & 0xffffu); }
__device__ __forceinline__ int px_lr(uint32_t px) { return static_cast<int>(px >> 16); }

__device__ __forceinline__ void start_pixel_sample(PathState& ps, const DevCamera& C, const DevJob& J,
                                                   uint32_t px, uint32_t sample) {
  const int i = px_i(px);
  const int j = J.row_begin + px_lr(px) * J.row_stride;
  const uint32_t pixel_id = static_cast<uint32_t>(j) * static_cast<uint32_t>(C.width) + static_cast<uint32_t>(i);
  start_sample(ps, C, J.seed_mix, pixel_id, sample, i, j);
}

// ---- per-tile combine through a ring of tile slots (DESIGN.md §4 "per-tile combine") ----
// A one-shot chunked frame keeps no full-frame partial buffers: tile t owns ring slot t mod R,
// [chunk][64 pixels] float4 partial sums. The wave that takes batch (t, c) writes its 64 partials
// there with write-through (sc1) stores; when the batch's last unit has finished, the wave drains its
// stores (s_waitcnt vmcnt(0)) and adds 1 to the slot's ticket (relaxed, agent scope). The wave whose
// add is the tile's last (ticket = (gen + 1) * chunks - 1, tickets count every generation of the
// slot) takes an agent-scope acquire, sums the tile's partials in chunk order
// (((p0 + p1) + p2) + ..., the order combine_kernel uses), writes the 64 pixels and hands the slot to
// tile t + R by storing gen + 1. A batch whose slot still belongs to tile t - R is pending: its wave
// keeps running the units it holds and hands none of the batch out until the slot is free; a wave that
// holds nothing but a pending batch sleeps on the slot word (bounded: counters[24] on timeout). Every
// batch of tile t - R was handed out before any of tile t (tile-major hand-out), and a wave that
// holds units never sleeps, so the oldest unfinished tile always progresses.
// The hand-off is the split-K fan-in form of cdna_hip_programming.md Guideline 16: every storing wave
// stores sc1 and drains before its counter add; the last adder, told by its add's return value, takes
// ONE agent acquire before its plain loads; the slot word is an agent-scope atomic store after the
// loader's own drain.
// batches one wave tracks at once (a batch lives in one wave): a 64-B table per wave in LDS (entry:
// tile << 7 | units of the batch not yet finished), so the count costs the render loop no SGPRs
// (kept in SGPRs, 4 entries cost config 2 +16 % and config 4 +34 %, 8 entries more: profiles/r03_i)
constexpr int kRingEntries = 16;
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(3))) uint32_t lu32;
typedef unsigned int ring_u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bool ring_slot_free(const DevJob& J, int tile) {
  const int slot = tile & ((1 << J.ring_log2) - 1);
  const uint32_t g = __hip_atomic_load((gu32*)(J.ring_words + slot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(g)) == static_cast<uint32_t>(tile >> J.ring_log2);
}

// A unit's partial sum: 16 B per lane, one write-through store (aux 16 = sc1).
__device__ __forceinline__ void ring_store(__amdgpu_buffer_rsrc_t rs, uint32_t unit, V3 a) {
  const ring_u4 v = {__float_as_uint(a.x), __float_as_uint(a.y), __float_as_uint(a.z), 0u};
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, static_cast<int>(unit << 4), 0, 16);
}

// The tile's combine, by the wave whose ticket add was the tile's last: ONE agent acquire, the
// partials in chunk order, the 64 pixels, then the slot to tile + R. It runs at the top of the render
// loop, where every lane's path and traversal state is live and the 96-register dual-launch build has
// no register to spare: one colour channel at a time through the ring's buffer descriptor keeps its
// temporaries to a few registers (a float4 accumulator + float4 loads spilled the traversal state
// across the trip loop: config 2 +14 %, config 4 +26 %, profiles/r03_m).
template <bool WIDE_REGS>
__device__ __forceinline__ void ring_combine(__amdgpu_buffer_rsrc_t rs, const DevCamera& C, const DevJob& J,
                                             int tile, int slot) {
  const int lane = __lane_id();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const int ty = tile / J.tiles_x;
  const int i = ((tile - ty * J.tiles_x) << J.tile_lw) + (lane & ((1 << J.tile_lw) - 1));
  const int lr = (ty << (6 - J.tile_lw)) + (lane >> J.tile_lw);
  // the pixel's byte offset in the frame (past the frame's end for pixels outside the image: the
  // buffer descriptor's range check drops those stores)
  const int frame_bytes = J.row_count * C.width * 12;
  const int pix = i < C.width && lr < J.row_count ? (lr * C.width + i) * 12 : frame_bytes;
  const __amdgpu_buffer_rsrc_t fs = __builtin_amdgcn_make_buffer_rsrc(J.out, 0, frame_bytes, 0x00020000);
  const int base = (slot * J.chunks * 64 + lane) << 4;  // byte offset of this lane's chunk-0 partial
  if constexpr (WIDE_REGS) {
    // registers to spare (the 128-VGPR treelet build): whole partials, eight loads in flight, the
    // adds still in chunk order
    const ring_u4 p0 = __builtin_amdgcn_raw_buffer_load_b128(rs, base, 0, 0);
    float ax = __uint_as_float(p0.x), ay = __uint_as_float(p0.y), az = __uint_as_float(p0.z);
    int c = 1;
    for (; c + 8 <= J.chunks; c += 8) {
      ring_u4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, base + ((c + k) << 10), 0, 0);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        ax = ax + __uint_as_float(v[k].x);
        ay = ay + __uint_as_float(v[k].y);
        az = az + __uint_as_float(v[k].z);
      }
    }
    for (; c < J.chunks; ++c) {
      const ring_u4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, base + (c << 10), 0, 0);
      ax = ax + __uint_as_float(v.x);
      ay = ay + __uint_as_float(v.y);
      az = az + __uint_as_float(v.z);
    }
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(C.scale * ax), fs, pix, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(C.scale * ay), fs, pix, 4, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(C.scale * az), fs, pix, 8, 0);
  } else {
    // the 96-VGPR builds: one colour channel at a time, one load in flight
    for (int ch = 0; ch < 3; ++ch) {
      float a = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, base, ch * 4, 0));
#pragma unroll 1
      for (int c = 1; c < J.chunks; ++c)
        a = a + __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, base + (c << 10), ch * 4, 0));
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(C.scale * a), fs, pix, ch * 4, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the slot's loads returned: hand it on
  if (lane == 0)
    __hip_atomic_store((gu32*)(J.ring_words + slot), static_cast<uint32_t>(tile >> J.ring_log2) + 1u,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Batch (tile, any chunk) finished in this wave: drain, ticket add, and the tile's combine if this
// add was the tile's last. Wave-uniform call (all 64 lanes active).
template <bool WIDE_REGS>
__device__ __forceinline__ void ring_batch_done(__amdgpu_buffer_rsrc_t rs, const DevCamera& C, const DevJob& J,
                                                int tile) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 partial stores have landed
  const int R = 1 << J.ring_log2;
  const int slot = tile & (R - 1);
  const uint32_t gen = static_cast<uint32_t>(tile >> J.ring_log2);
  uint32_t old = 0;
  if (__lane_id() == 0)
    old = __hip_atomic_fetch_add((gu32*)(J.ring_words + R + slot), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __builtin_amdgcn_readfirstlane(old);
  if (old + 1u != (gen + 1u) * static_cast<uint32_t>(J.chunks)) return;
  ring_combine<WIDE_REGS>(rs, C, J, tile, slot);
}

// One wave renders a stream of work units with the ballot-batched schedule. A unit is one pixel
// and one chunk of its samples: samples [c*K, min((c+1)*K, spp)) of chunk c (DESIGN.md §4 "sample
// chunks"); a lane walks the chunk's samples in order, accumulating them from zero, and stores the
// chunk's partial sum (or the pixel, when the pixel has one chunk). Units are handed out in batches
// = (8x8 tile, chunk) from the launch-wide atomic counter J.counters[6], tile-major, so the 64 units
// of a batch, and the next batch (same tile, next chunk), share one tile: a lane that finishes its
// unit takes the next unit of the wave's current batch, and the wave takes a new batch once its
// batch is handed out. Lanes only idle once the whole shard has been handed out, a wave holds at most
// 63 unstarted units then, and no single expensive pixel (a glass sphere seen through 50 bounces)
// can hold a wave for more than K samples.
// Within a loop trip every lane advances its own traversal one step; a trip is either a node step
// or a leaf step for the whole wave (leaf work waits until leaf_batch lanes have reached a leaf);
// the wave switches to shading once ceil(alive * shade_batch / 64) lanes have finished their
// closest-hit query, and lanes still traversing keep their stack and continue afterwards.
template <class Stk, bool COUNT, int WIDE, bool TEXF, int GEOM, bool RING, int PRIMS = kPrimsAny>
__device__ __forceinline__ void render_stream(const DevScene& S, const DevCamera& C, const DevJob& J,
                                              const Stk& stk, WaveStats<COUNT>& w, lu32* rtab) {
  const int lane = __lane_id();
  // max_depth <= 0: every pixel is black and no segment is traced (camera.hpp:183-186); rtg_render writes
  // that frame itself and launches nothing (round 6: the hand-out loop no longer carries a branch for it,
  // whose zero triple the textured kernel kept in scratch), so this exit is only a guard
  if (C.max_depth <= 0 || C.spp <= 0) return;
  const int num_batches = J.num_tiles * J.chunks;
  V3 acc = v3(0.0f, 0.0f, 0.0f);
  uint32_t px = 0;
  // su: the lane's unit, its current sample index in bits 0-25 and the samples it has left (1 .. 63) in bits
  // 26-31; 0: the lane holds no unit (an integer, not a bool, for the same reason as kTravDone: ballots of
  // it need no lane-mask copy). One register for the sample and the unit's end (round 6: the 96-VGPR
  // kernels had none to spare; the host keeps spp < 2^26 and K <= 63)
  constexpr uint32_t kSampleBits = 26, kSampleMask = (1u << kSampleBits) - 1u;
  uint32_t su = 0;
  uint32_t seg0 = 0;  // COUNT: the lane's segment count when its unit started (the tile-cost probe)
  int chunk = 0;
  auto has = [&]() { return su != 0; };
  // fresh: the lane starts sample (su & kSampleMask) of its unit at the top of the next loop trip (the one
  // start path for the next sample of a unit and the first sample of a new unit); cont: its path
  // continues with a new segment (ps.o / ps.d scattered)
  bool fresh = false, cont = false;
  // wave-uniform: the current batch's tile origin and chunk, and its next unassigned unit
  int bx = 0, by = 0, bc = 0, k_next = 64;
  bool exhausted = false;
  // tile ring (J.ring_log2 >= 0): the entries of rtab in use (the batches this wave holds), the
  // entry of the batch being handed out, whether that batch waits for its slot; a lane's `chunk`
  // then holds its unit's ring index | entry << 28, and `fin` marks a unit finished since the last
  // settle
  constexpr bool ring = RING;  // the host sets J.ring_log2 >= 0 exactly for the RING kernels
  uint32_t e_used = 0;
  int cur_e = 0;
  bool pending = false, fin = false, exhausted_by_timeout = false;
  uint32_t pend_spins = 0;  // empty trips spent waiting for the pending batch's slot
  // the tile of the batch being handed out (from its origin: no state of its own)
  auto cur_tile = [&]() { return (by >> (6 - J.tile_lw)) * J.tiles_x + (bx >> J.tile_lw); };
  __amdgpu_buffer_rsrc_t ring_rs = __builtin_amdgcn_make_buffer_rsrc(J.partial, 0, 0, 0x00020000);
  if (ring)
    ring_rs = __builtin_amdgcn_make_buffer_rsrc(
        J.partial, 0, static_cast<int>((static_cast<uint32_t>(J.chunks) << (J.ring_log2 + 10))), 0x00020000);
  PathState ps = {};
  Trav tr = {};
  tr.todo = kTravDone;
  const V3 bg = v3(C.background[0], C.background[1], C.background[2]);
  for (;;) {
    uint64_t t_top = 0;
    if (COUNT) t_top = __builtin_amdgcn_s_memtime();
    if (ring) {  // settle: count the units finished since the last trip, finish completed batches
      uint64_t fm = ballot(fin);
      if (fm != 0) {
        const int ent = static_cast<int>(static_cast<uint32_t>(chunk) >> 28);
        do {  // one LDS update per entry among the finished units (usually one)
          const int e = __builtin_amdgcn_readlane(ent, static_cast<int>(__builtin_ctzll(fm)));
          const uint64_t m = ballot(fin && ent == e);
          const uint32_t n = static_cast<uint32_t>(__popcll(m));
          uint32_t left = 0;
          if (lane == 0) left = __hip_atomic_fetch_sub(rtab + e, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT) - n;
          left = __builtin_amdgcn_readfirstlane(left);
          if ((left & 127u) == 0) {  // the batch's last unit: ticket (and the tile's combine)
            e_used &= ~(1u << e);
            ring_batch_done<false>(ring_rs, C, J, static_cast<int>(left >> 7));
          }
          fm &= ~m;
        } while (fm != 0);
        fin = false;
      }
      if (pending) {  // the held batch waits for its slot: one poll per trip (empty trips sleep)
        pending = !ring_slot_free(J, cur_tile());
        if (pending && ballot(has()) == 0) {  // an empty trip: sleep, bounded (~2^22 trips, seconds)
          __builtin_amdgcn_s_sleep(8);
          if (++pend_spins > (1u << 22)) {
            exhausted = exhausted_by_timeout = true;  // counters[24] after the loop; the wave drains
            pending = false;
          }
        }
      }
    }
    // hand the next units of the current batch (new batches as needed) to the lanes without one
    uint64_t want = ballot(!has());
    while (want != 0 && !exhausted && !pending) {
      if (k_next >= 64) {
        if (ring && e_used == (1u << kRingEntries) - 1u) break;  // every entry busy: lanes wait
        int b = 0;
        if (lane == 0) b = static_cast<int>(atomicAdd(&J.counters[6], 1ull));
        b = __builtin_amdgcn_readfirstlane(__shfl(b, 0, 64));
        if (b >= num_batches) {
          exhausted = true;
          break;
        }
        const int tpos = b / J.chunks;  // the batch's tile position in the hand-out order
        bc = J.chunk_begin + (b - tpos * J.chunks);
        // cost-ordered hand-out (rtg_scene_prepare's tile order): the tile at that position, the
        // most expensive first; tile-major without one, and always in the ring kernels (their slot hand-off
        // needs tile-major order). Only when a unit is rendered changes, never what it sums: frames identical
        int tile = tpos;
        if constexpr (!RING) {
          const int32_t* order = tile_order_late<COUNT>(J, w.corrupt);
          if (order != nullptr) tile = __builtin_amdgcn_readfirstlane(order[tpos]);  // wave-uniform: SALU below
        }
        const int ty = tile / J.tiles_x;
        bx = (tile - ty * J.tiles_x) << J.tile_lw;
        by = ty << (6 - J.tile_lw);
        k_next = 0;
        if (ring) {
          cur_e = __builtin_ctz(~e_used);
          e_used |= 1u << cur_e;
          if (lane == 0) rtab[cur_e] = (static_cast<uint32_t>(tile) << 7) | 64u;
          if (!ring_slot_free(J, tile)) {  // hand it out once its slot is free (top of the loop)
            if (COUNT && lane == 0) atomicAdd(&J.counters[25], 1ull);
            pending = true;
            pend_spins = 0;
            break;
          }
        }
      }
      const int take = min(__popcll(want), 64 - k_next);
      const int rank = static_cast<int>(__builtin_amdgcn_mbcnt_hi(
          static_cast<uint32_t>(want >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(want), 0u)));
      bool outside = false;  // a unit of the batch past the image edge: finished on hand-out
      if (!has() && rank < take) {
        const int k = k_next + rank;
        const int i = bx + (k & ((1 << J.tile_lw) - 1));
        const int lr = by + (k >> J.tile_lw);
        if (i < C.width && lr < J.row_count) {
          px = static_cast<uint32_t>(i) | (static_cast<uint32_t>(lr) << 16);
          fresh = true;
          chunk = ring ? ((((cur_tile() & ((1 << J.ring_log2) - 1)) * J.chunks + (bc - J.chunk_begin)) << 6) + k) |
                             (cur_e << 28)
                       : bc;
          if (COUNT) seg0 = w.segs;  // the tile-cost probe: this unit's segments are counted from here
          const int s0 = bc * J.chunk_samples;
          su = (static_cast<uint32_t>(min(s0 + J.chunk_samples, C.spp) - s0) << kSampleBits) | static_cast<uint32_t>(s0);
          acc = v3(0.0f, 0.0f, 0.0f);
        } else {
          outside = true;
        }
      }
      if (ring) {
        // units past the image edge finish on hand-out (a batch keeps >= 1 unit: its tile's origin)
        const uint32_t n_out = static_cast<uint32_t>(__popcll(ballot(outside)));
        if (n_out != 0 && lane == 0) rtab[cur_e] -= n_out;
      }
      k_next += take;
      want = ballot(!has());
    }
    uint64_t t_start = 0;
    if (COUNT) t_start = __builtin_amdgcn_s_memtime();
    if (fresh) start_pixel_sample(ps, C, J, px, su & kSampleMask);
    if (COUNT) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      w.diag[13] += t_start - t_top;  // unit hand-out
      w.diag[14] += t - t_start;      // camera rays of fresh samples
      t_start = t;
    }
    if (fresh || cont) {
      trav_begin<WIDE>(tr, S, ps.o, ps.d, ps.origin);
      if (S.occluder >= 0) {  // the scene-spanning sphere kept out of the BVH (DevScene::occluder)
        const float4* sp4 = S.spheres + static_cast<int64_t>(S.occluder) * S.sphere_f4;
        if (COUNT) w.cnt.prim += 1;
        const float th = sphere_t(sp4[0], sp4[1], ps.o, ps.d, tr.a, tr.inv_a, ps.time, kTMin, tr.tbest,
                                  S.occluder == ps.origin);
        if (th > 0.0f) {
          tr.tbest = th;
          tr.best = S.occluder;
          if (GEOM != kGeomLds) tr.mat = ibits(sp4[1].w);  // (LDS schedule: tie rank -1 from trav_begin)
        }
      }
    }
    fresh = false;
    cont = false;
    if (COUNT) w.diag[15] += __builtin_amdgcn_s_memtime() - t_start;  // trav_begin + occluder test
    const uint64_t has_m = ballot(has());  // constant over the trip loop: kept as an SGPR mask
    const int alive = __popcll(has_m);
    // the loop's one exit: nothing left to hand out and no unit in a lane. A wave whose only batch
    // waits for its slot runs an empty trip and sleeps on the slot at the top of the loop (a second
    // back edge here instead made the register allocator spill the traversal state: config 2 +14 %)
    if (alive == 0 && !pending) break;
    const int need = (alive * J.shade_batch + 63) >> 6;
    uint64_t t_trav0 = 0;
    if (COUNT) t_trav0 = __builtin_amdgcn_s_memtime();
    // traversal trips issue at wave priority 1, shading at 0: the SIMD's arbiter then prefers the
    // waves on the LDS-latency-bound node chain, and the VALU-dense shading fills the slots between
    // (same-box A/B, frames identical: book-1 -0.3 %, earth_perlin -0.6 %, 1M spheres -0.3 %,
    // Cornell +-0; shading first instead: neutral)
    __builtin_amdgcn_s_setprio(1);
    for (;;) {
      if (COUNT) {
        w.diag[0] += 1;
        w.diag[1] += __popcll(ballot(trav_active(tr)));
        w.diag[2] += __popcll(ballot(!has()));
      }
      const int at_leaf = __popcll(ballot(tr.todo < 0));
      const bool inner_left = ballot(at_inner(tr)) != 0;
      const bool leaf_trip = at_leaf >= J.leaf_batch || !inner_left;
      uint64_t tl = 0;
      if (COUNT) {
        if (leaf_trip) {
          w.diag[7] += 1;
          w.diag[10] += at_leaf;
          tl = __builtin_amdgcn_s_memtime();
        } else {
          w.diag[9] += __popcll(ballot(at_inner(tr)));
        }
      }
      if (leaf_trip && tr.todo < 0)
        leaf_step<Stk, COUNT, GEOM != kGeomLds, GEOM != kGeomLds, WIDE, GEOM, PRIMS, GEOM == kGeomLds || !RING>(
            tr, S, ps.o, ps.d, ps.time, stk, w.cnt, w.corrupt);
      // lanes at inner nodes step in every trip: in a leaf trip they would otherwise idle, and the
      // node step's LDS latency overlaps the primitive tests (measured -3% on book-1, -7% Cornell)
      // node steps per trip: 2 where nodes come through the caches (config 5 -2.1 %: half the trip
      // overhead, and a lane's second step overlaps the other lanes' load latency), 1 for LDS scenes
      // (2: neutral, 3: +3 %)
      constexpr int kNodeReps = GEOM == kGeomLds ? 1 : 2;
#pragma unroll
      for (int rep = 0; rep < kNodeReps; ++rep) {
        if (at_inner(tr)) {
          if constexpr (WIDE == 4)
            node_step4<Stk, COUNT, GEOM, (PRIMS & kPrimsKind) != kPrimsSpheres>(tr, S, stk, w.cnt, w.overflow,
                                                                                w.corrupt);
          else
            node_step<Stk, COUNT>(tr, S, stk, w.cnt, w.overflow, w.corrupt);
        }
      }
      if (COUNT && leaf_trip) w.diag[8] += __builtin_amdgcn_s_memtime() - tl;
      const uint64_t trav = ballot(trav_active(tr));
      const int ready = __popcll(ballot(!trav_active(tr)) & has_m);
      if (trav == 0 || ready >= need) break;
    }
    __builtin_amdgcn_s_setprio(0);
    uint64_t t_shade0 = 0;
    if (COUNT) {
      t_shade0 = __builtin_amdgcn_s_memtime();
      w.diag[5] += t_shade0 - t_trav0;
      w.diag[3] += 1;
      w.diag[4] += __popcll(ballot(!trav_active(tr) && has()));
    }
    if (!trav_active(tr) && has()) {
      ++w.segs;
      bool alive_path;
      if (tr.best < 0) {
        ps.L = vfma(ps.T, bg, ps.L);
        alive_path = false;
      } else {
        if (COUNT) ++w.hits;
        alive_path = shade<TEXF, GEOM != kGeomLds, PRIMS, GEOM == kGeomLds>(S, ps, tr.best, tr.tbest, tr.mat);
        if (alive_path && --ps.depth <= 0) alive_path = false;
      }
      uint64_t t_end = 0;
      if (COUNT) {
        t_end = __builtin_amdgcn_s_memtime();
        w.diag[11] += t_end - t_shade0;
      }
      cont = alive_path;
      if (!alive_path) {
        acc = add(acc, ps.L);
        su += 1u - (1u << kSampleBits);  // the next sample, one fewer left
        if ((su >> kSampleBits) != 0) {
          fresh = true;
        } else {
          const int64_t pix = static_cast<int64_t>(px_lr(px)) * C.width + px_i(px);
          if (ring) {  // the unit's partial sum into its tile's ring slot (settled next trip)
            ring_store(ring_rs, static_cast<uint32_t>(chunk & 0x0fffffff), acc);
            fin = true;
          } else if (J.partial == nullptr) {  // one chunk per pixel: the pixel mean directly
            float* o = J.out + pix * 3;
            o[0] = C.scale * acc.x;
            o[1] = C.scale * acc.y;
            o[2] = C.scale * acc.z;
          } else {  // progressive: chunk partial sum in the full-frame layout, combined by combine_kernel
            float* o = J.partial + (static_cast<int64_t>(chunk) * J.row_count * C.width + pix) * 3;
            o[0] = acc.x;
            o[1] = acc.y;
            o[2] = acc.z;
          }
          su = 0;  // the unit is done
          ++w.pixels;
          // the tile-cost probe (rtg_scene_prepare): the unit's segments into its tile's counter
          if (COUNT && J.tile_cost != nullptr)
            atomicAdd(J.tile_cost + (px_lr(px) >> (6 - J.tile_lw)) * J.tiles_x + (px_i(px) >> J.tile_lw), w.segs - seg0);
        }
      }
      if (COUNT) w.diag[12] += __builtin_amdgcn_s_memtime() - t_end;
    }
    if (COUNT) w.diag[6] += __builtin_amdgcn_s_memtime() - t_shade0;
  }
  // a slot wait that timed out, or (unreachable) a held batch never combined: the frame is incomplete
  if (ring && (exhausted_by_timeout || e_used != 0) && lane == 0) atomicAdd(&J.counters[24], 1ull);
}

// Schedule 4: the same loop on a plain grid of 256-thread workgroups (scene read through the
// caches; used when it does not fit in LDS). Waves take tiles from the same counter.
template <int STACK, bool SPILL, bool COUNT, int WIDE, bool TEXF, bool RING>
__global__ __launch_bounds__(256) void render_kernel(DevScene S, DevCamera C, DevJob J) {
  __shared__ int32_t s_stack[4 * STACK * 64];
  __shared__ uint32_t s_ring[RING ? 4 * kRingEntries : 1];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: an SGPR, not a VGPR held (or spilled) across the render loop
  const int slot = blockIdx.x * 4 + wave;
  lu32* rtab = (lu32*)(s_ring) + (RING ? __builtin_amdgcn_readfirstlane(wave) * kRingEntries : 0);
  int32_t* lstk = s_stack + wave * STACK * 64 + lane;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  WaveStats<COUNT> w;
  if constexpr (SPILL) {
    const SpillStack<STACK> stk{lstk, J.spill + static_cast<int64_t>(slot) * J.spill_depth * 64 + lane,
                                J.lds_stack, J.lds_stack + J.spill_depth};
    render_stream<SpillStack<STACK>, COUNT, WIDE, TEXF, kGeomGlobal, RING>(S, C, J, stk, w, rtab);
  } else {
    render_stream<LdsStack<STACK>, COUNT, WIDE, TEXF, kGeomGlobal, RING>(S, C, J, LdsStack<STACK>{lstk}, w, rtab);
  }
  flush_stats<COUNT>(J, w, lane_now());
  trace_wave(J, t0, w.pixels, lane_now(), slot, (blockIdx.x << 8) | wave);
}

// Schedule 3's body: the whole scene in the workgroup's LDS (render_kernel_lds with GEOM = kGeomLds).
template <int STACK, bool SPILL, bool COUNT, int WAVES, int WIDE, bool TEXF, bool RING, int PRIMS = kPrimsAny>
__device__ __forceinline__ void render_lds_scene(const DevScene& S, const DevCamera& C, const DevJob& J,
                                                 unsigned char* smem, int kFill, int wpb, uint64_t t0, int lane,
                                                 int wave, int32_t* lstk, int16_t* lstk16, lu32* rtab) {
  // the whole-scene LDS schedule of 4-wide trees without a stack spill and without image / noise
  // textures keeps 16-bit stack entries (the LDS room that lets book-1 run the dual launch; the
  // textured kernels keep 32-bit ones: earth_perlin +2 % with 16-bit)
  constexpr bool STK16 = WIDE == 4 && !SPILL && !TEXF;
  float4* l_nodes = reinterpret_cast<float4*>(smem + J.lds_nodes);
  int32_t* l_refs = reinterpret_cast<int32_t*>(smem + J.lds_refs);
  float4* l_spheres = reinterpret_cast<float4*>(smem + J.lds_spheres);
  float4* l_quads = reinterpret_cast<float4*>(smem + J.lds_quads);
  float4* l_materials = reinterpret_cast<float4*>(smem + J.lds_materials);
  float4* l_textures = reinterpret_cast<float4*>(smem + J.lds_textures);
  for (int k = threadIdx.x; k < S.num_materials * 2; k += kFill) l_materials[k] = S.materials[k];
  for (int k = threadIdx.x; k < S.num_textures * 2; k += kFill) l_textures[k] = S.textures[k];
  // LDS byte address of the node array (inner-node codes of the LDS copy are rebased onto it)
  const int32_t node_rebase = static_cast<int32_t>(static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) unsigned char*)smem))) + J.lds_nodes;
  for (int64_t k = threadIdx.x; k < S.num_nodes * (WIDE == 4 ? 7 : 4); k += kFill) {
    float4 v = S.nodes[k];
    if (WIDE == 4 && k % 7 == 6) {  // code row: inner-node codes become absolute LDS addresses
      int4 c = *reinterpret_cast<int4*>(&v);
      c.x = c.x >= 0 ? c.x + node_rebase : c.x;
      c.y = c.y >= 0 ? c.y + node_rebase : c.y;
      c.z = c.z >= 0 ? c.z + node_rebase : c.z;
      c.w = c.w >= 0 ? c.w + node_rebase : c.w;
      v = *reinterpret_cast<float4*>(&c);
    }
    l_nodes[k] = v;
  }
  // sphere records padded to J.lds_sphere_f4 float4s in LDS (3: 48-B stride, an odd number of 16-B
  // bank slots, so the ds_read_b128 of 16 lanes at different spheres spread over all 16 slots)
  for (int64_t k = threadIdx.x; k < S.num_spheres * 2; k += kFill)
    l_spheres[(k >> 1) * J.lds_sphere_f4 + (k & 1)] = S.spheres[k];
  for (int64_t k = threadIdx.x; k < S.num_quads * 5; k += kFill) l_quads[k] = S.quads[k];
  if (S.ref_mode == 0)
    for (int64_t k = threadIdx.x; k < S.num_refs; k += kFill) l_refs[k] = S.refs[k];
  float4* l_pvec = reinterpret_cast<float4*>(smem + J.lds_perlin_vec);
  uint32_t* l_pperm = reinterpret_cast<uint32_t*>(smem + J.lds_perlin_perm);
  if (TEXF) {
    // the Z words of table t carry the LDS address of its gradient rows in both 16-bit lanes (the host
    // plans them from LDS address 0: 4096-aligned, below 64 KiB, so an OR of disjoint bits); if the
    // dynamic-LDS base ever moves them elsewhere, report and render nothing
    const uint32_t vbase = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
                               (__attribute__((address_space(3))) unsigned char*)smem)) + J.lds_perlin_vec;
    if ((vbase & 4095u) != 0 || vbase + static_cast<uint32_t>(S.num_perlins) * 4096u > 65536u) {
      if (threadIdx.x == 0) atomicAdd(&J.counters[7], 1ull);
      return;
    }
    for (int k = threadIdx.x; k < S.num_perlins * 256; k += kFill) l_pvec[k] = S.perlin_vec[k];
    for (int k = threadIdx.x; k < S.num_perlins * kPerlinPermWords; k += kFill) {
      const int t = k / kPerlinPermWords;
      const uint32_t b = vbase + static_cast<uint32_t>(t) * 4096u;
      l_pperm[k] = S.perlin_perm[k] ^ (k - t * kPerlinPermWords >= 768 ? b * 0x10001u : 0u);
    }
  }
  __syncthreads();
  DevScene L = S;
  L.nodes = l_nodes;
  if (WIDE == 4) {  // inner-node codes are absolute LDS byte addresses
    L.root_code = node_rebase;
    L.node_limit = node_rebase + static_cast<int32_t>(S.num_nodes) * 112;
  }
  // 16-bit stack entries hold inner codes (absolute LDS addresses, so the node array must end below
  // 32 KB of LDS) and leaf codes (first primitive < 4096). The host plans the layout for a dynamic-LDS
  // base of 0; if that ever changes (e.g. a static __shared__ is added) report, render nothing
  if (STK16 && (L.node_limit > 32768 || S.num_refs > 4096)) {
    if (threadIdx.x == 0) atomicAdd(&J.counters[7], 1ull);
    return;
  }
  L.refs = l_refs;
  L.spheres = l_spheres;
  L.sphere_f4 = J.lds_sphere_f4;
  L.quads = l_quads;
  L.materials = l_materials;
  L.textures = l_textures;
  if (TEXF) {
    L.perlin_vec = l_pvec;
    L.perlin_perm = l_pperm;
  }
  WaveStats<COUNT> w;
  if constexpr (SPILL) {
    const int slot = blockIdx.x * wpb + wave;
    const SpillStack<STACK> stk{lstk, J.spill + static_cast<int64_t>(slot) * J.spill_depth * 64 + lane,
                                J.lds_stack, J.lds_stack + J.spill_depth};
    render_stream<SpillStack<STACK>, COUNT, WIDE, TEXF, kGeomLds, RING, PRIMS>(L, C, J, stk, w, rtab);
  } else if constexpr (STK16) {
    render_stream<LdsStack16<STACK>, COUNT, WIDE, TEXF, kGeomLds, RING, PRIMS>(L, C, J, LdsStack16<STACK>{lstk16}, w,
                                                                             rtab);
  } else {
    render_stream<LdsStack<STACK>, COUNT, WIDE, TEXF, kGeomLds, RING, PRIMS>(L, C, J, LdsStack<STACK>{lstk}, w, rtab);
  }
  flush_stats<COUNT>(J, w, lane_now());
  trace_wave(J, t0, w.pixels, lane_now(), blockIdx.x * wpb + wave, (blockIdx.x << 8) | wave);
}

// Schedule 3 (default when the geometry fits): persistent workgroups of WAVES waves, one per CU.
// The workgroup copies the traversal geometry (nodes, leaf refs, spheres, quads) into LDS once;
// afterwards every node / primitive fetch of the traversal is an LDS read instead of a divergent
// L1 gather. Each wave then pulls 8x8 pixel tiles from a global atomic counter until none are
// left (the exit every wave reaches), so the end of the launch has no tile-granularity tail.
//
// GEOM = kGeomTreelet (schedule 5, scenes too large for LDS such as the 1M-sphere field): the same
// persistent workgroups keep only the breadth-first top of the 4-wide tree in LDS (as many nodes as
// fit beside the stacks, S.treelet_bytes); deeper nodes, primitives, materials and textures are read
// through the caches. Every ray's first levels are then ds_reads instead of L1/L2 round trips.
template <int STACK, bool SPILL, bool COUNT, int WAVES, int WIDE, bool TEXF, int GEOM, bool RING,
          int PRIMS = kPrimsAny>
// WAVES = 4: compiled for 5 waves per SIMD (<= 96 VGPRs) and launched with 4-wave workgroups (small
// scenes, the dual launch's second workgroup) or 16-wave ones (book-1's main launch): one binary for
// both shapes of the dual launch, and its 96-register budget runs the 16-wave workgroup faster than
// the 104-register 16-wave build (dual -0.25 %, single -0.4 %, frames identical), so
// the workgroup size is read at run time (kFill, wpb) instead of from WAVES.
__global__ __launch_bounds__(WAVES == 4 ? 1024 : WAVES * 64, WAVES == 4 ? 5 : 4)
void render_kernel_lds(DevScene S, DevCamera C, DevJob J) {
  const int kFill = WAVES == 4 ? static_cast<int>(blockDim.x) : WAVES * 64;  // threads of the workgroup
  const int wpb = kFill >> 6;                                                // waves of the workgroup
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: an SGPR, not a VGPR held (or spilled) across the render loop
  int32_t* lstk = reinterpret_cast<int32_t*>(smem + J.lds_stacks) + wave * STACK * 64 + lane;
  int16_t* lstk16 = reinterpret_cast<int16_t*>(smem + J.lds_stacks) + wave * STACK * 64 + lane;
  lu32* rtab = (lu32*)(reinterpret_cast<uint32_t*>(smem + J.lds_ring)) +
               (RING ? __builtin_amdgcn_readfirstlane(wave) * kRingEntries : 0);
  if constexpr (GEOM == kGeomTreelet) {
    float4* l_top = reinterpret_cast<float4*>(smem + J.lds_nodes);
    for (int k = threadIdx.x; k < S.treelet_bytes / 16; k += kFill) l_top[k] = S.nodes[k];
    __syncthreads();
    DevScene L = S;
    L.treelet_lds = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
                        (__attribute__((address_space(3))) unsigned char*)smem)) +
                    static_cast<uint32_t>(J.lds_nodes);
    WaveStats<COUNT> w;
    if constexpr (SPILL) {
      // the LDS part of a spilling stack is J.lds_stack (<= STACK) entries per lane: the host may keep
      // fewer than STACK there to leave the treelet more room (RTG_TREELET_STACK)
      const int slot = blockIdx.x * wpb + wave;
      int32_t* tstk = reinterpret_cast<int32_t*>(smem + J.lds_stacks) + wave * J.lds_stack * 64 + lane;
      const SpillStack<STACK> stk{tstk, J.spill + static_cast<int64_t>(slot) * J.spill_depth * 64 + lane,
                                  J.lds_stack, J.lds_stack + J.spill_depth};
      render_stream<SpillStack<STACK>, COUNT, WIDE, TEXF, kGeomTreelet, RING, PRIMS>(L, C, J, stk, w, rtab);
    } else {
      render_stream<LdsStack<STACK>, COUNT, WIDE, TEXF, kGeomTreelet, RING, PRIMS>(L, C, J, LdsStack<STACK>{lstk}, w,
                                                                                rtab);
    }
    flush_stats<COUNT>(J, w, lane_now());
    trace_wave(J, t0, w.pixels, lane_now(), blockIdx.x * wpb + wave, (blockIdx.x << 8) | wave);
  } else {
    render_lds_scene<STACK, SPILL, COUNT, WAVES, WIDE, TEXF, RING, PRIMS>(S, C, J, smem, kFill, wpb, t0, lane, wave,
                                                                          lstk, lstk16, rtab);
  }
}



// write_color (color.hpp:14-58) in the reference's own precision: linear_to_gamma takes the
// square root in double (color.hpp:14-23), interval::clamp clamps in double to
// [0.000f, 0.999f] (the float literals widened, color.hpp:45, interval.hpp:35-46), and
// int(256 * x) truncates the double product — so every byte equals the reference's.
__global__ __launch_bounds__(256) void resolve_kernel(const float* __restrict__ in,
                                                      uint8_t* __restrict__ out, int64_t n) {
  const int64_t k = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k >= n * 3) return;
  double x = static_cast<double>(in[k]);
  x = x > 0.0 ? __builtin_sqrt(x) : 0.0;  // llvm.sqrt.f64: correctly rounded on gfx950
  const double lo = static_cast<double>(0.000f), hi = static_cast<double>(0.999f);
  x = x < lo ? lo : (x > hi ? hi : x);
  out[k] = static_cast<uint8_t>(static_cast<int>(256.0 * x));
}

// Pixel = scale * (((p_0 + p_1) + p_2) + ...): the chunk partial sums in chunk order.
__global__ __launch_bounds__(256) void combine_kernel(const float* __restrict__ partial, float* __restrict__ out,
                                                      int64_t n_pixels, int chunks, float scale) {
  const int64_t k = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k >= n_pixels * 3) return;
  float acc = partial[k];
  for (int c = 1; c < chunks; ++c) acc = acc + partial[static_cast<int64_t>(c) * n_pixels * 3 + k];
  out[k] = scale * acc;
}

constexpr int kLdsWaves = 16;  // 1024-thread persistent workgroups: 4 waves/SIMD at <= 128 VGPRs

template <int STACK, bool SPILL, int WIDE, bool TEXF, int GEOM = kGeomLds, int WAVES = kLdsWaves, int PRIMS = kPrimsAny>
KernelChoice lds_kernel(bool count, bool ring, int threads = WAVES * 64) {
  KernelChoice k;
  k.fn = count ? reinterpret_cast<const void*>(
                     &render_kernel_lds<STACK, SPILL, true, WAVES, WIDE, TEXF, GEOM, false, PRIMS>)
         : ring ? reinterpret_cast<const void*>(
                      &render_kernel_lds<STACK, SPILL, false, WAVES, WIDE, TEXF, GEOM, true, PRIMS>)
                : reinterpret_cast<const void*>(
                      &render_kernel_lds<STACK, SPILL, false, WAVES, WIDE, TEXF, GEOM, false, PRIMS>);
  k.block = threads;
  k.dynamic_lds = true;
  return k;
}

// the 4-wave whole-scene LDS build (five 4-wave workgroups per CU, or both shapes of the dual launch) for
// a primitive class
template <bool TEXF>
KernelChoice lds4_kernel(int prims, bool count, bool ring, int threads) {
  switch (prims) {
    case kPrimsSpheres: return lds_kernel<kLdsStack, false, 4, TEXF, kGeomLds, 4, kPrimsSpheres>(count, ring, threads);
    case kPrimsQuads: return lds_kernel<kLdsStack, false, 4, TEXF, kGeomLds, 4, kPrimsQuads>(count, ring, threads);
    case kPrimsAny | kPrimsDiffuse:
      return lds_kernel<kLdsStack, false, 4, TEXF, kGeomLds, 4, kPrimsAny | kPrimsDiffuse>(count, ring, threads);
    case kPrimsSpheres | kPrimsDiffuse:
      return lds_kernel<kLdsStack, false, 4, TEXF, kGeomLds, 4, kPrimsSpheres | kPrimsDiffuse>(count, ring, threads);
    case kPrimsQuads | kPrimsDiffuse:
      return lds_kernel<kLdsStack, false, 4, TEXF, kGeomLds, 4, kPrimsQuads | kPrimsDiffuse>(count, ring, threads);
    default: return lds_kernel<kLdsStack, false, 4, TEXF, kGeomLds, 4, kPrimsAny>(count, ring, threads);
  }
}

template <int STACK, bool SPILL, int WIDE, bool TEXF>
KernelChoice plain_kernel(bool count, bool ring) {
  KernelChoice k;
  k.fn = count ? reinterpret_cast<const void*>(&render_kernel<STACK, SPILL, true, WIDE, TEXF, false>)
         : ring ? reinterpret_cast<const void*>(&render_kernel<STACK, SPILL, false, WIDE, TEXF, true>)
                : reinterpret_cast<const void*>(&render_kernel<STACK, SPILL, false, WIDE, TEXF, false>);
  k.block = 256;
  return k;
}

// Schedule 5: the persistent kernel with an LDS treelet over a scene in HBM (4-wide trees only).
KernelChoice treelet_kernel(const DevScene& S, const DevJob& J, bool count) {
  if (J.lds_stack > kLdsStack || J.stack_esz != 4 || J.lds_waves != kLdsWaves) return {};
  const bool spill = J.spill_depth > 0, tex = S.tex_full != 0, ring = J.ring_log2 >= 0 && !count;
  if (S.node_width != 4) return {};
  // sphere-only scenes (the 1M field) get a build without the quad test (kPrimsSpheres, as default_kernel)
  const bool spheres = S.ref_mode == 1 && !tex;
  if (spill)
    return tex ? lds_kernel<kLdsStack, true, 4, true, kGeomTreelet>(count, ring)
               : spheres ? lds_kernel<kLdsStack, true, 4, false, kGeomTreelet, kLdsWaves, kPrimsSpheres>(count, ring)
                         : lds_kernel<kLdsStack, true, 4, false, kGeomTreelet>(count, ring);
  return tex ? lds_kernel<kLdsStack, false, 4, true, kGeomTreelet>(count, ring)
             : spheres ? lds_kernel<kLdsStack, false, 4, false, kGeomTreelet, kLdsWaves, kPrimsSpheres>(count, ring)
                       : lds_kernel<kLdsStack, false, 4, false, kGeomTreelet>(count, ring);
}

// The default schedules: persistent LDS kernel (16 LDS stack entries) or the plain grid (16, or 32
// with a global spill for deeper trees), each with / without the image-and-noise texture paths.
template <int WIDE>
KernelChoice default_kernel(const DevScene& S, const DevJob& J, bool count, int stack, bool lds) {
  const bool spill = J.spill_depth > 0;
  const bool tex = S.tex_full != 0;
  const bool ring = J.ring_log2 >= 0 && !count;
  if (lds) {
    if (stack != kLdsStack || J.lds_stack > kLdsStack) return {};
    // 4-wide trees keep 16-bit stack entries (J.stack_esz 2) unless their leaf codes do not fit 16
    // bits (the host then asks for 4-byte entries, which the spill variant holds, with no spill area
    // if none is needed); binary trees keep 32-bit entries
    const bool stk16 = WIDE == 4 && !spill && !tex && J.stack_esz == 2;
    if (J.stack_esz != (stk16 ? 2 : 4)) return {};
    if (spill || (WIDE == 4 && !tex && !stk16))
      return tex ? lds_kernel<kLdsStack, true, WIDE, true>(count, ring) : lds_kernel<kLdsStack, true, WIDE, false>(count, ring);
    // 4-wide trees with 16-bit stacks: the 4-wave build for both workgroup shapes (see render_kernel_lds),
    // one per primitive class (kPrimsAny...: the leaf test compiled for the scene's primitives only)
    // (a quad-only tree with a sphere occluder beside it shades spheres too: kPrimsAny)
    const int kind = S.ref_mode == 1 ? kPrimsSpheres : (S.ref_mode == 2 && S.occluder < 0 ? kPrimsQuads : kPrimsAny);
    const int prims = kind | (S.diffuse_only ? kPrimsDiffuse : 0);
    if (WIDE == 4 && !tex && J.lds_waves == kLdsWaves)
      return lds4_kernel<false>(prims, count, ring, kLdsWaves * 64);
    if (WIDE == 4 && J.lds_waves == 4)  // small scenes: five 4-wave workgroups per CU; the dual's second launch
      return tex ? lds4_kernel<true>(prims, count, ring, 4 * 64) : lds4_kernel<false>(prims, count, ring, 4 * 64);
    return tex ? lds_kernel<kLdsStack, false, WIDE, true>(count, ring) : lds_kernel<kLdsStack, false, WIDE, false>(count, ring);
  }
  if (stack > 32 || J.lds_stack > stack) return {};
  if (spill)  // (any LDS part <= 32 entries, J.lds_stack, plus the global spill)
    return tex ? plain_kernel<32, true, WIDE, true>(count, ring) : plain_kernel<32, true, WIDE, false>(count, ring);
  if (stack == 16)
    return tex ? plain_kernel<16, false, WIDE, true>(count, ring) : plain_kernel<16, false, WIDE, false>(count, ring);
  return tex ? plain_kernel<32, false, WIDE, true>(count, ring) : plain_kernel<32, false, WIDE, false>(count, ring);
}

}  // namespace

// The kernel a render of this plan runs (fn == nullptr: no kernel fits the plan).
KernelChoice choose_kernel(const DevScene& S, const DevJob& J, int stack, bool count, int variant) {
  if (variant == 5) return treelet_kernel(S, J, count);
  if (variant == 3 || variant == 0)
    return S.node_width == 4 ? default_kernel<4>(S, J, count, stack, variant == 3)
                             : default_kernel<2>(S, J, count, stack, variant == 3);
  return {};
}

hipError_t launch_render(const KernelChoice& k, const DevScene& S, const DevCamera& C, const DevJob& J,
                         int lds_bytes, int grid_blocks, hipStream_t stream) {
  if (J.row_count <= 0 || C.width <= 0) return hipSuccess;
  if (!k.fn) return hipErrorInvalidValue;
  if (k.dynamic_lds) {
    const hipError_t e = hipFuncSetAttribute(k.fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
    if (e != hipSuccess) return e;
  }
  const dim3 grid(grid_blocks);
  DevScene s = S;
  DevCamera c = C;
  DevJob j = J;
  void* args[] = {&s, &c, &j};
  return hipLaunchKernel(k.fn, grid, dim3(k.block), args, k.dynamic_lds ? lds_bytes : 0, stream);
}

// Registers / scratch of a compiled kernel (hipFuncGetAttributes on its code object).
KernelResources kernel_resources(const void* fn) {
  KernelResources r;
  if (!fn) return r;
  hipFuncAttributes a{};
  if (hipFuncGetAttributes(&a, fn) != hipSuccess) return r;
  r.ok = true;
  r.vgprs = a.numRegs;
  r.scratch = static_cast<int>(a.localSizeBytes);
  return r;
}


// Dynamic LDS bytes of the persistent kernel for this scene, or -1 when it does not fit in
// one CU's 160 KiB; fills the scene-copy offsets of the job.
int lds_layout(const DevScene& S, int stack, int waves, int esz, DevJob* J) {
  auto a16 = [](int64_t x) { return (x + 15) & ~int64_t(15); };
  // the node array first (at LDS address 0: inner-node codes are its byte offsets, <= 15 bits for
  // trees of <= 292 4-wide nodes, LdsStack16), then the traversal stacks (esz bytes per entry). Scenes
  // with noise textures (32-bit stacks) put the perlin gradient rows first instead: the noise lookup's
  // offsets carry the table's LDS address in 16 bits (perlin_noise), so at most 16 tables. Kernels
  // without image / noise textures (tex_full 0) copy no tables
  const int64_t perlins = S.tex_full ? S.num_perlins : 0;
  if (perlins > 16) return -1;
  const int64_t pvec = 0;
  const int64_t nodes = perlins * 256 * 16;
  int64_t off = a16(nodes + S.num_nodes * (S.node_width == 4 ? 112 : 64));
  const int64_t stacks = off;
  off = a16(off + int64_t(waves) * stack * 64 * esz);
  const int64_t spheres = off;
  off = a16(off + S.num_spheres * 16 * (J ? J->lds_sphere_f4 : 3));
  const int64_t quads = off;
  off = a16(off + S.num_quads * 80);
  const int64_t refs = off;
  off = a16(off + (S.ref_mode == 0 ? S.num_refs * 4 : 0));
  const int64_t materials = off;
  off = a16(off + int64_t(S.num_materials) * 32);
  const int64_t textures = off;
  off = a16(off + int64_t(S.num_textures) * 32);
  const int64_t pperm = off;
  off = a16(off + perlins * kPerlinPermWords * 4);
  const int64_t ring = off;  // RING kernels (J->ring_log2 >= 0): per-wave batch tables
  if (J && J->ring_log2 >= 0) off += int64_t(waves) * kRingEntries * 4;
  if (off > 160 * 1024) return -1;
  if (J) {
    J->lds_materials = static_cast<int32_t>(materials);
    J->lds_textures = static_cast<int32_t>(textures);
    J->lds_nodes = static_cast<int32_t>(nodes);
    J->lds_stacks = static_cast<int32_t>(stacks);
    J->lds_spheres = static_cast<int32_t>(spheres);
    J->lds_quads = static_cast<int32_t>(quads);
    J->lds_refs = static_cast<int32_t>(refs);
    J->lds_perlin_vec = static_cast<int32_t>(pvec);
    J->lds_perlin_perm = static_cast<int32_t>(pperm);
    J->lds_ring = static_cast<int32_t>(ring);
  }
  return static_cast<int>(off);
}

// Dynamic LDS of the treelet schedule: the stacks, then as many of the first (breadth-first) 4-wide
// nodes as fit in the rest of one CU's 160 KiB; sets S.treelet_bytes and J.lds_nodes.
int lds_layout_treelet(DevScene* S, int stack, int waves, DevJob* J) {
  const int64_t stacks = int64_t(waves) * stack * 64 * 4;
  const int64_t ring = J->ring_log2 >= 0 ? int64_t(waves) * kRingEntries * 4 : 0;  // RING: batch tables
  const int64_t room = 160 * 1024 - stacks - ring;
  const int64_t nb = node_bytes(S->node_width);
  if (S->node_width < 4 || room < nb) return -1;
  const int64_t nodes = std::min<int64_t>(S->num_nodes, room / nb);
  S->treelet_bytes = static_cast<int32_t>(nodes * nb);
  J->lds_ring = static_cast<int32_t>(stacks);
  J->lds_nodes = static_cast<int32_t>(stacks + ring);
  J->lds_stacks = 0;
  return static_cast<int>(stacks + ring + nodes * nb);
}

// The dual launch (rtg_api.cpp) needs the 16-wave workgroup's four waves and the 4-wave workgroup's
// one wave of a SIMD to fit its 512 registers per lane together (allocation granule 8): checked on the
// compiled kernel, so a later change that grows it drops the dual launch instead of leaving its
// second workgroup to run after the first has taken all the work.
bool dual_fits_registers(bool count, bool ring, bool verbose) {
  // both workgroups run the 4-wave build (default_kernel)
  const KernelResources r = kernel_resources(
      count  ? reinterpret_cast<const void*>(&render_kernel_lds<kLdsStack, false, true, 4, 4, false, kGeomLds, false>)
      : ring ? reinterpret_cast<const void*>(&render_kernel_lds<kLdsStack, false, false, 4, 4, false, kGeomLds, true>)
             : reinterpret_cast<const void*>(&render_kernel_lds<kLdsStack, false, false, 4, 4, false, kGeomLds, false>));
  if (verbose) std::fprintf(stderr, "[rtg] dual check: numRegs %d\n", r.vgprs);
  if (!r.ok) return false;
  return 5 * ((r.vgprs + 7) / 8 * 8) <= 512;
}

// Widen the culling margin of a node array in place (a camera farther out than the origin bound the boxes
// were padded for, rtg_api.cpp ensure_origin_bound): every finite box plane moves outward by delta (+ a
// 2^-22 |v| guard for this subtraction's own rounding); codes and empty slots (+-inf) are left alone.
// width 4: 28 floats per node (12 lo, 12 hi, 4 codes); width 2: 16 (lo, hi, lo, hi, 4 codes).
__global__ __launch_bounds__(256) void repad_nodes_kernel(float* __restrict__ nodes, int64_t n_floats, int width,
                                                          float delta) {
  const int64_t k = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k >= n_floats) return;
  const int w = static_cast<int>(k % (width == 4 ? 28 : 16));
  int side;  // -1 lo plane, +1 hi plane, 0 code
  if (width == 4)
    side = w < 12 ? -1 : (w < 24 ? 1 : 0);
  else
    side = w < 12 ? ((w % 6) < 3 ? -1 : 1) : 0;
  const float v = nodes[k];
  if (side == 0 || !(fabsf(v) < __builtin_inff())) return;
  const float g = delta + fabsf(v) * 0x1p-22f;
  nodes[k] = side < 0 ? v - g : v + g;
}

hipError_t launch_repad(float* nodes, int64_t num_nodes, int width, float delta, hipStream_t stream) {
  const int64_t n = num_nodes * (width == 4 ? 28 : 16);
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(repad_nodes_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, stream, nodes,
                     n, width, delta);
  return hipGetLastError();
}

hipError_t launch_combine(const float* partial, float* out, int64_t n_pixels, int chunks, float scale,
                          hipStream_t stream) {
  if (n_pixels <= 0) return hipSuccess;
  const unsigned blocks = static_cast<unsigned>((n_pixels * 3 + 255) / 256);
  hipLaunchKernelGGL(combine_kernel, dim3(blocks), dim3(256), 0, stream, partial, out, n_pixels, chunks, scale);
  return hipGetLastError();
}

hipError_t launch_resolve(const float* in, uint8_t* out, int64_t n_pixels, hipStream_t stream) {
  if (n_pixels <= 0) return hipSuccess;
  const int64_t total = n_pixels * 3;
  const unsigned blocks = static_cast<unsigned>((total + 255) / 256);
  hipLaunchKernelGGL(resolve_kernel, dim3(blocks), dim3(256), 0, stream, in, out, n_pixels);
  return hipGetLastError();
}

}  // namespace rtg
