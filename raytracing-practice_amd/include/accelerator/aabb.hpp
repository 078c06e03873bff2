// accelerator/aabb.hpp — axis-aligned box (aabb.hpp:12-173), host fp64.
#pragma once
#include "common/rtweekend.hpp"

class aabb {
 public:
  interval x, y, z;

  aabb() {}
  aabb(const interval& x, const interval& y, const interval& z) : x(x), y(y), z(z) { pad_to_minimums(); }
  aabb(const point3& a, const point3& b)
      : x(a[0] <= b[0] ? interval(a[0], b[0]) : interval(b[0], a[0])),
        y(a[1] <= b[1] ? interval(a[1], b[1]) : interval(b[1], a[1])),
        z(a[2] <= b[2] ? interval(a[2], b[2]) : interval(b[2], a[2])) {
    pad_to_minimums();
  }
  aabb(const aabb& box0, const aabb& box1)  // union, no padding
      : x(box0.x, box1.x), y(box0.y, box1.y), z(box0.z, box1.z) {}

  const interval& axis_interval(int n) const { return n == 1 ? y : (n == 2 ? z : x); }

  // Slab test; false when the clipped range is empty (max <= min).
  bool hit(const ray& r, interval ray_t) const {
    const point3& o = r.origin();
    const vec3& d = r.direction();
    for (int axis = 0; axis < 3; ++axis) {
      const interval& ax = axis_interval(axis);
      const double adinv = 1.0f / d[axis];
      const double t0 = (ax.min - o[axis]) * adinv;
      const double t1 = (ax.max - o[axis]) * adinv;
      const double lo = t0 < t1 ? t0 : t1, hi = t0 < t1 ? t1 : t0;
      if (lo > ray_t.min) ray_t.min = lo;
      if (hi < ray_t.max) ray_t.max = hi;
      if (ray_t.max <= ray_t.min) return false;
    }
    return true;
  }

  int longest_axis() const {
    if (x.size() > y.size()) return x.size() > z.size() ? 0 : 2;
    return y.size() > z.size() ? 1 : 2;
  }

  static const aabb empty, universe;

 private:
  void pad_to_minimums() {
    const double delta = 0.0001;
    if (x.size() < delta) x = x.expand(delta);
    if (y.size() < delta) y = y.expand(delta);
    if (z.size() < delta) z = z.expand(delta);
  }
};

inline const aabb aabb::empty = aabb(interval::empty, interval::empty, interval::empty);
inline const aabb aabb::universe = aabb(interval::universe, interval::universe, interval::universe);

inline aabb operator+(const aabb& b, const vec3& off) { return aabb(b.x + off.x(), b.y + off.y(), b.z + off.z()); }
inline aabb operator+(const vec3& off, const aabb& b) { return b + off; }
