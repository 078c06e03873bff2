// common/vec3.hpp — vec3 / point3 / color API of the reference (vec3.hpp:8-226), host fp64.
#pragma once
#include <cmath>
#include <iostream>

#include "common/random.hpp"

class vec3 {
 public:
  double e[3];

  vec3() : e{0, 0, 0} {}
  vec3(double x, double y, double z) : e{x, y, z} {}

  double x() const { return e[0]; }
  double y() const { return e[1]; }
  double z() const { return e[2]; }

  vec3 operator-() const { return vec3(-e[0], -e[1], -e[2]); }
  double operator[](int i) const { return e[i]; }
  double& operator[](int i) { return e[i]; }

  vec3& operator+=(const vec3& o) {
    for (int k = 0; k < 3; ++k) e[k] += o.e[k];
    return *this;
  }
  vec3& operator*=(double t) {
    for (double& c : e) c *= t;
    return *this;
  }
  vec3& operator/=(double t) { return *this *= 1 / t; }

  double length_squared() const { return e[0] * e[0] + e[1] * e[1] + e[2] * e[2]; }
  double length() const { return std::sqrt(length_squared()); }

  // Reproduces the reference's near_zero exactly, including fabs(e[1] < s) (hazard H5).
  bool near_zero() const {
    const double s = 1e-8;
    return std::fabs(e[0]) < s && std::fabs(double(e[1] < s)) != 0 && std::fabs(e[2]) < s;
  }

  // Draws are explicitly sequenced z, y, x: the order GCC gives the reference's
  // vec3(random_double(), random_double(), random_double()) (hazard H2), on any compiler.
  static vec3 random() {
    const double z = random_double(), y = random_double(), x = random_double();
    return vec3(x, y, z);
  }
  static vec3 random(double min, double max) {
    const double z = random_double(min, max), y = random_double(min, max), x = random_double(min, max);
    return vec3(x, y, z);
  }
};

using point3 = vec3;

inline std::ostream& operator<<(std::ostream& out, const vec3& v) {
  return out << v.e[0] << ' ' << v.e[1] << ' ' << v.e[2];
}
inline vec3 operator+(const vec3& a, const vec3& b) { return vec3(a.e[0] + b.e[0], a.e[1] + b.e[1], a.e[2] + b.e[2]); }
inline vec3 operator-(const vec3& a, const vec3& b) { return vec3(a.e[0] - b.e[0], a.e[1] - b.e[1], a.e[2] - b.e[2]); }
inline vec3 operator*(const vec3& a, const vec3& b) { return vec3(a.e[0] * b.e[0], a.e[1] * b.e[1], a.e[2] * b.e[2]); }
inline vec3 operator*(double t, const vec3& v) { return vec3(t * v.e[0], t * v.e[1], t * v.e[2]); }
inline vec3 operator*(const vec3& v, double t) { return t * v; }
inline vec3 operator/(vec3 v, double t) { return (1 / t) * v; }
inline double dot(const vec3& a, const vec3& b) { return a.e[0] * b.e[0] + a.e[1] * b.e[1] + a.e[2] * b.e[2]; }
inline vec3 cross(const vec3& a, const vec3& b) {
  return vec3(a.e[1] * b.e[2] - a.e[2] * b.e[1], a.e[2] * b.e[0] - a.e[0] * b.e[2],
              a.e[0] * b.e[1] - a.e[1] * b.e[0]);
}
inline vec3 unit_vector(vec3 v) { return v / v.length(); }

// Rejection samplers (vec3.hpp:158-204); draw order as GCC evaluates the reference (y then x).
inline vec3 random_in_unit_disk() {
  for (;;) {
    const double y = random_double(-1.0f, 1.0f);
    const double x = random_double(-1.0f, 1.0f);
    const vec3 p(x, y, 0.0f);
    if (p.length_squared() < 1.0f) return p;
  }
}
inline vec3 random_unit_vector() {
  for (;;) {
    const vec3 p = vec3::random(-1, 1);
    const double lensq = p.length_squared();
    if (1e-160 < lensq && lensq <= 1) return p / std::sqrt(lensq);
  }
}
inline vec3 random_on_hemisphere(const vec3& normal) {
  const vec3 v = random_unit_vector();
  return dot(v, normal) > 0.0f ? v : -v;
}
inline vec3 reflect(const vec3& v, const vec3& n) { return v - 2.0f * dot(v, n) * n; }
inline vec3 refract(const vec3& uv, const vec3& n, double etai_over_etat) {
  const double cos_theta = std::fmin(dot(-uv, n), 1.0f);
  const vec3 perp = etai_over_etat * (uv + cos_theta * n);
  const vec3 parallel = -std::sqrt(std::fabs(1.0f - perp.length_squared())) * n;
  return perp + parallel;
}
