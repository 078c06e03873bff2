// core/perlin.hpp — gradient noise with 256 random unit vectors and three permutations
// (perlin.hpp:9-266). Tables are drawn from rand() at construction in the reference's order.
#pragma once
#include "common/rtweekend.hpp"
#include "rtgpu.h"

class perlin {
 public:
  perlin() {
    for (int i = 0; i < point_count; ++i) randvec[i] = unit_vector(vec3::random(-1.0f, 1.0f));
    generate_perm(perm_x);
    generate_perm(perm_y);
    generate_perm(perm_z);
  }

  // The reference reads an uninitialised randfloat[] here (perlin.hpp:259); this mirror keeps
  // it zero-filled so both unused helpers are at least deterministic.
  double noise_hash(const point3& p) const {
    const int i = int(4 * p.x()) & 255, j = int(4 * p.y()) & 255, k = int(4 * p.z()) & 255;
    return randfloat[perm_x[i] ^ perm_y[j] ^ perm_z[k]];
  }
  double noise_trilinear(const point3& p) const {
    double u = p.x() - std::floor(p.x()), v = p.y() - std::floor(p.y()), w = p.z() - std::floor(p.z());
    u = u * u * (3 - 2 * u);
    v = v * v * (3 - 2 * v);
    w = w * w * (3 - 2 * w);
    const int i = int(std::floor(p.x())), j = int(std::floor(p.y())), k = int(std::floor(p.z()));
    auto accum = 0.0f;
    for (int di = 0; di < 2; ++di)
      for (int dj = 0; dj < 2; ++dj)
        for (int dk = 0; dk < 2; ++dk)
          accum += (di * u + (1 - di) * (1 - u)) * (dj * v + (1 - dj) * (1 - v)) *
                   (dk * w + (1 - dk) * (1 - w)) *
                   randfloat[perm_x[(i + di) & 255] ^ perm_y[(j + dj) & 255] ^ perm_z[(k + dk) & 255]];
    return accum;
  }

  double noise_perlin(const point3& p) const {
    const double u = p.x() - std::floor(p.x()), v = p.y() - std::floor(p.y()), w = p.z() - std::floor(p.z());
    const int i = int(std::floor(p.x())), j = int(std::floor(p.y())), k = int(std::floor(p.z()));
    const double uu = u * u * (3 - 2 * u), vv = v * v * (3 - 2 * v), ww = w * w * (3 - 2 * w);
    auto accum = 0.0f;  // float accumulator, as in the reference (H6)
    for (int di = 0; di < 2; ++di)
      for (int dj = 0; dj < 2; ++dj)
        for (int dk = 0; dk < 2; ++dk) {
          const vec3& c = randvec[perm_x[(i + di) & 255] ^ perm_y[(j + dj) & 255] ^ perm_z[(k + dk) & 255]];
          const vec3 weight_v(u - di, v - dj, w - dk);
          accum += (di * uu + (1 - di) * (1 - uu)) * (dj * vv + (1 - dj) * (1 - vv)) *
                   (dk * ww + (1 - dk) * (1 - ww)) * dot(c, weight_v);
        }
    return accum;
  }

  // Sum of |2^-k noise(2^k p)| over `depth` octaves (fp32 accumulator, H6).
  double turb(const point3& p, int depth) const {
    auto accum = 0.0f;
    point3 tp = p;
    auto weight = 1.0f;
    for (int i = 0; i < depth; ++i) {
      accum += weight * noise_perlin(tp);
      weight *= 0.5f;
      tp *= 2.0f;
    }
    return std::fabs(accum);
  }

  // Device export (extension).
  rtg_perlin tables() const {
    rtg_perlin t{};
    for (int i = 0; i < point_count; ++i)
      for (int a = 0; a < 3; ++a) t.randvec[i][a] = randvec[i][a];
    for (int i = 0; i < point_count; ++i) {
      t.perm_x[i] = perm_x[i];
      t.perm_y[i] = perm_y[i];
      t.perm_z[i] = perm_z[i];
    }
    return t;
  }

 private:
  static const int point_count = 256;
  double randfloat[point_count] = {};
  vec3 randvec[point_count];
  int perm_x[point_count], perm_y[point_count], perm_z[point_count];

  static void generate_perm(int* p) {
    for (int i = 0; i < point_count; ++i) p[i] = i;
    // Fisher-Yates from the top. random_int(0, i) can return i + 1 when random_double() rounds
    // to 1.0 (H3); kept as in the reference except at i = 255, where the reference would index
    // past the table (undefined behaviour) and this mirror clamps.
    for (int i = point_count - 1; i > 0; --i) {
      int target = random_int(0, i);
      if (target > point_count - 1) target = point_count - 1;
      const int tmp = p[i];
      p[i] = p[target];
      p[target] = tmp;
    }
  }
};
