// common/color.hpp — color alias and the PPM pixel writer (color.hpp:8-58).
#pragma once
#include <cmath>
#include <iostream>

#include "common/interval.hpp"
#include "common/vec3.hpp"

using color = vec3;

inline double linear_to_gamma(double linear_component) {
  return linear_component > 0.0f ? std::sqrt(linear_component) : 0.0f;
}

// gamma 2, clamp to [0, 0.999], scale to [0, 255]; same bytes as the reference.
inline void write_color(std::ostream& out, const color& pixel_color) {
  static const interval intensity(0.000f, 0.999f);
  const int r = int(256 * intensity.clamp(linear_to_gamma(pixel_color.x())));
  const int g = int(256 * intensity.clamp(linear_to_gamma(pixel_color.y())));
  const int b = int(256 * intensity.clamp(linear_to_gamma(pixel_color.z())));
  out << r << ' ' << g << ' ' << b << '\n';
}
