// common/random.hpp — the reference's host RNG helpers (rtweekend.hpp:23-39): glibc rand(), never
// seeded by the library. Scene construction code (e.g. bouncing_spheres) draws from it exactly as
// in the reference; rendering does NOT (the device uses the counter RNG of DESIGN.md §RNG).
#pragma once
#include <cstdlib>

inline double random_double() { return std::rand() / (RAND_MAX + 1.0f); }  // float division (H3)
inline double random_double(double min, double max) { return min + (max - min) * random_double(); }
inline int random_int(int min, int max) { return int(random_double(min, max + 1)); }
