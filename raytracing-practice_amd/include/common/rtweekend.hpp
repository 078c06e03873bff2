// common/rtweekend.hpp — umbrella header of the reference (rtweekend.hpp:1-47).
#pragma once
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <limits>
#include <memory>
#include <string>

#include "common/interval.hpp"
#include "common/random.hpp"

inline double degrees_to_radians(double degrees) { return degrees * pi / 180.0f; }

#include "common/color.hpp"
#include "common/ray.hpp"
#include "common/vec3.hpp"
