// common/interval.hpp — closed/open parameter range (interval.hpp:10-80).
#pragma once
#include <limits>

const double infinity = std::numeric_limits<double>::infinity();
const double pi = 3.1415926535897932385;

class interval {
 public:
  double min, max;

  interval() : min(+infinity), max(-infinity) {}
  interval(double lo, double hi) : min(lo), max(hi) {}
  interval(const interval& a, const interval& b)  // tightest interval enclosing both
      : min(a.min <= b.min ? a.min : b.min), max(a.max >= b.max ? a.max : b.max) {}

  double size() const { return max - min; }
  bool contains(double x) const { return min <= x && x <= max; }
  bool surrounds(double x) const { return min < x && x < max; }
  double clamp(double x) const { return x < min ? min : (x > max ? max : x); }
  interval expand(double delta) const {
    const double padding = delta / 2.0f;
    return interval(min - padding, max + padding);
  }

  static const interval empty, universe;
};

inline const interval interval::empty = interval(+infinity, -infinity);
inline const interval interval::universe = interval(-infinity, +infinity);

inline interval operator+(const interval& ival, double displacement) {
  return interval(ival.min + displacement, ival.max + displacement);
}
inline interval operator+(double displacement, const interval& ival) { return ival + displacement; }
