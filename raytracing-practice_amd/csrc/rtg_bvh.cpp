// rtg_bvh.cpp — host BVH construction for the device scene.
//
// RTG_BVH_MEDIAN reproduces bvh_node's topology (reference src/accelerator/bvh_node.hpp:25-77):
// node box = union of its objects' boxes, split axis = aabb::longest_axis (aabb.hpp:116-127),
// std::sort of the object range by bbox.min on that axis (bvh_node.hpp:69, 109-133), children
// [start, mid) / [mid, end) with mid = start + span/2; a 1-object node keeps that object once
// (the reference stores it as both children, H8), a 2-object node has two 1-object leaves.
// The tree is emitted in child-pair form: every node stores both children's boxes, so the
// traversal tests the two boxes the reference's left->hit / right->hit would test.
//
// RTG_BVH_SAH is this library's own binned-SAH builder (32 centroid bins on each of the three axes,
// leaves <= 4).
#include <array>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>

#include "rtg_internal.hpp"

namespace rtg {
namespace {

constexpr double kInf = std::numeric_limits<double>::infinity();

struct Box {
  double lo[3] = {kInf, kInf, kInf};
  double hi[3] = {-kInf, -kInf, -kInf};
};

// interval::expand / aabb::pad_to_minimums (interval.hpp:48-52, aabb.hpp:135-154)
void pad_to_minimums(Box& b) {
  const double delta = 0.0001;
  for (int a = 0; a < 3; ++a) {
    if (b.hi[a] - b.lo[a] < delta) {
      const double padding = delta / 2.0f;
      b.lo[a] -= padding;
      b.hi[a] += padding;
    }
  }
}

// aabb(point a, point b) (aabb.hpp:30-39)
Box box_from_points(const double a[3], const double b[3]) {
  Box r;
  for (int k = 0; k < 3; ++k) {
    if (a[k] <= b[k]) {
      r.lo[k] = a[k];
      r.hi[k] = b[k];
    } else {
      r.lo[k] = b[k];
      r.hi[k] = a[k];
    }
  }
  pad_to_minimums(r);
  return r;
}

// aabb(box0, box1) via interval(a, b) (aabb.hpp:42-48, interval.hpp:16-20)
Box box_union(const Box& a, const Box& b) {
  Box r;
  for (int k = 0; k < 3; ++k) {
    r.lo[k] = a.lo[k] <= b.lo[k] ? a.lo[k] : b.lo[k];
    r.hi[k] = a.hi[k] >= b.hi[k] ? a.hi[k] : b.hi[k];
  }
  return r;
}

int longest_axis(const Box& b) {
  const double sx = b.hi[0] - b.lo[0], sy = b.hi[1] - b.lo[1], sz = b.hi[2] - b.lo[2];
  if (sx > sy) return sx > sz ? 0 : 2;
  return sy > sz ? 1 : 2;
}

double half_area(const Box& b) {
  const double dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
  if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.0;
  return dx * dy + dy * dz + dz * dx;
}

struct Builder {
  const std::vector<Box>& boxes;
  Bvh& out;
  std::vector<int64_t>& ids;

  int32_t leaf(int64_t first, int64_t count) {
    const int64_t slot = static_cast<int64_t>(out.refs.size());
    for (int64_t i = 0; i < count; ++i) out.refs.push_back(ids[first + i]);
    (void)slot;
    return -(1 + static_cast<int32_t>(slot));
  }

  void set_child(int32_t node, int side, int32_t code, int32_t count, const Box& b) {
    BuildNode& n = out.nodes[node];
    n.child[side] = code;
    n.count[side] = count;
    for (int k = 0; k < 3; ++k) {
      n.lo[side][k] = b.lo[k];
      n.hi[side][k] = b.hi[k];
    }
  }

  int32_t new_node() {
    BuildNode n;
    for (int s = 0; s < 2; ++s) {
      n.child[s] = kEmptyChild;
      n.count[s] = 0;
      for (int k = 0; k < 3; ++k) {
        n.lo[s][k] = kInf;
        n.hi[s][k] = -kInf;
      }
    }
    out.nodes.push_back(n);
    return static_cast<int32_t>(out.nodes.size() - 1);
  }

  Box range_box(int64_t start, int64_t end) const {
    Box b;  // aabb::empty
    for (int64_t i = start; i < end; ++i) b = box_union(b, boxes[ids[i]]);
    return b;
  }

  // ---- bvh_node(objects, start, end) ----
  int32_t median(int64_t start, int64_t end, int depth) {
    out.depth = std::max(out.depth, depth);
    const int32_t node = new_node();
    const Box bbox = range_box(start, end);
    const int axis = longest_axis(bbox);
    const int64_t span = end - start;
    if (span == 1) {
      set_child(node, 0, leaf(start, 1), 1, boxes[ids[start]]);
    } else if (span == 2) {
      set_child(node, 0, leaf(start, 1), 1, boxes[ids[start]]);
      set_child(node, 1, leaf(start + 1, 1), 1, boxes[ids[start + 1]]);
    } else {
      const std::vector<Box>& bx = boxes;
      std::sort(ids.begin() + start, ids.begin() + end,
                [&bx, axis](int64_t a, int64_t b) { return bx[a].lo[axis] < bx[b].lo[axis]; });
      const int64_t mid = start + span / 2;
      const Box lb = range_box(start, mid);
      const int32_t l = median(start, mid, depth + 1);
      set_child(node, 0, l, 0, lb);
      const Box rb = range_box(mid, end);
      const int32_t r = median(mid, end, depth + 1);
      set_child(node, 1, r, 0, rb);
    }
    return node;
  }

  // ---- binned SAH ----
  static constexpr int kMaxBins = 64;
  // 32 bins on all three axes (round 2; round 1: 16 on the longest centroid axis): book-1 -2.3 %,
  // Cornell -5 %, config 5 -0.5 %, +1.5 s of host build for 1M spheres
  int kBins = 32;          // centroid bins per axis
  int axes = 3;            // 1: the centroid box's longest axis only, 3: the best split over all three
  int kMaxLeaf = 4;        // primitives per leaf (<= 8, the leaf code's count field)
  double trav_cost = 0.5;  // cost of one more level relative to one primitive test (measured best)

  // Returns a child code for the range; `node_depth` = depth of the node that would own it.
  int32_t sah_child(int64_t start, int64_t end, const Box& bbox, int depth, int32_t* count) {
    const int64_t n = end - start;
    if (n <= 1) {
      *count = static_cast<int32_t>(n);
      return leaf(start, n);
    }
    int64_t mid = -1;
    Box cb;
    for (int64_t i = start; i < end; ++i) {
      const Box& b = boxes[ids[i]];
      for (int k = 0; k < 3; ++k) {
        const double c = 0.5 * (b.lo[k] + b.hi[k]);
        cb.lo[k] = std::min(cb.lo[k], c);
        cb.hi[k] = std::max(cb.hi[k], c);
      }
    }
    const int long_axis = longest_axis(cb);
    int axis = long_axis;
    const double leaf_cost = static_cast<double>(n) * half_area(bbox);
    if (cb.hi[long_axis] - cb.lo[long_axis] > 0.0) {
      // binned SAH over the longest centroid axis (or all three): the best bin boundary
      double best = kInf;
      int best_split = -1, best_axis = long_axis;
      for (int ai = 0; ai < (axes == 3 ? 3 : 1); ++ai) {
        const int ax = axes == 3 ? ai : long_axis;
        const double extent = cb.hi[ax] - cb.lo[ax];
        if (!(extent > 0.0)) continue;
        Box bin_box[kMaxBins];
        int64_t bin_n[kMaxBins] = {0};
        const double k1 = kBins * (1.0 - 1e-9) / extent;
        for (int64_t i = start; i < end; ++i) {
          const Box& b = boxes[ids[i]];
          int bi = static_cast<int>((0.5 * (b.lo[ax] + b.hi[ax]) - cb.lo[ax]) * k1);
          bi = std::min(std::max(bi, 0), kBins - 1);
          bin_n[bi]++;
          bin_box[bi] = box_union(bin_box[bi], b);
        }
        double right_area[kMaxBins];
        int64_t right_n[kMaxBins];
        Box acc;
        int64_t accn = 0;
        for (int b = kBins - 1; b > 0; --b) {
          acc = box_union(acc, bin_box[b]);
          accn += bin_n[b];
          right_area[b] = half_area(acc);
          right_n[b] = accn;
        }
        Box lacc;
        int64_t lacc_n = 0;
        for (int b = 1; b < kBins; ++b) {
          lacc = box_union(lacc, bin_box[b - 1]);
          lacc_n += bin_n[b - 1];
          if (lacc_n == 0 || right_n[b] == 0) continue;
          const double cost = half_area(lacc) * lacc_n + right_area[b] * right_n[b];
          if (cost < best) {
            best = cost;
            best_split = b;
            best_axis = ax;
          }
        }
      }
      const double trav = trav_cost * half_area(bbox);
      if (n <= kMaxLeaf && leaf_cost <= best + trav) {
        *count = static_cast<int32_t>(n);
        return leaf(start, n);
      }
      if (best_split > 0) {
        axis = best_axis;
        const double k1 = kBins * (1.0 - 1e-9) / (cb.hi[axis] - cb.lo[axis]);
        auto it = std::partition(ids.begin() + start, ids.begin() + end, [&](int64_t id) {
          const Box& b = boxes[id];
          int bi = static_cast<int>((0.5 * (b.lo[axis] + b.hi[axis]) - cb.lo[axis]) * k1);
          return std::min(std::max(bi, 0), kBins - 1) < best_split;
        });
        mid = it - ids.begin();
      }
    } else if (n <= kMaxLeaf) {
      *count = static_cast<int32_t>(n);
      return leaf(start, n);
    }
    if (mid <= start || mid >= end) {  // degenerate: split by object median on the axis
      std::nth_element(ids.begin() + start, ids.begin() + start + n / 2, ids.begin() + end,
                       [&](int64_t a, int64_t b) {
                         return boxes[a].lo[axis] + boxes[a].hi[axis] <
                                boxes[b].lo[axis] + boxes[b].hi[axis];
                       });
      mid = start + n / 2;
    }
    *count = 0;
    const int32_t node = new_node();
    out.depth = std::max(out.depth, depth);
    const Box lb = range_box(start, mid);
    const Box rb = range_box(mid, end);
    int32_t lc = 0, rc = 0;
    const int32_t l = sah_child(start, mid, lb, depth + 1, &lc);
    set_child(node, 0, l, lc, lb);
    const int32_t r = sah_child(mid, end, rb, depth + 1, &rc);
    set_child(node, 1, r, rc, rb);
    return node;
  }
};

}  // namespace

void prim_bbox(const rtg_primitive& p, double lo[3], double hi[3]) {
  Box b;
  if (p.kind == RTG_PRIM_SPHERE) {
    const double r = p.radius;
    // center = ray(center1, center2 - center1) (sphere.hpp:32-44); static: direction 0.
    double dir[3], at0[3], at1[3];
    for (int k = 0; k < 3; ++k) {
      dir[k] = p.p1[k] - p.p0[k];
      at0[k] = p.p0[k] + 0.0 * dir[k];
      at1[k] = p.p0[k] + 1.0 * dir[k];
    }
    double a0[3], b0[3], a1[3], b1[3];
    for (int k = 0; k < 3; ++k) {
      a0[k] = at0[k] - r;
      b0[k] = at0[k] + r;
      a1[k] = at1[k] - r;
      b1[k] = at1[k] + r;
    }
    const bool moving = p.p1[0] != p.p0[0] || p.p1[1] != p.p0[1] || p.p1[2] != p.p0[2];
    if (!moving) {
      double sa[3], sb[3];
      for (int k = 0; k < 3; ++k) {
        sa[k] = p.p0[k] - r;
        sb[k] = p.p0[k] + r;
      }
      b = box_from_points(sa, sb);
    } else {
      b = box_union(box_from_points(a0, b0), box_from_points(a1, b1));
    }
  } else {
    double quv[3], qu[3], qv[3];
    for (int k = 0; k < 3; ++k) {
      qu[k] = p.p0[k] + p.p1[k];
      quv[k] = qu[k] + p.p2[k];
      qv[k] = p.p0[k] + p.p2[k];
    }
    b = box_union(box_from_points(p.p0, quv), box_from_points(qu, qv));
  }
  for (int k = 0; k < 3; ++k) {
    lo[k] = b.lo[k];
    hi[k] = b.hi[k];
  }
}

void collapse_bvh4(const Bvh& bin, Bvh4* out) {
  out->nodes.clear();
  out->depth = 0;
  out->max_pushes = 0;
  if (bin.nodes.empty()) return;
  struct Slot {
    int32_t code, count;
    Box box;
  };
  auto slot_of = [&](const BuildNode& n, int side) {
    Slot sl;
    sl.code = n.child[side];
    sl.count = n.count[side];
    for (int k = 0; k < 3; ++k) {
      sl.box.lo[k] = n.lo[side][k];
      sl.box.hi[k] = n.hi[side][k];
    }
    return sl;
  };
  // recursive collapse into pre-allocated nodes; tracks depth and stack pushes on the path
  struct Rec {
    const Bvh& bin;
    Bvh4* out;
    decltype(slot_of)& slot;
    std::vector<Slot> gather(int32_t b) {
      std::vector<Slot> slots;
      const BuildNode& n = bin.nodes[b];
      for (int side = 0; side < 2; ++side)
        if (n.child[side] != kEmptyChild) slots.push_back(slot(n, side));
      while (slots.size() < 4) {
        int best = -1;
        double best_area = -1.0;
        for (size_t i = 0; i < slots.size(); ++i) {
          if (slots[i].code < 0) continue;
          const double a = half_area(slots[i].box);
          if (a > best_area) {
            best_area = a;
            best = static_cast<int>(i);
          }
        }
        if (best < 0) break;
        const BuildNode& c = bin.nodes[slots[best].code];
        std::vector<Slot> kids;
        for (int side = 0; side < 2; ++side)
          if (c.child[side] != kEmptyChild) kids.push_back(slot(c, side));
        if (kids.size() + slots.size() - 1 > 4) break;
        slots.erase(slots.begin() + best);
        slots.insert(slots.begin() + best, kids.begin(), kids.end());
      }
      return slots;
    }
    std::array<int32_t, 4> children(const std::vector<Slot>& slots, int depth, int pushes) {
      out->depth = std::max(out->depth, depth);
      const int here = pushes + static_cast<int>(slots.size()) - 1;
      out->max_pushes = std::max(out->max_pushes, here);
      std::array<int32_t, 4> codes = {kEmptyChild, kEmptyChild, kEmptyChild, kEmptyChild};
      // the inner children of a node are allocated next to each other (then filled depth-first),
      // so the siblings a ray visits after the nearest one share its cache lines
      int32_t slot_ids[4] = {-1, -1, -1, -1};
      for (size_t i = 0; i < slots.size(); ++i)
        if (slots[i].code >= 0) {
          slot_ids[i] = static_cast<int32_t>(out->nodes.size());
          out->nodes.push_back(BuildNode4{});
        }
      for (size_t i = 0; i < slots.size(); ++i)
        codes[i] = slots[i].code >= 0 ? fill(slot_ids[i], slots[i].code, depth + 1, here) : slots[i].code;
      return codes;
    }
    int32_t fill(int32_t me, int32_t b, int depth, int pushes) {
      std::vector<Slot> slots = gather(b);
      std::array<int32_t, 4> codes = children(slots, depth, pushes);
      BuildNode4& o = out->nodes[me];
      for (int i = 0; i < 4; ++i) {
        o.child[i] = codes[i];
        o.count[i] = i < static_cast<int>(slots.size()) ? slots[i].count : 0;
        for (int k = 0; k < 3; ++k) {
          o.lo[i][k] = i < static_cast<int>(slots.size()) ? slots[i].box.lo[k] : kInf;
          o.hi[i][k] = i < static_cast<int>(slots.size()) ? slots[i].box.hi[k] : -kInf;
        }
      }
      return me;
    }
  } rec{bin, out, slot_of};
  out->nodes.push_back(BuildNode4{});  // the root is node 0
  rec.fill(0, 0, 1, 0);
}

void reorder_top_bfs(Bvh4* t, int64_t top) {
  const int64_t n = static_cast<int64_t>(t->nodes.size());
  if (n <= 1 || top <= 1) return;
  // the first `top` nodes of a breadth-first walk from the root, then the rest in their (depth-first)
  // order; a node's inner children stay next to each other in both parts
  std::vector<int32_t> order;
  order.reserve(n);
  std::vector<char> taken(n, 0);
  order.push_back(0);
  taken[0] = 1;
  for (size_t head = 0; head < order.size() && static_cast<int64_t>(order.size()) < top; ++head)
    for (int c = 0; c < 4 && static_cast<int64_t>(order.size()) < top; ++c) {
      const int32_t ch = t->nodes[order[head]].child[c];
      if (ch >= 0 && !taken[ch]) {
        taken[ch] = 1;
        order.push_back(ch);
      }
    }
  for (int32_t k = 0; k < n; ++k)
    if (!taken[k]) order.push_back(k);
  std::vector<int32_t> pos(n);
  for (int32_t k = 0; k < n; ++k) pos[order[k]] = k;
  std::vector<BuildNode4> out(n);
  for (int32_t k = 0; k < n; ++k) {
    out[k] = t->nodes[order[k]];
    for (int c = 0; c < 4; ++c)
      if (out[k].child[c] >= 0) out[k].child[c] = pos[out[k].child[c]];
  }
  t->nodes.swap(out);
}

bool build_bvh(const rtg_scene_desc* desc, Bvh* out, std::string* err) {
  out->nodes.clear();
  out->refs.clear();
  out->depth = 0;
  const int64_t n = desc->num_prims;
  if (n <= 0) return true;  // empty world: no nodes, every ray misses
  if (n > (int64_t(1) << 29)) {
    *err = "too many primitives";
    return false;
  }
  std::vector<Box> boxes(n);
  for (int64_t i = 0; i < n; ++i) prim_bbox(desc->prims[i], boxes[i].lo, boxes[i].hi);
  std::vector<int64_t> ids(n);
  for (int64_t i = 0; i < n; ++i) ids[i] = i;
  out->nodes.reserve(n * 2);
  out->refs.reserve(n);
  Builder b{boxes, *out, ids};
  // RTG_SAH_TUNE="trav_cost:max_leaf[:axes[:bins]]" overrides the SAH constants (tuning experiments only)
  if (const char* tune = std::getenv("RTG_SAH_TUNE")) {
    double ct = 0.0;
    int ml = 0, ax = 3, nb = 32;
    if (std::sscanf(tune, "%lf:%d:%d:%d", &ct, &ml, &ax, &nb) >= 2 && ct > 0.0 && ml >= 1 && ml <= 8) {
      b.trav_cost = ct;
      b.kMaxLeaf = ml;
      b.axes = ax == 3 ? 3 : 1;
      b.kBins = std::min(std::max(nb, 2), int(Builder::kMaxBins));
    }
  }
  if (desc->bvh_mode == RTG_BVH_MEDIAN) {
    b.median(0, n, 1);
  } else if (desc->bvh_mode == RTG_BVH_SAH) {
    Box all;
    for (int64_t i = 0; i < n; ++i) all = box_union(all, boxes[i]);
    int32_t cnt = 0;
    const int32_t code = b.sah_child(0, n, all, 1, &cnt);
    if (code < 0) {  // the whole scene is one leaf: wrap it into a root node
      const int32_t root = b.new_node();
      out->depth = 1;
      b.set_child(root, 0, code, cnt, all);
    }
  } else {
    *err = "unknown bvh_mode";
    return false;
  }
  return true;
}

}  // namespace rtg
