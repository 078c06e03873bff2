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
#include <cstring>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <new>
#include <thread>

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

// Data-parallel loop over [start, end) in T contiguous chunks (T-1 helper threads + this one).
template <class F>
void par_chunks(int64_t start, int64_t end, int T, F&& f) {
  if (T <= 1) {
    f(start, end, 0);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T - 1);
  const int64_t n = end - start;
  for (int t = 1; t < T; ++t)
    th.emplace_back([&, t]() { f(start + n * t / T, start + n * (t + 1) / T, t); });
  f(start, start + n / T, 0);
  for (auto& x : th) x.join();
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

};

// ---- binned SAH (RTG_BVH_SAH) ----
// Primitives travel with their boxes (one contiguous 56-B record each) instead of through an index
// array, and one pass per node bins every primitive on all three axes, keeping per bin the box, the
// centroid box and the count: the split's child boxes and child centroid boxes are unions of bins,
// so a node costs the binning pass and the partition (it was seven passes). Subtrees of large ranges
// build concurrently into their own buffers and are spliced back in depth-first order; the loops of
// the top levels run on the builder's threads. Unions are exact min / max and counts integers, and
// the partition is the sequential std::partition, so the tree is node for node the one the
// single-thread builder of round 2 produced (tests/test_host.py pins the hash).
struct PrimRec {
  double lo[3], hi[3];
  int64_t id;
};

struct SahBuilder {
  std::vector<PrimRec>& p;
  Bvh& out;
  int threads = 1;
  int kBins = 32;          // centroid bins per axis (round 2: 32 on all three axes; round 1: 16 on one)
  int axes = 3;            // 1: the centroid box's longest axis only, 3: the best split over all three
  int kMaxLeaf = 4;        // primitives per leaf (<= 8, the leaf code's count field)
  double trav_cost = 0.5;  // cost of one more level relative to one primitive test (measured best)
  bool parallel = false;   // build subtrees of large ranges concurrently
  static constexpr int kMaxBins = 64;
  static constexpr int64_t kParMin = 65536;    // ranges whose loops run data-parallel
  static constexpr int64_t kSpawnMin = 32768;  // ranges whose two subtrees build concurrently

  struct Bin {
    Box box, cbox;
    int64_t n = 0;
  };
  struct AxisBins {
    Bin b[3][kMaxBins];
  };

  static void add_point(Box& b, const double c[3]) {
    for (int k = 0; k < 3; ++k) {
      b.lo[k] = std::min(b.lo[k], c[k]);
      b.hi[k] = std::max(b.hi[k], c[k]);
    }
  }
  static void centroid(const PrimRec& r, double c[3]) {
    for (int k = 0; k < 3; ++k) c[k] = 0.5 * (r.lo[k] + r.hi[k]);
  }
  static Box box_of(const PrimRec& r) {
    Box b;
    for (int k = 0; k < 3; ++k) {
      b.lo[k] = r.lo[k];
      b.hi[k] = r.hi[k];
    }
    return b;
  }

  int32_t leaf(int64_t first, int64_t count) {
    const int64_t slot = static_cast<int64_t>(out.refs.size());
    for (int64_t i = 0; i < count; ++i) out.refs.push_back(p[first + i].id);
    return -(1 + static_cast<int32_t>(slot));
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
  void set_child(int32_t node, int side, int32_t code, int32_t count, const Box& b) {
    BuildNode& n = out.nodes[node];
    n.child[side] = code;
    n.count[side] = count;
    for (int k = 0; k < 3; ++k) {
      n.lo[side][k] = b.lo[k];
      n.hi[side][k] = b.hi[k];
    }
  }

  // box and centroid box of a range (root, and the rare degenerate split)
  void range_boxes(int64_t start, int64_t end, Box* bb, Box* cb) const {
    const int T = end - start >= kParMin ? threads : 1;
    std::vector<Box> pb(T), pc(T);
    par_chunks(start, end, T, [&](int64_t a, int64_t e, int t) {
      Box b, c;
      for (int64_t i = a; i < e; ++i) {
        double m[3];
        centroid(p[i], m);
        b = box_union(b, box_of(p[i]));
        add_point(c, m);
      }
      pb[t] = b;
      pc[t] = c;
    });
    *bb = Box{};
    *cb = Box{};
    for (int t = 0; t < T; ++t) {
      *bb = box_union(*bb, pb[t]);
      *cb = box_union(*cb, pc[t]);
    }
  }

  // Returns a child code for the range [start, end) with box `bbox` and centroid box `cb`.
  int32_t sah_child(int64_t start, int64_t end, const Box& bbox, const Box& cb, int depth, int32_t* count) {
    const int64_t n = end - start;
    if (n <= 1) {
      *count = static_cast<int32_t>(n);
      return leaf(start, n);
    }
    int64_t mid = -1;
    const int long_axis = longest_axis(cb);
    int axis = long_axis;
    const double leaf_cost = static_cast<double>(n) * half_area(bbox);
    Box lb, rb, lcb, rcb;
    bool child_boxes = false;
    if (cb.hi[long_axis] - cb.lo[long_axis] > 0.0) {
      bool use[3] = {false, false, false};
      double k1[3] = {0.0, 0.0, 0.0};
      for (int ai = 0; ai < (axes == 3 ? 3 : 1); ++ai) {
        const int ax = axes == 3 ? ai : long_axis;
        const double extent = cb.hi[ax] - cb.lo[ax];
        if (!(extent > 0.0)) continue;
        use[ax] = true;
        k1[ax] = kBins * (1.0 - 1e-9) / extent;
      }
      auto bin_of = [&](double c, int ax) {
        const int bi = static_cast<int>((c - cb.lo[ax]) * k1[ax]);
        return std::min(std::max(bi, 0), kBins - 1);
      };
      // bins are initialised on first touch and the sweeps visit the occupied ones only: a split
      // between two occupied bins costs the same wherever it falls between them, and the cost loop
      // keeps the first (strict <), i.e. the bin right after the lower one: the same split as a sweep
      // over every bin, without its fixed cost on the ~800k small nodes of a 1M-primitive tree
      Bin* bins[3];
      uint64_t occ[3] = {0, 0, 0};
      // uninitialised storage (a Bin's boxes start empty only when first touched: constructing all
      // 3 x 64 bins per node would write 20 KB for every node of the tree)
      alignas(Bin) unsigned char local_raw[sizeof(Bin) * 3 * kMaxBins];
      Bin* local = reinterpret_cast<Bin*>(local_raw);
      std::vector<AxisBins> part;
      const int T = n >= kParMin ? threads : 1;
      auto touch = [](Bin& bn, uint64_t& mask, int bi) {
        if (!(mask >> bi & 1)) {
          mask |= uint64_t(1) << bi;
          new (&bn) Bin();
        }
      };
      if (T == 1) {
        for (int ax = 0; ax < 3; ++ax) bins[ax] = local + ax * kMaxBins;
        for (int64_t i = start; i < end; ++i) {
          const PrimRec& r = p[i];
          double m[3];
          centroid(r, m);
          const Box bx = box_of(r);
          for (int ax = 0; ax < 3; ++ax) {
            if (!use[ax]) continue;
            const int bi = bin_of(m[ax], ax);
            Bin& bn = bins[ax][bi];
            touch(bn, occ[ax], bi);
            bn.n++;
            bn.box = box_union(bn.box, bx);
            add_point(bn.cbox, m);
          }
        }
      } else {
        part.resize(T);
        std::vector<std::array<uint64_t, 3>> pocc(T, std::array<uint64_t, 3>{0, 0, 0});
        par_chunks(start, end, T, [&](int64_t a, int64_t e, int t) {
          AxisBins& ab = part[t];
          for (int64_t i = a; i < e; ++i) {
            const PrimRec& r = p[i];
            double m[3];
            centroid(r, m);
            const Box bx = box_of(r);
            for (int ax = 0; ax < 3; ++ax) {
              if (!use[ax]) continue;
              const int bi = bin_of(m[ax], ax);
              Bin& bn = ab.b[ax][bi];
              touch(bn, pocc[t][ax], bi);
              bn.n++;
              bn.box = box_union(bn.box, bx);
              add_point(bn.cbox, m);
            }
          }
        });
        for (int ax = 0; ax < 3; ++ax) {
          bins[ax] = part[0].b[ax];
          occ[ax] = pocc[0][ax];
          for (int t = 1; t < T; ++t)
            for (int k = 0; k < kBins; ++k) {
              if (!(pocc[t][ax] >> k & 1)) continue;
              Bin& d = bins[ax][k];
              touch(d, occ[ax], k);
              const Bin& s = part[t].b[ax][k];
              d.n += s.n;
              d.box = box_union(d.box, s.box);
              d.cbox = box_union(d.cbox, s.cbox);
            }
        }
      }
      // the best bin boundary: the round-2 cost loop (axes in order, strict <: ties keep the first)
      double best = kInf;
      int best_split = -1, best_axis = long_axis;
      for (int ai = 0; ai < (axes == 3 ? 3 : 1); ++ai) {
        const int ax = axes == 3 ? ai : long_axis;
        if (!use[ax]) continue;
        int o[kMaxBins], m = 0;
        for (uint64_t w = occ[ax]; w; w &= w - 1) o[m++] = __builtin_ctzll(w);
        double right_area[kMaxBins];
        int64_t right_n[kMaxBins];
        Box acc;
        int64_t accn = 0;
        for (int j = m - 1; j > 0; --j) {
          acc = box_union(acc, bins[ax][o[j]].box);
          accn += bins[ax][o[j]].n;
          right_area[j] = half_area(acc);
          right_n[j] = accn;
        }
        Box lacc;
        int64_t lacc_n = 0;
        for (int j = 1; j < m; ++j) {
          lacc = box_union(lacc, bins[ax][o[j - 1]].box);
          lacc_n += bins[ax][o[j - 1]].n;
          const double cost = half_area(lacc) * lacc_n + right_area[j] * right_n[j];
          if (cost < best) {
            best = cost;
            best_split = o[j - 1] + 1;
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
        auto it = std::partition(p.begin() + start, p.begin() + end, [&](const PrimRec& r) {
          return bin_of(0.5 * (r.lo[axis] + r.hi[axis]), axis) < best_split;
        });
        mid = it - p.begin();
        for (uint64_t w = occ[axis]; w; w &= w - 1) {
          const int b = __builtin_ctzll(w);
          const Bin& bn = bins[axis][b];
          Box& box = b < best_split ? lb : rb;
          Box& cbox = b < best_split ? lcb : rcb;
          box = box_union(box, bn.box);
          cbox = box_union(cbox, bn.cbox);
        }
        child_boxes = true;
      }
    } else if (n <= kMaxLeaf) {
      *count = static_cast<int32_t>(n);
      return leaf(start, n);
    }
    if (mid <= start || mid >= end) {  // degenerate: split by object median on the axis
      std::nth_element(p.begin() + start, p.begin() + start + n / 2, p.begin() + end,
                       [&](const PrimRec& a, const PrimRec& b) {
                         return a.lo[axis] + a.hi[axis] < b.lo[axis] + b.hi[axis];
                       });
      mid = start + n / 2;
      child_boxes = false;
    }
    if (!child_boxes) {
      range_boxes(start, mid, &lb, &lcb);
      range_boxes(mid, end, &rb, &rcb);
    }
    *count = 0;
    const int32_t node = new_node();
    out.depth = std::max(out.depth, depth);
    int32_t lc = 0, rc = 0;
    if (parallel && n >= kSpawnMin) {
      // the two subtrees concurrently, each into its own buffers, then spliced in depth-first order.
      // Every range above kSpawnMin gets a thread of its own (~2n / kSpawnMin threads in all), so the
      // OS balances the uneven SAH subtrees over the cores; the data-parallel loops split the budget
      Bvh lt, rt;
      SahBuilder lb_{p, lt, std::max(1, threads / 2), kBins, axes, kMaxLeaf, trav_cost, parallel};
      SahBuilder rb_{p, rt, std::max(1, threads - threads / 2), kBins, axes, kMaxLeaf, trav_cost, parallel};
      int32_t lcode = 0, rcode = 0;
      std::thread left_thread([&]() { lcode = lb_.sah_child(start, mid, lb, lcb, depth + 1, &lc); });
      rcode = rb_.sah_child(mid, end, rb, rcb, depth + 1, &rc);
      left_thread.join();
      set_child(node, 0, splice(lt, lcode), lc, lb);
      set_child(node, 1, splice(rt, rcode), rc, rb);
      return node;
    }
    const int32_t l = sah_child(start, mid, lb, lcb, depth + 1, &lc);
    set_child(node, 0, l, lc, lb);
    const int32_t r = sah_child(mid, end, rb, rcb, depth + 1, &rc);
    set_child(node, 1, r, rc, rb);
    return node;
  }

  // Append a subtree built into its own buffers (root code `code`: node 0 of `t`, or a leaf) and
  // return its code in `out`: node indices shift by the nodes already in `out`, leaf slots by its refs
  // (the order a single-thread build would have numbered them in).
  int32_t splice(const Bvh& t, int32_t code) {
    const int32_t node_off = static_cast<int32_t>(out.nodes.size());
    const int32_t ref_off = static_cast<int32_t>(out.refs.size());
    auto fix = [&](int32_t c) {
      if (c == kEmptyChild) return c;
      return c >= 0 ? c + node_off : c - ref_off;  // leaf -(1 + slot) -> -(1 + slot + ref_off)
    };
    for (BuildNode n : t.nodes) {
      n.child[0] = fix(n.child[0]);
      n.child[1] = fix(n.child[1]);
      out.nodes.push_back(n);
    }
    out.refs.insert(out.refs.end(), t.refs.begin(), t.refs.end());
    out.depth = std::max(out.depth, t.depth);
    return fix(code);
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

// SAH-optimal W-wide collapse (the dynamic program of Ylitie, Karras and Laine, "Efficient
// Incoherent Ray Traversal on GPUs Through Compressed Wide BVHs", HPG 2017, at width W = 4 or 8): for
// every binary subtree and every budget i = 1..W of slots it may occupy under a wide parent, the cheapest
// representation by surface-area cost — one slot that is a merged leaf (its primitives are a
// contiguous ref range, <= max_leaf of them) or a wide node, or its two children sharing the budget.
// cost(wide node) = area x c_node + its slots; cost(leaf) = area x count x 1.
namespace {
template <int W>
struct CollapseDp {
  const Bvh& bin;
  double c_node;
  int max_leaf;
  std::vector<double> cost;   // [node][i], i = 0..W-1 for budgets 1..W
  std::vector<int8_t> pick;   // [node][i]: -1 = budget i-1 (i > 0), 0 = one slot, k = k slots to the left child
  std::vector<uint8_t> as_leaf;  // budget 1: merged leaf (1) or wide node (0)
  std::vector<int8_t> wide_k;    // slots of the left child when the node is a wide node (d[W])
  std::vector<int64_t> first, count;
  std::vector<Box> box;

  struct SlotRef {  // a child slot of a binary node: an inner node or a leaf range
    int32_t code, cnt;
    Box b;
  };
  SlotRef slot_of(int32_t node, int side) const {
    const BuildNode& n = bin.nodes[node];
    SlotRef s;
    s.code = n.child[side];
    s.cnt = n.count[side];
    for (int k = 0; k < 3; ++k) {
      s.b.lo[k] = n.lo[side][k];
      s.b.hi[k] = n.hi[side][k];
    }
    return s;
  }
  double slot_cost(const SlotRef& s, int i) const {  // budget i (1..W)
    if (s.code < 0) return half_area(s.b) * s.cnt;
    return cost[static_cast<size_t>(s.code) * W + (i - 1)];
  }

  void run() {
    const size_t n = bin.nodes.size();
    cost.assign(n * W, 0.0);
    pick.assign(n * W, 0);
    as_leaf.assign(n, 0);
    wide_k.assign(n, 0);
    first.assign(n, 0);
    count.assign(n, 0);
    box.assign(n, Box{});
    // node boxes from the parents' child slots (children follow their parent in depth-first order)
    box[0] = box_union(slot_of(0, 0).b, bin.nodes[0].child[1] != kEmptyChild ? slot_of(0, 1).b : Box{});
    for (size_t m = 0; m < n; ++m)
      for (int side = 0; side < 2; ++side) {
        const SlotRef s = slot_of(static_cast<int32_t>(m), side);
        if (s.code >= 0) box[s.code] = s.b;
      }
    for (size_t mm = n; mm-- > 0;) {
      const int32_t m = static_cast<int32_t>(mm);
      const BuildNode& nd = bin.nodes[m];
      int64_t f = INT64_MAX, c = 0;
      for (int side = 0; side < 2; ++side) {
        if (nd.child[side] == kEmptyChild) continue;
        const SlotRef s = slot_of(m, side);
        if (s.code < 0) {
          f = std::min<int64_t>(f, -(static_cast<int64_t>(s.code) + 1));
          c += s.cnt;
        } else {
          f = std::min(f, first[s.code]);
          c += count[s.code];
        }
      }
      first[m] = f;
      count[m] = c;
      const bool two = nd.child[1] != kEmptyChild;
      const SlotRef l = slot_of(m, 0);
      const SlotRef r = two ? slot_of(m, 1) : SlotRef{};
      double d[W + 1];  // d[j]: the two children sharing j slots
      int dk[W + 1];
      for (int j = 1; j <= W; ++j) {
        d[j] = kInf;
        dk[j] = 0;
        if (!two) {  // a single child: it takes the whole budget
          d[j] = slot_cost(l, j);
          dk[j] = j;
          continue;
        }
        for (int k = 1; k < j; ++k) {
          const double v = slot_cost(l, k) + slot_cost(r, j - k);
          if (v < d[j]) {
            d[j] = v;
            dk[j] = k;
          }
        }
      }
      const double a = half_area(box[m]);
      const double c_leaf = c <= max_leaf ? a * static_cast<double>(c) : kInf;
      const double c_int = a * c_node + d[W];
      double* cm = &cost[static_cast<size_t>(m) * W];
      int8_t* pm = &pick[static_cast<size_t>(m) * W];
      as_leaf[m] = c_leaf <= c_int;
      cm[0] = std::min(c_leaf, c_int);
      pm[0] = 0;
      for (int i = 2; i <= W; ++i) {
        if (d[i] < cm[i - 2]) {
          cm[i - 1] = d[i];
          pm[i - 1] = static_cast<int8_t>(dk[i]);
        } else {
          cm[i - 1] = cm[i - 2];
          pm[i - 1] = -1;
        }
      }
      wide_k[m] = static_cast<int8_t>(dk[W]);  // m as a wide node: its children share W slots so
    }
  }
};

}  // namespace

template <int W>
void collapse_bvh(const Bvh& bin, BvhW<W>* out, const CollapseParams& prm) {
  out->nodes.clear();
  out->depth = 0;
  out->max_pushes = 0;
  if (bin.nodes.empty()) return;
  CollapseDp<W> dp{bin, prm.c_node, prm.max_leaf, {}, {}, {}, {}, {}, {}, {}};
  if (prm.sah) dp.run();
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
    BvhW<W>* out;
    decltype(slot_of)& slot;
    const CollapseDp<W>* dp;  // SAH-optimal collapse, or null: greedy (open the largest-area inner child)
    // up to W slots, no heap (the collapse visits every node of a 1M-primitive tree)
    struct Slots {
      Slot s[W];
      size_t n = 0;
      size_t size() const { return n; }
      Slot& operator[](size_t i) { return s[i]; }
      const Slot& operator[](size_t i) const { return s[i]; }
    };
    // the DP's slots of wide node b: its children sharing W slots as the program chose
    void expand(Slots& out_slots, int32_t node, int side, int budget) const {
      const typename CollapseDp<W>::SlotRef s = dp->slot_of(node, side);
      if (s.code < 0) {  // a leaf of the binary tree stays a leaf
        Slot sl;
        sl.code = s.code;
        sl.count = s.cnt;
        sl.box = s.b;
        out_slots.s[out_slots.n++] = sl;
        return;
      }
      expand_node(out_slots, s.code, budget);
    }
    void expand_node(Slots& out_slots, int32_t m, int budget) const {
      const int8_t* pm = &dp->pick[static_cast<size_t>(m) * W];
      while (budget > 1 && pm[budget - 1] == -1) --budget;
      if (budget == 1) {
        Slot sl;
        sl.box = dp->box[m];
        if (dp->as_leaf[m]) {  // merged leaf: the subtree's contiguous refs
          sl.code = -(1 + static_cast<int32_t>(dp->first[m]));
          sl.count = static_cast<int32_t>(dp->count[m]);
        } else {
          sl.code = m;
          sl.count = 0;
        }
        out_slots.s[out_slots.n++] = sl;
        return;
      }
      const int k = pm[budget - 1];
      if (bin.nodes[m].child[1] == kEmptyChild) {
        expand(out_slots, m, 0, budget);
        return;
      }
      expand(out_slots, m, 0, k);
      expand(out_slots, m, 1, budget - k);
    }
    Slots gather(int32_t b) {
      Slots slots;
      const BuildNode& n = bin.nodes[b];
      if (dp) {  // b is a wide node: its two children share the W slots
        const int k = dp->wide_k[b];
        if (n.child[1] == kEmptyChild) {
          expand(slots, b, 0, W);
        } else {
          expand(slots, b, 0, k);
          expand(slots, b, 1, W - k);
        }
        return slots;
      }
      for (int side = 0; side < 2; ++side)
        if (n.child[side] != kEmptyChild) slots.s[slots.n++] = slot(n, side);
      while (slots.size() < W) {
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
        Slot kids[2];
        size_t nk = 0;
        for (int side = 0; side < 2; ++side)
          if (c.child[side] != kEmptyChild) kids[nk++] = slot(c, side);
        if (nk + slots.size() - 1 > W) break;
        // replace slot `best` by the kids, in place (the order a vector erase + insert gives)
        Slot next[W];
        size_t m = 0;
        for (size_t i = 0; i < slots.size(); ++i) {
          if (static_cast<int>(i) == best) {
            for (size_t k = 0; k < nk; ++k) next[m++] = kids[k];
          } else {
            next[m++] = slots[i];
          }
        }
        for (size_t i = 0; i < m; ++i) slots.s[i] = next[i];
        slots.n = m;
      }
      return slots;
    }
    std::array<int32_t, W> children(const Slots& slots, int depth, int pushes) {
      out->depth = std::max(out->depth, depth);
      const int here = pushes + static_cast<int>(slots.size()) - 1;
      out->max_pushes = std::max(out->max_pushes, here);
      std::array<int32_t, W> codes;
      codes.fill(kEmptyChild);
      // the inner children of a node are allocated next to each other (then filled depth-first),
      // so the siblings a ray visits after the nearest one share its cache lines
      int32_t slot_ids[W];
      std::fill(slot_ids, slot_ids + W, -1);
      for (size_t i = 0; i < slots.size(); ++i)
        if (slots[i].code >= 0) {
          slot_ids[i] = static_cast<int32_t>(out->nodes.size());
          out->nodes.push_back(BuildNodeW<W>{});
        }
      for (size_t i = 0; i < slots.size(); ++i)
        codes[i] = slots[i].code >= 0 ? fill(slot_ids[i], slots[i].code, depth + 1, here) : slots[i].code;
      return codes;
    }
    int32_t fill(int32_t me, int32_t b, int depth, int pushes) {
      const Slots slots = gather(b);
      std::array<int32_t, W> codes = children(slots, depth, pushes);
      BuildNodeW<W>& o = out->nodes[me];
      for (int i = 0; i < W; ++i) {
        o.child[i] = codes[i];
        o.count[i] = i < static_cast<int>(slots.size()) ? slots[i].count : 0;
        for (int k = 0; k < 3; ++k) {
          o.lo[i][k] = i < static_cast<int>(slots.size()) ? slots[i].box.lo[k] : kInf;
          o.hi[i][k] = i < static_cast<int>(slots.size()) ? slots[i].box.hi[k] : -kInf;
        }
      }
      return me;
    }
  } rec{bin, out, slot_of, prm.sah ? &dp : nullptr};
  out->nodes.reserve(bin.nodes.size() / 2 + 2);
  out->nodes.push_back(BuildNodeW<W>{});  // the root is node 0
  rec.fill(0, 0, 1, 0);
}
template void collapse_bvh<4>(const Bvh&, BvhW<4>*, const CollapseParams&);

template <int W>
void reorder_top_bfs(BvhW<W>* t, int64_t top) {
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
    for (int c = 0; c < W && static_cast<int64_t>(order.size()) < top; ++c) {
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
  std::vector<BuildNodeW<W>> out(n);
  for (int32_t k = 0; k < n; ++k) {
    out[k] = t->nodes[order[k]];
    for (int c = 0; c < W; ++c)
      if (out[k].child[c] >= 0) out[k].child[c] = pos[out[k].child[c]];
  }
  t->nodes.swap(out);
}
template void reorder_top_bfs<4>(BvhW<4>*, int64_t);

bool hot_order_nodes(int32_t* rec, int width, const uint32_t* visits, int64_t n, std::vector<int32_t>* order_out) {
  const int64_t words = 7 * width, bytes = 28 * width;  // a node: 6 plane rows + 1 code row of `width`
  std::vector<int32_t>& order = *order_out;
  order.resize(n);
  // every inner code must name a node of the array (the array may come from the device builder): a bad
  // one would index pos[] out of bounds below, so nothing is renumbered
  for (int64_t k = 0; k < n; ++k)
    for (int c = 0; c < width; ++c) {
      const int32_t code = rec[k * words + 6 * width + c];
      if (code >= 0 && (code % bytes != 0 || code / bytes >= n)) return false;
    }
  if (n <= 1) return true;
  for (int64_t k = 0; k < n; ++k) order[k] = static_cast<int32_t>(k);
  // the root stays node 0 (DevScene::root_code); the others by visits, ties in their previous order
  std::stable_sort(order.begin() + 1, order.end(),
                   [&](int32_t a, int32_t b) { return visits[a] > visits[b]; });
  std::vector<int32_t> pos(n);
  for (int64_t k = 0; k < n; ++k) pos[order[k]] = static_cast<int32_t>(k);
  std::vector<int32_t> out(static_cast<size_t>(n) * words);
  for (int64_t k = 0; k < n; ++k) {
    std::memcpy(&out[k * words], &rec[static_cast<int64_t>(order[k]) * words], bytes);
    int32_t* code = &out[k * words + 6 * width];
    for (int c = 0; c < width; ++c)
      if (code[c] >= 0) code[c] = static_cast<int32_t>(pos[code[c] / bytes] * bytes);  // inner: byte offset
  }
  std::memcpy(rec, out.data(), static_cast<size_t>(n) * bytes);
  return true;
}

// ---- bvh_node's leaf order (rtg_bvh_node_order) ----
// The permutation bvh_node(objects, 0, n) applies to `objects` (bvh_node.hpp:25-77): a node of three or
// more objects sorts its range by box min on its box's longest axis and splits it at the median, spans
// of 1 and 2 stay as they are; the final array is the leaves left to right. The sort is libstdc++'s
// std::sort as in the reference, run on (key, id) pairs instead of shared_ptrs: the same comparisons in
// the same sequence, so the same permutation, equal keys included (book-1's root sorts 483 equal y-mins).
// The two halves of a large range are ordered concurrently (disjoint ranges of ids and scratch).
namespace {
struct NodeOrder {
  struct KeyId {
    double key;
    int64_t id;
  };
  const Box* boxes;
  int64_t* ids;
  KeyId* scratch;

  void run(int64_t start, int64_t end, int spawn) {
    const int64_t span = end - start;
    if (span <= 2) return;
    Box b;
    for (int64_t i = start; i < end; ++i) b = box_union(b, boxes[ids[i]]);
    const int axis = longest_axis(b);
    KeyId* kv = scratch + start;
    for (int64_t k = 0; k < span; ++k) kv[k] = KeyId{boxes[ids[start + k]].lo[axis], ids[start + k]};
    std::sort(kv, kv + span, [](const KeyId& x, const KeyId& y) { return x.key < y.key; });
    for (int64_t k = 0; k < span; ++k) ids[start + k] = kv[k].id;
    const int64_t mid = start + span / 2;
    if (spawn > 0 && span >= 32768) {
      std::thread left([this, start, mid, spawn]() { run(start, mid, spawn - 1); });
      run(mid, end, spawn - 1);
      left.join();
    } else {
      run(start, mid, 0);
      run(mid, end, 0);
    }
  }
};
}  // namespace

void bvh_node_order(const double* boxes6, int64_t n, int64_t* order) {
  std::vector<Box> boxes(n);
  for (int64_t i = 0; i < n; ++i)
    for (int a = 0; a < 3; ++a) {
      boxes[i].lo[a] = boxes6[i * 6 + a];
      boxes[i].hi[a] = boxes6[i * 6 + 3 + a];
    }
  for (int64_t i = 0; i < n; ++i) order[i] = i;
  std::vector<NodeOrder::KeyId> scratch(n);
  NodeOrder o{boxes.data(), order, scratch.data()};
  o.run(0, n, 4);  // up to 16 concurrent subtrees (the GPU box's 16-core quota)
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
  // RTG_BUILD_THREADS, else the host's threads (at most 16: the GPU box's cgroup quota)
  int threads = static_cast<int>(std::thread::hardware_concurrency());
  if (const char* e = std::getenv("RTG_BUILD_THREADS")) threads = std::atoi(e);
  threads = std::min(16, std::max(1, threads));
  out->nodes.reserve(n * 2);
  out->refs.reserve(n);
  if (desc->bvh_mode == RTG_BVH_MEDIAN) {
    std::vector<Box> boxes(n);
    for (int64_t i = 0; i < n; ++i) prim_bbox(desc->prims[i], boxes[i].lo, boxes[i].hi);
    std::vector<int64_t> ids(n);
    for (int64_t i = 0; i < n; ++i) ids[i] = i;
    Builder b{boxes, *out, ids};
    b.median(0, n, 1);
    return true;
  }
  if (desc->bvh_mode != RTG_BVH_SAH) {
    *err = "unknown bvh_mode";
    return false;
  }
  std::vector<PrimRec> recs(n);
  par_chunks(0, n, n >= SahBuilder::kParMin ? threads : 1, [&](int64_t a, int64_t e, int) {
    for (int64_t i = a; i < e; ++i) {
      prim_bbox(desc->prims[i], recs[i].lo, recs[i].hi);
      recs[i].id = i;
    }
  });
  SahBuilder b{recs, *out, threads};
  b.parallel = threads > 1;
  // RTG_SAH_TUNE="trav_cost:max_leaf[:axes[:bins]]" overrides the SAH constants (tuning experiments only)
  if (const char* tune = std::getenv("RTG_SAH_TUNE")) {
    double ct = 0.0;
    int ml = 0, ax = 3, nb = 32;
    if (std::sscanf(tune, "%lf:%d:%d:%d", &ct, &ml, &ax, &nb) >= 2 && ct > 0.0 && ml >= 1 && ml <= 8) {
      b.trav_cost = ct;
      b.kMaxLeaf = ml;
      b.axes = ax == 3 ? 3 : 1;
      b.kBins = std::min(std::max(nb, 2), int(SahBuilder::kMaxBins));
    }
  }
  Box all, cb;
  b.range_boxes(0, n, &all, &cb);
  int32_t cnt = 0;
  const int32_t code = b.sah_child(0, n, all, cb, 1, &cnt);
  if (code < 0) {  // the whole scene is one leaf: wrap it into a root node
    const int32_t root = b.new_node();
    out->depth = 1;
    b.set_child(root, 0, code, cnt, all);
  }
  return true;
}

}  // namespace rtg
