// accelerator/bvh_node.hpp — host BVH node with the reference's topology (bvh_node.hpp:16-134):
// longest axis of the range box, std::sort by bbox.min on that axis, split at the median.
// On the device the library builds its own BVH over the flattened primitives (RTG_BVH_MEDIAN
// reproduces this topology, RTG_BVH_SAH is the fast default); flattening a bvh_node therefore
// emits the objects in the order of the list it was built from (the root keeps that order), so
// the flat scene lists objects exactly as the reference's hittable_list did, and records the order
// the reference's bvh_node::hit tests them in — its leaves left to right (rtg_bvh_node_order) — as
// the primitives' tie ranks (rtg_scene_desc.tie_rank): at an exactly equal t the reference keeps the
// first sphere and the last quad of THAT order (bvh_node.hpp:89-90, sphere.hpp:70, quad.hpp:62).
#pragma once
#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "accelerator/aabb.hpp"
#include "hittable/hittable.hpp"
#include "hittable/hittable_list.hpp"

class bvh_node : public hittable {
 public:
  // The root over a whole list (main.cpp:76). The reference builds the tree here; the mirror keeps
  // the list in insertion order, computes the root box (a union: order-independent, the same box) and
  // builds the host-side children only on the first host hit(): a render flattens the list and the
  // device builds its own BVH, so it never needs them, and config 5's 1M-sphere scene no longer pays
  // the reference's median build (4.2 s) before every upload.
  bvh_node(hittable_list list) : list_order(std::move(list.objects)) {
    bbox = aabb::empty;
    for (const auto& o : list_order) bbox = aabb(bbox, o->bounding_box());
  }

  // bvh_node.hpp:25-77 as the reference has it (sorts `objects` in place, builds eagerly)
  bvh_node(std::vector<std::shared_ptr<hittable>>& objects, size_t start, size_t end) {
    build(objects, start, end);
    built_ = true;
  }

 private:
  void ensure_built() const {
    std::call_once(once_, [this]() {
      if (built_) return;
      std::vector<std::shared_ptr<hittable>> objects(list_order);
      // the root's box was set in the constructor (the same union): not rewritten here, where other
      // threads may already read it through bounding_box()
      const_cast<bvh_node*>(this)->build(objects, 0, objects.size(), false);
      built_ = true;
    });
  }

  void build(std::vector<std::shared_ptr<hittable>>& objects, size_t start, size_t end, bool set_box = true) {
    if (start >= end) return;  // an empty list: no children, every ray misses the empty box
    aabb box = aabb::empty;
    for (size_t i = start; i < end; ++i) box = aabb(box, objects[i]->bounding_box());
    if (set_box) bbox = box;
    const int axis = box.longest_axis();
    const size_t span = end - start;
    if (span == 1) {
      left = right = objects[start];
    } else if (span == 2) {
      left = objects[start];
      right = objects[start + 1];
    } else {
      std::sort(objects.begin() + start, objects.begin() + end,
                [axis](const std::shared_ptr<hittable>& a, const std::shared_ptr<hittable>& b) {
                  return a->bounding_box().axis_interval(axis).min < b->bounding_box().axis_interval(axis).min;
                });
      const size_t mid = start + span / 2;
      left = std::make_shared<bvh_node>(objects, start, mid);
      right = std::make_shared<bvh_node>(objects, mid, end);
    }
  }

 public:
  bool hit(const ray& r, interval ray_t, hit_record& rec) const override {
    if (!built_) ensure_built();
    if (!left || !bbox.hit(r, ray_t)) return false;
    const bool hl = left->hit(r, ray_t, rec);
    const bool hr = right->hit(r, interval(ray_t.min, hl ? rec.t : ray_t.max), rec);
    return hl || hr;
  }
  aabb bounding_box() const override { return bbox; }

  bool rtg_flatten(rtgpu::scene_builder& sb, const vec3& offset) const override {
    if (!list_order.empty()) {
      const size_t n = list_order.size();
      sb.reserve(n);
      std::vector<size_t> first(n + 1);  // child k's primitives: [first[k], first[k + 1])
      std::vector<double> boxes(6 * n);  // child k's bounding_box(), the key the reference sorts by
      for (size_t k = 0; k < n; ++k) {
        first[k] = sb.prims.size();
        if (!list_order[k]->rtg_flatten(sb, offset)) return false;
        const aabb b = list_order[k]->bounding_box();
        for (int a = 0; a < 3; ++a) {
          boxes[6 * k + a] = b.axis_interval(a).min;
          boxes[6 * k + 3 + a] = b.axis_interval(a).max;
        }
      }
      first[n] = sb.prims.size();
      std::vector<int64_t> order(n);
      if (rtg_bvh_node_order(boxes.data(), static_cast<int64_t>(n), order.data()) != RTG_OK)
        return sb.fail(std::string("rtg_bvh_node_order: ") + rtg_last_error());
      bool identity = true;
      for (size_t k = 0; k < n && identity; ++k) identity = order[k] == static_cast<int64_t>(k);
      if (identity) return true;
      // the range's ranks: the children in leaf order, each child keeping its own primitives' order
      // (child k's ranks are a permutation of [first[k], first[k + 1]), identity unless it reordered them)
      sb.extend_ranks(first[n]);
      const std::vector<int64_t> own(sb.tie_rank.begin() + first[0], sb.tie_rank.begin() + first[n]);
      int64_t base = static_cast<int64_t>(first[0]);
      for (size_t pos = 0; pos < n; ++pos) {
        const size_t c = static_cast<size_t>(order[pos]);
        for (size_t i = first[c]; i < first[c + 1]; ++i)
          sb.tie_rank[i] = base + (own[i - first[0]] - static_cast<int64_t>(first[c]));
        base += static_cast<int64_t>(first[c + 1] - first[c]);
      }
      return true;
    }
    if (!left) return true;  // built over an empty list: nothing to flatten
    if (!left->rtg_flatten(sb, offset)) return false;
    return right == left || right->rtg_flatten(sb, offset);
  }

 private:
  std::vector<std::shared_ptr<hittable>> list_order;
  std::shared_ptr<hittable> left, right;
  aabb bbox;
  mutable std::once_flag once_;
  mutable std::atomic<bool> built_{false};
};
