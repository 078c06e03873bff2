// hittable/hittable_list.hpp — linear closest-hit list (hittable_list.hpp:21-76).
#pragma once
#include <vector>

#include "hittable/hittable.hpp"
#include "rtgpu/scene_builder.hpp"

class hittable_list : public hittable {
 public:
  std::vector<std::shared_ptr<hittable>> objects;

  hittable_list() {}
  hittable_list(std::shared_ptr<hittable> object) { add(object); }

  void clear() { objects.clear(); }
  void add(std::shared_ptr<hittable> object) {
    objects.push_back(object);
    bbox = aabb(bbox, object->bounding_box());
  }

  bool hit(const ray& r, interval ray_t, hit_record& rec) const override {
    hit_record candidate;
    bool any = false;
    double closest = ray_t.max;
    for (const auto& obj : objects) {
      if (obj->hit(r, interval(ray_t.min, closest), candidate)) {
        any = true;
        closest = candidate.t;
        rec = candidate;
      }
    }
    return any;
  }
  aabb bounding_box() const override { return bbox; }
  bool rtg_flatten(rtgpu::scene_builder& sb, const vec3& offset) const override {
    sb.reserve(objects.size());
    for (const auto& obj : objects)
      if (!obj->rtg_flatten(sb, offset)) return false;
    return true;
  }

 private:
  aabb bbox;
};
