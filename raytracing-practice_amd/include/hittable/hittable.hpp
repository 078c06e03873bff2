// hittable/hittable.hpp — hit_record, the hittable interface and translate (hittable.hpp:13-117).
//
// Extension over the reference: hittable::rtg_flatten appends the object's primitives to a flat
// device scene (rtgpu/scene_builder.hpp). camera::render renders a world only through that path;
// a user-defined hittable that does not override it makes render() fail loudly.
#pragma once
#include <memory>

#include "accelerator/aabb.hpp"
#include "common/rtweekend.hpp"

class material;
namespace rtgpu {
class scene_builder;
}

class hit_record {
 public:
  point3 p;
  vec3 normal;
  std::shared_ptr<material> mat;
  double t = 0, u = 0, v = 0;
  bool front_face = false;

  // outward_normal must be unit length; the stored normal faces against the ray.
  void set_face_normal(const ray& r, const vec3& outward_normal) {
    front_face = dot(r.direction(), outward_normal) < 0;
    normal = front_face ? outward_normal : -outward_normal;
  }
};

class hittable {
 public:
  virtual ~hittable() = default;
  virtual bool hit(const ray& r, interval ray_t, hit_record& rec) const = 0;
  virtual aabb bounding_box() const = 0;
  // Appends this object's primitives (moved by `offset`) to the flat scene; false = unsupported.
  virtual bool rtg_flatten(rtgpu::scene_builder& sb, const vec3& offset) const { return false; }
};

// Moves an object by a fixed offset (hittable.hpp:74-117).
class translate : public hittable {
 public:
  translate(std::shared_ptr<hittable> object, const vec3& offset)
      : object(object), offset(offset), bbox(object->bounding_box() + offset) {}

  bool hit(const ray& r, interval ray_t, hit_record& rec) const override {
    const ray moved(r.origin() - offset, r.direction(), r.time());
    if (!object->hit(moved, ray_t, rec)) return false;
    rec.p += offset;
    return true;
  }
  aabb bounding_box() const override { return bbox; }
  bool rtg_flatten(rtgpu::scene_builder& sb, const vec3& off) const override {
    return object->rtg_flatten(sb, off + offset);
  }

 private:
  std::shared_ptr<hittable> object;
  vec3 offset;
  aabb bbox;
};
