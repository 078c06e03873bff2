// hittable/sphere.hpp — static and moving spheres (sphere.hpp:7-119), host fp64 hit().
#pragma once
#include "hittable/hittable.hpp"
#include "rtgpu/scene_builder.hpp"

class sphere : public hittable {
 public:
  sphere(point3 static_center, double radius, std::shared_ptr<material> mat)
      : center(static_center, vec3(0.0f, 0.0f, 0.0f)), radius(radius), mat(mat) {
    const vec3 rvec(radius, radius, radius);
    bbox = aabb(static_center - rvec, static_center + rvec);
  }
  sphere(point3 center1, point3 center2, double radius, std::shared_ptr<material> mat)
      : center(center1, center2 - center1), radius(radius), mat(mat), moving(true) {
    const vec3 rvec(radius, radius, radius);
    const aabb b0(center.at(0.0f) - rvec, center.at(0.0f) + rvec);
    const aabb b1(center.at(1.0f) - rvec, center.at(1.0f) + rvec);
    bbox = aabb(b0, b1);
  }

  bool hit(const ray& r, interval ray_t, hit_record& rec) const override {
    const point3 c = center.at(r.time());
    const vec3 oc = r.origin() - c;
    const double a = r.direction().length_squared();
    const double half_b = dot(oc, r.direction());
    const double cc = oc.length_squared() - radius * radius;
    const double disc = half_b * half_b - a * cc;
    if (disc < 0) return false;
    const double sq = std::sqrt(disc);
    double root = (-half_b - sq) / a;  // nearer root first
    if (!ray_t.surrounds(root)) {
      root = (-half_b + sq) / a;
      if (!ray_t.surrounds(root)) return false;
    }
    rec.t = root;
    rec.p = r.at(root);
    const vec3 outward = (rec.p - c) / radius;
    rec.set_face_normal(r, outward);
    get_sphere_uv(outward, rec.u, rec.v);
    rec.mat = mat;
    return true;
  }
  aabb bounding_box() const override { return bbox; }

  bool rtg_flatten(rtgpu::scene_builder& sb, const vec3& offset) const override {
    rtg_primitive p{};
    p.kind = RTG_PRIM_SPHERE;
    p.material = sb.material_id(mat.get());
    if (p.material < 0) return false;
    const point3 c0 = center.origin() + offset;
    const point3 c1 = moving ? c0 + center.direction() : c0;
    for (int k = 0; k < 3; ++k) {
      p.p0[k] = c0[k];
      p.p1[k] = c1[k];
    }
    p.radius = radius;
    sb.prims.push_back(p);
    return true;
  }

 private:
  // p: point on the unit sphere at the origin; u from atan2 around Y, v from acos along -Y.
  static void get_sphere_uv(const point3& p, double& u, double& v) {
    const double theta = std::acos(-p.y());
    const double phi = std::atan2(-p.z(), p.x()) + pi;
    u = phi / (2.0f * pi);
    v = theta / pi;
  }

  ray center;  // origin = centre at time 0, direction = displacement over [0, 1]
  double radius;
  std::shared_ptr<material> mat;
  bool moving = false;
  aabb bbox;
};
