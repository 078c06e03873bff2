// hittable/quad.hpp — parallelogram Q + a*u + b*v and the six-sided box() (quad.hpp:8-159).
#pragma once
#include "hittable/hittable.hpp"
#include "hittable/hittable_list.hpp"
#include "rtgpu/scene_builder.hpp"

class quad : public hittable {
 public:
  quad(const point3& Q, const vec3& u, const vec3& v, std::shared_ptr<material> mat)
      : Q(Q), u(u), v(v), mat(mat) {
    const vec3 n = cross(u, v);
    normal = unit_vector(n);
    D = dot(normal, Q);
    w = n / dot(n, n);
    set_bounding_box();
  }

  virtual void set_bounding_box() { bbox = aabb(aabb(Q, Q + u + v), aabb(Q + u, Q + v)); }
  aabb bounding_box() const override { return bbox; }

  bool hit(const ray& r, interval ray_t, hit_record& rec) const override {
    const double denom = dot(normal, r.direction());
    if (std::fabs(denom) < 1e-8) return false;  // parallel to the plane
    const double t = (D - dot(normal, r.origin())) / denom;
    if (!ray_t.contains(t)) return false;
    const point3 at = r.at(t);
    const vec3 planar = at - Q;
    const double alpha = dot(w, cross(planar, v));
    const double beta = dot(w, cross(u, planar));
    if (!is_interior(alpha, beta, rec)) return false;
    rec.t = t;
    rec.p = at;
    rec.mat = mat;
    rec.set_face_normal(r, normal);
    return true;
  }

  virtual bool is_interior(double a, double b, hit_record& rec) const {
    const interval unit(0.0f, 1.0f);
    if (!unit.contains(a) || !unit.contains(b)) return false;
    rec.u = a;
    rec.v = b;
    return true;
  }

  bool rtg_flatten(rtgpu::scene_builder& sb, const vec3& offset) const override {
    rtg_primitive p{};
    p.kind = RTG_PRIM_QUAD;
    p.material = sb.material_id(mat.get());
    if (p.material < 0) return false;
    const point3 q = Q + offset;
    for (int k = 0; k < 3; ++k) {
      p.p0[k] = q[k];
      p.p1[k] = u[k];
      p.p2[k] = v[k];
    }
    sb.prims.push_back(p);
    return true;
  }

 private:
  point3 Q;
  vec3 u, v, w;
  std::shared_ptr<material> mat;
  aabb bbox;
  vec3 normal;
  double D;
};

// The six faces of the box spanned by opposite corners a and b.
inline std::shared_ptr<hittable_list> box(const point3& a, const point3& b, std::shared_ptr<material> mat) {
  auto sides = std::make_shared<hittable_list>();
  const point3 lo(std::fmin(a.x(), b.x()), std::fmin(a.y(), b.y()), std::fmin(a.z(), b.z()));
  const point3 hi(std::fmax(a.x(), b.x()), std::fmax(a.y(), b.y()), std::fmax(a.z(), b.z()));
  const vec3 dx(hi.x() - lo.x(), 0.0f, 0.0f), dy(0.0f, hi.y() - lo.y(), 0.0f), dz(0.0f, 0.0f, hi.z() - lo.z());
  sides->add(std::make_shared<quad>(point3(lo.x(), lo.y(), hi.z()), dx, dy, mat));   // front
  sides->add(std::make_shared<quad>(point3(hi.x(), lo.y(), hi.z()), -dz, dy, mat));  // right
  sides->add(std::make_shared<quad>(point3(hi.x(), lo.y(), lo.z()), -dx, dy, mat));  // back
  sides->add(std::make_shared<quad>(point3(lo.x(), lo.y(), lo.z()), dz, dy, mat));   // left
  sides->add(std::make_shared<quad>(point3(lo.x(), hi.y(), hi.z()), dx, -dz, mat));  // top
  sides->add(std::make_shared<quad>(point3(lo.x(), lo.y(), lo.z()), dx, dz, mat));   // bottom
  return sides;
}
