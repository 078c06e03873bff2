// core/material.hpp — material interface and the four materials (material.hpp:21-240), host
// fp64 scatter()/emitted() drawing from rand() like the reference, plus the rtg_export extension.
#pragma once
#include <memory>

#include "common/rtweekend.hpp"
#include "core/texture.hpp"
#include "hittable/hittable.hpp"
#include "rtgpu/scene_builder.hpp"

class material {
 public:
  virtual ~material() = default;
  virtual color emitted(double u, double v, const point3& p) const { return color(0.0f, 0.0f, 0.0f); }
  virtual bool scatter(const ray& r_in, const hit_record& rec, color& attenuation, ray& scattered) const {
    return false;
  }
  virtual int32_t rtg_export(rtgpu::scene_builder& sb) const { return -1; }
};

// Diffuse: scatter along normal + random unit vector (cosine-weighted).
class lambertian : public material {
 public:
  lambertian(const color& albedo) : tex(std::make_shared<solid_color>(albedo)) {}
  lambertian(std::shared_ptr<texture> tex) : tex(tex) {}

  bool scatter(const ray& r_in, const hit_record& rec, color& attenuation, ray& scattered) const override {
    vec3 dir = rec.normal + random_unit_vector();
    if (dir.near_zero()) dir = rec.normal;
    scattered = ray(rec.p, dir, r_in.time());
    attenuation = tex->value(rec.u, rec.v, rec.p);
    return true;
  }
  int32_t rtg_export(rtgpu::scene_builder& sb) const override {
    rtg_material m{};
    m.type = RTG_MAT_LAMBERTIAN;
    m.texture = sb.texture_id(tex.get());
    if (m.texture < 0) return -1;
    sb.materials.push_back(m);
    return static_cast<int32_t>(sb.materials.size() - 1);
  }

 private:
  std::shared_ptr<texture> tex;
};

// Mirror reflection perturbed by fuzz * random unit vector; absorbed below the surface.
class metal : public material {
 public:
  metal(const color& albedo, double fuzz) : albedo(albedo), fuzz(fuzz < 1.0f ? fuzz : 1.0f) {}

  bool scatter(const ray& r_in, const hit_record& rec, color& attenuation, ray& scattered) const override {
    vec3 reflected = reflect(r_in.direction(), rec.normal);
    reflected = unit_vector(reflected) + (fuzz * random_unit_vector());
    scattered = ray(rec.p, reflected, r_in.time());
    attenuation = albedo;
    return dot(scattered.direction(), rec.normal) > 0;
  }
  int32_t rtg_export(rtgpu::scene_builder& sb) const override {
    rtg_material m{};
    m.type = RTG_MAT_METAL;
    m.texture = -1;
    for (int k = 0; k < 3; ++k) m.albedo[k] = albedo[k];
    m.fuzz = fuzz;
    sb.materials.push_back(m);
    return static_cast<int32_t>(sb.materials.size() - 1);
  }

 private:
  color albedo;
  double fuzz;
};

// Glass: refract by Snell's law, reflect on total internal reflection or by Schlick's chance.
class dielectric : public material {
 public:
  dielectric(double refraction_index) : refraction_index(refraction_index) {}

  bool scatter(const ray& r_in, const hit_record& rec, color& attenuation, ray& scattered) const override {
    attenuation = color(1.0f, 1.0f, 1.0f);
    const double ri = rec.front_face ? (1.0f / refraction_index) : refraction_index;
    const vec3 ud = unit_vector(r_in.direction());
    const double cos_theta = std::fmin(dot(-ud, rec.normal), 1.0f);
    const double sin_theta = std::sqrt(1.0f - cos_theta * cos_theta);
    const bool cannot_refract = ri * sin_theta > 1.0f;
    const vec3 dir = (cannot_refract || reflectance(cos_theta, ri) > random_double())
                         ? reflect(ud, rec.normal)
                         : refract(ud, rec.normal, ri);
    scattered = ray(rec.p, dir, r_in.time());
    return true;
  }
  int32_t rtg_export(rtgpu::scene_builder& sb) const override {
    rtg_material m{};
    m.type = RTG_MAT_DIELECTRIC;
    m.texture = -1;
    m.refraction_index = refraction_index;
    sb.materials.push_back(m);
    return static_cast<int32_t>(sb.materials.size() - 1);
  }

 private:
  double refraction_index;
  static double reflectance(double cosine, double ri) {  // Schlick
    double r0 = (1.0f - ri) / (1.0f + ri);
    r0 = r0 * r0;
    return r0 + (1.0f - r0) * std::pow((1.0f - cosine), 5);
  }
};

class diffuse_light : public material {
 public:
  diffuse_light(std::shared_ptr<texture> tex) : tex(tex) {}
  diffuse_light(const color& emit) : tex(std::make_shared<solid_color>(emit)) {}
  color emitted(double u, double v, const point3& p) const override { return tex->value(u, v, p); }
  int32_t rtg_export(rtgpu::scene_builder& sb) const override {
    rtg_material m{};
    m.type = RTG_MAT_DIFFUSE_LIGHT;
    m.texture = sb.texture_id(tex.get());
    if (m.texture < 0) return -1;
    sb.materials.push_back(m);
    return static_cast<int32_t>(sb.materials.size() - 1);
  }

 private:
  std::shared_ptr<texture> tex;
};

inline int32_t rtgpu::scene_builder::material_id(const material* m) {
  if (!m) {
    fail("primitive without a material");
    return -1;
  }
  auto& memo = memo_table(kMaterial);
  auto it = memo.find(m);
  if (it != memo.end()) return it->second;
  const int32_t id = m->rtg_export(*this);
  if (id < 0) {
    fail("material type without a device export");
    return -1;
  }
  memo[m] = id;
  return id;
}
