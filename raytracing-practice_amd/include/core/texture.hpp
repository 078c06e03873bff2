// core/texture.hpp — texture interface and the four textures (texture.hpp:11-156), host fp64
// value() plus the rtg_export extension used to flatten them for the device.
#pragma once
#include <memory>

#include "common/rtweekend.hpp"
#include "core/perlin.hpp"
#include "core/rtw_stb_image.hpp"
#include "rtgpu/scene_builder.hpp"

class texture {
 public:
  virtual ~texture() = default;
  virtual color value(double u, double v, const point3& p) const = 0;
  // Appends this texture (and its children) to the flat scene; returns its index or -1.
  virtual int32_t rtg_export(rtgpu::scene_builder& sb) const { return -1; }
};

class solid_color : public texture {
 public:
  solid_color(const color& albedo) : albedo(albedo) {}
  solid_color(double red, double green, double blue) : solid_color(color(red, green, blue)) {}
  color value(double, double, const point3&) const override { return albedo; }
  int32_t rtg_export(rtgpu::scene_builder& sb) const override {
    rtg_texture t{};
    t.type = RTG_TEX_SOLID;
    for (int k = 0; k < 3; ++k) t.color[k] = albedo[k];
    sb.textures.push_back(t);
    return static_cast<int32_t>(sb.textures.size() - 1);
  }

 private:
  color albedo;
};

// 3-D checker on the world position: parity of floor(p / scale) summed over the axes.
class checker_texture : public texture {
 public:
  checker_texture(double scale, std::shared_ptr<texture> even, std::shared_ptr<texture> odd)
      : scale(scale), inv_scale(1.0f / scale), even(even), odd(odd) {}
  checker_texture(double scale, const color& c1, const color& c2)
      : checker_texture(scale, std::make_shared<solid_color>(c1), std::make_shared<solid_color>(c2)) {}

  color value(double u, double v, const point3& p) const override {
    const int xi = int(std::floor(inv_scale * p.x()));
    const int yi = int(std::floor(inv_scale * p.y()));
    const int zi = int(std::floor(inv_scale * p.z()));
    const bool is_even = (xi + yi + zi) % 2 == 0;  // C remainder: negative odd sums are odd (H13)
    return is_even ? even->value(u, v, p) : odd->value(u, v, p);
  }
  int32_t rtg_export(rtgpu::scene_builder& sb) const override {
    const int32_t e = sb.texture_id(even.get());
    const int32_t o = sb.texture_id(odd.get());
    if (e < 0 || o < 0) return -1;
    rtg_texture t{};
    t.type = RTG_TEX_CHECKER;
    t.even = e;
    t.odd = o;
    t.scale = scale;
    sb.textures.push_back(t);
    return static_cast<int32_t>(sb.textures.size() - 1);
  }

 private:
  double scale, inv_scale;
  std::shared_ptr<texture> even, odd;
};

class image_texture : public texture {
 public:
  image_texture(const char* filename) : image(filename) {}
  color value(double u, double v, const point3&) const override {
    if (image.height() <= 0) return color(0.0f, 1.0f, 1.0f);  // cyan: image missing
    u = interval(0.0f, 1.0f).clamp(u);
    v = 1.0f - interval(0.0f, 1.0f).clamp(v);  // image rows run top to bottom
    const auto* px = image.pixel_data(int(u * image.width()), int(v * image.height()));
    const auto s = 1.0f / 255.0f;
    return color(s * px[0], s * px[1], s * px[2]);
  }
  int32_t rtg_export(rtgpu::scene_builder& sb) const override {
    rtg_texture t{};
    t.type = RTG_TEX_IMAGE;
    t.image = sb.image_id(&image, image.width(), image.height(), image.bytes());
    sb.textures.push_back(t);
    return static_cast<int32_t>(sb.textures.size() - 1);
  }

 private:
  rtw_image image;
};

// Marble: 0.5 * (1 + sin(scale * z + 10 * turbulence(p))).
class noise_texture : public texture {
 public:
  noise_texture(double scale) : scale(scale) {}
  color value(double, double, const point3& p) const override {
    return color(0.5f, 0.5f, 0.5f) * (1.0f + std::sin(scale * p.z() + 10.0f * noise.turb(p, 7)));
  }
  int32_t rtg_export(rtgpu::scene_builder& sb) const override {
    rtg_texture t{};
    t.type = RTG_TEX_NOISE;
    t.perlin = sb.perlin_id(&noise, noise.tables());
    t.scale = scale;
    sb.textures.push_back(t);
    return static_cast<int32_t>(sb.textures.size() - 1);
  }

 private:
  perlin noise;
  double scale;
};

inline int32_t rtgpu::scene_builder::texture_id(const texture* t) {
  if (!t) {
    fail("null texture");
    return -1;
  }
  auto& memo = memo_table(kTexture);
  auto it = memo.find(t);
  if (it != memo.end()) return it->second;
  const int32_t id = t->rtg_export(*this);
  if (id < 0) {
    fail("texture type without a device export");
    return -1;
  }
  memo[t] = id;
  return id;
}
