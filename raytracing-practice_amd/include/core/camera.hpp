// core/camera.hpp — the camera of the reference (camera.hpp:10-245) with the same public fields
// and the same render(std::ostream&, const hittable&) entry point. render() no longer loops over
// pixels on the host: it flattens the world (hittable::rtg_flatten), uploads it once through the
// C-ABI of librtgpu (include/rtgpu.h) and runs the per-pixel sample loop on the MI355X, then
// writes the same P3 PPM. There is no CPU fallback: any device or scene error throws.
#pragma once
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "core/material.hpp"
#include "hittable/hittable.hpp"
#include "rtgpu.h"
#include "rtgpu/scene_builder.hpp"

namespace rtgpu {

inline void check(rtg_status st, const char* what) {
  if (st != RTG_OK)
    throw std::runtime_error(std::string("rtgpu: ") + what + " failed (" + std::to_string(st) +
                             "): " + rtg_last_error());
}

// A world flattened and uploaded once; render it as often as needed.
class device_scene {
 public:
  device_scene(const hittable& world, int device = 0, int bvh_mode = RTG_BVH_SAH) {
    scene_builder sb;
    if (!world.rtg_flatten(sb, vec3(0, 0, 0)))
      throw std::runtime_error("rtgpu: world cannot be flattened for the device: " +
                               (sb.error.empty() ? std::string("unsupported hittable") : sb.error));
    const rtg_scene_desc d = sb.desc(bvh_mode);
    check(rtg_scene_create(&d, device, &scene_), "rtg_scene_create");
  }
  ~device_scene() { rtg_scene_destroy(scene_); }
  device_scene(const device_scene&) = delete;
  device_scene& operator=(const device_scene&) = delete;
  rtg_scene* handle() const { return scene_; }

 private:
  rtg_scene* scene_ = nullptr;
};

}  // namespace rtgpu

class camera {
 public:
  double aspect_ratio = 1.0f;  // width / height
  int image_width = 100;
  int samples_per_pixel = 10;
  int max_depth = 10;  // ray segments per sample
  color background;

  double vfov = 90.0f;  // vertical field of view, degrees
  point3 lookfrom = point3(0.0f, 0.0f, 0.0f);
  point3 lookat = point3(0.0f, 0.0f, -1.0f);
  vec3 vup = vec3(0.0f, 1.0f, 0.0f);

  double defocus_angle = 0.0f;  // lens cone angle, degrees (0 = pinhole)
  double focus_dist = 10.0f;

  // ---- extensions (not in the reference) ----
  uint64_t seed = 0x5EED;          // counter-RNG run seed
  int device = 0;                  // HIP device to render on
  int bvh_mode = RTG_BVH_SAH;      // device BVH builder
  rtg_render_stats last_stats{};   // segments, samples, kernel time of the last render

  void render(std::ostream& output_stream, const hittable& world) {
    const std::vector<float> rgb = render_linear(world);
    const int H = image_height();
    output_stream << "P3\n" << image_width << ' ' << H << "\n255\n";
    for (size_t k = 0; k + 2 < rgb.size(); k += 3) write_color(output_stream, color(rgb[k], rgb[k + 1], rgb[k + 2]));
    std::printf("\rDone.                       \n");
    std::fflush(stdout);
  }

  // The linear, pre-gamma per-pixel mean (what the reference hands to write_color), H*W*3.
  std::vector<float> render_linear(const hittable& world) {
    rtgpu::device_scene scene(world, device, bvh_mode);
    return render_linear(scene);
  }
  std::vector<float> render_linear(const rtgpu::device_scene& scene) {
    const rtg_camera_desc cd = desc();
    std::vector<float> rgb(static_cast<size_t>(image_height()) * image_width * 3);
    rtg_render_desc job{};
    job.seed = seed;
    job.row_begin = 0;
    job.row_stride = 1;
    job.row_count = 0;
    rtgpu::check(rtg_render(scene.handle(), &cd, &job, rgb.data(), &last_stats), "rtg_render");
    return rgb;
  }

  int image_height() const {
    const int h = static_cast<int>(image_width / aspect_ratio);
    return h < 1 ? 1 : h;
  }

  rtg_camera_desc desc() const {
    rtg_camera_desc c{};
    c.aspect_ratio = aspect_ratio;
    c.image_width = image_width;
    c.samples_per_pixel = samples_per_pixel;
    c.max_depth = max_depth;
    c.vfov = vfov;
    c.defocus_angle = defocus_angle;
    c.focus_dist = focus_dist;
    for (int k = 0; k < 3; ++k) {
      c.background[k] = background[k];
      c.lookfrom[k] = lookfrom[k];
      c.lookat[k] = lookat[k];
      c.vup[k] = vup[k];
    }
    return c;
  }
};
