// core/camera.hpp — the camera of the reference (camera.hpp:10-245) with the same public fields
// and the same render(std::ostream&, const hittable&) entry point. render() no longer loops over
// pixels on the host: it flattens the world (hittable::rtg_flatten), uploads it once through the
// C-ABI of librtgpu (include/rtgpu.h) and runs the per-pixel sample loop on the MI355X, then
// writes the same P3 PPM. There is no CPU fallback: any device or scene error throws.
#pragma once
#include <algorithm>
#include <cstdio>
#include <exception>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
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
    flatten(world, sb);
    const rtg_scene_desc d = sb.desc(bvh_mode);
    check(rtg_scene_create(&d, device, &scene_), "rtg_scene_create");
  }
  device_scene(const rtg_scene_desc& d, int device) { check(rtg_scene_create(&d, device, &scene_), "rtg_scene_create"); }
  static void flatten(const hittable& world, scene_builder& sb) {
    if (!world.rtg_flatten(sb, vec3(0, 0, 0)))
      throw std::runtime_error("rtgpu: world cannot be flattened for the device: " +
                               (sb.error.empty() ? std::string("unsupported hittable") : sb.error));
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
  // row-interleaved shards on these devices, gathered over RCCL (rtg_render_frame); a device listed
  // twice (tests on a one-GPU box: RCCL takes one rank per device) renders from host threads instead
  std::vector<int> devices;
  int bvh_mode = RTG_BVH_SAH;      // device BVH builder
  rtg_render_stats last_stats{};   // segments, samples, kernel time of the last render

  void render(std::ostream& output_stream, const hittable& world) {
    const std::vector<float> rgb = render_linear(world);
    const int H = image_height();
    output_stream << "P3\n" << image_width << ' ' << H << "\n255\n";
    write_ppm_body(output_stream, rgb);
    std::printf("\rDone.                       \n");
    std::fflush(stdout);
  }

  // The linear, pre-gamma per-pixel mean (what the reference hands to write_color), H*W*3.
  std::vector<float> render_linear(const hittable& world) {
    if (!devices.empty()) {
      std::vector<int> sorted(devices);
      std::sort(sorted.begin(), sorted.end());
      if (std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end()) return render_linear_rccl(world);
      return render_linear_multi(world);
    }
    rtgpu::device_scene scene(world, device, bvh_mode);
    return render_linear(scene);
  }

  // One scene per device, rows r, r+N, ... on device r, one RCCL gather to devices[0] and the
  // de-interleave there (rtg_render_frame), then the frame to the host.
  std::vector<float> render_linear_rccl(const hittable& world) {
    rtgpu::scene_builder sb;
    rtgpu::device_scene::flatten(world, sb);
    const rtg_scene_desc d = sb.desc(bvh_mode);
    const rtg_camera_desc cd = desc();
    const std::vector<int32_t> devs(devices.begin(), devices.end());
    std::vector<std::unique_ptr<rtgpu::device_scene>> scenes;
    std::vector<rtg_scene*> handles;
    for (int32_t dv : devs) {
      scenes.emplace_back(new rtgpu::device_scene(d, dv));
      handles.push_back(scenes.back()->handle());
    }
    rtg_comm* comm = nullptr;
    rtgpu::check(rtg_comm_create_local(devs.data(), static_cast<int32_t>(devs.size()), &comm),
                 "rtg_comm_create_local");
    std::vector<float> rgb(static_cast<size_t>(image_height()) * image_width * 3);
    const rtg_status st = rtg_render_frame(comm, handles.data(), &cd, seed, 0, rgb.data(), &last_stats);
    const std::string err = st == RTG_OK ? std::string() : std::string(rtg_last_error());
    rtg_comm_destroy(comm);
    if (st != RTG_OK)
      throw std::runtime_error("rtgpu: rtg_render_frame failed (" + std::to_string(st) + "): " + err);
    return rgb;
  }

  // write_color (color.hpp:26-58) for every pixel, the text formatted on all host cores and
  // written in order: the same bytes as the reference's per-pixel stream writes.
  static void write_ppm_body(std::ostream& out, const std::vector<float>& rgb) {
    const size_t n = rgb.size() / 3;
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const size_t parts = std::max<size_t>(1, std::min<size_t>(hw, n / 4096));
    std::vector<std::string> text(parts);
    auto work = [&](size_t t) {
      std::string& s = text[t];
      const size_t b = n * t / parts, e = n * (t + 1) / parts;
      s.reserve((e - b) * 12);
      char buf[16];
      for (size_t k = b; k < e; ++k) {
        static const interval intensity(0.000f, 0.999f);
        for (int c = 0; c < 3; ++c) {
          const int v = int(256 * intensity.clamp(linear_to_gamma(rgb[3 * k + c])));
          const int len = std::snprintf(buf, sizeof(buf), c < 2 ? "%d " : "%d\n", v);
          s.append(buf, static_cast<size_t>(len));
        }
      }
    };
    std::vector<std::thread> pool;
    for (size_t t = 1; t < parts; ++t) pool.emplace_back(work, t);
    work(0);
    for (auto& th : pool) th.join();
    for (const std::string& s : text) out.write(s.data(), static_cast<std::streamsize>(s.size()));
  }

  // One host thread per entry of `devices` (used when a device is listed twice): device r renders
  // rows r, r+N, ... into host memory (the RNG is keyed by the global pixel, so the frame is
  // identical to a single-device render).
  std::vector<float> render_linear_multi(const hittable& world) {
    rtgpu::scene_builder sb;
    rtgpu::device_scene::flatten(world, sb);
    const rtg_scene_desc d = sb.desc(bvh_mode);
    const rtg_camera_desc cd = desc();
    const int N = static_cast<int>(devices.size()), H = image_height(), W = image_width;
    std::vector<std::vector<float>> shard(N);
    std::vector<rtg_render_stats> st(N);
    std::vector<std::exception_ptr> errs(N);
    std::vector<std::thread> pool;
    for (int r = 0; r < N; ++r)
      pool.emplace_back([&, r] {
        try {
          rtgpu::device_scene scene(d, devices[r]);
          const int rows = r < H ? (H - 1 - r) / N + 1 : 0;
          shard[r].assign(static_cast<size_t>(rows) * W * 3, 0.0f);
          if (rows == 0) return;
          rtg_render_desc job{};
          job.seed = seed;
          job.row_begin = r;
          job.row_stride = N;
          rtgpu::check(rtg_render(scene.handle(), &cd, &job, shard[r].data(), &st[r]), "rtg_render");
        } catch (...) {
          errs[r] = std::current_exception();
        }
      });
    for (auto& th : pool) th.join();
    for (auto& e : errs)
      if (e) std::rethrow_exception(e);
    std::vector<float> rgb(static_cast<size_t>(H) * W * 3);
    last_stats = rtg_render_stats{};
    for (int r = 0; r < N; ++r) {
      for (size_t k = 0; k * W * 3 < shard[r].size(); ++k)
        std::copy(shard[r].begin() + k * W * 3, shard[r].begin() + (k + 1) * W * 3,
                  rgb.begin() + (static_cast<size_t>(r) + k * N) * W * 3);
      last_stats.segments += st[r].segments;
      last_stats.samples += st[r].samples;
      last_stats.kernel_ms = std::max(last_stats.kernel_ms, st[r].kernel_ms);
    }
    return rgb;
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
