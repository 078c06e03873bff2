// scenes/scenes.hpp — the reference's seven scenes (main.cpp:12-346) plus the earth + Perlin
// composition of benchmark config 3, written against the C++ API mirror. Each builder returns the
// world and a camera configured as in the reference. Random draws in bouncing_spheres are
// explicitly sequenced in the order GCC evaluates main.cpp (hazard H2), so the scene is the
// reference's on every compiler.
#pragma once
#include <functional>
#include <map>
#include <string>

#include "accelerator/bvh_node.hpp"
#include "common/rtweekend.hpp"
#include "core/camera.hpp"
#include "core/material.hpp"
#include "core/texture.hpp"
#include "hittable/hittable.hpp"
#include "hittable/hittable_list.hpp"
#include "hittable/quad.hpp"
#include "hittable/sphere.hpp"

namespace scenes {

struct scene {
  std::shared_ptr<hittable> world;
  camera cam;
};

inline void sky_camera(camera& c, double vfov, point3 from, point3 at, color bg) {
  c.background = bg;
  c.vfov = vfov;
  c.lookfrom = from;
  c.lookat = at;
  c.vup = vec3(0.0f, 1.0f, 0.0f);
  c.defocus_angle = 0.0f;
}

// main.cpp:12-101 (grid = 11); grid = 500 gives the 1,000,001-object scene of config 5.
inline scene bouncing_spheres(int grid = 11) {
  hittable_list world;
  auto checker = std::make_shared<checker_texture>(0.32f, color(0.2f, 0.3f, 0.1f), color(0.9f, 0.9f, 0.9f));
  world.add(std::make_shared<sphere>(point3(0.0f, -1000.0f, -1.0f), 1000.0f, std::make_shared<lambertian>(checker)));
  for (int a = -grid; a < grid; a++) {
    for (int b = -grid; b < grid; b++) {
      const double choose_mat = random_double();
      const double rz = random_double();  // GCC evaluates the z argument first
      const double rx = random_double();
      const point3 center(a + 0.9f * rx, 0.2f, b + 0.9f * rz);
      if ((center - point3(4.0f, 0.2f, 0.0f)).length() <= 0.9f) continue;
      if (choose_mat < 0.8f) {
        const color second = color::random();  // right operand of '*' first (GCC)
        const color first = color::random();
        auto mat = std::make_shared<lambertian>(first * second);
        const point3 center2 = center + vec3(0.0f, random_double(0.0f, 0.5f), 0.0f);
        world.add(std::make_shared<sphere>(center, center2, 0.2f, mat));
      } else if (choose_mat < 0.95f) {
        const color albedo = color::random(0.5f, 1.0f);
        const double fuzz = random_double(0.0f, 0.5f);
        world.add(std::make_shared<sphere>(center, 0.2f, std::make_shared<metal>(albedo, fuzz)));
      } else {
        world.add(std::make_shared<sphere>(center, 0.2f, std::make_shared<dielectric>(1.5f)));
      }
    }
  }
  world.add(std::make_shared<sphere>(point3(0.0f, 1.0f, 0.0f), 1.0f, std::make_shared<dielectric>(1.5f)));
  world.add(std::make_shared<sphere>(point3(-4.0f, 1.0f, 0.0f), 1.0f, std::make_shared<lambertian>(color(0.4f, 0.2f, 0.1f))));
  world.add(std::make_shared<sphere>(point3(4.0f, 1.0f, 0.0f), 1.0f, std::make_shared<metal>(color(0.7f, 0.6f, 0.5f), 0.0f)));
  scene s;
  s.world = std::make_shared<hittable_list>(std::make_shared<bvh_node>(world));
  s.cam.image_width = 400;
  s.cam.aspect_ratio = 16.0f / 9.0f;
  s.cam.samples_per_pixel = 50;
  s.cam.max_depth = 20;
  sky_camera(s.cam, 20.0f, point3(13.0f, 2.0f, 3.0f), point3(0.0f, 0.0f, 0.0f), color(0.7f, 0.8f, 1.0f));
  s.cam.defocus_angle = 0.6f;
  s.cam.focus_dist = 10.0f;
  return s;
}

inline scene checkered_spheres() {  // main.cpp:104-138
  auto world = std::make_shared<hittable_list>();
  auto checker = std::make_shared<checker_texture>(0.32f, color(0.2f, 0.3f, 0.1f), color(0.9f, 0.9f, 0.9f));
  world->add(std::make_shared<sphere>(point3(0.0f, -10.0f, 0.0f), 10.0f, std::make_shared<lambertian>(checker)));
  world->add(std::make_shared<sphere>(point3(0.0f, 10.0f, 0.0f), 10.0f, std::make_shared<lambertian>(checker)));
  scene s{world, camera()};
  s.cam.image_width = 400;
  s.cam.aspect_ratio = 16.0f / 9.0f;
  s.cam.samples_per_pixel = 50;
  s.cam.max_depth = 20;
  sky_camera(s.cam, 20.0f, point3(13.0f, 2.0f, 3.0f), point3(0.0f, 0.0f, 0.0f), color(0.7f, 0.8f, 1.0f));
  return s;
}

inline scene earth() {  // main.cpp:141-171
  auto surface = std::make_shared<lambertian>(std::make_shared<image_texture>("earthmap.jpg"));
  auto world = std::make_shared<hittable_list>(std::make_shared<sphere>(point3(0.0f, 0.0f, 0.0f), 2.0f, surface));
  scene s{world, camera()};
  s.cam.image_width = 400;
  s.cam.aspect_ratio = 16.0f / 9.0f;
  s.cam.samples_per_pixel = 100;
  s.cam.max_depth = 50;
  sky_camera(s.cam, 20.0f, point3(0.0f, 0.0f, 12.0f), point3(0.0f, 0.0f, 0.0f), color(0.7f, 0.8f, 1.0f));
  return s;
}

inline scene perlin_sphere() {  // main.cpp:174-207
  auto world = std::make_shared<hittable_list>();
  auto pertext = std::make_shared<noise_texture>(4);
  world->add(std::make_shared<sphere>(point3(0.0f, -1000.0f, 0.0f), 1000.0f, std::make_shared<lambertian>(pertext)));
  world->add(std::make_shared<sphere>(point3(0.0f, 2.0f, 0.0f), 2.0f, std::make_shared<lambertian>(pertext)));
  scene s{world, camera()};
  s.cam.image_width = 400;
  s.cam.aspect_ratio = 16.0f / 9.0f;
  s.cam.samples_per_pixel = 100;
  s.cam.max_depth = 50;
  sky_camera(s.cam, 20.0f, point3(13.0f, 2.0f, 3.0f), point3(0.0f, 0.0f, 0.0f), color(0.7f, 0.8f, 1.0f));
  return s;
}

inline scene quads() {  // main.cpp:210-251
  auto world = std::make_shared<hittable_list>();
  world->add(std::make_shared<quad>(point3(-3.0f, -2.0f, 5.0f), vec3(0.0f, 0.0f, -4.0f), vec3(0.0f, 4.0f, 0.0f),
                                    std::make_shared<lambertian>(color(1.0f, 0.2f, 0.2f))));
  world->add(std::make_shared<quad>(point3(-2.0f, -2.0f, 0.0f), vec3(4.0f, 0.0f, 0.0f), vec3(0.0f, 4.0f, 0.0f),
                                    std::make_shared<lambertian>(color(0.2f, 1.0f, 0.2f))));
  world->add(std::make_shared<quad>(point3(3.0f, -2.0f, 1.0f), vec3(0.0f, 0.0f, 4.0f), vec3(0.0f, 4.0f, 0.0f),
                                    std::make_shared<lambertian>(color(0.2f, 0.2f, 1.0f))));
  world->add(std::make_shared<quad>(point3(-2.0f, 3.0f, 1.0f), vec3(4.0f, 0.0f, 0.0f), vec3(0.0f, 0.0f, 4.0f),
                                    std::make_shared<lambertian>(color(1.0f, 0.5f, 0.0f))));
  world->add(std::make_shared<quad>(point3(-2.0f, -3.0f, 5.0f), vec3(4.0f, 0.0f, 0.0f), vec3(0.0f, 0.0f, -4.0f),
                                    std::make_shared<lambertian>(color(0.2f, 0.8f, 0.8f))));
  scene s{world, camera()};
  s.cam.image_width = 400;
  s.cam.aspect_ratio = 1.0f;
  s.cam.samples_per_pixel = 100;
  s.cam.max_depth = 50;
  sky_camera(s.cam, 80.0f, point3(0.0f, 0.0f, 9.0f), point3(0.0f, 0.0f, 0.0f), color(0.7f, 0.8f, 1.0f));
  return s;
}

inline scene simple_light() {  // main.cpp:254-298
  auto world = std::make_shared<hittable_list>();
  auto pertext = std::make_shared<noise_texture>(4);
  world->add(std::make_shared<sphere>(point3(0.0f, -1000.0f, 0.0f), 1000.0f, std::make_shared<lambertian>(pertext)));
  world->add(std::make_shared<sphere>(point3(0.0f, 2.0f, 0.0f), 2.0f, std::make_shared<lambertian>(pertext)));
  auto light = std::make_shared<diffuse_light>(color(4.0f, 4.0f, 4.0f));
  world->add(std::make_shared<sphere>(point3(0.0f, 7.0f, 0.0f), 2.0f, light));
  world->add(std::make_shared<quad>(point3(3.0f, 1.0f, -2.0f), vec3(2.0f, 0.0f, 0.0f), vec3(0.0f, 2.0f, 0.0f), light));
  scene s{world, camera()};
  s.cam.image_width = 400;
  s.cam.aspect_ratio = 16.0f / 9.0f;
  s.cam.samples_per_pixel = 100;
  s.cam.max_depth = 50;
  sky_camera(s.cam, 20.0f, point3(26.0f, 3.0f, 6.0f), point3(0.0f, 2.0f, 0.0f), color(0.0f, 0.0f, 0.0f));
  return s;
}

inline scene cornell_box() {  // main.cpp:301-346
  auto world = std::make_shared<hittable_list>();
  auto red = std::make_shared<lambertian>(color(0.65f, 0.05f, 0.05f));
  auto white = std::make_shared<lambertian>(color(0.73f, 0.73f, 0.73f));
  auto green = std::make_shared<lambertian>(color(0.12f, 0.45f, 0.15f));
  auto light = std::make_shared<diffuse_light>(color(15.0f, 15.0f, 15.0f));
  const double L = 555.0f;
  world->add(std::make_shared<quad>(point3(L, 0.0f, 0.0f), vec3(0.0f, L, 0.0f), vec3(0.0f, 0.0f, L), green));
  world->add(std::make_shared<quad>(point3(0.0f, 0.0f, 0.0f), vec3(0.0f, L, 0.0f), vec3(0.0f, 0.0f, L), red));
  world->add(std::make_shared<quad>(point3(343.0f, 554.0f, 332.0f), vec3(-130.0f, 0.0f, 0.0f), vec3(0.0f, 0.0f, -105.0f), light));
  world->add(std::make_shared<quad>(point3(0.0f, 0.0f, 0.0f), vec3(L, 0.0f, 0.0f), vec3(0.0f, 0.0f, L), white));
  world->add(std::make_shared<quad>(point3(L, L, L), vec3(-L, 0.0f, 0.0f), vec3(0.0f, 0.0f, -L), white));
  world->add(std::make_shared<quad>(point3(0.0f, 0.0f, L), vec3(L, 0.0f, 0.0f), vec3(0.0f, L, 0.0f), white));
  world->add(box(point3(130.0f, 0.0f, 65.0f), point3(295.0f, 165.0f, 230.0f), white));
  world->add(box(point3(265.0f, 0.0f, 295.0f), point3(430.0f, 330.0f, 460.0f), white));
  scene s{world, camera()};
  s.cam.image_width = 600;
  s.cam.aspect_ratio = 1.0f;
  s.cam.samples_per_pixel = 100;
  s.cam.max_depth = 50;
  sky_camera(s.cam, 40.0f, point3(278.0f, 278.0f, -800.0f), point3(278.0f, 278.0f, 0.0f), color(0.0f, 0.0f, 0.0f));
  return s;
}

// Regression scene for translate (hittable.hpp:74-117; not in main.cpp): the Cornell box with its
// two boxes built at the origin and moved by translate (one of them by a translate of a translate)
// plus a translated metal sphere, so quads, spheres and nested offsets all go through
// translate::rtg_flatten. oracle/ref_harness.cpp builds the same scene with the reference's own
// translate class for the statistical golden.
inline scene cornell_translate() {
  scene s = cornell_box();
  auto world = std::make_shared<hittable_list>();
  auto& objs = std::static_pointer_cast<hittable_list>(s.world)->objects;
  for (size_t k = 0; k < 6; ++k) world->add(objs[k]);  // the five walls and the light
  auto white = std::make_shared<lambertian>(color(0.73f, 0.73f, 0.73f));
  auto chrome = std::make_shared<metal>(color(0.8f, 0.85f, 0.88f), 0.0f);
  world->add(std::make_shared<translate>(box(point3(0.0f, 0.0f, 0.0f), point3(165.0f, 330.0f, 165.0f), white),
                                         vec3(265.0f, 0.0f, 295.0f)));
  world->add(std::make_shared<translate>(
      std::make_shared<translate>(box(point3(0.0f, 0.0f, 0.0f), point3(165.0f, 165.0f, 165.0f), white),
                                  vec3(100.0f, 0.0f, 0.0f)),
      vec3(30.0f, 0.0f, 65.0f)));
  world->add(std::make_shared<translate>(std::make_shared<sphere>(point3(0.0f, 0.0f, 0.0f), 60.0f, chrome),
                                         vec3(420.0f, 90.0f, 120.0f)));
  s.world = world;
  return s;
}

// Benchmark config 3: Perlin ground of perlin_sphere + the earth globe, drawn in
// that order so the Perlin tables come first from the seed-1 stream.
inline scene earth_perlin() {
  auto world = std::make_shared<hittable_list>();
  auto pertext = std::make_shared<noise_texture>(4);
  world->add(std::make_shared<sphere>(point3(0.0f, -1000.0f, 0.0f), 1000.0f, std::make_shared<lambertian>(pertext)));
  auto globe = std::make_shared<lambertian>(std::make_shared<image_texture>("earthmap.jpg"));
  world->add(std::make_shared<sphere>(point3(0.0f, 2.0f, 0.0f), 2.0f, globe));
  scene s{world, camera()};
  s.cam.image_width = 1920;
  s.cam.aspect_ratio = 16.0 / 9.0;
  s.cam.samples_per_pixel = 500;
  s.cam.max_depth = 50;
  sky_camera(s.cam, 20.0f, point3(13.0f, 2.0f, 3.0f), point3(0.0f, 0.0f, 0.0f), color(0.7f, 0.8f, 1.0f));
  return s;
}

// Exact-t ties inside a bvh_node (not in main.cpp): groups of identical spheres,
// static spheres with a moving twin that coincides at time 0, coplanar quads of different extents and
// two identical compound children (hittable_lists of two quads) in the same plane, plus background
// spheres, every object emitting its own colour (so a pixel shows which object won). oracle/ref_harness.cpp
// "ties" builds the same objects with the reference's own classes and records the winners of exactly
// equal t, as a plain list and wrapped in bvh_node as main.cpp:76 wraps book-1 (tests/golden/ties.json).
// as_list = false: hittable_list(bvh_node(objects)), whose ties follow the median tree's leaf order.
inline scene tie_world(bool as_list = false) {
  hittable_list objs;
  int k = 0;
  auto mat = [&k]() {
    const double c = static_cast<double>(k++);
    return std::make_shared<diffuse_light>(color(0.1 + 0.02 * c, 1.0 - 0.02 * c, 0.5));
  };
  for (int m = 0; m < 4; ++m)  // 4 groups of 4 identical spheres, the list interleaving the groups
    for (int g = 0; g < 4; ++g) objs.add(std::make_shared<sphere>(point3(-9.0 + 6.0 * g, 4.0, 0.0), 1.5, mat()));
  for (int g = 0; g < 4; ++g) {  // a static sphere, then its moving twin (the same centre at time 0)
    const point3 c(-9.0 + 6.0 * g, -4.0, 0.0);
    objs.add(std::make_shared<sphere>(c, 1.5, mat()));
    objs.add(std::make_shared<sphere>(c, c + vec3(g % 2 ? 3.0 : -3.0, 0.0, 0.0), 1.5, mat()));
  }
  for (int q = 0; q < 4; ++q)  // coplanar quads in z = 3, box minima x = -2, -4, -6, -8
    objs.add(std::make_shared<quad>(point3(-2.0 - 2.0 * q, -1.0, 3.0), vec3(4.0 + 4.0 * q, 0.0, 0.0),
                                    vec3(0.0, 2.0, 0.0), mat()));
  for (int j = 0; j < 2; ++j) {  // two identical compound children in the same plane
    auto pane = std::make_shared<hittable_list>();
    pane->add(std::make_shared<quad>(point3(5.0, -1.0, 3.0), vec3(4.0, 0.0, 0.0), vec3(0.0, 2.0, 0.0), mat()));
    pane->add(std::make_shared<quad>(point3(5.0, -1.0, 3.0), vec3(2.0, 0.0, 0.0), vec3(0.0, 1.0, 0.0), mat()));
    objs.add(pane);
  }
  for (int b = 0; b < 8; ++b)  // background
    objs.add(std::make_shared<sphere>(point3(-14.0 + 4.0 * b, b % 2 ? -8.0 : 8.0, -6.0), 1.0, mat()));
  scene s{as_list ? std::make_shared<hittable_list>(objs)
                  : std::make_shared<hittable_list>(std::make_shared<bvh_node>(objs)),
          camera()};
  s.cam.image_width = 96;
  s.cam.aspect_ratio = 1.5;
  s.cam.samples_per_pixel = 4;
  s.cam.max_depth = 3;
  sky_camera(s.cam, 44.0, point3(0.0, 0.0, 30.0), point3(0.0, 0.0, 0.0), color(0.0, 0.0, 0.0));
  return s;
}

inline const std::map<std::string, std::function<scene(int)>>& registry() {
  static const std::map<std::string, std::function<scene(int)>> r = {
      {"bouncing_spheres", [](int g) { return bouncing_spheres(g > 0 ? g : 11); }},
      {"checkered_spheres", [](int) { return checkered_spheres(); }},
      {"earth", [](int) { return earth(); }},
      {"perlin_sphere", [](int) { return perlin_sphere(); }},
      {"quads", [](int) { return quads(); }},
      {"simple_light", [](int) { return simple_light(); }},
      {"cornell_box", [](int) { return cornell_box(); }},
      {"cornell_translate", [](int) { return cornell_translate(); }},
      {"earth_perlin", [](int) { return earth_perlin(); }},
      {"tie_world", [](int g) { return tie_world(g == 1); }},  // grid 1: the plain list
  };
  return r;
}

}  // namespace scenes
