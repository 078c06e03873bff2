// scenes/rts_scenes.cpp — librtscenes.so: builds a reference scene with the C++ API mirror and
// hands out its flattened rtg_scene_desc + camera (scenes/rts_scenes.hpp).
#include "rts_scenes.hpp"

#include <cstdlib>
#include <string>

#include "scenes.hpp"

namespace {
thread_local std::string g_err;
}

struct rts_scene {
  scenes::scene sc;
  rtgpu::scene_builder sb;
  rtg_scene_desc desc{};
  rtg_camera_desc cam{};
};

extern "C" {

const char* rts_last_error(void) { return g_err.c_str(); }

int32_t rts_build(const char* name, const rts_params* p, rts_scene** out) {
  if (!name || !out) {
    g_err = "null argument";
    return RTG_E_INVALID;
  }
  *out = nullptr;
  const auto& reg = scenes::registry();
  auto it = reg.find(name);
  if (it == reg.end()) {
    g_err = std::string("unknown scene '") + name + "'";
    return RTG_E_INVALID;
  }
  rts_params prm{};
  prm.max_depth = -1;
  prm.bvh_mode = RTG_BVH_SAH;
  prm.rand_seed = 1;
  if (p) prm = *p;
  std::srand(prm.rand_seed);
  auto* s = new rts_scene();
  s->sc = it->second(prm.grid);
  if (prm.image_width > 0) s->sc.cam.image_width = prm.image_width;
  if (prm.aspect_ratio > 0) s->sc.cam.aspect_ratio = prm.aspect_ratio;
  if (prm.samples_per_pixel > 0) s->sc.cam.samples_per_pixel = prm.samples_per_pixel;
  if (prm.max_depth >= 0) s->sc.cam.max_depth = prm.max_depth;
  if (!s->sc.world->rtg_flatten(s->sb, vec3(0, 0, 0))) {
    g_err = "flatten failed: " + s->sb.error;
    delete s;
    return RTG_E_INVALID;
  }
  s->desc = s->sb.desc(prm.bvh_mode);
  s->cam = s->sc.cam.desc();
  *out = s;
  return RTG_OK;
}

const rtg_scene_desc* rts_scene_desc(const rts_scene* s) { return s ? &s->desc : nullptr; }
const rtg_camera_desc* rts_scene_camera(const rts_scene* s) { return s ? &s->cam : nullptr; }
void rts_free(rts_scene* s) { delete s; }

}  // extern "C"
