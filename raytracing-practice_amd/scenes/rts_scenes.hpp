// scenes/rts_scenes.hpp — C-ABI of librtscenes.so: the reference's scenes (main.cpp:12-346) and
// the benchmark configurations built with the C++ API mirror, flattened for librtgpu.
#ifndef RTS_SCENES_H
#define RTS_SCENES_H
#include <stdint.h>

#include "rtgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rts_params {
  int32_t grid;              /* bouncing_spheres: a, b in [-grid, grid) (reference: 11) */
  int32_t image_width;       /* 0: the scene's own value */
  double aspect_ratio;       /* 0: the scene's own value */
  int32_t samples_per_pixel; /* 0: the scene's own value */
  int32_t max_depth;         /* < 0: the scene's own value */
  int32_t bvh_mode;          /* RTG_BVH_* used in the returned desc */
  uint32_t rand_seed;        /* srand() before building the scene (1 == the reference) */
} rts_params;

typedef struct rts_scene rts_scene;

/* names: bouncing_spheres, checkered_spheres, earth, perlin_sphere, quads, simple_light,
 * cornell_box, earth_perlin (benchmark config 3) */
int32_t rts_build(const char* name, const rts_params* params, rts_scene** out);
const rtg_scene_desc* rts_scene_desc(const rts_scene* s);
const rtg_camera_desc* rts_scene_camera(const rts_scene* s);
void rts_free(rts_scene* s);
const char* rts_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
