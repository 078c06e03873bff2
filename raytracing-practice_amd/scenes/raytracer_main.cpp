// scenes/raytracer_main.cpp — the reference's main() (main.cpp:348-397) on the device path:
//   raytracer [output.ppm] [scene] [width] [spp] [depth] [devices]
// Default scene cornell_box (the reference's switch(7)), default output output/image.ppm;
// devices = comma-separated HIP device ids to split the rows over (default: device 0).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>

#include "scenes.hpp"

int main(int argc, char* argv[]) {
  const std::string out_path = argc > 1 ? argv[1] : "output/image.ppm";
  const std::string name = argc > 2 ? argv[2] : "cornell_box";
  std::ofstream out(out_path);
  if (!out) {
    std::fprintf(stderr, "Error: could not open file %s for writing.\n", out_path.c_str());
    return 1;
  }
  const auto& reg = scenes::registry();
  auto it = reg.find(name);
  if (it == reg.end()) {
    std::fprintf(stderr, "Error: unknown scene %s\n", name.c_str());
    return 1;
  }
  scenes::scene s = it->second(11);
  if (argc > 3) s.cam.image_width = std::atoi(argv[3]);
  if (argc > 4) s.cam.samples_per_pixel = std::atoi(argv[4]);
  if (argc > 5) s.cam.max_depth = std::atoi(argv[5]);
  if (argc > 6) {
    std::stringstream ids(argv[6]);
    for (std::string id; std::getline(ids, id, ',');) s.cam.devices.push_back(std::atoi(id.c_str()));
  }
  s.cam.render(out, *s.world);
  std::fprintf(stderr, "segments=%llu samples=%llu kernel_ms=%.3f Mrays/s=%.1f\n",
               (unsigned long long)s.cam.last_stats.segments, (unsigned long long)s.cam.last_stats.samples,
               s.cam.last_stats.kernel_ms, s.cam.last_stats.segments / (s.cam.last_stats.kernel_ms * 1e3));
  return 0;
}
