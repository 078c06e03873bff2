// oracle/ref_harness.cpp — TEST INFRASTRUCTURE ONLY. Compiled (oracle/Makefile) against the
// reference's own headers under /root/reference/src to produce golden vectors that pin the oracle
// (oracle/cpu_ref.c). Output goes to oracle/_ref/ and, via oracle/gen_golden.py, to tests/golden/.
//
// Built from the reference: common/{rtweekend,vec3,ray,interval,color}.hpp,
// accelerator/{aabb,bvh_node}.hpp, hittable/{hittable,hittable_list,sphere,quad}.hpp,
// core/perlin.hpp — compiled with g++ 11 exactly as the reference would be (GCC evaluation
// order, hazard H2).
// NOT buildable here: core/{camera,material,texture,rtw_stb_image}.hpp, because texture.hpp
// includes <stb_image.h>, which the reference fetches from the network at configure time and
// which is absent from this image. The render loop below therefore restates camera::render /
// ray_color (camera.hpp:29-72, 139-232), the four materials (material.hpp:21-240) and the
// textures (texture.hpp:11-156) — ~150 lines — on top of the reference's geometry, BVH, RNG,
// vector and perlin code. DESIGN.md calls this build "ref-hybrid".
//
// Modes:
//   ref_harness golden                     -> JSON golden vectors on stdout
//   ref_harness ties                       -> exact-t tie winners, plain list vs bvh_node (JSON)
//   ref_harness render SCENE W H SPP DEPTH SEED OUT.bin   -> fp64 framebuffer + segment count
//   ref_harness bench SCENE W H SPP DEPTH PROCS [ROWSTEP] -> multi-process timing (JSON)
//   ref_harness moments SCENE W H SPP DEPTH PROCS SEED0 OUT.bin -> per-pixel sum L, sum L^2 (G5)
//   ref_harness records GRID OUT.bin                      -> bouncing_spheres records (G1')
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "common/rtweekend.hpp"
#include "accelerator/bvh_node.hpp"
#include "hittable/hittable.hpp"
#include "hittable/hittable_list.hpp"
#include "hittable/quad.hpp"
#include "hittable/sphere.hpp"
#include "core/perlin.hpp"

// ------------------------------------------------------------------------------------------
// Restated (unbuildable here) material.hpp / texture.hpp — same classes, same arithmetic.
class texture {
 public:
  virtual ~texture() = default;
  virtual color value(double u, double v, const point3& p) const = 0;
};
class solid_color : public texture {
 public:
  solid_color(const color& albedo) : albedo(albedo) {}
  color value(double, double, const point3&) const override { return albedo; }

 private:
  color albedo;
};
class checker_texture : public texture {
 public:
  checker_texture(double scale, std::shared_ptr<texture> even, std::shared_ptr<texture> odd)
      : inv_scale(1.0f / scale), even(even), odd(odd) {}
  checker_texture(double scale, const color& c1, const color& c2)
      : checker_texture(scale, std::make_shared<solid_color>(c1), std::make_shared<solid_color>(c2)) {}
  color value(double u, double v, const point3& p) const override {
    int xi = int(std::floor(inv_scale * p.x()));
    int yi = int(std::floor(inv_scale * p.y()));
    int zi = int(std::floor(inv_scale * p.z()));
    return ((xi + yi + zi) % 2 == 0) ? even->value(u, v, p) : odd->value(u, v, p);
  }

 private:
  double inv_scale;
  std::shared_ptr<texture> even, odd;
};
class noise_texture : public texture {
 public:
  noise_texture(double scale) : scale(scale) {}
  color value(double, double, const point3& p) const override {
    return color(0.5f, 0.5f, 0.5f) * (1.0f + std::sin(scale * p.z() + 10.0f * noise.turb(p, 7)));
  }

 private:
  perlin noise;  // the reference's perlin (perlin.hpp), tables drawn from rand() here
  double scale;
};

// rtw_image (rtw_stb_image.hpp:28-178) restated on the committed decoded texels: stb_image is absent
// (hazard H11), so tests/golden/earthmap.ppm holds earthmap.jpg decoded to 8-bit sRGB, and the load
// applies stbi_loadf's ldr-to-hdr step (pow(b / 255, 2.2), C double pow as in stb) then
// float_to_byte (rtw_stb_image.hpp:137-150), exactly the bytes rtw_image::convert_to_bytes keeps.
// pixel_data keeps the reference's clamp (x = high - 1 past the edge) and magenta fallback.
class rtw_image_ppm {
 public:
  explicit rtw_image_ppm(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) {
      std::fprintf(stderr, "ref_harness: cannot open %s\n", path.c_str());
      return;
    }
    int w = 0, h = 0, maxv = 0;
    char magic[3] = {0, 0, 0};
    if (std::fscanf(f, "%2s %d %d %d", magic, &w, &h, &maxv) == 4 && std::string(magic) == "P6" && maxv == 255 &&
        std::fgetc(f) != EOF) {
      std::vector<unsigned char> b(static_cast<size_t>(w) * h * 3);
      if (std::fread(b.data(), 1, b.size(), f) == b.size()) {
        for (auto& x : b) x = float_to_byte(static_cast<float>(::pow(x / 255.0f, 2.2f) * 1.0f));
        bdata.swap(b);
        image_width = w;
        image_height = h;
      }
    }
    std::fclose(f);
  }
  int width() const { return bdata.empty() ? 0 : image_width; }
  int height() const { return bdata.empty() ? 0 : image_height; }
  const unsigned char* pixel_data(int x, int y) const {
    static unsigned char magenta[] = {255, 0, 255};
    if (bdata.empty()) return magenta;
    x = clamp(x, 0, image_width);
    y = clamp(y, 0, image_height);
    return bdata.data() + y * image_width * 3 + x * 3;
  }

 private:
  static int clamp(int x, int low, int high) { return x < low ? low : (x < high ? x : high - 1); }
  static unsigned char float_to_byte(float value) {
    if (value <= 0.0f) return 0;
    if (value >= 1.0f) return 255;
    return static_cast<unsigned char>(256.0f * value);
  }
  std::vector<unsigned char> bdata;
  int image_width = 0, image_height = 0;
};

// tests/golden/earthmap.ppm: $RTG_EARTHMAP, else relative to this executable (oracle/_ref/)
static std::string earthmap_path() {
  if (const char* e = std::getenv("RTG_EARTHMAP")) return e;
  char buf[4096];
  const ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  std::string exe = n > 0 ? std::string(buf, static_cast<size_t>(n)) : std::string("oracle/_ref/ref_harness");
  return exe.substr(0, exe.find_last_of('/')) + "/../../tests/golden/earthmap.ppm";
}

// image_texture::value (texture.hpp:97-118)
class image_texture : public texture {
 public:
  explicit image_texture(const std::string& path) : image(path) {}
  color value(double u, double v, const point3&) const override {
    if (image.height() <= 0) return color(0.0f, 1.0f, 1.0f);
    u = interval(0.0f, 1.0f).clamp(u);
    v = 1.0f - interval(0.0f, 1.0f).clamp(v);
    auto i = int(u * image.width());
    auto j = int(v * image.height());
    auto pixel = image.pixel_data(i, j);
    auto color_scale = 1.0f / 255.0f;
    return color(color_scale * pixel[0], color_scale * pixel[1], color_scale * pixel[2]);
  }

 private:
  rtw_image_ppm image;
};

class material {
 public:
  virtual ~material() = default;
  virtual color emitted(double, double, const point3&) const { return color(0.0f, 0.0f, 0.0f); }
  virtual bool scatter(const ray&, const hit_record&, color&, ray&) const { return false; }
};
class lambertian : public material {
 public:
  lambertian(const color& a) : tex(std::make_shared<solid_color>(a)) {}
  lambertian(std::shared_ptr<texture> t) : tex(t) {}
  bool scatter(const ray& r_in, const hit_record& rec, color& att, ray& scattered) const override {
    vec3 dir = rec.normal + random_unit_vector();  // the reference's vec3.hpp sampler
    if (dir.near_zero()) dir = rec.normal;
    scattered = ray(rec.p, dir, r_in.time());
    att = tex->value(rec.u, rec.v, rec.p);
    return true;
  }

 private:
  std::shared_ptr<texture> tex;
};
class metal : public material {
 public:
  metal(const color& albedo, double fuzz) : albedo(albedo), fuzz(fuzz < 1.0f ? fuzz : 1.0f) {}
  bool scatter(const ray& r_in, const hit_record& rec, color& att, ray& scattered) const override {
    vec3 reflected = reflect(r_in.direction(), rec.normal);
    reflected = unit_vector(reflected) + (fuzz * random_unit_vector());
    scattered = ray(rec.p, reflected, r_in.time());
    att = albedo;
    return dot(scattered.direction(), rec.normal) > 0;
  }

 private:
  color albedo;
  double fuzz;
};
class dielectric : public material {
 public:
  dielectric(double ri) : refraction_index(ri) {}
  bool scatter(const ray& r_in, const hit_record& rec, color& att, ray& scattered) const override {
    att = color(1.0f, 1.0f, 1.0f);
    double ri = rec.front_face ? (1.0f / refraction_index) : refraction_index;
    vec3 ud = unit_vector(r_in.direction());
    double cos_theta = std::fmin(dot(-ud, rec.normal), 1.0f);
    double sin_theta = std::sqrt(1.0f - cos_theta * cos_theta);
    bool cannot = ri * sin_theta > 1.0f;
    vec3 direction;
    if (cannot || reflectance(cos_theta, ri) > random_double())
      direction = reflect(ud, rec.normal);
    else
      direction = refract(ud, rec.normal, ri);
    scattered = ray(rec.p, direction, r_in.time());
    return true;
  }
  static double reflectance(double cosine, double ri) {
    auto r0 = (1.0f - ri) / (1.0f + ri);
    r0 = r0 * r0;
    return r0 + (1.0f - r0) * std::pow((1.0f - cosine), 5);
  }

 private:
  double refraction_index;
};
class diffuse_light : public material {
 public:
  diffuse_light(const color& emit) : tex(std::make_shared<solid_color>(emit)) {}
  color emitted(double u, double v, const point3& p) const override { return tex->value(u, v, p); }

 private:
  std::shared_ptr<texture> tex;
};

// ------------------------------------------------------------------------------------------
// Restated camera (camera.hpp:13-245) with a segment counter at world.hit (camera.hpp:192).
struct cam_t {
  double aspect_ratio = 1.0f;
  int image_width = 100, samples_per_pixel = 10, max_depth = 10;
  color background;
  double vfov = 90.0f;
  point3 lookfrom = point3(0.0f, 0.0f, 0.0f), lookat = point3(0.0f, 0.0f, -1.0f);
  vec3 vup = vec3(0.0f, 1.0f, 0.0f);
  double defocus_angle = 0.0f, focus_dist = 10.0f;

  int image_height;
  double pixel_samples_scale;
  point3 center, pixel00_loc;
  vec3 pixel_delta_u, pixel_delta_v, u, v, w, defocus_disk_u, defocus_disk_v;
  unsigned long long segments = 0;

  void initialize() {
    image_height = static_cast<int>(image_width / aspect_ratio);
    image_height = (image_height < 1) ? 1 : image_height;
    pixel_samples_scale = 1.0f / samples_per_pixel;
    center = lookfrom;
    auto theta = degrees_to_radians(vfov);
    auto h = std::tan(theta / 2);
    auto vh = 2 * h * focus_dist;
    auto vw = vh * (static_cast<double>(image_width) / image_height);
    w = unit_vector(lookfrom - lookat);
    u = unit_vector(cross(vup, w));
    v = cross(w, u);
    auto vu = vw * u;
    auto vv = vh * -v;
    pixel_delta_u = vu / image_width;
    pixel_delta_v = vv / image_height;
    auto ul = center - (focus_dist * w) - vu / 2 - vv / 2;
    pixel00_loc = ul + 0.5 * (pixel_delta_u + pixel_delta_v);
    auto rad = focus_dist * std::tan(degrees_to_radians(defocus_angle) / 2.0f);
    defocus_disk_u = u * rad;
    defocus_disk_v = v * rad;
  }
  vec3 sample_square() const { return vec3(random_double() - 0.5f, random_double() - 0.5f, 0.0f); }
  point3 defocus_disk_sample() const {
    auto p = random_in_unit_disk();
    return center + (p[0] * defocus_disk_u) + (p[1] * defocus_disk_v);
  }
  ray get_ray(int i, int j) const {
    auto offset = sample_square();
    auto ps = pixel00_loc + ((i + offset.x()) * pixel_delta_u) + ((j + offset.y()) * pixel_delta_v);
    auto origin = (defocus_angle <= 0.0f) ? center : defocus_disk_sample();
    auto dir = ps - origin;
    auto t = random_double();
    return ray(origin, dir, t);
  }
  color ray_color(const ray& r, int depth, const hittable& world) {
    if (depth <= 0) return color(0.0f, 0.0f, 0.0f);
    hit_record rec;
    ++segments;
    if (!world.hit(r, interval(0.001, infinity), rec)) return background;
    color e = rec.mat->emitted(rec.u, rec.v, rec.p);
    ray scattered;
    color att;
    if (!rec.mat->scatter(r, rec, att, scattered)) return e;
    color s = att * ray_color(scattered, depth - 1, world);
    return e + s;
  }
  // Per-pixel first and second moments of one sample's radiance over every pixel of the image:
  // out[(j*W + i)*6 + c] += L_c, out[... + 3 + c] += L_c^2, for samples_per_pixel samples of
  // camera::render's loop order (camera.hpp:40-62). The statistical golden (G5) of the GPU.
  void render_moments(const hittable& world, double* out) {
    initialize();
    for (int j = 0; j < image_height; ++j)
      for (int i = 0; i < image_width; ++i) {
        double* q = out + ((long)j * image_width + i) * 6;
        for (int s = 0; s < samples_per_pixel; s++) {
          const color L = ray_color(get_ray(i, j), max_depth, world);
          for (int c = 0; c < 3; ++c) {
            q[c] += L[c];
            q[3 + c] += L[c] * L[c];
          }
        }
      }
  }
  // rows [r0, r0+nr): out = pixel_samples_scale * pixel_color (the input of write_color)
  void render(const hittable& world, int r0, int nr, double* out) {
    initialize();
    for (int j = r0; j < r0 + nr; ++j)
      for (int i = 0; i < image_width; ++i) {
        color pc(0.0f, 0.0f, 0.0f);
        for (int s = 0; s < samples_per_pixel; s++) pc += ray_color(get_ray(i, j), max_depth, world);
        color o = pixel_samples_scale * pc;
        double* q = out + ((long)(j - r0) * image_width + i) * 3;
        q[0] = o.x();
        q[1] = o.y();
        q[2] = o.z();
      }
  }
};

// ------------------------------------------------------------------------------------------
// Scenes (restated from main.cpp; the geometry / BVH / RNG / perlin code is the reference's).
struct sphere_rec {
  double c1[3], c2[3], r;
  int mat;  // 1 lambertian(albedo), 2 metal, 3 dielectric, 0 ground checker
  double albedo[3], fuzz, ri;
};
static std::vector<sphere_rec> g_book1;

// bouncing_spheres (main.cpp:12-76), grid half-width `g` (11 in the reference)
static hittable_list book1_world(int g, bool record) {
  hittable_list world;
  auto checker = std::make_shared<checker_texture>(0.32f, color(0.2f, 0.3f, 0.1f), color(0.9f, 0.9f, 0.9f));
  auto ground = std::make_shared<lambertian>(checker);
  world.add(std::make_shared<sphere>(point3(0.0f, -1000.0f, -1.0f), 1000.0f, ground));
  if (record) g_book1.push_back({{0, -1000, -1}, {0, -1000, -1}, 1000, 0, {0, 0, 0}, 0, 0});
  for (int a = -g; a < g; a++) {
    for (int b = -g; b < g; b++) {
      auto choose_mat = random_double();
      point3 center(a + 0.9f * random_double(), 0.2f, b + 0.9f * random_double());
      if ((center - point3(4.0f, 0.2f, 0.0f)).length() > 0.9f) {
        std::shared_ptr<material> m;
        sphere_rec sr{};
        sr.c1[0] = center.x();
        sr.c1[1] = center.y();
        sr.c1[2] = center.z();
        sr.r = 0.2f;
        if (choose_mat < 0.8f) {
          auto albedo = color::random() * color::random();
          m = std::make_shared<lambertian>(albedo);
          auto center2 = center + vec3(0.0f, random_double(0.0f, 0.5f), 0.0f);
          world.add(std::make_shared<sphere>(center, center2, 0.2f, m));
          sr.mat = 1;
          for (int k = 0; k < 3; ++k) {
            sr.albedo[k] = albedo[k];
            sr.c2[k] = center2[k];
          }
        } else if (choose_mat < 0.95f) {
          auto albedo = color::random(0.5f, 1.0f);
          auto fuzz = random_double(0.0f, 0.5f);
          m = std::make_shared<metal>(albedo, fuzz);
          world.add(std::make_shared<sphere>(center, 0.2f, m));
          sr.mat = 2;
          sr.fuzz = fuzz;
          for (int k = 0; k < 3; ++k) {
            sr.albedo[k] = albedo[k];
            sr.c2[k] = center[k];
          }
        } else {
          m = std::make_shared<dielectric>(1.5f);
          world.add(std::make_shared<sphere>(center, 0.2f, m));
          sr.mat = 3;
          sr.ri = 1.5f;
          for (int k = 0; k < 3; ++k) sr.c2[k] = center[k];
        }
        if (record) g_book1.push_back(sr);
      }
    }
  }
  world.add(std::make_shared<sphere>(point3(0.0f, 1.0f, 0.0f), 1.0f, std::make_shared<dielectric>(1.5f)));
  world.add(std::make_shared<sphere>(point3(-4.0f, 1.0f, 0.0f), 1.0f,
                                     std::make_shared<lambertian>(color(0.4f, 0.2f, 0.1f))));
  world.add(std::make_shared<sphere>(point3(4.0f, 1.0f, 0.0f), 1.0f,
                                     std::make_shared<metal>(color(0.7f, 0.6f, 0.5f), 0.0f)));
  if (record) {
    g_book1.push_back({{0, 1, 0}, {0, 1, 0}, 1.0f, 3, {0, 0, 0}, 0, 1.5f});
    g_book1.push_back({{-4, 1, 0}, {-4, 1, 0}, 1.0f, 1, {0.4f, 0.2f, 0.1f}, 0, 0});
    g_book1.push_back({{4, 1, 0}, {4, 1, 0}, 1.0f, 2, {0.7f, 0.6f, 0.5f}, 0.0f, 0});
  }
  return world;
}

static void setup_cam(const std::string& scene, cam_t& c) {
  c.background = color(0.7f, 0.8f, 1.0f);
  c.vup = vec3(0.0f, 1.0f, 0.0f);
  c.lookat = point3(0.0f, 0.0f, 0.0f);
  c.vfov = 20.0f;
  c.lookfrom = point3(13.0f, 2.0f, 3.0f);
  c.defocus_angle = 0.0f;
  c.focus_dist = 10.0f;
  if (scene == "book1" || scene == "book1_g500") {
    c.defocus_angle = 0.6f;
  } else if (scene == "cornell") {  // main.cpp:325-342
    c.background = color(0.0f, 0.0f, 0.0f);
    c.vfov = 40.0f;
    c.lookfrom = point3(278.0f, 278.0f, -800.0f);
    c.lookat = point3(278.0f, 278.0f, 0.0f);
  } else if (scene == "cornell_translate") {  // the Cornell camera
    c.background = color(0.0f, 0.0f, 0.0f);
    c.vfov = 40.0f;
    c.lookfrom = point3(278.0f, 278.0f, -800.0f);
    c.lookat = point3(278.0f, 278.0f, 0.0f);
  } else if (scene == "simple_light") {  // main.cpp:277-294
    c.background = color(0.0f, 0.0f, 0.0f);
    c.lookfrom = point3(26.0f, 3.0f, 6.0f);
    c.lookat = point3(0.0f, 2.0f, 0.0f);
  } else if (scene == "earth") {  // main.cpp:157-166
    c.lookfrom = point3(0.0f, 0.0f, 12.0f);
  } else if (scene == "quads") {  // main.cpp:234-246
    c.vfov = 80.0f;
    c.lookfrom = point3(0.0f, 0.0f, 9.0f);
  }  // earth_perlin (BASELINE config 3): perlin_sphere's camera, main.cpp:190-201; checkered: main.cpp:118-134
}

static std::shared_ptr<hittable> make_world(const std::string& scene) {
  if (scene == "book1" || scene == "book1_g500") {  // g500: BASELINE config 5's 1M-sphere field
    hittable_list w = book1_world(scene == "book1" ? 11 : 500, false);
    return std::make_shared<hittable_list>(std::make_shared<bvh_node>(w));  // main.cpp:76
  }
  auto w = std::make_shared<hittable_list>();
  if (scene == "cornell" || scene == "cornell_translate") {  // main.cpp:301-322
    auto red = std::make_shared<lambertian>(color(0.65f, 0.05f, 0.05f));
    auto white = std::make_shared<lambertian>(color(0.73f, 0.73f, 0.73f));
    auto green = std::make_shared<lambertian>(color(0.12f, 0.45f, 0.15f));
    auto light = std::make_shared<diffuse_light>(color(15.0f, 15.0f, 15.0f));
    w->add(std::make_shared<quad>(point3(555.0f, 0.0f, 0.0f), vec3(0.0f, 555.0f, 0.0f), vec3(0.0f, 0.0f, 555.0f), green));
    w->add(std::make_shared<quad>(point3(0.0f, 0.0f, 0.0f), vec3(0.0f, 555.0f, 0.0f), vec3(0.0f, 0.0f, 555.0f), red));
    w->add(std::make_shared<quad>(point3(343.0f, 554.0f, 332.0f), vec3(-130.0f, 0.0f, 0.0f), vec3(0.0f, 0.0f, -105.0f), light));
    w->add(std::make_shared<quad>(point3(0.0f, 0.0f, 0.0f), vec3(555.0f, 0.0f, 0.0f), vec3(0.0f, 0.0f, 555.0f), white));
    w->add(std::make_shared<quad>(point3(555.0f, 555.0f, 555.0f), vec3(-555.0f, 0.0f, 0.0f), vec3(0.0f, 0.0f, -555.0f), white));
    w->add(std::make_shared<quad>(point3(0.0f, 0.0f, 555.0f), vec3(555.0f, 0.0f, 0.0f), vec3(0.0f, 555.0f, 0.0f), white));
    if (scene == "cornell") {
      w->add(box(point3(130.0f, 0.0f, 65.0f), point3(295.0f, 165.0f, 230.0f), white));
      w->add(box(point3(265.0f, 0.0f, 295.0f), point3(430.0f, 330.0f, 460.0f), white));
    } else {  // the reference's own translate class (hittable.hpp:74-117), nested once
      auto chrome = std::make_shared<metal>(color(0.8f, 0.85f, 0.88f), 0.0f);
      w->add(std::make_shared<translate>(box(point3(0.0f, 0.0f, 0.0f), point3(165.0f, 330.0f, 165.0f), white),
                                         vec3(265.0f, 0.0f, 295.0f)));
      w->add(std::make_shared<translate>(
          std::make_shared<translate>(box(point3(0.0f, 0.0f, 0.0f), point3(165.0f, 165.0f, 165.0f), white),
                                      vec3(100.0f, 0.0f, 0.0f)),
          vec3(30.0f, 0.0f, 65.0f)));
      w->add(std::make_shared<translate>(std::make_shared<sphere>(point3(0.0f, 0.0f, 0.0f), 60.0f, chrome),
                                         vec3(420.0f, 90.0f, 120.0f)));
    }
  } else if (scene == "earth") {  // main.cpp:141-171
    auto surface = std::make_shared<lambertian>(std::make_shared<image_texture>(earthmap_path()));
    w->add(std::make_shared<sphere>(point3(0.0f, 0.0f, 0.0f), 2.0f, surface));
  } else if (scene == "earth_perlin") {  // BASELINE config 3: perlin ground, then the globe
    auto pertext = std::make_shared<noise_texture>(4);  // perlin tables first from the seed-1 stream
    w->add(std::make_shared<sphere>(point3(0.0f, -1000.0f, 0.0f), 1000.0f, std::make_shared<lambertian>(pertext)));
    auto globe = std::make_shared<lambertian>(std::make_shared<image_texture>(earthmap_path()));
    w->add(std::make_shared<sphere>(point3(0.0f, 2.0f, 0.0f), 2.0f, globe));
  } else if (scene == "checkered") {  // main.cpp:104-116
    auto checker = std::make_shared<checker_texture>(0.32f, color(0.2f, 0.3f, 0.1f), color(0.9f, 0.9f, 0.9f));
    w->add(std::make_shared<sphere>(point3(0.0f, -10.0f, 0.0f), 10.0f, std::make_shared<lambertian>(checker)));
    w->add(std::make_shared<sphere>(point3(0.0f, 10.0f, 0.0f), 10.0f, std::make_shared<lambertian>(checker)));
  } else if (scene == "quads") {  // main.cpp:210-225
    auto left_red = std::make_shared<lambertian>(color(1.0f, 0.2f, 0.2f));
    auto back_green = std::make_shared<lambertian>(color(0.2f, 1.0f, 0.2f));
    auto right_blue = std::make_shared<lambertian>(color(0.2f, 0.2f, 1.0f));
    auto upper_orange = std::make_shared<lambertian>(color(1.0f, 0.5f, 0.0f));
    auto lower_teal = std::make_shared<lambertian>(color(0.2f, 0.8f, 0.8f));
    w->add(std::make_shared<quad>(point3(-3.0f, -2.0f, 5.0f), vec3(0.0f, 0.0f, -4.0f), vec3(0.0f, 4.0f, 0.0f), left_red));
    w->add(std::make_shared<quad>(point3(-2.0f, -2.0f, 0.0f), vec3(4.0f, 0.0f, 0.0f), vec3(0.0f, 4.0f, 0.0f), back_green));
    w->add(std::make_shared<quad>(point3(3.0f, -2.0f, 1.0f), vec3(0.0f, 0.0f, 4.0f), vec3(0.0f, 4.0f, 0.0f), right_blue));
    w->add(std::make_shared<quad>(point3(-2.0f, 3.0f, 1.0f), vec3(4.0f, 0.0f, 0.0f), vec3(0.0f, 0.0f, 4.0f), upper_orange));
    w->add(std::make_shared<quad>(point3(-2.0f, -3.0f, 5.0f), vec3(4.0f, 0.0f, 0.0f), vec3(0.0f, 0.0f, -4.0f), lower_teal));
  } else if (scene == "simple_light" || scene == "perlin") {  // main.cpp:174-207, 254-298
    auto pertext = std::make_shared<noise_texture>(4);
    w->add(std::make_shared<sphere>(point3(0.0f, -1000.0f, 0.0f), 1000.0f, std::make_shared<lambertian>(pertext)));
    w->add(std::make_shared<sphere>(point3(0.0f, 2.0f, 0.0f), 2.0f, std::make_shared<lambertian>(pertext)));
    if (scene == "simple_light") {
      auto difflight = std::make_shared<diffuse_light>(color(4.0f, 4.0f, 4.0f));
      w->add(std::make_shared<sphere>(point3(0.0f, 7.0f, 0.0f), 2.0f, difflight));
      w->add(std::make_shared<quad>(point3(3.0f, 1.0f, -2.0f), vec3(2.0f, 0.0f, 0.0f), vec3(0.0f, 2.0f, 0.0f), difflight));
    }
  }
  return w;
}

// ------------------------------------------------------------------------------------------
// golden JSON
static void pj(const char* k, double v, bool comma = true) { printf("\"%s\": %.17g%s", k, v, comma ? ", " : ""); }
static void pv(const char* k, const vec3& v, bool comma = true) {
  printf("\"%s\": [%.17g, %.17g, %.17g]%s", k, v.x(), v.y(), v.z(), comma ? ", " : "");
}
static void pa(const double* v, int n) {
  printf("[");
  for (int i = 0; i < n; ++i) printf("%.17g%s", v[i], i + 1 < n ? ", " : "");
  printf("]");
}

// a deterministic generator for KAT inputs that does not touch rand()
static unsigned long long g_kat = 0x243F6A8885A308D3ull;
static double kat_u() {
  g_kat ^= g_kat << 13;
  g_kat ^= g_kat >> 7;
  g_kat ^= g_kat << 17;
  return (g_kat >> 11) * (1.0 / 9007199254740992.0);
}
static double kat_r(double a, double b) { return a + (b - a) * kat_u(); }

class logged : public hittable {
 public:
  logged(int id, std::shared_ptr<hittable> o, std::vector<int>* log) : id(id), obj(o), log(log) {}
  bool hit(const ray& r, interval t, hit_record& rec) const override {
    log->push_back(id);
    return obj->hit(r, t, rec);
  }
  aabb bounding_box() const override { return obj->bounding_box(); }

 private:
  int id;
  std::shared_ptr<hittable> obj;
  std::vector<int>* log;
};

static int golden() {
  printf("{\n");
  // 1. rand stream (rtweekend.hpp:23-39)
  printf("\"rand_default\": [");
  for (int i = 0; i < 64; ++i) printf("%.17g%s", random_double(), i < 63 ? ", " : "");
  printf("],\n");
  srand(7);
  printf("\"rand_seed7\": [");
  for (int i = 0; i < 16; ++i) printf("%.17g%s", random_double(), i < 15 ? ", " : "");
  printf("],\n");
  srand(11);
  printf("\"random_int_seed11\": [");
  for (int i = 0; i < 64; ++i) printf("%d%s", random_int(0, 255 - (i % 200)), i < 63 ? ", " : "");
  printf("],\n");

  // 2. samplers (vec3.hpp:158-184): value + the next draw (pins the draw count and order)
  printf("\"random_unit_vector\": [");
  for (int k = 1; k <= 48; ++k) {
    srand(k);
    vec3 v = random_unit_vector();
    double nxt = random_double();
    printf("{\"seed\": %d, ", k);
    pv("v", v);
    pj("next", nxt, false);
    printf("}%s", k < 48 ? ", " : "");
  }
  printf("],\n\"random_in_unit_disk\": [");
  for (int k = 1; k <= 48; ++k) {
    srand(k);
    vec3 v = random_in_unit_disk();
    double nxt = random_double();
    printf("{\"seed\": %d, ", k);
    pv("v", v);
    pj("next", nxt, false);
    printf("}%s", k < 48 ? ", " : "");
  }
  printf("],\n");

  // 3. sphere::hit (sphere.hpp:47-111)
  printf("\"sphere_hit\": [");
  for (int k = 0; k < 400; ++k) {
    point3 c1(kat_r(-3, 3), kat_r(-3, 3), kat_r(-3, 3));
    bool moving = (k % 3) == 0;
    point3 c2 = moving ? c1 + vec3(kat_r(-1, 1), kat_r(-1, 1), kat_r(-1, 1)) : c1;
    double rad = (k % 17 == 0) ? -kat_r(0.2, 2) : kat_r(0.2, 2);
    if (k % 50 == 7) rad = 1000.0;
    point3 o(kat_r(-6, 6), kat_r(-6, 6), kat_r(-6, 6));
    point3 target = c1 + vec3(kat_r(-2, 2), kat_r(-2, 2), kat_r(-2, 2));
    if (k % 50 == 7) {
      c1 = c2 = point3(0, -1000, -1);
      o = point3(kat_r(-5, 5), kat_r(0.0, 0.01), kat_r(-5, 5));
      target = o + vec3(kat_r(-1, 1), kat_r(-1, 1), kat_r(-1, 1));
    }
    vec3 d = target - o;
    double time = kat_u();
    double tmin = 0.001, tmax = (k % 5 == 0) ? kat_r(0.5, 8) : infinity;
    sphere s = moving ? sphere(c1, c2, rad, nullptr) : sphere(c1, rad, nullptr);
    hit_record rec;
    bool h = s.hit(ray(o, d, time), interval(tmin, tmax), rec);
    printf("{");
    pv("c1", c1);
    pv("c2", c2);
    pj("r", rad);
    printf("\"moving\": %d, ", moving ? 1 : 0);
    pv("o", o);
    pv("d", d);
    pj("time", time);
    pj("tmin", tmin);
    pj("tmax", tmax == infinity ? 1e300 : tmax);
    printf("\"hit\": %d", h ? 1 : 0);
    if (h) {
      printf(", ");
      pj("t", rec.t);
      pv("p", rec.p);
      pv("normal", rec.normal);
      printf("\"front\": %d, ", rec.front_face ? 1 : 0);
      pj("u", rec.u);
      pj("v", rec.v, false);
    }
    printf("}%s", k < 399 ? ", " : "");
  }
  printf("],\n");

  // 4. quad::hit (quad.hpp:44-114)
  printf("\"quad_hit\": [");
  for (int k = 0; k < 300; ++k) {
    point3 Q(kat_r(-3, 3), kat_r(-3, 3), kat_r(-3, 3));
    vec3 u(kat_r(-2, 2), kat_r(-2, 2), kat_r(-2, 2)), v(kat_r(-2, 2), kat_r(-2, 2), kat_r(-2, 2));
    if (k % 4 == 0) {
      u = vec3(kat_r(0.5, 3), 0, 0);
      v = vec3(0, 0, kat_r(0.5, 3));
    }
    point3 o(kat_r(-6, 6), kat_r(-6, 6), kat_r(-6, 6));
    point3 target = Q + kat_u() * u + kat_u() * v + vec3(kat_r(-0.3, 0.3), kat_r(-0.3, 0.3), kat_r(-0.3, 0.3));
    vec3 d = target - o;
    quad q(Q, u, v, nullptr);
    hit_record rec;
    double tmax = (k % 5 == 0) ? kat_r(0.5, 8) : infinity;
    bool h = q.hit(ray(o, d, 0.0), interval(0.001, tmax), rec);
    printf("{");
    pv("Q", Q);
    pv("u", u);
    pv("v", v);
    pv("o", o);
    pv("d", d);
    pj("tmax", tmax == infinity ? 1e300 : tmax);
    printf("\"hit\": %d", h ? 1 : 0);
    if (h) {
      printf(", ");
      pj("t", rec.t);
      pv("p", rec.p);
      pv("normal", rec.normal);
      printf("\"front\": %d, ", rec.front_face ? 1 : 0);
      pj("u_", rec.u);
      pj("v_", rec.v, false);
    }
    aabb bb = q.bounding_box();
    printf(", \"bbox\": [%.17g, %.17g, %.17g, %.17g, %.17g, %.17g]", bb.x.min, bb.y.min, bb.z.min,
           bb.x.max, bb.y.max, bb.z.max);
    printf("}%s", k < 299 ? ", " : "");
  }
  printf("],\n");

  // 5. aabb::hit (aabb.hpp:61-112)
  printf("\"aabb_hit\": [");
  for (int k = 0; k < 300; ++k) {
    point3 a(kat_r(-3, 3), kat_r(-3, 3), kat_r(-3, 3)), b(kat_r(-3, 3), kat_r(-3, 3), kat_r(-3, 3));
    if (k % 10 == 0) b = point3(a.x(), b.y(), b.z());  // flat box -> padding
    aabb box(a, b);
    point3 o(kat_r(-6, 6), kat_r(-6, 6), kat_r(-6, 6));
    vec3 d = point3(kat_r(-3, 3), kat_r(-3, 3), kat_r(-3, 3)) - o;
    if (k % 13 == 0) d = vec3(d.x(), 0.0, d.z());
    double tmax = (k % 4 == 0) ? kat_r(0.1, 3) : infinity;
    bool h = box.hit(ray(o, d, 0.0), interval(0.001, tmax));
    printf("{\"box\": [%.17g, %.17g, %.17g, %.17g, %.17g, %.17g], ", box.x.min, box.y.min, box.z.min,
           box.x.max, box.y.max, box.z.max);
    pv("a", a);
    pv("b", b);
    pv("o", o);
    pv("d", d);
    pj("tmax", tmax == infinity ? 1e300 : tmax);
    printf("\"hit\": %d, \"longest_axis\": %d}%s", h ? 1 : 0, box.longest_axis(), k < 299 ? ", " : "");
  }
  printf("],\n");

  // 6. reflect / refract (vec3.hpp:207-226)
  printf("\"reflect_refract\": [");
  for (int k = 0; k < 100; ++k) {
    vec3 v = unit_vector(vec3(kat_r(-1, 1), kat_r(-1, 1), kat_r(-1, 1)));
    vec3 n = unit_vector(vec3(kat_r(-1, 1), kat_r(-1, 1), kat_r(-1, 1)));
    if (dot(v, n) > 0) n = -n;
    double eta = kat_r(0.5, 1.6);
    printf("{");
    pv("v", v);
    pv("n", n);
    pj("eta", eta);
    pv("reflect", reflect(v, n));
    pv("refract", refract(v, n, eta), false);
    printf("}%s", k < 99 ? ", " : "");
  }
  printf("],\n");

  // 7. write_color (color.hpp:14-58)
  printf("\"write_color\": [");
  for (int k = 0; k < 200; ++k) {
    color c(kat_r(-0.2, 1.3), kat_r(0, 1), (k % 7 == 0) ? 0.0 : kat_r(0, 1.1));
    std::ostringstream os;  // write_color writes to an ostream
    write_color(os, c);
    const std::string s = os.str();
    int r, g, b;
    sscanf(s.c_str(), "%d %d %d", &r, &g, &b);
    printf("{");
    pv("c", c);
    printf("\"bytes\": [%d, %d, %d]}%s", r, g, b, k < 199 ? ", " : "");
  }
  printf("],\n");

  // 8. perlin tables drawn first from the seed-1 stream (perlin.hpp:12-31), noise + turbulence
  srand(1);
  {
    perlin pn;
    double after = random_double();
    printf("\"perlin_seed1\": {\"next_draw\": %.17g, \"points\": [", after);
    for (int k = 0; k < 200; ++k) {
      point3 p(kat_r(-20, 20), kat_r(-20, 20), kat_r(-20, 20));
      if (k % 10 == 0) p = point3(kat_r(-1200, 1200), kat_r(-5, 5), kat_r(-1200, 1200));
      printf("{");
      pv("p", p);
      pj("noise", pn.noise_perlin(p));
      pj("turb7", pn.turb(p, 7), false);
      printf("}%s", k < 199 ? ", " : "");
    }
    printf("]},\n");
  }

  // 9. book-1 scene from the default (seed 1) stream, GCC evaluation order (main.cpp:12-73)
  srand(1);
  g_book1.clear();
  hittable_list w = book1_world(11, true);
  double after_scene = random_double();
  printf("\"book1\": {\"next_draw\": %.17g, \"spheres\": [", after_scene);
  for (size_t i = 0; i < g_book1.size(); ++i) {
    const sphere_rec& s = g_book1[i];
    printf("{\"c1\": ");
    pa(s.c1, 3);
    printf(", \"c2\": ");
    pa(s.c2, 3);
    printf(", \"r\": %.17g, \"mat\": %d, \"albedo\": ", s.r, s.mat);
    pa(s.albedo, 3);
    printf(", \"fuzz\": %.17g, \"ri\": %.17g}%s", s.fuzz, s.ri, i + 1 < g_book1.size() ? ", " : "");
  }
  printf("]},\n");

  // 10. bvh_node traversal order over the book-1 spheres (bvh_node.hpp:25-94): per ray, the
  //     sequence of object ids whose hit() the reference calls, and the closest t.
  {
    std::vector<int> log;
    hittable_list lw;
    for (size_t i = 0; i < w.objects.size(); ++i)
      lw.add(std::make_shared<logged>((int)i, w.objects[i], &log));
    bvh_node root(lw);
    aabb rb = root.bounding_box();
    printf("\"book1_bvh\": {\"root_box\": [%.17g, %.17g, %.17g, %.17g, %.17g, %.17g], \"rays\": [",
           rb.x.min, rb.y.min, rb.z.min, rb.x.max, rb.y.max, rb.z.max);
    for (int k = 0; k < 160; ++k) {
      point3 o(kat_r(6, 14), kat_r(0.5, 4), kat_r(-4, 5));
      point3 tg(kat_r(-11, 11), kat_r(-0.5, 1.5), kat_r(-11, 11));
      vec3 d = tg - o;
      double time = kat_u();
      log.clear();
      hit_record rec;
      bool h = root.hit(ray(o, d, time), interval(0.001, infinity), rec);
      printf("{");
      pv("o", o);
      pv("d", d);
      pj("time", time);
      printf("\"hit\": %d, \"t\": %.17g, \"order\": [", h ? 1 : 0, h ? rec.t : -1.0);
      for (size_t i = 0; i < log.size(); ++i) printf("%d%s", log[i], i + 1 < log.size() ? ", " : "");
      printf("]}%s", k < 159 ? ", " : "");
    }
    printf("]}\n");
  }
  printf("}\n");
  return 0;
}

static int render_mode(const std::string& scene, int W, int H, int spp, int depth, unsigned seed,
                       const char* outpath) {
  srand(1);
  std::shared_ptr<hittable> world = make_world(scene);
  cam_t c;
  setup_cam(scene, c);
  c.image_width = W;
  c.aspect_ratio = static_cast<double>(W) / H;
  c.samples_per_pixel = spp;
  c.max_depth = depth;
  c.initialize();
  std::vector<double> fb(static_cast<size_t>(c.image_width) * c.image_height * 3);
  srand(seed);  // the render stream starts at the given seed (ref-hybrid)
  auto t0 = std::chrono::steady_clock::now();
  c.render(*world, 0, c.image_height, fb.data());
  double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  FILE* f = fopen(outpath, "wb");
  if (!f) return 1;
  fwrite(fb.data(), sizeof(double), fb.size(), f);
  fclose(f);
  printf("{\"width\": %d, \"height\": %d, \"segments\": %llu, \"seconds\": %.6f}\n", c.image_width,
         c.image_height, c.segments, sec);
  return 0;
}

// N processes, each renders every N-th row of the image with its own seed. ROWSTEP > 1 renders
// only rows 0, ROWSTEP, 2*ROWSTEP, ... (a bounded sample of the frame spread over its height).
static int bench_mode(const std::string& scene, int W, int H, int spp, int depth, int procs, int rowstep) {
  if (rowstep < 1) rowstep = 1;
  srand(1);
  std::shared_ptr<hittable> world = make_world(scene);
  std::vector<int> fds(procs);
  std::vector<pid_t> pids(procs);
  auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < procs; ++k) {
    int p[2];
    if (pipe(p) != 0) return 1;
    pid_t pid = fork();
    if (pid == 0) {
      close(p[0]);
      cam_t c;
      setup_cam(scene, c);
      c.image_width = W;
      c.aspect_ratio = static_cast<double>(W) / H;
      c.samples_per_pixel = spp;
      c.max_depth = depth;
      c.initialize();
      srand(1000 + k);
      std::vector<double> row(static_cast<size_t>(W) * 3);
      for (int j = k * rowstep; j < c.image_height; j += procs * rowstep) c.render(*world, j, 1, row.data());
      unsigned long long s = c.segments;
      if (write(p[1], &s, sizeof(s)) != (ssize_t)sizeof(s)) _exit(1);
      _exit(0);
    }
    close(p[1]);
    fds[k] = p[0];
    pids[k] = pid;
  }
  unsigned long long total = 0;
  for (int k = 0; k < procs; ++k) {
    unsigned long long s = 0;
    if (read(fds[k], &s, sizeof(s)) != (ssize_t)sizeof(s)) return 1;
    total += s;
    close(fds[k]);
    waitpid(pids[k], nullptr, 0);
  }
  double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("{\"segments\": %llu, \"seconds\": %.6f, \"procs\": %d, \"mrays_per_s\": %.6f}\n", total,
         sec, procs, total / sec / 1e6);
  return 0;
}

// G5: PROCS processes each render the whole image at SPP samples per pixel from their own
// srand(SEED0 + k) stream and return per-pixel moments (sum L, sum L^2, per channel); the parent
// writes their sum, (H, W, 6) doubles, to OUT. Every pixel then carries PROCS*SPP independent
// samples of the reference's estimator.
static int moments_mode(const std::string& scene, int W, int H, int spp, int depth, int procs,
                        unsigned seed0, const char* outpath) {
  srand(1);
  std::shared_ptr<hittable> world = make_world(scene);
  cam_t c0;
  setup_cam(scene, c0);
  c0.image_width = W;
  c0.aspect_ratio = static_cast<double>(W) / H;
  c0.samples_per_pixel = spp;
  c0.max_depth = depth;
  c0.initialize();
  const size_t n = static_cast<size_t>(c0.image_width) * c0.image_height * 6;
  const std::string base(outpath);
  std::vector<pid_t> pids(procs);
  for (int k = 0; k < procs; ++k) {
    pid_t pid = fork();
    if (pid == 0) {
      cam_t c = c0;
      srand(seed0 + k);
      std::vector<double> m(n, 0.0);
      c.render_moments(*world, m.data());
      FILE* f = fopen((base + ".part" + std::to_string(k)).c_str(), "wb");
      if (!f || fwrite(m.data(), sizeof(double), n, f) != n) _exit(1);
      fclose(f);
      printf("%llu\n", c.segments);
      fflush(stdout);
      _exit(0);
    }
    pids[k] = pid;
  }
  std::vector<double> sum(n, 0.0), part(n);
  for (int k = 0; k < procs; ++k) {
    int status = 0;
    waitpid(pids[k], &status, 0);
    if (!WIFEXITED(status) || WEXITSTATUS(status) != 0) return 1;
    const std::string p = base + ".part" + std::to_string(k);
    FILE* f = fopen(p.c_str(), "rb");
    if (!f || fread(part.data(), sizeof(double), n, f) != n) return 1;
    fclose(f);
    remove(p.c_str());
    for (size_t i = 0; i < n; ++i) sum[i] += part[i];
  }
  FILE* f = fopen(outpath, "wb");
  if (!f) return 1;
  fwrite(sum.data(), sizeof(double), n, f);
  fclose(f);
  printf("{\"width\": %d, \"height\": %d, \"samples_per_pixel\": %d}\n", c0.image_width, c0.image_height,
         spp * procs);
  return 0;
}

// G1': the bouncing_spheres records of grid half-width GRID (main.cpp:12-76 with the loop bounds
// generalised), from the default seed-1 stream, as (N, 13) doubles: c1[3] c2[3] r mat albedo[3]
// fuzz ri (mat: 0 ground checker, 1 lambertian, 2 metal, 3 dielectric).
static int records_mode(int grid, const char* outpath) {
  srand(1);
  g_book1.clear();
  book1_world(grid, true);
  FILE* f = fopen(outpath, "wb");
  if (!f) return 1;
  long counts[4] = {0, 0, 0, 0};
  for (const sphere_rec& s : g_book1) {
    const double row[13] = {s.c1[0], s.c1[1], s.c1[2], s.c2[0], s.c2[1], s.c2[2], s.r, double(s.mat),
                            s.albedo[0], s.albedo[1], s.albedo[2], s.fuzz, s.ri};
    fwrite(row, sizeof(double), 13, f);
    counts[s.mat]++;
  }
  fclose(f);
  printf("{\"records\": %zu, \"ground\": %ld, \"lambertian\": %ld, \"metal\": %ld, \"dielectric\": %ld}\n",
         g_book1.size(), counts[0], counts[1], counts[2], counts[3]);
  return 0;
}


// ------------------------------------------------------------------------------------------
// ties: the winner of exactly equal-t hits through the reference's own hittable_list, bvh_node,
// sphere and quad. The world holds groups of identical spheres, static spheres
// with a moving twin that coincides at time 0, coplanar quads of different extents and two compound
// children (hittable_lists of two quads) in the same plane, plus background spheres; every object has
// its own material, so rec.mat names the winner. Rays leave (0, 0, 30) at time 0 (and a few at 0.37)
// toward the tie regions. It is rendered as a plain hittable_list ("list": the list rule) and as
// hittable_list(bvh_node(list)) as main.cpp:76 wraps book-1 ("bvh": the median tree's leaf order).
// scenes/scenes.hpp tie_world builds the same objects with the C++ mirror; tests/golden/ties.json pins
// the oracle's tie rule (with the mirror's tie ranks) to these winners.
struct tie_obj {
  int kind;  // 1 sphere, 2 quad
  point3 c0, c1;
  double r;
  point3 Q;
  vec3 u, v;
};
static int ties_mode() {
  std::vector<tie_obj> prims;                       // flattened, list order
  std::vector<std::shared_ptr<material>> mats;      // one per primitive
  hittable_list objs;                               // the top-level children
  std::vector<int> child_prims;                     // primitives per child
  auto mat = [&]() {
    const double k = static_cast<double>(mats.size());
    mats.push_back(std::make_shared<diffuse_light>(color(0.1 + 0.02 * k, 1.0 - 0.02 * k, 0.5)));
    return mats.back();
  };
  auto sph = [&](point3 c0, point3 c1, double r) -> std::shared_ptr<hittable> {
    prims.push_back(tie_obj{1, c0, c1, r, point3(), vec3(), vec3()});
    if (c0.x() == c1.x() && c0.y() == c1.y() && c0.z() == c1.z()) return std::make_shared<sphere>(c0, r, mat());
    return std::make_shared<sphere>(c0, c1, r, mat());
  };
  auto qd = [&](point3 Q, vec3 u, vec3 v) -> std::shared_ptr<hittable> {
    prims.push_back(tie_obj{2, point3(), point3(), 0.0, Q, u, v});
    return std::make_shared<quad>(Q, u, v, mat());
  };
  for (int m = 0; m < 4; ++m)  // 4 groups of 4 identical spheres, the list interleaving the groups
    for (int g = 0; g < 4; ++g) {
      const point3 c(-9.0 + 6.0 * g, 4.0, 0.0);
      objs.add(sph(c, c, 1.5));
      child_prims.push_back(1);
    }
  for (int g = 0; g < 4; ++g) {  // a static sphere, then its moving twin (centre at time 0 the same)
    const point3 c(-9.0 + 6.0 * g, -4.0, 0.0);
    objs.add(sph(c, c, 1.5));
    objs.add(sph(c, c + vec3(g % 2 ? 3.0 : -3.0, 0.0, 0.0), 1.5));
    child_prims.push_back(1);
    child_prims.push_back(1);
  }
  for (int k = 0; k < 4; ++k) {  // coplanar quads in z = 3, box minima x = -2, -4, -6, -8
    objs.add(qd(point3(-2.0 - 2.0 * k, -1.0, 3.0), vec3(4.0 + 4.0 * k, 0.0, 0.0), vec3(0.0, 2.0, 0.0)));
    child_prims.push_back(1);
  }
  for (int j = 0; j < 2; ++j) {  // two identical compound children, in the same plane
    auto pane = std::make_shared<hittable_list>();
    pane->add(qd(point3(5.0, -1.0, 3.0), vec3(4.0, 0.0, 0.0), vec3(0.0, 2.0, 0.0)));
    pane->add(qd(point3(5.0, -1.0, 3.0), vec3(2.0, 0.0, 0.0), vec3(0.0, 1.0, 0.0)));
    objs.add(pane);
    child_prims.push_back(2);
  }
  for (int k = 0; k < 8; ++k) {  // background
    const point3 c(-14.0 + 4.0 * k, k % 2 ? -8.0 : 8.0, -6.0);
    objs.add(sph(c, c, 1.0));
    child_prims.push_back(1);
  }
  // rays
  std::vector<ray> rays;
  const point3 o(0.0, 0.0, 30.0);
  auto toward = [&](double x, double y, double z, double t) { rays.push_back(ray(o, point3(x, y, z) - o, t)); };
  for (int row = 0; row < 2; ++row)
    for (int g = 0; g < 4; ++g)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) toward(-9.0 + 6.0 * g + 0.5 * dx, (row ? -4.0 : 4.0) + 0.5 * dy, 0.0, 0.0);
  for (int g = 0; g < 4; ++g) toward(-9.0 + 6.0 * g + 0.25, -4.0 + 0.25, 0.0, 0.375);
  const double qx[] = {-7.5, -5.5, -3.5, -1.5, 0.0, 1.5, 3.5, 5.25, 5.5, 6.5, 7.5, 8.5};
  for (double x : qx)
    for (double y : {-0.5, 0.25}) toward(x, y, 3.0, 0.0);
  toward(0.0, 20.0, 0.0, 0.0);  // a miss
  hittable_list plain = objs;
  hittable_list tree(std::make_shared<bvh_node>(objs));
  std::map<const material*, int> who;
  for (size_t i = 0; i < mats.size(); ++i) who[mats[i].get()] = static_cast<int>(i);
  printf("{\"objects\": [");
  for (size_t i = 0; i < prims.size(); ++i) {
    const tie_obj& p = prims[i];
    printf("%s{", i ? ", " : "");
    if (p.kind == 1) {
      printf("\"kind\": \"sphere\", ");
      pv("c0", p.c0);
      pv("c1", p.c1);
      pj("r", p.r, false);
    } else {
      printf("\"kind\": \"quad\", ");
      pv("Q", p.Q);
      pv("u", p.u);
      pv("v", p.v, false);
    }
    printf("}");
  }
  printf("], \"child_prims\": [");
  for (size_t i = 0; i < child_prims.size(); ++i) printf("%s%d", i ? ", " : "", child_prims[i]);
  printf("], \"rays\": [");
  for (size_t k = 0; k < rays.size(); ++k) {
    printf("%s{", k ? ", " : "");
    pv("o", rays[k].origin());
    pv("d", rays[k].direction());
    pj("time", rays[k].time(), false);
    printf("}");
  }
  printf("]");
  const hittable* worlds[2] = {&plain, &tree};
  const char* names[2] = {"list", "bvh"};
  for (int w = 0; w < 2; ++w) {
    printf(", \"%s\": {\"winner\": [", names[w]);
    std::vector<double> ts;
    for (size_t k = 0; k < rays.size(); ++k) {
      hit_record rec;
      const bool h = worlds[w]->hit(rays[k], interval(0.001, infinity), rec);  // camera.hpp:192
      printf("%s%d", k ? ", " : "", h ? who.at(rec.mat.get()) : -1);
      ts.push_back(h ? rec.t : -1.0);
    }
    printf("], \"t\": ");
    pa(ts.data(), static_cast<int>(ts.size()));
    printf("}");
  }
  printf("}\n");
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && std::string(argv[1]) == "golden") return golden();
  if (argc >= 2 && std::string(argv[1]) == "ties") return ties_mode();
  if (argc >= 10 && std::string(argv[1]) == "moments")
    return moments_mode(argv[2], atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), atoi(argv[6]), atoi(argv[7]),
                        (unsigned)strtoul(argv[8], nullptr, 10), argv[9]);
  if (argc >= 4 && std::string(argv[1]) == "records") return records_mode(atoi(argv[2]), argv[3]);
  if (argc >= 9 && std::string(argv[1]) == "render")
    return render_mode(argv[2], atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), atoi(argv[6]),
                       (unsigned)strtoul(argv[7], nullptr, 10), argv[8]);
  if (argc >= 8 && std::string(argv[1]) == "bench")
    return bench_mode(argv[2], atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), atoi(argv[6]),
                      atoi(argv[7]), argc >= 9 ? atoi(argv[8]) : 1);
  fprintf(stderr,
          "usage: ref_harness golden | render SCENE W H SPP DEPTH SEED OUT | bench SCENE W H SPP DEPTH PROCS [ROWSTEP]\n");
  return 2;
}
