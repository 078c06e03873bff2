// core/rtw_stb_image.hpp — image loader behind image_texture (rtw_stb_image.hpp:28-178).
//
// The reference decodes with stb_image (fetched at configure time, not vendored; absent here),
// whose stbi_loadf() maps each 8-bit sRGB byte b to pow(b/255, 2.2) before convert_to_bytes()
// quantises it back with float_to_byte(). This mirror reads images that are already decoded to
// 8-bit sRGB as binary/ASCII PPM (P6/P3): a path that names a PPM is read directly, any other
// name (e.g. "earthmap.jpg") is looked up as "<stem>.ppm" next to it. The same byte -> float ->
// byte conversion is then applied, so the texels equal the reference's for the same decoded bytes.
#pragma once
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <memory>
#include <string>
#include <vector>

class rtw_image {
 public:
  rtw_image() {}
  explicit rtw_image(const char* image_filename) {
    const std::string name(image_filename);
    if (const char* dir = std::getenv("RTW_IMAGES"))
      if (load(std::string(dir) + "/" + name)) return;
    std::string prefix;
    if (load(name)) return;
    for (int up = 0; up < 7; ++up) {
      if (load(prefix + "images/" + name)) return;
      prefix += "../";
    }
    std::cerr << "ERROR: Could not load image file '" << image_filename << "'.\n";
  }

  bool load(const std::string& filename) {
    if (read_ppm(filename)) return true;
    const size_t dot = filename.find_last_of('.');
    if (dot != std::string::npos && filename.substr(dot) != ".ppm")
      return read_ppm(filename.substr(0, dot) + ".ppm");
    return false;
  }

  int width() const { return bdata ? image_width : 0; }
  int height() const { return bdata ? image_height : 0; }

  const unsigned char* pixel_data(int x, int y) const {
    static unsigned char magenta[] = {255, 0, 255};
    if (!bdata) return magenta;
    x = clamp(x, 0, image_width);
    y = clamp(y, 0, image_height);
    return bdata->data() + y * bytes_per_scanline + x * bytes_per_pixel;
  }

  // converted RGB8 texels (extension: shared with the device scene)
  std::shared_ptr<const std::vector<unsigned char>> bytes() const { return bdata; }

 private:
  static const int bytes_per_pixel = 3;
  std::shared_ptr<std::vector<unsigned char>> bdata;
  int image_width = 0, image_height = 0, bytes_per_scanline = 0;

  static int clamp(int x, int low, int high) { return x < low ? low : (x < high ? x : high - 1); }

  static unsigned char float_to_byte(float value) {
    if (value <= 0.0f) return 0;
    if (value >= 1.0f) return 255;
    return static_cast<unsigned char>(256.0f * value);
  }
  // stbi__ldr_to_hdr (gamma 2.2, scale 1) followed by float_to_byte
  static unsigned char srgb_byte_to_texel(unsigned char b) {
    const float f = static_cast<float>(std::pow(b / 255.0f, 2.2f) * 1.0f);
    return float_to_byte(f);
  }

  bool read_ppm(const std::string& path) {
    std::ifstream in(path, std::ios::binary);
    if (!in) return false;
    std::string magic;
    in >> magic;
    if (magic != "P6" && magic != "P3") return false;
    auto next_int = [&in](int& v) {
      for (;;) {
        in >> std::ws;
        if (in.peek() == '#') {
          std::string line;
          std::getline(in, line);
          continue;
        }
        return static_cast<bool>(in >> v);
      }
    };
    int w = 0, h = 0, maxv = 0;
    if (!next_int(w) || !next_int(h) || !next_int(maxv) || w <= 0 || h <= 0 || maxv != 255) return false;
    auto data = std::make_shared<std::vector<unsigned char>>(static_cast<size_t>(w) * h * 3);
    if (magic == "P6") {
      in.get();  // single whitespace after maxval
      in.read(reinterpret_cast<char*>(data->data()), static_cast<std::streamsize>(data->size()));
      if (in.gcount() != static_cast<std::streamsize>(data->size())) return false;
    } else {
      for (auto& b : *data) {
        int v;
        if (!next_int(v)) return false;
        b = static_cast<unsigned char>(v);
      }
    }
    unsigned char lut[256];
    for (int b = 0; b < 256; ++b) lut[b] = srgb_byte_to_texel(static_cast<unsigned char>(b));
    for (auto& b : *data) b = lut[b];
    bdata = data;
    image_width = w;
    image_height = h;
    bytes_per_scanline = w * bytes_per_pixel;
    return true;
  }
};
