// rtgpu/scene_builder.hpp — flattens the C++ object graph (hittable / material / texture, all
// shared_ptr-linked as in the reference) into the flat arrays of rtg_scene_desc (include/rtgpu.h).
// Materials, textures, images and perlin tables are de-duplicated by object identity, so a
// texture shared by many spheres (e.g. main.cpp:180-183) is uploaded once.
#pragma once
#include <cstdint>
#include <unordered_map>
#include <memory>
#include <string>
#include <vector>

#include "rtgpu.h"

class material;
class texture;

namespace rtgpu {

class scene_builder {
 public:
  std::vector<rtg_primitive> prims;
  std::vector<rtg_material> materials;
  std::vector<rtg_texture> textures;
  std::vector<rtg_image> images;
  std::vector<std::shared_ptr<const std::vector<uint8_t>>> image_bytes;
  std::vector<rtg_perlin> perlins;
  // Exact-t tie order (rtg_scene_desc.tie_rank, ABI 7): per primitive its position in the order the
  // reference's closest-hit walk tests it. Empty while that is the primitive order (hittable_list order);
  // a bvh_node's flatten permutes its own range into its median tree's leaf order (bvh_node.hpp:80-94).
  std::vector<int64_t> tie_rank;
  std::string error;

  // identity ranks for the primitives [tie_rank.size(), n) (before a bvh_node permutes a range)
  void extend_ranks(size_t n) {
    tie_rank.reserve(n);
    for (size_t i = tie_rank.size(); i < n; ++i) tie_rank.push_back(static_cast<int64_t>(i));
  }

  // Index of the flattened material / texture (exports on first use); -1 on failure.
  int32_t material_id(const material* m);  // defined in core/material.hpp
  int32_t texture_id(const texture* t);    // defined in core/texture.hpp
  enum memo_kind { kMaterial = 0, kTexture = 1, kImage = 2, kPerlin = 3 };

  int32_t image_id(const void* key, int w, int h, std::shared_ptr<const std::vector<uint8_t>> rgb) {
    auto& memo = memo_table(kImage);
    auto it = memo.find(key);
    if (it != memo.end()) return it->second;
    rtg_image im{w, h, rgb ? rgb->data() : nullptr};
    images.push_back(im);
    image_bytes.push_back(rgb);
    return memo[key] = static_cast<int32_t>(images.size() - 1);
  }
  int32_t perlin_id(const void* key, const rtg_perlin& p) {
    auto& memo = memo_table(kPerlin);
    auto it = memo.find(key);
    if (it != memo.end()) return it->second;
    perlins.push_back(p);
    return memo[key] = static_cast<int32_t>(perlins.size() - 1);
  }
  // Capacity for `n` more objects (each may bring a material and a texture of its own, as config 5's
  // 1M spheres do): one allocation per array and no rehashing while a large list flattens.
  void reserve(size_t n) {
    if (n < 1024) return;
    prims.reserve(prims.size() + n);
    materials.reserve(materials.size() + n);
    textures.reserve(textures.size() + n);
    memo_[kMaterial].reserve(memo_[kMaterial].size() + n);
    memo_[kTexture].reserve(memo_[kTexture].size() + n);
  }
  bool fail(const std::string& what) {
    if (error.empty()) error = what;
    return false;
  }
  // identity -> index table, one per exported object kind (hashed: config 5 flattens 1M materials)
  std::unordered_map<const void*, int32_t>& memo_table(memo_kind k) { return memo_[k]; }

  rtg_scene_desc desc(int32_t bvh_mode) {
    if (!tie_rank.empty()) extend_ranks(prims.size());
    rtg_scene_desc d{};
    d.abi_version = RTG_ABI_VERSION;
    d.bvh_mode = bvh_mode;
    d.prims = prims.data();
    d.num_prims = static_cast<int64_t>(prims.size());
    d.materials = materials.data();
    d.num_materials = static_cast<int32_t>(materials.size());
    d.textures = textures.data();
    d.num_textures = static_cast<int32_t>(textures.size());
    d.images = images.data();
    d.num_images = static_cast<int32_t>(images.size());
    d.perlins = perlins.data();
    d.num_perlins = static_cast<int32_t>(perlins.size());
    d.tie_rank = tie_rank.empty() ? nullptr : tie_rank.data();
    return d;
  }

 private:
  std::unordered_map<const void*, int32_t> memo_[4];
};

}  // namespace rtgpu
