// Host-side sphere BVH builder (host_bvh.cpp).
#pragma once

#include <cstdint>
#include <vector>

#include "device_layout.hpp"

namespace rtamd {

using BvhNodeHost = DevBvhNode;

struct BvhResult {
    std::vector<BvhNodeHost> nodes;
    std::vector<int32_t> order;     // order[k] = input index of the k-th sphere in leaf order
    int32_t root = 0;               // encoded pointer (node index, or ~leaf when the whole set is one leaf)
};

// Spheres (centre, radius); `pad` widens every box before f32 outward rounding.
BvhResult build_sphere_bvh(const std::vector<double>& cx, const std::vector<double>& cy, const std::vector<double>& cz,
                           const std::vector<double>& radius, double pad);

}  // namespace rtamd
