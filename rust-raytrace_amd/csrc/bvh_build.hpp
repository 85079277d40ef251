// Host-side sphere BVH builder (host_bvh.cpp).
#pragma once

#include <cstddef>
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

// Spheres (centre, radius); `pad` widens every box before f32 outward rounding;
// leaves hold at most `leaf_max` (1..8) spheres.
BvhResult build_sphere_bvh(const std::vector<double>& cx, const std::vector<double>& cy, const std::vector<double>& cz,
                           const std::vector<double>& radius, double pad, int leaf_max);

// 4-wide BVH collapsed from a binary one (same leaves, same f32 boxes), in
// the device's plane-major layout (device_layout.hpp, DevBvh4): plane k of
// node i at planes[k * n_nodes + i].
struct Bvh4Result {
    std::vector<DevBvh4Plane> planes;   // kBvh4Planes * n_nodes
    int32_t n_nodes = 0;
    int32_t root = 0;                   // encoded pointer, as in DevBvhNode
};
Bvh4Result collapse_bvh4(const BvhResult& b2);

// Worst-case traversal stack depth of a 4-wide tree: the largest sum, over
// the nodes of a root-to-leaf path, of (children - 1) pending siblings, + 1.
int bvh4_stack_need(const Bvh4Result& b4);
// Depth of a binary tree (its traversal pushes at most one entry per level).
int bvh_depth(const BvhResult& b2);

// The binary tree's nodes with binary16 bounds rounded outward (DevBvhNodeH);
// empty when some bound is not finite or lies outside the half range.
std::vector<DevBvhNodeH> half_nodes(const BvhResult& b2);
// binary16 helpers (exact decode; the largest half <= v / smallest half >= v)
float half_to_float(uint16_t h);
bool half_round_down(float v, uint16_t& out);
bool half_round_up(float v, uint16_t& out);

// The 4-wide tree with 8-bit child bounds in a per-node frame (DevQNode4),
// every decoded box containing the f32 child box; empty when some bound is not
// finite or too large, a node's leaf children lie more than 4094 spheres apart,
// the tree has 32768 nodes or more, or the root is a leaf.
std::vector<DevQNode4> quantize_bvh4(const Bvh4Result& b4);

}  // namespace rtamd

namespace rtamd {

// Light-view grids for point-light shadow queries (host_lightgrid.cpp,
// DESIGN.md "Light-view grids").  Per point light: a cube map of R x R cells
// per face around the light; cell c lists every sphere whose padded box has a
// point whose direction from the light falls in c (a conservative superset),
// sorted by the box's distance from the light.  `r_leaf` are the radii and
// `spheres` the centres in leaf order (the indices the lists hold).
struct LightGridResult {
    std::vector<DevLightGrid> grids;    // one per light (R = 0: no grid, e.g. not a point light)
    std::vector<uint32_t> off;          // cell offsets into ent (per face rect: w * h + 1)
    std::vector<DevLgEntry> ent;
};
LightGridResult build_light_grids(const std::vector<DevSphere>& spheres, const std::vector<double>& r_leaf,
                                  const std::vector<DevLight>& lights, double pad, int r_override);
// The camera's view grid (the same cube-map layout, one grid centred on `pos`)
// for the camera rays' nearest-hit query; R halves until the lists hold at
// most max_entries entries.
LightGridResult build_view_grid(const std::vector<DevSphere>& spheres, const std::vector<double>& r_leaf,
                                const double pos[3], double pad, int R, size_t max_entries);
// Host mirror of the device's candidate list (test / diagnostic).
bool light_grid_candidates(const LightGridResult& lg, int light, const double p[3], std::vector<int32_t>& out);

}  // namespace rtamd
