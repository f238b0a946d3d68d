// rt_bvh.h -- sphere BVH shared by the host builder (rt_bvh.cpp) and the
// device traversal (rt_device.h).
//
// Stackless layout ("skip pointers"): nodes in depth-first preorder; a node's
// first child is the next node, `skip` is the first node after its subtree.
// Boxes are fp32, rounded outward from the fp64 sphere bounds [c - |r|, c + |r|];
// the traversal adds a scene-scale margin at run time (see rt_device.h), so a
// box test never rejects a sphere the reference's fp64 test could report.
#pragma once
#include <cstdint>
#include <vector>

namespace rtk {

struct BvhNode {  // 32 B
  float lo[3];
  int32_t skip;   // index of the node after this subtree (== node count at the end)
  float hi[3];
  int32_t leaf;   // leaf: (first << 4) | count (count 1..15); internal: -1
};

// Builds the BVH over spheres (centres cx,cy,cz, radii r).  `prims` receives
// the sphere indices in leaf order.  Leaves hold at most `max_leaf` (<= 15)
// spheres; depth is unlimited (the traversal is stackless).
void build_bvh(const double *cx, const double *cy, const double *cz, const double *r, int n, int max_leaf,
               std::vector<BvhNode> &nodes, std::vector<int32_t> &prims);

}  // namespace rtk
