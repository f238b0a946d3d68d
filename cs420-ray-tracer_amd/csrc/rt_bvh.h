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

// Two-child node for ordered (near-first) traversal: both children's boxes
// in one 64-B record.  Child reference c >= 0: internal node c of this array;
// c < 0: leaf -(c + 1) = (first << 4) | count, as BvhNode::leaf.
struct BvhNode2 {  // 64 B
  float lo0[3], hi0[3], lo1[3], hi1[3];
  int32_t c0, c1;
  int32_t pad[2];
};

// Four-child node for the ordered 4-wide walk: the grandchildren of a binary
// node (a leaf child stands for itself), boxes in SoA order so child k's slab
// test reads lox[k] .. hiz[k].  Unused slots have NaN boxes (every slab
// comparison with them is false, so they are never entered).  Child
// references as BvhNode2 (>= 0: internal node of this array, < 0: leaf).
struct BvhNode4 {  // 128 B
  float lox[4], loy[4], loz[4], hix[4], hiy[4], hiz[4];
  int32_t c[4];
  int32_t pad[4];
};

// Derives the two-child layout from the preorder one; returns the root's
// reference (a leaf reference when the whole tree is one leaf) and the tree
// depth (the most far-children an ordered walk can have pending).
int32_t build_bvh2(const std::vector<BvhNode> &nodes, std::vector<BvhNode2> &out, int &depth);

// Derives the four-child layout; returns the root's reference and, in
// `stack`, the most entries an ordered 4-wide walk can have pending (the
// largest sum over a root-to-leaf path of (children - 1) per node).
int32_t build_bvh4(const std::vector<BvhNode> &nodes, std::vector<BvhNode4> &out, int &stack);

// Builds the BVH over spheres (centres cx,cy,cz, radii r).  `prims` receives
// the sphere indices in leaf order.  Leaves hold at most `max_leaf` (<= 15)
// spheres; depth is unlimited (the traversal is stackless).
void build_bvh(const double *cx, const double *cy, const double *cz, const double *r, int n, int max_leaf,
               std::vector<BvhNode> &nodes, std::vector<int32_t> &prims);

}  // namespace rtk
