// rt_bvh.h -- sphere BVH shared by the host builder (rt_bvh.cpp) and the
// device traversal (rt_device.h).
//
// Stackless layout ("skip pointers"): nodes in depth-first preorder; a node's
// first child is the next node, `skip` is the first node after its subtree.
// Boxes are fp32, rounded outward from the fp64 sphere bounds [c - |r|, c + |r|];
// the traversal adds a scene-scale margin at run time (see rt_device.h), so a
// box test never rejects a sphere the reference's fp64 test could report.
#pragma once
#include <cstddef>
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

// Behind grid: a uniform grid of sphere lists for the part of a closest-hit
// line BEHIND the ray origin.  There the reference's test (sphere.h:26-59) can
// only report the negative tangent root (disc == 0, sphere.h:43-47) -- any
// other root of a sphere wholly behind the origin is negative and discarded --
// so the ordered walks skip boxes wholly behind the origin when this grid
// exists, and the device visits the cells along the backward half-line instead
// (rt_device.h behind_cells), testing every listed sphere exactly.  Cells are
// cubes of edge cs from the origin (gx, gy, gz) (coordinates relative to the
// BVH centre c0, fp32); a sphere is listed in every cell its box grown by
// reg_margin meets.  Spheres of radius above 2 cells (a ground sphere) are not
// listed but in `glob`, tested for every line.  Cell (x, y, z) = k in
// [start[c], start[c + 1]), c = (z * ny + y) * nx + x.
// The device reads a cell as one 64-B record of four slots (UgRec: centre -
// c0 and |radius| rounded up, fp32; w = -1: no further entry; a cell with more
// than four entries keeps three and, in slot 3, w = -2 and the bit patterns
// of [k0, k1): its remaining entries q[k], ids[k] of the overflow list); rid
// holds the slots' sphere ids.
struct UgRec {
  float x, y, z, w;
};
struct UgridHost {
  float gx = 0, gy = 0, gz = 0, cs = 0;
  int nx = 0, ny = 0, nz = 0;
  float reg_margin = 0;  // listing margin (>= the device's prefilter margin + DDA error, checked per launch)
  float extent = 0;      // largest edge of the grid (the DDA error scale)
  std::vector<int32_t> start, ids, glob;  // CSR lists (ids: every entry, in cell order)
  std::vector<UgRec> rec;                  // [cell][4]
  std::vector<int32_t> rid;                // [cell][4]
  std::vector<UgRec> q;                    // per CSR entry (the overflow lists index it)
};
// Builds the grid over spheres (centres relative to c0, radii r), about
// cells_per_sphere cells per listed sphere; false (no grid) for an empty
// scene, non-finite values, more than 64 global spheres or more than
// max_entries list entries.
bool build_ugrid(const double *cx, const double *cy, const double *cz, const double *r, int n, size_t max_entries,
                 UgridHost &out, double cells_per_sphere = 2.0);

}  // namespace rtk
