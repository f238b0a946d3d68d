// rt_device.h -- device-side math shared by every render pipeline in
// rt_kernel.hip: Vec3 algebra, the exact ray-sphere test, the wave-level
// conservative cull and the closest-hit / shadow sweeps.  Numerics follow the
// reference's serial fp64 path operation by operation.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "rt_bvh.h"
#include "rt_lightgrid.h"
#include "rt_pow.h"

#pragma clang fp contract(off)

namespace rtk {

constexpr double kEps = 0.001;  // ray_math_constants.h:22
constexpr double kInf = 1e20;   // ray_math_constants.h:23
constexpr double kSpec = 0.5;   // scene.h:38
constexpr int kBlock = 256;
constexpr size_t kLdsBudget = 64 * 1024;
constexpr int kCounters = 6;  // primary, shadow, reflect, negative, exact tests, cull tests
// Statistics counters are sharded: 64 copies, 256 B apart, picked by workgroup
// id.  A single contended word serialises device atomics (~88/us, MI355X
// microarch "dequeue" row); the host sums the shards.
constexpr int kShards = 64;
constexpr int kShardStride = 32;  // u64 per shard (256 B)
__device__ __forceinline__ unsigned long long *counter_shard(unsigned long long *counters) {
  const unsigned wg = blockIdx.x + blockIdx.y * gridDim.x;
  return counters + (size_t)(wg % kShards) * kShardStride;
}

// ---------------------------------------------------------------------------
// Bounds-checked build (-DRT_CHECK: variants/librt_hip_check.so; SURVEY 5's
// "HIP bounds-checked debug build").  RT_CK(site, i, bound) is `i` itself in
// every other build.  In the checked build each index the kernels take out
// of a host-built structure -- grid CSR starts and list ids, uniform-grid
// cells, records and overflow lists, BVH node references and leaf slots, the
// tile order, deferred-queue and reflection-stack slots, LDS queue and
// pixel-buffer slots -- is compared with the size of what it indexes.  A
// violation is recorded (the first one's site, index and bound, and a count)
// and the access goes to element 0 instead, so the launch still drains and
// rt_render_stats returns RT_ERR_CHECK naming the site, rather than the
// queue faulting or a pixel coming out silently wrong.
enum CkSite {
  kCkSphere = 1,  // a sphere index from a list, grid, leaf or hit (geometry, material)
  kCkLgStart,     // light grid: CSR start of (light, cell)
  kCkLgId,        // light grid: list slot
  kCkCgStart,     // camera grid: CSR start of a cell
  kCkCgEnt,       // camera / sphere grid: list slot
  kCkSgStart,     // sphere grid: CSR start of (grid, cell)
  kCkSgKey,       // sphere grid: the sphere a reflection ray leaves
  kCkUgCell,      // uniform grid: cell record
  kCkUgOver,      // uniform grid: overflow-list slot
  kCkBvhNode,     // BVH node reference
  kCkBvhLeaf,     // BVH leaf slot (prefilter record, sphere id)
  kCkTile,        // tile order slot / tile id
  kCkDeferQ,      // deferred-queue slot
  kCkStack,       // reflection-stack slot
  kCkLdsQueue,    // merge_tiles' LDS ray-queue slot
  kCkPixbuf,      // merge_tiles' LDS finished-pixel slot
  kCkOut,         // framebuffer byte offset of a tile row or deferred pixel
  kCkCgBuild,     // camera-grid build: disk, (disk, block) pair, cell count and list slot
  kCkHome,        // stack-home pool: no free home after kHomeSweeps sweeps of its bitmap
  kCkSites
};
#ifdef RT_CHECK
struct CheckRec {
  unsigned long long count, site, idx, bound;
};
__device__ CheckRec g_check;
__device__ __attribute__((noinline)) void ck_fail(int site, long long i, long long bound) {
  if (atomicAdd(&g_check.count, 1ull) == 0ull) {  // the first violation names itself
    g_check.site = (unsigned long long)site;
    g_check.idx = (unsigned long long)i;
    g_check.bound = (unsigned long long)bound;
  }
}
template <class I>
__host__ __device__ __forceinline__ I ck(int site, I i, long long bound) {
#ifdef __HIP_DEVICE_COMPILE__
  if (__builtin_expect(!((long long)i >= 0 && (long long)i < bound), 0)) {
    ck_fail(site, (long long)i, bound);
    return (I)0;
  }
#endif
  return i;
}
#define RT_CK(site, i, bound) ::rtk::ck((site), (i), (long long)(bound))
#else
#define RT_CK(site, i, bound) (i)
#endif

struct __attribute__((aligned(32))) SphGeo {
  double cx, cy, cz, rr;  // rr = radius*radius, rounded once on the host as sphere.h:33 does
};
struct SphMat {
  double cr, cg, cb, refl, shin, pad;
};
struct LightD {
  double px, py, pz, cr, cg, cb;
};

struct D3 {
  double x, y, z;
};
// One entry of a pixel's reflection stack (main.cpp:54): A = shade*(1-refl), and refl.
struct StackEnt {  // 32 B
  double ax, ay, az, refl;
};
__device__ __forceinline__ D3 mk(double x, double y, double z) { return D3{x, y, z}; }
__device__ __forceinline__ D3 add(D3 a, D3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ D3 sub(D3 a, D3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ D3 mul(D3 a, D3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ D3 scale(D3 a, double t) { return mk(a.x * t, a.y * t, a.z * t); }
__device__ __forceinline__ double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ double length(D3 a) { return __builtin_sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }

// (a.x / b, a.y / b, a.z / b), bit-identical to three IEEE divisions.  The
// compiler lowers one fp64 division to v_div_scale (x2), v_rcp_f64, two
// Newton steps on the reciprocal, q = x*r, e = fma(-b, q, x), v_div_fmas
// (= fma(e, r, q) when no scaling was applied) and v_div_fixup (only the sign
// and special values).  The reciprocal and its refinement depend on b alone,
// so for three numerators they are computed once.  v_div_scale leaves both
// operands unscaled (and VCC clear) exactly when b is a normal number whose
// reciprocal is normal, x is 0 or neither tiny (exponent <= 53) nor 2^768
// larger than b, and x/b is not subnormal; the guard below is a subset of
// that (b in [2^-300, 2^300], x == 0 or |x| in [2^-600, 2^400]), and for it
// v_div_fixup returns the fma result with the sign of x ^ b = the sign of x
// (so 0/b keeps the sign of the zero).  Anything else -- zero, NaN, infinite
// or extreme operands -- takes the ordinary divisions.
#ifndef RT_FASTDIV
#define RT_FASTDIV 0
#endif

__device__ __forceinline__ bool div_num_ok(double x) {
  const double m = __builtin_fabs(x);
  return x == 0.0 || (m >= 0x1p-600 && m <= 0x1p400);
}
__device__ __forceinline__ D3 div3(D3 a, double b) {
#if RT_FASTDIV
  if (__builtin_expect(b >= 0x1p-300 && b <= 0x1p300 && div_num_ok(a.x) && div_num_ok(a.y) && div_num_ok(a.z), 1)) {
    double r = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    auto one = [&](double x) {
      const double q = x * r;
      const double res = __builtin_fma(-b, q, x);
      return __builtin_copysign(__builtin_fma(res, r, q), x);
    };
    return mk(one(a.x), one(a.y), one(a.z));
  }
#endif
  return mk(a.x / b, a.y / b, a.z / b);
}
__device__ __forceinline__ D3 normalized(D3 a) {
  double len = length(a);
  return div3(a, len);  // vec3.h:26-29: x/len, y/len, z/len
}
// normalized(a), bit-identical, with a fast path for |a| within a few ulps of
// 1 -- the renderer normalises already-normalised directions again (Ray()'s
// constructor, ray.h:12: the camera ray and the shadow direction, scene.h:72)
// and reflections of unit vectors (main.cpp:46).  With u = 2^-53 and
// s = (x*x + y*y) + z*z (length()'s sum, same order), s - 1 is exact near 1
// and s = 1 + t u with t in {-4..0} or {2, 4, 6} (the grid spacing is u below
// 1, 2u above).  sqrt(1 + t u) = 1 + t u / 2 - O(u^2), so the correctly
// rounded length is 1 - ceil(-t/2) u below 1 (an odd -t is a midpoint minus
// the O(u^2) term: it rounds away from 1) and 1 + 2 floor(t/4) u above:
//   t in {0, 2} -> len 1;  {-1, -2} -> 1 - u;  {-3, -4} -> 1 - 2u;  {4, 6} -> 1 + 2u.
// Each quotient x / len is then Markstein's correction with the correctly
// rounded reciprocal rcp = RN(1/len) (1, 1 + 2u, 1 + 2u, 1 - 2u):
// q0 = x rcp, r = fma(-q0, len, x) (exact), q = fma(r, rcp, q0) = RN(x / len)
// -- valid while nothing underflows (|x| >= 2^-959); copysign keeps the sign
// of a zero numerator (x = -0 gives -0, as -0 / len).  Checked against IEEE
// division for 500 M numerators over the exponent range and at binade edges
// and for random, reflected and perturbed vectors (tests/native/renorm_check.cpp).
// Any other length, a tiny component or a NaN takes normalized().
__device__ __forceinline__ D3 renormalized(D3 a) {
  constexpr double u = 0x1p-53;
  const double s = (a.x * a.x + a.y * a.y) + a.z * a.z;
  const double t = (s - 1.0) * 0x1p53;
  auto usable = [](double x) { return __builtin_fabs(x) >= 0x1p-959 || x == 0.0; };
  if (__builtin_expect(t >= -4.0 && t <= 6.0 && usable(a.x) && usable(a.y) && usable(a.z), 1)) {
    const double len = t > 3.0 ? 1.0 + 2.0 * u : (t > -0.5 ? 1.0 : (t > -2.5 ? 1.0 - u : 1.0 - 2.0 * u));
    const double rcp = t > 3.0 ? 1.0 - 2.0 * u : (t > -0.5 ? 1.0 : 1.0 + 2.0 * u);
    auto q = [&](double x) {
      const double q0 = x * rcp;
      return __builtin_copysign(__builtin_fma(__builtin_fma(-q0, len, x), rcp, q0), x);
    };
    return mk(q(a.x), q(a.y), q(a.z));
  }
  return normalized(a);
}

// pow(x, y) outside int_pow's domain -- a shininess that is not a whole number
// in 1..1024 (the parser takes any double, scene_loader.h:66-70).  dd_pow
// (rt_pow.h) is the correctly rounded x^y in nearly all cases, so it agrees
// with the reference's glibc pow (scene.h:113) wherever glibc is correctly
// rounded (99.9 % of renderer-shaped operands; ocml's pow: 86 %); ocml's pow
// remains for zero or non-finite operands and |y ln x| > 700.  Called out of
// line: inlined, it would hold its registers across the whole render loop.
__device__ __attribute__((noinline)) double pow_call(double x, double y) {
  double v;
  if (dd_pow_ok(x, y) && dd_pow(x, y, v)) return v;
  return pow(x, y);
}

// pow(x, n) for the specular term's usual operands -- x in (0, 1 + 2^-40],
// n a whole shininess in [1, 1024] (every scene here uses 5..200) -- by
// left-to-right binary exponentiation in double-double: each step (square,
// times x) keeps the product as an unevaluated sum hi + lo, exact to ~2^-104
// relative (products split with fma, renormalised by fast two-sum), so after
// at most 20 steps hi + lo is within ~2^-99 of x^n and its rounding hi is the
// correctly rounded x^n unless x^n lies within that distance of a rounding
// boundary (probability ~2^-47 per call) -- the result glibc's pow (the
// reference, correctly rounded in nearly all cases) returns.  ~6 fp64
// operations per step instead of ocml's general pow (~220 instructions).
// int_pow_ok() is the domain: also n * floor(log2 x) >= -900, so no partial
// product leaves the normal range.
__device__ __forceinline__ bool int_pow_ok(double x, double y, int &n) {
  n = (int)y;
  if (!(x > 0.0 && x <= 1.0 + 0x1p-40 && y >= 1.0 && y <= 1024.0 && (double)n == y)) return false;
  const int ex = (int)((__double_as_longlong(x) >> 52) & 0x7ff) - 1023;
  return ex * n >= -900;
}
__device__ __forceinline__ double int_pow(double x, int n) {
  double h = x, l = 0.0;
  for (int i = 30 - __builtin_clz((unsigned)n); i >= 0; --i) {
    // (h, l)^2: h*h exactly as p + e, plus the cross term 2 h l (l^2 is below 2^-200 relative)
    double p = h * h;
    double e = __builtin_fma(h, h, -p);
    e = __builtin_fma(h + h, l, e);
    h = p + e;
    l = e - (h - p);
    if ((n >> i) & 1) {  // (h, l) * x
      p = h * x;
      e = __builtin_fma(h, x, -p);
      e = __builtin_fma(l, x, e);
      h = p + e;
      l = e - (h - p);
    }
  }
  return h;
}

__device__ __forceinline__ double max0(double x) { return (0.0 < x) ? x : 0.0; }  // std::max(0.0, x)
__device__ __forceinline__ double min1(double x) { return (x < 1.0) ? x : 1.0; }  // std::min(1.0, x)

// Sphere::intersect (sphere.h:26-59) for a ray whose a = dot(d,d) is hoisted:
// a4 = 4*a, a2 = 2*a (both exact scalings).  Returns true and t on a hit.
__host__ __device__ __forceinline__ bool intersect(const SphGeo &s, D3 o, D3 d, double a4, double a2, double &t) {
  double ocx = o.x - s.cx, ocy = o.y - s.cy, ocz = o.z - s.cz;
  double b = 2.0 * ((ocx * d.x + ocy * d.y) + ocz * d.z);
  double c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - s.rr;
  double disc = b * b - a4 * c;
  if (!(disc >= 0.0)) return false;  // disc < 0 -> miss; a NaN disc can never be recorded either
  if (disc == 0.0) {
    t = -b / a2;  // tangent root, kept even when negative (sphere.h:43-47)
    return true;
  }
  double sq = __builtin_sqrt(disc);
  double t1 = (-b - sq) / a2;
  double t2 = (-b + sq) / a2;
  double tmx = (t1 < t2) ? t2 : t1;
  if (tmx < 0.0) return false;
  double tmn = (t2 < t1) ? t2 : t1;
  t = (tmn < 0.0) ? tmx : tmn;
  return true;
}

// Division-free form of the same test.  With a2 = 2a > 0, t1 = fl(n1/a2) and
// t2 = fl(n2/a2) where n1 = fl(-b - sq) <= n2 = fl(-b + sq) are exactly the
// reference's numerators (sphere.h:49-50).  Division by a2 > 0 is monotone and
// for |n| >= 2^-900, a2 in [2^-60, 2^60] it can neither underflow to a signed
// zero nor change sign, so the root choice of sphere.h:51-57 (t2 < 0 -> miss;
// t = t1 < 0 ? t2 : t1) is made on the numerators: t = fl(num / a2).
// Returns 0 = miss, 1 = hit with numerator `num`, 2 = "decide with the exact
// intersect()" (a numerator too close to zero, or a2 out of range), 3 = a hit
// whose t lies below the caller's bound (qocc, see below), num not formed.
// Two cases of disc > 0 are decided without the square root:
//  * b > 0 with disc < b^2 (1 - 2^-50) (b^2 normal): sqrt(disc) rounds below
//    b, so n2 = -b + sq < 0 and both roots are negative: a miss (the same
//    bound as shadow_cells' own-sphere test).  Spheres behind the origin
//    that the line runs through (the sorted lists' behind entries, the light
//    lists' spheres beyond the shaded point) end here;
//  * c > 0 and b < 0 (the origin outside, the centre ahead): disc =
//    fl(b^2 - fl(a4 c)) <= fl(b^2), so sq <= fl(sqrt(fl(b^2))) = |b| and
//    0 <= n1 = fl(|b| - sq) <= |b|: the reference's t is t1 = fl(n1/a2) >= 0
//    (also through intersect() when n1 is tiny).  With -b below qocc (a
//    shadow query's q(1-2^-48), where a numerator gives t < T) that is an
//    occluder.  qocc < 0 (closest hits) never takes it.
constexpr double kTinyNum = 0x1p-900;
__host__ __device__ __forceinline__ int intersect_num(const SphGeo &s, D3 o, D3 d, double a4, double &num,
                                                      double qocc = -1.0) {
  double ocx = o.x - s.cx, ocy = o.y - s.cy, ocz = o.z - s.cz;
  double b = 2.0 * ((ocx * d.x + ocy * d.y) + ocz * d.z);
  double c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - s.rr;
  double p = b * b;
  double disc = p - a4 * c;
  if (!(disc >= 0.0)) return 0;
  if (disc == 0.0) {
    num = -b;  // t = -b / a2, negative roots included (sphere.h:43-47)
    return 1;
  }
  if (b > 0.0) {
    if (p > 1e-290 && disc < p * (1.0 - 0x1p-50)) return 0;
  } else if (c > 0.0 && -b < qocc) {
    return 3;
  }
  double sq = __builtin_sqrt(disc);
  double n1 = -b - sq, n2 = -b + sq;
  if (__builtin_fabs(n1) < kTinyNum || __builtin_fabs(n2) < kTinyNum) return 2;
  if (n2 < 0.0) return 0;
  num = (n1 < 0.0) ? n2 : n1;
  return 1;
}
__host__ __device__ __forceinline__ bool a2_ok(double a2) { return a2 >= 0x1p-60 && a2 <= 0x1p60; }

// ---------------------------------------------------------------------------
// Wave-wide reductions.  Called only where all 64 lanes are active.
__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ double wmax(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    double o = __shfl_xor(v, off, 64);
    v = (o > v) ? o : v;
  }
  return v;
}
__device__ __forceinline__ double wmin(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    double o = __shfl_xor(v, off, 64);
    v = (o < v) ? o : v;
  }
  return v;
}
// x rounded up to fp32 (the walks' prune bound: an entry t above it is above
// x too).  NaN stays NaN (every comparison with it keeps the box).
__host__ __device__ __forceinline__ float float_up(double x) {
  float f = (float)x;
  if ((double)f < x) {  // one float up: f is finite here (x > f)
    const int b = __builtin_bit_cast(int, f);
    f = f == 0.0f ? 0x1p-149f : __builtin_bit_cast(float, f > 0.0f ? b + 1 : b - 1);
  }
  return f;
}

// An upper bound of the wave's maximum of a double, wave-uniform: each lane's
// value rounded UP to fp32 (float_up; negatives count as 0, NaN stays NaN and
// wins), reduced on the 32-bit patterns -- ordered like the values for
// non-negative floats, NaN above +inf -- with DPP row shifts and broadcasts
// (no LDS crossbar), the result read from lane 63.  Called only where all 64
// lanes are active.
__device__ __forceinline__ double wmax_up(double v) {
  const float f = float_up(v);
  unsigned b = f >= 0.0f ? __float_as_uint(f) : (f != f ? 0x7fc00000u : 0u);
  auto step = [&](unsigned x) { b = x > b ? x : b; };
  step((unsigned)__builtin_amdgcn_update_dpp(0, (int)b, 0x111, 0xf, 0xf, false));  // row_shr:1
  step((unsigned)__builtin_amdgcn_update_dpp(0, (int)b, 0x112, 0xf, 0xf, false));  // row_shr:2
  step((unsigned)__builtin_amdgcn_update_dpp(0, (int)b, 0x113, 0xf, 0xf, false));  // row_shr:3
  step((unsigned)__builtin_amdgcn_update_dpp(0, (int)b, 0x114, 0xf, 0xe, false));  // row_shr:4, banks 1-3
  step((unsigned)__builtin_amdgcn_update_dpp(0, (int)b, 0x118, 0xf, 0xc, false));  // row_shr:8, banks 2-3
  step((unsigned)__builtin_amdgcn_update_dpp(0, (int)b, 0x142, 0xa, 0xf, false));  // row_bcast:15, rows 1, 3
  step((unsigned)__builtin_amdgcn_update_dpp(0, (int)b, 0x143, 0xc, 0xf, false));  // row_bcast:31, rows 2, 3
  return (double)__uint_as_float(__builtin_amdgcn_readlane(b, 63));
}

// Make a wave-uniform double live in SGPRs (the value is identical in every lane).
__device__ __forceinline__ double uni(double v) {
  unsigned long long b = __double_as_longlong(v);
  unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
  unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// ---------------------------------------------------------------------------
// Exact conservative culling of spheres per wave and per sweep.
//
// The active lanes' rays are treated as infinite LINES o_i + t d_i.  With a
// reference point P (camera for primary rays, the light for shadow rays, an
// active lane's origin for reflections) and a unit axis a (from the first and
// last active lanes' directions), let theta be the widest line angle between
// any d_i and a, rho_i the distance from P to line i and reach_i = |o_i - P|_1.
// For a sphere centre C with v = C - P every line satisfies
//     dist(C, line_i) >= |v x a| cos(theta) - |v . a| sin(theta) - rho_i.
// A sphere is culled only when that bound exceeds r + m_i for every lane, with
//     m_i = 1e-6 * (|v|_1 + r + reach_i)   (so |oc_i| <= |v|_1 + reach_i).
// The reference test (sphere.h:29-35) computes disc = 4|d|^2 (r^2 - dist'^2) + e
// with |e| <= ~20 * 2^-53 * 4|d|^2 (2|oc|^2 + r^2) and dist' within 2^-53 |oc| of
// dist, so dist >= r + m forces the computed disc < 0 with >100x slack: every
// culled sphere is a miss for every active lane in the reference's own fp64
// arithmetic -- including its disc == 0 (negative-root) quirk, which needs
// disc == 0 exactly.  Candidates are still tested in file order with the exact
// test, so closest-hit ties keep the lowest index.  NaN anywhere makes the
// comparison false, i.e. keeps the sphere.  Two wave reductions per sweep:
// max sin^2(theta_i) and max slack_i = |po x d|_1 + 1e-6 reach_i
// (|po x d|_1 >= rho_i |d|, |d| = 1 +- 2^-52).  ("Culling".)
struct Bound {
  double px, py, pz, ax, ay, az, cos2, sin_t, slack;
  bool cull;
};

__device__ __forceinline__ double lane_bcast(double v, int l) {
  unsigned long long b = __double_as_longlong(v);
  unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l);
  unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ Bound make_bound(bool act, D3 o, D3 d, D3 P) {
  Bound B;
  const unsigned long long am = __ballot(act);
  const int l0 = __builtin_ctzll(am), l1 = 63 - __builtin_clzll(am);
  double sx = lane_bcast(d.x, l0) + lane_bcast(d.x, l1);
  double sy = lane_bcast(d.y, l0) + lane_bcast(d.y, l1);
  double sz = lane_bcast(d.z, l0) + lane_bcast(d.z, l1);
  double len = __builtin_sqrt(sx * sx + sy * sy + sz * sz);
  D3 a = (len > 0.0) ? mk(sx / len, sy / len, sz / len) : mk(1.0, 0.0, 0.0);
  D3 cr = mk(d.y * a.z - d.z * a.y, d.z * a.x - d.x * a.z, d.x * a.y - d.y * a.x);
  double s2 = act ? dot(cr, cr) : 0.0;
  D3 po = sub(P, o);
  D3 pc = mk(po.y * d.z - po.z * d.y, po.z * d.x - po.x * d.z, po.x * d.y - po.y * d.x);
  double slack = act ? (__builtin_fabs(pc.x) + __builtin_fabs(pc.y) + __builtin_fabs(pc.z)) * (1.0 + 1e-9) +
                           1e-6 * (__builtin_fabs(po.x) + __builtin_fabs(po.y) + __builtin_fabs(po.z))
                     : 0.0;
  const double s2max = wmax_up(s2);
  B.slack = wmax_up(slack);
  B.px = uni(P.x);
  B.py = uni(P.y);
  B.pz = uni(P.z);
  B.ax = uni(a.x);
  B.ay = uni(a.y);
  B.az = uni(a.z);
  // theta from the widest sine; 1e-9 covers the rounding of |a|, |d_i| and the products.
  B.sin_t = __builtin_sqrt(s2max) + 1e-9;
  const double c = __builtin_sqrt(1.0 - (s2max < 1.0 ? s2max : 1.0)) - 1e-9;
  B.cos2 = c * c;
  B.cull = c > 0.0 && B.sin_t < 1.0;
  return B;
}

// True unless the sphere provably misses every active line (see above).
__device__ __forceinline__ bool keep(const Bound &B, double cx, double cy, double cz, double r) {
  double vx = cx - B.px, vy = cy - B.py, vz = cz - B.pz;
  double va = __builtin_fabs(vx * B.ax + vy * B.ay + vz * B.az);
  double wx = vy * B.az - vz * B.ay, wy = vz * B.ax - vx * B.az, wz = vx * B.ay - vy * B.ax;
  double vp2 = wx * wx + wy * wy + wz * wz;
  double m = 1e-6 * (__builtin_fabs(vx) + __builtin_fabs(vy) + __builtin_fabs(vz) + r);
  double rhs = r + B.slack + m + va * B.sin_t;
  return !(B.cull && vp2 * B.cos2 > rhs * rhs);
}

// Candidate mask of the 64 spheres [base, base+64) for this wave's bound.
template <bool kCull>
__device__ __forceinline__ unsigned long long candidates(const SphGeo *__restrict__ g, const double *__restrict__ rad,
                                                         int n, int base, const Bound &B) {
  if (!kCull) {
    const int cnt = n - base;
    return cnt >= 64 ? ~0ull : ((1ull << cnt) - 1ull);
  }
  const int s = base + (int)(threadIdx.x & 63);
  bool k = false;
  if (s < n) {
    const SphGeo q = g[s];
    k = keep(B, q.cx, q.cy, q.cz, rad[s]);
  }
  return __ballot(k);
}

// Scene::find_intersection (scene.h:41-61): all candidate spheres in file
// order, strict '<' (so ties keep the lowest index), t starts at 1e20.
// Work counters, per lane (summed over the wave when flushed): exact = exact
// ray-sphere tests this lane executed; cull = conservative tests it evaluated
// (one sphere vs the wave's bound in a cull sweep, one box in a BVH walk).
struct Work {
  unsigned long long exact = 0, cull = 0;
#ifdef RT_STAMPS
  // Diagnostic build only (-DRT_STAMPS): s_memtime cycles per phase, per wave.
  unsigned long long st[12] = {};
  unsigned long long iters = 0, sweeps = 0, it_closest = 0, sw_closest = 0, it_prim = 0;
#endif
};
#ifdef RT_STAMPS
// Each stamp first drains outstanding memory operations and fences the
// scheduler, so a phase's latency is charged to that phase.
__device__ __forceinline__ unsigned long long rt_stamp() {
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define RT_T0(v) const unsigned long long v = rt_stamp()
#define RT_ACC(w, slot, v) (w).st[slot] += rt_stamp() - (v)
#define RT_CNT(w, f, n) (w).f += (n)
#else
#define RT_CNT(w, f, n)
#define RT_T0(v)
#define RT_ACC(w, slot, v)
#endif
// stamp slots: 0 bound, 1 cull, 2 candidate tests, 3 per-light setup, 4 shading, 5 whole wave

// ---------------------------------------------------------------------------
// Per-lane BVH traversal (the fallback for groups whose cull bound is loose).
// Stackless: nodes in preorder with skip pointers (rt_bvh.h).  The LINE
// o + t d is tested against each box (both directions of t, so the reference's
// disc == 0 negative-root hits behind the origin are still found), in fp32
// relative to the scene centre c0, with every box grown by `margin` =
// 1e-6 * (scene diameter + largest radius) -- at least the 1e-6 (|oc| + r) that
// the cull proof above needs, and far above the fp32 rounding (~1e-7 of the
// diameter) of the slab arithmetic.  Closest-hit prunes a box only when its
// entry t exceeds the current best by a margin; any-hit prunes beyond T.
// The uniform grid (rt_bvh.h UgridHost) on the device: on = 1 when this
// launch may use it (the host checked its listing margin against pmargin and
// the DDA error bound).  A record slot or overflow entry q = centre - c0
// (fp32) and |radius| rounded up.
struct UgArgs {
  const float4 *rec;   // [cell][4] list records (grid_line)
  const int32_t *rid;  // [cell][4] their sphere ids
  const float4 *q;     // overflow lists: q[k], ids[k]
  const int32_t *ids;
  const int32_t *glob;
  int nglob;
  int nx, ny, nz;
  float gx, gy, gz, cs;
  int on;
  int closest;  // 1: closest hits walk the grid along the whole line (grid_closest_line) instead of the BVH
  float tol;    // 1e-4 * the grid's extent: the DDA's error bound, with room to spare
  int nq;       // overflow-list entries (RT_CHECK bound)
};
struct BvhArgs {
  const BvhNode *nodes;
  const int32_t *prims;
  const float4 *pf;     // per leaf slot: sphere centre - c0 (fp32) and |radius| rounded up
  float pmargin;        // prefilter margin (4x the box margin)
  int nnodes;
  float margin;
  double c0x, c0y, c0z;
  double diam;          // scene diameter bound used for the t margins
  int min_cands;        // switch a group to the BVH above this many cull candidates
  int always;           // 1: skip the cull and traverse for every group
  int max_groups;       // lanes of groups beyond this many go straight to the BVH
  // ordered (near-first) traversal: two-child nodes, the root's reference, and
  // this lane's LDS stack ([entry][lane], kOrderedStack entries); ostk ==
  // nullptr selects the stackless preorder walk
  const BvhNode2 *n2;
  int root_ref;
  // 4-wide ordered walk (wide = 1): grandchild nodes, root reference; odepth is
  // then the 4-wide walk's worst-case pending entries (build_bvh4)
  const BvhNode4 *n4;
  int root4;
  int wide;
  int ordered;  // the host allows the ordered walk (tree depth <= kOrderedStack)
  int odepth;   // stack entries per lane (the tree depth)
  int2 *ostk;
  int ostk_off;  // ostk == nullptr: the stacks sit at this byte offset of dynamic LDS ([wave][entry][lane]); -1 none
  // the ordered 4-wide closest-hit walks enter a box only if its (grown) exit
  // t is >= tf_min: 0 with the behind grid (ug.on; boxes wholly behind the
  // origin are then behind_cells' part), -inf without it
  float tf_min;
  UgArgs ug;
  int nn2, nn4, nprims;  // two-child / 4-wide nodes and leaf slots (RT_CHECK bounds)
};
constexpr int kOrderedStack = 24;  // pending far children; the host requires depth <= this

// Dynamic LDS (every extern __shared__ array starts at its base).
extern __shared__ __attribute__((aligned(32))) unsigned char rt_dyn_lds[];

// This lane's entry 0 of the ordered walk's stack.
__device__ __forceinline__ int2 *ordered_stack(const BvhArgs &bv) {
  int2 *base = bv.ostk ? bv.ostk
                       : reinterpret_cast<int2 *>(rt_dyn_lds + bv.ostk_off) +
                             (size_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * bv.odepth * 64;
  return base + (threadIdx.x & 63);
}
__device__ __forceinline__ bool has_ordered_stack(const BvhArgs &bv) { return bv.ostk || bv.ostk_off >= 0; }
// The same entry when the stacks are known to sit in dynamic LDS (ostk ==
// nullptr, the kFast kernels): an LDS-typed pointer, so pushes and pops are
// ds_write / ds_read instead of flat accesses (which also wait for the
// outstanding global loads).
// An entry is (node reference, entry t bits) = int2 {x, y}, read and written
// here as one 64-bit word (x in the low half).
typedef __attribute__((address_space(3))) unsigned long long LdsU64;
__device__ __forceinline__ LdsU64 *ordered_stack_lds(const BvhArgs &bv) {
  typedef __attribute__((address_space(3))) unsigned char LdsByte;
  LdsByte *base = (LdsByte *)(rt_dyn_lds) + bv.ostk_off;
  return reinterpret_cast<LdsU64 *>(base) + (size_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * bv.odepth * 64 +
         (threadIdx.x & 63);
}
__device__ __forceinline__ unsigned long long stk_entry(int ref, float t) {
  return ((unsigned long long)(unsigned)__float_as_int(t) << 32) | (unsigned)ref;
}


// Visits every leaf whose (grown) box the line meets and whose entry does not
// exceed tmax_fn() (re-read per node: closest-hit tightens it); calls
// leaf_fn(sphere index) for each sphere of such leaves.  leaf_fn returns
// false to stop the walk (any-hit found).
template <typename T, typename F>
__device__ __forceinline__ void bvh_walk(const BvhArgs &bv, D3 o, D3 d, T &&tmax_fn, Work &work, F &&leaf_fn) {
  const float ox = (float)(o.x - bv.c0x), oy = (float)(o.y - bv.c0y), oz = (float)(o.z - bv.c0z);
  const float dx = (float)d.x, dy = (float)d.y, dz = (float)d.z;
  const float ix = 1.0f / dx, iy = 1.0f / dy, iz = 1.0f / dz;
  const float dd = (dx * dx + dy * dy + dz * dz) * (1.0f + 1e-5f);
  const float m = bv.margin;
  int i = 0;
  while (i < bv.nnodes) {
    const BvhNode nd = bv.nodes[RT_CK(kCkBvhNode, i, bv.nnodes)];
    const float ax = (nd.lo[0] - m - ox) * ix, bx = (nd.hi[0] + m - ox) * ix;
    const float ay = (nd.lo[1] - m - oy) * iy, by = (nd.hi[1] + m - oy) * iy;
    const float az = (nd.lo[2] - m - oz) * iz, bz = (nd.hi[2] + m - oz) * iz;
    const float tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    const bool in = tn <= tf && !((double)tn > tmax_fn());
    work.cull += 1;
    RT_CNT(work, st[7], 1);
#ifdef RT_STAMPS
    if (__builtin_amdgcn_readfirstlane((int)(threadIdx.x & 63)) == (int)(threadIdx.x & 63)) work.st[10] += 1;
#endif
    if (in && nd.leaf >= 0) {
      const int first = nd.leaf >> 4, cnt = nd.leaf & 15;
      for (int k = 0; k < cnt; ++k) {
        // fp32 prefilter: the line misses the sphere grown by pmargin (fp32
        // rounding of the distance is < 6e-7 * diameter, the fp64 test can
        // only hit within 2e-8 * diameter of the surface; NaN passes)
        const float4 q = bv.pf[RT_CK(kCkBvhLeaf, first + k, bv.nprims)];
        const float wx = q.x - ox, wy = q.y - oy, wz = q.z - oz;
        const float cx = wy * dz - wz * dy, cy = wz * dx - wx * dz, cz = wx * dy - wy * dx;
        const float R = q.w + bv.pmargin;
        if (cx * cx + cy * cy + cz * cz > R * R * dd) continue;
        if (!leaf_fn((int)bv.prims[RT_CK(kCkBvhLeaf, first + k, bv.nprims)])) return;
      }
      i = nd.skip;
    } else {
      i = in ? i + 1 : nd.skip;
    }
  }
}

// Ordered closest-hit walk: at an internal node both child boxes are tested
// (same grown fp32 slab test, both directions of the line, as bvh_walk), the
// nearer child is entered and the farther pushed with its entry t; pops skip
// entries whose entry exceeds tmax_fn().  A box is pruned only against the
// current best (with bvh_walk's margin), so every leaf that can still hold a
// closer root is visited and the lexicographic (t, index) minimum is the one
// bvh_walk finds, in fewer steps.
template <typename T, typename F>
__device__ __forceinline__ void bvh_walk_ordered(const BvhArgs &bv, D3 o, D3 d, T &&tmax_fn, Work &work,
                                                 F &&leaf_fn) {
  const float ox = (float)(o.x - bv.c0x), oy = (float)(o.y - bv.c0y), oz = (float)(o.z - bv.c0z);
  const float dx = (float)d.x, dy = (float)d.y, dz = (float)d.z;
  const float ix = 1.0f / dx, iy = 1.0f / dy, iz = 1.0f / dz;
  const float dd = (dx * dx + dy * dy + dz * dz) * (1.0f + 1e-5f);
  const float m = bv.margin;
  auto slab = [&](const float *lo, const float *hi, float &tn) {
    const float ax = (lo[0] - m - ox) * ix, bx = (hi[0] + m - ox) * ix;
    const float ay = (lo[1] - m - oy) * iy, by = (hi[1] + m - oy) * iy;
    const float az = (lo[2] - m - oz) * iz, bz = (hi[2] + m - oz) * iz;
    tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    return tn <= tf && !((double)tn > tmax_fn());
  };
  int2 *st = ordered_stack(bv);
  int sp = 0;
  float tn;
  if (!slab(bv.nodes[0].lo, bv.nodes[0].hi, tn)) return;
  int ref = bv.root_ref;
  for (;;) {
    work.cull += 1;
    if (ref >= 0) {
      const BvhNode2 nd = bv.n2[RT_CK(kCkBvhNode, ref, bv.nn2)];
      float t0, t1;
      const bool h0 = slab(nd.lo0, nd.hi0, t0), h1 = slab(nd.lo1, nd.hi1, t1);
      if (h0 && h1) {
        const bool first0 = t0 <= t1;
        st[sp * 64] = make_int2(first0 ? nd.c1 : nd.c0, __float_as_int(first0 ? t1 : t0));
        ++sp;
        ref = first0 ? nd.c0 : nd.c1;
        continue;
      }
      if (h0 || h1) {
        ref = h0 ? nd.c0 : nd.c1;
        continue;
      }
    } else {
      const int leaf = -(ref + 1), first = leaf >> 4, cnt = leaf & 15;
      for (int k = 0; k < cnt; ++k) {
        const float4 q = bv.pf[RT_CK(kCkBvhLeaf, first + k, bv.nprims)];  // fp32 prefilter, as bvh_walk
        const float wx = q.x - ox, wy = q.y - oy, wz = q.z - oz;
        const float cx = wy * dz - wz * dy, cy = wz * dx - wx * dz, cz = wx * dy - wy * dx;
        const float R = q.w + bv.pmargin;
        if (cx * cx + cy * cy + cz * cz > R * R * dd) continue;
        if (!leaf_fn((int)bv.prims[RT_CK(kCkBvhLeaf, first + k, bv.nprims)])) return;
      }
    }
    bool more = false;
    while (sp > 0) {
      --sp;
      const int2 e = st[sp * 64];
      if (!((double)__int_as_float(e.y) > tmax_fn())) {
        ref = e.x;
        more = true;
        break;
      }
    }
    if (!more) return;
  }
}

// The fp32 form of a closest-hit line for the ordered 4-wide walks
// (bvh_walk_ordered4, walk4_step): origin and direction relative to the BVH
// centre c0, the slab reciprocals, |d|^2 grown for the prefilter, the slab
// planes' origins moved by the box margin once per ray ((lo - m - o) regrouped
// as lo - (o + m): one subtraction per plane; the two roundings stay ~2^-24 of
// the diameter, far inside the margin m = 1e-6 of it, so the grown slab still
// contains the exact one), and the walk's lower bound on a box's exit t.
// Host-callable, so tests/native/margin_check.cpp runs the walk's own box and
// prefilter arithmetic on the CPU.
struct Walk4Ray {
  float ox, oy, oz, dx, dy, dz, ix, iy, iz, dd, lx, ly, lz, hx, hy, hz, tfm;
};
__host__ __device__ __forceinline__ Walk4Ray walk4_ray(const BvhArgs &bv, D3 o, D3 d) {
  Walk4Ray r;
  r.ox = (float)(o.x - bv.c0x), r.oy = (float)(o.y - bv.c0y), r.oz = (float)(o.z - bv.c0z);
  r.dx = (float)d.x, r.dy = (float)d.y, r.dz = (float)d.z;
  r.ix = 1.0f / r.dx, r.iy = 1.0f / r.dy, r.iz = 1.0f / r.dz;
  r.dd = (r.dx * r.dx + r.dy * r.dy + r.dz * r.dz) * (1.0f + 1e-5f);
  const float m = bv.margin;
  r.lx = r.ox + m, r.ly = r.oy + m, r.lz = r.oz + m, r.hx = r.ox - m, r.hy = r.oy - m, r.hz = r.oz - m;
  r.tfm = bv.tf_min;
  return r;
}
// The grown fp32 slab test of one box, both directions of the line (so the
// disc == 0 negative tangent roots behind the origin are never pruned): true
// when the line meets it and its entry tn is not above the prune bound tmf (an
// upper bound of the best t, float_up); tf is its exit (the walks also require
// tf >= r.tfm below the root).  NaN boxes (unused 4-wide slots) give false.
__host__ __device__ __forceinline__ bool box4_hit(const Walk4Ray &r, float lox, float loy, float loz, float hix,
                                                  float hiy, float hiz, float tmf, float &tn, float &tf) {
  const float ax = (lox - r.lx) * r.ix, bx = (hix - r.hx) * r.ix;
  const float ay = (loy - r.ly) * r.iy, by = (hiy - r.hy) * r.iy;
  const float az = (loz - r.lz) * r.iz, bz = (hiz - r.hz) * r.iz;
  tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
  tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
  return tn <= tf && !(tn > tmf);
}
// The leaves' fp32 sphere prefilter: false when the line provably misses the
// sphere grown by pmargin (|w x d|^2 > R^2 |d|^2 with |d|^2 grown by 1e-5; the
// fp32 rounding of the distance is < 6e-7 * diameter, the fp64 test can only
// hit within 2e-8 * diameter of the surface; NaN passes).  q: centre - c0 and
// |radius| rounded up.
__host__ __device__ __forceinline__ bool pf_keep(const Walk4Ray &r, float qx, float qy, float qz, float qw,
                                                 float pmargin) {
  const float wx = qx - r.ox, wy = qy - r.oy, wz = qz - r.oz;
  const float cx = wy * r.dz - wz * r.dy, cy = wz * r.dx - wx * r.dz, cz = wx * r.dy - wy * r.dx;
  const float R = qw + pmargin;
  return !(cx * cx + cy * cy + cz * cz > R * R * r.dd);
}

// Ordered closest-hit walk over the 4-wide nodes (rt_bvh.h BvhNode4): the
// same grown fp32 slab test as bvh_walk_ordered on up to four child boxes,
// the nearest entered, the other hits pushed farthest first (so the nearest
// pending one is popped next), pops pruned against the current best.  Half
// the iterations of the two-child walk (scripts/bvh_sim.cpp: 29 -> 15 wave
// node-steps per primary query, 89 -> 46 per secondary, synth10k), each one
// with four independent box tests.  Every leaf that can hold a closer root is
// still visited, so the lexicographic (t, index) minimum is unchanged.
template <bool kLdsStack = false, typename T, typename F>
__device__ __forceinline__ void bvh_walk_ordered4(const BvhArgs &bv, D3 o, D3 d, T &&tmax_fn, Work &work,
                                                  F &&leaf_fn) {
  const Walk4Ray r = walk4_ray(bv, o, d);
  // The prune bound in fp32, rounded up (re-read after every leaf, where the
  // best t can shrink): an entry t > tmf is > tmax_fn() too, so every box the
  // fp64 comparison keeps is kept (a box at tmax < t <= tmf is kept as well,
  // which costs a visit, never a result); NaNs keep boxes either way.
  auto tmax_f = [&] { return float_up(tmax_fn()); };
  float tmf = tmax_f();
  {
    const BvhNode &r0 = bv.nodes[0];
    float tn, tf;
    if (!box4_hit(r, r0.lo[0], r0.lo[1], r0.lo[2], r0.hi[0], r0.hi[1], r0.hi[2], tmf, tn, tf)) return;
  }
  auto st = [&] {
    if constexpr (kLdsStack) return ordered_stack_lds(bv);
    else return reinterpret_cast<unsigned long long *>(ordered_stack(bv));
  }();
  int sp = 0;
  int ref = bv.root4;
  for (;;) {
    work.cull += 1;
    if (ref >= 0) {
      const BvhNode4 *nd = bv.n4 + RT_CK(kCkBvhNode, ref, bv.nn4);
      float t[4];
      int c[4];
      int hits = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float tn, tf;
        const bool h = box4_hit(r, nd->lox[k], nd->loy[k], nd->loz[k], nd->hix[k], nd->hiy[k], nd->hiz[k], tmf, tn,
                                tf) && tf >= r.tfm;
        hits += h ? 1 : 0;
        // sort key: a hit sorts below every miss (fminf keeps it finite-or-below-inf)
        t[k] = h ? fminf(tn, 3.0e38f) : __builtin_inff();
        c[k] = nd->c[k];
      }
      auto ce = [&](int a, int b) {  // compare-exchange, ascending
        const bool sw = t[b] < t[a];
        const float ta = sw ? t[b] : t[a], tb = sw ? t[a] : t[b];
        const int ca = sw ? c[b] : c[a], cb = sw ? c[a] : c[b];
        t[a] = ta, t[b] = tb, c[a] = ca, c[b] = cb;
      };
      ce(0, 1);
      ce(2, 3);
      ce(0, 2);
      ce(1, 3);
      ce(1, 2);
      if (hits > 0) {
        if (hits > 3) st[(sp++) * 64] = stk_entry(c[3], t[3]);
        if (hits > 2) st[(sp++) * 64] = stk_entry(c[2], t[2]);
        if (hits > 1) st[(sp++) * 64] = stk_entry(c[1], t[1]);
        ref = c[0];
        continue;
      }
    } else {
      const int leaf = -(ref + 1), first = leaf >> 4, cnt = leaf & 15;
      for (int k = 0; k < cnt; ++k) {
        const float4 q = bv.pf[RT_CK(kCkBvhLeaf, first + k, bv.nprims)];  // fp32 prefilter, as bvh_walk
        if (!pf_keep(r, q.x, q.y, q.z, q.w, bv.pmargin)) continue;
        if (!leaf_fn((int)bv.prims[RT_CK(kCkBvhLeaf, first + k, bv.nprims)])) return;
      }
      tmf = tmax_f();
    }
    bool more = false;
    while (sp > 0) {
      --sp;
      const unsigned long long e = st[sp * 64];
      if (!(__int_as_float((int)(e >> 32)) > tmf)) {
        ref = (int)(unsigned)e;
        more = true;
        break;
      }
    }
    if (!more) return;
  }
}

// bvh_walk_ordered4 (LDS stacks) as a resumable state machine, for a kernel
// whose lanes are at different stages of their rays (render_deferred_walk):
// walk4_begin tests the root box, each walk4_step visits the pending node or
// leaf and pops the next pending entry (false: the walk is over).  The
// visits, their order and the pruning are bvh_walk_ordered4's, so the closest
// hit is the same.  The fp32 form of the ray (walk4_ray) is recomputed
// wherever a kernel resumes walks, so it is not live across other work.
__device__ __forceinline__ bool walk4_begin(const BvhArgs &bv, const Walk4Ray &r, float tmf, int &ref, int &sp) {
  const BvhNode &r0 = bv.nodes[0];
  float tn, tf;
  ref = bv.root4;
  sp = 0;
  return box4_hit(r, r0.lo[0], r0.lo[1], r0.lo[2], r0.hi[0], r0.hi[1], r0.hi[2], tmf, tn, tf);
}
// leaf_fn(sphere index) tests one sphere; tmf_fn() is the current prune bound
// (float_up of the closest-hit margin), re-read after a leaf.
template <typename T, typename F>
__device__ __forceinline__ bool walk4_step(const BvhArgs &bv, const Walk4Ray &r, T &&tmf_fn, Work &work, F &&leaf_fn,
                                           int &ref, int &sp, float &tmf) {
  LdsU64 *st = ordered_stack_lds(bv);
  work.cull += 1;
  if (ref >= 0) {
    const BvhNode4 *nd = bv.n4 + RT_CK(kCkBvhNode, ref, bv.nn4);
    float t[4];
    int c[4];
    int hits = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float tn, tf;
      const bool h = box4_hit(r, nd->lox[k], nd->loy[k], nd->loz[k], nd->hix[k], nd->hiy[k], nd->hiz[k], tmf, tn, tf) &&
                     tf >= r.tfm;
      hits += h ? 1 : 0;
      t[k] = h ? fminf(tn, 3.0e38f) : __builtin_inff();
      c[k] = nd->c[k];
    }
    auto ce = [&](int a, int b) {
      const bool sw = t[b] < t[a];
      const float ta = sw ? t[b] : t[a], tb = sw ? t[a] : t[b];
      const int ca = sw ? c[b] : c[a], cb = sw ? c[a] : c[b];
      t[a] = ta, t[b] = tb, c[a] = ca, c[b] = cb;
    };
    ce(0, 1);
    ce(2, 3);
    ce(0, 2);
    ce(1, 3);
    ce(1, 2);
    if (hits > 0) {
      if (hits > 3) st[(sp++) * 64] = stk_entry(c[3], t[3]);
      if (hits > 2) st[(sp++) * 64] = stk_entry(c[2], t[2]);
      if (hits > 1) st[(sp++) * 64] = stk_entry(c[1], t[1]);
      ref = c[0];
      return true;
    }
  } else {
    const int leaf = -(ref + 1), first = leaf >> 4, cnt = leaf & 15;
    for (int k = 0; k < cnt; ++k) {
      const float4 q = bv.pf[RT_CK(kCkBvhLeaf, first + k, bv.nprims)];  // fp32 prefilter, as bvh_walk
      if (!pf_keep(r, q.x, q.y, q.z, q.w, bv.pmargin)) continue;
      leaf_fn((int)bv.prims[RT_CK(kCkBvhLeaf, first + k, bv.nprims)]);
    }
    tmf = tmf_fn();
  }
  while (sp > 0) {
    --sp;
    const unsigned long long e = st[sp * 64];
    if (!(__int_as_float((int)(e >> 32)) > tmf)) {
      ref = (int)(unsigned)e;
      return true;
    }
  }
  return false;
}

// One candidate of the closest-hit search (sweep_closest's exact test): (bt,
// bi) is the lexicographic (t, index) minimum so far and bn its numerator.
__device__ __forceinline__ void closest_test(const SphGeo &s, int i, D3 o, D3 d, double a4, double a2, bool fast,
                                             double &bt, double &bn, int &bi) {
  double num;
  const int r = fast ? intersect_num(s, o, d, a4, num) : 2;
  if (r == 1) {
    if (num < bn || i < bi) {
      const double t = num / a2;
      if (t < bt || (t == bt && i < bi)) {
        bt = t;
        bn = num;
        bi = i;
      }
    }
  } else if (r == 2) {
    double t;
    if (intersect(s, o, d, a4, a2, t) && (t < bt || (t == bt && i < bi))) {
      bt = t;
      bn = __builtin_inf();  // no numerator for this best: every later candidate divides
      bi = i;
    }
  }
}

// The grid walks (bv.ug, the uniform grid of rt_bvh.h UgridHost): a 3-D DDA
// in fp32 along a closest-hit line, visiting its cells in order and handing
// every sphere listed there that the line passes near to test_fn (which folds
// it into the lexicographic (t, index) minimum, so a sphere tested twice is
// harmless).  Two uses:
//
// behind_cells -- the part of the line BEHIND its origin, when the ordered
// walks skipped the boxes wholly behind it (bv.tf_min = 0).  A box whose
// grown exit t is < 0 in the walk's fp32 slab test (error ~2^-23 of the
// diameter, far inside the 1e-6 margin) holds only spheres all of whose
// points lie at t < 0.  For such a sphere the reference's test
// (sphere.h:26-59) reports a hit only through its disc == 0 branch (the
// tangent root -b/2a, kept whatever its sign, sphere.h:43-47): with disc > 0
// both roots are negative by more than their rounding (|oc| 2^-50 << the
// margin), so max(t1, t2) < 0 is a miss; and disc == 0 needs the line within
// ~2e-8 of the diameter of the sphere's surface (the cull proof's bound,
// above).  So it suffices to test every sphere whose surface the backward
// half-line {o + t d, t <= 0} passes within the prefilter margin of.
//
// grid_closest_line -- the whole closest hit (bv.ug.closest, instead of the
// BVH walk): the line from where it enters the grid, in order along +d; the
// walk stops after the first cell whose exit t is beyond the best t + tol: a
// sphere with a root t* below the best has that root's point on its surface,
// inside a cell entered at t <= t* that the DDA has visited.
//
// Coverage: the global spheres (listed in no cell) are tested first; every
// other sphere is listed in every cell its box grown by reg_margin meets, and
// reg_margin >= pmargin + tol, tol = 1e-4 * the grid's extent (the host's
// per-launch check): every line point within R + pmargin of a listed centre
// lies within reg_margin - tol of that sphere's cells, and the visited cells
// miss no line point by more than the DDA's fp32 error (a few ulps of the
// extent, << tol).  Prefilter (fp32, as the BVH walks' leaves): a sphere is
// skipped when the line misses it grown by pmargin, and -- in cells wholly
// behind the origin -- when the line runs deep inside it (disc > 0 there,
// both roots negative; a root ahead lies in a cell ahead, where the sphere
// is listed too and tested).  NaN lines return at once (the reference's
// test never records a NaN t).
//
// A cell's list is one 64-B record of four float4 slots (centre - c0, |r|
// rounded up; w = -1: no more entries; w = -2 in slot 3: entries x..y of the
// overflow list continue the cell), so a cell is one 64-B load, issued one
// cell ahead; sphere ids are read only for the spheres that pass.
template <bool kWhole, typename F, typename B>
__host__ __device__ __forceinline__ void grid_line(const BvhArgs &bv, D3 o, D3 d, Work &work, F &&test_fn,
                                                   B &&best_fn) {
  const UgArgs &ug = bv.ug;
  for (int k = 0; k < ug.nglob; ++k) {
    work.exact += 1;
    test_fn((int)ug.glob[k]);
  }
  const float ox = (float)(o.x - bv.c0x), oy = (float)(o.y - bv.c0y), oz = (float)(o.z - bv.c0z);
  const float dx = (float)d.x, dy = (float)d.y, dz = (float)d.z;
  const float d2 = dx * dx + dy * dy + dz * dz;
  const float dd_hi = d2 * (1.0f + 1e-5f), dd_lo = d2 * (1.0f - 1e-5f);
  const float pm = bv.pmargin;
  const float cs = ug.cs;
  const float p0 = ox - ug.gx, p1 = oy - ug.gy, p2 = oz - ug.gz;  // the origin in grid coordinates
  // walk direction: +d for the whole line, -d behind the origin (then s = -t)
  const float v0 = kWhole ? dx : -dx, v1 = kWhole ? dy : -dy, v2 = kWhole ? dz : -dz;
  const float i0 = 1.0f / v0, i1 = 1.0f / v1, i2 = 1.0f / v2;  // +-inf for a zero component
  // the walked part inside the grid box [0, n cs]^3: s in [s0, s1]
  float s0 = kWhole ? -__builtin_inff() : 0.0f, s1 = __builtin_inff();
  auto clip = [&](float p, float iv, int n) {
    const float ta = (0.0f - p) * iv, tb = ((float)n * cs - p) * iv;  // a zero component: +-inf or NaN
    if (iv == __builtin_inff() || iv == -__builtin_inff()) {
      if (!(p >= 0.0f && p <= (float)n * cs)) s1 = -__builtin_inff();  // parallel to the slab and outside it
    } else {
      s0 = fmaxf(s0, fminf(ta, tb));
      s1 = fminf(s1, fmaxf(ta, tb));
    }
  };
  clip(p0, i0, ug.nx);
  clip(p1, i1, ug.ny);
  clip(p2, i2, ug.nz);
  if (!(s0 <= s1)) return;  // misses the grid (or NaN)
  const float ics = 1.0f / cs;
  auto cell_of = [&](float p, float v, int n) {
    const int c = (int)floorf((p + v * s0) * ics);
    return c < 0 ? 0 : (c >= n ? n - 1 : c);
  };
  int c0 = cell_of(p0, v0, ug.nx), c1 = cell_of(p1, v1, ug.ny), c2 = cell_of(p2, v2, ug.nz);
  const int st0 = v0 > 0.0f ? 1 : -1, st1 = v1 > 0.0f ? 1 : -1, st2 = v2 > 0.0f ? 1 : -1;
  // the exit s of the current cell along each axis (re-derived per step, not accumulated)
  auto exit_s = [&](int c, float p, float iv, int st) {
    return (iv == __builtin_inff() || iv == -__builtin_inff()) ? __builtin_inff()
                                                              : ((float)(c + (st > 0 ? 1 : 0)) * cs - p) * iv;
  };
  int ci = RT_CK(kCkUgCell, (c2 * ug.ny + c1) * ug.nx + c0, ug.nx * ug.ny * ug.nz);
  float4 r0 = ug.rec[4 * ci], r1 = ug.rec[4 * ci + 1], r2 = ug.rec[4 * ci + 2], r3 = ug.rec[4 * ci + 3];
  int guard = ug.nx + ug.ny + ug.nz + 2;  // every step leaves the cell along one axis for good
  int last = -1;                          // the sphere tested last (spheres span neighbouring cells)
  // the current cell's exit s per axis; a step re-derives only the stepped axis's
  float e0 = exit_s(c0, p0, i0, st0), e1 = exit_s(c1, p1, i1, st1), e2 = exit_s(c2, p2, i2, st2);
  while (true) {
    // the next cell first, so its record is in flight while this one's slots are tested
    const float ex = fminf(e0, fminf(e1, e2));  // this cell's exit
    bool more = false;
    if (--guard > 0) {
      if (e0 <= e1 && e0 <= e2) {
        c0 += st0;
        more = e0 <= s1 && c0 >= 0 && c0 < ug.nx;
        e0 = exit_s(c0, p0, i0, st0);
      } else if (e1 <= e2) {
        c1 += st1;
        more = e1 <= s1 && c1 >= 0 && c1 < ug.ny;
        e1 = exit_s(c1, p1, i1, st1);
      } else {
        c2 += st2;
        more = e2 <= s1 && c2 >= 0 && c2 < ug.nz;
        e2 = exit_s(c2, p2, i2, st2);
      }
    }
    const int cur = ci;
    float4 n0 = r0, n1 = r1, n2 = r2, n3 = r3;
    if (more) {
      ci = RT_CK(kCkUgCell, (c2 * ug.ny + c1) * ug.nx + c0, ug.nx * ug.ny * ug.nz);
      n0 = ug.rec[4 * ci];
      n1 = ug.rec[4 * ci + 1];
      n2 = ug.rec[4 * ci + 2];
      n3 = ug.rec[4 * ci + 3];
    }
    work.cull += 1;
    // cells wholly behind the origin: the deep-inside skip applies
    const bool behind = kWhole ? ex < 0.0f : true;
    auto one = [&](const float4 &q, int id_at, const int32_t *ids) {
      const float wx = q.x - ox, wy = q.y - oy, wz = q.z - oz;
      const float cx = wy * dz - wz * dy, cy = wz * dx - wx * dz, cz = wx * dy - wy * dx;
      const float x2 = cx * cx + cy * cy + cz * cz;  // (distance to the line)^2 |d|^2
      const float ro = q.w + pm, ri = q.w * (1.0f - 0x1p-22f) - pm;
      if (x2 > ro * ro * dd_hi) return;                          // misses the grown sphere
      if (behind && ri > 0.0f && x2 < ri * ri * dd_lo) return;  // runs deep inside it
      const int id = (int)ids[id_at];
      if (id == last) return;
      last = id;
      work.exact += 1;
      test_fn(id);
    };
    // false: no slot after this one
    auto slot = [&](const float4 &q, int j) {
      if (q.w >= 0.0f) {
        one(q, 4 * cur + j, ug.rid);
        return true;
      }
      if (q.w == -2.0f)  // the cell continues in the overflow list
        for (int k = __builtin_bit_cast(int, q.x), ke = __builtin_bit_cast(int, q.y); k < ke; ++k)
          one(ug.q[RT_CK(kCkUgOver, k, ug.nq)], RT_CK(kCkUgOver, k, ug.nq), ug.ids);
      return false;
    };
    if (slot(r0, 0) && slot(r1, 1) && slot(r2, 2)) slot(r3, 3);
    if (!more) break;
    if (kWhole && (double)ex > best_fn() + (double)ug.tol) break;
    r0 = n0;
    r1 = n1;
    r2 = n2;
    r3 = n3;
  }
}

// Host-callable too (tests/native/ug_check.cpp runs this same code on the CPU).
template <typename F>
__host__ __device__ __forceinline__ void behind_cells(const BvhArgs &bv, D3 o, D3 d, Work &work, F &&test_fn) {
  grid_line<false>(bv, o, d, work, test_fn, [] { return 0.0; });
}
template <typename F, typename B>
__host__ __device__ __forceinline__ void grid_closest_line(const BvhArgs &bv, D3 o, D3 d, Work &work, F &&test_fn,
                                                           B &&best_fn) {
  grid_line<true>(bv, o, d, work, test_fn, best_fn);
}

// LDS layout of a staged scene: sphere geometry, radii, lights and, when the
// scene is staged (lds_geo) and has a BVH, its nodes and leaf sphere indices.
// The host sizes the dynamic LDS with the same function.
#ifndef RT_MAT_LDS
#define RT_MAT_LDS 0
#endif
struct LdsLayout {
  size_t rad, light, nodes, pf, prims, mat, end;
};
__host__ __device__ inline LdsLayout lds_layout(bool lds_geo, int n, int nl, int nnodes) {
  LdsLayout L;
  L.rad = lds_geo ? (size_t)n * sizeof(SphGeo) : 0;
  L.light = lds_geo ? (size_t)n * (sizeof(SphGeo) + sizeof(double)) : 0;
  // lights: staged only with a staged scene (stage_scene); otherwise read with scalar loads
  size_t e = (L.light + (lds_geo ? (size_t)nl * sizeof(LightD) : 0) + 15) & ~(size_t)15;
  const bool bvh = lds_geo && nnodes > 0;
  L.nodes = e;
  if (bvh) e += (size_t)nnodes * sizeof(BvhNode);
  L.pf = e;
  if (bvh) e += (size_t)n * sizeof(float4);
  L.prims = e;
  if (bvh) e += (size_t)n * sizeof(int32_t);
  // materials (read once per hit) after the BVH, when staged
  L.mat = (e + 15) & ~(size_t)15;
  if (lds_geo && RT_MAT_LDS) e = L.mat + (size_t)n * sizeof(SphMat);
  L.end = e;
  return L;
}

// Copies the scene (and, with kLdsGeo, its BVH and materials) into LDS; g/rad/sm/lights and
// bv.nodes/bv.prims then point at the LDS copies.  Ends with a barrier.
template <bool kLdsGeo>
__device__ __forceinline__ void stage_scene(unsigned char *smem, const SphGeo *geo, const double *radius,
                                            const SphMat *mat, const LightD *lights, int n, int nl, BvhArgs &bv,
                                            const SphGeo *&g, const double *&rad, const SphMat *&sm,
                                            const LightD *&sl) {
  const LdsLayout L = lds_layout(kLdsGeo, n, nl, bv.nnodes);
  SphGeo *sgeo = reinterpret_cast<SphGeo *>(smem);
  double *srad = reinterpret_cast<double *>(smem + L.rad);
  LightD *slight = reinterpret_cast<LightD *>(smem + L.light);
  BvhNode *snodes = reinterpret_cast<BvhNode *>(smem + L.nodes);
  int32_t *sprims = reinterpret_cast<int32_t *>(smem + L.prims);
  float4 *spf = reinterpret_cast<float4 *>(smem + L.pf);
  SphMat *smat = reinterpret_cast<SphMat *>(smem + L.mat);
  const int tid = (int)threadIdx.x, nt = (int)blockDim.x;
  if (kLdsGeo) {
    for (int i = tid; i < n; i += nt) {
      sgeo[i] = geo[i];
      srad[i] = radius[i];
      if (RT_MAT_LDS) smat[i] = mat[i];
    }
    if (bv.nnodes > 0) {
      for (int i = tid; i < bv.nnodes; i += nt) snodes[i] = bv.nodes[i];
      for (int i = tid; i < n; i += nt) {
        sprims[i] = bv.prims[i];
        spf[i] = bv.pf[i];
      }
    }
  }
  // lights: staged with a staged scene; otherwise read from global memory at
  // wave-uniform indices, i.e. scalar loads into SGPRs instead of LDS reads
  // into VGPRs (the light loop is where VGPR pressure peaks)
  if (kLdsGeo)
    for (int i = tid; i < nl; i += nt) slight[i] = lights[i];
  __syncthreads();
  g = kLdsGeo ? sgeo : geo;
  rad = kLdsGeo ? srad : radius;
  sm = (kLdsGeo && RT_MAT_LDS) ? smat : mat;
  sl = kLdsGeo ? slight : lights;
  if (kLdsGeo) {
    bv.nodes = snodes;
    bv.prims = sprims;
    bv.pf = spf;
  }
}

// Lanes of a wave are swept in coherent groups: lanes whose rays leave the
// same sphere (`key` = that sphere's index; -1 for camera rays) share one
// bound, so a wave whose secondary rays leave several spheres does not pay the
// candidate union of all of them.  Each lane takes part in exactly one group
// pass and only its own pass updates it, so results (and closest-hit ties) are
// unchanged.  `P` of a group is the origin of its first lane.
__device__ __forceinline__ unsigned long long next_group(unsigned long long todo, int key) {
  const int first = __builtin_ctzll(todo);
  const int kf = __builtin_amdgcn_readlane(key, first);
  return __ballot(key == kf) & todo;
}

// Scene::find_intersection (scene.h:41-61): all candidate spheres in file
// order, strict '<' (so ties keep the lowest index), t starts at 1e20.
// kFast: the default configuration only (ordered 4-wide BVH walk); the other
// walks are not compiled in, which keeps the default kernel's register
// allocation free of their cold paths (render_kernel's kFast).
template <bool kCull, bool kFast = false>
__device__ __forceinline__ int sweep_closest(const SphGeo *__restrict__ g, const double *__restrict__ rad, int n,
                                             bool act, D3 o, D3 d, int key, const BvhArgs &bv, double &best_t,
                                             Work &work) {
  const double a = dot(d, d);
  const double a4 = 4.0 * a, a2 = 2.0 * a;
  double bt = kInf, bn = __builtin_inf();
  int bi = -1;
  const bool fast = a2_ok(a2);
  const int lane = (int)(threadIdx.x & 63);
  // Lexicographic (t, index) minimum == the reference's strict-< scan in file
  // order (scene.h:50-58); in file order the index tie-break never fires.
  // A numerator >= the best's with a larger index cannot win, so it skips the
  // division.
  auto test = [&](int i) {
    double num;
    const int r = fast ? intersect_num(g[RT_CK(kCkSphere, i, n)], o, d, a4, num) : 2;
    if (r == 1) {
      if (num < bn || i < bi) {
        const double t = num / a2;
        if (t < bt || (t == bt && i < bi)) {
          bt = t;
          bn = num;
          bi = i;
        }
      }
    } else if (r == 2) {
      double t;
      if (intersect(g[i], o, d, a4, a2, t) && (t < bt || (t == bt && i < bi))) {
        bt = t;
        bn = __builtin_inf();  // no numerator for this best: every later candidate divides
        bi = i;
      }
    }
  };
  unsigned long long todo = __ballot(act);
  RT_CNT(work, sw_closest, 1);
  // Lanes whose group bound is loose (or that come after max_groups groups)
  // are collected in `need` and walk the BVH together after the group passes,
  // so the divergent walks of different groups overlap instead of queueing.
  const bool have_bvh = kCull && bv.nnodes > 0;
  bool need = false;
  int groups = 0;
  while (todo) {
    if (have_bvh && (bv.always || groups >= bv.max_groups)) {
      need = need || ((todo >> lane) & 1ull);
      break;
    }
    const unsigned long long grp = kCull ? next_group(todo, key) : todo;
    todo &= ~grp;
    ++groups;
    const bool gact = (grp >> lane) & 1ull;
    if (kCull) {
      Bound B;
      RT_T0(tb);
      const int fl = __builtin_ctzll(grp);
      B = make_bound(gact, o, d, mk(lane_bcast(o.x, fl), lane_bcast(o.y, fl), lane_bcast(o.z, fl)));
      RT_ACC(work, 0, tb);
      RT_CNT(work, sweeps, 1);
      int seen = 0;
      for (int base = 0; base < n; base += 64) {
        RT_T0(tc);
        unsigned long long mask = candidates<kCull>(g, rad, n, base, B);
        RT_ACC(work, 1, tc);
        work.cull += base + lane < n ? 1u : 0u;  // this lane's keep() test
        seen += __popcll(mask);
        if (have_bvh && seen > bv.min_cands) {  // loose bound: this group walks the BVH
          need = need || gact;
          break;
        }
        RT_T0(tt);
        if (gact) {
          work.exact += (unsigned)__popcll(mask);
          while (mask) {
            const int i = base + __builtin_ctzll(mask);
            mask &= mask - 1;
            RT_CNT(work, iters, 1);
            RT_CNT(work, it_closest, 1);
            test(i);
          }
        }
        RT_ACC(work, 2, tt);
      }
    } else {
      for (int base = 0; base < n; base += 64) {
        unsigned long long mask = candidates<false>(g, rad, n, base, Bound{});
        if (gact) {
          work.exact += (unsigned)__popcll(mask);
          while (mask) {
            const int i = base + __builtin_ctzll(mask);
            mask &= mask - 1;
            test(i);
          }
        }
      }
    }
  }
#ifdef RT_STAMPS
  const bool any_need = have_bvh && __ballot(need) != 0;
  RT_T0(tv);
#endif
  if (have_bvh && need) {
    // a box whose entry is beyond the best t (by the margin) holds no closer root;
    // spheres a group pass already tested are harmless to test again
    auto tmax = [&] { return bt + 2e-6 * (bv.diam + __builtin_fabs(bt)); };
    auto leaf = [&](int i) {
      work.exact += 1;
      test(i);
      return true;
    };
    if constexpr (kFast) {
      if (bv.ug.on && bv.ug.closest) {
        grid_closest_line(bv, o, d, work, test, [&] { return bt; });
      } else {
        bvh_walk_ordered4<true>(bv, o, d, tmax, work, leaf);
        if (bv.ug.on) behind_cells(bv, o, d, work, test);
      }
    } else {
      if (bv.ug.on && bv.ug.closest) {
        grid_closest_line(bv, o, d, work, test, [&] { return bt; });
      } else if (has_ordered_stack(bv) && bv.wide) {
        bvh_walk_ordered4(bv, o, d, tmax, work, leaf);
        if (bv.ug.on) behind_cells(bv, o, d, work, test);
      } else if (has_ordered_stack(bv)) {
        bvh_walk_ordered(bv, o, d, tmax, work, leaf);
      } else {
        bvh_walk(bv, o, d, tmax, work, leaf);
      }
    }
  }
#ifdef RT_STAMPS
  if (any_need) RT_ACC(work, 6, tv);
#endif
  best_t = bt;
  return bi;
}

// Scene::in_shadow (scene.h:65-86) as an any-hit over the candidates: some
// sphere with t < 1e20 (the find_intersection start value) and t < dist.  A
// group leaves as soon as the ballot of its still-unoccluded lanes is empty.
// All shadow rays of a light pass (up to rounding) through the light, so P is
// the light for every group; the key still splits lanes by surface sphere.
template <bool kCull>
__device__ __forceinline__ bool sweep_shadow(const SphGeo *__restrict__ g, const double *__restrict__ rad, int n,
                                             bool act, D3 o, D3 d, D3 P, int key, double dist, const BvhArgs &bv,
                                             Work &work) {
  unsigned long long todo = __ballot(act);
  if (todo == 0) return false;
  const double a = dot(d, d);
  const double a4 = 4.0 * a, a2 = 2.0 * a;
  // occluded <=> t < T, T = min(dist, 1e20).  With q = fl(a2*T), a numerator
  // below q(1-2^-48) gives fl(num/a2) < T and one above q(1+2^-48) gives
  // fl(num/a2) > T (both with >2^-50 relative room), so only the band between
  // needs the exact division.
  const double T = dist < kInf ? dist : kInf;
  const bool fast = a2_ok(a2) && dist == dist && T >= 0x1p-900;
  const double q = a2 * T, qlo = q * (1.0 - 0x1p-48), qhi = q * (1.0 + 0x1p-48);
  const int lane = (int)(threadIdx.x & 63);
  bool occ = false;
  auto test = [&](int i) {
    double num;
    const int r = fast ? intersect_num(g[RT_CK(kCkSphere, i, n)], o, d, a4, num, qlo) : 2;
    if (r == 3) {
      occ = true;
    } else if (r == 1) {
      if (num < qlo) occ = true;
      else if (!(num > qhi)) {
        const double t = num / a2;
        occ = t < kInf && t < dist;
      }
    } else if (r == 2) {
      double t;
      occ = intersect(g[i], o, d, a4, a2, t) && t < kInf && t < dist;
    }
  };
  const bool have_bvh = kCull && bv.nnodes > 0;
  bool need = false;
  int groups = 0;
  while (todo) {
    if (have_bvh && (bv.always || groups >= bv.max_groups)) {
      need = need || ((todo >> lane) & 1ull);
      break;
    }
    const unsigned long long grp = kCull ? next_group(todo, key) : todo;
    todo &= ~grp;
    ++groups;
    const bool gact = (grp >> lane) & 1ull;
    unsigned long long live = grp;
    Bound B;
    RT_T0(tb);
    if (kCull) B = make_bound(gact, o, d, P);
    RT_ACC(work, 0, tb);
    RT_CNT(work, sweeps, 1);
    int seen = 0;
    for (int base = 0; base < n && live; base += 64) {
      RT_T0(tc);
      unsigned long long mask = candidates<kCull>(g, rad, n, base, B);
      RT_ACC(work, 1, tc);
      if (kCull) {
        work.cull += base + lane < n ? 1u : 0u;  // this lane's keep() test
        seen += __popcll(mask);
        if (have_bvh && seen > bv.min_cands) {
          need = need || (gact && !occ);
          break;
        }
      }
      RT_T0(tt);
      while (mask) {
        const int i = base + __builtin_ctzll(mask);
        mask &= mask - 1;
        RT_CNT(work, iters, 1);
        if (gact && !occ) {
          work.exact += 1;
          test(i);
        }
        live = __ballot(gact && !occ);
        if (live == 0) break;
      }
      RT_ACC(work, 2, tt);
    }
  }
#ifdef RT_STAMPS
  const bool any_need = have_bvh && __ballot(need && !occ) != 0;
  RT_T0(tv);
#endif
  if (have_bvh && need && !occ) {
    // boxes entirely beyond T (by the margin) cannot occlude; boxes behind the
    // origin are still visited (negative tangent roots count, sphere.h:43-47)
    const double tmax = T + 2e-6 * (bv.diam + T);
    bvh_walk(bv, o, d, [&] { return tmax; }, work, [&](int i) {
      work.exact += 1;
      test(i);
      return !occ;
    });
  }
#ifdef RT_STAMPS
  if (any_need) RT_ACC(work, 6, tv);
#endif
  return act && occ;
}

// Shadow query through the light's direction grid (rt_lightgrid.h): each lane
// tests the list of the cell its direction (from the light towards the shaded
// point) falls in and the global list, with the same exact test and early
// exit as sweep_shadow.  A lane whose direction cannot be binned (degenerate or
// non-finite) or whose line misses the light by more than max_off tests every
// sphere.
struct LgArgs {
  const int32_t *start;
  const int32_t *ids;
  int N;
  int on;          // 0: shadow rays use sweep_shadow
  double max_off;  // largest distance of a ray's line from its light the grid margins cover
  long long nstart, nids;  // CSR starts and list ids (RT_CHECK bounds)
  int off_free;    // 1: every query's line provably within max_off of its light (the host's bound, below)
};

// The cell list a shadow query of light l from point hp will test: the cell
// of direction hp - L (within 1e-15 rad of the query line's -d, far inside
// the grid's slack).  cb = -1: direction not binnable, test every sphere.
// Issued one light ahead so the load overlaps the previous light's work.
struct LgRange {
  int cb, ce;
};
// lg_cell (rt_lightgrid.h) with the two quotients p/m, q/m formed as p * rcp(m)
// (v_rcp_f32, within 1 ulp): each within 2^-22 relative of the IEEE
// quotient, an angle error far inside the grids' 4e-6 rad slack;
// tests/native/lg_check.cpp checks the lists against cells binned with
// +-2^-22 quotient errors.
__device__ __forceinline__ int lg_cell_rcp(float ux, float uy, float uz, int N) {
  const float ax = __builtin_fabsf(ux), ay = __builtin_fabsf(uy), az = __builtin_fabsf(uz);
  int face;
  float m, p, q;
  if (ax >= ay && ax >= az) {
    face = ux >= 0 ? 0 : 1;
    m = ax, p = uy, q = uz;
  } else if (ay >= az) {
    face = uy >= 0 ? 2 : 3;
    m = ay, p = ux, q = uz;
  } else {
    face = uz >= 0 ? 4 : 5;
    m = az, p = ux, q = uy;
  }
  if (!(m > 1e-30f) || !(m <= 3.4e38f) || p != p || q != q) return -1;
  const float r = __builtin_amdgcn_rcpf(m);
  const float fa = (p * r + 1.0f) * 0.5f * (float)N, fb = (q * r + 1.0f) * 0.5f * (float)N;
  int i = (int)(fa < 0.f ? 0.f : fa), j = (int)(fb < 0.f ? 0.f : fb);
  i = i > N - 1 ? N - 1 : i;
  j = j > N - 1 ? N - 1 : j;
  return (face * N + j) * N + i;
}

__device__ __forceinline__ LgRange lg_range(const LgArgs &lg, int l, D3 hp, D3 lp, bool act) {
  LgRange r{0, 0};
  if (act) {
    const int N = lg.N, cells = 6 * N * N;
    const int c = lg_cell_rcp((float)(hp.x - lp.x), (float)(hp.y - lp.y), (float)(hp.z - lp.z), N);
    if (c < 0) {
      r.cb = -1;
    } else {
      const int32_t *st = lg.start + (size_t)l * (size_t)(cells + 2);
      const int cc = RT_CK(kCkLgStart, c, lg.nstart - 1 - (long long)l * (cells + 2));
      r.cb = st[cc];
      r.ce = st[cc + 1];
    }
  }
  return r;
}

__device__ __forceinline__ int lg_first(const LgArgs &lg, LgRange r) {
  return (r.cb >= 0 && r.ce > r.cb) ? lg.ids[RT_CK(kCkLgId, r.cb, lg.nids)] : 0;
}

// `pre` >= 0: the sphere the shaded point lies on (see below).
__device__ __forceinline__ bool shadow_cells(const SphGeo *__restrict__ g, int n, bool act, D3 o, D3 d, D3 lp,
                                             double dist, const LgArgs &lg, int l, LgRange cell, int id0,
                                             Work &work, int pre = -1) {
  if (__ballot(act) == 0) return false;
  const double a = dot(d, d);
  const double a4 = 4.0 * a, a2 = 2.0 * a;
  const double T = dist < kInf ? dist : kInf;
  const bool fast = a2_ok(a2) && dist == dist && T >= 0x1p-900;
  const double q = a2 * T, qlo = q * (1.0 - 0x1p-48), qhi = q * (1.0 + 0x1p-48);
  bool occ = false;
  auto test = [&](int i) {
    double num;
    const int r = fast ? intersect_num(g[RT_CK(kCkSphere, i, n)], o, d, a4, num, qlo) : 2;
    if (r == 3) {
      occ = true;
    } else if (r == 1) {
      if (num < qlo) occ = true;
      else if (!(num > qhi)) {
        const double t = num / a2;
        occ = t < kInf && t < dist;
      }
    } else if (r == 2) {
      double t;
      occ = intersect(g[i], o, d, a4, a2, t) && t < kInf && t < dist;
    }
  };
  // The lane's own sphere `pre` (the shaded point lies on it) is on almost
  // every list, and its test is decided by the first steps of the
  // reference's arithmetic (sphere.h:29-35, the same roundings as
  // intersect_num), without the square root:
  //  * c < 0, the origin inside the sphere: disc > 0 and the exit root t2 is
  //    in [0, 2.42 |r|] (|oc| <= |r|(1+2u), |b| <= 2|r|(1+6u),
  //    disc <= 8 r^2 (1+15u), so n2 <= 4.83 |r| and t2 <= 2.415 |r|), the
  //    reference's t is t2 (or 0), so with dist^2 > 6 r^2 (and |r| < 1e19,
  //    t < 1e20; r^2 > 1e-200 keeps every term normal) the point is in shadow
  //    (scene.h:78-82) whatever the other spheres give; `fast` (a finite
  //    direction) guards both cases: a NaN direction makes the reference's t
  //    NaN, which is never recorded;
  //  * c > 0 and b > 0 (both roots negative in exact arithmetic): disc < 0
  //    is a miss; 0 < disc < b^2 (1 - 2^-50) makes sqrt(disc) round below
  //    b (b^2 normal), so n2 = -b + sq < 0 and both roots are negative: a miss; the lists
  //    then skip that sphere.  disc == 0 (the negative tangent root the
  //    reference keeps, sphere.h:43-47) and every other case take the test.
  bool self_miss = false;
  if (act && pre >= 0 && fast) {
    const SphGeo s = g[RT_CK(kCkSphere, pre, n)];
    const double ocx = o.x - s.cx, ocy = o.y - s.cy, ocz = o.z - s.cz;
    const double c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - s.rr;
    if (c < 0.0) {
      occ = dist * dist > 6.0 * s.rr && s.rr < 1e38 && s.rr > 1e-200;
    } else if (c > 0.0) {
      const double b = 2.0 * ((ocx * d.x + ocy * d.y) + ocz * d.z);
      const double p = b * b, disc = p - a4 * c;
      self_miss = b > 0.0 && (disc < 0.0 || (disc > 0.0 && p > 1e-290 && disc < p * (1.0 - 0x1p-50)));
    }
  }
  const int skip = self_miss ? pre : -1;
  if (act && !occ) {
    const int N = lg.N, cells = 6 * N * N;
    const int32_t *st = lg.start + (size_t)l * (size_t)(cells + 2);
    // The line o + t d passes (up to rounding) through the light; the grid's
    // margins assume it does within max_off -- checked here, per ray, unless
    // the host has bounded it for the whole scene (off_free: |hit point|,
    // |light| <= B, so the line's distance from the light, as computed here,
    // is below 60 u (4B + 2 EPSILON) + the cross product's rounding, far
    // under 2^-41 (1.01 B + 0.01) <= max_off; tests/native/num_check.cpp)
    bool off_ok = true;
    if (!lg.off_free) {
      const D3 w = sub(lp, o);
      const double off = __builtin_fabs(w.y * d.z - w.z * d.y) + __builtin_fabs(w.z * d.x - w.x * d.z) +
                         __builtin_fabs(w.x * d.y - w.y * d.x);
      off_ok = off <= lg.max_off;
    }
    // the cell's list (first id prefetched), then the global list; a lane
    // whose line cannot use the grid tests every sphere (ids 0 .. n-1) in the
    // same loop
    const bool all = !off_ok || cell.cb < 0;
    const int cl = RT_CK(kCkLgStart, cells, lg.nstart - 1 - (long long)l * (cells + 2));
    const int gb = st[cl], ge = st[cl + 1];
    const int len1 = all ? n : cell.ce - cell.cb, len = all ? n : len1 + (ge - gb);
    int k = 0;
    int nxt = all ? 0 : id0;
    if (!all && len1 == 0 && len > 0) nxt = lg.ids[RT_CK(kCkLgId, gb, lg.nids)];
    while (k < len && !occ) {
      const int i = nxt;
      ++k;
      if (k < len) nxt = all ? k : lg.ids[RT_CK(kCkLgId, k < len1 ? cell.cb + k : gb + (k - len1), lg.nids)];
      if (i != skip) {
        work.exact += 1;
        test(i);
      }
    }
  }
  return act && occ;
}

// Closest hit of camera rays through the camera grid (rt_lightgrid.h
// build_point_grid's cube map and lists, built on the device by
// rt_kernel.hip's cg_*_kernel passes): the rays leave the grid's
// point P exactly, so every sphere the reference's test can report lies on
// the list of the cell of d (spheres containing or nearly containing P are
// on every list, tlo = -inf); a cell's list ascends by a lower bound tlo of
// the sphere's t, so the scan stops at the first entry whose bound exceeds
// the best t found so far (every later entry can only give a larger t: no
// strict-< win, no tie).  The result is the lexicographic (t, index) minimum
// over all spheres, as sweep_closest's.  A lane whose direction cannot be
// binned tests every sphere; a lane whose cell overflowed the builder's K
// slots is told to sweep.
constexpr int kCgSlots = 48;  // entries per cell; a cell with more has its rays sweep
struct CgArgs {
  const int32_t *count;   // [grid][6N^2] entries of each cell (> kCgSlots: overflowed, its rays sweep)
  const int2 *ent;        // [grid][6N^2][kCgSlots] (sphere, tlo bits), ascending by (tlo, index)
  int N;
  int on;         // the launch's frames have grids
  int per_frame;  // 1: frame f scans grid f; 0: every frame grid 0 (one camera position)
  int ngrid;      // (RT_CHECK bound)
};
// The scan of one grid's cell list for the closest hit; this lane's grid
// starts at start + sbase (camera grid: sbase = 0; sphere grids: the grid of
// the sphere the ray leaves).
__device__ __forceinline__ int grid_closest(const SphGeo *__restrict__ g, int n, bool act, D3 o, D3 d,
                                            const int32_t *__restrict__ start, const int2 *__restrict__ ent, int N,
                                            int sbase, long long nstart, long long nent, double &best_t,
                                            Work &work) {
  const double a = dot(d, d);
  const double a4 = 4.0 * a, a2 = 2.0 * a;
  double bt = kInf, bn = __builtin_inf();
  int bi = -1;
  const bool fast = a2_ok(a2);
  int cb = 0, len = 0;
  bool all = false;
  if (act) {
    const int c = lg_cell_rcp((float)d.x, (float)d.y, (float)d.z, N);
    if (c < 0) {
      all = true;
      len = n;
    } else {
      const int cc = RT_CK(kCkCgStart, c, nstart - 1 - sbase);
      cb = start[sbase + cc];
      len = start[sbase + cc + 1] - cb;
    }
  }
  int k = 0;
  int2 e = (len > 0 && !all) ? ent[RT_CK(kCkCgEnt, cb, nent)] : make_int2(0, (int)0xff800000u);  // -inf
  while (k < len) {
    const int i = all ? k : e.x;
    if ((double)__int_as_float(e.y) > bt) break;
    ++k;
    if (k < len && !all) e = ent[RT_CK(kCkCgEnt, cb + k, nent)];  // the next entry, loaded during this test
    work.exact += 1;
    closest_test(g[RT_CK(kCkSphere, i, n)], i, o, d, a4, a2, fast, bt, bn, bi);
  }
  best_t = bt;
  return bi;
}
__device__ __forceinline__ int cam_closest(const SphGeo *__restrict__ g, int n, bool act, D3 o, D3 d,
                                           const CgArgs &cg, int grid, bool &sweep, double &best_t, Work &work) {
  const double a = dot(d, d);
  const double a4 = 4.0 * a, a2 = 2.0 * a;
  double bt = kInf, bn = __builtin_inf();
  int bi = -1;
  sweep = false;
  const bool fast = a2_ok(a2);
  const int cells = 6 * cg.N * cg.N;  // the host keeps grid * cells * kCgSlots below 2^31
  unsigned cb = 0;
  int len = 0;
  bool all = false;
  if (act) {
    const int c = lg_cell_rcp((float)d.x, (float)d.y, (float)d.z, cg.N);
    if (c < 0) {
      all = true;
      len = n;
    } else {
      const unsigned gc = (unsigned)(RT_CK(kCkCgStart, grid, cg.ngrid) * cells + RT_CK(kCkCgStart, c, cells));
      len = cg.count[gc];
      if (len > kCgSlots) {  // overflowed: this lane sweeps
        sweep = true;
        len = 0;
      }
      cb = gc * (unsigned)kCgSlots;
    }
  }
  int k = 0;
  int2 e = (len > 0 && !all) ? cg.ent[RT_CK(kCkCgEnt, cb, (long long)cg.ngrid * cells * kCgSlots)]
                              : make_int2(0, (int)0xff800000u);  // -inf
  while (k < len) {
    const int i = all ? k : RT_CK(kCkSphere, e.x, n);
    if ((double)__int_as_float(e.y) > bt) break;
    ++k;
    if (k < len && !all)  // the next entry, loaded during this test
      e = cg.ent[RT_CK(kCkCgEnt, cb + (unsigned)k, (long long)cg.ngrid * cells * kCgSlots)];
    work.exact += 1;
    closest_test(g[i], i, o, d, a4, a2, fast, bt, bn, bi);
  }
  best_t = bt;
  return bi;
}

// Closest hit of reflection rays through the sphere grids (rt_lightgrid.h
// build_sphere_grids): a ray leaving sphere `key` whose origin lies in the
// ball the grid of `key` was built for (|o - C|^2 <= rho2[key]: checked here
// per ray; rho2 < 0 where there is no grid) scans that grid's cell of d as the
// camera rays scan theirs -- the candidate set holds every sphere the
// reference's test can report for such a ray, with a lower bound of its t.
struct SgArgs {
  const int32_t *start;  // [n][6N^2 + 1]
  const int2 *ent;       // (sphere, tlo bits)
  const double *rho2;    // [n] squared origin-ball radius, < 0: no grid
  int N;
  int on;
  long long nstart, nent;  // CSR starts and list entries (RT_CHECK bounds)
  int nsph;                // spheres (RT_CHECK bound of the grid key)
};
__device__ __forceinline__ bool sg_usable(const SphGeo *__restrict__ g, const SgArgs &sg, bool act, D3 o, int key) {
  if (!act || key < 0) return false;
  const int k = RT_CK(kCkSgKey, key, sg.nsph);
  const SphGeo s = g[k];
  const double ox = o.x - s.cx, oy = o.y - s.cy, oz = o.z - s.cz;
  return (ox * ox + oy * oy) + oz * oz <= sg.rho2[k];
}

struct Cam {
  double px, py, pz, fx, fy, fz, rx, ry, rz, ux, uy, uz, scale;
};
struct Rows {
  int band, first, stride, count;
};

__device__ __forceinline__ int quantize(double c) {
  double m = 255.99 * min1(c);  // main.cpp:85
  return (int)m;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned v) {
  unsigned long long s = v;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  return s;
}

__device__ __forceinline__ unsigned long long wave_sum64(unsigned long long s) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  return s;
}

}  // namespace rtk
