// rt_kernel.hip -- gfx950 (MI355X / CDNA4) render loop + device half of the C-ABI.
//
// One lane per pixel, wave64 over an 8x8 pixel tile, 256-thread workgroups
// (2x2 waves = 16x16 pixels).  Sphere geometry (cx,cy,cz,r*r as fp64, 32 B) and
// the light list are staged into LDS per workgroup and read as wave-uniform
// broadcasts; materials (48 B) are read from global memory only on a hit.
// Shadow rays exit early once no lane of the wave is still unoccluded
// (__ballot).  Reflections are walked iteratively; each level's
// (shade*(1-refl), refl) is pushed on a per-lane stack and unwound at the end,
// which reproduces the reference recursion's rounding exactly.
//
// Numerics follow the serial fp64 path operation by operation:
// vec3.h:13-33, ray.h:12, camera.h:17-25, sphere.h:26-64, scene.h:41-121,
// main.cpp:16-58 and the quantiser main.cpp:85-87.  Build with
// -ffp-contract=off (also forced below): no FMA contraction, IEEE division and
// sqrt, so the output bytes equal ray_serial's.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <string>

#include "rt_hip.h"

#pragma clang fp contract(off)

#include "rt_device.h"
#include "rt_cgbuild.h"
#include "rt_sched.h"

#include <chrono>
#include <cmath>
#include <vector>

namespace rtk {

#ifdef RT_STAMPS
// Diagnostic timeline: per wave {start, end} (s_memrealtime, 100 MHz) and
// {HW_ID, XCC_ID}; dumped by rt_render_stats when RT_HIP_STAMPS_FILE is set.
constexpr int kTimelineWaves = 1 << 17;
constexpr int kTl = 16;  // u64 per wave
__device__ unsigned long long g_timeline[kTimelineWaves * kTl];
#endif


// Output of a launch.  RT_FB_RGB8 with full = 0: rows.count x W RGB8 (the
// rows of `rows`, rt_render); RT_FB_RGB8 with full = 1: a W x H RGB8 image in
// PPM row order; RT_FB_F32X3 / RT_FB_F64X3: the reference's framebuffer,
// index j*W + x with j = 0 the bottom row (src/main.cpp:156, kernel.cu:112),
// unquantised.  Pixels x0 <= x < x0 + xw are written.  Frame f of a
// multi-frame launch (RT_FB_RGB8, full = 0) starts fstride bytes after frame f-1.
struct OutDesc {
  void *ptr;
  int fmt, full, x0, xw;
  long long fstride;
};

// A queued ray of the merged levels (merge_tiles' LDS queue, render_deferred's
// global queue): origin, direction, stack level, depth left, the sphere it
// leaves, and its pixel.
struct QRay {  // 64 B
  double ox, oy, oz, dx, dy, dz;
  int orig, dleft, key, pix;
};
// All arguments of render_kernel in one struct: its only kernel parameter, so
// it sits at offset 0 of the kernarg segment and a member can be re-read from
// there by offsetof (kernarg_late).
struct RenderArgs {
  const SphGeo *geo;
  const double *radius;
  const SphMat *mat;
  const LightD *lights;
  int n, nl;
  D3 amb;
  Cam cam[RT_MAX_FRAMES];  // frame f's camera (rt_render_frames_async); cam[0] otherwise
  int frames;              // frames of this launch: launch slot b renders frame b % frames of tile slot b / frames
  int W, H, depth;
  Rows rows;
  BvhArgs bv;
  LgArgs lg;
  CgArgs cg;  // camera grid of the launch's (shared) camera position; cg.on = 0: none
  SgArgs sg;  // sphere grids (reflection rays); sg.on = 0: none
  OutDesc od;
  StackEnt *gstack;               // kStackGlobal: [depth-1][launch pixels]
  StackEnt *homes;                // kStackMerge: [home][depth-1][kMergeTiles * 64] (a wave's group of tiles)
  unsigned long long *home_bits;  // kStackMerge: the homes taken (a bit each)
  int home_words;                 // kStackMerge: 64-bit words of home_bits
  StackEnt *dstack;               // kStackMerge: deferred rays' stacks, [depth-1][kShards * dq_cap]
  unsigned long long *counters;
  int ntx, ntiles;
  int nslots;                     // wave slots per frame: kStackMerge tile groups, kStackGlobal with perm
                                  // the listed blocks, else ntiles
  const int *perm;
  unsigned long long *zero_next;  // counters of the next launch, zeroed by workgroup 0 (or nullptr)
  QRay *dq;                       // kStackMerge: deferred deep rays, [kShards][dq_cap] (render_deferred)
  int dq_cap;                     // entries per shard segment; 0 = no deferral
  int merge_q;                    // kStackMerge: LDS ray-queue entries per wave (16..64)
  int nsingle;                    // kStackMerge: the first nsingle tile slots (heaviest class) get a wave each
  int merge_end;                  // kStackMerge: slots [nsingle, merge_end) go kMergeTiles per wave, the rest
                                  // (the launch's tail: its lightest tiles) one per wave again
  int pix_off;                    // kStackMerge: LDS offset of the wave's finished pixels (flush_tile)
  int rows_dword;                 // kStackMerge: every 8-pixel tile row starts dword aligned (flush_tile)
  int defer_level;                // kStackMerge: rays of this reflection level and deeper are deferred
  int xcd_frames;                 // multi-frame launches: every frame of a tile group on one XCD (render_kernel)
};
// the whole struct is the kernel's argument block (kernarg segment, at most 4 KiB)
static_assert(sizeof(RenderArgs) <= 4096, "RenderArgs exceeds the kernel-argument segment");

// Member `x` (at offset kOff of RenderArgs) re-read from the kernarg segment
// here.  Kernel arguments are otherwise loaded into SGPRs at entry and live
// for the whole kernel; the big loop-invariant ones (BVH and light-grid
// descriptors) then spill to VGPR lanes, paid for with v_readlane /
// v_writelane in the level and light loops.  The empty asm makes the kernarg
// pointer opaque, so the scalar loads happen at this point and their
// registers are free again afterwards.  kLate = false returns x itself.
template <bool kLate, size_t kOff, class T>
__device__ __forceinline__ const T &kernarg_late(const T &x);

// Frame f's camera, read from the kernarg segment (a dynamic index into the
// by-value kernel argument would copy the array to scratch).
__device__ __forceinline__ const Cam &kernarg_cam(int f) {
  typedef const __attribute__((address_space(4))) unsigned char KB;
  KB *p = (KB *)__builtin_amdgcn_kernarg_segment_ptr();
  return *(const Cam *)(p + offsetof(RenderArgs, cam) + (size_t)f * sizeof(Cam));
}

template <bool kLate, size_t kOff, class T>
__device__ __forceinline__ const T &kernarg_late(const T &x) {
  if constexpr (!kLate) {
    return x;
  } else {
    typedef const __attribute__((address_space(4))) unsigned char KB;
    KB *p = (KB *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const T *)(p + kOff);
  }
}

// One bounce of trace_ray (src/main.cpp:16-58) for the wave's `alive` lanes:
// closest hit, sky on a miss, Phong shading with per-light shadow queries,
// and the reflection decision (main.cpp:43-55).  Outcome per alive lane:
// kEnded (colour = the level's final colour: sky, shade, or shade*(1-refl)
// when no depth is left) or kSpawned (colour = shade*(1-refl), refl, and the
// reflection ray no/nd leaving sphere nkey).  Wave-uniform control flow.
enum { kEnded = 1, kSpawned = 2 };

// kArgMem: bv and lg are the kernel's own arguments (kernarg segment), so they
// are re-read where needed (kernarg_late) instead of held in SGPRs throughout.
// kFast: only the default paths (ordered 4-wide BVH walk, light-grid shadow
// queries) are compiled in; the host picks it when the scene uses them.
// The part of bounce() after the closest hit (bi, bt) is known: sky or
// shading with the shadow queries, and the reflection decision.  Lanes with
// alive = false take no part; it has no wave-wide operation that needs every
// lane active (render_deferred_walk calls it for the lanes whose walk ended).
// Position of the k-th (from 0) set bit of m (k < popcount(m)).
__device__ __forceinline__ int nth_set_bit(unsigned long long m, int k) {
  int pos = 0;
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) {
    const unsigned long long low = m & ((1ull << s) - 1ull);
    const int c = __popcll(low);
    if (k >= c) {
      k -= c;
      m >>= s;
      pos += s;
    } else {
      m = low;
    }
  }
  return pos;
}

// kWide (one-frame launches): a wave whose hit lanes are at most half of it
// spreads the light loop over the lanes -- in passes of lpp = 64 / hits lights,
// lane j handles light l0 + j % lpp of the (j / lpp)-th hit lane: its shadow
// query and Phong terms, computed with the same operands and operations as the
// loop below (the hit lane's normal and view direction passed over) -- and each
// hit lane then adds its lights' terms in file order (scene.h:117): the same
// bits, in ceil(lights / lpp) passes instead of one per light.
template <bool kCull, bool kArgMem = false, bool kFast = false, bool kWide = false>
__device__ __forceinline__ void shade_hit(const SphGeo *__restrict__ g, const double *__restrict__ rad,
                                          const SphMat *__restrict__ mat, const LightD *__restrict__ slight, int n,
                                          int nl, D3 amb, const BvhArgs &bv, const LgArgs &lg_arg, bool alive, D3 o,
                                          D3 d, int key, int dleft, int bi, double bt, Work &work, unsigned &c_shadow,
                                          int &outcome, D3 &color, double &refl, D3 &no, D3 &nd, int &nkey) {
  outcome = 0;
  const bool hit = alive && bi >= 0;
  if (alive && !hit) {  // sky, main.cpp:26-30
    const double st = 0.5 * (d.y + 1.0);
    color = add(scale(mk(1.0, 1.0, 1.0), 1.0 - st), scale(mk(0.5, 0.7, 1.0), st));
    outcome = kEnded;
  }
  const int hi = RT_CK(kCkSphere, hit ? bi : 0, n > 0 ? n : 1);
  const D3 hp = add(o, scale(d, bt));                            // main.cpp:32
  D3 col;
  {
    const SphMat m0 = mat[hi];
    col = mul(amb, mk(m0.cr, m0.cg, m0.cb));                   // scene.h:91
  }
  // the normal (sphere.h:62-64), used by the shading and by the reflection
  // (main.cpp:44-46: the same expression, formed once), and the view direction
  D3 nrm = mk(0.0, 0.0, 0.0), view = nrm;
  if (hit) {
    const SphGeo sg = g[hi];
    nrm = normalized(sub(hp, mk(sg.cx, sg.cy, sg.cz)));
    view = normalized(sub(o, hp));  // main.cpp:38
  }
    // scene.h:94-120: per light in file order, the shadow query then (if lit)
    // the Phong terms with the same ldir -- skipped by a wave (or the active
    // lanes of one) whose rays all left the scene
    bool wide_done = false;
    if constexpr (kWide && kFast) {
      const unsigned long long hm = __ballot(hit);
      const int nh = __popcll(hm);
      const LgArgs &lgw = kernarg_late<kArgMem, offsetof(RenderArgs, lg)>(lg_arg);
      const int lpp = nh ? (64 / nh < nl ? 64 / nh : nl) : 0;  // lights per pass
      if (nl >= 2 && lpp >= 2 && lgw.on) {                   // wave-uniform
        const int lane = (int)(threadIdx.x & 63);
        const int rank = (int)__popcll(hm & ((1ull << lane) - 1ull));
        for (int l0 = 0; l0 < nl; l0 += lpp) {  // lights l0 .. l0 + cnt - 1 in this pass
          const int cnt = nl - l0 < lpp ? nl - l0 : lpp;
          const bool helper = lane < nh * cnt;
          const int r = helper ? lane / cnt : 0, lh = l0 + (helper ? lane - r * cnt : 0);
          const int src = nth_set_bit(hm, r);
          // the owner's hit point, sphere, normal and view direction
          const D3 hq = mk(__shfl(hp.x, src, 64), __shfl(hp.y, src, 64), __shfl(hp.z, src, 64));
          const D3 nq = mk(__shfl(nrm.x, src, 64), __shfl(nrm.y, src, 64), __shfl(nrm.z, src, 64));
          const D3 vq = mk(__shfl(view.x, src, 64), __shfl(view.y, src, 64), __shfl(view.z, src, 64));
          const int hq_i = RT_CK(kCkSphere, __shfl(hi, src, 64), n > 0 ? n : 1);
          D3 t = mk(0.0, 0.0, 0.0);
          bool lit = false;
          {
            const SphMat m = mat[hq_i];
            const D3 mc = mk(m.cr, m.cg, m.cb);
            const LightD L = slight[lh];
            const D3 lp = mk(L.px, L.py, L.pz);
            const LgRange cell = lg_range(lgw, lh, hq, lp, helper);
            const int id0 = lg_first(lgw, cell);
            const D3 to_light = sub(lp, hq);
            const double dist = length(to_light);
            const D3 ldir = normalized(to_light);
            const D3 so = add(hq, scale(ldir, kEps)), sd = renormalized(ldir);
            const bool occ = shadow_cells(g, n, helper, so, sd, lp, dist, lgw, lh, cell, id0, work, hq_i);
            if (helper && !occ) {  // the terms of the loop below, same operands and order
              const double ndl = max0(dot(nq, ldir));
              const D3 diffuse = scale(scale(mc, 1.0 - m.refl), ndl);
              const D3 nl2 = scale(ldir, -1.0);
              const D3 rdir = sub(nl2, scale(scale(nq, 2.0), dot(nl2, nq)));
              const double rdv = max0(dot(rdir, vq));
              double spec = 0.0;
              int ipow = 0;
              if (!(rdv == 0.0 && m.shin > 0.0))
                spec = int_pow_ok(rdv, m.shin, ipow) ? int_pow(rdv, ipow) : pow_call(rdv, m.shin);
              const D3 specular = scale(scale(mk(L.cr, L.cg, L.cb), kSpec), spec);
              t = add(specular, diffuse);
              lit = true;
            }
          }
          // each hit lane adds this pass's lights' terms in file order (scene.h:117)
          const unsigned long long litm = __ballot(lit);
          for (int l = 0; l < cnt; ++l) {
            const int sl = hit ? rank * cnt + l : 0;
            const D3 tl = mk(__shfl(t.x, sl, 64), __shfl(t.y, sl, 64), __shfl(t.z, sl, 64));
            if (hit && ((litm >> sl) & 1ull)) col = add(tl, col);
          }
        }
        wide_done = true;
      }
    }
    if (!wide_done && __ballot(hit)) {
      const SphMat m = mat[hi];
      const D3 mc = mk(m.cr, m.cg, m.cb);
      LgRange next{0, 0};
      {
        const LgArgs &lg0 = kernarg_late<kArgMem, offsetof(RenderArgs, lg)>(lg_arg);
        if (lg0.on && nl > 0) next = lg_range(lg0, 0, hp, mk(slight[0].px, slight[0].py, slight[0].pz), hit);
      }
      for (int l = 0; l < nl; ++l) {
        const LgArgs &lg = kernarg_late<kArgMem, offsetof(RenderArgs, lg)>(lg_arg);
        RT_T0(t_setup);
        // this light's first list id, and the next light's cell range, are
        // loaded now and consumed after the setup arithmetic below
        const LgRange cell = next;
        const int id0 = lg.on ? lg_first(lg, cell) : 0;
        if (lg.on && l + 1 < nl) next = lg_range(lg, l + 1, hp, mk(slight[l + 1].px, slight[l + 1].py, slight[l + 1].pz), hit);
        const LightD L = slight[l];
        const D3 lp = mk(L.px, L.py, L.pz);
        const D3 to_light = sub(lp, hp);
        const double dist = length(to_light);
        const D3 ldir = normalized(to_light);
        const bool need = hit;
        RT_ACC(work, 3, t_setup);
        RT_T0(t_sh);
        bool occ = false;
        if (__ballot(need)) {
          const D3 so = add(hp, scale(ldir, kEps)), sd = renormalized(ldir);
          if constexpr (kFast) {
            occ = shadow_cells(g, n, need, so, sd, lp, dist, lg, l, cell, id0, work, hi);
          }
          else
            occ = lg.on ? shadow_cells(g, n, need, so, sd, lp, dist, lg, l, cell, id0, work, hi)
                        : sweep_shadow<kCull>(g, rad, n, need, so, sd, lp, hi, dist,
                                              kernarg_late<kArgMem, offsetof(RenderArgs, bv)>(bv), work);
        }
        RT_ACC(work, 9, t_sh);
        RT_T0(t_shade);
        if (hit && !occ) {
          const double ndl = max0(dot(nrm, ldir));
          const D3 diffuse = scale(scale(mc, 1.0 - m.refl), ndl);
          const D3 nl2 = scale(ldir, -1.0);
          const D3 rdir = sub(nl2, scale(scale(nrm, 2.0), dot(nl2, nrm)));  // reflect(), vec3.h:31-33
          const double rdv = max0(dot(rdir, view));
          // pow(+0, y > 0) is +0 exactly (C99 F.10.4.4), so most lanes skip ocml's pow.
          double spec = 0.0;
          int ipow = 0;
          if (!(rdv == 0.0 && m.shin > 0.0))
            spec = int_pow_ok(rdv, m.shin, ipow) ? int_pow(rdv, ipow) : pow_call(rdv, m.shin);
          const D3 specular = scale(scale(mk(L.cr, L.cg, L.cb), kSpec), spec);
          col = add(add(specular, diffuse), col);                  // scene.h:117
        }
        RT_ACC(work, 4, t_shade);
      }
    }
  if (hit) {
    c_shadow += (unsigned)nl;
    const SphMat m = mat[hi];
    if (m.refl > 0.0) {                                         // main.cpp:43-55
      const double w = 1.0 - m.refl;
      const D3 A = mk(col.x * w, col.y * w, col.z * w);
      color = A;  // with no depth left trace_ray(depth 0) is black: A + (0,0,0)*refl == A
      outcome = kEnded;
      if (dleft - 1 >= 1) {
        const D3 rd = sub(d, scale(scale(nrm, 2.0), dot(d, nrm)));
        no = add(hp, scale(nrm, kEps));
        nd = renormalized(rd);
        nkey = hi;
        refl = m.refl;
        outcome = kSpawned;
      }
    } else {
      color = col;
      outcome = kEnded;
    }
  }
}

// The closest hit of bounce() (scene.h:41-61) for the `alive` lanes: sphere
// index (-1: none) and t.  Wave-uniform control flow.
template <bool kCull, bool kArgMem = false, bool kFast = false>
__device__ __forceinline__ int closest_hit(const SphGeo *__restrict__ g, const double *__restrict__ rad, int n,
                                           const BvhArgs &bv, bool alive, D3 o, D3 d, int key, Work &work,
                                           double &bt_out, bool cam_pass = false, int frame = 0) {
  double bt = kInf;
  RT_T0(t_cl);
  int bi = -1;
  // cam_pass (kFast merged kernels, wave-uniform): every alive lane holds a
  // camera ray of a frame whose position is the camera grid's point.  The
  // lanes a grid cannot serve (`rest`) take the one sweep below.
  bool rest = alive;
  if constexpr (kFast && kArgMem) {
    if (cam_pass) {
      const CgArgs &cg = kernarg_late<true, offsetof(RenderArgs, cg)>(CgArgs{});
      bi = cam_closest(g, n, alive, o, d, cg, cg.per_frame ? frame : 0, rest, bt, work);
    } else if (kernarg_late<true, offsetof(RenderArgs, sg)>(SgArgs{}).on) {
      // reflection rays through the sphere grid of the sphere they leave; the
      // lanes whose origin fails the grid's check sweep as before
      bool grid;
      {
        const SgArgs &sg = kernarg_late<true, offsetof(RenderArgs, sg)>(SgArgs{});
        grid = sg_usable(g, sg, alive, o, key);
      }
      if (__ballot(grid)) {
        const SgArgs &sg = kernarg_late<true, offsetof(RenderArgs, sg)>(SgArgs{});
        bi = grid_closest(g, n, grid, o, d, sg.start, sg.ent, sg.N, grid ? key * (6 * sg.N * sg.N + 1) : 0, sg.nstart,
                          sg.nent, bt, work);
      }
      rest = alive && !grid;
    }
  }
  if (__ballot(rest)) {
    double bt2 = kInf;
    const int bi2 = sweep_closest<kCull, kFast>(g, rad, n, rest, o, d, key,
                                                kernarg_late<kArgMem, offsetof(RenderArgs, bv)>(bv), bt2, work);
    if (rest) {
      bi = bi2;
      bt = bt2;
    }
  }
  RT_ACC(work, 8, t_cl);
  bt_out = bt;
  return bi;
}

template <bool kCull, bool kArgMem = false, bool kFast = false, bool kWide = false>
__device__ __forceinline__ void bounce(const SphGeo *__restrict__ g, const double *__restrict__ rad,
                                       const SphMat *__restrict__ mat, const LightD *__restrict__ slight, int n,
                                       int nl, D3 amb, const BvhArgs &bv, const LgArgs &lg_arg, bool alive, D3 o, D3 d,
                                       int key, int dleft, Work &work, unsigned &c_shadow, int &outcome, D3 &color,
                                       double &refl, D3 &no, D3 &nd, int &nkey, bool cam_pass = false) {
  double bt;
  const int bi = closest_hit<kCull, kArgMem, kFast>(g, rad, n, bv, alive, o, d, key, work, bt, cam_pass);
  shade_hit<kCull, kArgMem, kFast, kWide>(g, rad, mat, slight, n, nl, amb, bv, lg_arg, alive, o, d, key, dleft, bi, bt,
                                          work, c_shadow, outcome, color, refl, no, nd, nkey);
}

// trace_ray for one camera ray per lane, the wave walking the levels together
// (lanes masked by `alive`); the lane's reflection stack entries are
// sbase[sidx + level * sstride] (depth - 1 levels), unwound innermost first.
// The wave-uniform base and a 32-bit lane index (not a per-lane 64-bit
// pointer) keep the stack address out of the registers that spill.
// kPark: a lane's final colour is parked in LDS (park[lane], this wave's
// slice) when its chain ends instead of being held in registers while the
// wave's other lanes keep bouncing (6 VGPRs fewer in the level loop).
template <bool kCull, bool kArgMem = false, bool kPark = false>
__device__ __forceinline__ D3 trace_wave(const SphGeo *__restrict__ g, const double *__restrict__ rad,
                                         const SphMat *__restrict__ mat, const LightD *__restrict__ slight, int n,
                                         int nl, D3 amb, int depth, const BvhArgs &bv, const LgArgs &lg, bool live,
                                         D3 o, D3 d, StackEnt *sbase, unsigned sidx, unsigned sstride, Work &work, unsigned &c_prim,
                                         unsigned &c_shadow, unsigned &c_reflect, D3 *park = nullptr) {
  int lev = 0;
  int dleft = depth;
  D3 res = mk(0.0, 0.0, 0.0);     // depth <= 0 -> black (main.cpp:17-18)
  bool alive = live && depth >= 1;
  const bool traced = alive;
  int key = -1;  // sphere the current ray leaves (-1: camera), groups lanes in sweeps
  c_prim += alive ? 1u : 0u;
  while (__ballot(alive)) {
    int outcome, nkey = 0;
    D3 color = kPark ? mk(0.0, 0.0, 0.0) : res, no = o, nd = d;
    double refl = 0.0;
    bounce<kCull, kArgMem>(g, rad, mat, slight, n, nl, amb, bv, lg, alive, o, d, key, dleft, work, c_shadow, outcome,
                           color, refl, no, nd, nkey);
    if (alive) {
      if (outcome == kSpawned) {
        sbase[RT_CK(kCkStack, sidx + (unsigned)lev * sstride, (long long)(depth - 1) * sstride)] =
            StackEnt{color.x, color.y, color.z, refl};
        ++lev;
        o = no;
        d = nd;
        key = nkey;
        --dleft;
        ++c_reflect;
      } else {
        if (kPark) park[threadIdx.x & 63] = color;
        else res = color;
        alive = false;
      }
    }
  }
  if (kPark && traced) res = park[threadIdx.x & 63];
  while (lev > 0) {  // unwind: shade*(1-refl) + reflected*refl, innermost first
    --lev;
    const StackEnt e = sbase[RT_CK(kCkStack, sidx + (unsigned)lev * sstride, (long long)(depth - 1) * sstride)];
    res = mk(e.ax + res.x * e.refl, e.ay + res.y * e.refl, e.az + res.z * e.refl);
  }
  return res;
}

// One 8x8 tile of pixels, one lane per pixel; `samples` = 1 (the serial
// path) or 4 (main_gpu.cu:249-333's antialias offsets, in fp64 serial
// semantics: samples summed in order, then * 0.25).  Adds the tile's ray
// counts to the wave sums.
struct CompactArgs {
  D3 *park;          // kStackGlobal with kernarg-resident arguments: this wave's parked colours (LDS)
  StackEnt *gstack;  // [depth-1][npx]
  size_t npx;        // level stride: pixels of all frames of the launch
  unsigned fpx;      // this wave's frame's first stack entry (frame * pixels per frame)
};

// Reflection stack placement: kStackGlobal = [level][pixel] in global memory
// (any depth, one tile per wave: trace_wave); kStackMerge = the same stack with
// merged reflection levels (merge_tiles, below).
enum { kStackGlobal = 1, kStackMerge = 4 };
template <bool kCull, int kSamples, int kStack, bool kArgMem = false>
__device__ __forceinline__ void trace_tile(const SphGeo *__restrict__ g, const double *__restrict__ rad,
                                           const SphMat *__restrict__ mat, const LightD *__restrict__ slight, int n,
                                           int nl, D3 amb, const Cam &cam, int W_arg, int H_arg, int depth,
                                           const Rows &rows_arg, const BvhArgs &bv, const LgArgs &lg,
                                           const OutDesc &od_arg, int x0, int k0, const CompactArgs &ca, Work &work,
                                           unsigned long long (&sums)[4], int frame = 0) {
  const int W = W_arg, H = H_arg;
  const Rows &rows = rows_arg;
  const OutDesc &od = od_arg;
  const int lane = threadIdx.x & 63;
  const int x = x0 + (lane & 7);
  const int k = k0 + (lane >> 3);
  const bool in_tile = x < W && x < od.x0 + od.xw && k < rows.count;
  const long long y = (long long)(k / rows.band) * rows.band * rows.stride + (long long)rows.first * rows.band +
                      (k % rows.band);
  const bool in_img = in_tile && y < H;
  const int j = H - 1 - (int)(in_img ? y : 0);  // reference row (main.cpp:74)
  unsigned c_prim = 0, c_shadow = 0, c_reflect = 0, c_neg = 0;
  D3 acc = mk(0.0, 0.0, 0.0);
#pragma unroll 1
  for (int s = 0; s < kSamples; ++s) {
    // Camera ray, camera.h:17-25 and main.cpp:151-154: ((u-0.5)*scale)*aspect,
    // aspect = 1.0; antialias offsets main_gpu.cu:253-256 (x + 0.0 == x exactly)
    const double ox = (double)(s & 1) * 0.5, oy = s >= 2 ? 0.5 : 0.0;
    const double u = ((double)x + ox) / (W - 1), v = ((double)j + oy) / (H - 1);
    const double su = ((u - 0.5) * cam.scale) * 1.0, sv = (v - 0.5) * cam.scale;
    const D3 dir = add(add(mk(cam.fx, cam.fy, cam.fz), scale(mk(cam.rx, cam.ry, cam.rz), su)),
                       scale(mk(cam.ux, cam.uy, cam.uz), sv));
    const D3 d = renormalized(normalized(dir));  // get_ray normalises, Ray() normalises again
    const D3 o = mk(cam.px, cam.py, cam.pz);
    const int pix = k * od.xw + (x - od.x0);
    const D3 c = trace_wave<kCull, kArgMem, kArgMem>(g, rad, mat, slight, n, nl, amb, depth, bv, lg, in_img, o, d,
                                                     ca.gstack, (unsigned)pix + ca.fpx, (unsigned)ca.npx, work,
                                                     c_prim, c_shadow, c_reflect, ca.park);
    acc = kSamples == 1 ? c : add(acc, c);  // serial: the colour itself; AA: from 0 in sample order (main_gpu.cu:250, 327)
  }
  const D3 res = kSamples == 4 ? scale(acc, 0.25) : acc;  // main_gpu.cu:331, 1/4 is exact
  // The pixel's coordinates are recomputed from the lane id (mbcnt) rather
  // than kept live across the trace, which would spill them to scratch; the
  // output descriptors are re-read from the kernarg segment (kArgMem).
  {
    const OutDesc &od = kernarg_late<kArgMem, offsetof(RenderArgs, od)>(od_arg);
    const Rows &rows = kernarg_late<kArgMem, offsetof(RenderArgs, rows)>(rows_arg);
    const int W = kernarg_late<kArgMem, offsetof(RenderArgs, W)>(W_arg);
    const int H = kernarg_late<kArgMem, offsetof(RenderArgs, H)>(H_arg);
    const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    const int x = x0 + (lane & 7);
    const int k = k0 + (lane >> 3);
    const bool in_tile = x < W && x < od.x0 + od.xw && k < rows.count;
    const long long y = (long long)(k / rows.band) * rows.band * rows.stride + (long long)rows.first * rows.band +
                        (k % rows.band);
    const bool in_img = in_tile && y < H;
    const int j = H - 1 - (int)(in_img ? y : 0);
  if (od.fmt == RT_FB_RGB8) {
    // RGB8: a tile row of 8 pixels is 24 contiguous bytes.  When the whole row
    // is written and dword aligned, lanes 0-5 of the row store it as 6 dwords
    // assembled with two shuffles; otherwise every lane stores its 3 bytes.
    unsigned v = 0;  // r | g << 8 | b << 16
    if (in_img) {
      const int q0 = quantize(res.x), q1 = quantize(res.y), q2 = quantize(res.z);
      c_neg = (q0 < 0) + (q1 < 0) + (q2 < 0);
      v = (unsigned)(q0 < 0 ? 0 : q0) | (unsigned)(q1 < 0 ? 0 : q1) << 8 | (unsigned)(q2 < 0 ? 0 : q2) << 16;
    }
    const bool put = in_tile && (in_img || !od.full);  // padding rows of a shard are zero-filled
    const int c = lane & 7, rb = lane & ~7;
    const unsigned long long rowmask = 0xFFull << rb;
    const bool whole = (__ballot(put) & rowmask) == rowmask;
    uint8_t *row = static_cast<uint8_t *>(od.ptr) + (size_t)frame * (size_t)od.fstride +
                   ((size_t)(od.full ? y : k) * W + (x - c)) * 3;
    const bool packed = whole && ((reinterpret_cast<uintptr_t>(row) & 3u) == 0);
    const int p0 = (4 * c) / 3;  // dword c holds bytes 4c..4c+3: pixels p0, p0+1
    const unsigned v0 = __shfl(v, rb + (p0 < 7 ? p0 : 7), 64), v1 = __shfl(v, rb + (p0 + 1 < 7 ? p0 + 1 : 7), 64);
    if (packed) {
      if (c < 6) {
        const unsigned long long both = (unsigned long long)v0 | (unsigned long long)v1 << 24;
        reinterpret_cast<unsigned *>(row)[c] = (unsigned)(both >> (8 * (4 * c - 3 * p0)));
      }
    } else if (put) {
      uint8_t *px = row + c * 3;
      px[0] = (uint8_t)v;
      px[1] = (uint8_t)(v >> 8);
      px[2] = (uint8_t)(v >> 16);
    }
  } else if (in_tile && in_img) {
    const size_t i = ((size_t)j * W + x) * 3;
    if (od.fmt == RT_FB_F64X3) {
      double *f = static_cast<double *>(od.ptr) + i;
      f[0] = res.x;
      f[1] = res.y;
      f[2] = res.z;
    } else {
      float *f = static_cast<float *>(od.ptr) + i;
      f[0] = (float)res.x;
      f[1] = (float)res.y;
      f[2] = (float)res.z;
    }
  }
  }
  sums[0] += wave_sum(c_prim);
  sums[1] += wave_sum(c_shadow);
  sums[2] += wave_sum(c_reflect);
  sums[3] += wave_sum(c_neg);
}

// kStackMerge: one wave traces kMergeTiles tiles and merges their reflection
// rays before tracing them.  Level 0 runs tile by tile (one lane per pixel,
// coherent); a pixel whose chain ends there is stored at once.  The rays it
// spawns (typically a handful per tile: 0.34 M reflection rays for 2.07 M
// pixels on synth200) wait in a per-wave LDS queue (< 64 entries) until a
// tile's spawns and the queue fill a wave: then those 64 rays run their
// remaining levels together (chain), each lane unwinding its own pixel's
// [level][pixel] stack and storing it.  So the incoherent levels cost one
// wave pass per 64 rays instead of one per tile that has any: measured per
// reflection level, level 2 of synth200 (41 K rays) cost 0.047 ms and level 3
// (8 K rays) 0.021 ms with one tile per wave.  No barriers: the wave is its
// own workgroup.  RGB8 row-compact output, one sample per pixel.
#ifndef RT_MERGE_TILES
#define RT_MERGE_TILES 4
#endif
constexpr int kMergeTiles = RT_MERGE_TILES;
// Rays of reflection level >= kDeferLevel leave the merged megakernel for
// render_deferred, a second kernel over all deferred rays of the launch; the
// per-shard count lives in u64 slot kDeferSlot of the launch's counter shards.
#ifndef RT_DEFER_LEVEL
#define RT_DEFER_LEVEL 2
#endif
constexpr int kDeferLevel = RT_DEFER_LEVEL;
#ifndef RT_DEFER_WGS
#define RT_DEFER_WGS 48  // render_deferred workgroups (one wave each) per shard segment
#endif
#ifndef RT_DEFER_CAP_DIV
#define RT_DEFER_CAP_DIV 8  // deferred-queue room: 1 / RT_DEFER_CAP_DIV of the launch's pixels
#endif
constexpr int kDeferSlot = 7;
// merge_tiles' LDS: the finished pixels (RGB8, 192 B per tile), then the tile ids
constexpr size_t kPixbufIds = (size_t)kMergeTiles * 64 * 3;
constexpr size_t kPixbufBytes = kPixbufIds + (size_t)kMergeTiles * 8;  // + (tile id, row-0 offset) per tile
// u64 slot of a counter shard: the deferred kernels' next queue entry of that
// shard segment (lanes take entries dynamically; zeroed with the launch's counters)
constexpr int kFetchSlot = 24;
constexpr long long kSchedMinTiles = 1024;  // launches with fewer 8x8 tiles keep scanline order

// A pixel's final colour quantised as write_ppm (main.cpp:85), packed r | g << 8 | b << 16.
__device__ __forceinline__ unsigned pack_px(D3 c, unsigned &c_neg) {
  const int q0 = quantize(c.x), q1 = quantize(c.y), q2 = quantize(c.z);
  c_neg += (q0 < 0) + (q1 < 0) + (q2 < 0);
  return (unsigned)(q0 < 0 ? 0 : q0) | (unsigned)(q1 < 0 ? 0 : q1) << 8 | (unsigned)(q2 < 0 ? 0 : q2) << 16;
}

// A deferred ray's pixel (render_deferred*): its 3 bytes at out + 3 pix are
// OR-ed into the one or two dwords that hold them.  merge_tiles stored the
// pixel's tile as dword rows with zero bytes in this pixel's place, and the
// neighbours in those dwords may be other deferred pixels being OR-ed at the
// same time: a dword atomic OR per covered dword, no byte stores.
__device__ __forceinline__ void or_px(uint8_t *out, unsigned pix, unsigned v) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(out) + (uintptr_t)pix * 3;
  unsigned *d = reinterpret_cast<unsigned *>(a & ~(uintptr_t)3);
  const unsigned sh = (unsigned)(a & 3) * 8;
  const unsigned long long w = (unsigned long long)v << sh;  // bytes sh/8 .. sh/8 + 2 of a dword pair
  if ((unsigned)w) atomicOr(d, (unsigned)w);
  if (sh > 8 && (unsigned)(w >> 32)) atomicOr(d + 1, (unsigned)(w >> 32));
}

// kMergeTiles tiles of one frame for one wave (see kStackMerge).  Every lane
// holds at most one ray: (o, d, key = the sphere it leaves, dleft = depth
// left, pix, lev = stack entries its pixel has).  One bounce() per iteration
// for all lanes holding a ray:
//   * a tile pass loads the next tile's camera rays into all lanes (level 0);
//     the reflection rays it spawns join the queue unless they and the queue
//     fill the wave (or no tile is left), then the queued rays fill the lanes
//     that spawned none;
//   * a chain pass bounces the lanes' rays (any level >= 1) and refills the
//     lanes whose chain ended from the queue.
// A chain that ends unwinds its pixel's stack (sbase[sidx + level * sstride],
// innermost first, main.cpp:54) and stores the pixel.
// One pixel's 3 bytes at p (any alignment) written with dword atomics: its
// bytes of each covering dword cleared (AND), then set (OR); the other bytes,
// other pixels', are untouched whoever writes them meanwhile.
__device__ __forceinline__ void put_px(uint8_t *p, unsigned v) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  unsigned *d = reinterpret_cast<unsigned *>(a & ~(uintptr_t)3);
  const unsigned sh = (unsigned)(a & 3) * 8;
  const unsigned long long m = 0xFFFFFFull << sh, w = (unsigned long long)v << sh;
  atomicAnd(d, ~(unsigned)m);
  if ((unsigned)w) atomicOr(d, (unsigned)w);
  if (sh > 8) {
    atomicAnd(d + 1, ~(unsigned)(m >> 32));
    if ((unsigned)(w >> 32)) atomicOr(d + 1, (unsigned)(w >> 32));
  }
}

// The finished pixels of a merge_tiles group wait in LDS as RGB8 bytes laid
// out like the tiles' rows (tile slot t, row y, pixel x at t * 192 + y * 24 +
// x * 3) until every pixel of their tile is final, then go out as the tile's
// 24-byte rows, one dword per lane (flush_tile); a deferred pixel's bytes stay
// 0 for render_deferred's or_px.
typedef __attribute__((address_space(3))) unsigned char LdsU8;
typedef __attribute__((address_space(3))) unsigned LdsU32;
__device__ __forceinline__ void flush_tile(const RenderArgs &a, int tile, int frame, const LdsU8 *pb) {
  const int lane = (int)(threadIdx.x & 63);
  const OutDesc &od = kernarg_late<true, offsetof(RenderArgs, od)>(a.od);
  const Rows &rows = kernarg_late<true, offsetof(RenderArgs, rows)>(a.rows);
  const int W = kernarg_late<true, offsetof(RenderArgs, W)>(a.W);
  const int ntx = kernarg_late<true, offsetof(RenderArgs, ntx)>(a.ntx);
  const int rows_dword = kernarg_late<true, offsetof(RenderArgs, rows_dword)>(a.rows_dword);
  uint8_t *out = static_cast<uint8_t *>(od.ptr) + (size_t)frame * (size_t)od.fstride;
  const int x0 = (tile % ntx) * 8, ty = tile / ntx;
  // a row of 8 pixels is 24 bytes = 6 dwords when it is whole and dword aligned
  auto row_at = [&](int r) { return out + ((size_t)(ty * 8 + r) * W + x0) * 3; };
  if (rows_dword && x0 + 8 <= W && ty * 8 + 8 <= rows.count) {  // wave-uniform: the usual case
    if (lane < 48) {  // lane: row lane / 6, dword lane % 6 = LDS dword lane
      const unsigned v = reinterpret_cast<const LdsU32 *>(pb)[lane];
      *reinterpret_cast<unsigned *>(row_at(0) + (unsigned)(lane / 6) * (unsigned)W * 3u +
                                    4u * (unsigned)(lane - 6 * (lane / 6))) = v;
    }
    return;
  }
  auto whole = [&](int r) {
    return ty * 8 + r < rows.count && x0 + 8 <= W && (reinterpret_cast<uintptr_t>(row_at(r)) & 3) == 0;
  };
  {
    const int r = lane / 6, c = lane - 6 * (lane / 6);  // lanes 0..47: row r, dword c = LDS dword lane
    if (lane < 48 && whole(r)) reinterpret_cast<unsigned *>(row_at(r))[c] = reinterpret_cast<const LdsU32 *>(pb)[lane];
  }
  {
    // rows that are not whole (the image's right edge, odd widths): the
    // lane's own pixel into the dwords it shares with its neighbours (which
    // other waves may be writing): its bytes cleared and set by dword atomics
    const int r = lane >> 3, x = x0 + (lane & 7);
    if (!whole(r) && ty * 8 + r < rows.count && x < W) {
      const LdsU8 *p = pb + lane * 3;
      put_px(row_at(r) + (lane & 7) * 3, (unsigned)p[0] | (unsigned)p[1] << 8 | (unsigned)p[2] << 16);
    }
  }
}

// A merged wave's reflection stack lives in a "home": [depth-1][kMergeTiles *
// 64] entries, one per pixel of its group (lidx) and level, taken from the
// context's pool when the wave's first reflection ray spawns and returned
// when the wave ends.  The pool has twice as many homes as waves can be
// resident on the device (the host sizes it by the occupancy API), so a free
// one exists whenever a wave asks; the bitmap is searched from a word picked
// by the workgroup id, one atomic OR per try.  The stack memory of a launch
// is bounded by the pool, not by its pixels (kStackGlobal keeps the
// per-pixel stack).
constexpr int kHomePx = kMergeTiles * 64;
__device__ __forceinline__ int home_acquire(unsigned long long *bits, int nwords) {
  int h = -1;
  if ((threadIdx.x & 63) == 0) {
    int w = (int)(blockIdx.x % (unsigned)nwords);
    // the first try: a bit picked by the workgroup id as well (a half-full word
    // then takes one atomic, not two); it learns the word.  (Lowest-free-bit
    // first, to keep the homes in use few and L2-resident, measured the same
    // HBM writes and frame time: profiles/r7f/.)
    unsigned long long cur = ~(1ull << ((blockIdx.x / (unsigned)nwords) & 63u));
#ifdef RT_CHECK
    long long spins = 0;
#endif
    while (h < 0) {
      while (~cur) {
        const int bit = __builtin_ctzll(~cur);
        const unsigned long long old = atomicOr(bits + w, 1ull << bit);
        if (!((old >> bit) & 1ull)) {
          h = w * 64 + bit;
          break;
        }
        cur = old | (1ull << bit);
      }
      if (h < 0) {
        w = w + 1 == nwords ? 0 : w + 1;
        cur = 0ull;
#ifdef RT_CHECK
        // the pool holds twice the resident waves, so a wave finds a home
        // within a sweep or two; a wave still spinning after kHomeSweeps full
        // sweeps means a leaked home or an under-sized pool: record it and
        // share home 0 (wrong pixels, RT_ERR_CHECK) so the launch drains
        // instead of hanging
        constexpr long long kHomeSweeps = 4096;
        if (++spins >= kHomeSweeps * nwords) {
          ck_fail(kCkHome, spins, kHomeSweeps * nwords);
          h = 0;
        }
#endif
      }
    }
  }
  return __shfl(h, 0, 64);
}
__device__ __forceinline__ void home_release(unsigned long long *bits, int h) {
  if ((threadIdx.x & 63) == 0) atomicAnd(bits + (h >> 6), ~(1ull << (h & 63)));
}

template <bool kCull, bool kFast, bool kWide = false>
__device__ __forceinline__ void merge_tiles(const SphGeo *__restrict__ g, const double *__restrict__ rad,
                                            const SphMat *__restrict__ mat, const LightD *__restrict__ slight,
                                            const RenderArgs &a, int group, int frame, const CompactArgs &ca,
                                            QRay *q, Work &work, unsigned long long (&sums)[4]) {
  const int lane = (int)(threadIdx.x & 63);
  const unsigned long long lt = (1ull << lane) - 1ull;
  unsigned c_prim = 0, c_shadow = 0, c_reflect = 0, c_neg = 0;
  // the finished pixels (flush_tile), at an LDS offset the host placed after the walk stacks
  auto pixbuf = [&]() { return (LdsU8 *)rt_dyn_lds + kernarg_late<true, offsetof(RenderArgs, pix_off)>(a.pix_off); };
#pragma unroll
  for (int i = 0; i < (int)((kPixbufIds + 255) / 256); ++i)  // padding, depth 0 and deferred pixels: 0
    if ((size_t)(i * 256 + lane * 4) < kPixbufIds) reinterpret_cast<LdsU32 *>(pixbuf())[i * 64 + lane] = 0u;
  const int depth = a.depth;
  int qn = 0;        // queued rays q[0 .. qn), wave-uniform, < Q between passes
  const int Q = kernarg_late<true, offsetof(RenderArgs, merge_q)>(a.merge_q);
  int next = 0;      // next tile of the group
  bool act = false;  // this lane holds a ray
  D3 o = mk(0.0, 0.0, 0.0), d = o;
  int key = -1, dleft = 0, lev = 0;
  unsigned pix = 0;
  int lidx = 0;  // the pixel's place in the group: tile slot * 64 + y * 8 + x (pixbuf byte 3 * lidx)
  int home = -1;  // the group's stack home (home_acquire), once a reflection ray spawned
  auto hs = [&]() {
    return kernarg_late<true, offsetof(RenderArgs, homes)>(a.homes) + (size_t)home * (size_t)(depth - 1) * kHomePx;
  };
  auto hslot = [&](int l) {
    return RT_CK(kCkStack, (size_t)l * kHomePx + (size_t)lidx, (long long)(depth - 1) * kHomePx);
  };
  // pops queued rays into the lanes without one (lanes ranked by lane id)
  auto refill = [&](unsigned long long busy) {
    const int take = (64 - __popcll(busy)) < qn ? (64 - __popcll(busy)) : qn;
    const int r = (int)__popcll(~busy & lt);
    if (!act && r < take) {
      const QRay &e = q[RT_CK(kCkLdsQueue, qn - 1 - r, Q)];
      o = mk(e.ox, e.oy, e.oz);
      d = mk(e.dx, e.dy, e.dz);
      key = e.key;
      dleft = e.dleft;
      pix = (unsigned)e.pix;
      lidx = e.orig;
      lev = 1;
      act = true;
    }
    qn -= take;
  };
  while (true) {
    // the group's tile slots: [base, base + nt) -- one slot for the first nsingle
    // groups (the heaviest tiles: their own reflection rays fill the wave, and
    // a frame's critical path is its slowest wave), kMergeTiles up to
    // merge_end, then one slot per group again (the launch's last, lightest
    // tiles: the waves that end a launch are short, so fewer slots idle while
    // the last ones finish)
    const int ns = kernarg_late<true, offsetof(RenderArgs, nsingle)>(a.nsingle);
    const int me = kernarg_late<true, offsetof(RenderArgs, merge_end)>(a.merge_end);
    const int nm = (me - ns + kMergeTiles - 1) / kMergeTiles;
    int base, nt;
    if (group < ns) {
      base = group, nt = 1;
    } else if (group < ns + nm) {
      base = ns + (group - ns) * kMergeTiles, nt = me - base < kMergeTiles ? me - base : kMergeTiles;
    } else {
      base = me + (group - ns - nm), nt = 1;
    }
    bool tile_pass = false;
    if (__ballot(act) == 0) {
      if (next < nt) {  // camera rays of the next tile: camera.h:17-25, main.cpp:151-154 (as trace_tile)
        const int *perm = kernarg_late<true, offsetof(RenderArgs, perm)>(a.perm);
        const int slot = base + next;
        const int tile = RT_CK(kCkTile, perm ? perm[RT_CK(kCkTile, slot, a.ntiles)] : slot, a.ntiles);
        const int ntx = kernarg_late<true, offsetof(RenderArgs, ntx)>(a.ntx);
        const int tx = tile % ntx, ty = tile / ntx;
        const OutDesc &od = kernarg_late<true, offsetof(RenderArgs, od)>(a.od);
        const Rows &rows = kernarg_late<true, offsetof(RenderArgs, rows)>(a.rows);
        const int W = kernarg_late<true, offsetof(RenderArgs, W)>(a.W);
        const int H = kernarg_late<true, offsetof(RenderArgs, H)>(a.H);
        const int x = tx * 8 + (lane & 7);
        const int k = ty * 8 + (lane >> 3);
        const bool in_tile = x < W && k < rows.count;
        const long long y = (long long)(k / rows.band) * rows.band * rows.stride +
                            (long long)rows.first * rows.band + (k % rows.band);
        const bool in_img = in_tile && y < H;
        const int j = H - 1 - (int)(in_img ? y : 0);  // reference row (main.cpp:74)
        const Cam &cam = kernarg_cam(frame);
        const double u = (double)x / (W - 1), v = (double)j / (H - 1);
        const double su = ((u - 0.5) * cam.scale) * 1.0, sv = (v - 0.5) * cam.scale;
        const D3 dir = add(add(mk(cam.fx, cam.fy, cam.fz), scale(mk(cam.rx, cam.ry, cam.rz), su)),
                           scale(mk(cam.ux, cam.uy, cam.uz), sv));
        d = renormalized(normalized(dir));
        o = mk(cam.px, cam.py, cam.pz);
        pix = (unsigned)(k * W + x);
        lidx = next * 64 + lane;
        key = -1;
        dleft = depth;
        lev = 0;
        act = in_img && depth >= 1;
        c_prim += act ? 1u : 0u;
        // depth <= 0 -> black (main.cpp:17-18), padding rows -> zeros: pixbuf's 0
        (void)od;
        // for the flush at the group's end: the tile id and, when the tile is
        // whole and its rows dword aligned, the byte offset of its first row in
        // the frame (else ~0: flush_tile's general path)
        if (lane == 0) {
          const size_t off = ((size_t)ty * 8 * W + (size_t)tx * 8) * 3;
          const bool whole = kernarg_late<true, offsetof(RenderArgs, rows_dword)>(a.rows_dword) && tx * 8 + 8 <= W &&
                             ty * 8 + 8 <= rows.count && off < 0xFFFFFFFFull;
          LdsU32 *ids = reinterpret_cast<LdsU32 *>(pixbuf() + kPixbufIds);
          ids[2 * next] = (unsigned)tile;
          ids[2 * next + 1] = whole ? (unsigned)off : 0xFFFFFFFFu;
        }
        ++next;
        tile_pass = true;
        if (__ballot(act) == 0) continue;
      } else if (qn > 0) {
        refill(0ull);
      } else {
        break;
      }
    }
    int outcome = 0, nkey = 0;
    D3 color = mk(0.0, 0.0, 0.0), no = o, nd = d;
    double refl = 0.0;
    double bt;
    const int bi = closest_hit<kCull, true, kFast>(g, rad, a.n, a.bv, act, o, d, key, work, bt,
                                             kFast && tile_pass && kernarg_late<true, offsetof(RenderArgs, cg)>(a.cg).on,
                                             frame);
    shade_hit<kCull, true, kFast, kWide>(g, rad, mat, slight, a.n, a.nl, a.amb, a.bv, a.lg, act, o, d, key, dleft, bi, bt,
                                  work, c_shadow, outcome, color, refl, no, nd, nkey);
    const unsigned sidx = pix + ca.fpx;
    bool defer = false;
    if (home < 0 && __ballot(act && outcome == kSpawned))
      home = home_acquire(kernarg_late<true, offsetof(RenderArgs, home_bits)>(a.home_bits),
                          kernarg_late<true, offsetof(RenderArgs, home_words)>(a.home_words));
    if (act) {
      if (outcome == kSpawned) {
        hs()[hslot(lev)] = StackEnt{color.x, color.y, color.z, refl};
        ++lev;
        o = no;
        d = nd;
        key = nkey;
        --dleft;
        ++c_reflect;
        defer = lev >= kernarg_late<true, offsetof(RenderArgs, defer_level)>(a.defer_level);
      } else {  // the chain ends: unwind its pixel's stack and store it
        D3 res = color;
        while (lev > 0) {
          --lev;
          const StackEnt e = hs()[hslot(lev)];
          res = mk(e.ax + res.x * e.refl, e.ay + res.y * e.refl, e.az + res.z * e.refl);
        }
        {
          const unsigned v = pack_px(res, c_neg);
          LdsU8 *p = pixbuf() + 3 * RT_CK(kCkPixbuf, lidx, kMergeTiles * 64);
          p[0] = (unsigned char)v;
          p[1] = (unsigned char)(v >> 8);
          p[2] = (unsigned char)(v >> 16);
        }
        act = false;
      }
    }
    // rays of level >= kDeferLevel go to the launch's deferred queue (render_deferred),
    // as far as its shard segment has room; the others continue here
    const unsigned long long dm = __ballot(defer);
    if (dm) {
      const int cap = kernarg_late<true, offsetof(RenderArgs, dq_cap)>(a.dq_cap);
      if (cap > 0) {
        unsigned long long base = 0;
        const int first = __builtin_ctzll(dm);
        if (lane == first) base = atomicAdd(&counter_shard(kernarg_late<true, offsetof(RenderArgs, counters)>(a.counters))[kDeferSlot],
                                            (unsigned long long)__popcll(dm));
        base = __shfl(base, first, 64);
        const unsigned long long slot = base + (unsigned long long)__popcll(dm & lt);
        if (defer && slot < (unsigned long long)cap) {
          QRay *dq = kernarg_late<true, offsetof(RenderArgs, dq)>(a.dq);
          const unsigned wg = blockIdx.x;
          const size_t gslot = RT_CK(kCkDeferQ, (size_t)(wg % kShards) * (size_t)cap + slot, (long long)kShards * cap);
          dq[gslot] = QRay{o.x, o.y, o.z, d.x, d.y, d.z, lev, dleft, key, (int)sidx};
          // its stack entries so far go with it: render_deferred continues the chain at its queue slot
          StackEnt *ds = kernarg_late<true, offsetof(RenderArgs, dstack)>(a.dstack);
          const size_t dtot = (size_t)kShards * (size_t)cap;
          for (int l = 0; l < lev; ++l)
            ds[RT_CK(kCkStack, (size_t)l * dtot + gslot, (long long)(depth - 1) * (long long)dtot)] = hs()[hslot(l)];
          act = false;
        }
      }
    }
    const unsigned long long busy = __ballot(act);
    if (tile_pass && next < nt && __popcll(busy) + qn < Q) {
      // this tile's reflection rays wait for the next tiles' (queue < Q entries)
      if (act)
        q[RT_CK(kCkLdsQueue, qn + (int)__popcll(busy & lt), Q)] =
            QRay{o.x, o.y, o.z, d.x, d.y, d.z, lidx, dleft, key, (int)pix};
      qn += __popcll(busy);
      act = false;
    } else if (qn > 0 && busy != ~0ull) {
      refill(busy);  // lanes without a ray take queued ones
    }
  }
  // every pixel of the group is final (or deferred, 0 bytes): its tiles go
  // out, a whole aligned tile as 48 dword stores at its recorded offset
  {
    const OutDesc &od = kernarg_late<true, offsetof(RenderArgs, od)>(a.od);
    const int W = kernarg_late<true, offsetof(RenderArgs, W)>(a.W);
    uint8_t *out = static_cast<uint8_t *>(od.ptr) + (size_t)frame * (size_t)od.fstride;
    const unsigned roff = (unsigned)(lane / 6) * (unsigned)W * 3u + 4u * (unsigned)(lane - 6 * (lane / 6));
    const LdsU32 *ids = reinterpret_cast<const LdsU32 *>(pixbuf() + kPixbufIds);
#pragma unroll
    for (int t = 0; t < kMergeTiles; ++t) {
      if (t >= next) break;
      const unsigned off = __builtin_amdgcn_readfirstlane(ids[2 * t + 1]);
      if (off != 0xFFFFFFFFu) {
        if (lane < 48) {
          const unsigned v = reinterpret_cast<const LdsU32 *>(pixbuf() + 192 * t)[lane];
          *reinterpret_cast<unsigned *>(
              out + RT_CK(kCkOut, (size_t)off + roff,
                          (long long)(kernarg_late<true, offsetof(RenderArgs, rows)>(a.rows).count) * W * 3 - 3)) = v;
        }
      } else {
        flush_tile(a, (int)__builtin_amdgcn_readfirstlane(ids[2 * t]), frame, pixbuf() + 192 * t);
      }
    }
  }
  if (home >= 0) home_release(kernarg_late<true, offsetof(RenderArgs, home_bits)>(a.home_bits), home);
  sums[0] += wave_sum(c_prim);
  sums[1] += wave_sum(c_shadow);
  sums[2] += wave_sum(c_reflect);
  sums[3] += wave_sum(c_neg);
}

// Flushes a wave's ray counts and work counters into its counter shard.
// Called with every lane of the wave active (the per-lane work counters are
// summed over the wave here).
__device__ __forceinline__ void flush_counts(unsigned long long *counters, const unsigned long long (&sums)[4],
                                             const Work &work) {
  const unsigned long long exact = wave_sum64(work.exact), cull = wave_sum64(work.cull);
  if ((threadIdx.x & 63) == 0) {
    unsigned long long *sc = counter_shard(counters);
#ifdef RT_STAMPS
    for (int q = 0; q < 6; q++) atomicAdd(&sc[8 + q], work.st[q]);
    atomicAdd(&sc[20], work.st[6]);
    atomicAdd(&sc[21], work.st[8]);  // closest hits
    atomicAdd(&sc[22], work.st[9]);  // shadow queries
    atomicAdd(&sc[14], 1ull);
    atomicAdd(&sc[15], work.iters);
    atomicAdd(&sc[16], work.sweeps);
    atomicAdd(&sc[17], work.it_closest);
    atomicAdd(&sc[18], work.sw_closest);
    atomicAdd(&sc[19], work.it_prim);
#endif
    for (int q = 0; q < 4; q++)
      if (sums[q]) atomicAdd(&sc[q], sums[q]);
    if (exact) atomicAdd(&sc[4], exact);
    if (cull) atomicAdd(&sc[5], cull);
  }
}

#ifdef RT_STAMPS
__device__ __forceinline__ void record_timeline(unsigned wave_id, unsigned long long t_real0, const Work &work) {
  const int lane = threadIdx.x & 63;
  const unsigned long long bvh_steps_max = (unsigned long long)wmax((double)work.st[7]);
  const unsigned long long wave_trips = wave_sum((unsigned)work.st[10]);
  if (lane == 0) {
    const unsigned wid = wave_id;
    if (wid < (unsigned)kTimelineWaves) {
      unsigned long long *tl = g_timeline + (size_t)kTl * wid;
      tl[0] = t_real0;
      tl[1] = __builtin_amdgcn_s_memrealtime();
      const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
      const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));
      tl[2] = ((unsigned long long)xcc << 32) | hw;
      tl[3] = work.st[0];  // bound cycles
      tl[4] = work.st[1];  // cull
      tl[5] = work.st[2];  // candidates
      tl[6] = work.st[4];  // shading
      tl[7] = work.st[5];  // total
      tl[8] = work.iters | (work.sweeps << 32);
      tl[10] = work.st[6];  // bvh walks
      tl[11] = work.st[3];  // per-light setup
      tl[12] = work.st[8];  // closest sweeps
      tl[13] = work.st[9];  // shadow sweeps
      tl[14] = wave_trips;  // bvh loop trips of the wave
      tl[9] = bvh_steps_max;  // most BVH node visits of one lane
    }
  }
}
#endif

#ifndef RT_MIN_WAVES_PER_EU
#define RT_MIN_WAVES_PER_EU 3  // caps VGPRs at 168: three waves per SIMD
#endif
// Waves per render_kernel workgroup: 4 (2x2 tiles of 8x8 pixels) when the
// workgroup shares a scene staged in LDS; 1 otherwise, so no wave's slot
// waits for its slowest neighbour.
template <bool kLdsGeo>
constexpr int wg_waves() {
  return kLdsGeo ? 4 : 1;
}

template <bool kLdsGeo, bool kCull, int kSamples, int kStack, bool kFast = false, bool kWide = false>
__global__ __launch_bounds__((64 * wg_waves<kLdsGeo>()), RT_MIN_WAVES_PER_EU) void render_kernel(
    const RenderArgs a) {
  // Workgroups are dealt to the 8 XCDs round robin (b % 8), so every image
  // region is spread over all XCDs.  perm: the host's launch order (rt_sched.h).
  const int b = blockIdx.x;
  if (b == 0 && a.zero_next)
    for (int i = (int)threadIdx.x; i < kShards * kShardStride; i += (int)blockDim.x) a.zero_next[i] = 0ull;
  // the frames of a multi-frame launch share the tile order, so every frame's
  // copy of a heavy tile starts early.  Workgroups are dealt to the 8 XCDs
  // round robin (b % 8); with xcd_frames the k-th workgroup of XCD x renders
  // frame k % F of tile group 8 (k / F) + x, so all F copies of a group run on
  // the XCD whose L2 holds that group's scene lists and nodes (the grid is
  // padded to a multiple of 8 groups; the padding exits); otherwise the F
  // copies of a group are adjacent (b / F, b % F) and spread over the XCDs
  const int nf = a.frames;
  int slot = b, frame = 0;
  if (nf > 1) {
    if (a.xcd_frames) {
      const int k = b >> 3;
      slot = (k / nf) * 8 + (b & 7);
      frame = k - (k / nf) * nf;
    } else {
      slot = b / nf;
      frame = b - slot * nf;
    }
  }
  int tile = slot;
  if constexpr (kStack == kStackMerge) {
    if (slot >= a.nslots) return;  // slot = this wave's group of tile slots (merge_tiles)
  } else {
    if (a.perm) {
      if (slot >= a.nslots) return;
      tile = a.perm[RT_CK(kCkTile, slot, a.nslots)];  // heaviest predicted tiles first, or a batch's listed blocks
    }
    if (tile >= a.ntiles) return;  // workgroup-uniform, before any barrier
  }
  const int tx = tile % a.ntx, ty = tile / a.ntx;
  extern __shared__ __attribute__((aligned(32))) unsigned char smem[];
  const SphGeo *g;
  const double *rad;
  const LightD *slight;
  const SphMat *sm;
  // With the scene staged in LDS the BVH arguments are a modified local copy;
  // otherwise the kernel argument itself is used (re-read from the kernarg
  // segment where needed: kernarg_late) and the ordered walk finds its LDS
  // stacks at bv.ostk_off (set by the host).
  BvhArgs bv_local = a.bv;
  stage_scene<kLdsGeo>(smem, a.geo, a.radius, a.mat, a.lights, a.n, a.nl, bv_local, g, rad, sm, slight);
  const size_t stack_off = (lds_layout(kLdsGeo, a.n, a.nl, a.bv.nnodes).end + 31) & ~(size_t)31;
  // the ordered BVH walk's per-lane stacks, [wave][entry][lane], after the scene
  if (kLdsGeo && bv_local.ordered)
    bv_local.ostk = reinterpret_cast<int2 *>(smem + stack_off) + (size_t)(threadIdx.x >> 6) * bv_local.odepth * 64;
  const BvhArgs &bv = kLdsGeo ? bv_local : a.bv;
  constexpr int kWg = wg_waves<kLdsGeo>();
  constexpr int kWx = kWg == 4 ? 2 : 1;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: keeps tile coordinates in SGPRs
  CompactArgs ca;
  ca.park = nullptr;
  if (!kLdsGeo)  // after the ordered walk's stacks (launch_tiles sizes both)
    ca.park = reinterpret_cast<D3 *>(smem + stack_off + (a.bv.ordered ? (size_t)kWg * a.bv.odepth * 64 * sizeof(int2) : 0)) +
              (size_t)wave * 64;
  ca.gstack = a.gstack;
  ca.npx = (size_t)a.rows.count * a.od.xw * nf;
  ca.fpx = (unsigned)((size_t)a.rows.count * a.od.xw * frame);
  Work work;
  unsigned long long sums[4] = {0, 0, 0, 0};
  RT_T0(t_wave);
#ifdef RT_STAMPS
  const unsigned long long t_real0 = __builtin_amdgcn_s_memrealtime();
#endif
  if constexpr (kStack == kStackMerge && !kLdsGeo && kSamples == 1) {
    // the wave's ray queue sits where trace_wave parks colours, after the
    // finished-pixel bytes (launch_tiles)
    QRay *q = reinterpret_cast<QRay *>(reinterpret_cast<unsigned char *>(ca.park) + kPixbufBytes);
    merge_tiles<kCull, kFast, kWide>(g, rad, sm, slight, a, slot, frame, ca, q, work, sums);
  } else {
    trace_tile<kCull, kSamples, kStack, !kLdsGeo>(g, rad, sm, slight, a.n, a.nl, a.amb, kernarg_cam(frame), a.W, a.H,
                                                  a.depth, a.rows, bv, a.lg, a.od,
                                                  a.od.x0 + tx * (8 * kWx) + (wave % kWx) * 8,
                                                  ty * (8 * (kWg / kWx)) + (wave / kWx) * 8, ca, work,
                                                  sums, frame);
  }
  RT_ACC(work, 5, t_wave);
#ifdef RT_STAMPS
  // merged kernels: one entry per workgroup of the launch (slot b = group b / F of frame b % F)
  record_timeline(kStack == kStackMerge ? (unsigned)blockIdx.x : (unsigned)(tile * kWg + wave), t_real0, work);
#endif
  flush_counts(kernarg_late<!kLdsGeo, offsetof(RenderArgs, counters)>(a.counters), sums, work);
}

// The deferred rays of a kStackMerge launch (level >= kDeferLevel, typically
// 2-3 % of its rays but the least coherent): one wave per workgroup,
// workgroup b serves shard segment b % kShards and takes its chunks of 64
// rays b / kShards, + gridDim / kShards, ...  Each lane runs its ray's chain
// to the end exactly as merge_tiles would have (bounce, stack entries at its
// queue slot's [level][slot] entries of dstack), unwinds the chain's whole
// stack -- the levels merge_tiles copied there at the deferral first -- and
// stores the pixel.
template <bool kCull, bool kFast = false, bool kWide = false>
__global__ __launch_bounds__(64, RT_MIN_WAVES_PER_EU) void render_deferred(const RenderArgs a) {
  const unsigned shard = blockIdx.x % kShards, first = blockIdx.x / kShards;
  const int cap = a.dq_cap;
  const unsigned long long cnt = a.counters[(size_t)shard * kShardStride + kDeferSlot];
  const unsigned n_dq = (unsigned)(cnt < (unsigned long long)cap ? cnt : (unsigned long long)cap);
  if (first * 64u >= n_dq) return;
  const int lane = (int)(threadIdx.x & 63);
  const unsigned npx_frame = (unsigned)((size_t)a.rows.count * a.od.xw);
  const unsigned sstride = (unsigned)kShards * (unsigned)cap;  // the chain's stack: dstack[level][queue slot]
  Work work;
  unsigned c_shadow = 0, c_reflect = 0, c_neg = 0;
  // Lanes without a ray take the shard segment's next entries (one
  // wave-aggregated atomic on its fetch slot), so the wave stays full until
  // the segment runs out and the workgroups of a segment finish together
  // instead of each finishing its own static stream's longest chains.
  const unsigned long long lt = (1ull << lane) - 1ull;
  bool act = false, more = true;
  D3 o = mk(0.0, 0.0, 0.0), d = o;
  int key = -1, dleft = 0, lev = 0;
  unsigned pixg = 0, qslot = 0;  // the ray's output pixel (launch index) and queue slot
  unsigned long long *fetch = kernarg_late<true, offsetof(RenderArgs, counters)>(a.counters) +
                              (size_t)shard * kShardStride + kFetchSlot;
  while (true) {
    const unsigned long long idle = ~__ballot(act);
    if (idle && more) {
      const int fi = __builtin_ctzll(idle);
      unsigned long long base = 0;
      if (lane == fi) base = atomicAdd(fetch, (unsigned long long)__popcll(idle));
      base = __shfl(base, fi, 64);
      const unsigned long long i = base + (unsigned long long)__popcll(idle & lt);
      more = base + (unsigned long long)__popcll(idle) < n_dq;
      if (!act && i < n_dq) {
        const QRay &e = kernarg_late<true, offsetof(RenderArgs, dq)>(a.dq)[RT_CK(kCkDeferQ, (size_t)shard * (size_t)cap + i, (long long)kShards * cap)];
        o = mk(e.ox, e.oy, e.oz);
        d = mk(e.dx, e.dy, e.dz);
        lev = e.orig;
        dleft = e.dleft;
        key = e.key;
        pixg = (unsigned)e.pix;
        qslot = shard * (unsigned)cap + (unsigned)i;
        act = true;
      }
    }
    if (__ballot(act) == 0) break;
    {
      int outcome = 0, nkey = 0;
      D3 color = mk(0.0, 0.0, 0.0), no = o, nd = d;
      double refl = 0.0;
      bounce<kCull, true, kFast, kWide>(a.geo, a.radius, a.mat, a.lights, a.n, a.nl, a.amb, a.bv, a.lg, act, o, d, key,
                                        dleft, work, c_shadow, outcome, color, refl, no, nd, nkey);
      if (act) {
        StackEnt *gs = kernarg_late<true, offsetof(RenderArgs, dstack)>(a.dstack);
        if (outcome == kSpawned) {
          gs[RT_CK(kCkStack, qslot + (unsigned)lev * sstride, (long long)(a.depth - 1) * sstride)] =
              StackEnt{color.x, color.y, color.z, refl};
          ++lev;
          o = no;
          d = nd;
          key = nkey;
          --dleft;
          ++c_reflect;
        } else {
          D3 res = color;
          while (lev > 0) {  // main.cpp:54, innermost first
            --lev;
            const StackEnt e = gs[RT_CK(kCkStack, qslot + (unsigned)lev * sstride, (long long)(a.depth - 1) * sstride)];
            res = mk(e.ax + res.x * e.refl, e.ay + res.y * e.refl, e.az + res.z * e.refl);
          }
          const OutDesc &od = kernarg_late<true, offsetof(RenderArgs, od)>(a.od);
          const unsigned f = pixg / npx_frame;
          or_px(static_cast<uint8_t *>(od.ptr) + (size_t)RT_CK(kCkOut, f, a.frames) * (size_t)od.fstride, pixg - f * npx_frame,
                pack_px(res, c_neg));
          act = false;
        }
      }
    }
  }
  unsigned long long sums[4] = {0ull, wave_sum(c_shadow), wave_sum(c_reflect), wave_sum(c_neg)};
  flush_counts(kernarg_late<true, offsetof(RenderArgs, counters)>(a.counters), sums, work);
}

// render_deferred for scenes with a BVH, with the walks decoupled from the
// shading (kFast configuration).  A lane's closest-hit walk advances one node
// or leaf per step (walk4_step); a lane whose walk ended waits, and the wave
// shades once kShadeAt lanes are ready (or no lane is walking): shade_hit for
// the ready lanes only, after which a spawned reflection ray starts its walk
// and an ended chain stores its pixel and takes the next queued ray.  In
// render_deferred a wave's walk lasts as long as its longest one (the
// level >= 2 rays' walks are long-tailed: scripts/bvh_sim.cpp models 0.36 of
// the lanes busy); here the lanes whose walks end early start the next ray's.
// Same tests, same per-ray results: the closest hit of each ray is its
// lexicographic (t, index) minimum (walk4_step, closest_test), shading and
// the stack unwinding are render_deferred's.
#ifndef RT_SHADE_AT
#define RT_SHADE_AT 40
#endif
constexpr int kShadeAt = RT_SHADE_AT;
__global__ __launch_bounds__(64, RT_MIN_WAVES_PER_EU) void render_deferred_walk(const RenderArgs a) {
  const unsigned shard = blockIdx.x % kShards, first = blockIdx.x / kShards;
  const int cap = a.dq_cap;
  const unsigned long long cnt = a.counters[(size_t)shard * kShardStride + kDeferSlot];
  const unsigned n_dq = (unsigned)(cnt < (unsigned long long)cap ? cnt : (unsigned long long)cap);
  if (first * 64u >= n_dq) return;
  const int lane = (int)(threadIdx.x & 63);
  const unsigned npx_frame = (unsigned)((size_t)a.rows.count * a.od.xw);
  const unsigned sstride = (unsigned)kShards * (unsigned)cap;  // the chain's stack: dstack[level][queue slot]
  Work work;
  unsigned c_shadow = 0, c_reflect = 0, c_neg = 0;
  const unsigned long long lt = (1ull << lane) - 1ull;
  bool act = false, walking = false, more = true;
  unsigned long long *fetch = kernarg_late<true, offsetof(RenderArgs, counters)>(a.counters) +
                              (size_t)shard * kShardStride + kFetchSlot;  // as render_deferred
  D3 o = mk(0.0, 0.0, 0.0), d = o;
  int key = -1, dleft = 0, lev = 0;
  unsigned pixg = 0, qslot = 0;  // the ray's output pixel (launch index) and queue slot
  // the walk of this lane's ray: pending reference and stack depth, the best
  // hit so far (t, numerator, sphere) and the fp32 prune bound
  int ref = 0, sp = 0, bi = -1;
  double bt = kInf, bn = __builtin_inf();
  float tmf = 0.0f;
  auto prune = [&](const BvhArgs &bv) { return float_up(bt + 2e-6 * (bv.diam + __builtin_fabs(bt))); };
  auto begin = [&](const BvhArgs &bv) {  // a new ray: an empty best, the root box
    bt = kInf;
    bn = __builtin_inf();
    bi = -1;
    tmf = prune(bv);
    walking = walk4_begin(bv, walk4_ray(bv, o, d), tmf, ref, sp);
  };
  while (true) {
    {
      const unsigned long long idle = ~__ballot(act);
      if (idle && more) {
        const int fi = __builtin_ctzll(idle);
        unsigned long long base = 0;
        if (lane == fi) base = atomicAdd(fetch, (unsigned long long)__popcll(idle));
        base = __shfl(base, fi, 64);
        const unsigned long long i = base + (unsigned long long)__popcll(idle & lt);
        more = base + (unsigned long long)__popcll(idle) < n_dq;
        if (!act && i < n_dq) {
          const QRay &e = kernarg_late<true, offsetof(RenderArgs, dq)>(a.dq)[RT_CK(kCkDeferQ, (size_t)shard * (size_t)cap + i, (long long)kShards * cap)];
          o = mk(e.ox, e.oy, e.oz);
          d = mk(e.dx, e.dy, e.dz);
          lev = e.orig;
          dleft = e.dleft;
          key = e.key;
          pixg = (unsigned)e.pix;
          qslot = shard * (unsigned)cap + (unsigned)i;
          act = true;
          begin(kernarg_late<true, offsetof(RenderArgs, bv)>(a.bv));
        }
      }
    }
    if (__ballot(act) == 0) break;
    // walk until enough lanes are ready to shade (or no lane walks)
    if (__ballot(walking)) {
      const BvhArgs &bv = kernarg_late<true, offsetof(RenderArgs, bv)>(a.bv);
      const Walk4Ray r = walk4_ray(bv, o, d);
      const double a4 = 4.0 * dot(d, d), a2 = 0.5 * a4;
      const bool fast = a2_ok(a2);
      const SphGeo *__restrict__ g = a.geo;
      while (true) {
        const unsigned long long wm = __ballot(walking);
        if (wm == 0 || __popcll(__ballot(act) & ~wm) >= kShadeAt) break;
        if (walking) {
          auto leaf = [&](int i) {
            work.exact += 1;
            closest_test(g[RT_CK(kCkSphere, i, a.n)], i, o, d, a4, a2, fast, bt, bn, bi);
          };
          walking = walk4_step(bv, r, [&] { return prune(bv); }, work, leaf, ref, sp, tmf);
        }
      }
    }
    const bool ready = act && !walking;
    if (__ballot(ready)) {
      {
        // the line's part behind its origin (the walk skipped boxes wholly behind it)
        const BvhArgs &bv = kernarg_late<true, offsetof(RenderArgs, bv)>(a.bv);
        if (bv.ug.on && ready) {
          const double a4 = 4.0 * dot(d, d), a2 = 0.5 * a4;
          const bool fast = a2_ok(a2);
          const SphGeo *__restrict__ g = a.geo;
          behind_cells(bv, o, d, work, [&](int i) { closest_test(g[RT_CK(kCkSphere, i, a.n)], i, o, d, a4, a2, fast, bt, bn, bi); });
        }
      }
      int outcome = 0, nkey = 0;
      D3 color = mk(0.0, 0.0, 0.0), no = o, nd = d;
      double refl = 0.0;
      shade_hit<true, true, true>(a.geo, a.radius, a.mat, a.lights, a.n, a.nl, a.amb, a.bv, a.lg, ready, o, d, key,
                                   dleft, bi, bt, work, c_shadow, outcome, color, refl, no, nd, nkey);
      bool spawned = false;
      if (ready) {
        StackEnt *gs = kernarg_late<true, offsetof(RenderArgs, dstack)>(a.dstack);
        if (outcome == kSpawned) {
          gs[RT_CK(kCkStack, qslot + (unsigned)lev * sstride, (long long)(a.depth - 1) * sstride)] =
              StackEnt{color.x, color.y, color.z, refl};
          ++lev;
          o = no;
          d = nd;
          key = nkey;
          --dleft;
          ++c_reflect;
          spawned = true;
        } else {
          D3 res = color;
          while (lev > 0) {  // main.cpp:54, innermost first
            --lev;
            const StackEnt e = gs[RT_CK(kCkStack, qslot + (unsigned)lev * sstride, (long long)(a.depth - 1) * sstride)];
            res = mk(e.ax + res.x * e.refl, e.ay + res.y * e.refl, e.az + res.z * e.refl);
          }
          const OutDesc &od = kernarg_late<true, offsetof(RenderArgs, od)>(a.od);
          const unsigned f = pixg / npx_frame;
          or_px(static_cast<uint8_t *>(od.ptr) + (size_t)RT_CK(kCkOut, f, a.frames) * (size_t)od.fstride, pixg - f * npx_frame,
                pack_px(res, c_neg));
          act = false;
        }
      }
      if (spawned) begin(kernarg_late<true, offsetof(RenderArgs, bv)>(a.bv));
    }
  }
  unsigned long long sums[4] = {0ull, wave_sum(c_shadow), wave_sum(c_reflect), wave_sum(c_neg)};
  flush_counts(kernarg_late<true, offsetof(RenderArgs, counters)>(a.counters), sums, work);
}

// Reassemble rank-major shards into PPM row order (one workgroup per row).
__global__ __launch_bounds__(kBlock) void unpermute_kernel(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                           int W, int H, int band, int G, int R) {
  const int y = blockIdx.x;
  if (y >= H) return;
  const int b = y / band;
  const int r = b % G;
  const int k = (b / G) * band + (y % band);
  const uint8_t *s = src + ((size_t)r * R + k) * (size_t)W * 3;
  uint8_t *d = dst + (size_t)y * W * 3;
  const int nb = W * 3;
  // 16-byte (else 4-byte) vector copies when both rows allow it (1080p: a row
  // is 360 x 16 B), bytes otherwise; the condition is uniform per row
  if (((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d) | (uintptr_t)nb) & 15) == 0) {
    const uint4 *s4 = reinterpret_cast<const uint4 *>(s);
    uint4 *d4 = reinterpret_cast<uint4 *>(d);
    for (int i = threadIdx.x; i < nb / 16; i += kBlock) d4[i] = s4[i];
  } else if (((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d) | (uintptr_t)nb) & 3) == 0) {
    const unsigned *s1 = reinterpret_cast<const unsigned *>(s);
    unsigned *d1 = reinterpret_cast<unsigned *>(d);
    for (int i = threadIdx.x; i < nb / 4; i += kBlock) d1[i] = s1[i];
  } else {
    for (int i = threadIdx.x; i < nb; i += kBlock) d[i] = s[i];
  }
}

// ---------------------------------------------------------------------------
// The camera grid, built on the device for each camera position of a launch:
// build_point_grid (rt_lightgrid.cpp) on the GPU.  Every sphere's two disks
// seen from the grid's point P -- along +u with tlo = (D - R)(1 - 1e-9), along
// -u (the negative tangent root, sphere.h:43-47) with -(D + R)(1 + 1e-9), R
// the light grids' grown radius, each disk's angular radius asin(R / D) +
// kLgSlack -- are listed in every cell they meet, by the host builder's patch
// hierarchy and tests (faces, blocks of 8 x 8 tiles, tiles of 8 x 8 cells -- a
// tile well inside a disk takes all its cells untested -- cells against the
// per-(i, j) table), the same patches and margins; a sphere that contains (or
// nearly contains) P, or has non-finite data, is one disk of every direction
// with tlo = -inf (on every list).  A cell keeps K entries; one that
// overflows is marked by its count, and its rays sweep.  Passes:
// cg_disk_kernel (a wave per grid and sphere: the disks and the (disk, block)
// pairs they meet), cg_bin_kernel (a wave per quarter pair: tiles, cells,
// slots), cg_sort_kernel (a thread per cell: (tlo, index) order).
struct CgBuild {
  const SphGeo *geo;
  const double *rad;
  const CubePatch *faces, *blocks, *tiles;
  const double *cell_cbsb;
  int32_t *count;
  int2 *ent;            // [grid][cell][K] the lists (count: their lengths)
  CgDisk *disks;        // [grid][sphere][side]
  int2 *pairs;          // [grid][maxp] (disk, block) pairs whose block the disk meets
  unsigned *npairs;     // [grid * kCgCntStride] their counts (a 256-byte line per grid's counter)
  int n, N, NT, NB, K, ngrid, maxp;
  double px[RT_MAX_FRAMES], py[RT_MAX_FRAMES], pz[RT_MAX_FRAMES], diam[RT_MAX_FRAMES];
};
static_assert(sizeof(CgBuild) <= 4096, "CgBuild exceeds the kernel-argument segment");

constexpr int kCgCntStride = 64;
// Pass 1, a wave per (grid, sphere): its two disks (one for a global sphere), and
// every (disk, block) pair whose face and block patches the disk meets (a
// lane per block, one atomic on the grid's pair count per wave and side).
__global__ __launch_bounds__(256) void cg_disk_kernel(const CgBuild a) {
  const int t = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6), lane = (int)(threadIdx.x & 63);
  if (t >= a.n * a.ngrid) return;
  const int grid = t / a.n, s = t - grid * a.n;
  const SphGeo sp = a.geo[s];
  const CgView v = cg_view(sp.cx, sp.cy, sp.cz, a.rad[s], a.px[grid], a.py[grid], a.pz[grid], a.diam[grid]);
  const int nb = 6 * a.NB * a.NB;
  for (int side = 0; side < (v.global ? 1 : 2); ++side) {
    const CgDisk k = cg_side(v, side, s);
    const int di = 2 * t + side;
    if (lane == 0) a.disks[RT_CK(kCkCgBuild, di, 2LL * a.n * a.ngrid)] = k;
    for (int b0 = 0; b0 < nb; b0 += 64) {
      const int b = b0 + lane;
      const bool m = b < nb && cg_block(k, a.faces, a.blocks, a.NB, b);
      const unsigned long long bm = __ballot(m);
      if (!bm) continue;
      unsigned q0 = 0;
      if (lane == 0) q0 = atomicAdd(&a.npairs[grid * kCgCntStride], (unsigned)__builtin_popcountll(bm));
      q0 = (unsigned)__builtin_amdgcn_readfirstlane((int)q0);
      // a grid whose pairs exceed maxp keeps the first maxp; cg_sort_kernel
      // then marks all its cells overflowed (its rays sweep)
      const unsigned qi = q0 + (unsigned)__builtin_popcountll(bm & ((1ull << lane) - 1));
      if (m && qi < (unsigned)a.maxp) a.pairs[RT_CK(kCkCgBuild, (size_t)grid * a.maxp + qi, (long long)a.ngrid * a.maxp)] =
          make_int2(di, b);
    }
  }
}

// Pass 2, a wave per quarter of a (disk, block) pair (a fixed grid of waves
// walks the grids' pair lists): the block's 64 tiles (a tile well inside the
// disk takes all its cells untested), then the cells of each tile of the
// quarter it meets; each listed cell takes a slot (count) and, below K, the
// entry (sphere, tlo).
__global__ __launch_bounds__(64) void cg_bin_kernel(const CgBuild a) {
  const int lane = (int)(threadIdx.x & 63);
  const long long cells = 6LL * a.N * a.N;
  // work items per grid (4 per stored pair; the host keeps 4 ngrid maxp < 2^32), then their prefix
  unsigned incl = lane < a.ngrid ? 4u * min(a.npairs[lane * kCgCntStride], (unsigned)a.maxp) : 0u;
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned v = __shfl_up(incl, off, 64);
    if (lane >= off) incl += v;
  }
  const unsigned total = __shfl(incl, 63, 64);
  for (unsigned v = blockIdx.x; v < total; v += gridDim.x) {
    const int grid = __builtin_popcountll(__ballot(incl <= v));
    const unsigned item = v - (grid ? __shfl(incl, grid - 1, 64) : 0u);
    const int2 pr = a.pairs[RT_CK(kCkCgBuild, (size_t)grid * a.maxp + (item >> 2), (long long)a.ngrid * a.maxp)];
    const CgDisk k = a.disks[RT_CK(kCkCgBuild, pr.x, 2LL * a.n * a.ngrid)];
    const bool wide = cg_wide(k);
    const int bb = pr.y;
    const int f = bb / (a.NB * a.NB), bj = (bb / a.NB) % a.NB, bi = bb % a.NB;
    bool tm, inside;
    cg_tile(k, a.tiles, a.NT, f, bi, bj, lane, tm, inside);
    unsigned long long tmask = __ballot(tm) & (0xffffull << (16 * (item & 3)));
    const unsigned long long imask = __ballot(inside);
    while (tmask) {  // up to 4 tiles a round: their cells' slot atomics in flight together
      int gcs[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        gcs[u] = -1;
        if (!tmask) continue;
        const int tl = __builtin_ctzll(tmask);
        tmask &= tmask - 1;
        gcs[u] = cg_cell(k, wide, a.cell_cbsb, a.N, f, bi, bj, tl, lane, (imask >> tl) & 1ull);
      }
      int slots[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        slots[u] = gcs[u] >= 0 ? atomicAdd(&a.count[RT_CK(kCkCgBuild, (long long)grid * cells + gcs[u], a.ngrid * cells)], 1)
                               : a.K;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (slots[u] < a.K)
          a.ent[RT_CK(kCkCgBuild, ((long long)grid * cells + gcs[u]) * a.K + slots[u], a.ngrid * cells * a.K)] =
              make_int2(k.s, __float_as_int(k.tlo));
    }
  }
}

// Pass 3, a thread per cell: its list sorted by (tlo, index) in place (lists
// are short: insertion sort; an overflowed cell's rays sweep, its list unread).
__global__ __launch_bounds__(256) void cg_sort_kernel(const CgBuild a) {
  const long long cells = 6LL * a.N * a.N;
  const long long gc = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gc >= cells * a.ngrid) return;
  if (a.npairs[(gc / cells) * kCgCntStride] > (unsigned)a.maxp) {  // pass 1 dropped pairs: the grid is incomplete
    a.count[gc] = a.K + 1;                                           // every cell overflowed, its rays sweep
    return;
  }
  const int cnt = a.count[gc];
  if (cnt > a.K) return;
  int2 *e = a.ent + gc * a.K;
  for (int k = 1; k < cnt; ++k) {
    const int2 x = e[k];
    const float tx = __int_as_float(x.y);
    int m = k - 1;
    while (m >= 0 && (__int_as_float(e[m].y) > tx || (__int_as_float(e[m].y) == tx && e[m].x > x.x))) {
      e[m + 1] = e[m];
      --m;
    }
    e[m + 1] = x;
  }
}

// ---------------------------------------------------------------------------
// Point grids built on the device at upload: the sphere grids
// (build_sphere_grids, rt_lightgrid.cpp) -- one cube-map grid per reflective
// sphere s, seen from the ball B(C_s, rho_s) that holds the origins of the
// reflection rays leaving s (main.cpp:46), both disks of every sphere, the
// spheres within reach of the ball (global) on every list, entries (sphere,
// tlo) ascending by (tlo, index) -- and the light grids (build_light_grid)
// -- one grid per light, seen from the light (rho = 0), the disk ahead only,
// global spheres on a separate list (the grid's slot `cells`), ids
// ascending.  The camera grid's per-lane disk / block / tile / cell tests
// (rt_cgbuild.h) and the host builders' CSR layouts.  Grids go through in
// batches (their disks and pair lists are scratch); passes:
//   pg_disk_kernel   a wave per (grid, sphere): its disks and (disk, block)
//                    pairs (pairs past maxp and global spheres counted per
//                    grid: the host refuses a sphere grid with more than
//                    kSgMaxGlobal globals or dropped pairs, as
//                    build_sphere_grids refuses it); a light grid's global
//                    sphere goes to its global list (counted, then filled)
//   pg_bin_kernel    a wave per quarter pair, as cg_bin_kernel: <count> adds
//                    1 per listed cell, <fill> takes a slot there and writes
//                    the entry at the cell's CSR offset
//   scan_*           the exclusive prefix of the counts (CSR offsets)
//   sg_sort_kernel / ids_sort_kernel   a thread per list: (tlo, index) / (nearest distance, index) order
//   sg_start_kernel / lg_start_kernel  the host builders' start arrays
struct GridPt {  // a grid's point and origin-ball radius
  double x, y, z, rho;
};
struct SgBuild {
  const SphGeo *geo;
  const double *rad;
  const GridPt *pts;             // [ng] the batch's grids
  const unsigned char *allglob;  // [ng] or nullptr: 1 = every sphere global (a non-finite light)
  const CubePatch *faces, *blocks, *tiles;
  const double *cell_cbsb;
  CgDisk *disks;         // [ng][n][2]
  int2 *pairs;           // [ng][maxp]
  unsigned *npairs;      // [ng * 16]: pairs per grid (one 64-B line each)
  unsigned *nglob;       // [ng * 16]: global spheres per grid
  const unsigned *woff;  // [ng + 1]: work items (4 per kept pair) before grid j; refused grids have none
  int *cnt;              // [ng][row] (count pass: list lengths; fill pass: slots taken)
  const int *off;        // [(g0 + j) row + c]: the CSR offset of the batch's grid j's list c
  int2 *ent;             // sphere grids: (sphere, tlo bits)
  int32_t *ids;          // light grids: sphere ids
  long long nent;        // entries of all grids (the fill pass's bound)
  int n, ng, g0, N, NT, NB, maxp;
  int row;               // lists per grid: 6 N^2 cells (+ 1 global list: light grids)
  int sides;             // 2: both disks (sphere grids), 1: the disk ahead (light grids)
  int globlist;          // 1: global spheres on the grid's list `row - 1`, not in every cell
  int fill;              // the pass: 0 count, 1 fill
  double diam;
};
static_assert(sizeof(SgBuild) <= 4096, "SgBuild exceeds the kernel-argument segment");
constexpr int kSgCntStride = 16;

// a list entry: at the CSR offset of list ci (batch-local) plus its slot
__device__ __forceinline__ void pg_put(const SgBuild &a, long long ci, int slot, int s, float tlo) {
  const long long e = RT_CK(kCkCgBuild, (long long)a.off[(long long)a.g0 * a.row + ci] + slot, a.nent);
  if (a.ids)
    a.ids[e] = s;
  else
    a.ent[e] = make_int2(s, __float_as_int(tlo));
}

__global__ __launch_bounds__(256) void pg_disk_kernel(const SgBuild a) {
  const int t = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6), lane = (int)(threadIdx.x & 63);
  if (t >= a.n * a.ng) return;
  const int j = t / a.n, i = t - j * a.n;
  const GridPt P = a.pts[j];
  const SphGeo sp = a.geo[i];
  // light grids (one side): spheres within a shadow ray's overshoot of the light are global (kLgOvershoot)
  CgView v = cg_view(sp.cx, sp.cy, sp.cz, a.rad[i], P.x, P.y, P.z, a.diam, P.rho, a.sides == 1 ? kLgOvershoot : 0.0);
  if (a.allglob && a.allglob[j]) v = cg_view(0.0, 0.0, 0.0, __builtin_inf(), 0.0, 0.0, 0.0, 0.0);  // global
  if (v.global && lane == 0) {
    atomicAdd(&a.nglob[j * kSgCntStride], 1u);
    if (a.globlist) {  // the grid's global list
      const long long ci = RT_CK(kCkCgBuild, (long long)j * a.row + a.row - 1, (long long)a.ng * a.row);
      const int slot = atomicAdd(&a.cnt[ci], 1);
      if (a.fill) pg_put(a, ci, slot, i, -__builtin_inff());
    }
  }
  if (v.global && a.globlist) return;
  const int nb = 6 * a.NB * a.NB;
  for (int side = 0; side < (v.global ? 1 : a.sides); ++side) {
    const CgDisk k = cg_side(v, side, i);
    const int di = 2 * t + side;
    if (lane == 0) a.disks[RT_CK(kCkCgBuild, di, 2LL * a.n * a.ng)] = k;
    for (int b0 = 0; b0 < nb; b0 += 64) {
      const int b = b0 + lane;
      const bool m = b < nb && cg_block(k, a.faces, a.blocks, a.NB, b);
      const unsigned long long bm = __ballot(m);
      if (!bm) continue;
      unsigned q0 = 0;
      if (lane == 0) q0 = atomicAdd(&a.npairs[j * kSgCntStride], (unsigned)__builtin_popcountll(bm));
      q0 = (unsigned)__builtin_amdgcn_readfirstlane((int)q0);
      const unsigned qi = q0 + (unsigned)__builtin_popcountll(bm & ((1ull << lane) - 1));
      if (m && qi < (unsigned)a.maxp)
        a.pairs[RT_CK(kCkCgBuild, (size_t)j * a.maxp + qi, (long long)a.ng * a.maxp)] = make_int2(di, b);
    }
  }
}

__global__ __launch_bounds__(64) void pg_bin_kernel(const SgBuild a) {
  const int lane = (int)(threadIdx.x & 63);
  const unsigned total = a.woff[a.ng];
  for (unsigned v = blockIdx.x; v < total; v += gridDim.x) {
    int lo = 0, hi = a.ng;  // the grid of work item v: woff[j] <= v < woff[j + 1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (a.woff[mid] <= v) lo = mid; else hi = mid;
    }
    const int j = lo;
    const unsigned item = v - a.woff[j];
    const int2 pr = a.pairs[RT_CK(kCkCgBuild, (size_t)j * a.maxp + (item >> 2), (long long)a.ng * a.maxp)];
    const CgDisk k = a.disks[RT_CK(kCkCgBuild, pr.x, 2LL * a.n * a.ng)];
    const bool wide = cg_wide(k);
    const int bb = pr.y;
    const int f = bb / (a.NB * a.NB), bj = (bb / a.NB) % a.NB, bi = bb % a.NB;
    bool tm, inside;
    cg_tile(k, a.tiles, a.NT, f, bi, bj, lane, tm, inside);
    unsigned long long tmask = __ballot(tm) & (0xffffull << (16 * (item & 3)));
    const unsigned long long imask = __ballot(inside);
    while (tmask) {
      const int tl = __builtin_ctzll(tmask);
      tmask &= tmask - 1;
      const int gc = cg_cell(k, wide, a.cell_cbsb, a.N, f, bi, bj, tl, lane, (imask >> tl) & 1ull);
      if (gc >= 0) {
        const long long ci = RT_CK(kCkCgBuild, (long long)j * a.row + gc, (long long)a.ng * a.row);
        const int slot = atomicAdd(&a.cnt[ci], 1);
        if (a.fill) pg_put(a, ci, slot, k.s, k.tlo);
      }
    }
  }
}

// Exclusive prefix sum of n ints (x -> y, y[n] = the total), in chunks of
// kScanChunk per 256-thread block: chunk sums, their prefix (one block), then
// each chunk's prefix from its base.
constexpr int kScanChunk = 4096;
__device__ __forceinline__ int block_excl_scan256(int x, int *sh, int &total) {
  const int t = (int)threadIdx.x;
  sh[t] = x;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const int v = t >= o ? sh[t - o] : 0;
    __syncthreads();
    sh[t] += v;
    __syncthreads();
  }
  total = sh[255];
  const int incl = sh[t];
  __syncthreads();
  return incl - x;
}
__global__ __launch_bounds__(256) void scan_chunk_sums(const int *x, long long n, long long *bsum) {
  __shared__ long long sh[256];
  const long long b0 = (long long)blockIdx.x * kScanChunk;
  long long s = 0;
  for (int k = threadIdx.x; k < kScanChunk; k += 256)
    if (b0 + k < n) s += x[b0 + k];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) bsum[blockIdx.x] = sh[0];
}
// in place, exclusive, in 64 bits (bsum[nb] = the total: the caller refuses
// totals past 32 bits before using the offsets); a few thousand chunk sums at
// most, serially in one thread
__global__ __launch_bounds__(64) void scan_sums(long long *bsum, int nb) {
  if (threadIdx.x != 0) return;
  long long run = 0;
  for (int k = 0; k < nb; ++k) {
    const long long v = bsum[k];
    bsum[k] = run;
    run += v;
  }
  bsum[nb] = run;
}
__global__ __launch_bounds__(256) void scan_apply(const int *x, long long n, const long long *bsum, int *y) {
  __shared__ int sh[256];
  constexpr int kPer = kScanChunk / 256;
  const long long b0 = (long long)blockIdx.x * kScanChunk + (long long)threadIdx.x * kPer;
  int v[kPer], s = 0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    v[k] = b0 + k < n ? x[b0 + k] : 0;
    s += v[k];
  }
  int tot;
  int run = (int)bsum[blockIdx.x] + block_excl_scan256(s, sh, tot);
#pragma unroll
  for (int k = 0; k < kPer; ++k)
    if (b0 + k < n) {
      y[b0 + k] = run;
      run += v[k];
    }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) y[n] = (int)bsum[gridDim.x];
}

// Sphere s's row of CSR starts (every sphere has one, as on the host): its
// grid's offsets, or an empty list everywhere (no grid / refused).
__global__ __launch_bounds__(256) void sg_start_kernel(const int *gidx, const unsigned char *ok, const int *off,
                                                       int n, long long cells, int *start) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x, row = cells + 1;
  if (k >= (long long)n * row) return;
  const int s = (int)(k / row);
  const long long c = k - (long long)s * row;
  const int j = gidx[s];
  start[k] = (j >= 0 && ok[j]) ? off[(long long)j * cells + c] : 0;
}

// A light grid's start row (build_light_grid: stride 6N^2 + 2, the global
// list last): the CSR offsets of its 6N^2 + 1 lists and their end.
__global__ __launch_bounds__(256) void lg_start_kernel(const int *off, int nl, long long cells, int *start) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x, row = cells + 2;
  if (k >= (long long)nl * row) return;
  const long long l = k / row, c = k - l * row;
  start[k] = off[l * (cells + 1) + c];  // c = cells + 1: the next light's first offset (or the total)
}

// A thread per list: ascending ids (insertion sort); with `near` (light
// grids) ascending by the sphere's nearest distance from the grid's point
// (|C - P| - |r|, then the id), so a shadow query meets the spheres between
// its point and the light before those beyond it -- the lists' order is free:
// a shadow query is an any-hit test (scene.h:78-82).
__device__ __forceinline__ double near_key(const SphGeo *geo, const GridPt &p, int i) {
  const SphGeo s = geo[i];
  const double dx = s.cx - p.x, dy = s.cy - p.y, dz = s.cz - p.z;
  return __builtin_sqrt(dx * dx + dy * dy + dz * dz) - __builtin_sqrt(s.rr);
}
__global__ __launch_bounds__(256) void ids_sort_kernel(const int *off, long long nlists, int32_t *ids,
                                                       const SphGeo *geo, const GridPt *pts, long long row, int near) {
  const long long gc = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gc >= nlists) return;
  int32_t *e = ids + off[gc];
  const int cnt = off[gc + 1] - off[gc];
  const GridPt p = near ? pts[gc / row] : GridPt{};
  for (int k = 1; k < cnt; ++k) {
    const int32_t x = e[k];
    const double kx = near ? near_key(geo, p, x) : 0.0;
    int m = k - 1;
    while (m >= 0) {
      const double km = near ? near_key(geo, p, e[m]) : 0.0;
      if (!(kx < km || (!(km < kx) && x < e[m]))) break;
      e[m + 1] = e[m];
      --m;
    }
    e[m + 1] = x;
  }
}

// A thread per cell of every grid: its list in (tlo, index) order (insertion sort).
__global__ __launch_bounds__(256) void sg_sort_kernel(const int *off, long long ncells, int2 *ent) {
  const long long gc = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gc >= ncells) return;
  int2 *e = ent + off[gc];
  const int cnt = off[gc + 1] - off[gc];
  for (int k = 1; k < cnt; ++k) {
    const int2 x = e[k];
    const float tx = __int_as_float(x.y);
    int m = k - 1;
    while (m >= 0 && cg_before(tx, x.x, __int_as_float(e[m].y), e[m].x)) {
      e[m + 1] = e[m];
      --m;
    }
    e[m + 1] = x;
  }
}

}  // namespace rtk

using namespace rtk;

constexpr int kBvhAlwaysAbove = 1024;
constexpr size_t kUgMaxEntries = size_t(64) << 20;  // behind-grid list entries (20 B each)

struct rt_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t switch_ev = nullptr;  // rt_set_stream: orders the new stream after the old one
  SphGeo *d_geo = nullptr;
  double *d_rad = nullptr;  // |radius|, for the conservative cull only
  SphMat *d_mat = nullptr;
  bool cull = true;
  // BVH over the spheres (fallback for incoherent groups), built at upload
  BvhNode *d_bvh = nullptr;
  int32_t *d_prims = nullptr;
  float4 *d_pf = nullptr;
  BvhNode2 *d_bvh2 = nullptr;
  int bvh2_root = -1, bvh_depth = 0, bvh_ordered = 1;  // RT_HIP_BVH_ORDERED
  BvhNode4 *d_bvh4 = nullptr;  // 4-wide nodes for the ordered walk (RT_HIP_BVH4=0: two-child walk)
  int bvh4_root = -1, bvh4_stack = 0, bvh_wide = 1;
  int bvh_nodes = 0;
  int bvh2_nodes = 0, bvh4_nodes = 0, bvh_prims = 0;  // sizes the RT_CHECK build checks node / leaf indices against
  // per-light direction grids for shadow rays (rt_lightgrid.h), built at upload
  int32_t *d_lg_start = nullptr, *d_lg_ids = nullptr;
  int lg_n = 128, lg_on = 1;  // lg_n: the grid of the uploaded scene
  long long lg_nstart = 0, lg_nids = 0;
  int lg_n_opt = 0;            // RT_HIP_SHADOW_GRID_N; 0 = 128, or 768 above kBvhAlwaysAbove spheres
  double lg_max_off = 0.0;
  bool lg_off_free = false;  // shadow queries skip the per-ray max_off check (light_grids)
  // camera grids (rt_device.h CgArgs), built on the device per camera
  // position of a launch (cg_bin_kernel / cg_sort_kernel) and kept while the
  // positions and the scene stay the same
  int cg_mode = 1;    // RT_HIP_CAM_GRID: 0 off, 1 auto (a one-frame launch at a new position sweeps), 2 every launch
  int cg_n_opt = 0;   // RT_HIP_CAM_GRID_N (tuning build); 0 = kCgNStatic / kCgNMoving
  long long cg_budget_opt = -1;  // RT_HIP_CAM_GRID_BUDGET (tuning build): bytes for a launch's grids; -1 = kCgBudgetBytes
  long long cg_maxp_opt = -1;    // RT_HIP_CAM_GRID_MAXP (tuning build): pairs per grid kept; -1 = the pair budget
  int32_t *d_cg_count = nullptr;
  int2 *d_cg_ent = nullptr;
  CgDisk *d_cg_disks = nullptr;
  int2 *d_cg_pairs = nullptr;
  unsigned *d_cg_npairs = nullptr;
  size_t cg_count_cap = 0, cg_ent_cap = 0, cg_disks_cap = 0, cg_pairs_cap = 0, cg_npairs_cap = 0;  // bytes
  int cg_n = 0, cg_ngrid = 0;
  std::vector<double> cg_pos;          // the grids' points (3 per grid)
  std::vector<double> cg_seen;         // the previous launch's camera positions
  unsigned long long cg_seen_gen = ~0ull;
  unsigned long long cg_gen = ~0ull;   // scene_gen they were built for
  struct CgTables {                    // the cube map's patch tables of one N on the device
    int N = 0, NT = 0, NB = 0;
    CubePatch *faces = nullptr, *blocks = nullptr, *tiles = nullptr;
    double *cell = nullptr;
  };
  CgTables cg_tab[2];
  int cg_tab_next = 0;
  std::vector<double> h_sx, h_sy, h_sz, h_sr;  // sphere centres and radii (grid builds)
  // sphere grids (rt_lightgrid.h build_sphere_grids): the closest hit of
  // reflection rays in the kFast kernels, built at upload for the reflective
  // spheres
  int sg_mode = -1;  // RT_HIP_SPHERE_GRID: -1 auto (scenes of up to kSgMaxSpheres spheres), 0 off, 1 on
  int sg_n_opt = 0;  // RT_HIP_SPHERE_GRID_N; 0 = kSgN
  int32_t *d_sg_start = nullptr;
  int2 *d_sg_ent = nullptr;
  double *d_sg_rho2 = nullptr;
  int sg_n = 0, sg_grids = 0;
  long long sg_nstart = 0, sg_nent = 0;
  bool sg_ok = false;
  size_t sg_entries = 0;
  double sg_build_ms = 0.0;
  // RT_HIP_SPHERE_GRID auto: the grids are built by the scene's first launch
  // of more than one frame, or its second launch -- not by rt_upload_scene: a
  // one-image render (the drop-in ray_serial) spends ~1.8 ms building 143
  // grids (synth200) that save it ~0.05 ms of kernel time
  std::vector<rt_sphere> sg_src;  // the uploaded spheres (centres, radii, reflectivities)
  double sg_diam = 0.0;
  bool sg_pending = false;
  long long scene_launches = 0;  // render launches since the scene was uploaded
  double bvh_build_ms = 0.0, lg_build_ms = 0.0;  // rt_upload_scene's host builds (rt_info)
  int nsph_up = 0;  // spheres of the scene being uploaded (the device grid builders)
  // behind grid (rt_bvh.h build_ugrid): the backward half of the ordered
  // walks' closest-hit lines (rt_device.h behind_cells), built at upload
  int ug_mode = -1;  // RT_HIP_BEHIND_GRID: -1 auto (scenes above kBvhAlwaysAbove spheres), 0 off, 1 on
  // RT_HIP_GRID_CLOSEST: 1 (default) = with the grid, closest hits walk it along the whole line instead of the
  // BVH (rt_device.h grid_closest_line; synth10k 3.03 -> 2.93 ms per frame, profiles/r3u); 0 = the ordered BVH
  // walk ahead of the origin + behind_cells behind it (3.15 ms: the grid walk behind the origin costs more than
  // the BVH boxes it replaces)
  int ug_closest = 1;
  int32_t *d_ug_rid = nullptr, *d_ug_ids = nullptr, *d_ug_glob = nullptr;
  UgRec *d_ug_rec = nullptr, *d_ug_q = nullptr;
  double ug_cells = 2.0;  // RT_HIP_GRID_CELLS: cells per listed sphere
  UgArgs ug{};        // its device arguments (on = 0 until a launch allows it)
  float ug_reg_margin = 0.0f, ug_extent = 0.0f;
  bool ug_ok = false;
  bool ug_last = false;  // the most recent launch used it
  size_t ug_entries = 0;
  double ug_build_ms = 0.0;
  double c0[3] = {0, 0, 0};
  double lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};  // bounds of spheres and lights
  double rmax = 0;
  int bvh_min = 24, bvh_on = 1, bvh_groups = 2, bvh_leaf = 4;
  // RT_HIP_BVH_LEAF; 0 = 2, or 1 above kBvhAlwaysAbove spheres (rt_upload_scene)
  int bvh_leaf_opt = 0;
  // -1 (auto): every group walks the BVH when the scene has more than
  // kBvhAlwaysAbove spheres (a linear cull sweep is O(n) per group)
  int bvh_always = -1;
  int n_cu = 256;
  LightD *d_lights = nullptr;
  int nsph = 0, nlight = 0;
  double amb[3] = {0, 0, 0};
  bool has_scene = false;
  // Counters: two halves of one allocation, alternating by launch; d_counters
  // is the half of the latest launch (what rt_render_stats reads).  A
  // render_kernel launch zeroes the other half for the next launch, so the
  // default path needs no separate memset (a fill kernel per frame).
  unsigned long long *d_counters = nullptr;
  unsigned long long *d_ctr_base = nullptr;
  bool ctr_clean[2] = {true, true};
  bool zero_pending = false;  // the launch being enqueued zeroes the other half
  unsigned long long *h_counters = nullptr;  // pinned
  // In-stream HIP events around every render launch (a ring), so a caller can
  // time a whole region of launches and read the per-launch durations after.
  static constexpr int kRing = 256;
  hipEvent_t ev0[kRing] = {}, ev1[kRing] = {};
  long long launches = 0, hist_begin = 0;
  uint8_t *d_tmp = nullptr;
  size_t tmp_bytes = 0;
  int samples = 1;  // 4: the antialias mode (rt_set_antialias)
  int stack_mode = 4;  // RT_HIP_STACK: 4 merged reflection levels (default), 1 per-pixel global stack (one tile per wave)
  // RT_HIP_DEFER: kStackMerge defers rays of level >= kDeferLevel to render_deferred
  // (-1, default: in multi-frame launches only; 0 never; 1 always).  A one-frame
  // launch ends on its slowest chains either way, and the second kernel's own
  // ramp and tail come after them (synth200 single frame 0.455 -> 0.384 ms
  // without it, profiles/r3n/ab_knobs.log; 32-frame launches are 13 % slower
  // per frame without it)
  int defer = -1;
  bool defer_walk = true;  // RT_HIP_DEFER_WALK: deferred rays of a scene whose closest hits always walk the BVH use render_deferred_walk
  int merge_q = 64;           // kStackMerge: the launch's LDS queue entries per wave (launch_render4 picks it)
  int merge_q_max = 64;       // RT_HIP_MERGE_Q: longest queue tried (8, 16, 32 or 64)
  int defer_level = kDeferLevel;  // RT_HIP_DEFER_LEVEL (>= 1)
  int defer_div = RT_DEFER_CAP_DIV;  // RT_HIP_DEFER_DIV (tuning build): queue room = launch pixels / defer_div
  QRay *dq_buf = nullptr;     // its queue (and its slots' stacks), grow-only
  // kStackMerge: the merged waves' stack homes (merge_tiles, home_acquire),
  // twice as many as the render kernel can have resident, and their bitmap
  StackEnt *d_homes = nullptr;
  size_t homes_bytes = 0;
  unsigned long long *d_home_bits = nullptr;
  int home_words = 0;
  const void *occ_kernel = nullptr;  // the occupancy of the last kernel asked (blocks per CU at occ_lds)
  size_t occ_lds = 0;
  int occ_blocks = 0;
  size_t dq_bytes = 0;
  // frames of the launch being enqueued (rt_render_frames_async; 1 otherwise) and their cameras
  int nframes = 1;
  const rt_camera *fcams = nullptr;
  // rt_render_tiles: the requested tiles of the launch being enqueued, and the
  // launch-order buffer of the blocks covering them
  const rt_tile *req_tiles = nullptr;
  int req_n = 0;
  int *d_bperm = nullptr, *h_bperm = nullptr;  // h_bperm pinned
  size_t bperm_cap = 0;
  unsigned char *cstack_buf = nullptr;
  size_t cstack_bytes = 0;
  // RT_HIP_LDS_SCENE=1: stage scenes that fit (<= kLdsBudget) in LDS, 4-wave
  // workgroups.  Off by default: one-wave workgroups reading the scene through
  // L2 free each wave's slot as soon as its own tile is done (synth200:
  // 0.473 -> 0.428 ms), which beats the LDS latency advantage.
  int lds_scene = 0;
  // Launch order of the tiles (rt_sched.h), rebuilt when the view or the
  // scene changes; RT_HIP_SCHED=0 dispatches in scanline order.
  int sched = 1;
  std::vector<SchedSphere> h_refl;  // reflective spheres of the scene
  unsigned long long scene_gen = 0;
  SchedView perm_view{};
  unsigned long long perm_gen = ~0ull;
  int *d_perm = nullptr, *h_perm = nullptr;  // h_perm pinned
  size_t perm_cap = 0;
  long long perm_cls[kSchedClasses] = {};  // tiles per class of the cached order
  // kStackMerge: tiles of this class and above get a wave each (RT_HIP_SINGLE_CLASS
  // for every launch; kSchedClasses = none).  Default: every tile (class >= 0)
  // in one-frame launches, whose end is their slowest wave -- with no deferred
  // kernel after them (defer, below): synth200 0.780 -> 0.372 ms, complex
  // 0.652 -> 0.332 ms (profiles/r3r/ab_knobs.log); none in multi-frame
  // launches, where the other frames fill that tail and four tiles per wave
  // share their reflection rays' passes (class >= 1 there: 0.2285 -> 0.2364 ms
  // per frame, profiles/r3c/ab_single.log)
  int single_class = -1;
  // RT_HIP_TAIL: launches give their last tiles (the lightest, about one per
  // wave slot of the chip: tail_waves per CU over the frames) a wave each
  // (merge_end); 0: four per wave to the end.  RT_HIP_TAIL_WAVES (tuning build)
  int tail = 1;
  int tail_waves = 12;
  // RT_HIP_WIDE (tuning build): the render kernel whose sparse waves spread
  // their light loop over the lanes (shade_hit kWide).  3 (default): the
  // render and the deferred kernels of every fp64 launch; 2: the render kernel
  // only; 1: one-frame launches only; 0: the lane-per-ray loop (synth200 one
  // frame 0.297 -> 0.279 ms, 20 frames 0.1965 -> 0.1932 ms per frame; complex
  // 0.1797 -> 0.1755; profiles/r5o, profiles/r5p/ab_wide.log)
  int wide_mode = 3;
  // RT_HIP_XCD_FRAMES: multi-frame launches put every frame of a tile group on
  // one XCD (render_kernel).  -1 (default): for scenes with the uniform grid
  // (large scenes, whose lists and nodes outgrow an XCD's L2: synth10k 2.58 ->
  // 2.49 ms per frame); synth200 keeps the adjacent order (0.1943 vs 0.1958
  // ms per frame at 32 frames, equal at 20; profiles/r3u/ab_xcd_frames.log)
  int xcd_frames = -1;
  // rt_get_info: host-side builds made by the render calls
  bool cg_last = false;
  int cg_last_n = 0;
  unsigned long long cg_builds = 0, perm_builds = 0;
  double cg_build_ms = 0.0, perm_build_ms = 0.0, upload_ms = 0.0;
  std::string err;
};

namespace {
double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
}  // namespace

namespace {

int fail(rt_ctx *c, hipError_t e, const char *what) {
  if (c) c->err = std::string(what) + ": " + hipGetErrorString(e);
  return e == hipErrorOutOfMemory ? RT_ERR_OUT_OF_MEMORY : RT_ERR_HIP;
}

#define RT_TRY(ctx, call)                           \
  do {                                              \
    hipError_t e_ = (call);                         \
    if (e_ != hipSuccess) return fail(ctx, e_, #call); \
  } while (0)

void free_scene(rt_ctx *c) {
  if (c->d_geo) (void)hipFree(c->d_geo);
  if (c->d_rad) (void)hipFree(c->d_rad);
  if (c->d_mat) (void)hipFree(c->d_mat);
  if (c->d_lights) (void)hipFree(c->d_lights);
  if (c->d_bvh) (void)hipFree(c->d_bvh);
  if (c->d_prims) (void)hipFree(c->d_prims);
  if (c->d_pf) (void)hipFree(c->d_pf);
  c->d_pf = nullptr;
  if (c->d_bvh2) (void)hipFree(c->d_bvh2);
  c->d_bvh2 = nullptr;
  if (c->d_bvh4) (void)hipFree(c->d_bvh4);
  c->d_bvh4 = nullptr;
  if (c->d_lg_start) (void)hipFree(c->d_lg_start);
  if (c->d_lg_ids) (void)hipFree(c->d_lg_ids);
  c->d_lg_start = c->d_lg_ids = nullptr;
  c->cg_gen = ~0ull;
  if (c->d_sg_start) (void)hipFree(c->d_sg_start);
  if (c->d_sg_ent) (void)hipFree(c->d_sg_ent);
  if (c->d_sg_rho2) (void)hipFree(c->d_sg_rho2);
  c->d_sg_start = nullptr;
  c->d_sg_ent = nullptr;
  c->d_sg_rho2 = nullptr;
  c->sg_ok = false;
  c->sg_pending = false;
  c->sg_grids = 0;
  c->sg_entries = 0;
  if (c->d_ug_rec) (void)hipFree(c->d_ug_rec);
  if (c->d_ug_rid) (void)hipFree(c->d_ug_rid);
  if (c->d_ug_ids) (void)hipFree(c->d_ug_ids);
  if (c->d_ug_glob) (void)hipFree(c->d_ug_glob);
  if (c->d_ug_q) (void)hipFree(c->d_ug_q);
  c->d_ug_rid = c->d_ug_ids = c->d_ug_glob = nullptr;
  c->d_ug_rec = c->d_ug_q = nullptr;
  c->ug = UgArgs{};
  c->ug_ok = false;
  c->ug_entries = 0;
  c->d_bvh = nullptr;
  c->d_prims = nullptr;
  c->bvh_nodes = 0;
  c->d_geo = nullptr;
  c->d_rad = nullptr;
  c->d_mat = nullptr;
  c->d_lights = nullptr;
  c->has_scene = false;
}

// BVH arguments for one render: the scene extent includes the camera (the
// origin of primary rays); margin = 1e-6 * (diameter + largest radius).
BvhArgs bvh_args(const rt_ctx *c, const Cam &cam) {
  BvhArgs b{};
  b.nodes = c->d_bvh;
  b.prims = c->d_prims;
  b.pf = c->d_pf;
  b.n2 = c->d_bvh2;
  b.root_ref = c->bvh2_root;
  b.nnodes = (c->bvh_on && c->cull) ? c->bvh_nodes : 0;
  b.nn2 = c->bvh2_nodes;
  b.nn4 = c->bvh4_nodes;
  b.nprims = c->bvh_prims;
  b.n4 = c->d_bvh4;
  b.root4 = c->bvh4_root;
  b.wide = (c->bvh_wide && c->d_bvh4 && c->bvh4_stack <= kOrderedStack) ? 1 : 0;
  b.ordered = (c->bvh_ordered && b.nnodes > 0 && (b.wide || (c->d_bvh2 && c->bvh_depth <= kOrderedStack))) ? 1 : 0;
  if (!b.ordered) b.wide = 0;
  b.odepth = std::max(1, b.wide ? c->bvh4_stack : c->bvh_depth);
  b.ostk = nullptr;  // set in the kernel (LDS), or found at ostk_off
  b.ostk_off = -1;
  b.c0x = c->c0[0];
  b.c0y = c->c0[1];
  b.c0z = c->c0[2];
  const double cp[3] = {cam.px, cam.py, cam.pz};
  double d2 = 0.0;
  for (int k = 0; k < 3; k++) {
    const double l = std::min(c->lo[k], cp[k]), h = std::max(c->hi[k], cp[k]);
    d2 += (h - l) * (h - l);
  }
  b.diam = std::sqrt(d2) + 0.01;  // + the 0.001 origin offsets of secondary rays
  const double m = 1e-6 * (b.diam + c->rmax);
  b.margin = std::isfinite(m) ? (float)(m * (1.0 + 1e-6)) : INFINITY;
  b.pmargin = 4.0f * b.margin;
  if (!std::isfinite(b.diam)) b.diam = INFINITY;
  b.min_cands = c->bvh_min;
  b.always = c->bvh_always >= 0 ? c->bvh_always : (c->nsph > kBvhAlwaysAbove ? 1 : 0);
  b.max_groups = c->bvh_groups;
  // the behind grid, when its listing margin covers this view's prefilter
  // margin plus the DDA's error bound (rt_device.h behind_cells); the ordered
  // walks then skip boxes wholly behind the origin
  b.tf_min = -INFINITY;
  b.ug = UgArgs{};
  if (c->ug_ok && b.nnodes > 0 && b.ordered && b.wide && std::isfinite(b.pmargin) &&
      (double)b.pmargin + 1e-4 * (double)c->ug_extent <= (double)c->ug_reg_margin) {
    b.ug = c->ug;
    b.ug.on = 1;
    b.ug.closest = c->ug_closest;
    b.tf_min = 0.0f;
    // no closest hit walks the BVH then (the shadow queries use the light
    // grids or the stackless walk): no LDS stacks for the ordered walk, so
    // merge_tiles keeps its longest ray queue
    if (b.ug.closest) b.odepth = 0;
  }
  return b;
}

LgArgs lg_args(const rt_ctx *c) {
  LgArgs g{};
  g.start = c->d_lg_start;
  g.ids = c->d_lg_ids;
  g.N = c->lg_n;
  g.on = (c->lg_on && c->cull && c->d_lg_start) ? 1 : 0;
  g.max_off = c->lg_max_off;
  g.off_free = c->lg_off_free ? 1 : 0;
  g.nstart = c->lg_nstart;
  g.nids = c->lg_nids;
  return g;
}

// camera grid cells per cube-map face edge (profiles/r4e/ab_camgrid_n.log,
// per frame of 32-frame launches at one position, synth200 / complex: 512
// 0.1914 / 0.1761 ms, 256 0.1914 / 0.1766, 128 0.1925 / 0.1770, 64 0.1950 /
// 0.1791, no grid 0.2177 / 0.1980): 256 for a launch at one position, 128 for
// a grid per frame (a quarter of the cells to build)
constexpr int kCgNStatic = 256, kCgNMoving = 128;

void free_tables(rt_ctx::CgTables &t);
int upload_tables(rt_ctx *c, int N, rt_ctx::CgTables &t);

// The device patch tables of the cube map with N cells per face edge (two
// kept; replacing one waits for the launches in flight).
int cg_tables(rt_ctx *c, int N, const rt_ctx::CgTables *&out) {
  for (const auto &t : c->cg_tab)
    if (t.N == N) {
      out = &t;
      return RT_OK;
    }
  rt_ctx::CgTables &t = c->cg_tab[c->cg_tab_next];
  c->cg_tab_next ^= 1;
  RT_TRY(c, hipStreamSynchronize(c->stream));
  free_tables(t);
  const int rc = upload_tables(c, N, t);
  if (rc != RT_OK) return rc;
  out = &t;
  return RT_OK;
}

void free_tables(rt_ctx::CgTables &t) {
  for (void *p : {(void *)t.faces, (void *)t.blocks, (void *)t.tiles, (void *)t.cell})
    if (p) (void)hipFree(p);
  t = rt_ctx::CgTables{};
}

// The cube map's patch tables for N cells per face edge, on the device.
int upload_tables(rt_ctx *c, int N, rt_ctx::CgTables &t) {
  std::vector<CubePatch> faces, blocks, tiles;
  std::vector<double> cell;
  int NT = 0, NB = 0;
  cube_tables(N, faces, blocks, tiles, cell, NT, NB);
  RT_TRY(c, hipMalloc(&t.faces, faces.size() * sizeof(CubePatch)));
  RT_TRY(c, hipMalloc(&t.blocks, blocks.size() * sizeof(CubePatch)));
  RT_TRY(c, hipMalloc(&t.tiles, tiles.size() * sizeof(CubePatch)));
  RT_TRY(c, hipMalloc(&t.cell, cell.size() * sizeof(double)));
  RT_TRY(c, hipMemcpy(t.faces, faces.data(), faces.size() * sizeof(CubePatch), hipMemcpyHostToDevice));
  RT_TRY(c, hipMemcpy(t.blocks, blocks.data(), blocks.size() * sizeof(CubePatch), hipMemcpyHostToDevice));
  RT_TRY(c, hipMemcpy(t.tiles, tiles.data(), tiles.size() * sizeof(CubePatch), hipMemcpyHostToDevice));
  RT_TRY(c, hipMemcpy(t.cell, cell.data(), cell.size() * sizeof(double), hipMemcpyHostToDevice));
  t.N = N;
  t.NT = NT;
  t.NB = NB;
  return RT_OK;
}

// grow-only device buffer
template <class T>
int grow(rt_ctx *c, T *&p, size_t &cap, size_t bytes) {
  if (cap >= bytes) return RT_OK;
  RT_TRY(c, hipStreamSynchronize(c->stream));  // launches in flight may read the old one
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  RT_TRY(c, hipMalloc(&p, bytes));
  cap = bytes;
  return RT_OK;
}

// grow-only device buffer that may fail softly: false (error cleared, buffer
// freed) when the memory is not there -- for optional structures
template <class T>
bool grow_soft(rt_ctx *c, T *&p, size_t &cap, size_t bytes) {
  if (cap >= bytes) return true;
  if (hipStreamSynchronize(c->stream) != hipSuccess) return false;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  if (hipMalloc(&p, bytes) != hipSuccess) {
    (void)hipGetLastError();
    p = nullptr;
    return false;
  }
  cap = bytes;
  return true;
}

// Camera-grid memory: the (disk, block) pair lists of one launch's grids take
// at most kCgPairBytes (a grid with more pairs is marked overflowed on the
// device and its rays sweep), and all of a launch's grid buffers at most
// kCgBudgetBytes and half the device's free memory -- the grid is a speed-up,
// so past that (or when an allocation fails) the launch sweeps (RT_OK).
constexpr size_t kCgPairBytes = size_t(128) << 20;
constexpr size_t kCgBudgetBytes = size_t(2) << 30;

// What cam_grid_prepare decided for a launch.
struct CgPlan {
  bool use = false;    // the launch scans grids
  bool build = false;  // ... built by cam_grid_enqueue first
  int N = 0, ngrid = 0, maxp = 0;
  long long nblocks = 0;
  std::vector<double> pos;
  const rt_ctx::CgTables *tab = nullptr;
};

// The camera grids of this launch (plan.use = false: the launch sweeps as
// before): one grid when every frame shares the camera position, else one per
// frame; kept while the positions and the scene stay the same.  The host part
// -- policy, tables, buffers (which may wait for the stream) -- runs before
// the launch's start event; cam_grid_enqueue puts the device passes on the
// stream ahead of the render kernel.
int cam_grid_prepare(rt_ctx *c, const Cam &cam, int nf, CgPlan &p) {
  p = CgPlan{};
  if (c->cg_mode == 0 || !c->cull || c->nsph == 0) return RT_OK;
  std::vector<double> pos{cam.px, cam.py, cam.pz};
  bool same = true;
  for (int f = 1; f < nf; f++) same = same && std::memcmp(c->fcams[f].position, pos.data(), 3 * sizeof(double)) == 0;
  const int ngrid = same ? 1 : nf;
  for (int f = 1; f < ngrid; f++) pos.insert(pos.end(), c->fcams[f].position, c->fcams[f].position + 3);
  const int N = c->cg_n_opt ? c->cg_n_opt : (same ? kCgNStatic : kCgNMoving);
  const size_t cells = 6 * (size_t)N * N;
  if (ngrid * cells * kCgSlots >= (size_t(1) << 31)) return RT_OK;  // the scan's 32-bit slot index: no grid
  const bool cached = c->cg_gen == c->scene_gen && c->cg_n == N && c->cg_ngrid == ngrid && c->cg_pos == pos;
  if (!cached && nf == 1 && c->cg_mode == 1 && !(c->cg_seen_gen == c->scene_gen && c->cg_seen == pos)) {
    // one frame from a position the previous launch did not use: the build
    // (~0.05 ms) costs more than the grid saves that frame (profiles/r4j/);
    // the position's next launch gets the grid
    c->cg_seen = pos;
    c->cg_seen_gen = c->scene_gen;
    return RT_OK;
  }
  c->cg_seen = pos;
  c->cg_seen_gen = c->scene_gen;
  if (cached) {
    p.use = true;
    p.N = N;
    p.ngrid = ngrid;
    return RT_OK;
  }
  // from here the buffers change: the cached grids are gone whatever happens
  c->cg_gen = ~0ull;
  const rt_ctx::CgTables *tab = nullptr;
  int rc = cg_tables(c, N, tab);
  if (rc != RT_OK) return rc;
  const long long nblocks = 6LL * tab->NB * tab->NB;
  // pairs per grid: every (disk, block) pair at most, within the pair budget
  // (a grid past it is marked overflowed on the device), and 4 work items per
  // pair of all grids countable in 32 bits (cg_bin_kernel)
  const unsigned long long worst = 2ull * (unsigned long long)c->nsph * (unsigned long long)nblocks;
  const unsigned long long cap32 = ((1ull << 32) - 1) / (4ull * (unsigned long long)ngrid);
  const unsigned long long budget = std::max<unsigned long long>(1, kCgPairBytes / sizeof(int2) / ngrid);
  int maxp = (int)std::min({worst, cap32, budget, (unsigned long long)INT32_MAX});
  if (c->cg_maxp_opt >= 0) maxp = (int)std::max<long long>(1, std::min<long long>(maxp, c->cg_maxp_opt));
  const size_t b_count = ngrid * cells * sizeof(int32_t), b_ent = ngrid * cells * kCgSlots * sizeof(int2),
               b_np = (size_t)ngrid * kCgCntStride * sizeof(unsigned),
               b_disks = 2 * (size_t)c->nsph * ngrid * sizeof(CgDisk), b_pairs = (size_t)ngrid * maxp * sizeof(int2);
  const size_t total = b_count + b_ent + b_np + b_disks + b_pairs;
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
    (void)hipGetLastError();
    free_b = 0;
  }
  // what the grids hold now counts as available: growing frees it first
  const size_t held = c->cg_count_cap + c->cg_ent_cap + c->cg_npairs_cap + c->cg_disks_cap + c->cg_pairs_cap;
  const size_t limit = c->cg_budget_opt >= 0 ? (size_t)c->cg_budget_opt : kCgBudgetBytes;
  if (total > limit || total > (free_b + held) / 2) return RT_OK;
  if (!grow_soft(c, c->d_cg_count, c->cg_count_cap, b_count) || !grow_soft(c, c->d_cg_ent, c->cg_ent_cap, b_ent) ||
      !grow_soft(c, c->d_cg_npairs, c->cg_npairs_cap, b_np) || !grow_soft(c, c->d_cg_disks, c->cg_disks_cap, b_disks) ||
      !grow_soft(c, c->d_cg_pairs, c->cg_pairs_cap, b_pairs))
    return RT_OK;  // no memory for the grid: this launch sweeps
  p.use = p.build = true;
  p.N = N;
  p.ngrid = ngrid;
  p.maxp = maxp;
  p.nblocks = nblocks;
  p.pos = std::move(pos);
  p.tab = tab;
  return RT_OK;
}

int cam_grid_enqueue(rt_ctx *c, const CgPlan &p, CgArgs &out) {
  out = CgArgs{};
  if (!p.use) return RT_OK;
  const size_t cells = 6 * (size_t)p.N * p.N;
  if (p.build) {
    const auto t0 = std::chrono::steady_clock::now();
    const rt_ctx::CgTables *tab = p.tab;
    const int ngrid = p.ngrid;
    CgBuild b{};
    b.geo = c->d_geo;
    b.rad = c->d_rad;
    b.faces = tab->faces;
    b.blocks = tab->blocks;
    b.tiles = tab->tiles;
    b.cell_cbsb = tab->cell;
    b.count = c->d_cg_count;
    b.ent = c->d_cg_ent;
    b.disks = c->d_cg_disks;
    b.pairs = c->d_cg_pairs;
    b.npairs = c->d_cg_npairs;
    b.maxp = p.maxp;
    b.n = c->nsph;
    b.N = p.N;
    b.NT = tab->NT;
    b.NB = tab->NB;
    b.K = kCgSlots;
    b.ngrid = ngrid;
    for (int g = 0; g < ngrid; g++) {
      b.px[g] = p.pos[3 * g];
      b.py[g] = p.pos[3 * g + 1];
      b.pz[g] = p.pos[3 * g + 2];
      double d2 = 0.0;  // the scene's extent with the point (the grown radius' margin)
      for (int k = 0; k < 3; k++) {
        const double l = std::min(c->lo[k], p.pos[3 * g + k]), h = std::max(c->hi[k], p.pos[3 * g + k]);
        d2 += (h - l) * (h - l);
      }
      b.diam[g] = std::sqrt(d2);
    }
    RT_TRY(c, hipMemsetAsync(c->d_cg_count, 0, ngrid * cells * sizeof(int32_t), c->stream));
    RT_TRY(c, hipMemsetAsync(c->d_cg_npairs, 0, ngrid * kCgCntStride * sizeof(unsigned), c->stream));
    const int nthr = c->nsph * ngrid;
    hipLaunchKernelGGL(cg_disk_kernel, dim3((unsigned)((nthr + 3) / 4)), dim3(256), 0, c->stream, b);
    hipLaunchKernelGGL(cg_bin_kernel, dim3((unsigned)std::min<long long>(8192, 8LL * nthr * p.nblocks)), dim3(64), 0,
                       c->stream, b);
    hipLaunchKernelGGL(cg_sort_kernel, dim3((unsigned)((ngrid * cells + 255) / 256)), dim3(256), 0, c->stream, b);
    RT_TRY(c, hipGetLastError());
    // the grids are valid for later launches only once their passes are on the stream
    c->cg_gen = c->scene_gen;
    c->cg_n = p.N;
    c->cg_ngrid = ngrid;
    c->cg_pos = p.pos;
    c->cg_builds++;
    c->cg_build_ms += ms_since(t0);
  }
  out = CgArgs{c->d_cg_count, c->d_cg_ent, p.N, 1, p.ngrid > 1 ? 1 : 0, p.ngrid};
  return RT_OK;
}

// sphere grid cells per cube-map face edge: 32 up to kSgFineSpheres spheres,
// else 16 (r3s: synth200 0.2031 / 0.2014 / 0.2003 ms per frame at 16 / 24 / 32,
// a 61 / 138 ms build at 16 / 32)
constexpr int kSgN = 16, kSgNFine = 32, kSgFineSpheres = 512;
constexpr int kSgMaxSpheres = 2048;     // RT_HIP_SPHERE_GRID=-1: larger scenes keep the BVH walks
constexpr int kSgMaxGlobal = 32;        // spheres overlapping an origin ball (on every list of its grid)
constexpr size_t kSgMaxEntries = size_t(256) << 20;  // 2 GiB of lists (built on the device)

// device scratch of one upload-time build, freed on every exit path
struct DevScratch {
  std::vector<void *> p;
  template <class T>
  hipError_t alloc(T *&out, size_t bytes) {
    out = nullptr;
    void *q = nullptr;
    const hipError_t e = hipMalloc(&q, bytes ? bytes : 1);
    if (e == hipSuccess) {
      p.push_back(q);
      out = static_cast<T *>(q);
    }
    return e;
  }
  ~DevScratch() {
    for (void *q : p) (void)hipFree(q);
  }
};

// The exclusive prefix sum of x[0 .. n) into y[0 .. n] (y[n] = the total) on
// the stream; `total` the sum in 64 bits (y holds it only when below 2^31).
int device_scan(rt_ctx *c, const int *x, long long n, int *y, long long &total) {
  const long long nb = std::max(1LL, (n + kScanChunk - 1) / kScanChunk);
  DevScratch sc;
  long long *bsum = nullptr;
  RT_TRY(c, sc.alloc(bsum, sizeof(long long) * (size_t)(nb + 1)));
  hipLaunchKernelGGL(scan_chunk_sums, dim3((unsigned)nb), dim3(256), 0, c->stream, x, n, bsum);
  hipLaunchKernelGGL(scan_sums, dim3(1), dim3(64), 0, c->stream, bsum, (int)nb);
  hipLaunchKernelGGL(scan_apply, dim3((unsigned)nb), dim3(256), 0, c->stream, x, n, bsum, y);
  RT_TRY(c, hipGetLastError());
  RT_TRY(c, hipMemcpyAsync(&total, bsum + nb, sizeof(long long), hipMemcpyDeviceToHost, c->stream));
  RT_TRY(c, hipStreamSynchronize(c->stream));  // bsum is freed on return
  return RT_OK;
}

// Point grids on the device (pg_*_kernel passes) for the grids `pts`, each
// with N cells per cube-map face edge: per grid ok (sphere grids: refused past
// max_global global spheres or dropped pairs; light grids: never), the CSR
// offsets of the ng x row lists (device, ng * row + 1 ints, held by `keep`)
// and the entries (`out`: int2 (sphere, tlo) or, for light grids, int ids;
// the caller owns it; nullptr when the lists would exceed max_entries).
struct PgMode {
  int sides, globlist, max_global;
  size_t max_entries;
  // light grids: lists by distance from the point (ids_sort_kernel; synth10k
  // 2.439 -> 2.386 ms per frame against sphere-index order, synth200 and
  // complex within +-0.3 %, profiles/r5x/ab_lg_order.log)
  int near = 0;
};
int point_grids(rt_ctx *c, const std::vector<GridPt> &pts, const std::vector<unsigned char> &allglob, double diam,
                int N, const PgMode &md, DevScratch &keep, int *&d_off, std::vector<unsigned char> &ok,
                long long &total, void *&out) {
  const int n = c->nsph_up, ng = (int)pts.size();
  const long long cells = 6LL * N * N, row = cells + (md.globlist ? 1 : 0);
  out = nullptr;
  total = 0;
  ok.assign((size_t)ng, 0);
  rt_ctx::CgTables tab;
  int rc = upload_tables(c, N, tab);
  struct TabGuard {
    rt_ctx::CgTables &t;
    ~TabGuard() { free_tables(t); }
  } tab_guard{tab};
  if (rc != RT_OK) return rc;
  const long long nblocks = 6LL * tab.NB * tab.NB;
  // pairs kept per grid (past it a sphere grid is refused, as one past the
  // host builder's entry cap; a light grid keeps every pair); grids in batches
  // whose disks and pairs fit kPgScratch
  constexpr size_t kPgScratch = size_t(128) << 20;
  const long long worst = (long long)md.sides * n * nblocks;
  const long long maxp = std::max(1LL, md.globlist ? worst : std::min<long long>(worst, 1 << 22));
  const size_t per_grid = 2 * (size_t)n * sizeof(CgDisk) + (size_t)maxp * sizeof(int2);
  const int batch = (int)std::max<long long>(
      1, std::min<long long>({(long long)ng, (long long)(kPgScratch / per_grid),
                              (long long)(((1ull << 32) - 1) / (4ull * (unsigned long long)maxp))}));
  if (4ull * (unsigned long long)maxp >= (1ull << 32)) return RT_OK;  // a grid's work items past 32 bits: none
  DevScratch sc;
  GridPt *d_pts = nullptr;
  unsigned char *d_ag = nullptr;
  int *d_cnt = nullptr;
  CgDisk *d_disks = nullptr;
  int2 *d_pairs = nullptr;
  unsigned *d_np = nullptr, *d_woff = nullptr;
  RT_TRY(c, sc.alloc(d_pts, sizeof(GridPt) * (size_t)ng));
  RT_TRY(c, sc.alloc(d_ag, (size_t)ng));
  RT_TRY(c, sc.alloc(d_cnt, sizeof(int) * (size_t)(ng * row)));
  RT_TRY(c, keep.alloc(d_off, sizeof(int) * (size_t)(ng * row + 1)));
  RT_TRY(c, sc.alloc(d_disks, 2 * (size_t)std::max(n, 1) * batch * sizeof(CgDisk)));
  RT_TRY(c, sc.alloc(d_pairs, (size_t)maxp * batch * sizeof(int2)));
  RT_TRY(c, sc.alloc(d_np, 2 * sizeof(unsigned) * kSgCntStride * (size_t)batch));
  RT_TRY(c, sc.alloc(d_woff, sizeof(unsigned) * (size_t)(batch + 1)));
  RT_TRY(c, hipMemcpy(d_pts, pts.data(), sizeof(GridPt) * (size_t)ng, hipMemcpyHostToDevice));
  RT_TRY(c, hipMemcpy(d_ag, allglob.data(), (size_t)ng, hipMemcpyHostToDevice));
  RT_TRY(c, hipMemsetAsync(d_cnt, 0, sizeof(int) * (size_t)(ng * row), c->stream));
  SgBuild b{};
  b.geo = c->d_geo;
  b.rad = c->d_rad;
  b.faces = tab.faces;
  b.blocks = tab.blocks;
  b.tiles = tab.tiles;
  b.cell_cbsb = tab.cell;
  b.disks = d_disks;
  b.pairs = d_pairs;
  b.npairs = d_np;
  b.nglob = d_np + kSgCntStride * (size_t)batch;
  b.woff = d_woff;
  b.off = d_off;
  b.n = n;
  b.N = N;
  b.NT = tab.NT;
  b.NB = tab.NB;
  b.maxp = (int)maxp;
  b.row = (int)row;
  b.sides = md.sides;
  b.globlist = md.globlist;
  b.diam = diam;
  std::vector<std::vector<unsigned>> woffs;
  // one batch of grids: disks and pairs (pass 1) -- and, counting, the
  // grids' refusals and work offsets -- then the bin pass
  auto run_batch = [&](int g0, bool fill) -> int {
    const int nbg = std::min(batch, ng - g0);
    b.pts = d_pts + g0;
    b.allglob = d_ag + g0;
    b.ng = nbg;
    b.g0 = g0;
    b.cnt = d_cnt + (size_t)g0 * row;
    b.fill = fill ? 1 : 0;
    RT_TRY(c, hipMemsetAsync(d_np, 0, 2 * sizeof(unsigned) * kSgCntStride * (size_t)batch, c->stream));
    const long long waves = (long long)n * nbg;
    if (waves > 0) hipLaunchKernelGGL(pg_disk_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, c->stream, b);
    RT_TRY(c, hipGetLastError());
    if (!fill) {
      std::vector<unsigned> hn(2 * kSgCntStride * (size_t)batch);
      RT_TRY(c, hipMemcpyAsync(hn.data(), d_np, sizeof(unsigned) * hn.size(), hipMemcpyDeviceToHost, c->stream));
      RT_TRY(c, hipStreamSynchronize(c->stream));
      std::vector<unsigned> wo((size_t)nbg + 1, 0);
      for (int j = 0; j < nbg; j++) {
        const unsigned np = hn[(size_t)j * kSgCntStride], nglob = hn[((size_t)batch + j) * kSgCntStride];
        const bool g_ok = nglob <= (unsigned)md.max_global && np <= (unsigned)maxp;
        ok[(size_t)(g0 + j)] = g_ok ? 1 : 0;
        wo[(size_t)j + 1] = wo[(size_t)j] + (g_ok ? 4u * np : 0u);
      }
      woffs.push_back(wo);
    }
    const std::vector<unsigned> &wo = woffs[(size_t)(g0 / batch)];
    RT_TRY(c, hipMemcpyAsync(d_woff, wo.data(), sizeof(unsigned) * wo.size(), hipMemcpyHostToDevice, c->stream));
    const unsigned items = wo.back();
    if (items) {
      hipLaunchKernelGGL(pg_bin_kernel, dim3((unsigned)std::min<unsigned>(items, 16384u)), dim3(64), 0, c->stream, b);
      RT_TRY(c, hipGetLastError());
    }
    // the host copy of the work offsets is read by the stream: wait before the next batch rewrites them
    RT_TRY(c, hipStreamSynchronize(c->stream));
    return RT_OK;
  };
  for (int g0 = 0; g0 < ng; g0 += batch)
    if ((rc = run_batch(g0, false)) != RT_OK) return rc;
  if (md.globlist)  // a refused light grid's global list holds spheres too: keep it out of the counts
    for (int j = 0; j < ng; j++)
      if (!ok[(size_t)j]) return RT_OK;
  if ((rc = device_scan(c, d_cnt, (long long)ng * row, d_off, total)) != RT_OK) return rc;
  if ((size_t)total > md.max_entries || total > INT32_MAX) return RT_OK;
  const size_t esz = md.globlist ? sizeof(int32_t) : sizeof(int2);
  RT_TRY(c, hipMalloc(&out, esz * ((size_t)total + 1)));
  b.ent = md.globlist ? nullptr : static_cast<int2 *>(out);
  b.ids = md.globlist ? static_cast<int32_t *>(out) : nullptr;
  b.nent = total;
  RT_TRY(c, hipMemsetAsync(d_cnt, 0, sizeof(int) * (size_t)(ng * row), c->stream));
  for (int g0 = 0; g0 < ng; g0 += batch)
    if ((rc = run_batch(g0, true)) != RT_OK) return rc;
  const long long nlists = (long long)ng * row;
  if (md.globlist)
    hipLaunchKernelGGL(ids_sort_kernel, dim3((unsigned)((nlists + 255) / 256)), dim3(256), 0, c->stream, d_off, nlists,
                       b.ids, c->d_geo, d_pts, row, md.near);
  else
    hipLaunchKernelGGL(sg_sort_kernel, dim3((unsigned)((nlists + 255) / 256)), dim3(256), 0, c->stream, d_off, nlists,
                       b.ent);
  RT_TRY(c, hipGetLastError());
  RT_TRY(c, hipStreamSynchronize(c->stream));  // the scratch is freed on return
  return RT_OK;
}

// Sphere grids for the reflective spheres of the scene being uploaded (the
// origins of reflection rays, main.cpp:46, lie within |r| + 0.001 of their
// sphere's centre up to the rounding of the hit point; the ball is grown by a
// relative 1e-6 and the device checks every ray against it), built on the
// device (point_grids; the geometry is on the device already).  No grids (and
// RT_OK) when disabled, too large, or refused.
int sphere_grids(rt_ctx *c) {
  const int n = (int)c->sg_src.size();
  const double diam = c->sg_diam;
  c->sg_pending = false;
  if (c->sg_mode == 0 || (c->sg_mode < 0 && n > kSgMaxSpheres) || n == 0 || !std::isfinite(diam)) return RT_OK;
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<double> rho((size_t)n, -1.0);
  std::vector<int> gidx((size_t)n, -1);
  std::vector<GridPt> pts;
  for (int i = 0; i < n; i++) {
    const rt_sphere &sp = c->sg_src[(size_t)i];
    const double r = std::fabs(sp.radius);
    const double mag = std::fabs(sp.center[0]) + std::fabs(sp.center[1]) + std::fabs(sp.center[2]);
    if (sp.reflectivity > 0.0 && std::isfinite(r) && std::isfinite(mag))  // main.cpp:43
      rho[(size_t)i] = (r + kEps) * (1.0 + 1e-6) + 1e-12 * mag + 1e-9 * diam;
    if (rho[(size_t)i] >= 0.0 && std::isfinite(rho[(size_t)i])) {  // (build_sphere_grids: a finite ball)
      gidx[(size_t)i] = (int)pts.size();
      pts.push_back(GridPt{sp.center[0], sp.center[1], sp.center[2], rho[(size_t)i]});
    }
  }
  const int N = c->sg_n_opt ? c->sg_n_opt : (n <= kSgFineSpheres ? kSgNFine : kSgN);
  // the device indexes grid key's starts at key * (6 N^2 + 1) in 32 bits, and
  // every sphere has its row of starts: refuse grids that would overflow it
  // or hold more than 1 GiB of starts
  const long long cells = 6LL * N * N;
  const size_t nstart = (size_t)n * (size_t)(cells + 1);
  if (nstart > (size_t)INT32_MAX || nstart * sizeof(int32_t) > ((size_t)1 << 30)) return RT_OK;
  const int ng = (int)pts.size();
  c->sg_grids = 0;
  c->sg_entries = 0;
  if (ng == 0 || (long long)ng * cells >= INT32_MAX) {  // (32-bit CSR offsets)
    c->sg_build_ms = ms_since(t0);
    return RT_OK;
  }
  DevScratch keep;
  int *d_off = nullptr;
  std::vector<unsigned char> ok;
  long long total = 0;
  void *ent = nullptr;
  int rc = point_grids(c, pts, std::vector<unsigned char>((size_t)ng, 0), diam, N,
                       PgMode{2, 0, kSgMaxGlobal, kSgMaxEntries}, keep, d_off, ok, total, ent);
  c->d_sg_ent = static_cast<int2 *>(ent);  // owned by the context from here (free_scene)
  if (rc != RT_OK) return rc;
  int grids = 0;
  for (int j = 0; j < ng; j++) grids += ok[(size_t)j];
  if (!ent || grids == 0) {  // as build_sphere_grids past max_entries: no grids
    c->sg_build_ms = ms_since(t0);
    return RT_OK;
  }
  DevScratch sc;
  int *d_gidx = nullptr;
  unsigned char *d_ok = nullptr;
  RT_TRY(c, sc.alloc(d_gidx, sizeof(int) * (size_t)n));
  RT_TRY(c, sc.alloc(d_ok, (size_t)ng));
  RT_TRY(c, hipMemcpy(d_gidx, gidx.data(), sizeof(int) * (size_t)n, hipMemcpyHostToDevice));
  RT_TRY(c, hipMemcpy(d_ok, ok.data(), (size_t)ng, hipMemcpyHostToDevice));
  RT_TRY(c, hipMalloc(&c->d_sg_start, sizeof(int32_t) * nstart));
  RT_TRY(c, hipMalloc(&c->d_sg_rho2, sizeof(double) * (size_t)n));
  hipLaunchKernelGGL(sg_start_kernel, dim3((unsigned)((nstart + 255) / 256)), dim3(256), 0, c->stream, d_gidx, d_ok,
                     d_off, n, cells, c->d_sg_start);
  RT_TRY(c, hipGetLastError());
  std::vector<double> rho2((size_t)n);
  for (int i = 0; i < n; i++) {
    const int j = gidx[(size_t)i];
    rho2[(size_t)i] = (j >= 0 && ok[(size_t)j]) ? rho[(size_t)i] * rho[(size_t)i] : -1.0;
  }
  RT_TRY(c, hipMemcpy(c->d_sg_rho2, rho2.data(), sizeof(double) * (size_t)n, hipMemcpyHostToDevice));
  RT_TRY(c, hipStreamSynchronize(c->stream));  // the scratch is freed on return
  c->sg_n = N;
  c->sg_nstart = (long long)nstart;
  c->sg_nent = total;
  c->sg_ok = true;
  c->sg_grids = grids;
  c->sg_entries = (size_t)total;
  c->sg_build_ms = ms_since(t0);
  return RT_OK;
}

// The per-light direction grids for shadow rays (rt_lightgrid.h
// build_light_grid's lists and layout), built on the device (point_grids,
// one side, global lists); the host builder when the device lists would not
// fit 32-bit offsets.
int light_grids(rt_ctx *c, const rt_scene *s, double diam) {
  const auto t0 = std::chrono::steady_clock::now();
  const int n = s->num_spheres, nl = s->num_lights, N = c->lg_n;
  const long long cells = 6LL * N * N;
  c->lg_max_off = std::isfinite(diam) ? 1e-7 * diam : 0.0;
  {
    // every hit point lies on a finite sphere, inside the scene box up to
    // rounding, and every light inside it: with B the box's largest |coordinate|
    // the shadow lines' computed distance from their light stays below
    // 2^-41 (1.01 B + 0.01) (shadow_cells), so the per-ray check can go
    double B = 0.0;
    for (int k = 0; k < 3; k++) B = std::max(B, std::max(std::fabs(c->lo[k]), std::fabs(c->hi[k])));
    c->lg_off_free = std::isfinite(B) && c->lg_max_off > 0.0 && 0x1p-41 * (1.01 * B + 0.01) <= c->lg_max_off;
  }
  const double dm = std::isfinite(diam) ? diam : 0.0;
  std::vector<GridPt> pts((size_t)nl);
  std::vector<unsigned char> allglob((size_t)nl);
  for (int l = 0; l < nl; l++) {
    const rt_light &L = s->lights[l];
    pts[(size_t)l] = GridPt{L.position[0], L.position[1], L.position[2], 0.0};
    allglob[(size_t)l] = !(std::isfinite(L.position[0]) && std::isfinite(L.position[1]) && std::isfinite(L.position[2]));
  }
  int32_t *ids = nullptr;
  long long total = 0;
  bool dev = nl > 0 && (long long)nl * (cells + 2) < INT32_MAX;
  if (dev) {
    DevScratch keep;
    int *d_off = nullptr;
    std::vector<unsigned char> ok;
    void *out = nullptr;
    int rc = point_grids(c, pts, allglob, dm, N, PgMode{1, 1, INT32_MAX, (size_t)INT32_MAX, 1}, keep, d_off,
                         ok, total, out);
    ids = static_cast<int32_t *>(out);
    c->d_lg_ids = ids;  // owned by the context from here (free_scene)
    if (rc != RT_OK) return rc;
    if (ids) {
      const long long nstart = (long long)nl * (cells + 2);
      RT_TRY(c, hipMalloc(&c->d_lg_start, sizeof(int32_t) * (size_t)(nstart + 1)));
      hipLaunchKernelGGL(lg_start_kernel, dim3((unsigned)((nstart + 255) / 256)), dim3(256), 0, c->stream, d_off, nl,
                         cells, c->d_lg_start);
      RT_TRY(c, hipGetLastError());
      RT_TRY(c, hipStreamSynchronize(c->stream));  // d_off is freed on return
      c->lg_nstart = nstart;
      c->lg_nids = total;
    } else {
      dev = false;
    }
  }
  if (!dev) {  // no lights, or lists past 32 bits: the host builder
    std::vector<double> lx((size_t)nl), ly((size_t)nl), lz((size_t)nl);
    for (int l = 0; l < nl; l++) {
      lx[(size_t)l] = s->lights[l].position[0];
      ly[(size_t)l] = s->lights[l].position[1];
      lz[(size_t)l] = s->lights[l].position[2];
    }
    std::vector<int32_t> lg_start, lg_ids;
    build_light_grid(c->h_sx.data(), c->h_sy.data(), c->h_sz.data(), c->h_sr.data(), n, lx.data(), ly.data(),
                     lz.data(), nl, diam, N, lg_start, lg_ids);
    c->lg_nstart = (long long)lg_start.size();
    c->lg_nids = (long long)lg_ids.size();
    if (c->d_lg_ids) (void)hipFree(c->d_lg_ids);
    c->d_lg_ids = nullptr;
    RT_TRY(c, hipMalloc(&c->d_lg_start, sizeof(int32_t) * (lg_start.size() + 1)));
    RT_TRY(c, hipMalloc(&c->d_lg_ids, sizeof(int32_t) * (lg_ids.size() + 1)));
    if (!lg_start.empty())
      RT_TRY(c, hipMemcpy(c->d_lg_start, lg_start.data(), sizeof(int32_t) * lg_start.size(), hipMemcpyHostToDevice));
    if (!lg_ids.empty())
      RT_TRY(c, hipMemcpy(c->d_lg_ids, lg_ids.data(), sizeof(int32_t) * lg_ids.size(), hipMemcpyHostToDevice));
  }
  c->lg_build_ms = ms_since(t0);
  return RT_OK;
}

Cam to_cam(const rt_camera &cm) {
  return Cam{cm.position[0], cm.position[1], cm.position[2], cm.forward[0], cm.forward[1], cm.forward[2],
             cm.right[0],    cm.right[1],    cm.right[2],    cm.up[0],      cm.up[1],      cm.up[2],
             cm.scale};
}

// The tile launch order for this view (rt_sched.h), on the device; rebuilt
// only when the camera, the image/shard geometry, the tile size or the scene
// changed since the last build.
int tile_perm(rt_ctx *c, const Cam &cam, int W, int H, const Rows &rows, const OutDesc &od, int tw, int th,
              long long ntiles, const int *&out) {
  SchedView v{};
  v.px = cam.px, v.py = cam.py, v.pz = cam.pz, v.fx = cam.fx, v.fy = cam.fy, v.fz = cam.fz;
  v.rx = cam.rx, v.ry = cam.ry, v.rz = cam.rz, v.ux = cam.ux, v.uy = cam.uy, v.uz = cam.uz, v.scale = cam.scale;
  v.W = W, v.H = H, v.band = rows.band, v.first = rows.first, v.stride = rows.stride, v.count = rows.count;
  v.x0 = od.x0, v.xw = od.xw, v.tw = tw, v.th = th;
  if (c->perm_gen == c->scene_gen && std::memcmp(&v, &c->perm_view, sizeof v) == 0 && c->d_perm) {
    out = c->d_perm;
    return RT_OK;
  }
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<int> perm;
  long long cls[kSchedClasses] = {};
  tile_order(v, c->h_refl, perm, cls);
  if ((long long)perm.size() != ntiles) return RT_ERR_INVALID_ARG;
  const size_t bytes = perm.size() * sizeof(int);
  RT_TRY(c, hipStreamSynchronize(c->stream));  // the previous order may still be in flight from h_perm
  if (c->perm_cap < bytes) {
    if (c->d_perm) (void)hipFree(c->d_perm);
    if (c->h_perm) (void)hipHostFree(c->h_perm);
    c->d_perm = c->h_perm = nullptr;
    c->perm_cap = 0;
    c->perm_gen = ~0ull;
    RT_TRY(c, hipMalloc(&c->d_perm, bytes));
    RT_TRY(c, hipHostMalloc(&c->h_perm, bytes, hipHostMallocDefault));
    c->perm_cap = bytes;
  }
  std::memcpy(c->h_perm, perm.data(), bytes);
  RT_TRY(c, hipMemcpyAsync(c->d_perm, c->h_perm, bytes, hipMemcpyHostToDevice, c->stream));
  c->perm_view = v;
  c->perm_gen = c->scene_gen;
  for (int k = 0; k < kSchedClasses; k++) c->perm_cls[k] = cls[k];
  out = c->d_perm;
  c->perm_builds++;
  c->perm_build_ms += ms_since(t0);
  return RT_OK;
}

// (Re-)records the launch's start event just before its first kernel: the
// host-side builds a launch may make first (tile order, camera grid) are not
// kernel time.  enqueue() has recorded it already for launches with no kernel.
hipError_t mark_start(rt_ctx *c) { return hipEventRecord(c->ev0[(int)(c->launches % rt_ctx::kRing)], c->stream); }

template <bool kLds, bool kCull, int kSamples, int kStack>
int launch_tiles(rt_ctx *c, size_t lds, const Cam &cam, int W, int H, int depth, const Rows &rows,
                 const OutDesc &od) {
  BvhArgs bv = bvh_args(c, cam);
  const LgArgs lg = lg_args(c);
  constexpr int kWg = wg_waves<kLds>(), kWx = kWg == 4 ? 2 : 1, kWy = kWg / kWx;
  // the ordered walk's stacks follow the scene in LDS (render_kernel)
  if (bv.ordered)
    bv.ostk_off = (int)((lds_layout(kLds, c->nsph, c->nlight, bv.nnodes).end + 31) & ~(size_t)31);
  const int ntx = (od.xw + 8 * kWx - 1) / (8 * kWx), nty = (rows.count + 8 * kWy - 1) / (8 * kWy);
  const long long ntiles = (long long)ntx * nty;
  // frames of this launch (rt_render_frames_async)
  const int nf = c->nframes;
  if (nf < 1 || nf > RT_MAX_FRAMES) return RT_ERR_INVALID_ARG;
  // kStackMerge: one wave per kMergeTiles consecutive tile slots
  long long nslots = kStack == kStackMerge ? (ntiles + kMergeTiles - 1) / kMergeTiles : ntiles;
  if (ntiles * nf > (1LL << 30)) return RT_ERR_INVALID_ARG;
  // rt_render_tiles: the launch visits the blocks (launch tiles) that overlap
  // a requested tile, in scanline order of the blocks
  const int *batch_perm = nullptr;
  if constexpr (kStack == kStackGlobal) {
    if (c->req_tiles) {
      const int bw = 8 * kWx, bh = 8 * kWy;
      std::vector<unsigned char> mark((size_t)ntiles, 0);
      for (int i = 0; i < c->req_n; i++) {
        const rt_tile &t = c->req_tiles[i];
        // in 64 bits: a caller's x + width near INT_MAX must still clip to the image
        const int x1 = (int)std::min<long long>(W, (long long)t.x + t.width);
        const int j1 = (int)std::min<long long>(H, (long long)t.y + t.height);
        if (t.x >= x1 || t.y >= j1) continue;
        // framebuffer rows j (0 = bottom) are PPM rows H-1-j
        const int y0 = H - j1, y1 = H - 1 - t.y;
        for (int by = y0 / bh; by <= y1 / bh; by++)
          for (int bx = t.x / bw; bx <= (x1 - 1) / bw; bx++) mark[(size_t)by * ntx + bx] = 1;
      }
      std::vector<int> list;
      for (long long b = 0; b < ntiles; b++)
        if (mark[(size_t)b]) list.push_back((int)b);
      nslots = (long long)list.size();
      if (nslots == 0) return RT_OK;
      const size_t bytes = list.size() * sizeof(int);
      RT_TRY(c, hipStreamSynchronize(c->stream));  // the previous list may still be in flight from h_bperm
      if (c->bperm_cap < bytes) {
        if (c->d_bperm) (void)hipFree(c->d_bperm);
        if (c->h_bperm) (void)hipHostFree(c->h_bperm);
        c->d_bperm = c->h_bperm = nullptr;
        c->bperm_cap = 0;
        RT_TRY(c, hipMalloc(&c->d_bperm, bytes));
        RT_TRY(c, hipHostMalloc(&c->h_bperm, bytes, hipHostMallocDefault));
        c->bperm_cap = bytes;
      }
      std::memcpy(c->h_bperm, list.data(), bytes);
      RT_TRY(c, hipMemcpyAsync(c->d_bperm, c->h_bperm, bytes, hipMemcpyHostToDevice, c->stream));
      batch_perm = c->d_bperm;
    }
  }
  D3 amb{c->amb[0], c->amb[1], c->amb[2]};
  lds = (lds + 31) & ~(size_t)31;
  // the kernel places the ordered walk's stacks from these same arguments
  if (bv.ordered)
    lds += (size_t)kWg * bv.odepth * 64 * sizeof(int2);
  if (!kLds && kStack == kStackGlobal) lds += (size_t)kWg * 64 * sizeof(D3);  // parked colours (trace_wave)
  if (kStack == kStackMerge)  // the wave's ray queue and finished pixels (merge_tiles)
    lds += (size_t)c->merge_q * sizeof(QRay) + kPixbufBytes;
  StackEnt *gstack = nullptr;
  if (depth > 1 && kStack == kStackGlobal) {
    // the kernel indexes the stack with 32 bits: entry + level * npx < 2^32
    if ((unsigned long long)(depth - 1) * rows.count * od.xw * nf >= (1ull << 32)) return RT_ERR_INVALID_ARG;
    // grow-only: sized for this launch's frames; a later launch of as many
    // frames or fewer (a last partial batch) reuses it
    const size_t need = (size_t)(depth - 1) * rows.count * od.xw * nf * sizeof(StackEnt);
    if (c->cstack_bytes < need) {
      RT_TRY(c, hipStreamSynchronize(c->stream));
      if (c->cstack_buf) (void)hipFree(c->cstack_buf);
      c->cstack_buf = nullptr;
      c->cstack_bytes = 0;
      RT_TRY(c, hipMalloc(&c->cstack_buf, need));
      c->cstack_bytes = need;
    }
    gstack = reinterpret_cast<StackEnt *>(c->cstack_buf);
  }
  const int *perm = nullptr;
  int nsingle = 0;
  long long tail = 0;
  // The heavy-first order pays off when a launch has many more tiles than the
  // chip has wave slots; a small launch (a hybrid driver's 64x64 tile) keeps
  // scanline order and skips building and uploading one (which waits for the
  // stream whenever the tile shape changes).
  if (batch_perm) {
    perm = batch_perm;
  } else if (c->sched && ntiles >= kSchedMinTiles) {
    int rc = tile_perm(c, cam, W, H, rows, od, 8 * kWx, 8 * kWy, ntiles, perm);
    if (rc != RT_OK) return rc;
    if (kStack == kStackMerge) {  // the heaviest classes lead the order: one wave per tile for them
      // one-frame launches: the tiles under reflective spheres (class >= 1) a
      // wave each, the rest four per wave, the last ones (tail) single again
      // (synth200 0.314 -> 0.298 ms, complex 0.293 -> 0.286 against every tile
      // single, profiles/r5g/); multi-frame launches merge every class
      const int sc = c->single_class >= 0 ? c->single_class : (nf == 1 ? 1 : kSchedClasses);
      long long heavy = 0;
      for (int k = sc; k < kSchedClasses; k++) heavy += c->perm_cls[k];
      nsingle = (int)std::min<long long>(heavy, ntiles);
      // multi-frame launches end on their lightest tiles one per wave: about
      // as many as the chip holds waves (12 per CU), over the launch's frames
      if (c->tail)
        tail = std::min<long long>(ntiles - nsingle, ((long long)c->n_cu * c->tail_waves + nf - 1) / nf);
      nslots = nsingle + (ntiles - nsingle - tail + kMergeTiles - 1) / kMergeTiles + tail;
    }
  }
  const bool xcd_frames = nf > 1 && (c->xcd_frames > 0 || (c->xcd_frames < 0 && bv.ug.on));
  const dim3 grid((unsigned)((xcd_frames ? (nslots + 7) / 8 * 8 : nslots) * nf));
  RenderArgs ra{};
  ra.geo = c->d_geo;
  ra.radius = c->d_rad;
  ra.mat = c->d_mat;
  ra.lights = c->d_lights;
  ra.n = c->nsph;
  ra.nl = c->nlight;
  ra.amb = amb;
  ra.cam[0] = cam;
  for (int f = 1; f < nf; f++) ra.cam[f] = to_cam(c->fcams[f]);
  ra.frames = nf;
  ra.W = W;
  ra.H = H;
  ra.depth = depth;
  ra.rows = rows;
  ra.bv = bv;
  c->ug_last = bv.ug.on != 0;
  ra.lg = lg;
  ra.od = od;
  ra.gstack = gstack;
  ra.counters = c->d_counters;
  ra.ntx = ntx;
  ra.ntiles = (int)ntiles;
  ra.nslots = (int)nslots;
  ra.perm = perm;
  // zero the other counter half for the next launch (enqueue's alternation)
  const int next = (int)((c->launches + 1) & 1);
  ra.zero_next = c->d_ctr_base + (size_t)next * kShards * kShardStride;
  c->zero_pending = true;
  ra.dq = nullptr;
  ra.dq_cap = 0;
  ra.merge_q = c->merge_q;
  ra.nsingle = nsingle;
  ra.merge_end = (int)(ntiles - tail);
  // merge_tiles' pixel bytes: after the scene and the walk stacks, where render_kernel's park/queue region starts
  ra.pix_off = (int)(((lds_layout(kLds, c->nsph, c->nlight, bv.nnodes).end + 31) & ~(size_t)31) +
                     (bv.ordered ? (size_t)kWg * bv.odepth * 64 * sizeof(int2) : 0));
  // row k of frame f starts at ptr + f fstride + 3 (k W + x): dword aligned for every k, f and x = 8i
  ra.rows_dword = ((reinterpret_cast<uintptr_t>(od.ptr) | (uintptr_t)(3 * (size_t)W) | (uintptr_t)od.fstride) & 3) == 0;
  ra.defer_level = c->defer_level;
  ra.xcd_frames = xcd_frames ? 1 : 0;
  if (kStack == kStackMerge && (c->defer > 0 || (c->defer < 0 && nf > 1)) && depth > c->defer_level) {
    // room for 1/8 of the launch's pixels (deferred rays are ~2 % on synth200); a ray
    // that finds its shard segment full simply continues in its merge_tiles lane.
    // Each queue slot has its chain's stack after the queue: [depth-1][kShards * cap]
    const size_t npx = (size_t)rows.count * od.xw * nf;
    const size_t cap = std::max<size_t>(64, ((npx / kShards / (size_t)c->defer_div) + 63) & ~(size_t)63);
    const size_t need = cap * kShards * (sizeof(QRay) + (size_t)(depth - 1) * sizeof(StackEnt));
    // the queue is a speed-up: past the 32-bit slot-stack index, or when the
    // memory is not there (grow_soft), the launch runs without deferral
    if (cap < (size_t)1 << 30 && (unsigned long long)cap * kShards * (unsigned)(depth - 1) < (1ull << 32) &&
        grow_soft(c, c->dq_buf, c->dq_bytes, need)) {
      ra.dq = c->dq_buf;
      ra.dq_cap = (int)cap;
      ra.dstack = reinterpret_cast<StackEnt *>(c->dq_buf + cap * kShards);
    }
  }
  if constexpr (kStack == kStackMerge && !kLds && kSamples == 1) {
    // the default configuration (ordered 4-wide BVH walk, light grids) has kernels
    // compiled with only those paths (kFast): no registers held for the others
    const bool fast = bv.ordered && bv.wide && lg.on;
    // the light loop of sparse waves spread over the lanes (shade_hit kWide, the default)
    const bool wide = fast && (c->wide_mode >= 2 || (nf == 1 && c->wide_mode == 1));
    if (depth > 1) {  // the stack homes: 2 x the render kernel's resident waves
      const void *kf = wide   ? reinterpret_cast<const void *>(&render_kernel<kLds, kCull, kSamples, kStack, true, true>)
                       : fast ? reinterpret_cast<const void *>(&render_kernel<kLds, kCull, kSamples, kStack, true>)
                              : reinterpret_cast<const void *>(&render_kernel<kLds, kCull, kSamples, kStack>);
      if (kf != c->occ_kernel || lds != c->occ_lds) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kf, 64 * kWg, lds) != hipSuccess || nb < 1) {
          (void)hipGetLastError();
          nb = 32;  // the most waves a CU holds
        }
        c->occ_kernel = kf;
        c->occ_lds = lds;
        c->occ_blocks = nb;
      }
      const int words = (int)(((long long)2 * c->occ_blocks * kWg * c->n_cu + 63) / 64);
      const size_t hb = (size_t)words * 64 * (size_t)(depth - 1) * kHomePx * sizeof(StackEnt);
      if (c->homes_bytes < hb || c->home_words < words) {
        RT_TRY(c, hipStreamSynchronize(c->stream));  // launches in flight hold homes
        if (c->d_homes) (void)hipFree(c->d_homes);
        if (c->d_home_bits) (void)hipFree(c->d_home_bits);
        c->d_homes = nullptr;
        c->d_home_bits = nullptr;
        c->homes_bytes = 0;
        c->home_words = 0;
        RT_TRY(c, hipMalloc(&c->d_homes, hb));
        RT_TRY(c, hipMalloc(&c->d_home_bits, (size_t)words * sizeof(unsigned long long)));
        // zero once: every wave returns the home it took, so a drained launch leaves the bitmap zero
        RT_TRY(c, hipMemset(c->d_home_bits, 0, (size_t)words * sizeof(unsigned long long)));
        c->homes_bytes = hb;
        c->home_words = words;
      }
      ra.homes = c->d_homes;
      ra.home_bits = c->d_home_bits;
      ra.home_words = c->home_words;
    }
    // the sphere grids, lazily (sg_pending): the scene's first multi-frame
    // launch or its second launch builds them, before the launch's timing
    // (a speed-up: if its build fails the launch runs without the grids)
    if (fast && kCull && c->sg_pending && (nf > 1 || c->scene_launches > 0)) {
      if (sphere_grids(c) != RT_OK) {
        (void)hipGetLastError();
        c->err.clear();
        c->sg_ok = false;
      }
    }
    // the camera grids' host part (policy, tables, buffers) first; the
    // launch's timing starts after it: the grids' device passes ahead of the
    // render kernel are part of the launch
    CgPlan plan;
    if (fast && kCull) {
      const int rc = cam_grid_prepare(c, cam, nf, plan);
      if (rc != RT_OK) return rc;
    }
    RT_TRY(c, mark_start(c));
    {
      const int rc = cam_grid_enqueue(c, plan, ra.cg);
      if (rc != RT_OK) return rc;
    }
    if (fast && kCull && c->sg_ok)
      ra.sg = SgArgs{c->d_sg_start, c->d_sg_ent, c->d_sg_rho2, c->sg_n, 1, c->sg_nstart, c->sg_nent, c->nsph};
    c->cg_last = ra.cg.on != 0;
    c->cg_last_n = ra.cg.on ? ra.cg.N : 0;
    if (wide)
      hipLaunchKernelGGL((render_kernel<kLds, kCull, kSamples, kStack, true, true>), grid, dim3(64 * kWg), lds, c->stream,
                         ra);
    else if (fast)
      hipLaunchKernelGGL((render_kernel<kLds, kCull, kSamples, kStack, true>), grid, dim3(64 * kWg), lds, c->stream, ra);
    else
      hipLaunchKernelGGL((render_kernel<kLds, kCull, kSamples, kStack>), grid, dim3(64 * kWg), lds, c->stream, ra);
    if (ra.dq_cap > 0) {  // 48 one-wave workgroups per shard segment
      // the walk kernel where every closest hit walks the BVH anyway (large
      // scenes: synth10k 12.2 -> 11.0 ms per 8-frame launch); small scenes keep
      // the cull sweeps (synth200 1 % slower on the walk kernel)
      if (kCull && fast && c->defer_walk && bv.nnodes > 0 && bv.always && !(bv.ug.on && bv.ug.closest))
        hipLaunchKernelGGL(render_deferred_walk, dim3(RT_DEFER_WGS * kShards), dim3(64), lds, c->stream, ra);
      else if (fast && c->wide_mode == 3)  // the deferred waves' tails spread their light loops too
        hipLaunchKernelGGL((render_deferred<kCull, true, true>), dim3(RT_DEFER_WGS * kShards), dim3(64), lds, c->stream,
                           ra);
      else if (fast)
        hipLaunchKernelGGL((render_deferred<kCull, true>), dim3(RT_DEFER_WGS * kShards), dim3(64), lds, c->stream, ra);
      else
        hipLaunchKernelGGL((render_deferred<kCull>), dim3(RT_DEFER_WGS * kShards), dim3(64), lds, c->stream, ra);
    }
  } else {
    RT_TRY(c, mark_start(c));
    hipLaunchKernelGGL((render_kernel<kLds, kCull, kSamples, kStack>), grid, dim3(64 * kWg), lds, c->stream, ra);
    if constexpr (kStack == kStackMerge) {
      if (ra.dq_cap > 0)
        hipLaunchKernelGGL((render_deferred<kCull>), dim3(RT_DEFER_WGS * kShards), dim3(64), lds, c->stream, ra);
    }
  }
  return RT_OK;
}

template <bool kLds, bool kCull, int kSamples>
int launch_render4(rt_ctx *c, size_t lds, const Cam &cam, int W, int H, int depth, const Rows &rows,
                   const OutDesc &od) {
  if (c->stack_mode == kStackMerge) {
    // merged reflection levels: RGB8 row-compact output, one sample, scene through L2,
    // and only while the wave's LDS (BVH stacks + ray queue) still allows the
    // 12 waves per CU its registers allow (synth10k's 22-entry stacks do not:
    // 10 waves, 12 % slower); otherwise the per-pixel global stack
    if constexpr (!kLds && kSamples == 1) {
      const BvhArgs bv = bvh_args(c, cam);
      const size_t stacks = bv.ordered ? (size_t)bv.odepth * 64 * sizeof(int2) : 0;
      if (od.fmt == RT_FB_RGB8 && !od.full && od.x0 == 0 && od.xw == W)
        for (int q = c->merge_q_max; q >= 8; q /= 2)  // the longest queue that keeps 12 waves per CU
          if (12 * (stacks + (size_t)q * sizeof(QRay) + kPixbufBytes + ((lds + 31) & ~(size_t)31)) <= 160 * 1024) {
            c->merge_q = q;
            return launch_tiles<kLds, kCull, 1, kStackMerge>(c, lds, cam, W, H, depth, rows, od);
          }
    }
    return launch_tiles<kLds, kCull, kSamples, kStackGlobal>(c, lds, cam, W, H, depth, rows, od);
  }
  return launch_tiles<kLds, kCull, kSamples, kStackGlobal>(c, lds, cam, W, H, depth, rows, od);
}

int launch_render(rt_ctx *c, bool lds_geo, size_t lds, const Cam &cam, int W, int H, int depth, const Rows &rows,
                  const OutDesc &od) {
  const bool aa = c->samples == 4;
  if (lds_geo) {
    if (c->cull) return aa ? launch_render4<true, true, 4>(c, lds, cam, W, H, depth, rows, od)
                           : launch_render4<true, true, 1>(c, lds, cam, W, H, depth, rows, od);
    return aa ? launch_render4<true, false, 4>(c, lds, cam, W, H, depth, rows, od)
              : launch_render4<true, false, 1>(c, lds, cam, W, H, depth, rows, od);
  }
  if (c->cull) return aa ? launch_render4<false, true, 4>(c, lds, cam, W, H, depth, rows, od)
                         : launch_render4<false, true, 1>(c, lds, cam, W, H, depth, rows, od);
  return aa ? launch_render4<false, false, 4>(c, lds, cam, W, H, depth, rows, od)
            : launch_render4<false, false, 1>(c, lds, cam, W, H, depth, rows, od);
}

int validate(rt_ctx *c, const rt_camera *cam, int W, int H, int depth, const rt_rows *rows, const void *out,
             Rows &r) {
  if (!c || !cam || !out || W <= 0 || H <= 0) return RT_ERR_INVALID_ARG;
  if (!c->has_scene) return RT_ERR_NO_SCENE;
  if (depth > RT_MAX_DEPTH) return RT_ERR_DEPTH;
  r = rows ? Rows{rows->band, rows->first, rows->stride, rows->count} : Rows{1, 0, 1, H};
  if (r.band < 1 || r.stride < 1 || r.first < 0 || r.count < 0) return RT_ERR_INVALID_ARG;
  if ((long long)W * 3 * (long long)r.count > (1LL << 40)) return RT_ERR_INVALID_ARG;
  return RT_OK;
}

int enqueue(rt_ctx *c, const rt_camera *cm, int W, int H, int depth, const Rows &r, const OutDesc &od) {
  RT_TRY(c, hipSetDevice(c->device));
  const int half = (int)(c->launches & 1);
  c->d_counters = c->d_ctr_base + (size_t)half * kShards * kShardStride;
  if (!c->ctr_clean[half])
    RT_TRY(c, hipMemsetAsync(c->d_counters, 0, kShards * kShardStride * sizeof(unsigned long long), c->stream));
  c->ctr_clean[half] = false;
  c->zero_pending = false;
  const int slot = (int)(c->launches % rt_ctx::kRing);
  RT_TRY(c, hipEventRecord(c->ev0[slot], c->stream));
  c->cg_last = false;
  c->cg_last_n = 0;
  if (r.count > 0) {
    const Cam cam = to_cam(*cm);
    // the scene and its BVH are staged in LDS when they fit (lds_layout)
    const int nn = (c->bvh_on && c->cull) ? c->bvh_nodes : 0;
    const bool lds_geo = c->lds_scene && lds_layout(true, c->nsph, c->nlight, nn).end <= kLdsBudget;
    const size_t lds = lds_layout(lds_geo, c->nsph, c->nlight, nn).end;
    if (lds > kLdsBudget) {
      c->err = "light list does not fit in LDS";
      return RT_ERR_INVALID_ARG;
    }
    int rc = launch_render(c, lds_geo, lds, cam, W, H, depth, r, od);
    if (rc != RT_OK) return rc;
    RT_TRY(c, hipGetLastError());
  }
  RT_TRY(c, hipEventRecord(c->ev1[slot], c->stream));
  if (c->zero_pending) c->ctr_clean[(c->launches + 1) & 1] = true;
  c->zero_pending = false;
  c->launches++;
  c->scene_launches++;
  return RT_OK;  // the counters are read back by rt_render_stats, after the stream drains
}

}  // namespace

extern "C" {

int rt_device_count(int *count) {
  if (!count) return RT_ERR_INVALID_ARG;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  *count = e == hipSuccess ? n : 0;
  return e == hipSuccess ? RT_OK : RT_ERR_NO_DEVICE;
}

int rt_create(int device, rt_ctx **out) {
  if (!out) return RT_ERR_INVALID_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return RT_ERR_NO_DEVICE;
  if (device < 0 || device >= n) return RT_ERR_INVALID_ARG;
  rt_ctx *c = new rt_ctx();
  c->device = device;
  // Environment knobs.  The product build reads two: RT_HIP_LDS_SCENE (the
  // north star's sphere array and light list staged in LDS per workgroup) and
  // RT_HIP_CAM_GRID (when the camera grid is built: 0 never, 1 auto, 2 for
  // every launch).  The tuning build (-DRT_TUNING: variants/librt_hip_tuning.so)
  // also reads the layout and grid knobs that the parity tests sweep and the
  // A/B scripts measured; every default below is the measured optimum.
  if (const char *e = std::getenv("RT_HIP_LDS_SCENE")) c->lds_scene = std::atoi(e) != 0;
  if (const char *e = std::getenv("RT_HIP_CAM_GRID")) c->cg_mode = std::max(0, std::min(2, std::atoi(e)));
#ifdef RT_TUNING
  if (const char *e = std::getenv("RT_HIP_BVH")) c->bvh_on = std::atoi(e) != 0;
  if (const char *e = std::getenv("RT_HIP_BVH_MIN")) c->bvh_min = std::atoi(e);
  if (const char *e = std::getenv("RT_HIP_BVH_ALWAYS")) c->bvh_always = std::atoi(e) != 0;
  if (const char *e = std::getenv("RT_HIP_BVH_GROUPS")) c->bvh_groups = std::max(1, std::atoi(e));
  if (const char *e = std::getenv("RT_HIP_SHADOW_GRID")) c->lg_on = std::atoi(e) != 0;
  if (const char *e = std::getenv("RT_HIP_SCHED")) c->sched = std::atoi(e) != 0;
  if (const char *e = std::getenv("RT_HIP_STACK")) c->stack_mode = std::atoi(e) == kStackGlobal ? kStackGlobal : kStackMerge;
  if (const char *e = std::getenv("RT_HIP_BVH_ORDERED")) c->bvh_ordered = std::atoi(e) != 0;
  if (const char *e = std::getenv("RT_HIP_BVH4")) c->bvh_wide = std::atoi(e) != 0;
  if (const char *e = std::getenv("RT_HIP_BVH_LEAF")) c->bvh_leaf_opt = std::max(1, std::min(15, std::atoi(e)));
  if (const char *e = std::getenv("RT_HIP_DEFER")) c->defer = std::atoi(e) != 0 ? 1 : 0;
  if (const char *e = std::getenv("RT_HIP_DEFER_WALK")) c->defer_walk = std::atoi(e) != 0;
  if (const char *e = std::getenv("RT_HIP_DEFER_LEVEL")) c->defer_level = std::max(1, std::min(RT_MAX_DEPTH, std::atoi(e)));
  if (const char *e = std::getenv("RT_HIP_MERGE_Q")) c->merge_q_max = std::max(8, std::min(64, std::atoi(e)));
  if (const char *e = std::getenv("RT_HIP_SHADOW_GRID_N")) c->lg_n_opt = std::max(1, std::min(1024, std::atoi(e)));
  if (const char *e = std::getenv("RT_HIP_CAM_GRID_N")) c->cg_n_opt = std::max(1, std::min(1024, std::atoi(e)));
  if (const char *e = std::getenv("RT_HIP_CAM_GRID_BUDGET")) c->cg_budget_opt = std::max(0LL, std::atoll(e));
  if (const char *e = std::getenv("RT_HIP_CAM_GRID_MAXP")) c->cg_maxp_opt = std::max(1LL, std::atoll(e));
  if (const char *e = std::getenv("RT_HIP_SPHERE_GRID")) c->sg_mode = std::max(-1, std::min(1, std::atoi(e)));
  if (const char *e = std::getenv("RT_HIP_SPHERE_GRID_N")) c->sg_n_opt = std::max(1, std::min(256, std::atoi(e)));
  if (const char *e = std::getenv("RT_HIP_BEHIND_GRID")) c->ug_mode = std::max(-1, std::min(1, std::atoi(e)));
  if (const char *e = std::getenv("RT_HIP_GRID_CLOSEST")) c->ug_closest = std::atoi(e) != 0 ? 1 : 0;  // (see ug_closest)
  if (const char *e = std::getenv("RT_HIP_XCD_FRAMES")) c->xcd_frames = std::max(-1, std::min(1, std::atoi(e)));
  if (const char *e = std::getenv("RT_HIP_TAIL")) c->tail = std::atoi(e) != 0;
  if (const char *e = std::getenv("RT_HIP_TAIL_WAVES")) c->tail_waves = std::max(1, std::min(64, std::atoi(e)));
  if (const char *e = std::getenv("RT_HIP_WIDE")) c->wide_mode = std::max(0, std::min(3, std::atoi(e)));
  if (const char *e = std::getenv("RT_HIP_DEFER_DIV")) c->defer_div = std::max(1, std::min(1024, std::atoi(e)));
  if (const char *e = std::getenv("RT_HIP_GRID_CELLS")) c->ug_cells = std::max(0.05, std::min(64.0, std::atof(e)));
  if (const char *e = std::getenv("RT_HIP_SINGLE_CLASS"))
    c->single_class = std::max(0, std::min(kSchedClasses, std::atoi(e)));
#endif
  auto bail = [&](int rc) {
    rt_destroy(c);
    return rc;
  };
  if (hipSetDevice(device) != hipSuccess) return bail(RT_ERR_HIP);
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
      c->n_cu = prop.multiProcessorCount;
  }
  // A blocking stream: it is ordered with the legacy NULL stream (torch's
  // default stream), so buffers a caller fills there are ready before a
  // render on the context's own stream reads or overwrites them, and the
  // caller's later NULL-stream work sees the render's output.
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamDefault) != hipSuccess) return bail(RT_ERR_HIP);
  if (hipEventCreateWithFlags(&c->switch_ev, hipEventDisableTiming) != hipSuccess) return bail(RT_ERR_HIP);
  c->stream = c->own_stream;
  if (hipMalloc(&c->d_ctr_base, 2 * kShards * kShardStride * sizeof(unsigned long long)) != hipSuccess)
    return bail(RT_ERR_OUT_OF_MEMORY);
  if (hipMemset(c->d_ctr_base, 0, 2 * kShards * kShardStride * sizeof(unsigned long long)) != hipSuccess)
    return bail(RT_ERR_HIP);
  c->d_counters = c->d_ctr_base;
  if (hipHostMalloc(&c->h_counters, kShards * kShardStride * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess)
    return bail(RT_ERR_OUT_OF_MEMORY);
  std::memset(c->h_counters, 0, kShards * kShardStride * sizeof(unsigned long long));
  for (int i = 0; i < rt_ctx::kRing; i++)
    if (hipEventCreate(&c->ev0[i]) != hipSuccess || hipEventCreate(&c->ev1[i]) != hipSuccess) return bail(RT_ERR_HIP);
  // The HIP runtime's one-time work in a process, done here rather than
  // inside the first render: the kernels' code object loads at the first
  // launch, and the first blocking host-to-device copy, the first large
  // asynchronous copy (the staging path) each cost ~8 ms on the box
  // (scripts/copy_warm_probe.cpp).  So a drop-in's first render -- the time
  // ray_serial prints, main.cpp:139-163 -- is the render alone.  Once per
  // process and device.
  {
    static std::mutex warm_mu;
    static std::vector<int> warmed;
    std::lock_guard<std::mutex> lk(warm_mu);
    if (std::find(warmed.begin(), warmed.end(), device) == warmed.end()) {
      hipFuncAttributes fa;
      (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(&render_kernel<false, true, 1, kStackMerge, true, true>));
      std::vector<unsigned char> h((size_t)1 << 20);
      void *d = nullptr;
      if (hipMalloc(&d, h.size()) == hipSuccess) {
        (void)hipMemcpy(d, h.data(), 8, hipMemcpyHostToDevice);
        (void)hipMemcpyAsync(d, h.data(), h.size(), hipMemcpyHostToDevice, c->stream);
        (void)hipMemcpyAsync(h.data(), d, h.size(), hipMemcpyDeviceToHost, c->stream);
        (void)hipStreamSynchronize(c->stream);
        (void)hipFree(d);
      }
      (void)hipGetLastError();
      warmed.push_back(device);
    }
  }
  *out = c;
  return RT_OK;
}

void rt_destroy(rt_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
  if (c->stream && c->stream != c->own_stream) (void)hipStreamSynchronize(c->stream);
  free_scene(c);
  if (c->d_ctr_base) (void)hipFree(c->d_ctr_base);
  if (c->h_counters) (void)hipHostFree(c->h_counters);
  if (c->d_tmp) (void)hipFree(c->d_tmp);
  if (c->cstack_buf) (void)hipFree(c->cstack_buf);
  if (c->dq_buf) (void)hipFree(c->dq_buf);
  if (c->d_homes) (void)hipFree(c->d_homes);
  if (c->d_home_bits) (void)hipFree(c->d_home_bits);
  if (c->d_perm) (void)hipFree(c->d_perm);
  if (c->h_perm) (void)hipHostFree(c->h_perm);
  if (c->d_bperm) (void)hipFree(c->d_bperm);
  if (c->h_bperm) (void)hipHostFree(c->h_bperm);
  if (c->d_cg_count) (void)hipFree(c->d_cg_count);
  if (c->d_cg_ent) (void)hipFree(c->d_cg_ent);
  if (c->d_cg_disks) (void)hipFree(c->d_cg_disks);
  if (c->d_cg_pairs) (void)hipFree(c->d_cg_pairs);
  if (c->d_cg_npairs) (void)hipFree(c->d_cg_npairs);
  for (auto &t : c->cg_tab) {
    if (t.faces) (void)hipFree(t.faces);
    if (t.blocks) (void)hipFree(t.blocks);
    if (t.tiles) (void)hipFree(t.tiles);
    if (t.cell) (void)hipFree(t.cell);
  }
  for (int i = 0; i < rt_ctx::kRing; i++) {
    if (c->ev0[i]) (void)hipEventDestroy(c->ev0[i]);
    if (c->ev1[i]) (void)hipEventDestroy(c->ev1[i]);
  }
  if (c->switch_ev) (void)hipEventDestroy(c->switch_ev);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
}

const char *rt_last_error(const rt_ctx *c) { return c ? c->err.c_str() : "null context"; }

int rt_set_stream(rt_ctx *c, void *s) {
  if (!c) return RT_ERR_INVALID_ARG;
  hipStream_t next = s ? (hipStream_t)s : c->own_stream;
  if (next != c->stream) {
    // The context's scratch (reflection stack, deferred queue, counters, tile
    // order) is shared by every launch: work enqueued on the new stream waits
    // for everything already enqueued on the old one.
    RT_TRY(c, hipSetDevice(c->device));
    RT_TRY(c, hipEventRecord(c->switch_ev, c->stream));
    RT_TRY(c, hipStreamWaitEvent(next, c->switch_ev, 0));
    c->stream = next;
  }
  return RT_OK;
}

int rt_set_culling(rt_ctx *c, int enable) {
  if (!c) return RT_ERR_INVALID_ARG;
  c->cull = enable != 0;
  return RT_OK;
}

int rt_upload_scene(rt_ctx *c, const rt_scene *s) {
  if (!c || !s || s->num_spheres < 0 || s->num_lights < 0) return RT_ERR_INVALID_ARG;
  if ((s->num_spheres > 0 && !s->spheres) || (s->num_lights > 0 && !s->lights)) return RT_ERR_INVALID_ARG;
  const auto t_upload = std::chrono::steady_clock::now();
  RT_TRY(c, hipSetDevice(c->device));
  RT_TRY(c, hipStreamSynchronize(c->stream));
  free_scene(c);
  const int n = s->num_spheres, nl = s->num_lights;
  SphGeo *hg = new SphGeo[n + 1];
  double *hr = new double[n + 1];
  SphMat *hm = new SphMat[n + 1];
  LightD *hl = new LightD[nl + 1];
  for (int i = 0; i < n; i++) {
    const rt_sphere &sp = s->spheres[i];
    hg[i] = SphGeo{sp.center[0], sp.center[1], sp.center[2], sp.radius * sp.radius};
    hr[i] = sp.radius < 0 ? -sp.radius : sp.radius;
    hm[i] = SphMat{sp.color[0], sp.color[1], sp.color[2], sp.reflectivity, sp.shininess, 0.0};
  }
  for (int i = 0; i < nl; i++) {
    const rt_light &L = s->lights[i];
    hl[i] = LightD{L.position[0], L.position[1], L.position[2], L.color[0], L.color[1], L.color[2]};
  }
  // scene bounds (spheres and lights), centre, largest radius; BVH relative to the centre
  double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300}, rmax = 0.0;
  auto grow = [&](const double *p, double r) {
    for (int k = 0; k < 3; k++) {
      lo[k] = std::min(lo[k], p[k] - r);
      hi[k] = std::max(hi[k], p[k] + r);
    }
  };
  for (int i = 0; i < n; i++) {
    const double r = std::fabs(s->spheres[i].radius);
    grow(s->spheres[i].center, r);
    if (r > rmax || r != r) rmax = r != r ? INFINITY : r;
  }
  for (int i = 0; i < nl; i++) grow(s->lights[i].position, 0.0);
  double c0[3] = {0, 0, 0};
  if (n + nl > 0)
    for (int k = 0; k < 3; k++) c0[k] = std::isfinite(lo[k] + hi[k]) ? 0.5 * (lo[k] + hi[k]) : 0.0;
  std::vector<double> bx(n), by(n), bz(n), br(n);
  for (int i = 0; i < n; i++) {
    bx[i] = s->spheres[i].center[0] - c0[0];
    by[i] = s->spheres[i].center[1] - c0[1];
    bz[i] = s->spheres[i].center[2] - c0[2];
    br[i] = s->spheres[i].radius;
  }
  const bool big = n > kBvhAlwaysAbove;
  const auto t_bvh = std::chrono::steady_clock::now();
  // leaves of 2 spheres (+0.6..0.9 % over 4 on synth200 with the merged levels);
  // 1 above kBvhAlwaysAbove, where every closest hit walks (synth10k 4.37 -> 4.16 ms)
  c->bvh_leaf = c->bvh_leaf_opt ? c->bvh_leaf_opt : (big ? 1 : 2);
  c->lg_n = c->lg_n_opt ? c->lg_n_opt : (big ? 768 : 128);
  std::vector<BvhNode> nodes;
  std::vector<int32_t> prims;
  build_bvh(bx.data(), by.data(), bz.data(), br.data(), n, c->bvh_leaf, nodes, prims);
  // prefilter records in leaf order (centre - c0 in fp32, |radius| rounded up)
  std::vector<float4> pf(prims.size());
  for (size_t k = 0; k < prims.size(); k++) {
    const int id = prims[k];
    float rr = (float)std::fabs(br[id]);
    if ((double)rr < std::fabs(br[id])) rr = std::nextafter(rr, INFINITY);
    pf[k] = make_float4((float)bx[id], (float)by[id], (float)bz[id], rr);
  }
  std::vector<BvhNode2> nodes2;
  int depth2 = 0;
  const int32_t root2 = build_bvh2(nodes, nodes2, depth2);
  std::vector<BvhNode4> nodes4;
  int stack4 = 0;
  const int32_t root4 = build_bvh4(nodes, nodes4, stack4);
  int rc = RT_OK;
  hipError_t e = hipSuccess;
  if ((e = hipMalloc(&c->d_bvh2, sizeof(BvhNode2) * (nodes2.size() + 1))) != hipSuccess ||
      (e = hipMalloc(&c->d_bvh4, sizeof(BvhNode4) * (nodes4.size() + 1))) != hipSuccess ||
      (!nodes4.empty() && (e = hipMemcpy(c->d_bvh4, nodes4.data(), sizeof(BvhNode4) * nodes4.size(),
                                         hipMemcpyHostToDevice)) != hipSuccess) ||
      (!nodes2.empty() && (e = hipMemcpy(c->d_bvh2, nodes2.data(), sizeof(BvhNode2) * nodes2.size(),
                                         hipMemcpyHostToDevice)) != hipSuccess) ||
      (e = hipMalloc(&c->d_pf, sizeof(float4) * (pf.size() + 1))) != hipSuccess ||
      (!pf.empty() && (e = hipMemcpy(c->d_pf, pf.data(), sizeof(float4) * pf.size(), hipMemcpyHostToDevice)) !=
                          hipSuccess) ||
      (e = hipMalloc(&c->d_bvh, sizeof(BvhNode) * (nodes.size() + 1))) != hipSuccess ||
      (e = hipMalloc(&c->d_prims, sizeof(int32_t) * (prims.size() + 1))) != hipSuccess ||
      (!nodes.empty() &&
       (e = hipMemcpy(c->d_bvh, nodes.data(), sizeof(BvhNode) * nodes.size(), hipMemcpyHostToDevice)) != hipSuccess) ||
      (!prims.empty() &&
       (e = hipMemcpy(c->d_prims, prims.data(), sizeof(int32_t) * prims.size(), hipMemcpyHostToDevice)) != hipSuccess)) {
    rc = fail(c, e, "rt_upload_scene(bvh)");
    free_scene(c);
    delete[] hg;
    delete[] hr;
    delete[] hm;
    delete[] hl;
    return rc;
  }
  c->bvh_build_ms = ms_since(t_bvh);
  if (c->ug_mode > 0 || (c->ug_mode < 0 && big)) {
    const auto t_ug = std::chrono::steady_clock::now();
    UgridHost ug;
    if (build_ugrid(bx.data(), by.data(), bz.data(), br.data(), n, kUgMaxEntries, ug, c->ug_cells)) {
      if ((e = hipMalloc(&c->d_ug_rec, sizeof(UgRec) * ug.rec.size())) != hipSuccess ||
          (e = hipMalloc(&c->d_ug_rid, sizeof(int32_t) * ug.rid.size())) != hipSuccess ||
          (e = hipMalloc(&c->d_ug_q, sizeof(UgRec) * ug.q.size())) != hipSuccess ||
          (e = hipMalloc(&c->d_ug_ids, sizeof(int32_t) * (ug.ids.size() + 1))) != hipSuccess ||
          (e = hipMalloc(&c->d_ug_glob, sizeof(int32_t) * (ug.glob.size() + 1))) != hipSuccess ||
          (e = hipMemcpy(c->d_ug_rec, ug.rec.data(), sizeof(UgRec) * ug.rec.size(), hipMemcpyHostToDevice)) !=
              hipSuccess ||
          (e = hipMemcpy(c->d_ug_rid, ug.rid.data(), sizeof(int32_t) * ug.rid.size(), hipMemcpyHostToDevice)) !=
              hipSuccess ||
          (e = hipMemcpy(c->d_ug_q, ug.q.data(), sizeof(UgRec) * ug.q.size(), hipMemcpyHostToDevice)) != hipSuccess ||
          (!ug.ids.empty() && (e = hipMemcpy(c->d_ug_ids, ug.ids.data(), sizeof(int32_t) * ug.ids.size(),
                                             hipMemcpyHostToDevice)) != hipSuccess) ||
          (!ug.glob.empty() && (e = hipMemcpy(c->d_ug_glob, ug.glob.data(), sizeof(int32_t) * ug.glob.size(),
                                              hipMemcpyHostToDevice)) != hipSuccess)) {
        rc = fail(c, e, "rt_upload_scene(uniform grid)");
        free_scene(c);
        delete[] hg;
        delete[] hr;
        delete[] hm;
        delete[] hl;
        return rc;
      }
      c->ug = UgArgs{reinterpret_cast<const float4 *>(c->d_ug_rec), c->d_ug_rid,
                     reinterpret_cast<const float4 *>(c->d_ug_q), c->d_ug_ids, c->d_ug_glob, (int)ug.glob.size(),
                     ug.nx, ug.ny, ug.nz, ug.gx, ug.gy, ug.gz, ug.cs, 0, 0, (float)(1e-4 * (double)ug.extent),
                     (int)ug.q.size()};
      c->ug_reg_margin = ug.reg_margin;
      c->ug_extent = ug.extent;
      c->ug_entries = ug.ids.size();
      c->ug_ok = true;
    }
    c->ug_build_ms = ms_since(t_ug);
  }
  c->bvh_nodes = (int)nodes.size();
  c->bvh2_nodes = (int)nodes2.size();
  c->bvh4_nodes = (int)nodes4.size();
  c->bvh_prims = (int)prims.size();
  c->bvh2_root = root2;
  c->bvh_depth = depth2;
  c->bvh4_root = root4;
  c->bvh4_stack = stack4;
  double scene_diam = 0.0;
  {
    double d2 = 0.0;
    for (int k = 0; k < 3; k++) d2 += (hi[k] - lo[k]) * (hi[k] - lo[k]);
    const double diam = n + nl > 0 ? std::sqrt(d2) : 0.0;
    std::vector<double> sx(n), sy(n), sz(n);
    for (int i = 0; i < n; i++) {
      sx[i] = s->spheres[i].center[0];
      sy[i] = s->spheres[i].center[1];
      sz[i] = s->spheres[i].center[2];
    }
    c->h_sx = sx;
    c->h_sy = sy;
    c->h_sz = sz;
    c->h_sr = br;
    scene_diam = diam;
  }
  for (int k = 0; k < 3; k++) {
    c->c0[k] = c0[k];
    c->lo[k] = lo[k];
    c->hi[k] = hi[k];
  }
  c->rmax = rmax;
  if ((e = hipMalloc(&c->d_geo, sizeof(SphGeo) * (n + 1))) != hipSuccess ||
      (e = hipMalloc(&c->d_rad, sizeof(double) * (n + 1))) != hipSuccess ||
      (e = hipMalloc(&c->d_mat, sizeof(SphMat) * (n + 1))) != hipSuccess ||
      (e = hipMalloc(&c->d_lights, sizeof(LightD) * (nl + 1))) != hipSuccess ||
      (e = hipMemcpy(c->d_geo, hg, sizeof(SphGeo) * n, hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMemcpy(c->d_rad, hr, sizeof(double) * n, hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMemcpy(c->d_mat, hm, sizeof(SphMat) * n, hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMemcpy(c->d_lights, hl, sizeof(LightD) * nl, hipMemcpyHostToDevice)) != hipSuccess) {
    rc = fail(c, e, "rt_upload_scene");
    free_scene(c);
  } else if ((c->nsph_up = n, rc = light_grids(c, s, scene_diam)) != RT_OK ||  // built on the device from d_geo /
             (c->sg_src.assign(s->spheres, s->spheres + n), c->sg_diam = scene_diam, c->scene_launches = 0,
              c->sg_pending = c->sg_mode < 0, rc = c->sg_mode > 0 ? sphere_grids(c) : RT_OK) != RT_OK) {  // d_rad
    free_scene(c);
  } else {
    c->nsph = n;
    c->nlight = nl;
    c->h_refl.clear();
    for (int i = 0; i < n; i++)
      if (s->spheres[i].reflectivity > 0.0)  // main.cpp:43
        c->h_refl.push_back(SchedSphere{s->spheres[i].center[0], s->spheres[i].center[1], s->spheres[i].center[2],
                                        s->spheres[i].radius});
    c->scene_gen++;
    for (int q = 0; q < 3; q++) c->amb[q] = s->ambient[q];
    c->has_scene = true;
    c->upload_ms = ms_since(t_upload);
  }
  delete[] hg;
  delete[] hr;
  delete[] hm;
  delete[] hl;
  return rc;
}

int rt_render_async(rt_ctx *c, const rt_camera *cam, int W, int H, int depth, const rt_rows *rows, uint8_t *out) {
  Rows r;
  int rc = validate(c, cam, W, H, depth, rows, out, r);
  if (rc != RT_OK) return rc;
  return enqueue(c, cam, W, H, depth, r, OutDesc{out, RT_FB_RGB8, 0, 0, W});
}

int rt_render_frames_async(rt_ctx *c, const rt_camera *cams, int nframes, int W, int H, int depth,
                           const rt_rows *rows, uint8_t *out, size_t frame_stride) {
  Rows r;
  int rc = validate(c, cams, W, H, depth, rows, out, r);
  if (rc != RT_OK) return rc;
  if (nframes < 1 || nframes > RT_MAX_FRAMES) return RT_ERR_INVALID_ARG;
  if (nframes > 1 && (frame_stride < (size_t)r.count * W * 3 || frame_stride > (size_t)1 << 62))
    return RT_ERR_INVALID_ARG;
  c->nframes = nframes;
  c->fcams = cams;
  rc = enqueue(c, cams, W, H, depth, r, OutDesc{out, RT_FB_RGB8, 0, 0, W, (long long)frame_stride});
  c->nframes = 1;
  c->fcams = nullptr;
  return rc;
}

int rt_render_stats(rt_ctx *c, rt_stats *st) {
  if (!c || !st) return RT_ERR_INVALID_ARG;
  RT_TRY(c, hipSetDevice(c->device));
  RT_TRY(c, hipStreamSynchronize(c->stream));
  float ms = 0.f;
  if (c->launches > 0) {
    const int slot = (int)((c->launches - 1) % rt_ctx::kRing);
    RT_TRY(c, hipEventElapsedTime(&ms, c->ev0[slot], c->ev1[slot]));
  }
  RT_TRY(c, hipMemcpy(c->h_counters, c->d_counters, kShards * kShardStride * sizeof(unsigned long long),
                      hipMemcpyDeviceToHost));
  unsigned long long sum[kCounters] = {};
  for (int sh = 0; sh < kShards; sh++)
    for (int q = 0; q < kCounters; q++) sum[q] += c->h_counters[sh * kShardStride + q];
  st->rays_primary = sum[0];
  st->rays_shadow = sum[1];
  st->rays_reflect = sum[2];
  st->negative_clamped = sum[3];
  st->tests_exact = sum[4];
  st->tests_cull = sum[5];
#ifdef RT_CHECK
  {
    // the first out-of-range device index of the launches since the last
    // read (rt_device.h RT_CK), then cleared for the next ones
    static const char *const kSiteNames[kCkSites] = {
        "?", "sphere index", "light-grid start", "light-grid list slot", "camera-grid start",
        "camera/sphere-grid list slot", "sphere-grid start", "sphere-grid key", "uniform-grid cell",
        "uniform-grid overflow slot", "BVH node reference", "BVH leaf slot", "tile order slot / tile id",
        "deferred-queue slot", "reflection-stack slot", "LDS ray-queue slot", "LDS pixel slot",
        "framebuffer offset", "camera-grid build slot", "stack-home pool exhausted"};
    CheckRec rec{};
    RT_TRY(c, hipMemcpyFromSymbol(&rec, HIP_SYMBOL(g_check), sizeof rec));
    if (rec.count) {
      const CheckRec zero{};
      RT_TRY(c, hipMemcpyToSymbol(HIP_SYMBOL(g_check), &zero, sizeof zero));
      c->err = std::string("RT_CHECK: ") + (rec.site < (unsigned long long)kCkSites ? kSiteNames[rec.site] : "?") +
               " index " + std::to_string((long long)rec.idx) + " outside [0, " + std::to_string(rec.bound) +
               ") (" + std::to_string(rec.count) + " violations)";
      return RT_ERR_CHECK;
    }
  }
#endif
#ifdef RT_STAMPS
  if (const char *tf = std::getenv("RT_HIP_STAMPS_FILE")) {
    static unsigned long long host_tl[kTimelineWaves * kTl];
    if (hipMemcpyFromSymbol(host_tl, HIP_SYMBOL(g_timeline), sizeof(host_tl)) == hipSuccess) {
      if (FILE *f = std::fopen(tf, "wb")) {
        std::fwrite(host_tl, sizeof(host_tl), 1, f);
        std::fclose(f);
      }
    }
  }
#endif
#ifdef RT_STAMPS
  if (std::getenv("RT_HIP_STAMPS")) {  // diagnostic builds (-DRT_STAMPS) fill slots 8..14
    unsigned long long d[12] = {};
    for (int sh = 0; sh < kShards; sh++)
      for (int q = 0; q < 12; q++) d[q] += c->h_counters[sh * kShardStride + 8 + q];
    const double nw = (double)(d[6] ? d[6] : 1);
    unsigned long long bvh = 0;
    for (int sh = 0; sh < kShards; sh++) bvh += c->h_counters[sh * kShardStride + 20];
    std::fprintf(stderr,
                 "RT_STAMPS per wave: candidate iterations %.1f (closest %.1f, of which primary %.1f), sweeps %.2f "
                 "(closest %.2f), bvh cycles %.0f\n",
                 d[7] / nw, d[9] / nw, d[11] / nw, d[8] / nw, d[10] / nw, bvh / nw);
    unsigned long long cl = 0, sh = 0;
    for (int s2 = 0; s2 < kShards; s2++) {
      cl += c->h_counters[s2 * kShardStride + 21];
      sh += c->h_counters[s2 * kShardStride + 22];
    }
    std::fprintf(stderr, "RT_STAMPS cycles/wave: closest hits %.0f, shadow queries %.0f\n", cl / nw, sh / nw);
    std::fprintf(stderr, "RT_STAMPS waves=%llu cycles/wave: bound %.0f cull %.0f cand %.0f setup %.0f shade %.0f total %.0f\n",
                 d[6], (double)d[0] / (d[6] ? d[6] : 1), (double)d[1] / (d[6] ? d[6] : 1),
                 (double)d[2] / (d[6] ? d[6] : 1), (double)d[3] / (d[6] ? d[6] : 1),
                 (double)d[4] / (d[6] ? d[6] : 1), (double)d[5] / (d[6] ? d[6] : 1));
  }
#endif
  st->kernel_ms = ms;
  return RT_OK;
}

int rt_render(rt_ctx *c, const rt_camera *cam, int W, int H, int depth, const rt_rows *rows, uint8_t *out,
              int out_on_device, rt_stats *st) {
  Rows r;
  int rc = validate(c, cam, W, H, depth, rows, out, r);
  if (rc != RT_OK) return rc;
  RT_TRY(c, hipSetDevice(c->device));
  size_t bytes = (size_t)r.count * W * 3;
  uint8_t *dst = out;
  if (!out_on_device) {
    if (c->tmp_bytes < bytes) {
      RT_TRY(c, hipStreamSynchronize(c->stream));
      if (c->d_tmp) (void)hipFree(c->d_tmp);
      c->d_tmp = nullptr;
      c->tmp_bytes = 0;
      RT_TRY(c, hipMalloc(&c->d_tmp, bytes ? bytes : 1));
      c->tmp_bytes = bytes;
    }
    dst = c->d_tmp;
  }
  rc = enqueue(c, cam, W, H, depth, r, OutDesc{dst, RT_FB_RGB8, 0, 0, W});
  if (rc != RT_OK) return rc;
  if (!out_on_device && bytes) RT_TRY(c, hipMemcpyAsync(out, dst, bytes, hipMemcpyDeviceToHost, c->stream));
  rt_stats tmp;
  rc = rt_render_stats(c, st ? st : &tmp);
  return rc;
}

int rt_set_antialias(rt_ctx *c, int samples) {
  if (!c || (samples != 1 && samples != 4)) return RT_ERR_INVALID_ARG;
  c->samples = samples;
  return RT_OK;
}

int rt_render_tile(rt_ctx *c, const rt_camera *cam, int W, int H, int depth, int tile_x, int tile_y, int tile_w,
                   int tile_h, int fb_format, void *fb_device) {
  if (!c || !cam || !fb_device || W <= 0 || H <= 0 || tile_w < 0 || tile_h < 0 || tile_x < 0 || tile_y < 0)
    return RT_ERR_INVALID_ARG;
  if (fb_format != RT_FB_RGB8 && fb_format != RT_FB_F32X3 && fb_format != RT_FB_F64X3) return RT_ERR_INVALID_ARG;
  if (!c->has_scene) return RT_ERR_NO_SCENE;
  if (depth > RT_MAX_DEPTH) return RT_ERR_DEPTH;
  // the reference kernel clips the tile to the image (kernel.cu:103)
  const int xe = (int)std::min<long long>(W, (long long)tile_x + tile_w);  // 64-bit: no overflow near INT_MAX
  const int ye = (int)std::min<long long>(H, (long long)tile_y + tile_h);
  const int xw = std::max(0, xe - tile_x), th = std::max(0, ye - tile_y);
  // framebuffer rows j = tile_y .. ye-1 (j = 0 the bottom row) are PPM rows H-ye .. H-1-tile_y
  const Rows r{1, H - ye, 1, xw > 0 ? th : 0};
  RT_TRY(c, hipSetDevice(c->device));
  return enqueue(c, cam, W, H, depth, r, OutDesc{fb_device, fb_format, 1, tile_x, xw});
}

int rt_render_tiles(rt_ctx *c, const rt_camera *cam, int W, int H, int depth, const rt_tile *tiles, int ntiles,
                    int fb_format, void *fb_device) {
  if (!c || !cam || !fb_device || W <= 0 || H <= 0 || ntiles < 0 || (ntiles > 0 && !tiles)) return RT_ERR_INVALID_ARG;
  if (fb_format != RT_FB_RGB8 && fb_format != RT_FB_F32X3 && fb_format != RT_FB_F64X3) return RT_ERR_INVALID_ARG;
  for (int i = 0; i < ntiles; i++)
    if (tiles[i].x < 0 || tiles[i].y < 0 || tiles[i].width < 0 || tiles[i].height < 0) return RT_ERR_INVALID_ARG;
  if (!c->has_scene) return RT_ERR_NO_SCENE;
  if (depth > RT_MAX_DEPTH) return RT_ERR_DEPTH;
  RT_TRY(c, hipSetDevice(c->device));
  c->req_tiles = tiles;
  c->req_n = ntiles;
  const int rc = enqueue(c, cam, W, H, depth, Rows{1, 0, 1, H}, OutDesc{fb_device, fb_format, 1, 0, W});
  c->req_tiles = nullptr;
  c->req_n = 0;
  return rc;
}

int rt_kernel_times(rt_ctx *c, double *ms_out, int max_n, int *n_out) {
  if (!c || !n_out || max_n < 0 || (max_n > 0 && !ms_out)) return RT_ERR_INVALID_ARG;
  RT_TRY(c, hipSetDevice(c->device));
  RT_TRY(c, hipStreamSynchronize(c->stream));
  long long avail = c->launches - c->hist_begin;
  if (avail > rt_ctx::kRing) avail = rt_ctx::kRing;
  if (avail > max_n) avail = max_n;
  for (long long i = 0; i < avail; i++) {
    const int slot = (int)((c->launches - avail + i) % rt_ctx::kRing);
    float ms = 0.f;
    RT_TRY(c, hipEventElapsedTime(&ms, c->ev0[slot], c->ev1[slot]));
    ms_out[i] = ms;
  }
  *n_out = (int)avail;
  c->hist_begin = c->launches;
  return RT_OK;
}

int rt_get_info(rt_ctx *c, rt_info *out) {
  if (!c || !out) return RT_ERR_INVALID_ARG;
  *out = rt_info{};
  out->cam_grid_last = c->cg_last ? 1 : 0;
  out->cam_grid_n = c->cg_last_n;
  out->cam_grid_builds = c->cg_builds;
  out->cam_grid_build_ms = c->cg_build_ms;
  out->tile_order_builds = c->perm_builds;
  out->tile_order_build_ms = c->perm_build_ms;
  out->upload_ms = c->upload_ms;
  out->launches = (uint64_t)c->launches;
  out->sphere_grids = c->sg_ok ? c->sg_grids : 0;
  out->sphere_grid_n = c->sg_ok ? c->sg_n : 0;
  out->sphere_grid_entries = c->sg_ok ? (uint64_t)c->sg_entries : 0;
  out->sphere_grid_build_ms = c->sg_build_ms;
  out->behind_grid = c->ug_ok ? 1 : 0;
  out->behind_grid_last = c->ug_last ? 1 : 0;
  out->behind_grid_cells = c->ug_ok ? (uint64_t)c->ug.nx * (uint64_t)c->ug.ny * (uint64_t)c->ug.nz : 0;
  out->behind_grid_entries = c->ug_ok ? (uint64_t)c->ug_entries : 0;
  out->behind_grid_build_ms = c->ug_build_ms;
  out->bvh_build_ms = c->bvh_build_ms;
  out->light_grid_build_ms = c->lg_build_ms;
  out->scratch_bytes = (uint64_t)(c->cstack_bytes + c->dq_bytes + c->homes_bytes +
                                  (size_t)c->home_words * sizeof(unsigned long long) + c->cg_count_cap + c->cg_ent_cap +
                                  c->cg_disks_cap + c->cg_pairs_cap + c->cg_npairs_cap + c->perm_cap);
  out->shadow_line_bounded = c->lg_off_free ? 1 : 0;
  out->reserved0 = 0;
  return RT_OK;
}

int rt_unpermute_rows(rt_ctx *c, const uint8_t *gathered, uint8_t *image, int W, int H, int band, int G, int R) {
  if (!c || !gathered || !image || W <= 0 || H <= 0 || band < 1 || G < 1 || R < 0) return RT_ERR_INVALID_ARG;
  const long long bands = (H + band - 1) / band;
  if ((long long)((bands + G - 1) / G) * band > R) return RT_ERR_INVALID_ARG;
  RT_TRY(c, hipSetDevice(c->device));
  hipLaunchKernelGGL(unpermute_kernel, dim3(H), dim3(kBlock), 0, c->stream, gathered, image, W, H, band, G, R);
  RT_TRY(c, hipGetLastError());
  return RT_OK;
}

}  // extern "C"
