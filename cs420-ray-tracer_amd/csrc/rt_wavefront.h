// rt_wavefront.h -- the wavefront (queue) render pipeline, included by rt_kernel.hip.
//
// The per-pixel recursion of trace_ray (src/main.cpp:16-58) is split into
// level-synchronous passes over compacted queues, so every kernel keeps little
// live state (high occupancy hides the fp64 dependency chains) and no lane
// idles on sky pixels or on sparse reflection levels:
//
//   wf_primary      one lane per pixel: camera ray (camera.h:17-25), closest hit
//                   (scene.h:41-61); misses write the sky colour, hits are
//                   appended to the hit queue (wave-aggregated atomics).
//   wf_shade(L)     one lane per hit of level L (persistent grid-stride loop):
//                   Phong + per-light shadow sweeps (scene.h:65-121); a
//                   reflective hit pushes (shade*(1-refl), refl) on the pixel's
//                   stack and appends the reflection ray (main.cpp:43-55).
//   wf_reflect(L)   one lane per reflection ray of level L: closest hit, sky on
//                   a miss, hit records for wf_shade(L).
//   wf_resolve      one lane per pixel: unwinds the stack innermost-first
//                   (shade*(1-refl) + reflected*refl, bit-identical to the
//                   recursion) and quantises (main.cpp:85-87) into RGB8.
//
// Queues are split into kShards segments, each with its own append counter:
// a producer workgroup appends to segment (workgroup id % kShards), and the
// consumer workgroups of segment s are exactly those with id % kShards == s
// (grid-stride inside the segment).  One contended word serialises device
// atomics (~88/us); 64 words in separate lines do not.  Capacity: segment s of
// the primary hit queue receives at most ceil(WGs/kShards) * 256 hits, and each
// later pass maps segment s to segment s with at most one output per input, so
// every queue segment needs the same `seg_cap` entries.  Segment order follows
// the producing waves (runs of up to 64 hits from one 8x8 tile), so consumer
// waves stay spatially coherent and the per-wave cull stays tight.
#pragma once
#include "rt_device.h"

namespace rtk {

struct __attribute__((aligned(16))) RayRec {  // 64 B
  double ox, oy, oz, dx, dy, dz;
  int pix, dleft;
  int key, pad;  // key: sphere the ray leaves
};
struct __attribute__((aligned(16))) HitRec {  // 80 B
  double ox, oy, oz, dx, dy, dz, t;
  int pix, sph, dleft, pad;
  double pad2;
};
struct StackEnt {  // 32 B: A = shade*(1-refl), and refl
  double ax, ay, az, refl;
};
struct Term {  // terminal colour of a pixel's chain
  double r, g, b;
};

// Wave-aggregated append: returns this lane's slot (valid where `want`).
__device__ __forceinline__ unsigned wave_append(bool want, unsigned *counter) {
  const unsigned long long m = __ballot(want);
  unsigned base = 0;
  if ((threadIdx.x & 63) == 0 && m) base = atomicAdd(counter, (unsigned)__popcll(m));
  base = __shfl(base, 0, 64);
  const unsigned below = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
  return base + below;
}

struct WfArgs {
  const SphGeo *geo;
  const double *rad;
  const SphMat *mat;
  const LightD *lights;
  int n, nl;
  D3 amb;
  Cam cam;
  int W, H, depth;
  Rows rows;
  int npx;            // rows.count * W
  int seg_cap;        // entries per queue segment
  HitRec *hitq;       // [kShards][seg_cap]
  RayRec *rayq;       // [kShards][seg_cap]
  unsigned *hit_cnt;  // [depth+1][kShards]
  unsigned *ray_cnt;  // [depth+1][kShards]
  Term *term;
  uint8_t *nlev;
  StackEnt *stack;    // [(depth-1) * npx]
  uint8_t *out;
  unsigned long long *counters;
  BvhArgs bv;
  LgArgs lg;
};

// Stage sphere geometry/radii (if they fit) and lights into LDS.
template <bool kLdsGeo>
__device__ __forceinline__ void stage(const WfArgs &a, unsigned char *smem, const SphGeo *&g, const double *&rad,
                                      const LightD *&lights, BvhArgs &bv) {
  bv = a.bv;
  const SphMat *sm;  // the queue kernels read materials from a.mat
  stage_scene<kLdsGeo>(smem, a.geo, a.rad, a.mat, a.lights, a.n, a.nl, bv, g, rad, sm, lights);
}

__device__ __forceinline__ void flush_work(const Work &w, unsigned long long *counters) {
  if ((threadIdx.x & 63) == 0) {
    unsigned long long *sc = counter_shard(counters);
    if (w.exact) atomicAdd(&sc[4], w.exact);
    if (w.cull) atomicAdd(&sc[5], w.cull);
  }
}

__device__ __forceinline__ D3 sky(D3 d) {  // main.cpp:26-30
  const double st = 0.5 * (d.y + 1.0);
  return add(scale(mk(1.0, 1.0, 1.0), 1.0 - st), scale(mk(0.5, 0.7, 1.0), st));
}

// ---- pass 1: camera rays (one lane per pixel, 8x8 tile per wave) -----------
template <bool kLdsGeo, bool kCull>
__global__ __launch_bounds__(256) void wf_primary(WfArgs a) {
  extern __shared__ __attribute__((aligned(32))) unsigned char smem[];
  const SphGeo *g;
  const double *rad;
  const LightD *lights;
  BvhArgs bv;
  stage<kLdsGeo>(a, smem, g, rad, lights, bv);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
  const int k = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
  const long long y = (long long)(k / a.rows.band) * a.rows.band * a.rows.stride +
                      (long long)a.rows.first * a.rows.band + (k % a.rows.band);
  const bool in_img = x < a.W && k < a.rows.count && y < a.H;
  const int pix = k * a.W + x;
  // camera.h:17-25 and main.cpp:151-154: u = i/(W-1), v = j/(H-1), ((u-0.5)*scale)*aspect
  const int j = a.H - 1 - (int)(in_img ? y : 0);
  const double u = (double)x / (a.W - 1), v = (double)j / (a.H - 1);
  const double su = ((u - 0.5) * a.cam.scale) * 1.0, sv = (v - 0.5) * a.cam.scale;
  const D3 dir = add(add(mk(a.cam.fx, a.cam.fy, a.cam.fz), scale(mk(a.cam.rx, a.cam.ry, a.cam.rz), su)),
                     scale(mk(a.cam.ux, a.cam.uy, a.cam.uz), sv));
  const D3 d = normalized(normalized(dir));  // get_ray normalises, Ray() normalises again
  const D3 o = mk(a.cam.px, a.cam.py, a.cam.pz);
  const bool alive = in_img && a.depth >= 1;
  Work work;
  double bt;
  const int bi = sweep_closest<kCull>(g, rad, a.n, alive, o, d, -1, bv, bt, work);
  const bool hit = alive && bi >= 0;
  if (in_img && !hit) {
    const D3 c = alive ? sky(d) : mk(0.0, 0.0, 0.0);  // depth <= 0 is black (main.cpp:17-18)
    a.term[pix] = Term{c.x, c.y, c.z};
    a.nlev[pix] = 0;
  }
  const unsigned shard = (blockIdx.x + blockIdx.y * gridDim.x) % kShards;
  const unsigned slot = wave_append(hit, &a.hit_cnt[shard]);
  if (hit) {
    HitRec h;
    h.ox = o.x; h.oy = o.y; h.oz = o.z;
    h.dx = d.x; h.dy = d.y; h.dz = d.z;
    h.t = bt;
    h.pix = pix;
    h.sph = bi;
    h.dleft = a.depth;
    h.pad = 0;
    h.pad2 = 0;
    a.hitq[(size_t)shard * a.seg_cap + slot] = h;
  }
  const unsigned np = (unsigned)__popcll(__ballot(alive));
  if (lane == 0 && np) atomicAdd(&counter_shard(a.counters)[0], (unsigned long long)np);
  flush_work(work, a.counters);
}

// ---- hybrid pass 0: camera rays + their whole first level, per 8x8 tile -----
// The coherent part of the frame stays in one kernel (one wave per 8x8 tile,
// like the megakernel); reflection rays leave through the level-1 queue, so
// the incoherent levels are spread over many waves by wf_reflect / wf_shade.
template <bool kLdsGeo, bool kCull>
__global__ __launch_bounds__(64) void wf_level0(WfArgs a) {
  extern __shared__ __attribute__((aligned(32))) unsigned char smem[];
  const SphGeo *g;
  const double *rad;
  const LightD *lights;
  BvhArgs bv;
  stage<kLdsGeo>(a, smem, g, rad, lights, bv);
  const int lane = threadIdx.x & 63;
  const int x = blockIdx.x * 8 + (lane & 7);
  const int k = blockIdx.y * 8 + (lane >> 3);
  const long long y = (long long)(k / a.rows.band) * a.rows.band * a.rows.stride +
                      (long long)a.rows.first * a.rows.band + (k % a.rows.band);
  const bool in_img = x < a.W && k < a.rows.count && y < a.H;
  const int pix = k * a.W + x;
  const int j = a.H - 1 - (int)(in_img ? y : 0);  // camera.h:17-25, main.cpp:151-154
  const double u = (double)x / (a.W - 1), v = (double)j / (a.H - 1);
  const double su = ((u - 0.5) * a.cam.scale) * 1.0, sv = (v - 0.5) * a.cam.scale;
  const D3 dir = add(add(mk(a.cam.fx, a.cam.fy, a.cam.fz), scale(mk(a.cam.rx, a.cam.ry, a.cam.rz), su)),
                     scale(mk(a.cam.ux, a.cam.uy, a.cam.uz), sv));
  const D3 d = normalized(normalized(dir));
  const D3 o = mk(a.cam.px, a.cam.py, a.cam.pz);
  const bool alive = in_img && a.depth >= 1;
  Work work;
  double bt;
  const int bi = sweep_closest<kCull>(g, rad, a.n, alive, o, d, -1, bv, bt, work);
  const bool hit = alive && bi >= 0;
  if (in_img && !hit) {
    const D3 c = alive ? sky(d) : mk(0.0, 0.0, 0.0);  // depth <= 0 is black (main.cpp:17-18)
    a.term[pix] = Term{c.x, c.y, c.z};
    a.nlev[pix] = 0;
  }
  const int hi = hit ? bi : 0;
  const D3 hp = add(o, scale(d, bt));  // main.cpp:32
  D3 col;
  {
    const SphMat m0 = a.mat[hi];
    col = mul(a.amb, mk(m0.cr, m0.cg, m0.cb));  // scene.h:91
  }
  // scene.h:94-120 in two phases per block of 64 lights (see render_kernel)
  for (int l0 = 0; l0 < a.nl; l0 += 64) {
    const int lend = a.nl - l0 < 64 ? a.nl : l0 + 64;
    unsigned long long occm = 0;
    for (int l = l0; l < lend; ++l) {
      const LightD L = lights[l];
      const D3 lp = mk(L.px, L.py, L.pz);
      const D3 to_light = sub(lp, hp);
      const double dist = length(to_light);
      const D3 ldir = normalized(to_light);
      const D3 so = add(hp, scale(ldir, kEps)), sd = normalized(ldir);
      const LgRange cr = a.lg.on ? lg_range(a.lg, l, hp, lp, hit) : LgRange{0, 0};
      const bool occ = a.lg.on ? shadow_cells(g, a.n, hit, so, sd, lp, dist, a.lg, l, cr, lg_first(a.lg, cr), work)
                               : sweep_shadow<kCull>(g, rad, a.n, hit, so, sd, lp, hi, dist, bv, work);
      if (occ) occm |= 1ull << (l - l0);
    }
    if (hit && occm != ~0ull >> (64 - (lend - l0))) {
      const SphGeo sg = g[hi];
      const SphMat m = a.mat[hi];
      const D3 nrm = normalized(sub(hp, mk(sg.cx, sg.cy, sg.cz)));  // sphere.h:62-64
      const D3 view = normalized(sub(o, hp));                       // main.cpp:38
      const D3 mc = mk(m.cr, m.cg, m.cb);
      for (int l = l0; l < lend; ++l) {
        if (occm >> (l - l0) & 1ull) continue;
        const LightD L = lights[l];
        const D3 ldir = normalized(sub(mk(L.px, L.py, L.pz), hp));
        const double ndl = max0(dot(nrm, ldir));
        const D3 diffuse = scale(scale(mc, 1.0 - m.refl), ndl);
        const D3 nl2 = scale(ldir, -1.0);
        const D3 rdir = sub(nl2, scale(scale(nrm, 2.0), dot(nl2, nrm)));  // reflect(), vec3.h:31-33
        const double rdv = max0(dot(rdir, view));
        const double spec = (rdv == 0.0 && m.shin > 0.0) ? 0.0 : pow_call(rdv, m.shin);
        const D3 specular = scale(scale(mk(L.cr, L.cg, L.cb), kSpec), spec);
        col = add(add(specular, diffuse), col);  // scene.h:117
      }
    }
  }
  bool spawn = false;
  D3 ro = mk(0.0, 0.0, 0.0), rd = ro;
  if (hit) {
    const SphMat m = a.mat[hi];
    if (m.refl > 0.0) {  // main.cpp:43-55
      const double w = 1.0 - m.refl;
      const D3 A = mk(col.x * w, col.y * w, col.z * w);
      if (a.depth - 1 >= 1) {
        a.stack[pix] = StackEnt{A.x, A.y, A.z, m.refl};  // level 0
        const SphGeo sg = g[hi];
        const D3 nrm = normalized(sub(hp, mk(sg.cx, sg.cy, sg.cz)));
        rd = normalized(sub(d, scale(scale(nrm, 2.0), dot(d, nrm))));
        ro = add(hp, scale(nrm, kEps));
        spawn = true;
      } else {
        a.term[pix] = Term{A.x, A.y, A.z};
        a.nlev[pix] = 0;
      }
    } else {
      a.term[pix] = Term{col.x, col.y, col.z};
      a.nlev[pix] = 0;
    }
  }
  const unsigned shard = (blockIdx.x + blockIdx.y * gridDim.x) % kShards;
  const unsigned slot = wave_append(spawn, &a.ray_cnt[1 * kShards + shard]);
  if (spawn) a.rayq[(size_t)shard * a.seg_cap + slot] = RayRec{ro.x, ro.y, ro.z, rd.x, rd.y, rd.z, pix, a.depth - 1, hi, 0};
  const unsigned np = (unsigned)__popcll(__ballot(alive));
  const unsigned nh = (unsigned)__popcll(__ballot(hit));
  const unsigned ns = (unsigned)__popcll(__ballot(spawn));
  if (lane == 0) {
    unsigned long long *sc = counter_shard(a.counters);
    if (np) atomicAdd(&sc[0], (unsigned long long)np);
    if (nh) atomicAdd(&sc[1], (unsigned long long)nh * (unsigned)a.nl);
    if (ns) atomicAdd(&sc[2], (unsigned long long)ns);
  }
  flush_work(work, a.counters);
}

// ---- pass 2 (per level): shading + shadow rays, spawns reflection rays -------
template <bool kLdsGeo, bool kCull>
__global__ __launch_bounds__(256) void wf_shade(WfArgs a, int level) {
  const unsigned shard = blockIdx.x % kShards, j = blockIdx.x / kShards, nj = gridDim.x / kShards;
  const unsigned cnt = a.hit_cnt[level * kShards + shard];
  if (j * 256u >= cnt) return;  // uniform: nothing for this workgroup
  const HitRec *__restrict__ hq = a.hitq + (size_t)shard * a.seg_cap;
  extern __shared__ __attribute__((aligned(32))) unsigned char smem[];
  const SphGeo *g;
  const double *rad;
  const LightD *lights;
  BvhArgs bv;
  stage<kLdsGeo>(a, smem, g, rad, lights, bv);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  Work work;
  unsigned long long n_shadow = 0, n_reflect = 0;
  const unsigned stride = nj * 256u;
  for (unsigned base = j * 256u + wave * 64u; base < cnt; base += stride) {
    const unsigned idx = base + lane;
    const bool hit = idx < cnt;
    const HitRec h = hq[hit ? idx : base];
    const D3 o = mk(h.ox, h.oy, h.oz), d = mk(h.dx, h.dy, h.dz);
    const SphGeo sg = g[h.sph];
    const SphMat m = a.mat[h.sph];
    const D3 hp = add(o, scale(d, h.t));                          // main.cpp:32
    const D3 nrm = normalized(sub(hp, mk(sg.cx, sg.cy, sg.cz)));  // sphere.h:62-64
    const D3 view = normalized(sub(o, hp));                       // main.cpp:38
    const D3 mc = mk(m.cr, m.cg, m.cb);
    D3 col = mul(a.amb, mc);                                      // scene.h:91
    for (int l = 0; l < a.nl; ++l) {                              // scene.h:94-120
      const LightD L = lights[l];
      const D3 lp = mk(L.px, L.py, L.pz);
      const D3 to_light = sub(lp, hp);
      const double dist = length(to_light);
      const D3 ldir = normalized(to_light);
      const D3 so = add(hp, scale(ldir, kEps)), sd = normalized(ldir);
      const LgRange cr = a.lg.on ? lg_range(a.lg, l, hp, lp, hit) : LgRange{0, 0};
      const bool occ = a.lg.on ? shadow_cells(g, a.n, hit, so, sd, lp, dist, a.lg, l, cr, lg_first(a.lg, cr), work)
                               : sweep_shadow<kCull>(g, rad, a.n, hit, so, sd, lp, h.sph, dist, bv, work);
      if (hit && !occ) {
        const double ndl = max0(dot(nrm, ldir));
        const D3 diffuse = scale(scale(mc, 1.0 - m.refl), ndl);
        const D3 nl2 = scale(ldir, -1.0);
        const D3 rdir = sub(nl2, scale(scale(nrm, 2.0), dot(nl2, nrm)));  // reflect(), vec3.h:31-33
        const double rdv = max0(dot(rdir, view));
        // pow(+0, y > 0) is +0 exactly (C99 F.10.4.4), so most lanes skip ocml's pow.
        const double spec = (rdv == 0.0 && m.shin > 0.0) ? 0.0 : pow(rdv, m.shin);
        const D3 specular = scale(scale(mk(L.cr, L.cg, L.cb), kSpec), spec);
        col = add(add(specular, diffuse), col);                   // scene.h:117
      }
    }
    n_shadow += (unsigned long long)__popcll(__ballot(hit)) * (unsigned)a.nl;
    bool spawn = false;
    D3 ro = mk(0.0, 0.0, 0.0), rd = ro;
    if (hit) {
      if (m.refl > 0.0) {                                         // main.cpp:43-55
        const double w = 1.0 - m.refl;
        const D3 A = mk(col.x * w, col.y * w, col.z * w);
        if (h.dleft - 1 >= 1) {
          a.stack[(size_t)level * a.npx + h.pix] = StackEnt{A.x, A.y, A.z, m.refl};
          rd = normalized(sub(d, scale(scale(nrm, 2.0), dot(d, nrm))));
          ro = add(hp, scale(nrm, kEps));
          spawn = true;
        } else {
          a.term[h.pix] = Term{A.x, A.y, A.z};  // trace_ray(depth 0) is black: A + 0*refl == A
          a.nlev[h.pix] = (uint8_t)level;
        }
      } else {
        a.term[h.pix] = Term{col.x, col.y, col.z};
        a.nlev[h.pix] = (uint8_t)level;
      }
    }
    const unsigned slot = wave_append(spawn, &a.ray_cnt[(level + 1) * kShards + shard]);
    if (spawn)
      a.rayq[(size_t)shard * a.seg_cap + slot] = RayRec{ro.x, ro.y, ro.z, rd.x, rd.y, rd.z, h.pix, h.dleft - 1, h.sph, 0};
    n_reflect += (unsigned long long)__popcll(__ballot(spawn));
  }
  if (lane == 0) {
    if (n_shadow) atomicAdd(&counter_shard(a.counters)[1], n_shadow);
    if (n_reflect) atomicAdd(&counter_shard(a.counters)[2], n_reflect);
  }
  flush_work(work, a.counters);
}

// ---- pass 3 (per level >= 1): reflection rays -> hits ------------------------
template <bool kLdsGeo, bool kCull>
__global__ __launch_bounds__(256) void wf_reflect(WfArgs a, int level) {
  const unsigned shard = blockIdx.x % kShards, j = blockIdx.x / kShards, nj = gridDim.x / kShards;
  const unsigned cnt = a.ray_cnt[level * kShards + shard];
  if (j * 256u >= cnt) return;
  const RayRec *__restrict__ rq = a.rayq + (size_t)shard * a.seg_cap;
  extern __shared__ __attribute__((aligned(32))) unsigned char smem[];
  const SphGeo *g;
  const double *rad;
  const LightD *lights;
  BvhArgs bv;
  stage<kLdsGeo>(a, smem, g, rad, lights, bv);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  Work work;
  const unsigned stride = nj * 256u;
  for (unsigned base = j * 256u + wave * 64u; base < cnt; base += stride) {
    const unsigned idx = base + lane;
    const bool alive = idx < cnt;
    const RayRec r = rq[alive ? idx : base];
    const D3 o = mk(r.ox, r.oy, r.oz), d = mk(r.dx, r.dy, r.dz);
    double bt;
    const int bi = sweep_closest<kCull>(g, rad, a.n, alive, o, d, r.key, bv, bt, work);
    const bool hit = alive && bi >= 0;
    if (alive && !hit) {
      const D3 c = sky(d);
      a.term[r.pix] = Term{c.x, c.y, c.z};
      a.nlev[r.pix] = (uint8_t)level;
    }
    const unsigned slot = wave_append(hit, &a.hit_cnt[level * kShards + shard]);
    if (hit) {
      HitRec h;
      h.ox = o.x; h.oy = o.y; h.oz = o.z;
      h.dx = d.x; h.dy = d.y; h.dz = d.z;
      h.t = bt;
      h.pix = r.pix;
      h.sph = bi;
      h.dleft = r.dleft;
      h.pad = 0;
      h.pad2 = 0;
      a.hitq[(size_t)shard * a.seg_cap + slot] = h;
    }
  }
  flush_work(work, a.counters);
}

// ---- pass 4: unwind + quantise into RGB8 (one lane per output pixel) ---------
__global__ __launch_bounds__(256) void wf_resolve(WfArgs a) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int k = blockIdx.y * 4 + (threadIdx.x >> 6);
  unsigned neg = 0;
  if (x < a.W && k < a.rows.count) {
    const long long y = (long long)(k / a.rows.band) * a.rows.band * a.rows.stride +
                        (long long)a.rows.first * a.rows.band + (k % a.rows.band);
    uint8_t *px = a.out + ((size_t)k * a.W + x) * 3;
    if (y < a.H) {
      const int pix = k * a.W + x;
      const Term t = a.term[pix];
      D3 res = mk(t.r, t.g, t.b);
      for (int lev = (int)a.nlev[pix] - 1; lev >= 0; --lev) {  // innermost first
        const StackEnt e = a.stack[(size_t)lev * a.npx + pix];
        res = mk(e.ax + res.x * e.refl, e.ay + res.y * e.refl, e.az + res.z * e.refl);
      }
      const int q0 = quantize(res.x), q1 = quantize(res.y), q2 = quantize(res.z);
      neg = (q0 < 0) + (q1 < 0) + (q2 < 0);
      px[0] = (uint8_t)(q0 < 0 ? 0 : q0);
      px[1] = (uint8_t)(q1 < 0 ? 0 : q1);
      px[2] = (uint8_t)(q2 < 0 ? 0 : q2);
    } else {
      px[0] = px[1] = px[2] = 0;
    }
  }
  const unsigned long long sn = wave_sum(neg);
  if ((threadIdx.x & 63) == 0 && sn) atomicAdd(&counter_shard(a.counters)[3], sn);
}

}  // namespace rtk
