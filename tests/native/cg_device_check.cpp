// Check of the camera grids' device builder (rt_kernel.hip cg_disk_kernel /
// cg_bin_kernel / cg_sort_kernel) on the CPU: the kernels' per-lane functions
// (csrc/rt_cgbuild.h, shared with the kernels) run lane by lane in the
// kernels' pass structure -- pass 1 a wave per (grid, sphere) appending
// (disk, block) pairs to its grid's list, pass 2 a wave per quarter pair
// (tiles, then cells of up to 4 tiles a round, slots counted per cell), pass 3
// the (tlo, index) sort -- for 1-3 camera positions per scene (one grid per
// position, as a moving-camera launch builds them).  Checked per grid:
//   * every cell that did not overflow its K = 48 slots lists exactly the
//     host builder's entries (build_point_grid, the same N and point), in
//     ascending (tlo, index) order;
//   * for random camera rays (uniform, and aimed at sphere silhouettes ahead
//     of and behind the camera), every sphere the reference's test reports a
//     hit for (either sign of t) is on the looked-up cell's list with
//     tlo <= t, and the scan of rt_device.h cam_closest (stop at the first
//     tlo > best t) returns find_intersection's (t, index); a ray whose cell
//     overflowed sweeps (not checked here).
// Prints "checked <rays> <hit pairs> cells <cells> overflow <cells> differ <n>
// missed <n> wrong <n>".
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <set>
#include <utility>
#include <vector>

#include "rt_cgbuild.h"

namespace {
struct V {
  double x, y, z;
};
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V add(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V scl(V a, double s) { return {a.x * s, a.y * s, a.z * s}; }
double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V nrm(V a) {
  const double l = std::sqrt(dot(a, a));
  return {a.x / l, a.y / l, a.z / l};
}
bool hit(V c, double r, V o, V d, double &t) {  // sphere.h:26-59
  V oc = sub(o, c);
  double a = dot(d, d), b = 2.0 * dot(oc, d), cc = dot(oc, oc) - r * r;
  double disc = b * b - 4 * a * cc;
  if (disc < 0) return false;
  if (disc == 0) {
    t = -b / (2 * a);
    return true;
  }
  double t1 = (-b - std::sqrt(disc)) / (2 * a), t2 = (-b + std::sqrt(disc)) / (2 * a);
  if (std::fmax(t1, t2) < 0) return false;
  t = std::fmin(t1, t2);
  if (t < 0) t = std::fmax(t1, t2);
  return true;
}
int popc(unsigned long long m) { return __builtin_popcountll(m); }

constexpr int K = 48;  // rt_device.h kCgSlots
struct Ent {
  int s;
  float tlo;
};
// The device builder's passes for ngrid points, as the kernels run them.
struct DevGrids {
  int N, ngrid;
  std::vector<int> count;  // [grid][cell]
  std::vector<Ent> ent;    // [grid][cell][K]
};
DevGrids build_device(const std::vector<double> &cx, const std::vector<double> &cy, const std::vector<double> &cz,
                      const std::vector<double> &r, const std::vector<V> &pts, const std::vector<double> &diam, int N) {
  const int n = (int)cx.size(), ngrid = (int)pts.size();
  std::vector<rtk::CubePatch> faces, blocks, tiles;
  std::vector<double> cell;
  int NT = 0, NB = 0;
  rtk::cube_tables(N, faces, blocks, tiles, cell, NT, NB);
  const int nb = 6 * NB * NB;
  const long long cells = 6LL * N * N;
  DevGrids g{N, ngrid, std::vector<int>(ngrid * cells, 0), std::vector<Ent>(ngrid * cells * K)};
  // pass 1
  std::vector<rtk::CgDisk> disks(2 * (size_t)n * ngrid);
  std::vector<std::vector<std::pair<int, int>>> pairs(ngrid);
  for (int t = 0; t < n * ngrid; t++) {
    const int grid = t / n, s = t - grid * n;
    const rtk::CgView v =
        rtk::cg_view(cx[s], cy[s], cz[s], std::fabs(r[s]), pts[grid].x, pts[grid].y, pts[grid].z, diam[grid]);
    for (int side = 0; side < (v.global ? 1 : 2); ++side) {
      const rtk::CgDisk k = rtk::cg_side(v, side, s);
      const int di = 2 * t + side;
      disks[di] = k;
      for (int b0 = 0; b0 < nb; b0 += 64)
        for (int lane = 0; lane < 64; lane++) {
          const int b = b0 + lane;
          if (b < nb && rtk::cg_block(k, faces.data(), blocks.data(), NB, b)) pairs[grid].push_back({di, b});
        }
    }
  }
  // pass 2 (quarter items: tiles of rows 2q, 2q + 1 of the block)
  for (int grid = 0; grid < ngrid; grid++)
    for (const auto &pr : pairs[grid])
      for (int q = 0; q < 4; q++) {
        const rtk::CgDisk &k = disks[pr.first];
        const bool wide = rtk::cg_wide(k);
        const int bb = pr.second;
        const int f = bb / (NB * NB), bj = (bb / NB) % NB, bi = bb % NB;
        unsigned long long tmask = 0, imask = 0;
        for (int lane = 0; lane < 64; lane++) {
          bool tm, inside;
          rtk::cg_tile(k, tiles.data(), NT, f, bi, bj, lane, tm, inside);
          if (tm) tmask |= 1ull << lane;
          if (inside) imask |= 1ull << lane;
        }
        tmask &= 0xffffull << (16 * q);
        while (tmask) {
          for (int u = 0; u < 4 && tmask; ++u) {
            const int tl = __builtin_ctzll(tmask);
            tmask &= tmask - 1;
            for (int lane = 0; lane < 64; lane++) {
              const int gc = rtk::cg_cell(k, wide, cell.data(), N, f, bi, bj, tl, lane, (imask >> tl) & 1ull);
              if (gc < 0) continue;
              const long long c = (long long)grid * cells + gc;
              const int slot = g.count[c]++;
              if (slot < K) g.ent[c * K + slot] = Ent{k.s, k.tlo};
            }
          }
        }
      }
  // pass 3
  for (long long c = 0; c < (long long)ngrid * cells; c++) {
    const int cnt = g.count[c];
    if (cnt > K) continue;
    Ent *e = &g.ent[c * K];
    for (int k = 1; k < cnt; ++k) {
      const Ent x = e[k];
      int m = k - 1;
      while (m >= 0 && rtk::cg_before(x.tlo, x.s, e[m].tlo, e[m].s)) {
        e[m + 1] = e[m];
        --m;
      }
      e[m + 1] = x;
    }
  }
  return g;
}
}  // namespace

int main(int argc, char **argv) {
  const int seeds = argc > 1 ? std::atoi(argv[1]) : 20;
  long rays = 0, npairs = 0, ncells = 0, overflow = 0, differ = 0, missed = 0, wrong = 0;
  for (int seed = 0; seed < seeds; seed++) {
    std::mt19937_64 rng(5000 + seed);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    const double scale = std::pow(10.0, (int)(rng() % 5) - 1);  // 0.1 .. 1000
    const double shift = (rng() % 3 == 0) ? 1e5 * scale : 0.0;
    const int n = 20 + (int)(rng() % 200);
    const int N = (int[]){1, 3, 16, 64, 128, 256}[rng() % 6];
    std::vector<double> cx(n), cy(n), cz(n), r(n);
    for (int i = 0; i < n; i++) {
      cx[i] = shift + scale * 10 * U(rng);
      cy[i] = shift + scale * 10 * U(rng);
      cz[i] = shift + scale * 10 * U(rng);
      const int kind = (int)(rng() % 10);
      r[i] = scale * (kind == 0 ? 1e-4 : kind == 1 ? 5.0 : 0.05 + 1.5 * std::fabs(U(rng)));
      if (kind == 2) r[i] = -r[i];  // the parser accepts negative radii
    }
    // 1-3 camera points: free, inside a sphere, or just off a sphere's surface
    const int ngrid = 1 + (int)(rng() % 3);
    std::vector<V> pts;
    std::vector<double> diam;
    for (int gi = 0; gi < ngrid; gi++) {
      V P{shift + scale * 12 * U(rng), shift + scale * 12 * U(rng), shift + scale * 12 * U(rng)};
      const int pk = (int)(rng() % 4);
      if (pk == 1) {
        const int s = (int)(rng() % n);
        P = add({cx[s], cy[s], cz[s]}, scl(nrm({U(rng), U(rng), U(rng)}), 0.5 * std::fabs(r[s])));
      } else if (pk == 2) {
        const int s = (int)(rng() % n);
        P = add({cx[s], cy[s], cz[s]}, scl(nrm({U(rng), U(rng), U(rng)}), std::fabs(r[s]) * (1.0 + 1e-12)));
      }
      double lo[3] = {P.x, P.y, P.z}, hi[3] = {P.x, P.y, P.z};
      for (int i = 0; i < n; i++) {
        const double p[3] = {cx[i], cy[i], cz[i]};
        for (int k = 0; k < 3; k++) {
          lo[k] = std::fmin(lo[k], p[k] - std::fabs(r[i]));
          hi[k] = std::fmax(hi[k], p[k] + std::fabs(r[i]));
        }
      }
      double d2 = 0;
      for (int k = 0; k < 3; k++) d2 += (hi[k] - lo[k]) * (hi[k] - lo[k]);
      pts.push_back(P);
      diam.push_back(std::sqrt(d2));
    }
    const DevGrids dev = build_device(cx, cy, cz, r, pts, diam, N);
    const long long cells = 6LL * N * N;
    for (int gi = 0; gi < ngrid; gi++) {
      const V P = pts[gi];
      std::vector<int32_t> start, ent;
      const bool host_ok = rtk::build_point_grid(cx.data(), cy.data(), cz.data(), r.data(), n, P.x, P.y, P.z, diam[gi],
                                                 N, 1 << 30, size_t(64) << 20, start, ent);
      const int *cnt = &dev.count[gi * cells];
      const Ent *de = &dev.ent[gi * cells * K];
      for (long long c = 0; c < cells; c++) {
        ncells++;
        if (cnt[c] > K) {
          overflow++;
          continue;
        }
        for (int k = 1; k < cnt[c]; k++)
          if (!rtk::cg_before(de[c * K + k - 1].tlo, de[c * K + k - 1].s, de[c * K + k].tlo, de[c * K + k].s)) {
            if (++differ < 10) std::printf("ORDER seed %d grid %d cell %lld\n", seed, gi, c);
          }
        if (!host_ok) continue;
        std::set<std::pair<int, float>> ds, hs;
        for (int k = 0; k < cnt[c]; k++) ds.insert({de[c * K + k].s, de[c * K + k].tlo});
        for (int k = start[c]; k < start[c + 1]; k++) {
          float b;
          std::memcpy(&b, &ent[2 * k + 1], sizeof b);
          hs.insert({ent[2 * k], b});
        }
        if (ds != hs && ++differ < 10)
          std::printf("DIFF seed %d N %d grid %d cell %lld device %zu host %zu\n", seed, N, gi, c, ds.size(), hs.size());
      }
      for (int q = 0; q < 1500; q++) {
        V dir;
        if (q % 3 == 0) {
          dir = {U(rng), U(rng), U(rng)};
        } else {  // towards a point just on/off a sphere's silhouette
          const int s = (int)(rng() % n);
          V c{cx[s], cy[s], cz[s]};
          V w = sub(c, P);
          V perp = nrm({w.y - w.z, w.z - w.x, w.x - w.y});
          if (!(dot(perp, perp) > 0.5)) perp = nrm({1.0, 2.0, 3.0});
          const double f = 1.0 + ((int)(rng() % 5) - 2) * 1e-12;
          dir = sub(add(c, scl(perp, std::fabs(r[s]) * f)), P);
          if (q % 3 == 2) dir = scl(dir, -1.0);  // a silhouette behind the camera
        }
        V d = nrm(nrm(dir));  // camera.h:24 then ray.h:12
        int bi_ref = -1;
        double bt_ref = 1e20;
        for (int i = 0; i < n; i++) {  // scene.h:41-61
          double t;
          if (hit({cx[i], cy[i], cz[i]}, r[i], P, d, t) && t < bt_ref) bt_ref = t, bi_ref = i;
        }
        rays++;
        const float fx = (float)d.x, fy = (float)d.y, fz = (float)d.z;
        for (float rel : {0.0f, -0x1p-22f, 0x1p-22f}) {
          const int c = rtk::lg_cell(fx, fy, fz, N, rel);
          if (c < 0 || cnt[c] > K) continue;  // the device tests every sphere / sweeps
          std::vector<float> tlo(n, NAN);
          for (int k = 0; k < cnt[c]; k++) tlo[de[c * K + k].s] = de[c * K + k].tlo;
          for (int i = 0; i < n; i++) {
            double t;
            if (!hit({cx[i], cy[i], cz[i]}, r[i], P, d, t)) continue;
            if (rel == 0.0f) npairs++;
            if (!((double)tlo[i] <= t) && !(t != t)) {
              if (++missed < 10)
                std::printf("MISS seed %d N %d grid %d sphere %d t %.17g tlo %.9g\n", seed, N, gi, i, t, (double)tlo[i]);
            }
          }
          double bt = 1e20;  // cam_closest's scan
          int bi = -1;
          for (int k = 0; k < cnt[c]; k++) {
            if ((double)de[c * K + k].tlo > bt) break;
            const int i = de[c * K + k].s;
            double t;
            if (hit({cx[i], cy[i], cz[i]}, r[i], P, d, t) && (t < bt || (t == bt && i < bi))) bt = t, bi = i;
          }
          if (bi != bi_ref || (bi >= 0 && bt != bt_ref)) {
            if (++wrong < 10)
              std::printf("WRONG seed %d N %d grid %d got %d %.17g want %d %.17g\n", seed, N, gi, bi, bt, bi_ref, bt_ref);
          }
        }
      }
    }
  }
  std::printf("checked %ld %ld cells %ld overflow %ld differ %ld missed %ld wrong %ld\n", rays, npairs, ncells, overflow,
              differ, missed, wrong);
  return (differ != 0 || missed != 0 || wrong != 0) ? 1 : 0;
}
