// Check of the device point-grid builder (rt_kernel.hip pg_disk_kernel /
// pg_bin_kernel / the scan / sg_sort_kernel, ids_sort_kernel / sg_start_kernel,
// lg_start_kernel) on the CPU, for the sphere grids and the light grids:
// the kernels' per-lane functions (csrc/rt_cgbuild.h: cg_view with the origin
// ball's rho, cg_side, cg_block, cg_tile, cg_cell, cg_before) run lane by
// lane in the kernels' pass structure -- pass 1 a wave per (grid, sphere)
// appending (disk, block) pairs and counting global spheres, the host's
// refusal of a grid with more than 32 globals, the bin pass per quarter pair
// counting then filling CSR lists, the (tlo, index) sort -- against the host
// builder (rt_lightgrid.cpp build_sphere_grids, the one rt_upload_scene used
// before) on random scenes: which spheres get a grid, and for every grid and
// cell the exact list (sphere, tlo bits) in order.  The light grids (one side,
// global spheres on a separate list, nearest first) against build_light_grid
// (ids ascending): every light's start row and the same ids in every list,
// lights with non-finite positions included.
// Prints "scenes <n> grids <n> refused <n> cells <n> entries <n> differ <n>
// lights <n> light_entries <n> light_differ <n>".
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "rt_cgbuild.h"

namespace {
struct E {
  int s;
  float tlo;
};

// the device build for the grid spheres gsph (rho per sphere): per grid ok and
// per-cell lists in the kernels' final order
void build_device(const std::vector<double> &cx, const std::vector<double> &cy, const std::vector<double> &cz,
                  const std::vector<double> &r, const std::vector<double> &rho, const std::vector<int> &gsph,
                  double diam, int N, int max_global, std::vector<unsigned char> &ok,
                  std::vector<std::vector<E>> &lists) {
  const int n = (int)cx.size(), ng = (int)gsph.size();
  std::vector<rtk::CubePatch> faces, blocks, tiles;
  std::vector<double> cell;
  int NT = 0, NB = 0;
  rtk::cube_tables(N, faces, blocks, tiles, cell, NT, NB);
  const int nb = 6 * NB * NB;
  const long long cells = 6LL * N * N;
  ok.assign((size_t)ng, 0);
  lists.assign((size_t)(ng * cells), {});
  for (int j = 0; j < ng; j++) {
    const int gs = gsph[j];
    std::vector<rtk::CgDisk> disks(2 * (size_t)n);
    std::vector<std::pair<int, int>> pairs;
    int nglob = 0;
    for (int i = 0; i < n; i++) {  // pass 1: a wave per (grid, sphere)
      const rtk::CgView v = rtk::cg_view(cx[i], cy[i], cz[i], std::fabs(r[i]), cx[gs], cy[gs], cz[gs], diam, rho[gs]);
      nglob += v.global ? 1 : 0;
      for (int side = 0; side < (v.global ? 1 : 2); ++side) {
        const rtk::CgDisk k = rtk::cg_side(v, side, i);
        disks[2 * i + side] = k;
        for (int b = 0; b < nb; b++)
          if (rtk::cg_block(k, faces.data(), blocks.data(), NB, b)) pairs.push_back({2 * i + side, b});
      }
    }
    if (nglob > max_global) continue;  // refused: no lists
    ok[(size_t)j] = 1;
    for (const auto &pr : pairs)  // the bin pass, all four quarters
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
          const int tl = __builtin_ctzll(tmask);
          tmask &= tmask - 1;
          for (int lane = 0; lane < 64; lane++) {
            const int gc = rtk::cg_cell(k, wide, cell.data(), N, f, bi, bj, tl, lane, (imask >> tl) & 1ull);
            if (gc >= 0) lists[(size_t)(j * cells + gc)].push_back(E{k.s, k.tlo});
          }
        }
      }
    for (long long c = 0; c < cells; c++) {  // sg_sort_kernel: insertion sort by (tlo, index)
      std::vector<E> &e = lists[(size_t)(j * cells + c)];
      for (size_t k = 1; k < e.size(); ++k) {
        const E x = e[k];
        long m = (long)k - 1;
        while (m >= 0 && rtk::cg_before(x.tlo, x.s, e[(size_t)m].tlo, e[(size_t)m].s)) {
          e[(size_t)m + 1] = e[(size_t)m];
          --m;
        }
        e[(size_t)m + 1] = x;
      }
    }
  }
}
// the device build of the light grids: per light, lists for the 6N^2 cells
// and the global list (index 6N^2), nearest first
std::vector<std::vector<int>> build_device_lights(const std::vector<double> &cx, const std::vector<double> &cy,
                                                  const std::vector<double> &cz, const std::vector<double> &r,
                                                  const std::vector<double> &lx, const std::vector<double> &ly,
                                                  const std::vector<double> &lz, double diam, int N) {
  const int n = (int)cx.size(), nl = (int)lx.size();
  std::vector<rtk::CubePatch> faces, blocks, tiles;
  std::vector<double> cell;
  int NT = 0, NB = 0;
  rtk::cube_tables(N, faces, blocks, tiles, cell, NT, NB);
  const int nb = 6 * NB * NB;
  const long long cells = 6LL * N * N, row = cells + 1;
  const double dm = std::isfinite(diam) ? diam : 0.0;
  std::vector<std::vector<int>> lists((size_t)(nl * row));
  for (int l = 0; l < nl; l++) {
    const bool allglob = !(std::isfinite(lx[l]) && std::isfinite(ly[l]) && std::isfinite(lz[l]));
    for (int i = 0; i < n; i++) {
      rtk::CgView v = rtk::cg_view(cx[i], cy[i], cz[i], std::fabs(r[i]), lx[l], ly[l], lz[l], dm, 0.0, rtk::kLgOvershoot);
      if (allglob) v = rtk::cg_view(0.0, 0.0, 0.0, INFINITY, 0.0, 0.0, 0.0, 0.0);
      if (v.global) {
        lists[(size_t)(l * row + cells)].push_back(i);
        continue;
      }
      const rtk::CgDisk k = rtk::cg_side(v, 0, i);
      for (int b = 0; b < nb; b++) {
        if (!rtk::cg_block(k, faces.data(), blocks.data(), NB, b)) continue;
        const bool wide = rtk::cg_wide(k);
        const int f = b / (NB * NB), bj = (b / NB) % NB, bi = b % NB;
        unsigned long long tmask = 0, imask = 0;
        for (int lane = 0; lane < 64; lane++) {
          bool tm, inside;
          rtk::cg_tile(k, tiles.data(), NT, f, bi, bj, lane, tm, inside);
          if (tm) tmask |= 1ull << lane;
          if (inside) imask |= 1ull << lane;
        }
        while (tmask) {
          const int tl = __builtin_ctzll(tmask);
          tmask &= tmask - 1;
          for (int lane = 0; lane < 64; lane++) {
            const int gc = rtk::cg_cell(k, wide, cell.data(), N, f, bi, bj, tl, lane, (imask >> tl) & 1ull);
            if (gc >= 0) lists[(size_t)(l * row + gc)].push_back(i);
          }
        }
      }
    }
  }
  // ids_sort_kernel with `near`: each list by (|C - L| - |r|, id), the
  // kernel's insertion sort and comparison (NaN keys fall back to the id)
  for (int l = 0; l < nl; l++)
    for (long long c = 0; c < row; c++) {
      std::vector<int> &e = lists[(size_t)(l * row + c)];
      auto key = [&](int i) {
        const double dx = cx[i] - lx[l], dy = cy[i] - ly[l], dz = cz[i] - lz[l];
        return std::sqrt(dx * dx + dy * dy + dz * dz) - std::sqrt(r[i] * r[i]);
      };
      std::sort(e.begin(), e.end());  // the fill order is arbitrary on the device: start from a fixed one
      for (size_t k = 1; k < e.size(); ++k) {
        const int x = e[k];
        const double kx = key(x);
        long m = (long)k - 1;
        while (m >= 0) {
          const double km = key(e[(size_t)m]);
          if (!(kx < km || (!(km < kx) && x < e[(size_t)m]))) break;
          e[(size_t)m + 1] = e[(size_t)m];
          --m;
        }
        e[(size_t)m + 1] = x;
      }
    }
  return lists;
}
}  // namespace

int main(int argc, char **argv) {
  const int seeds = argc > 1 ? std::atoi(argv[1]) : 20;
  long scenes = 0, grids = 0, refused = 0, ncells = 0, entries = 0, differ = 0, lights = 0, lentries = 0,
       ldiffer = 0;
  for (int seed = 0; seed < seeds; seed++) {
    std::mt19937_64 rng(9100 + seed);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    const double scale = std::pow(10.0, (int)(rng() % 5) - 1);  // 0.1 .. 1000
    const double shift = (rng() % 3 == 0) ? 1e5 * scale : 0.0;
    const int n = 5 + (int)(rng() % 120);
    const bool dense = rng() % 4 == 0;  // overlapping clusters: grids with many globals, some refused
    const int N = (int[]){1, 3, 8, 16, 32}[rng() % 5];
    std::vector<double> cx(n), cy(n), cz(n), r(n), refl(n);
    for (int i = 0; i < n; i++) {
      const double sp = dense ? 1.0 : 10.0;
      cx[i] = shift + scale * sp * U(rng);
      cy[i] = shift + scale * sp * U(rng);
      cz[i] = shift + scale * sp * U(rng);
      const int kind = (int)(rng() % 10);
      r[i] = scale * (kind == 0 ? 1e-4 : kind == 1 ? 5.0 : 0.05 + 1.5 * std::fabs(U(rng)));
      if (kind == 2) r[i] = -r[i];  // the parser accepts negative radii
      refl[i] = rng() % 4 == 0 ? 0.0 : 0.5;
    }
    if (n > 3) r[3] = scale * 200.0;  // a ground-like sphere
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    for (int i = 0; i < n; i++) {
      const double p[3] = {cx[i], cy[i], cz[i]};
      for (int k = 0; k < 3; k++) {
        lo[k] = std::fmin(lo[k], p[k] - std::fabs(r[i]));
        hi[k] = std::fmax(hi[k], p[k] + std::fabs(r[i]));
      }
    }
    double d2 = 0;
    for (int k = 0; k < 3; k++) d2 += (hi[k] - lo[k]) * (hi[k] - lo[k]);
    const double diam = std::sqrt(d2);
    // rho and the grid spheres exactly as rt_kernel.hip sphere_grids
    std::vector<double> rho((size_t)n, -1.0);
    std::vector<int> gsph;
    for (int i = 0; i < n; i++) {
      const double rr = std::fabs(r[i]), mag = std::fabs(cx[i]) + std::fabs(cy[i]) + std::fabs(cz[i]);
      if (refl[i] > 0.0 && std::isfinite(rr) && std::isfinite(mag))
        rho[(size_t)i] = (rr + 0.001) * (1.0 + 1e-6) + 1e-12 * mag + 1e-9 * diam;
      if (rho[(size_t)i] >= 0.0 && std::isfinite(rho[(size_t)i])) gsph.push_back(i);
    }
    const int max_global = dense ? 4 : 32;
    std::vector<int32_t> start, ent;
    std::vector<uint8_t> hok;
    rtk::build_sphere_grids(cx.data(), cy.data(), cz.data(), r.data(), n, rho.data(), diam, N, max_global,
                            size_t(64) << 20, start, ent, hok);
    std::vector<unsigned char> dok;
    std::vector<std::vector<E>> lists;
    build_device(cx, cy, cz, r, rho, gsph, diam, N, max_global, dok, lists);
    const long long cells = 6LL * N * N;
    scenes++;
    std::vector<int> gidx((size_t)n, -1);
    for (size_t j = 0; j < gsph.size(); j++) gidx[(size_t)gsph[j]] = (int)j;
    for (int s = 0; s < n; s++) {
      const int j = gidx[(size_t)s];
      const bool d_ok = j >= 0 && dok[(size_t)j];
      if (d_ok != (hok[(size_t)s] != 0)) {
        differ++;
        continue;
      }
      if (j >= 0 && !d_ok) refused++;
      if (!d_ok) continue;
      grids++;
      for (long long c = 0; c < cells; c++) {
        const std::vector<E> &dl = lists[(size_t)(j * cells + c)];
        const size_t b = (size_t)start[(size_t)s * (cells + 1) + c], e = (size_t)start[(size_t)s * (cells + 1) + c + 1];
        ncells++;
        entries += (long)dl.size();
        bool same = dl.size() == e - b;
        for (size_t k = 0; same && k < dl.size(); k++) {
          float ht;
          std::memcpy(&ht, &ent[2 * (b + k) + 1], sizeof ht);
          same = dl[k].s == ent[2 * (b + k)] && std::memcmp(&dl[k].tlo, &ht, sizeof ht) == 0;
        }
        differ += same ? 0 : 1;
      }
    }
    // light grids: 1-6 lights (one maybe non-finite, one inside a sphere), N as drawn (or 128 / 768-like sizes)
    const int nl = 1 + (int)(rng() % 6);
    std::vector<double> lx(nl), ly(nl), lz(nl);
    for (int l = 0; l < nl; l++) {
      lx[l] = shift + scale * 15 * U(rng);
      ly[l] = shift + scale * 15 * U(rng);
      lz[l] = shift + scale * 15 * U(rng);
    }
    if (nl > 1 && rng() % 3 == 0) lx[1] = NAN;
    if (nl > 2) lx[2] = cx[0], ly[2] = cy[0], lz[2] = cz[0];  // a light at a sphere's centre
    const int NL = (int[]){1, 3, 16, 64, 128}[rng() % 5];
    std::vector<int32_t> lstart, lids;
    rtk::build_light_grid(cx.data(), cy.data(), cz.data(), r.data(), n, lx.data(), ly.data(), lz.data(), nl, diam, NL,
                          lstart, lids);
    const std::vector<std::vector<int>> dl = build_device_lights(cx, cy, cz, r, lx, ly, lz, diam, NL);
    const long long lcells = 6LL * NL * NL;
    // the device's start row is the exclusive prefix of its list lengths (lg_start_kernel)
    long long off = 0;
    for (int l = 0; l < nl; l++) {
      lights++;
      bool same = true;
      for (long long c = 0; c <= lcells; c++) {
        const std::vector<int> &e = dl[(size_t)(l * (lcells + 1) + c)];
        same = same && lstart[(size_t)(l * (lcells + 2) + c)] == off &&
               lstart[(size_t)(l * (lcells + 2) + c + 1)] == off + (long long)e.size();
        // the same ids (the host builder's ascending, the device's nearest-first)
        std::vector<int> asc(e);
        std::sort(asc.begin(), asc.end());
        for (size_t k = 0; same && k < asc.size(); k++) same = lids[(size_t)off + k] == asc[k];
        off += (long long)e.size();
        lentries += (long)e.size();
      }
      ldiffer += same ? 0 : 1;
    }
  }
  std::printf("scenes %ld grids %ld refused %ld cells %ld entries %ld differ %ld lights %ld light_entries %ld "
              "light_differ %ld\n",
              scenes, grids, refused, ncells, entries, differ, lights, lentries, ldiffer);
  return differ || ldiffer ? 1 : 0;
}
