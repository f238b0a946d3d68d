// Host ASan/UBSan driver (SURVEY 5 "sanitizers"): every host-side builder
// whose output decides what the GPU may skip or how it reads memory -- the
// scene parser and P3/P6 writer (rt_host.cpp), the BVH builders (rt_bvh.cpp),
// the light direction grids (rt_lightgrid.cpp), the tile scheduler
// (rt_sched.cpp), ray_hybrid's CPU tile worker (rt_cpu.cpp) -- and the oracle
// (oracle/rt_oracle.c) run on random and hostile inputs.  Built with
// -fsanitize=address,undefined -fno-sanitize-recover=all by
// tests/test_sanitize.py; any report aborts the process.  Structural checks on
// the outputs (indices in range, lists sorted) are asserted here too.
//   host_sanitize SCENE_DIR TMP_DIR ITERATIONS
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "rt_bvh.h"
#include "rt_cpu.h"
#include "rt_hip.h"
#include "rt_lightgrid.h"
#include "rt_sched.h"

extern "C" {
#include "rt_oracle.h"
}

#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::abort();                                                     \
    }                                                                   \
  } while (0)

namespace {

std::mt19937_64 rng(20261016);

double uni(double a, double b) { return std::uniform_real_distribution<double>(a, b)(rng); }
int irand(int a, int b) { return std::uniform_int_distribution<int>(a, b)(rng); }

// A number token, sometimes hostile.
std::string num() {
  switch (irand(0, 11)) {
    case 0: return "nan";
    case 1: return "inf";
    case 2: return "-inf";
    case 3: return "1e400";
    case 4: return "-0";
    case 5: return "0x1p3";
    case 6: return "abc";
    case 7: return std::to_string(irand(-3, 3));
    default: {
      char b[64];
      std::snprintf(b, sizeof b, "%.6g", uni(-50, 50));
      return b;
    }
  }
}

std::string random_scene_text() {
  static const char *kw[] = {"sphere", "light", "ambient", "camera", "#", "bogus", "", "  sphere", "\tlight"};
  static const int nargs[] = {10, 7, 3, 7, 2, 1, 0, 10, 7};
  std::ostringstream s;
  const int lines = irand(0, 60);
  for (int i = 0; i < lines; ++i) {
    const int k = irand(0, 8);
    s << kw[k];
    const int n = nargs[k] + irand(-2, 2);
    for (int j = 0; j < n; ++j) s << (irand(0, 9) == 0 ? "\t" : " ") << num();
    s << (irand(0, 20) == 0 ? "\r\n" : "\n");
  }
  if (irand(0, 5) == 0) s << std::string((size_t)irand(0, 5000), 'x');  // a long unterminated line
  return s.str();
}

void parse_and_use(const std::string &text, const char *tmp) {
  rt_scene sc;
  if (rt_scene_parse(text.c_str(), &sc, 0) != RT_OK) return;
  CHECK(sc.num_spheres >= 0 && sc.num_lights >= 0);
  rt_camera cam;
  rt_camera_from_scene(&sc, &cam);
  // the oracle parses the same text the same way
  orc_scene os;
  if (orc_parse_scene(text.c_str(), &os, 0) == 0) {
    CHECK(os.num_spheres == sc.num_spheres && os.num_lights == sc.num_lights);
    orc_free_scene(&os);
  }
  if (sc.num_spheres <= 40 && sc.num_lights <= 6) {
    rtc::CpuTracer cpu(sc, cam);
    std::vector<rtc::V3> fb(7 * 5);
    cpu.render_tile(0, 0, 7, 5, 7, 5, irand(0, 4), fb.data());
    (void)cpu.tile_complexity(0, 0, 7, 5, 7, 5);
  }
  (void)tmp;
  rt_scene_free(&sc);
}

void bvh_case(int n) {
  std::vector<double> cx(n), cy(n), cz(n), r(n);
  const double spread = std::pow(10.0, uni(-3, 6));
  for (int i = 0; i < n; ++i) {
    cx[i] = uni(-spread, spread), cy[i] = uni(-spread, spread), cz[i] = uni(-spread, spread);
    r[i] = uni(-1, 1) * spread * 0.1;
    switch (irand(0, 40)) {
      case 0: cx[i] = std::numeric_limits<double>::quiet_NaN(); break;
      case 1: r[i] = std::numeric_limits<double>::infinity(); break;
      case 2: r[i] = 0; break;
      case 3: if (i) cx[i] = cx[i - 1], cy[i] = cy[i - 1], cz[i] = cz[i - 1]; break;
    }
  }
  std::vector<rtk::BvhNode> nodes;
  std::vector<int32_t> prims;
  rtk::build_bvh(cx.data(), cy.data(), cz.data(), r.data(), n, irand(1, 15), nodes, prims);
  CHECK(prims.size() == (size_t)n);
  std::vector<char> seen((size_t)n, 0);
  for (int32_t p : prims) {
    CHECK(p >= 0 && p < n && !seen[(size_t)p]);
    seen[(size_t)p] = 1;
  }
  for (size_t i = 0; i < nodes.size(); ++i) {
    CHECK(nodes[i].skip > (int32_t)i && nodes[i].skip <= (int32_t)nodes.size());
    if (nodes[i].leaf >= 0) CHECK((nodes[i].leaf >> 4) + (nodes[i].leaf & 15) <= n);
  }
  if (!nodes.empty()) {
    std::vector<rtk::BvhNode2> n2;
    std::vector<rtk::BvhNode4> n4;
    int depth = 0, stack = 0;
    const int32_t r2 = rtk::build_bvh2(nodes, n2, depth);
    const int32_t r4 = rtk::build_bvh4(nodes, n4, stack);
    CHECK(r2 < (int32_t)n2.size() && r4 < (int32_t)n4.size() && depth >= 0 && stack >= 0);
    for (const auto &q : n2) CHECK(q.c0 < (int32_t)n2.size() && q.c1 < (int32_t)n2.size());
    for (const auto &q : n4)
      for (int k = 0; k < 4; ++k) CHECK(q.c[k] < (int32_t)n4.size());
  }
}

// The uniform grid (rt_bvh.h build_ugrid): CSR, cell records and overflow
// entries consistent, for spreads 1e-3 .. 1e6, duplicate centres, zero /
// negative / non-finite radii and a few huge spheres.
void ugrid_case(int n) {
  std::vector<double> cx(n), cy(n), cz(n), r(n);
  const double spread = std::pow(10.0, uni(-3, 6));
  const bool flat = irand(0, 3) == 0;  // every centre in one plane
  for (int i = 0; i < n; ++i) {
    cx[i] = uni(-spread, spread), cy[i] = flat ? 0.0 : uni(-spread, spread), cz[i] = uni(-spread, spread);
    r[i] = uni(-1, 1) * spread * 0.05;
    switch (irand(0, 60)) {
      case 0: cx[i] = std::numeric_limits<double>::quiet_NaN(); break;
      case 1: r[i] = std::numeric_limits<double>::infinity(); break;
      case 2: r[i] = 0; break;
      case 3: if (i) cx[i] = cx[i - 1], cy[i] = cy[i - 1], cz[i] = cz[i - 1]; break;
      case 4: r[i] = spread * 3; break;  // wider than the cloud: a global sphere
    }
  }
  rtk::UgridHost g;
  if (!rtk::build_ugrid(cx.data(), cy.data(), cz.data(), r.data(), n, size_t(1) << 20, g, uni(0.3, 6))) return;
  const size_t cells = (size_t)g.nx * g.ny * g.nz;
  CHECK(g.nx >= 1 && g.ny >= 1 && g.nz >= 1 && g.cs > 0.0f);
  CHECK(g.start.size() == cells + 1 && g.start[0] == 0 && (size_t)g.start[cells] == g.ids.size());
  CHECK(g.rec.size() == 4 * cells && g.rid.size() == 4 * cells && g.q.size() >= g.ids.size());
  for (int32_t k : g.glob) CHECK(k >= 0 && k < n);
  for (size_t c = 0; c < cells; ++c) {
    const int32_t b = g.start[c], e = g.start[c + 1];
    CHECK(b <= e);
    for (int32_t k = b; k < e; ++k) CHECK(g.ids[(size_t)k] >= 0 && g.ids[(size_t)k] < n);
    for (int j = 0; j < 4; ++j) {
      const rtk::UgRec &q = g.rec[4 * c + j];
      if (q.w >= 0.0f) {
        CHECK(g.rid[4 * c + j] == g.ids[(size_t)b + j]);
      } else if (q.w == -2.0f) {
        int32_t k0, k1;
        std::memcpy(&k0, &q.x, sizeof k0);
        std::memcpy(&k1, &q.y, sizeof k1);
        CHECK(j == 3 && k0 == b + 3 && k1 == e);
      } else {
        CHECK(q.w == -1.0f && j >= e - b);  // past the last entry
      }
    }
  }
}

void grid_case(int n, int nl) {
  std::vector<double> cx(n), cy(n), cz(n), r(n), lx(nl), ly(nl), lz(nl);
  for (int i = 0; i < n; ++i) {
    cx[i] = uni(-20, 20), cy[i] = uni(-5, 5), cz[i] = uni(-40, 0), r[i] = uni(0.01, 3);
    if (irand(0, 50) == 0) r[i] = std::numeric_limits<double>::quiet_NaN();
  }
  for (int l = 0; l < nl; ++l) {
    lx[l] = uni(-20, 20), ly[l] = uni(-5, 15), lz[l] = uni(-40, 5);
    if (n && irand(0, 4) == 0) {  // a light on a sphere's surface
      const int i = irand(0, n - 1);
      lx[l] = cx[i] + r[i], ly[l] = cy[i], lz[l] = cz[i];
    }
  }
  const int N = irand(1, 24);
  std::vector<int32_t> start, ids;
  rtk::build_light_grid(cx.data(), cy.data(), cz.data(), r.data(), n, lx.data(), ly.data(), lz.data(), nl, 200.0, N,
                        start, ids);
  const size_t stride = 6 * (size_t)N * N + 2;
  CHECK(start.size() >= stride * (size_t)nl);
  for (int l = 0; l < nl; ++l)
    for (size_t c = 0; c + 1 < stride; ++c) {
      const int32_t b = start[l * stride + c], e = start[l * stride + c + 1];
      CHECK(b >= 0 && b <= e && e <= (int32_t)ids.size());
      for (int32_t k = b; k < e; ++k) {
        CHECK(ids[(size_t)k] >= 0 && ids[(size_t)k] < n);
        if (k > b) CHECK(ids[(size_t)k] > ids[(size_t)k - 1]);
      }
    }
  for (int k = 0; k < 1000; ++k) {
    const int c = rtk::lg_cell((float)uni(-1, 1), (float)uni(-1, 1), (float)uni(-1, 1), N);
    CHECK(c >= -1 && c < 6 * N * N);
  }
  // the camera grid around a random point or a sphere's centre
  std::vector<int32_t> cst, cent;
  const int s0 = n > 0 ? irand(0, n - 1) : 0;
  const bool at_centre = n > 0 && irand(0, 1) == 1;
  const double qx = at_centre ? cx[s0] : uni(-20, 20), qy = at_centre ? cy[s0] : uni(-20, 20),
               qz = at_centre ? cz[s0] : uni(-20, 20);
  if (rtk::build_point_grid(cx.data(), cy.data(), cz.data(), r.data(), n, qx, qy, qz, 200.0, N, 8,
                            size_t(1) << 22, cst, cent)) {
    const size_t cells = 6 * (size_t)N * N;
    CHECK(cst.size() == cells + 1 && cst[0] == 0 && (size_t)cst[cells] * 2 == cent.size());
    for (size_t c = 0; c < cells; ++c) {
      CHECK(cst[c] <= cst[c + 1]);
      for (int32_t k = cst[c]; k < cst[c + 1]; ++k) {
        CHECK(cent[2 * (size_t)k] >= 0 && cent[2 * (size_t)k] < n);
        float t0, t1;
        std::memcpy(&t1, &cent[2 * (size_t)k + 1], sizeof t1);
        if (k > cst[c]) {
          std::memcpy(&t0, &cent[2 * (size_t)k - 1], sizeof t0);
          CHECK(!(t1 < t0));  // ascending bounds
        }
      }
    }
  }
}

void sched_case() {
  rtk::SchedView v{};
  v.px = uni(-5, 5), v.py = uni(-5, 5), v.pz = uni(0, 20);
  v.fx = 0, v.fy = 0, v.fz = -1, v.rx = 1, v.ry = 0, v.rz = 0, v.ux = 0, v.uy = 1, v.uz = 0;
  v.scale = uni(0.1, 2);
  v.W = irand(1, 700), v.H = irand(1, 500);
  v.band = irand(1, 8);
  const int G = irand(1, 8);
  v.first = irand(0, G - 1), v.stride = G;
  const int nb = (v.H + v.band - 1) / v.band;
  v.count = ((nb + G - 1) / G) * v.band;
  v.x0 = irand(0, v.W - 1), v.xw = irand(1, v.W - v.x0);
  v.tw = 8, v.th = 8;
  std::vector<rtk::SchedSphere> refl;
  for (int i = irand(0, 30); i > 0; --i) refl.push_back({uni(-10, 10), uni(-5, 5), uni(-40, 0), uni(-2, 2)});
  std::vector<int> perm;
  rtk::tile_order(v, refl, perm);
  const int ntx = (v.xw + v.tw - 1) / v.tw, nty = (v.count + v.th - 1) / v.th;
  CHECK(perm.size() == (size_t)ntx * nty);
  std::vector<char> seen(perm.size(), 0);
  for (int p : perm) {
    CHECK(p >= 0 && p < (int)perm.size() && !seen[(size_t)p]);
    seen[(size_t)p] = 1;
  }
}

}  // namespace

int main(int argc, char **argv) {
  if (argc != 4) return 2;
  const std::string dir = argv[1], tmp = argv[2];
  const int iters = std::atoi(argv[3]);
  for (const char *name : {"simple", "medium", "complex", "synth200"}) {
    std::ifstream f(dir + "/" + name + ".txt");
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string text = ss.str();
    parse_and_use(text, tmp.c_str());
    rt_scene sc;
    CHECK(rt_scene_load((dir + "/" + name + ".txt").c_str(), &sc, 0) == RT_OK);
    // the oracle on a tiny image of the real scene
    orc_scene os;
    CHECK(orc_parse_scene(text.c_str(), &os, 0) == 0);
    std::vector<uint8_t> rgb(9 * 7 * 3);
    orc_counts cnt;
    CHECK(orc_render(&os, 9, 7, 4, 1, 0, 1, 7, rgb.data(), nullptr, &cnt, 1) == 0);
    orc_free_scene(&os);
    rt_scene_free(&sc);
  }
  CHECK(rt_scene_load((tmp + "/does_not_exist.txt").c_str(), nullptr, 0) == RT_ERR_INVALID_ARG);
  {
    rt_scene none;
    CHECK(rt_scene_load((tmp + "/does_not_exist.txt").c_str(), &none, 0) == RT_ERR_IO);
    rt_scene_free(&none);
  }
  for (int i = 0; i < iters; ++i) {
    parse_and_use(random_scene_text(), tmp.c_str());
    bvh_case(irand(0, 300));
    ugrid_case(irand(0, 400));
    grid_case(irand(0, 80), irand(0, 5));
    sched_case();
    if (i % 16 == 0) {
      const int W = irand(1, 17), H = irand(1, 17);
      std::vector<uint8_t> rgb((size_t)W * H * 3);
      for (auto &b : rgb) b = (uint8_t)irand(0, 255);
      CHECK(rt_write_ppm((tmp + "/p.ppm").c_str(), rgb.data(), W, H, i & 1) == RT_OK);
      CHECK(orc_write_p3((tmp + "/q.ppm").c_str(), rgb.data(), W, H) == 0);
    }
  }
  CHECK(rt_write_ppm((tmp + "/no_such_dir/x.ppm").c_str(), nullptr, 1, 1, 0) != RT_OK);
  std::printf("sanitized %d iterations ok\n", iters);
  return 0;
}
