// Host check of ray_hybrid's CPU tile worker (csrc/rt_cpu.cpp) without a GPU:
//   cpu_tiles_check SCENE W H DEPTH TILE OUT_RGB OUT_COSTS
// renders the image tile by tile (process_tile_cpu's order of tiles and pixels
// does not matter: every pixel is independent), quantises it in write_ppm's
// PPM row order (main.cpp:69-91) into OUT_RGB, and writes every tile's
// estimate_tile_complexity (scanline order of tiles) to OUT_COSTS, one per
// line.  tests/test_hybrid.py compares both with the oracle.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rt_cpu.h"
#include "rt_hip.h"

int main(int argc, char **argv) {
  if (argc != 8) return 2;
  const int W = std::atoi(argv[2]), H = std::atoi(argv[3]), D = std::atoi(argv[4]), ts = std::atoi(argv[5]);
  rt_scene sc;
  if (rt_scene_load(argv[1], &sc, 0) != RT_OK) return 3;
  rt_camera cam;
  rt_camera_from_scene(&sc, &cam);
  rtc::CpuTracer cpu(sc, cam);
  std::vector<rtc::V3> fb((size_t)W * H);
  FILE *costs = std::fopen(argv[7], "w");
  for (int y = 0; y < H; y += ts)
    for (int x = 0; x < W; x += ts) {
      const int x1 = std::min(x + ts, W), y1 = std::min(y + ts, H);
      cpu.render_tile(x, y, x1, y1, W, H, D, fb.data());
      std::fprintf(costs, "%d\n", cpu.tile_complexity(x, y, x1, y1, W, H));
    }
  std::fclose(costs);
  std::vector<unsigned char> rgb;
  for (int j = H - 1; j >= 0; --j)
    for (int i = 0; i < W; ++i) {
      const rtc::V3 c = fb[(size_t)j * W + i];
      for (double ch : {c.x, c.y, c.z}) {
        const int q = int(255.99 * std::min(1.0, ch));
        rgb.push_back((unsigned char)(q < 0 ? 0 : q));
      }
    }
  FILE *out = std::fopen(argv[6], "wb");
  std::fwrite(rgb.data(), 1, rgb.size(), out);
  std::fclose(out);
  rt_scene_free(&sc);
  return 0;
}
