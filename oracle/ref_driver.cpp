// ref_driver.cpp -- parameterised driver around the REFERENCE's own render code.
//
// TEST INFRASTRUCTURE ONLY.  Built by oracle/Makefile together with the
// unmodified /root/reference/src/main.cpp (its `main` renamed at compile time
// with -Dmain=cs420_reference_main so this file can provide the entry point).
// It calls the reference's trace_ray (src/main.cpp:16), load_scene
// (include/scene_loader.h:27), Camera (include/camera.h:10) and write_ppm
// (src/main.cpp:69) exactly as the reference's serial loop does
// (src/main.cpp:146-157), but with W/H/depth taken from argv, so golden images
// at BASELINE.json sizes come from the reference code itself.
//
//   ref_render <scene> <W> <H> <depth> [--out FILE.ppm] [--rows-every K] [--threads T]
//
// --rows-every K renders only rows j % K == 0 (a bounded CPU-baseline sample).
// --threads T runs the loop as the reference's OpenMP variant does
// (src/main.cpp:185: parallel for, schedule(dynamic), collapse(2)) on T threads.
// Prints "Serial time: X seconds" (the reference's own line, main.cpp:161).
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "camera.h"
#include "scene_loader.h"

Vec3 trace_ray(const Ray &ray, const Scene &scene, int depth);  // src/main.cpp:16
void write_ppm(const std::string &filename, const std::vector<Vec3> &framebuffer, int width,
               int height);                                      // src/main.cpp:69

int main(int argc, char **argv) {
  if (argc < 5) {
    std::cerr << "usage: ref_render scene W H depth [--out F] [--rows-every K]\n";
    return 2;
  }
  std::string scene_file = argv[1];
  int width = std::atoi(argv[2]), height = std::atoi(argv[3]), max_depth = std::atoi(argv[4]);
  std::string out;
  int every = 1, threads = 1;
  for (int i = 5; i < argc; i++) {
    if (!std::strcmp(argv[i], "--out") && i + 1 < argc) out = argv[++i];
    else if (!std::strcmp(argv[i], "--rows-every") && i + 1 < argc) every = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--threads") && i + 1 < argc) threads = std::atoi(argv[++i]);
  }
  Scene scene = load_scene(scene_file);
  Camera camera(scene.camera.position, scene.camera.look_at, scene.camera.fov);
  std::vector<Vec3> framebuffer(width * height);
  const int rows = (height + every - 1) / every;
  const long long pixels = (long long)rows * width;
  auto start = std::chrono::high_resolution_clock::now();
#ifdef _OPENMP
  omp_set_num_threads(threads > 0 ? threads : 1);
#pragma omp parallel for schedule(dynamic) collapse(2)
#endif
  for (int r = 0; r < rows; r++) {
    for (int i = 0; i < width; i++) {
      const int j = r * every;
      double u = double(i) / (width - 1);
      double v = double(j) / (height - 1);
      Ray ray = camera.get_ray(u, v);
      framebuffer[j * width + i] = trace_ray(ray, scene, max_depth);
    }
  }
  auto end = std::chrono::high_resolution_clock::now();
  std::chrono::duration<double> diff = end - start;
  std::cout << "Serial time: " << diff.count() << " seconds\n";
  std::cout << "Pixels: " << pixels << "\n";
  if (!out.empty()) write_ppm(out, framebuffer, width, height);
  return 0;
}
