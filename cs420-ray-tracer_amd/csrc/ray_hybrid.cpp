// ray_hybrid.cpp -- the hybrid CPU+GPU tile renderer, a
// drop-in for the reference's ray_hybrid (src/main_hybrid.cpp:321-830).
//
//   ray_hybrid [--pipeline|-p] [--tile-size|-t N] [--output|-o FILE] [--help|-h] [scene]
//
// Same argv grammar, defaults (1080x720, depth 3, 64x64 tiles, scenes/simple.txt,
// output_hybrid.ppm; main_hybrid.cpp:41-42, 726-753) and stdout lines.  The
// image is split into tiles; estimate_tile_complexity (5 camera rays per tile)
// sends tiles above a threshold (7, or 9 with --pipeline) to the CPU workers and
// the rest to the GPU, rendered through librt_hip.so's rt_render_tile on
// NUM_STREAMS contexts round robin (render_hybrid, :351-460: one download per
// tile; render_hybrid_pipeline, :462-590: every GPU tile launched, then one
// download).  As upstream, --pipeline always uses 64x64 tiles (:790 passes no
// tile size).
//
// Both halves compute the serial fp64 colours (the GPU through the HIP
// kernels, the CPU through rt_cpu.cpp), so output_hybrid.ppm is ray_serial's
// image of the same size byte for byte, whatever the split -- upstream's GPU
// tiles were the fp32 CUDA kernel's approximation.
//
// Extra options: --width W --height H --depth D, --threads N (CPU workers,
// default: OMP_NUM_THREADS, else hardware threads - 1), --cpu-threshold N (complexity above N goes to
// the CPU; -1 sends every tile there), --device N, --streams N, and --dynamic: instead of the static
// split, tiles sorted by estimated cost form one deque; the GPU thread takes
// the costliest from the front in batches (one rt_render_tiles launch each),
// each CPU worker the cheapest from the back, until it is empty.  With
// --pipeline every GPU tile goes into ONE rt_render_tiles launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rt_cpu.h"
#include "rt_hip.h"

namespace {

struct Opts {
  bool pipeline = false, dynamic = false;
  int tile = 64, width = 1080, height = 720, depth = 3;  // main_hybrid.cpp:41-42, 736-738
  int threads = -1, threshold = INT_MIN, device = 0, streams = 3;  // INT_MIN: the reference's threshold
  std::string out = "output_hybrid.ppm", scene = "scenes/simple.txt";
};

struct Tile {
  int x0, y0, x1, y1, cost;
  bool gpu, done;
};

int usage(const char *argv0) {  // main_hybrid.cpp:741-750
  std::printf("Usage: %s [options] [scene_file]\n", argv0);
  std::printf("Options:\n");
  std::printf("  --pipeline, -p        Use pipelined execution\n");
  std::printf("  --tile-size, -t SIZE  Set tile size (default: 64)\n");
  std::printf("  --output, -o FILE     Output filename\n");
  std::printf("  --help, -h            Show this help message\n");
  std::printf("  --width W --height H --depth D, --threads N, --cpu-threshold N,\n"
              "  --device N, --streams N, --dynamic   (extensions)\n");
  std::printf("\nPositional arguments:\n");
  std::printf("  scene_file            Scene file to load (default: scenes/simple.txt)\n");
  return 0;
}

#define CK(call)                                                                    \
  do {                                                                              \
    int rc_ = (call);                                                               \
    if (rc_ != RT_OK) {                                                             \
      std::fprintf(stderr, "%s failed: %s\n", #call, rt_error_string(rc_));          \
      return 1;                                                                     \
    }                                                                               \
  } while (0)
#define HK(call)                                                                    \
  do {                                                                              \
    hipError_t e_ = (call);                                                         \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s failed: %s\n", #call, hipGetErrorString(e_));         \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

// The GPU half: NUM_STREAMS contexts (each its own stream and scene copy) over
// one full-image device framebuffer of doubles (RT_FB_F64X3 = the serial
// framebuffer layout, main.cpp:156).
struct Gpu {
  std::vector<rt_ctx *> ctx;
  std::vector<hipStream_t> st;
  double *dfb = nullptr;
  int W = 0, H = 0, depth = 0, next = 0;
  rt_camera cam{};

  int open(const Opts &o, const rt_scene &sc, const rt_camera &c) {
    W = o.width, H = o.height, depth = o.depth, cam = c;
    HK(hipSetDevice(o.device));
    HK(hipMalloc(&dfb, (size_t)W * H * 3 * sizeof(double)));
    for (int i = 0; i < o.streams; ++i) {
      rt_ctx *x = nullptr;
      CK(rt_create(o.device, &x));
      ctx.push_back(x);
      hipStream_t s;
      HK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      st.push_back(s);
      CK(rt_set_stream(x, s));
      CK(rt_upload_scene(x, &sc));
    }
    return 0;
  }
  // launch_gpu_kernel for one tile (main_hybrid.cpp:457-463), round robin over the streams
  int launch(const Tile &t, int &k) {
    k = next;
    next = (next + 1) % (int)ctx.size();
    CK(rt_render_tile(ctx[(size_t)k], &cam, W, H, depth, t.x0, t.y0, t.x1 - t.x0, t.y1 - t.y0, RT_FB_F64X3, dfb));
    return 0;
  }
  // several tiles in ONE launch (rt_render_tiles) on the next context
  int launch_batch(const std::vector<Tile *> &ts, int &k) {
    k = next;
    next = (next + 1) % (int)ctx.size();
    std::vector<rt_tile> rects;
    for (const Tile *t : ts) rects.push_back(rt_tile{t->x0, t->y0, t->x1 - t->x0, t->y1 - t->y0});
    CK(rt_render_tiles(ctx[(size_t)k], &cam, W, H, depth, rects.data(), (int)rects.size(), RT_FB_F64X3, dfb));
    return 0;
  }
  // download_tile (main_hybrid.cpp:281-309): the tile's rows straight into the host framebuffer
  int download(const Tile &t, int k, rtc::V3 *fb) {
    const size_t pitch = (size_t)W * sizeof(rtc::V3);
    HK(hipMemcpy2DAsync(fb + (size_t)t.y0 * W + t.x0, pitch, dfb + ((size_t)t.y0 * W + t.x0) * 3, pitch,
                        (size_t)(t.x1 - t.x0) * sizeof(rtc::V3), (size_t)(t.y1 - t.y0), hipMemcpyDeviceToHost,
                        st[(size_t)k]));
    HK(hipStreamSynchronize(st[(size_t)k]));
    return 0;
  }
  int sync_all() {
    for (hipStream_t s : st) HK(hipStreamSynchronize(s));
    return 0;
  }
  ~Gpu() {
    for (rt_ctx *x : ctx) rt_destroy(x);
    for (hipStream_t s : st) (void)hipStreamDestroy(s);
    if (dfb) (void)hipFree(dfb);
  }
};

// CPU workers over a list of tiles, each taking the next unclaimed one
// (process_tile_cpu per tile, main_hybrid.cpp:162-173 / :571-581).
void cpu_workers(const rtc::CpuTracer &cpu, std::vector<Tile *> &list, int n, const Opts &o, rtc::V3 *fb) {
  std::atomic<size_t> next{0};
  auto work = [&] {
    for (size_t i; (i = next.fetch_add(1)) < list.size();) {
      Tile *t = list[i];
      cpu.render_tile(t->x0, t->y0, t->x1, t->y1, o.width, o.height, o.depth, fb);
      t->done = true;
    }
  };
  std::vector<std::thread> pool;
  for (int i = 0; i < n; ++i) pool.emplace_back(work);
  for (auto &th : pool) th.join();
}

int render_static(const Opts &o, const rtc::CpuTracer &cpu, Gpu &gpu, std::vector<Tile> &tiles, rtc::V3 *fb) {
  std::vector<Tile *> cpu_q, gpu_q;
  for (Tile &t : tiles) (t.gpu ? gpu_q : cpu_q).push_back(&t);
  int rc = 0;
  // the CPU section and the GPU section run concurrently (main_hybrid.cpp:410-475)
  std::thread cpu_side([&] { cpu_workers(cpu, cpu_q, o.threads, o, fb); });
  if (!o.pipeline) {
    for (Tile *t : gpu_q) {
      int k;
      if ((rc = gpu.launch(*t, k)) || (rc = gpu.download(*t, k, fb))) break;
      t->done = true;
    }
    if (!rc) rc = gpu.sync_all();
  } else {
    // every GPU tile launched -- here all in one launch (rt_render_tiles) --
    // then one download of the whole device framebuffer and a copy of the GPU
    // tiles' pixels (main_hybrid.cpp:535-600)
    if (!gpu_q.empty()) {
      int k;
      rc = gpu.launch_batch(gpu_q, k);
      if (!rc)
        for (Tile *t : gpu_q) t->done = true;
    }
    std::vector<rtc::V3> all;
    if (!rc && !(rc = gpu.sync_all())) {
      all.resize((size_t)o.width * o.height);
      if (hipMemcpy(all.data(), gpu.dfb, all.size() * sizeof(rtc::V3), hipMemcpyDeviceToHost) != hipSuccess) rc = 1;
    }
    cpu_side.join();
    if (!rc)
      for (Tile *t : gpu_q)
        for (int y = t->y0; y < t->y1; ++y)
          std::memcpy(fb + (size_t)y * o.width + t->x0, all.data() + (size_t)y * o.width + t->x0,
                      (size_t)(t->x1 - t->x0) * sizeof(rtc::V3));
    return rc;
  }
  cpu_side.join();
  return rc;
}

// --dynamic: one deque of tiles, costliest first; the GPU takes batches from
// the front, the CPU workers single tiles from the back.
int render_dynamic(const Opts &o, const rtc::CpuTracer &cpu, Gpu &gpu, std::vector<Tile> &tiles, rtc::V3 *fb) {
  std::vector<Tile *> order;
  for (Tile &t : tiles) order.push_back(&t);
  std::stable_sort(order.begin(), order.end(), [](const Tile *a, const Tile *b) { return a->cost > b->cost; });
  std::mutex mu;
  size_t front = 0, back = order.size();
  auto cpu_work = [&] {
    for (;;) {
      Tile *t;
      {
        std::lock_guard<std::mutex> l(mu);
        if (front >= back) return;
        t = order[--back];
      }
      t->gpu = false;
      cpu.render_tile(t->x0, t->y0, t->x1, t->y1, o.width, o.height, o.depth, fb);
      t->done = true;
    }
  };
  std::vector<std::thread> pool;
  for (int i = 0; i < o.threads; ++i) pool.emplace_back(cpu_work);
  int rc = 0;
  // the GPU takes a quarter of what is left per batch (at least 8 tiles): few
  // launches while the deque is long, small ones near the end
  const size_t min_batch = 8;
  for (;;) {
    size_t b, e;
    {
      std::lock_guard<std::mutex> l(mu);
      b = front;
      e = std::min(back, front + std::max(min_batch, (back - front) / 4));
      front = e;
    }
    if (b >= e) break;
    std::vector<Tile *> mine(order.begin() + (long)b, order.begin() + (long)e);
    int k = 0;
    for (Tile *t : mine) t->gpu = true;
    rc = gpu.launch_batch(mine, k);  // the batch in one launch, then its tiles' rows
    for (size_t i = 0; i < mine.size() && !rc; ++i) {
      rc = gpu.download(*mine[i], k, fb);
      mine[i]->done = true;
    }
    if (rc) break;
  }
  for (auto &th : pool) th.join();
  if (!rc) rc = gpu.sync_all();
  return rc;
}

}  // namespace

int main(int argc, char **argv) {
  Opts o;
  bool tile_set = false, threads_set = false;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto num = [&](int &dst) {
      if (i + 1 < argc) dst = std::atoi(argv[++i]);
    };
    if (a == "--pipeline" || a == "-p") o.pipeline = true;
    else if (a == "--tile-size" || a == "-t") { num(o.tile); tile_set = true; }
    else if (a == "--output" || a == "-o") { if (i + 1 < argc) o.out = argv[++i]; }
    else if (a == "--help" || a == "-h") return usage(argv[0]);
    else if (a == "--width") num(o.width);
    else if (a == "--height") num(o.height);
    else if (a == "--depth") num(o.depth);
    else if (a == "--threads") { num(o.threads); threads_set = true; }
    else if (a == "--cpu-threshold") num(o.threshold);
    else if (a == "--device") num(o.device);
    else if (a == "--streams") num(o.streams);
    else if (a == "--dynamic") o.dynamic = true;
    else o.scene = a;  // main_hybrid.cpp:751-753
  }
  (void)tile_set;
  if (o.width < 1 || o.height < 1 || o.tile < 1 || o.streams < 1) {
    std::fprintf(stderr, "invalid size, tile size or stream count\n");
    return 2;
  }
  if (threads_set && o.threads < 1) {  // no CPU worker would render the CPU tiles
    std::fprintf(stderr, "--threads must be at least 1\n");
    return 2;
  }
  if (o.threads < 0) {  // OMP_NUM_THREADS (the reference's CPU section is OpenMP), else the cores but one
    const char *omp = std::getenv("OMP_NUM_THREADS");
    o.threads = omp && std::atoi(omp) > 0 ? std::atoi(omp) : (int)std::thread::hardware_concurrency() - 1;
    o.threads = std::max(1, o.threads);
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {  // main_hybrid.cpp:755-761
    std::fprintf(stderr, "No HIP devices found. Cannot run hybrid version.\n");
    return 1;
  }
  hipDeviceProp_t props;
  HK(hipGetDeviceProperties(&props, o.device));
  std::printf("Using GPU: %s\n", props.name[0] ? props.name : props.gcnArchName);
  std::printf("Tile size: %dx%d\n", o.tile, o.tile);
  std::printf("Loading scene from: %s\n", o.scene.c_str());
  rt_scene sc;
  if (rt_scene_load(o.scene.c_str(), &sc, 1) != RT_OK) {
    std::fprintf(stderr, "terminate called after throwing an instance of 'std::runtime_error'\n"
                         "  what():  Could not open scene file: %s\n", o.scene.c_str());
    return 134 - 128;  // the reference aborts on the uncaught exception
  }
  rt_camera cam;
  rt_camera_from_scene(&sc, &cam);  // Camera(lookfrom, lookat, vfov), main_hybrid.cpp:773-781
  const int W = o.width, H = o.height;
  std::vector<rtc::V3> fb((size_t)W * H, rtc::V3{0, 0, 0});

  rtc::CpuTracer cpu(sc, cam);
  Gpu gpu;
  int rc = gpu.open(o, sc, cam);
  if (!rc) {
    std::printf(o.pipeline ? "Hybrid Pipeline Rendering...\n" : "Hybrid Rendering...\n");
    const int ts = o.pipeline ? 64 : o.tile;  // render_hybrid_pipeline gets the default tile size (:790)
    std::vector<Tile> tiles;
    for (int y = 0; y < H; y += ts)
      for (int x = 0; x < W; x += ts) tiles.push_back(Tile{x, y, std::min(x + ts, W), std::min(y + ts, H), 0, true, false});
    std::printf("Created %zu tiles of size %dx%d\n", tiles.size(), ts, ts);
    for (Tile &t : tiles) t.cost = cpu.tile_complexity(t.x0, t.y0, t.x1, t.y1, W, H);
    const int thr = o.threshold != INT_MIN ? o.threshold : (o.pipeline ? 9 : 7);  // :386 / :516
    size_t ncpu = 0;
    for (Tile &t : tiles) {
      t.gpu = !(t.cost > thr);
      ncpu += t.gpu ? 0 : 1;
    }
    if (!o.dynamic)
      std::printf("Distribution: %zu tiles to CPU, %zu tiles to GPU\n", ncpu, tiles.size() - ncpu);
    std::fflush(stdout);
    const auto t0 = std::chrono::high_resolution_clock::now();
    rc = o.dynamic ? render_dynamic(o, cpu, gpu, tiles, fb.data()) : render_static(o, cpu, gpu, tiles, fb.data());
    const auto t1 = std::chrono::high_resolution_clock::now();
    if (!rc) {
      if (o.dynamic) {
        size_t on_cpu = 0;
        for (const Tile &t : tiles) on_cpu += t.gpu ? 0 : 1;
        std::printf("Distribution: %zu tiles to CPU, %zu tiles to GPU\n", on_cpu, tiles.size() - on_cpu);
      }
      std::printf("Hybrid rendering time: %g seconds\n", std::chrono::duration<double>(t1 - t0).count());
      size_t missing = 0;
      for (const Tile &t : tiles) missing += t.done ? 0 : 1;
      if (missing) std::fprintf(stderr, "Warning: %zu tiles not processed!\n", missing);  // :478-486
    }
  }
  if (!rc) {
    // write_ppm (main_hybrid.cpp:47-75 = main.cpp:69-91): rows j = H-1 .. 0
    std::vector<uint8_t> rgb((size_t)W * H * 3);
    size_t neg = 0;
    for (int j = H - 1, k = 0; j >= 0; --j)
      for (int i = 0; i < W; ++i) {
        const rtc::V3 c = fb[(size_t)j * W + i];
        for (double ch : {c.x, c.y, c.z}) {
          const int q = int(255.99 * std::min(1.0, ch));
          neg += q < 0 ? 1 : 0;
          rgb[(size_t)k++] = (uint8_t)(q < 0 ? 0 : q);
        }
      }
    if (neg) std::fprintf(stderr, "warning: %zu channels quantised below 0 were stored as 0\n", neg);
    if (rt_write_ppm(o.out.c_str(), rgb.data(), W, H, 0) != RT_OK) {
      std::fprintf(stderr, "Error: Could not open file %s\n", o.out.c_str());
      rc = 1;
    } else {
      std::printf("Image written to %s\n", o.out.c_str());
    }
  }
  rt_scene_free(&sc);
  return rc;
}
