// rt_host.cpp -- host half of librt_hip.so: scene text parser, camera basis,
// PPM writer, status strings.  No device code here.
//
// The parser keeps the reference loader's record grammar and its quirks
// (include/scene_loader.h:27-135): '#' comments (also after leading
// spaces/tabs), `sphere x y z r  R G B  metallic roughness shininess`,
// `light x y z R G B intensity`, `ambient R G B`, `camera px py pz lx ly lz fov`;
// last ambient/camera wins; malformed records are skipped with a warning;
// trailing tokens are ignored.  Numbers go through std::istream >> double, the
// same extractor the reference uses, so parsed doubles are identical.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>
#include <atomic>
#include <memory>
#include <thread>

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include "rt_hip.h"

namespace {

struct Grow {
  std::vector<rt_sphere> spheres;
  std::vector<rt_light> lights;
};

void set3(double *d, double x, double y, double z) {
  d[0] = x;
  d[1] = y;
  d[2] = z;
}

int parse_stream(std::istream &in, rt_scene *out, int verbose) {
  std::memset(out, 0, sizeof(*out));
  set3(out->cam_look_at, 0, 0, -1);  // CameraConfig() defaults, scene.h:22
  out->cam_fov = 60.0;
  Grow g;
  std::string line;
  int line_number = 0;
  while (std::getline(in, line)) {
    line_number++;
    if (line.empty() || line[0] == '#') continue;
    size_t start = line.find_first_not_of(" \t");
    if (start == std::string::npos) continue;
    if (line[start] == '#') continue;
    std::istringstream iss(line.substr(start));
    std::string type;
    iss >> type;
    double v[10];
    auto read = [&](int n) {
      for (int i = 0; i < n; i++)
        if (!(iss >> v[i])) return false;
      return true;
    };
    auto warn = [&](const char *what) {
      out->warnings++;
      if (verbose) std::cerr << "Warning: Invalid " << what << " at line " << line_number << ", skipping\n";
    };
    if (type == "sphere") {
      if (!read(10)) { warn("sphere"); continue; }
      rt_sphere s;
      set3(s.center, v[0], v[1], v[2]);
      s.radius = v[3];
      set3(s.color, v[4], v[5], v[6]);
      s.reflectivity = v[7];  // "metallic"; v[8] (roughness) is dropped as upstream
      s.shininess = v[9];
      g.spheres.push_back(s);
    } else if (type == "light") {
      if (!read(7)) { warn("light"); continue; }
      rt_light l;
      set3(l.position, v[0], v[1], v[2]);
      set3(l.color, v[3], v[4], v[5]);
      l.intensity = v[6];
      g.lights.push_back(l);
    } else if (type == "ambient") {
      if (!read(3)) { warn("ambient"); continue; }
      set3(out->ambient, v[0], v[1], v[2]);
    } else if (type == "camera") {
      if (!read(7)) { warn("camera"); continue; }
      set3(out->cam_position, v[0], v[1], v[2]);
      set3(out->cam_look_at, v[3], v[4], v[5]);
      out->cam_fov = v[6];
      out->has_camera = 1;
    } else {
      out->warnings++;
      if (verbose) std::cerr << "Warning: Unknown type '" << type << "' at line " << line_number << ", skipping\n";
    }
  }
  out->num_spheres = (int32_t)g.spheres.size();
  out->num_lights = (int32_t)g.lights.size();
  out->spheres = (rt_sphere *)std::malloc(sizeof(rt_sphere) * (g.spheres.size() + 1));
  out->lights = (rt_light *)std::malloc(sizeof(rt_light) * (g.lights.size() + 1));
  if (!out->spheres || !out->lights) return RT_ERR_OUT_OF_MEMORY;
  if (!g.spheres.empty()) std::memcpy(out->spheres, g.spheres.data(), sizeof(rt_sphere) * g.spheres.size());
  if (!g.lights.empty()) std::memcpy(out->lights, g.lights.data(), sizeof(rt_light) * g.lights.size());
  if (verbose)
    std::cout << "Loaded scene: " << out->num_spheres << " spheres, " << out->num_lights << " lights\n";
  return RT_OK;
}

// Vec3 algebra of include/vec3.h:13-29, used only for the per-frame camera basis.
struct V {
  double x, y, z;
};
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
V normalized(V a) {
  double len = std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
  return {a.x / len, a.y / len, a.z / len};
}
void put(double *d, V v) { set3(d, v.x, v.y, v.z); }

// Runs fn(k) for k in [0, nchunk) on up to nthr threads (the caller is one
// of them).  A thread that cannot be started (resource limits) leaves its
// share to the others; every started thread is joined on every path, so no
// exception leaves the C ABI and no joinable thread is destroyed.
template <typename F>
void run_chunks(size_t nthr, size_t nchunk, F &&fn) {
  std::atomic<size_t> next{0};
  auto worker = [&]() {
    for (size_t k; (k = next.fetch_add(1)) < nchunk;) fn(k);
  };
  std::vector<std::thread> th;
  for (size_t t = 1; t < nthr; t++) {
    try {
      th.emplace_back(worker);
    } catch (...) {
      break;  // the threads already started and this one do the rest
    }
  }
  worker();
  for (auto &t : th) t.join();
}

}  // namespace

extern "C" {

int rt_abi_version(void) { return RT_HIP_ABI_VERSION; }

int rt_rows_for_shard(int height, int band, int rank, int num_shards, rt_rows *out) {
  if (!out || height < 0 || band < 1 || num_shards < 1 || rank < 0 || rank >= num_shards) return RT_ERR_INVALID_ARG;
  const long long nb = ((long long)height + band - 1) / band;          // bands of the image
  const long long per = (nb + num_shards - 1) / num_shards;           // bands per rank
  if (per * band > 0x7fffffffLL) return RT_ERR_INVALID_ARG;
  *out = rt_rows{band, rank, num_shards, (int32_t)(per * band)};
  return RT_OK;
}

const char *rt_error_string(int status) {
  switch (status) {
    case RT_OK: return "ok";
    case RT_ERR_INVALID_ARG: return "invalid argument";
    case RT_ERR_NO_DEVICE: return "no HIP device";
    case RT_ERR_HIP: return "HIP runtime error";
    case RT_ERR_OUT_OF_MEMORY: return "out of memory";
    case RT_ERR_NO_SCENE: return "no scene uploaded";
    case RT_ERR_IO: return "I/O error";
    case RT_ERR_DEPTH: return "depth exceeds RT_MAX_DEPTH";
    case RT_ERR_CHECK: return "device index out of range (bounds-checked build)";
    default: return "unknown status";
  }
}

int rt_scene_parse(const char *text, rt_scene *out, int verbose) {
  if (!text || !out) return RT_ERR_INVALID_ARG;
  std::istringstream in{std::string(text)};
  return parse_stream(in, out, verbose);
}

int rt_scene_load(const char *path, rt_scene *out, int verbose) {
  if (!path || !out) return RT_ERR_INVALID_ARG;
  std::ifstream f(path);
  if (!f.is_open()) {  // the reference throws "Could not open scene file: ..." (scene_loader.h:33-35)
    std::memset(out, 0, sizeof(*out));
    if (verbose) std::cerr << "Could not open scene file: " << path << "\n";
    return RT_ERR_IO;
  }
  return parse_stream(f, out, verbose);
}

void rt_scene_free(rt_scene *scene) {
  if (!scene) return;
  std::free(scene->spheres);
  std::free(scene->lights);
  scene->spheres = nullptr;
  scene->lights = nullptr;
  scene->num_spheres = scene->num_lights = 0;
}

int rt_camera_from_scene(const rt_scene *s, rt_camera *c) {
  if (!s || !c) return RT_ERR_INVALID_ARG;
  V pos{s->cam_position[0], s->cam_position[1], s->cam_position[2]};
  V look{s->cam_look_at[0], s->cam_look_at[1], s->cam_look_at[2]};
  V fwd = normalized(sub(look, pos));        // camera.h:12
  V right = normalized(cross(fwd, {0, 1, 0}));  // camera.h:13
  V up = normalized(cross(right, fwd));      // camera.h:14
  put(c->position, pos);
  put(c->forward, fwd);
  put(c->right, right);
  put(c->up, up);
  c->scale = std::tan(s->cam_fov * 0.5 * M_PI / 180.0);  // camera.h:19 (glibc tan, host)
  return RT_OK;
}

// P3 text identical to write_ppm (src/main.cpp:69-91) -- "r g b\n" per pixel,
// top row first -- formatted from a 256-entry table, in parallel, straight into
// the file: a sizing pass gives every pixel range's offset, the file is sized
// once and mapped, and each range is formatted in place (no intermediate
// buffers, no copy through stdio; 1.85 s at 1080p upstream).  Where the file
// cannot be mapped (a pipe, a special file) the ranges are formatted into
// buffers and written in order.
int rt_write_ppm(const char *path, const uint8_t *rgb, int width, int height, int binary) {
  if (!path || !rgb || width < 0 || height < 0) return RT_ERR_INVALID_ARG;
  const size_t n = (size_t)width * (size_t)height;
  char hdr[64];
  const int hn = std::snprintf(hdr, sizeof hdr, "%s\n%d %d\n255\n", binary ? "P6" : "P3", width, height);
  if (binary) {
    FILE *f = std::fopen(path, "wb");
    if (!f) return RT_ERR_IO;
    int rc = std::fwrite(hdr, 1, (size_t)hn, f) == (size_t)hn ? RT_OK : RT_ERR_IO;
    if (rc == RT_OK && n && std::fwrite(rgb, 1, n * 3, f) != n * 3) rc = RT_ERR_IO;
    if (std::fclose(f) != 0) rc = RT_ERR_IO;
    return rc;
  }
  // "0".."255" and their lengths, built once (a function-local static: safe
  // when several threads write images at the same time)
  struct Tab {
    char s[256][4];
    unsigned char n[256];
    Tab() {
      for (int v = 0; v < 256; v++) n[v] = (unsigned char)std::snprintf(s[v], 4, "%d", v);
    }
  };
  static const Tab T;
  const unsigned hw = std::thread::hardware_concurrency();
  const size_t nthr = n < ((size_t)1 << 16) ? 1 : std::max<size_t>(1, std::min<size_t>(hw ? hw : 1, 16));
  const size_t nchunk = nthr == 1 ? 1 : nthr * 4;
  auto lo = [&](size_t k) { return n * k / nchunk; };
  // bytes of each pixel range: the three numbers' digits + 2 spaces + newline
  std::vector<size_t> off(nchunk + 1, 0);
  run_chunks(nthr, nchunk, [&](size_t k) {
    size_t b = 0;
    for (size_t i = 3 * lo(k), e = 3 * lo(k + 1); i < e; i++) b += T.n[rgb[i]];
    off[k + 1] = b + 3 * (lo(k + 1) - lo(k));
  });
  off[0] = (size_t)hn;
  for (size_t k = 0; k < nchunk; k++) off[k + 1] += off[k];
  const size_t total = off[nchunk];
  // range k formatted at o (exactly off[k + 1] - off[k] bytes): each number
  // as its 4-byte table slot (the next write overwrites the slot's tail), the
  // range's last pixel through a bounce buffer so that nothing lands past the
  // range (the next range may be another thread's)
  auto format = [&](size_t k, char *o) {
    auto pixel = [&](size_t p, char *w) {
      for (int c = 0; c < 3; c++) {
        const unsigned v = rgb[3 * p + c];
        std::memcpy(w, T.s[v], 4);
        w += T.n[v];
        *w++ = c == 2 ? '\n' : ' ';
      }
      return w;
    };
    const size_t p0 = lo(k), p1 = lo(k + 1);
    if (p1 == p0) return;
    for (size_t p = p0; p + 1 < p1; p++) o = pixel(p, o);
    char tail[16];
    std::memcpy(o, tail, (size_t)(pixel(p1 - 1, tail) - tail));
  };
  const int fd = ::open(path, O_RDWR | O_CREAT | O_TRUNC, 0666);
  if (fd < 0) return RT_ERR_IO;
  int rc = RT_OK;
  void *m = MAP_FAILED;
  if (::ftruncate(fd, (off_t)total) == 0) m = ::mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (m != MAP_FAILED) {
    char *base = static_cast<char *>(m);
    std::memcpy(base, hdr, (size_t)hn);
    run_chunks(nthr, nchunk, [&](size_t k) { format(k, base + off[k]); });
    if (::munmap(m, total) != 0) rc = RT_ERR_IO;
  } else {  // not mappable (nothing written yet: the file position is 0): format into buffers, write in order
    std::vector<std::unique_ptr<char[]>> bufs(nchunk);
    run_chunks(nthr, nchunk, [&](size_t k) {
      bufs[k].reset(new (std::nothrow) char[off[k + 1] - off[k]]);
      if (bufs[k]) format(k, bufs[k].get());
    });
    auto put = [&](const char *p, size_t len) {
      while (rc == RT_OK && len > 0) {
        const ssize_t w = ::write(fd, p, len);
        if (w <= 0) rc = RT_ERR_IO;
        else p += w, len -= (size_t)w;
      }
    };
    put(hdr, (size_t)hn);
    for (size_t k = 0; k < nchunk; k++) {
      if (!bufs[k]) rc = RT_ERR_IO;
      put(bufs[k].get(), off[k + 1] - off[k]);
    }
  }
  if (::close(fd) != 0) rc = RT_ERR_IO;
  return rc;
}

}  // extern "C"
