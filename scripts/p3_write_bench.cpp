// Write strategies for a 24 MB P3 file on the box's file systems (a builder's
// probe for rt_write_ppm, not a test): (a) pixel ranges formatted on N
// threads into buffers, written in order as they complete (fwrite), (b) the
// same with write(2), (c) everything formatted, then one write(2), (d)
// pwrite(2) of each range from its own thread, (e) mmap of the sized file.
//   g++ -O2 -std=c++17 -pthread p3_write_bench.cpp -o p3wb && ./p3wb DIR [threads]
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static char S[256][4];
static unsigned char L[256];
static double now() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
int main(int argc, char **argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const int nthr = argc > 2 ? std::atoi(argv[2]) : 16;
  for (int v = 0; v < 256; v++) L[v] = (unsigned char)std::snprintf(S[v], 4, "%d", v);
  const size_t n = 1920 * 1080;
  std::vector<unsigned char> rgb(n * 3);
  unsigned x = 12345;
  for (auto &c : rgb) c = (unsigned char)((x = x * 1103515245u + 12345u) >> 24 | 0x60);  // mostly 3-digit
  const size_t nchunk = (size_t)nthr * 4;
  auto lo = [&](size_t k) { return n * k / nchunk; };
  std::vector<size_t> off(nchunk + 1, 0);
  for (size_t k = 0; k < nchunk; k++) {
    size_t b = 0;
    for (size_t i = 3 * lo(k); i < 3 * lo(k + 1); i++) b += L[rgb[i]];
    off[k + 1] = off[k] + b + 3 * (lo(k + 1) - lo(k));
  }
  const size_t total = off[nchunk];
  auto fmt = [&](size_t k, char *o) {
    for (size_t p = lo(k); p < lo(k + 1); p++)
      for (int c = 0; c < 3; c++) {
        const unsigned v = rgb[3 * p + c];
        std::memcpy(o, S[v], 4);
        o += L[v];
        *o++ = c == 2 ? '\n' : ' ';
      }
  };
  auto par = [&](auto &&fn) {
    std::atomic<size_t> next{0};
    std::vector<std::thread> th;
    auto w = [&] { for (size_t k; (k = next++) < nchunk;) fn(k); };
    for (int t = 1; t < nthr; t++) th.emplace_back(w);
    w();
    for (auto &t : th) t.join();
  };
  const std::string path = dir + "/p3wb_test.ppm";
  for (int rep = 0; rep < 3; rep++) {
    // (a)/(b): ordered writes as ranges complete
    for (int use_fwrite = 1; use_fwrite >= 0; use_fwrite--) {
      double t0 = now();
      std::vector<char *> bufs(nchunk, nullptr);
      std::vector<std::atomic<int>> done(nchunk);
      for (auto &d : done) d = 0;
      std::atomic<size_t> next{0};
      std::vector<std::thread> th;
      auto w = [&] {
        for (size_t k; (k = next++) < nchunk;) {
          bufs[k] = (char *)std::malloc(off[k + 1] - off[k] + 4);
          fmt(k, bufs[k]);
          done[k].store(1, std::memory_order_release);
        }
      };
      for (int t = 0; t < nthr; t++) th.emplace_back(w);
      FILE *f = use_fwrite ? std::fopen(path.c_str(), "wb") : nullptr;
      int fd = use_fwrite ? -1 : ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0666);
      for (size_t k = 0; k < nchunk; k++) {
        while (!done[k].load(std::memory_order_acquire)) std::this_thread::yield();
        if (f) std::fwrite(bufs[k], 1, off[k + 1] - off[k], f);
        else if (::write(fd, bufs[k], off[k + 1] - off[k]) < 0) return 1;
        std::free(bufs[k]);
      }
      for (auto &t : th) t.join();
      if (f) std::fclose(f);
      else ::close(fd);
      std::printf("%s ordered %s: %.3f ms\n", dir.c_str(), use_fwrite ? "fwrite" : "write", now() - t0);
    }
    {  // (c) all formatted, one write
      double t0 = now();
      char *buf = (char *)std::malloc(total + 4);
      par([&](size_t k) { fmt(k, buf + off[k]); });
      double t1 = now();
      int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0666);
      if (::write(fd, buf, total) != (ssize_t)total) return 1;
      ::close(fd);
      std::free(buf);
      std::printf("%s one write: %.3f ms (format %.3f)\n", dir.c_str(), now() - t0, t1 - t0);
    }
    {  // (d) pwrite per range
      double t0 = now();
      int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0666);
      par([&](size_t k) {
        char *b = (char *)std::malloc(off[k + 1] - off[k] + 4);
        fmt(k, b);
        if (::pwrite(fd, b, off[k + 1] - off[k], (off_t)off[k]) < 0) std::abort();
        std::free(b);
      });
      ::close(fd);
      std::printf("%s pwrite: %.3f ms\n", dir.c_str(), now() - t0);
    }
    {  // (e) mmap
      double t0 = now();
      int fd = ::open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0666);
      if (::ftruncate(fd, (off_t)total) != 0) return 1;
      char *m = (char *)::mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      par([&](size_t k) {
        char tmp[64];
        (void)tmp;
        fmt(k, m + off[k]);  // (overrun into the next range: timing only)
      });
      ::munmap(m, total);
      ::close(fd);
      std::printf("%s mmap: %.3f ms\n", dir.c_str(), now() - t0);
    }
  }
  ::unlink(path.c_str());
  return 0;
}
