// renorm_gpu_check.hip -- GPU check that rtk::renormalized (rt_device.h: the
// second normalisation's fast path) returns the bits of rtk::normalized (sqrt
// and three IEEE divisions as the compiler lowers them) on the device itself.
// Kinds: 0 = a random vector normalised once, then renormalised (the camera
// ray and shadow direction, ray.h:12); 1 = the reflection d - 2 (d.n) n of
// unit vectors (main.cpp:46); 2 = a unit vector scaled by 1 + k 2^-53,
// k in -8..8 (every length class and its neighbours); 3 = special
// components (zeros, subnormals, tiny, guard boundaries, NaN).  Built by
// tests/native/Makefile into librenormcheck.so; driven by
// tests/test_gpu_renorm.py.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../cs420-ray-tracer_amd/csrc/rt_device.h"

namespace {

__device__ uint64_t mix(uint64_t z) {  // splitmix64 finaliser
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ double unit(uint64_t z) { return (double)(z >> 11) * 0x1p-53; }

__device__ rtk::D3 operand(uint64_t seed, uint64_t i, int kind) {
  const uint64_t z0 = mix(seed ^ (i * 4 + kind)), z1 = mix(z0), z2 = mix(z1), z3 = mix(z2), z4 = mix(z3);
  const double s = __builtin_ldexp(1.0, (int)(z3 % 40) - 20);
  rtk::D3 v = rtk::mk((unit(z0) - 0.5) * s, (unit(z1) - 0.5) * s, (unit(z2) - 0.5) * s);
  if ((z4 >> 8) % 16 == 0) v.x = 0.0;
  if ((z4 >> 12) % 32 == 0) v.y = -0.0;
  const rtk::D3 d = rtk::normalized(v);
  if (kind == 0) return d;
  if (kind == 1) {
    const rtk::D3 n = rtk::normalized(rtk::mk(unit(z3) - 0.5, unit(z4) - 0.5, unit(mix(z4)) - 0.5));
    const double dn = rtk::dot(d, n);
    return rtk::sub(d, rtk::scale(rtk::scale(n, 2.0), dn));  // main.cpp:46 (reflect, vec3.h:31-33)
  }
  if (kind == 2) {
    const double f = 1.0 + (double)((int)(z4 % 17) - 8) * 0x1p-53;
    return rtk::mk(d.x * f, d.y * f, d.z * f);
  }
  const double edge[] = {0.0, -0.0, 0x1p-1074, -0x1p-1060, 0x1p-1022, 0x1p-960, 0x1p-959, -0x1p-959, 0x1p-958,
                         1e-300, 0x1.fffffffffffffp-1, 1.0, -1.0, 0.5, __builtin_nan("")};
  const int ne = sizeof(edge) / sizeof(edge[0]);
  rtk::D3 a = d;
  const int which = (int)(z4 % 3);
  const double e = edge[(z4 >> 4) % ne];
  if (which == 0) a.x = e;
  if (which == 1) a.y = e;
  if (which == 2) a.z = e;
  return a;
}

__device__ bool same(double x, double y) {
  return __double_as_longlong(x) == __double_as_longlong(y) || (x != x && y != y);
}

__global__ void check(uint64_t seed, uint64_t n, unsigned long long *out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (int kind = 0; kind < 4; ++kind) {
    const rtk::D3 a = operand(seed, i, kind);
    const rtk::D3 f = rtk::renormalized(a);
    volatile double vx = a.x, vy = a.y, vz = a.z;  // the reference computed apart from renormalized's code
    const rtk::D3 r = rtk::normalized(rtk::mk(vx, vy, vz));
    const double s = (a.x * a.x + a.y * a.y) + a.z * a.z, t = (s - 1.0) * 0x1p53;
    const bool fast = t >= -4.0 && t <= 6.0;
    const bool ok = same(f.x, r.x) && same(f.y, r.y) && same(f.z, r.z);
    atomicAdd(&out[kind * 3 + 0], 1ull);
    if (fast) atomicAdd(&out[kind * 3 + 1], 1ull);
    if (!ok) {
      atomicAdd(&out[kind * 3 + 2], 1ull);
      out[12] = __double_as_longlong(a.x);
      out[13] = __double_as_longlong(a.y);
    }
  }
}

}  // namespace

// counts[14]: per kind {tested, length class in the fast range, mismatches},
// then the last mismatching (a.x, a.y) bit patterns.  Returns 0 on success,
// else a hipError_t.
extern "C" int renormcheck_run(unsigned long long seed, unsigned long long n, unsigned long long *counts) {
  unsigned long long *d = nullptr;
  hipError_t e = hipMalloc(&d, 14 * sizeof(unsigned long long));
  if (e != hipSuccess) return (int)e;
  e = hipMemset(d, 0, 14 * sizeof(unsigned long long));
  if (e == hipSuccess) {
    const unsigned blocks = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(check, dim3(blocks), dim3(256), 0, 0, (uint64_t)seed, (uint64_t)n, d);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(counts, d, 14 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  return (int)e;
}
