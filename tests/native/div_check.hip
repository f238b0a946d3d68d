// div_check.hip -- GPU check that rtk::div3 (the shared-reciprocal fast path
// of normalized(), rt_device.h) is bit-identical to three IEEE divisions as
// the compiler lowers them, over random and edge-case operands.  Built by
// tests/native/Makefile into libdivcheck.so; driven by tests/test_gpu_divcheck.py.
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

// One operand triple per (thread, kind): kind 0 = normalize a random scene
// vector (b = |a|, the renderer's use), 1 = normalize a near-unit vector,
// 2 = random signs/exponents over the whole double range (b positive),
// 3 = edge values (zeros, subnormals, infinities, NaN, guard boundaries).
__device__ void operands(uint64_t seed, uint64_t i, int kind, rtk::D3 &a, double &b) {
  const uint64_t z0 = mix(seed ^ (i * 4 + kind)), z1 = mix(z0), z2 = mix(z1), z3 = mix(z2);
  if (kind == 0 || kind == 1) {
    const double s = kind == 0 ? __builtin_ldexp(1.0, (int)(z3 % 64) - 32) : 1.0;
    a = rtk::mk((unit(z0) - 0.5) * s, (unit(z1) - 0.5) * s, (unit(z2) - 0.5) * s);
    if (kind == 1) a = rtk::normalized(a);  // |a| within a few ulp of 1 (the shadow direction case)
    if ((z3 >> 20) % 16 == 0) a.y = 0.0;
    if ((z3 >> 24) % 32 == 0) a.x = -0.0;
    b = rtk::length(a);
    return;
  }
  if (kind == 2) {
    auto rnd = [](uint64_t z) {
      const int e = (int)(z % 2100) - 1075;
      return __builtin_copysign(__builtin_ldexp(1.0 + unit(mix(z)), e), (z >> 63) ? -1.0 : 1.0);
    };
    a = rtk::mk(rnd(z0), rnd(z1), rnd(z2));
    b = __builtin_fabs(rnd(z3));
    return;
  }
  const double edge[] = {0.0, -0.0, 0x1p-1074, -0x1p-1070, 0x1p-1022, 0x1p-601, 0x1p-600, -0x1p-600, 0x1p-599,
                         0x1p-300, 0x1p-299, 0x1p300, 0x1p301, 0x1p399, 0x1p400, 0x1p401, 1.0, -1.0,
                         1.0 + 0x1p-52, 1.0 - 0x1p-53, __builtin_inf(), -__builtin_inf(), __builtin_nan(""),
                         3.0, 0.1, 1e300, 1e-300, 2.5e-200};
  const int ne = sizeof(edge) / sizeof(edge[0]);
  a = rtk::mk(edge[z0 % ne], edge[z1 % ne], edge[z2 % ne]);
  b = __builtin_fabs(edge[z3 % ne]) * ((z3 >> 40) % 3 == 0 ? (1.0 + unit(z2)) : 1.0);
}

__device__ bool same(double x, double y) {
  return __double_as_longlong(x) == __double_as_longlong(y) || (x != x && y != y);
}

__global__ void check(uint64_t seed, uint64_t n, unsigned long long *out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (int kind = 0; kind < 4; ++kind) {
    rtk::D3 a;
    double b;
    operands(seed, i, kind, a, b);
    const rtk::D3 f = rtk::div3(a, b);
    volatile double vb = b;  // keep the reference divisions independent of div3's code
    const double bb = vb;
    const rtk::D3 r = rtk::mk(a.x / bb, a.y / bb, a.z / bb);
    const bool ok = same(f.x, r.x) && same(f.y, r.y) && same(f.z, r.z);
    const bool fast = b >= 0x1p-300 && b <= 0x1p300 && rtk::div_num_ok(a.x) && rtk::div_num_ok(a.y) &&
                      rtk::div_num_ok(a.z);
    atomicAdd(&out[kind * 3 + 0], 1ull);
    if (fast) atomicAdd(&out[kind * 3 + 1], 1ull);
    if (!ok) {
      atomicAdd(&out[kind * 3 + 2], 1ull);
      out[12] = __double_as_longlong(a.x);
      out[13] = __double_as_longlong(b);
    }
  }
}

}  // namespace

// counts[14]: per kind {tested, fast path, mismatches}, then the last
// mismatching (a.x, b) bit patterns.  Returns 0 on success, else a hipError_t.
extern "C" int divcheck_run(unsigned long long seed, unsigned long long n, unsigned long long *counts) {
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
