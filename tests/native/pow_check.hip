// GPU-side check of the specular pow (tests/test_gpu_powcheck.py): for host-given
// (x, n) pairs, writes ocml's pow(x, n) and rtk::int_pow(x, n) (rt_device.h) so
// the test can compare both with the host's glibc pow -- the reference's.
#include <hip/hip_runtime.h>

#include "../../cs420-ray-tracer_amd/csrc/rt_device.h"

__global__ void pow_kernel(const double *x, const int *n, double *ocml, double *dd, long long count) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  ocml[i] = pow(x[i], (double)n[i]);
  int k = 0;
  dd[i] = rtk::int_pow_ok(x[i], (double)n[i], k) ? rtk::int_pow(x[i], k) : -1.0;
}

extern "C" int powcheck_run(const double *hx, const int *hn, double *hocml, double *hdd, long long count) {
  double *x = nullptr, *o = nullptr, *d = nullptr;
  int *n = nullptr;
  const size_t bd = (size_t)count * sizeof(double), bi = (size_t)count * sizeof(int);
  if (hipMalloc(&x, bd) != hipSuccess || hipMalloc(&o, bd) != hipSuccess || hipMalloc(&d, bd) != hipSuccess ||
      hipMalloc(&n, bi) != hipSuccess)
    return 1;
  int rc = 0;
  if (hipMemcpy(x, hx, bd, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(n, hn, bi, hipMemcpyHostToDevice) != hipSuccess)
    rc = 2;
  if (!rc) {
    hipLaunchKernelGGL(pow_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, 0, x, n, o, d, count);
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(hocml, o, bd, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(hdd, d, bd, hipMemcpyDeviceToHost) != hipSuccess)
      rc = 3;
  }
  (void)hipFree(x);
  (void)hipFree(o);
  (void)hipFree(d);
  (void)hipFree(n);
  return rc;
}
