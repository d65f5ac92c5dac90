// rocprofv3 exit-crash control: one HIP kernel, no libfisdf, no torch.
// Built two ways by run.sh: a plain executable (control) and a shared library (libcontrol.so)
// that ctl.py drives through ctypes, so the three controls separate "any HIP program under
// rocprofv3" from "a Python process" and from "torch's bundled HIP runtime".
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__global__ void axpy(double* y, const double* x, double a, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] += a * x[i];
}

// D: the same work plus one cooperative launch (hipLaunchCooperativeKernel), the launch mode
// of libfisdf's selection kernels
__global__ void coop_touch(double* y, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] += 1.0;
}

extern "C" int control_coop(int n) {
  double* y = nullptr;
  if (hipMalloc(&y, sizeof(double) * n) != hipSuccess) return 1;
  if (hipMemset(y, 0, sizeof(double) * n) != hipSuccess) return 1;
  void* args[] = {(void*)&y, (void*)&n};
  if (hipLaunchCooperativeKernel((const void*)coop_touch, dim3(64), dim3(256), args, 0, 0) != hipSuccess)
    return 3;
  double h = -1.0;
  if (hipMemcpy(&h, y, sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  if (hipFree(y) != hipSuccess) return 1;
  return h == 1.0 ? 0 : 2;
}

extern "C" int control_run(int n) {
  double *x = nullptr, *y = nullptr;
  if (hipMalloc(&x, sizeof(double) * n) != hipSuccess) return 1;
  if (hipMalloc(&y, sizeof(double) * n) != hipSuccess) return 1;
  hipMemset(x, 0, sizeof(double) * n);
  hipMemset(y, 0, sizeof(double) * n);
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(axpy, dim3((n + 255) / 256), dim3(256), 0, 0, y, x, 2.0, n);
  double h = -1.0;
  hipMemcpy(&h, y, sizeof(double), hipMemcpyDeviceToHost);
  hipFree(x);
  hipFree(y);
  return h == 0.0 ? 0 : 2;
}

#ifdef CONTROL_MAIN
int main(int argc, char** argv) {
  int rc = control_run(1 << 20);
  printf("control_run rc=%d\n", rc);
  if (argc > 2) {  // D: one cooperative launch too
    rc = control_coop(1 << 14);
    printf("control_coop rc=%d\n", rc);
  }
  if (argc > 1) {  // the address map, to symbolize a crash in the exit handlers
    FILE* src = fopen("/proc/self/maps", "r");
    FILE* dst = fopen(argv[1], "w");
    char buf[4096];
    size_t k;
    while (src && dst && (k = fread(buf, 1, sizeof(buf), src)) > 0) fwrite(buf, 1, k, dst);
    if (src) fclose(src);
    if (dst) fclose(dst);
  }
  return rc;
}
#endif
