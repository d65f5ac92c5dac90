#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ __launch_bounds__(256) void p16(int iters, double* out) {
  f64x4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f64x4{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.0) out[0] = s;
}
template <int NACC>
__global__ __launch_bounds__(256) void p4(int iters, double* out) {
  double acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = 0;
  double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i];
  if (s == 12345.0) out[0] = s;
}
template <int NACC>
__global__ __launch_bounds__(256) void pv(int iters, double* out) {
  double acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = threadIdx.x;
  double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = fma(a, acc[i], b);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i];
  if (s == 12345.0) out[0] = s;
}
int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  int ncu = p.multiProcessorCount;
  double* out; hipMalloc(&out, 8);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  float ms;
  for (int bpc : {1, 2, 4}) {
    int blocks = ncu * bpc, iters = 2000;
    p16<8><<<blocks, 256>>>(10, out);
    hipEventRecord(a); p16<8><<<blocks, 256>>>(iters, out); hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("16x16x4 f64 blocks/CU %d: %.2f TF/s\n", bpc, 2048.0 * 8 * iters * blocks * 4 / ms / 1e9);
    p4<16><<<blocks, 256>>>(10, out);
    hipEventRecord(a); p4<16><<<blocks, 256>>>(iters, out); hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("4x4x4 f64 (4 blocks) blocks/CU %d: %.2f TF/s\n", bpc, 512.0 * 16 * iters * blocks * 4 / ms / 1e9);
    pv<16><<<blocks, 256>>>(10, out);
    hipEventRecord(a); pv<16><<<blocks, 256>>>(iters, out); hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("VALU fma f64 blocks/CU %d: %.2f TF/s\n", bpc, 2.0 * 16 * iters * blocks * 256 / ms / 1e9);
  }
  return 0;
}
