// Microbenchmark: achievable v_mfma_f64_16x16x4_f64 rate on this GPU (no memory traffic).
// hipcc --offload-arch=gfx950 -O3 tools/mfma_peak.hip -o /tmp/mfma_peak && /tmp/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void peak(int iters, double* out) {
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
void run(int blocks_per_cu) {
  int ncu = 256;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  ncu = p.multiProcessorCount;
  int iters = 4000;
  int blocks = ncu * blocks_per_cu;
  double* out;
  hipMalloc(&out, 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  peak<NACC><<<blocks, 256>>>(10, out);
  hipEventRecord(a);
  peak<NACC><<<blocks, 256>>>(iters, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  double flop = 2048.0 * NACC * iters * (blocks * 4.0);
  printf("NACC=%d blocks/CU=%d CUs=%d clock(kHz)=%d: %.3f ms  %.2f TF/s\n", NACC, blocks_per_cu,
         ncu, p.clockRate, ms, flop / ms / 1e9);
  hipFree(out);
}

int main() {
  run<4>(1);
  run<8>(1);
  run<8>(2);
  run<16>(1);
  run<16>(3);
  return 0;
}
