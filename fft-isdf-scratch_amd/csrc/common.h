// fisdf — MI355X-native FFT-ISDF kernels: shared device/host helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <set>
#include <string>
#include <tuple>

namespace fisdf {

typedef double2 cplx;  // interleaved complex128 (matches NumPy complex128)
typedef __attribute__((ext_vector_type(4))) double f64x4;

// ---- error plumbing (C-ABI returns 0 / negative code, message via fisdf_last_error)
void set_error(const std::string& msg);

#define FISDF_HIP(call)                                                              \
  do {                                                                               \
    hipError_t _e = (call);                                                          \
    if (_e != hipSuccess) {                                                          \
      (void)hipGetLastError(); /* reported here: do not leave it for the next caller */ \
      ::fisdf::set_error(std::string("HIP error '") + hipGetErrorString(_e) +        \
                         "' at " __FILE__ ":" + std::to_string(__LINE__) + " in " #call); \
      return -2;                                                                     \
    }                                                                                \
  } while (0)

#define FISDF_CHECK(cond, msg)                                                       \
  do {                                                                               \
    if (!(cond)) {                                                                   \
      ::fisdf::set_error(std::string("fisdf: ") + (msg) + " [" #cond "] at " __FILE__ ":" + \
                         std::to_string(__LINE__));                                  \
      return -1;                                                                     \
    }                                                                                \
  } while (0)

#define FISDF_TRY(call)        \
  do {                         \
    int _r = (call);           \
    if (_r != 0) return _r;    \
  } while (0)

// ---- hipFuncAttributeMaxDynamicSharedMemorySize, set once per (kernel, device, size): safe from
// the rank threads of a fisdf_group (several devices, concurrent first calls)
inline int func_max_lds(const void* fn, int bytes) {
  static std::mutex m;
  static std::set<std::tuple<const void*, int, int>> done;
  int dev = 0;
  FISDF_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(m);
  if (done.count({fn, dev, bytes})) return 0;
  FISDF_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  done.insert({fn, dev, bytes});
  return 0;
}

// ---- kernel-exact stage timing: when set, the next zgemm()/herk() call's kernels record their
// execution span {first workgroup start, last wave end} (s_memrealtime, 100 MHz ticks) into
// `span` — the kernels' own time, what rocprofv3's kernel trace reports, rather than the stream
// positions around them (which, beside other fit lanes, also count the wait for free CUs); the
// call clears it.  Host-thread local (one context per thread).
struct LaunchEvents {
  unsigned long long* span = nullptr;
};
LaunchEvents& launch_events();

// record a kernel's execution span: span[0] = min start, span[1] = ~(max end) (both kept as
// minima so one all-ones fill initialises a slot); span may be null
__device__ __forceinline__ void span_begin(unsigned long long* span) {
  if (span && threadIdx.x == 0) atomicMin(span, (unsigned long long)__builtin_amdgcn_s_memrealtime());
}
__device__ __forceinline__ void span_end(unsigned long long* span) {
  if (span && (threadIdx.x & 63) == 0)
    atomicMin(span + 1, ~(unsigned long long)__builtin_amdgcn_s_memrealtime());
}

// ---- complex helpers (device + host)
__host__ __device__ inline cplx cmk(double r, double i) { cplx c; c.x = r; c.y = i; return c; }
__host__ __device__ inline cplx cadd(cplx a, cplx b) { return cmk(a.x + b.x, a.y + b.y); }
__host__ __device__ inline cplx csub(cplx a, cplx b) { return cmk(a.x - b.x, a.y - b.y); }
__host__ __device__ inline cplx cmul(cplx a, cplx b) { return cmk(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
__host__ __device__ inline cplx cconj(cplx a) { return cmk(a.x, -a.y); }
__host__ __device__ inline cplx cscale(cplx a, double s) { return cmk(a.x * s, a.y * s); }

// ---- GEMM op codes: bit0 = transpose, bit1 = conjugate
enum Op { OP_N = 0, OP_T = 1, OP_R = 2 /*conj only*/, OP_C = 3 /*conj-transpose*/ };

// ---- kernels (launchers return 0 or negative; all asynchronous on `stream`)
// C[b] = alpha * op(A[b]) * op(B[b]) + beta * C[b]; lda/ldb/ldc in complex elements,
// strides sA/sB/sC per batch in complex elements. ksplit>1 uses `work` (ksplit*M*N cplx).
// epilogues: EPI_STREAM: C = alpha acc (beta = 0) with non-temporal stores (a large output
// read back only much later, e.g. the y build's fx blocks)
// EPI_CSQUARE: C = (alpha acc)^2 elementwise (beta = 0), max |Im(alpha acc)| recorded in *mon
// EPI_REAL: C = Re(alpha acc) written as REAL doubles (C is a double*, ldc in doubles; batch 1);
// EPI_WSRHO: C = aux Re(alpha acc) + 0i with aux real (a double* passed as `work`, row stride
// ldaux doubles); both record max |Im(alpha acc)| in *mon (nullable)
enum Epi { EPI_NONE = 0, EPI_STREAM = 2, EPI_CSQUARE = 4, EPI_REAL = 5, EPI_WSRHO = 6 };
// arithmetic modes (MFMA work skipped): GEMM_A_REAL: Im(op(A)) is taken as zero (2 of the 4
// real MFMAs per complex block); GEMM_RE_ONLY: only Re(C) is formed (Im(C) written as 0).
// Supported for (N,N), (C,N) and the HERK; other op pairs require mode 0.
// GEMM_A_LOWER: op(A) = A (OP_N) is lower triangular: each M-tile stops its K loop at the
// tile's last row (the zero upper part is never read or multiplied).
// GEMM_A_UPPER: op(A) = A^H (OP_C) is upper triangular (A lower): each M-tile starts its K loop
// at its own first row (no split-K)
enum GemmMode { GEMM_FULL = 0, GEMM_A_REAL = 1, GEMM_RE_ONLY = 2, GEMM_A_LOWER = 4, GEMM_A_UPPER = 8 };
int zgemm(hipStream_t s, int opA, int opB, int M, int N, int K, cplx alpha,
          const cplx* A, long lda, long sA, const cplx* B, long ldb, long sB, cplx beta,
          cplx* C, long ldc, long sC, int batch, int ksplit = 1, cplx* work = nullptr,
          int epi = EPI_NONE, unsigned long long* mon = nullptr, int mode = GEMM_FULL,
          long ldaux = 0);

// the 64 x 128-tile kernel for big single NN products (zgemm_wide.hip); zgemm() routes there
bool wide_gemm_enabled();
bool zgemm_wide_applies(int opA, int opB, int M, int N, int K, long lda, long ldb, int batch,
                        int ksplit, int epi,
                        int mode);
int zgemm_nn_wide(hipStream_t s, int M, int N, int K, cplx alpha, const cplx* A, long lda,
                  const cplx* B, long ldb, cplx beta, cplx* C, long ldc, int mode,
                  unsigned long long* span);

// C = alpha A A^H (Hermitian rank-K update; lower tiles computed, upper mirrored)
int herk(hipStream_t s, int n, int K, double alpha, const cplx* A, long lda, cplx* C, long ldc,
         int ksplit = 1, cplx* work = nullptr, int mode = GEMM_FULL);

// C[b] = alpha A[b] A[b]^H + beta C[b] (lower tiles + mirror), batched, no split-K
int herk_batched(hipStream_t s, int n, int K, double alpha, const cplx* A, long lda, long sA,
                 double beta, cplx* C, long ldc, long sC, int batch);

// batched pivoted Cholesky of Hermitian PSD matrices (fftisdf.py:381-382, A4 factorisation)
// trail: pchol_trail_elems(n, batch) complex elements (the blocked path's trailing copy)
int pchol(hipStream_t s, const cplx* A, long lda, long sA, int n, int batch, int rmax,
          double tol_rel, double tol_abs, cplx* L /*batch, n, rmax*/, int* piv /*batch, rmax*/,
          int* rank /*batch, device*/, double* d /*batch,n*/, int* flags /*batch*/,
          double* work /*batch*(1+rmax)*/, cplx* trail);
size_t pchol_trail_elems(int n, int batch);

// unpivoted blocked Cholesky (full-rank fast path); see pchol.hip
int chol_unpivoted(hipStream_t s, cplx* W, int n, int batch, double tol_rel, int* piv, int* rank,
                   int* fail, cplx* work);
// selection pivots from the real Gram Re(X2)^2*scale (cooperative kernel, else blocked, real;
// n <= 4096): *handled=false otherwise.  work: n*n + 17*n + 1 doubles; piv (rmax), rank (1),
// flags (1) device.  When the cooperative kernel ran (allow_coop), *coop_err is the device address
// of its error flag: nonzero after the stream completes = a stalled step, redo with
// allow_coop = false.
// progress (device int, nullable): the cooperative kernel publishes the count of final pivots
// every kSelPublish pivots and kSelDone at its end, with piv[] written agent-coherent, so work
// on other streams can start on the first pivots while the selection runs (the streamed y
// build, api.hip); *publishes tells whether the kernel that ran does so (the other paths
// publish nothing: their consumers see only the kSelDone the caller writes after the kernel)
// whether the selection kernels go through hipLaunchCooperativeKernel (FISDF_COOP_LAUNCH=0/1;
// default: cooperative on HIP runtimes >= 7.2, else a plain launch after the occupancy check,
// pchol.hip coop_launch_enabled / launch_coresident)
bool coop_launch_enabled();
constexpr int kSelPublish = 16;
constexpr int kSelDone = 1 << 30;
int pchol_select_real(hipStream_t s, const cplx* X2, double scale, int n, int rmax, double tol,
                      int* piv, int* rank, double* work, int* flags, bool* handled,
                      bool allow_coop, const int** coop_err, int* progress = nullptr,
                      bool* publishes = nullptr);

// Where plane i0 of input row r lives when the rows arrive in grid slices (the all-to-all
// pieces of a k-sharded build): in + base + r * ld, one entry per plane (device table)
struct PlaneRef {
  long base;
  long ld;
};

// 3-D FFT (unnormalised forward, numpy.fft.fftn sign) over `rows` rows of length n0*n1*n2.
// in-row gather `rowidx` (may be null), pre-multiply by exp(-i (f.kd)) where f are the
// fftfreq fractions (if kd != null), post-multiply by weight[G] (if weight != null).
// planes (device, n0 entries, may be null): sliced input — plane i0 of row r at
// in + planes[i0].base + r * planes[i0].ld (in_ld unused); needs fft3d_reads_slices(mesh)
// herm (3 ints or null): the input is real up to the phase, so its transform pairs up as
// out(j') = conj(out(j)) with j' = -j - herm (mod mesh) (a self-conjugate q, m = 2 k_q); only the
// prefix planes j0 < half_prefix_planes(n0, herm[0]) of out are written (the half-grid fit reads
// nothing else) and the register path moves half of the intermediate planes.
// in_real: the input rows are doubles (in cast to double*, same in_ld and plane offsets)
int fft3d(hipStream_t s, const cplx* in, long in_ld, const int* rowidx, cplx* out, long out_ld,
          int rows, int n0, int n1, int n2, const double* kd /*3 or null*/,
          const double* weight /*ngrid or null*/, cplx* work, const PlaneRef* planes = nullptr,
          const int* herm = nullptr, bool in_real = false);
// whether fft3d takes sliced input for this mesh (its first pass is a per-plane kernel)
bool fft3d_reads_slices(int n0, int n1, int n2);
// whether fft3d takes real input (in_real: rows of doubles at the same strides) for this mesh
bool fft3d_reads_real(int n0, int n1, int n2);

}  // namespace fisdf
