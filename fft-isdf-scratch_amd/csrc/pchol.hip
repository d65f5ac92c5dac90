// Batched greedy (full-pivot) Cholesky of Hermitian PSD matrices.
//
// Serves two call sites of the reference:
//  * interpolation-point selection: LAPACK dpstrf on the real parent-grid Gram x4
//    (fftisdf.py:381-384 via pyscf.lib.scipy_helper.pivoted_cholesky); only the first
//    nip = min(nao*c0, rank) pivots are produced, rank is detected by the same
//    relative tolerance LAPACK uses (tol <= 0 -> n*eps*max(diag)).
//  * the per-q factorisation of x4_q that replaces zgelsy's rank-revealing QRCP
//    (fftisdf.py:108): rank cut at tol_rel * max(diag) (SURVEY.md A3 — applied in
//    factored order downstream, never as an explicit inverse).
//
// Left-looking, one pivot per step: step j computes column j of L for every row
// (one wave per row, dot product over the j previous columns with a wave reduction),
// updates the residual diagonal d, then a per-matrix arg-max picks pivot j+1
// (first index on ties, as LAPACK's MAXLOC).  Chosen rows are marked d = -1.
#include <cstdio>
#include <cstring>
#include <vector>

#include <mutex>

#include "common.h"

namespace fisdf {

namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// d <- Re(diag A); choose pivot 0.
__global__ void pchol_init(const cplx* __restrict__ A, long lda, long sA, int n, int rmax,
                           double tol_rel, double tol_abs, int* __restrict__ piv,
                           double* __restrict__ pval, int* __restrict__ rank,
                           double* __restrict__ d, int* __restrict__ flags,
                           double* __restrict__ dmax0) {
  const int b = blockIdx.x;
  A += (long)b * sA;
  d += (long)b * n;
  __shared__ double sv[1024];
  __shared__ int si[1024];
  double best = -1.0;
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    double v = A[(long)i * lda + i].x;
    d[i] = v;
    if (v > best || (v == best && i < bi)) { best = v; bi = i; }
  }
  sv[threadIdx.x] = best;
  si[threadIdx.x] = bi;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      double o = sv[threadIdx.x + s];
      int oi = si[threadIdx.x + s];
      if (o > sv[threadIdx.x] || (o == sv[threadIdx.x] && oi < si[threadIdx.x])) {
        sv[threadIdx.x] = o;
        si[threadIdx.x] = oi;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double m = sv[0];
    double tol = tol_rel > 0 ? tol_rel * m : (double)n * 2.220446049250313e-16 * m;
    if (tol_abs > tol) tol = tol_abs;
    dmax0[b] = tol;  // store the absolute stopping threshold
    if (!(m > tol) || rmax <= 0) {
      flags[b] = 1;
      rank[b] = 0;
    } else {
      flags[b] = 0;
      rank[b] = 0;
      piv[(long)b * rmax] = si[0];
      pval[(long)b * rmax] = m;
    }
  }
}

// column j of L for all rows; one wave per row
__global__ __launch_bounds__(256) void pchol_step(const cplx* __restrict__ A, long lda, long sA,
                                                  int n, int rmax, int j,
                                                  const int* __restrict__ piv,
                                                  const double* __restrict__ pval,
                                                  cplx* __restrict__ L, double* __restrict__ d,
                                                  const int* __restrict__ flags) {
  const int b = blockIdx.y;
  if (flags[b]) return;
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (i >= n) return;
  A += (long)b * sA;
  L += (long)b * n * rmax;
  d += (long)b * n;
  const int p = piv[(long)b * rmax + j];
  const double dp = pval[(long)b * rmax + j];
  const double di = d[i];
  if (di <= -1e299 && i != p) {  // already a pivot row
    if (lane == 0) L[(long)i * rmax + j] = cmk(0, 0);
    return;
  }
  // s = sum_{t<j} L[i,t] * conj(L[p,t])
  double sr = 0, si = 0;
  const cplx* Li = L + (long)i * rmax;
  const cplx* Lp = L + (long)p * rmax;
  for (int t = lane; t < j; t += 64) {
    cplx a = Li[t], c = Lp[t];
    sr += a.x * c.x + a.y * c.y;
    si += a.y * c.x - a.x * c.y;
  }
  sr = wave_sum(sr);
  si = wave_sum(si);
  if (lane == 0) {
    const double sq = sqrt(dp);
    if (i == p) {
      L[(long)i * rmax + j] = cmk(sq, 0.0);
      d[i] = -1e300;
    } else {
      cplx aip = A[(long)i * lda + p];
      cplx l = cmk((aip.x - sr) / sq, (aip.y - si) / sq);
      L[(long)i * rmax + j] = l;
      d[i] = di - (l.x * l.x + l.y * l.y);
    }
  }
}

// arg-max of the residual diagonal -> pivot j+1, or stop
__global__ void pchol_pick(int n, int rmax, int j, int* __restrict__ piv, double* __restrict__ pval,
                           int* __restrict__ rank, const double* __restrict__ d,
                           int* __restrict__ flags, const double* __restrict__ thr) {
  const int b = blockIdx.x;
  if (flags[b]) return;
  d += (long)b * n;
  __shared__ double sv[1024];
  __shared__ int si[1024];
  double best = -1.0;
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    double v = d[i];
    if (v > best || (v == best && i < bi)) { best = v; bi = i; }
  }
  sv[threadIdx.x] = best;
  si[threadIdx.x] = bi;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      double o = sv[threadIdx.x + s];
      int oi = si[threadIdx.x + s];
      if (o > sv[threadIdx.x] || (o == sv[threadIdx.x] && oi < si[threadIdx.x])) {
        sv[threadIdx.x] = o;
        si[threadIdx.x] = oi;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    rank[b] = j + 1;
    if (j + 1 >= rmax || !(sv[0] > thr[b])) {
      flags[b] = 1;
    } else {
      piv[(long)b * rmax + j + 1] = si[0];
      pval[(long)b * rmax + j + 1] = sv[0];
    }
  }
}

// ---- blocked variant (dpstrf-style): one workgroup per matrix factors a panel of NB
// pivots with the panel held in registers (GEMV only over the panel's own columns), then
// one batched ZGEMM applies the panel to the trailing matrix W -= L_panel L_panel^H.
// 2 launches per NB pivots instead of 2 per pivot; trailing traffic 2|W| per panel.
constexpr int PB_THREADS = 1024;

template <int NB>
__global__ __launch_bounds__(PB_THREADS) void pchol_panel(const cplx* __restrict__ W, long sW,
                                                          int n, int rmax, int j0,
                                                          cplx* __restrict__ L,
                                                          int* __restrict__ piv,
                                                          int* __restrict__ rank,
                                                          double* __restrict__ d,
                                                          int* __restrict__ flags,
                                                          const double* __restrict__ thr) {
  const int b = blockIdx.x;
  if (flags[b]) return;
  W += b * sW;
  L += (long)b * n * rmax;
  piv += (long)b * rmax;
  d += (long)b * n;
  __shared__ double s_v[PB_THREADS / 64];
  __shared__ int s_i[PB_THREADS / 64];
  __shared__ cplx s_lp[NB];
  __shared__ int s_p, s_stop;
  __shared__ double s_dp;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int i = tid;  // one row per thread (n <= PB_THREADS)
  const bool live = i < n;
  double dd = live ? d[i] : -1e300;
  cplx lp[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) lp[c] = cmk(0, 0);
  const double t = thr[b];
  int jdone = j0;
  bool stopped = false;
  // lp[c] stays zero for columns not yet computed, so every dot runs over all NB columns and
  // lp is only ever indexed with compile-time indices (no scratch)
  for (int jj = 0; jj < NB; ++jj) {
    const int j = j0 + jj;
    if (!stopped && j < rmax) {
      // arg-max of the residual diagonal, first index on ties (LAPACK MAXLOC)
      double bv = live ? dd : -1e300;
      int bi = live ? i : 0x7fffffff;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        double ov = __shfl_xor(bv, o, 64);
        int oi = __shfl_xor(bi, o, 64);
        if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
      }
      if (lane == 0) { s_v[wid] = bv; s_i[wid] = bi; }
      __syncthreads();
      if (wid == 0) {
        bv = lane < PB_THREADS / 64 ? s_v[lane] : -1e300;
        bi = lane < PB_THREADS / 64 ? s_i[lane] : 0x7fffffff;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          double ov = __shfl_xor(bv, o, 64);
          int oi = __shfl_xor(bi, o, 64);
          if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
        }
        if (lane == 0) {
          s_p = bi;
          s_dp = bv;
          s_stop = !(bv > t);
          if (!s_stop) piv[j] = bi;
        }
      }
      __syncthreads();
      const int p = s_p;
      const double dp = s_dp;
      if (s_stop) {
        stopped = true;
      } else {
        if (i == p) {
#pragma unroll
          for (int c = 0; c < NB; ++c) s_lp[c] = lp[c];
        }
        __syncthreads();
        cplx l = cmk(0, 0);
        if (live) {
          const double sq = sqrt(dp);
          if (i == p) {
            l = cmk(sq, 0.0);
            dd = -1e300;
          } else if (dd > -1e299) {
            cplx w = cconj(W[(long)p * n + i]);  // W[i][p] of the Hermitian trailing matrix
#pragma unroll
            for (int c = 0; c < NB; ++c) w = csub(w, cmul(lp[c], cconj(s_lp[c])));
            l = cmk(w.x / sq, w.y / sq);
            dd -= l.x * l.x + l.y * l.y;
          }
        }
#pragma unroll
        for (int c = 0; c < NB; ++c)
          if (c == jj) lp[c] = l;
        jdone = j + 1;
        __syncthreads();  // s_lp reused by the next pivot
      }
    }
  }
  if (live) {
    d[i] = dd;
    cplx* Li = L + (long)i * rmax + j0;
#pragma unroll
    for (int c = 0; c < NB; ++c)
      if (j0 + c < rmax) Li[c] = lp[c];
  }
  if (tid == 0) {
    rank[b] = jdone;
    if (stopped || jdone >= rmax) flags[b] = 1;
  }
}

// ---- real blocked variant for the interpolation-point selection --------------------------
// The selection Gram x4 = Re(x2)^2 / nk is real (fftisdf.py:376-379).  Right-looking blocked
// pivoted Cholesky (dpstrf structure) on a real n x n trailing matrix W: one 512-thread
// workgroup factors a panel of NB pivots with its rows' panel entries in registers (RPT rows per
// thread; the pivot row of W is one coalesced read per pivot), then a tiled real rank-NB
// update W -= L_panel L_panel^T.  Same pivot choice as LAPACK: arg-max of the residual
// diagonal, first index on ties; tol <= 0 -> n * eps * max(diag).
constexpr int PR_THREADS = 512;

template <int RPT, int NB>
__global__ __launch_bounds__(PR_THREADS) void pchol_real_panel(const double* __restrict__ W, int n,
                                                               int rmax, int j0, double tol,
                                                               double* __restrict__ Lpan,
                                                               int* __restrict__ piv,
                                                               int* __restrict__ rank,
                                                               double* __restrict__ d,
                                                               int* __restrict__ flags,
                                                               double* __restrict__ thr) {
  if (flags[0]) return;
  __shared__ double s_v[PR_THREADS / 64];
  __shared__ int s_i[PR_THREADS / 64];
  __shared__ double s_lp[NB];
  __shared__ int s_p, s_stop;
  __shared__ double s_dp, s_thr;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  double dd[RPT];
  double lp[RPT][NB];
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int i = tid + PR_THREADS * r;
    dd[r] = i < n ? d[i] : -1e300;
#pragma unroll
    for (int c = 0; c < NB; ++c) lp[r][c] = 0.0;
  }
  // block arg-max of (value, index): larger value, then smaller index
  auto argmax = [&](double v, int idx, double* ov, int* oi) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double v2 = __shfl_xor(v, o, 64);
      const int i2 = __shfl_xor(idx, o, 64);
      if (v2 > v || (v2 == v && i2 < idx)) { v = v2; idx = i2; }
    }
    if (lane == 0) { s_v[wid] = v; s_i[wid] = idx; }
    __syncthreads();
    v = lane < PR_THREADS / 64 ? s_v[lane] : -1e300;
    idx = lane < PR_THREADS / 64 ? s_i[lane] : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double v2 = __shfl_xor(v, o, 64);
      const int i2 = __shfl_xor(idx, o, 64);
      if (v2 > v || (v2 == v && i2 < idx)) { v = v2; idx = i2; }
    }
    *ov = v;
    *oi = idx;
  };
  if (j0 == 0) {  // stopping threshold from the initial diagonal
    double bv = -1e300;
    int bi = 0x7fffffff;
#pragma unroll
    for (int r = 0; r < RPT; ++r)
      if (dd[r] > bv) { bv = dd[r]; bi = tid + PR_THREADS * r; }
    double m;
    int mi;
    argmax(bv, bi, &m, &mi);
    if (tid == 0) {
      s_thr = tol > 0 ? tol * m : (double)n * 2.220446049250313e-16 * m;
      thr[0] = s_thr;
    }
  } else if (tid == 0) {
    s_thr = thr[0];
  }
  __syncthreads();
  const double t = s_thr;
  int jdone = j0;
  bool stopped = false;
#pragma unroll
  for (int jj = 0; jj < NB; ++jj) {
    const int j = j0 + jj;
    if (stopped || j >= rmax) break;  // uniform over the workgroup
    double bv = -1e300;
    int bi = 0x7fffffff;
#pragma unroll
    for (int r = 0; r < RPT; ++r)
      if (dd[r] > bv) { bv = dd[r]; bi = tid + PR_THREADS * r; }
    double v;
    int p;
    argmax(bv, bi, &v, &p);
    if (tid == 0) {
      s_p = p;
      s_dp = v;
      s_stop = !(v > t);
      if (!s_stop) piv[j] = p;
    }
    __syncthreads();
    p = s_p;
    const double dp = s_dp;
    if (s_stop) {
      stopped = true;
      break;
    }
#pragma unroll
    for (int r = 0; r < RPT; ++r)
      if (tid + PR_THREADS * r == p) {
#pragma unroll
        for (int c = 0; c < NB; ++c) s_lp[c] = lp[r][c];
      }
    // column p of the trailing matrix from its lower triangle (the only part the rank-NB
    // updates keep current): row p for i < p (coalesced), column p below the diagonal
    double wrow[RPT];
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      const int i = tid + PR_THREADS * r;
      wrow[r] = i < n ? W[i < p ? (long)p * n + i : (long)i * n + p] : 0.0;
    }
    __syncthreads();
    const double sq = sqrt(dp), inv = 1.0 / sq;
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      const int i = tid + PR_THREADS * r;
      double l = 0.0;
      if (i == p) {
        l = sq;
        dd[r] = -1e300;
      } else if (i < n && dd[r] > -1e299) {
        double w = wrow[r];
#pragma unroll
        for (int c = 0; c < NB; ++c) w -= lp[r][c] * s_lp[c];
        l = w * inv;
        dd[r] -= l * l;
      }
      lp[r][jj] = l;
    }
    jdone = j + 1;
    __syncthreads();  // s_lp / s_p reused by the next pivot
  }
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int i = tid + PR_THREADS * r;
    if (i < n) {
      d[i] = dd[r];
#pragma unroll
      for (int c = 0; c < NB; ++c) Lpan[(long)i * NB + c] = lp[r][c];
    }
  }
  if (tid == 0) {
    rank[0] = jdone;
    if (stopped || jdone >= rmax) flags[0] = 1;
  }
}

// W -= Lpan Lpan^T on the lower triangle of tiles (64 x 64 tile per 256-thread workgroup,
// 4 x 4 elements per thread, the two NB-wide panel slices in LDS); 1-D grid over the
// T(T+1)/2 tiles with row >= column
template <int NB>
__global__ __launch_bounds__(256) void syrk_real_update(double* __restrict__ W, int n,
                                                        const double* __restrict__ Lpan,
                                                        const int* __restrict__ flags) {
  if (flags[0]) return;
  __shared__ double Li[64][NB + 1], Lj[64][NB + 1];
  const int t = blockIdx.x;
  int bi = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((bi + 1) * (bi + 2) / 2 <= t) ++bi;
  while (bi * (bi + 1) / 2 > t) --bi;
  const int bj = t - bi * (bi + 1) / 2;
  const int i0 = bi * 64, j0 = bj * 64;
  const int tid = threadIdx.x;
  for (int e = tid; e < 64 * NB; e += 256) {
    const int r = e / NB, c = e % NB;
    Li[r][c] = i0 + r < n ? Lpan[(long)(i0 + r) * NB + c] : 0.0;
    Lj[r][c] = j0 + r < n ? Lpan[(long)(j0 + r) * NB + c] : 0.0;
  }
  __syncthreads();
  const int ti = (tid >> 4) * 4, tj = (tid & 15) * 4;
  double acc[4][4] = {};
#pragma unroll 2
  for (int c = 0; c < NB; ++c)
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] += Li[ti + a][c] * Lj[tj + b][c];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int i = i0 + ti + a;
    if (i >= n) continue;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int j = j0 + tj + b;
      if (j < n) W[(long)i * n + j] -= acc[a][b];
    }
  }
}

// ---- cooperative left-looking variant (default for the selection) ----------------------
// One pivot per step over a co-resident grid (launch_coresident): workgroup w owns
// rows [w*RW, w*RW+RW) with their L rows in LDS (and a copy in the row-major global L) and
// their residual diagonal.  Step j:
//   post: the local arg-max of the residual diagonal as one 16-byte record {value, row, step}
//     (a single agent-coherent dwordx4 store);
//   poll: thread g waits for workgroup g's record of step j; block arg-max (larger value,
//     then smaller row: LAPACK's first index on ties) -> pivot p, d_p;
//   gather: L[p, :j] from the global L and x4[p, owned rows] = Re(x2[p, rows])^2 * scale;
//   column: L[rows, j] = (x4[rows, p] - L[rows, :j] L[p, :j]^T) / sqrt(d_p), 8 threads per row;
//     d -= L^2; the new entries go to LDS and to the global L (completed before the next post,
//     so a reader that sees step j+1's record sees row p's entries up to j).
// No trailing matrix is formed or updated.  Exchange traffic uses agent-coherent (sc1) loads
// and stores (no per-step L2 write-back/invalidate).  Records are double-buffered by step
// parity (a workgroup runs at most one step ahead).  Every wait is bounded: a stalled step
// sets *err and every workgroup exits (the caller then falls back to the blocked path).
// 512 threads: the column step's dot products over the owned L rows take 16 threads per row at C3
// (27 rows) instead of 8, halving the dependent LDS-load chain of the step's longest phase
// (per-step phase timing, FISDF_SEL_PROF: 1.86 of ≈ 5.9 us at 256 threads)
constexpr int SC_THREADS = 512;
constexpr int SC_MAXRW = SC_THREADS / 8;  // at least 8 threads per owned row
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void sc_store_rec(u32x4* addr, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(addr), "v"(v) : "memory");
}
__device__ __forceinline__ u32x4 sc_load_rec(const u32x4* addr) {
  u32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)"
               : "=v"(r)
               : "v"(addr)
               : "memory");
  return r;
}
__device__ __forceinline__ bool sc_better(double v2, int i2, double v, int i) {
  return v2 > v || (v2 == v && i2 < i);
}

__global__ __launch_bounds__(SC_THREADS) void pchol_select_coop(
    const cplx* __restrict__ X2, double scale, int n, int rmax, double tol, int RW, int K, int tpr,
    int* __restrict__ piv, int* __restrict__ rank, u32x4* __restrict__ rec,
    double* __restrict__ Lg, int* __restrict__ err, unsigned long long* __restrict__ prof,
    int* __restrict__ progress) {
  extern __shared__ double sm[];
  double* Lr = sm;                    // RW x K, row-major (columns >= K only in the global L)
  double* Lp = Lr + (long)RW * K;     // pivot row L[p, :j]
  double* dd = Lp + rmax;             // residual diagonal of the owned rows
  double* w0 = dd + RW;               // x4[p, owned rows]
  __shared__ double s_v[SC_THREADS / 64];
  __shared__ int s_i[SC_THREADS / 64];
  __shared__ int s_p, s_stop;
  __shared__ double s_dp, s_thr;
  const int G = gridDim.x, w = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r0 = w * RW, nr = max(0, min(RW, n - r0));
  // with a streamed consumer (progress) other kernels share the CUs: the dependent pivot chain
  // issues first
  if (progress) __builtin_amdgcn_s_setprio(3);
  if (tid < RW) {
    double v = -1e300;
    if (tid < nr) {
      const double x = X2[(long)(r0 + tid) * n + r0 + tid].x;
      v = x * x * scale;
    }
    dd[tid] = v;
  }
  if (tid == 0) s_stop = 0;
  __syncthreads();
  for (int j = 0;; ++j) {
    // ---- post ----
    if (wid == 0) {
      double v = lane < nr ? dd[lane] : -1e300;
      int i = lane < nr ? r0 + lane : 0x7fffffff;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const double v2 = __shfl_xor(v, o, 64);
        const int i2 = __shfl_xor(i, o, 64);
        if (sc_better(v2, i2, v, i)) { v = v2; i = i2; }
      }
      if (lane == 0) {
        const unsigned long long vb = (unsigned long long)__double_as_longlong(v);
        u32x4 r;
        r.x = (unsigned)vb;
        r.y = (unsigned)(vb >> 32);
        r.z = (unsigned)i;
        r.w = (unsigned)(j + 1);
        sc_store_rec(rec + (j & 1) * G + w, r);
      }
    }
    // timing probe (FISDF_SEL_PROF): workgroup 0's phase boundaries of every step
    const bool pr = prof != nullptr && w == 0 && tid == 0 && j < rmax;
    if (pr) prof[4L * j] = __builtin_amdgcn_s_memrealtime();
    // ---- poll ----
    {
      double v = -1e300;
      int i = 0x7fffffff;
      bool bad = false;
      for (int g = tid; g < G; g += SC_THREADS) {
        u32x4 r;
        long spins = 0;
        for (;;) {
          r = sc_load_rec(rec + (j & 1) * G + g);
          if (r.w == (unsigned)(j + 1)) break;
          __builtin_amdgcn_s_sleep(1);
          if (++spins > (1L << 22) ||
              ((spins & 1023) == 0 &&
               __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
            bad = true;
            break;
          }
        }
        if (bad) break;
        const double v2 =
            __longlong_as_double((long long)(((unsigned long long)r.y << 32) | r.x));
        const int i2 = (int)r.z;
        if (sc_better(v2, i2, v, i)) { v = v2; i = i2; }
      }
      if (bad) {
        atomicExch(err, 1);
        s_stop = 1;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const double v2 = __shfl_xor(v, o, 64);
        const int i2 = __shfl_xor(i, o, 64);
        if (sc_better(v2, i2, v, i)) { v = v2; i = i2; }
      }
      if (lane == 0) { s_v[wid] = v; s_i[wid] = i; }
      __syncthreads();
      if (s_stop) return;
      if (tid == 0) {
        for (int q = 1; q < SC_THREADS / 64; ++q)
          if (sc_better(s_v[q], s_i[q], v, i)) { v = s_v[q]; i = s_i[q]; }
        if (j == 0) s_thr = tol > 0 ? tol * v : (double)n * 2.220446049250313e-16 * v;
        const bool stop = !(v > s_thr) || i == 0x7fffffff;
        s_stop = stop;
        s_p = i;
        s_dp = v;
        if (w == 0) {
          if (progress) {
            // streamed consumers (the y build behind the selection, api.hip) read piv[] while
            // the kernel runs: the pivot goes out agent-coherent, and every kSelPublish pivots
            // (and at the end) the count follows once the pivot stores have completed
            if (!stop) __hip_atomic_store(&piv[j], i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const bool last = stop || j + 1 >= rmax;
            if (last || ((j + 1) % kSelPublish) == 0) {
              asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
              __hip_atomic_store(progress, last ? kSelDone : j + 1, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
            }
          } else if (!stop) {
            piv[j] = i;
          }
          if (stop || j + 1 >= rmax) rank[0] = stop ? j : j + 1;
        }
      }
      __syncthreads();
      if (s_stop) return;
    }
    const int p = s_p;
    const double dp = s_dp;
    if (pr) prof[4L * j + 1] = __builtin_amdgcn_s_memrealtime();
    // ---- gather ----
#ifndef FISDF_EXP_NOGATHER  // timing experiment only (stale pivot row)
    for (int c = tid; c < j; c += SC_THREADS)
      Lp[c] = __hip_atomic_load(&Lg[(long)p * rmax + c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
    for (int r = tid; r < nr; r += SC_THREADS) {
      const double x = X2[(long)p * n + r0 + r].x;
      w0[r] = x * x * scale;
    }
    __syncthreads();
    if (pr) prof[4L * j + 2] = __builtin_amdgcn_s_memrealtime();
    // ---- column j ----
    {
      const double sq = sqrt(dp), inv = 1.0 / sq;
      const int r = tid / tpr, part = tid & (tpr - 1);
      if (r < nr) {
        const double* lr = Lr + (long)r * K;
        const int jl = min(j, K);
        double a0 = 0.0, a1 = 0.0;
        int c = part;
        for (; c + tpr < jl; c += 2 * tpr) {
          a0 += lr[c] * Lp[c];
          a1 += lr[c + tpr] * Lp[c + tpr];
        }
        if (c < jl) a0 += lr[c] * Lp[c];
        if (j > K) {  // this workgroup's own entries past the LDS columns, written by earlier steps
          const double* lg = Lg + (long)(r0 + r) * rmax;
          for (c = K + part; c < j; c += tpr)
            a1 += __hip_atomic_load(lg + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * Lp[c];
        }
        double acc = a0 + a1;
        for (int o = 1; o < tpr; o <<= 1) acc += __shfl_xor(acc, o, 64);
        if (part == 0) {
          const int i = r0 + r;
          double l = 0.0;
          if (i == p) {
            l = sq;
            dd[r] = -1e300;
          } else if (dd[r] > -1e299) {
            l = (w0[r] - acc) * inv;
            dd[r] -= l * l;
          }
          if (j < K) Lr[(long)r * K + j] = l;
          __hip_atomic_store(&Lg[(long)i * rmax + j], l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifndef FISDF_EXP_NOSTOREWAIT  // timing experiment only (breaks the hand-off)
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
        }
      }
    }
    __syncthreads();
    if (pr) prof[4L * j + 3] = __builtin_amdgcn_s_memrealtime();
    if (j + 1 >= rmax) return;
  }
}

// ---- batched-candidate selection (default where the owned rows fit, C1-C4) -------------------
// pchol_select_coop needs a grid-wide arg-max and a pivot-row hand-off for EVERY pivot: two
// dependent cross-XCD round trips, ~6 us per pivot at C3 whatever the exchange's shape
// (4.0 ms of every k-shard rank).  Here the grid exchanges once per BATCH:
//  * owners (workgroups 0..G-1, RW <= 16 rows each, their L rows in LDS and in the row-major
//    global L) post their residual diagonal as tagged 16-byte granules {d, row, batch};
//  * the leader (workgroup G) reads them all and takes as candidates C the 4 best rows (value
//    desc, row asc: LAPACK's first index on ties) of each of its 8 waves' share, and as the bound
//    B the best row left out; it forms the candidates' residual block R = x4[C,C] - L[C,:j]
//    L[C,:j]^T on FP64 MFMA from the global L rows and runs the greedy steps on R alone while the
//    chosen diagonal beats B.  No other row can win such a step: its residual diagonal only
//    decreases (d -= l^2) and was <= B at the batch start, so every accepted step is exactly the
//    greedy (dpstrf) pivot of the whole matrix;
//  * the leader publishes the batch (pivots, their d, the candidates' new L entries and
//    residuals); each owner forms its rows' new columns with one MFMA pass against the pivot
//    rows (acc = L[rows,:j] L[piv,:j]^T) plus the in-batch triangular part, and posts again.
// Simulated on the C3 parent grid (n 3375, 600 pivots): 99 batches of 32 per-wave candidates
// (100 with the exact top 16, 165 with 2 per wave).  Hand-offs: every handed-off byte is stored
// sc1 (write-through) and loaded sc1; the owners' L stores wait (vmcnt) behind a barrier before
// their next post; the published granules carry their batch and a stale one is re-read.  Every
// wait is bounded: a stalled wait sets *err and the grid drains (the caller then falls back).
constexpr int SB_THREADS = 512;
constexpr int SB_TW = 4;                    // candidates per leader wave
constexpr int SB_M = 8 * SB_TW;             // candidates per batch
constexpr int SB_S = 16;                    // pivots per batch at most (one MFMA N block)
constexpr int SB_GR = 8;                    // granules per leader thread: n <= 8 * 512
constexpr int SB_KCH = 20;                  // K steps (4 columns) per wave and load chunk
constexpr int SB_NPUB = 1 + SB_M + SB_S + SB_M * SB_S;  // granules of one publish
constexpr long SB_SPIN = 1L << 22;

// The leader's publish: SB_NPUB 16-byte granules {payload lo, payload hi, aux, batch}, each
// written whole by one sc1 store (untorn), so a reader checks every granule's batch word and
// re-reads a stale one — no flag-after-payload ordering is needed:
//   [0]                  {s, stop, rank, b}
//   [1 + c]              {dnew_c (the candidate's residual after the batch, -1e300 chosen), row_c}
//   [1 + M + k]          {d of pivot k when chosen, candidate index of pivot k}
//   [1 + M + S + c S + k] {L[cand c, j + k] (the batch's columns of the candidates), index}
__device__ __forceinline__ double sb_dbl(u32x4 g) {
  return __longlong_as_double((long long)(((unsigned long long)g.y << 32) | g.x));
}
__device__ __forceinline__ u32x4 sb_gran(double v, unsigned aux, unsigned tag) {
  const unsigned long long vb = (unsigned long long)__double_as_longlong(v);
  u32x4 g;
  g.x = (unsigned)vb;
  g.y = (unsigned)(vb >> 32);
  g.z = aux;
  g.w = tag;
  return g;
}
__device__ __forceinline__ void sb_st_d(double* a, double v) {
  __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double sb_ld_d(const double* a) {
  return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// re-read a granule until its batch word is `tag`; false on a stall or another workgroup's error
__device__ __forceinline__ bool sb_repoll(const u32x4* gp, unsigned tag, int* err, u32x4* g) {
  for (long spins = 0; g->w != tag; ++spins) {
    __builtin_amdgcn_s_sleep(2);
    if (spins > SB_SPIN ||
        ((spins & 1023) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
      atomicExch(err, 1);
      return false;
    }
    *g = sc_load_rec(gp);
  }
  return true;
}
// one DPP step of the wave arg-max (value desc, row asc); out-of-row sources keep the own key
template <int CTRL, int RMASK>
__device__ __forceinline__ void sb_dpp_step(double& v, int& r) {
  const long long b = __double_as_longlong(v);
  const int lo = (int)b, hi = (int)(b >> 32);
  const int lo2 = __builtin_amdgcn_update_dpp(lo, lo, CTRL, RMASK, 0xf, false);
  const int hi2 = __builtin_amdgcn_update_dpp(hi, hi, CTRL, RMASK, 0xf, false);
  const int r2 = __builtin_amdgcn_update_dpp(r, r, CTRL, RMASK, 0xf, false);
  const double v2 = __longlong_as_double(((long long)hi2 << 32) | (unsigned)lo2);
  if (sc_better(v2, r2, v, r)) {
    v = v2;
    r = r2;
  }
}
// the wave's best key, uniform in every lane: row_shr 1/2/4/8 leaves each row's best in its
// lane 15, row_bcast 15/31 carry them up to lane 63
__device__ __forceinline__ void sb_wave_best(double& v, int& r) {
  sb_dpp_step<0x111, 0xf>(v, r);
  sb_dpp_step<0x112, 0xf>(v, r);
  sb_dpp_step<0x114, 0xf>(v, r);
  sb_dpp_step<0x118, 0xf>(v, r);
  sb_dpp_step<0x142, 0xa>(v, r);
  sb_dpp_step<0x143, 0xc>(v, r);
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, 63);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  v = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
  r = __builtin_amdgcn_readlane(r, 63);
}
template <int A, int B>
__device__ __forceinline__ void sb_cx(double (&v)[SB_GR], int (&r)[SB_GR]) {
  if (sc_better(v[B], r[B], v[A], r[A])) {
    const double tv = v[A];
    const int tr = r[A];
    v[A] = v[B];
    r[A] = r[B];
    v[B] = tv;
    r[B] = tr;
  }
}

__global__ __launch_bounds__(SB_THREADS) void pchol_select_batch(
    const cplx* __restrict__ X2, double scale, int n, int rmax, double tol, int RW,
    int* __restrict__ piv, int* __restrict__ rank, u32x4* __restrict__ ddg,
    u32x4* __restrict__ pub, double* __restrict__ Lg, int* __restrict__ err,
    unsigned long long* __restrict__ prof) {
  extern __shared__ double sm[];
  constexpr int M = SB_M, S = SB_S;
  const int G = gridDim.x - 1, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i16 = lane & 15, kq = lane >> 4;
  double* red = sm;  // MFMA partials
  __shared__ int s_i[M + S + 8];
  __shared__ double s_d[M + S + M + 8];
  __shared__ int s_bad;
  if (tid == 0) s_bad = 0;
  if ((int)blockIdx.x < G) {
    // ======================= owner: rows [r0, r0 + nr) =======================
    double* Lr = red + 8 * 256;     // RW x rmax, row-major
    double* Lnew = Lr + (long)RW * rmax;  // [candidate][k]: the batch's columns of the candidates
    double* x4p = Lnew + M * S;     // [row][k] = x4[row, p_k]
    double* acc = x4p + 16 * S;     // [row][k] = L[row, :j] . L[p_k, :j]
    int* cand = s_i;                // candidates (rows, -1 none)
    int* pidx = s_i + M;            // candidate index of pivot k
    int* hdr = s_i + M + S;         // s, stop
    double* dnew = s_d;
    double* dpv = s_d + M;
    const int r0 = blockIdx.x * RW, nr = max(0, min(RW, n - r0));
    double dd = -1e300;             // thread r < nr: residual diagonal of row r0 + r
    if (tid < nr) {
      const double x = X2[(long)(r0 + tid) * n + r0 + tid].x;
      dd = x * x * scale;
    }
    int j = 0;
    for (unsigned b = 1;; ++b) {
      if (tid < nr) sc_store_rec(ddg + r0 + tid, sb_gran(dd, (unsigned)(r0 + tid), b));  // post
      // the leader's publish of this batch: one lane waits for the header (211 pollers, not
      // 211 x 512: polling traffic slows everybody's loads), then every granule is read in one
      // round and a stale one re-read
      if (tid == 0) {
        u32x4 h = sc_load_rec(pub);
        if (!sb_repoll(pub, b, err, &h)) s_bad = 1;
      }
      __syncthreads();
      if (s_bad) return;
      u32x4 g0 = sc_load_rec(pub + tid), g1;
      const bool two = tid + SB_THREADS < SB_NPUB;
      if (two) g1 = sc_load_rec(pub + tid + SB_THREADS);
      bool ok = true;
      if (g0.w != b) {
        u32x4 g = sc_load_rec(pub + tid);
        ok = sb_repoll(pub + tid, b, err, &g);
        g0 = g;
      }
      if (two && ok && g1.w != b) {
        u32x4 g = sc_load_rec(pub + tid + SB_THREADS);
        ok = sb_repoll(pub + tid + SB_THREADS, b, err, &g);
        g1 = g;
      }
      if (!ok) s_bad = 1;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = tid + h * SB_THREADS;
        if (h == 1 && !two) break;
        const u32x4 g = h ? g1 : g0;
        const double v = sb_dbl(g);
        if (e == 0) {
          hdr[0] = (int)g.x;
          hdr[1] = (int)g.y;
        } else if (e < 1 + M) {
          cand[e - 1] = (int)g.z;
          dnew[e - 1] = v;
        } else if (e < 1 + M + S) {
          pidx[e - 1 - M] = (int)g.z;
          dpv[e - 1 - M] = v;
        } else {
          Lnew[e - 1 - M - S] = v;
        }
      }
      __syncthreads();
      if (s_bad) return;
      const int s = hdr[0], stop = hdr[1];
      if (s > 0) {
        // acc[r][k] = sum_{l < j} L[r0 + r, l] L[p_k, l]: FP64 MFMA, A = the owned rows (LDS),
        // B = the pivot rows (global L), K split over the 8 waves, a chunk's loads issued up front
        const int nks = (j + 3) >> 2;
        const int prow = cand[pidx[min(i16, s - 1)]];
        const double* lgp = Lg + (long)prow * rmax;
        const bool bok = i16 < s, aok = i16 < nr;
        // x4[row, p_k] (row p_k of x4 is contiguous over this workgroup's rows)
        double xv = 0.0;
        const int xr = tid & 15, xk = (tid >> 4) & 15;
        if (tid < 16 * S && xr < nr && xk < s) xv = X2[(long)cand[pidx[xk]] * n + r0 + xr].x;
        f64x4 D = {0, 0, 0, 0};
        for (int c0 = 0; c0 < nks; c0 += 8 * SB_KCH) {
          double bv[SB_KCH];
#pragma unroll
          for (int u = 0; u < SB_KCH; ++u) {
            const int ks = c0 + w + 8 * u, l = ks * 4 + kq;
            bv[u] = 0.0;
            if (ks < nks) {
              const double t = sb_ld_d(lgp + min(l, j - 1));
              bv[u] = (bok && l < j) ? t : 0.0;
            }
          }
#pragma unroll
          for (int u = 0; u < SB_KCH; ++u) {
            const int ks = c0 + w + 8 * u, l = ks * 4 + kq;
            if (ks < nks) {  // wave-uniform
              const double a = (aok && l < j) ? Lr[(long)i16 * rmax + l] : 0.0;
              D = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bv[u], D, 0, 0, 0);
            }
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) red[w * 256 + (kq + 4 * r) * 16 + i16] = D[r];
        if (tid < 16 * S) x4p[xr * S + xk] = xv * xv * scale;
        __syncthreads();
        if (tid < 256) {
          double t = 0.0;
#pragma unroll
          for (int q = 0; q < 8; ++q) t += red[q * 256 + tid];
          acc[(tid >> 4) * S + (tid & 15)] = t;
        }
        __syncthreads();
        // the batch's columns of each owned row, in order (one thread per row)
        if (tid < nr) {
          const int row = r0 + tid;
          int ci = -1;
#pragma unroll
          for (int c = 0; c < M; ++c)
            if (cand[c] == row) ci = c;
          double* lr = Lr + (long)tid * rmax + j;
          double* lg = Lg + (long)row * rmax + j;
          if (ci >= 0) {  // a candidate: the leader's entries and residual (a pivot: -1e300)
            for (int k = 0; k < s; ++k) {
              const double l = Lnew[ci * S + k];
              lr[k] = l;
              sb_st_d(lg + k, l);
            }
            dd = dnew[ci];
          } else {
            for (int k = 0; k < s; ++k) {
              double l = 0.0;
              if (dd > -1e299) {
                const double* lp = Lnew + pidx[k] * S;  // L[p_k, j + k'] for k' < k
                double v = x4p[tid * S + k] - acc[tid * S + k];
                for (int k2 = 0; k2 < k; ++k2) v -= lr[k2] * lp[k2];
                l = v / sqrt(dpv[k]);
                dd -= l * l;
              }
              lr[k] = l;
              sb_st_d(lg + k, l);
            }
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // before the next post (barrier)
        }
      }
      __syncthreads();
      j += s;
      if (stop) return;
    }
  }
  // ======================= leader =======================
  double* Rs = red + 3 * 8 * 256;   // M x M candidates' residual block
  double* Lb = Rs + M * M;          // the step's column, broadcast through LDS
  double* Ldn = Lb + 64;            // [c][k] the batch's columns of the candidates
  double* wbv = Ldn + M * S;        // per-wave bound (value, row)
  int* wbi = (int*)(wbv + 8);
  int* cand = s_i;                  // candidates (rows; -1 none)
  int* pidx = s_i + M;
  int* st = s_i + M + S;            // s, stop, rank, Brow
  double* cd = s_d;                 // candidates' residual diagonal (batch start)
  double* dpv = s_d + M;
  double* dn = s_d + M + S;         // candidates' residual after the batch
  double* misc = s_d + 2 * M + S;   // thr, Bv
  int j = 0;
  for (unsigned b = 1;; ++b) {
    const bool pr = prof != nullptr && tid == 0 && b <= 8192;
    // ---- every row's residual diagonal: all loads in flight, stale granules re-read ----
    double v[SB_GR];
    int rw[SB_GR];
    unsigned tg[SB_GR];
#pragma unroll
    for (int u = 0; u < SB_GR; ++u) {
      const u32x4 g = sc_load_rec(ddg + min(tid + SB_THREADS * u, n - 1));
      v[u] = sb_dbl(g);
      tg[u] = g.w;
    }
    bool bad = false;
#pragma unroll
    for (int u = 0; u < SB_GR; ++u) {
      const int row = tid + SB_THREADS * u;
      double x = v[u];
      v[u] = -1e300;
      rw[u] = 0x7fffffff;
      if (row < n && !bad) {
        u32x4 g;
        g.w = tg[u];
        if (tg[u] != b) {
          g = sc_load_rec(ddg + row);
          if (!sb_repoll(ddg + row, b, err, &g)) bad = true;
          x = sb_dbl(g);
        }
        if (!bad && x > -1e299) {
          v[u] = x;
          rw[u] = row;
        }
      }
    }
    if (bad) s_bad = 1;
    // ---- candidates: each wave's SB_TW best keys; the bound B: the best key left out ----
    // sorting network (19 compare-exchanges) puts each thread's 8 keys in order
    sb_cx<0, 1>(v, rw); sb_cx<2, 3>(v, rw); sb_cx<4, 5>(v, rw); sb_cx<6, 7>(v, rw);
    sb_cx<0, 2>(v, rw); sb_cx<1, 3>(v, rw); sb_cx<4, 6>(v, rw); sb_cx<5, 7>(v, rw);
    sb_cx<1, 2>(v, rw); sb_cx<5, 6>(v, rw); sb_cx<0, 4>(v, rw); sb_cx<3, 7>(v, rw);
    sb_cx<1, 5>(v, rw); sb_cx<2, 6>(v, rw);
    sb_cx<1, 4>(v, rw); sb_cx<3, 6>(v, rw);
    sb_cx<2, 4>(v, rw); sb_cx<3, 5>(v, rw);
    sb_cx<3, 4>(v, rw);
    for (int rd = 0; rd <= SB_TW; ++rd) {
      double mv = v[0];
      int mi = rw[0];
      sb_wave_best(mv, mi);
      if (rd < SB_TW) {
        if (lane == 0) {
          const bool valid = mi != 0x7fffffff;
          cand[w * SB_TW + rd] = valid ? mi : -1;
          cd[w * SB_TW + rd] = valid ? mv : -1e300;
        }
        if (mi != 0x7fffffff && rw[0] == mi) {  // the winner's lane moves on to its next key
#pragma unroll
          for (int u = 0; u + 1 < SB_GR; ++u) {
            v[u] = v[u + 1];
            rw[u] = rw[u + 1];
          }
          v[SB_GR - 1] = -1e300;
          rw[SB_GR - 1] = 0x7fffffff;
        }
      } else if (lane == 0) {
        wbv[w] = mv;
        wbi[w] = mi;
      }
    }
    __syncthreads();
    if (s_bad) return;
    if (pr) prof[4L * (b - 1)] = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
      double bv = -1e300;
      int bi = 0x7fffffff;
      for (int q = 0; q < 8; ++q)
        if (sc_better(wbv[q], wbi[q], bv, bi)) { bv = wbv[q]; bi = wbi[q]; }
      misc[1] = bv;
      st[3] = bi;
      if (b == 1) {  // dpstrf's tolerance from the largest diagonal
        double mx = -1e300;
        for (int c = 0; c < M; ++c) mx = fmax(mx, cd[c]);
        misc[0] = tol > 0 ? tol * mx : (double)n * 2.220446049250313e-16 * mx;
      }
    }
    // ---- R = x4[C,C] - L[C,:j] L[C,:j]^T (FP64 MFMA: blocks 00, 01, 11; K over the waves) ----
    {
      const int nks = (j + 3) >> 2;
      const int c0r = cand[i16], c1r = cand[16 + i16];
      const double* l0 = Lg + (long)max(c0r, 0) * rmax;
      const double* l1 = Lg + (long)max(c1r, 0) * rmax;
      double xv[2] = {0.0, 0.0};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = tid + h * SB_THREADS, a = e >> 5, c = e & 31;
        if (cand[a] >= 0 && cand[c] >= 0) xv[h] = X2[(long)cand[a] * n + cand[c]].x;
      }
      f64x4 D00 = {0, 0, 0, 0}, D01 = {0, 0, 0, 0}, D11 = {0, 0, 0, 0};
      for (int k0 = 0; k0 < nks; k0 += 8 * SB_KCH) {
        double a0[SB_KCH], a1[SB_KCH];
#pragma unroll
        for (int u = 0; u < SB_KCH; ++u) {
          const int ks = k0 + w + 8 * u, l = ks * 4 + kq;
          a0[u] = 0.0;
          a1[u] = 0.0;
          if (ks < nks) {
            const double t0 = sb_ld_d(l0 + min(l, j - 1)), t1 = sb_ld_d(l1 + min(l, j - 1));
            a0[u] = (c0r >= 0 && l < j) ? t0 : 0.0;
            a1[u] = (c1r >= 0 && l < j) ? t1 : 0.0;
          }
        }
#pragma unroll
        for (int u = 0; u < SB_KCH; ++u) {
          if (k0 + w + 8 * u < nks) {  // wave-uniform
            D00 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[u], a0[u], D00, 0, 0, 0);
            D01 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[u], a1[u], D01, 0, 0, 0);
            D11 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[u], a1[u], D11, 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = (kq + 4 * r) * 16 + i16;
        red[(0 * 8 + w) * 256 + o] = D00[r];
        red[(1 * 8 + w) * 256 + o] = D01[r];
        red[(2 * 8 + w) * 256 + o] = D11[r];
      }
      __syncthreads();
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = tid + h * SB_THREADS, a = e >> 5, c = e & 31;
        // block of (a, c): 00, 01 (a < 16 <= c), 10 = 01^T, 11
        const int blk = (a < 16) ? (c < 16 ? 0 : 1) : (c < 16 ? 1 : 2);
        const int ra = (a < 16 || blk == 2) ? (a & 15) : (c & 15);
        const int rc = (a < 16 || blk == 2) ? (c & 15) : (a & 15);
        double t = 0.0;
#pragma unroll
        for (int q = 0; q < 8; ++q) t += red[(blk * 8 + q) * 256 + ra * 16 + rc];
        Rs[e] = xv[h] * xv[h] * scale - t;
      }
      __syncthreads();
    }
    if (pr) prof[4L * (b - 1) + 1] = __builtin_amdgcn_s_memrealtime();
    // ---- the greedy steps on the candidates (wave 0; lane c < M holds candidate c's R row) ----
    if (w == 0) {
      const double thr = misc[0], Bv = misc[1];
      const int Brow = st[3];
      const int myrow = lane < M ? cand[lane] : -1;
      double d = lane < M ? cd[lane] : -1e300;
      bool chosen = myrow < 0;
      double Rr[M];
#pragma unroll
      for (int c = 0; c < M; ++c) Rr[c] = lane < M ? Rs[lane * M + c] : 0.0;
      int k = 0, stop = 0, rk = 0;
      for (;;) {
        if (j + k >= rmax) { stop = 1; rk = rmax; break; }
        if (k == S) break;  // the owners' MFMA block holds S pivots: next batch
        double mv = (lane < M && !chosen) ? d : -1e300;
        int mi = (lane < M && !chosen) ? myrow : 0x7fffffff;
        sb_wave_best(mv, mi);
        if (mi == 0x7fffffff) {  // every candidate chosen
          if (Brow == 0x7fffffff) { stop = 1; rk = j + k; }  // ... and no other row left
          break;
        }
        if (!sc_better(mv, mi, Bv, Brow)) break;  // a non-candidate could win the next step
        if (!(mv > thr)) { stop = 1; rk = j + k; break; }  // the global max is below dpstrf's tol
        const int pc = __builtin_amdgcn_readfirstlane(
            __ffsll((long long)__ballot(lane < M && myrow == mi)) - 1);
        const double sq = sqrt(mv), inv = 1.0 / sq;
        double rp = 0.0;
#pragma unroll
        for (int c = 0; c < M; ++c) rp = c == pc ? Rr[c] : rp;
        double l = 0.0;
        if (lane < M) {
          l = lane == pc ? sq : (chosen ? 0.0 : rp * inv);
          Ldn[lane * S + k] = l;
          Lb[lane] = l;
        }
        if (lane == 0) {
          pidx[k] = pc;
          dpv[k] = mv;
          piv[j + k] = mi;
        }
        __builtin_amdgcn_wave_barrier();
        // rank-1 update of the candidates' residual block (every lane reads the column)
        const bool upd = lane < M && !chosen && lane != pc;
#pragma unroll
        for (int c = 0; c < M; c += 2) {
          const double2 lc = *(const double2*)(Lb + c);
          if (upd) {
            Rr[c] -= l * lc.x;
            Rr[c + 1] -= l * lc.y;
          }
        }
        if (upd) d -= l * l;
        if (lane == pc) {
          chosen = true;
          d = -1e300;
        }
        __builtin_amdgcn_wave_barrier();
        ++k;
      }
      if (k == 0 && !stop) {  // cannot happen (the top candidate beats B); never spin on it
        stop = 1;
        rk = j;
        if (lane == 0) atomicExch(err, 1);
      }
      if (lane < M) dn[lane] = d;
      if (lane == 0) {
        st[0] = k;
        st[1] = stop;
        st[2] = rk;
        if (stop) rank[0] = rk;
      }
    }
    __syncthreads();
    if (pr) prof[4L * (b - 1) + 2] = __builtin_amdgcn_s_memrealtime();
    // ---- publish: the granules, header included (readers re-read stale ones) ----
    const int s = st[0], stop = st[1];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = tid + h * SB_THREADS;
      if (e >= SB_NPUB) break;
      u32x4 gr;
      if (e == 0) {
        gr.x = (unsigned)s;
        gr.y = (unsigned)stop;
        gr.z = (unsigned)st[2];
        gr.w = b;
      } else if (e < 1 + M) {
        gr = sb_gran(dn[e - 1], (unsigned)cand[e - 1], b);
      } else if (e < 1 + M + S) {
        const int k = e - 1 - M;
        gr = sb_gran(k < s ? dpv[k] : 1.0, k < s ? (unsigned)pidx[k] : 0u, b);
      } else {
        const int q = e - 1 - M - S;
        gr = sb_gran((q % S) < s ? Ldn[q] : 0.0, (unsigned)q, b);
      }
      sc_store_rec(pub + e, gr);
    }
    if (pr) prof[4L * (b - 1) + 3] = __builtin_amdgcn_s_memrealtime();
    j += s;
    if (stop) return;
    __syncthreads();  // the shared lists are rewritten by the next batch
  }
}

__global__ void real_square_scale_kernel(const cplx* __restrict__ in, double s,
                                         double* __restrict__ out, double* __restrict__ d,
                                         long n2, int n) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n2;
       e += (long)gridDim.x * blockDim.x) {
    const double r = in[e].x;
    const double v = r * r * s;
    out[e] = v;
    if (e / n == e % n) d[e / n] = v;
  }
}

// ---- unpivoted blocked Cholesky (full-rank fast path of the x4_q factorisation) -----------
// Right-looking, 64-column blocks, batched over q: the diagonal block is factored and inverted
// in LDS by one workgroup per matrix, the panel below is multiplied by the block inverse^H
// (in-place ZGEMM) and the trailing matrix gets a ZGEMM rank-64 update.  A matrix whose pivot
// falls to <= tol_rel * max(initial diag) is flagged (the caller then uses the pivoted,
// rank-revealing pchol for the batch).  Pivots = identity, rank = n on success.
__global__ void diag_max_kernel(const cplx* __restrict__ A, int n, long sA, double tol_rel,
                                double* __restrict__ thr, int* __restrict__ fail) {
  A += blockIdx.x * sA;
  __shared__ double sv[256];
  double m = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) m = fmax(m, A[(long)i * n + i].x);
  sv[threadIdx.x] = m;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) sv[threadIdx.x] = fmax(sv[threadIdx.x], sv[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    thr[blockIdx.x] = tol_rel * sv[0];
    fail[blockIdx.x] = 0;
  }
}

// factor + invert the m x m diagonal block at (b0, b0) of W (ld n); writes L_bb (lower) in
// place and L_bb^{-1} to Linv (64 x 64, batch stride 4096; identity on the padding).
// Register-blocked: thread t owns the 4 x 4 block (rows 4 (t >> 4), cols 4 (t & 15)) of both the
// trailing matrix A and the inverse X, and one step k does the right-looking Cholesky update and
// the matching forward-substitution step of X = L^{-1} together: column k of A and row k of X go
// through LDS (double-buffered by parity, one barrier per step), then every thread updates
//   A[i][j] -= l_ik conj(l_jk)   (i, j > k)        X[i][:] -= l_ik X[k][:] / l_kk   (i > k)
// with the masks folded into zeroed operands (no divergent branches in the update).  The
// round-2 kernel factored first and then inverted by 16 x 16 blocks with exec-masked branches
// around every element update (89 us per 64-column block at batch 4, the serial chain of the
// N-rank factorisation).
__global__ __launch_bounds__(256) void chol_diag_kernel(cplx* __restrict__ W, int n, long sW,
                                                        int b0, int m,
                                                        const double* __restrict__ thr,
                                                        int* __restrict__ fail,
                                                        cplx* __restrict__ Linv) {
  const int b = blockIdx.x;
  W += b * sW;
  Linv += (long)b * 4096;
  // the diagonal blocks are the serial chain of the factorisation, which runs beside the y
  // build's throughput kernels on the same CUs: raise the wave priority so the SIMD arbiter
  // issues this chain's instructions first
  __builtin_amdgcn_s_setprio(3);
  __shared__ cplx colA[2][64];  // column k of A, by step parity
  __shared__ cplx rowX[2][64];  // row k of X (not yet scaled by 1 / l_kk), by step parity
  const int t = threadIdx.x;
  const int bi = t >> 4, bj = t & 15, r0 = bi * 4, c0 = bj * 4;
  cplx a[4][4], x[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int i = r0 + r, j = c0 + c;
      a[r][c] = (i < m && j <= i) ? W[(long)(b0 + i) * n + b0 + j] : cmk(0, 0);
      x[r][c] = cmk(i == j ? 1.0 : 0.0, 0.0);
    }
  const double th = thr[b];
  bool bad = false;
  // k = 4 kb + kc with kc unrolled: register arrays are indexed with compile-time indices
  // only (a runtime index demotes them to scratch memory)
  for (int kb = 0; 4 * kb < m; ++kb) {
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) {
      const int k = 4 * kb + kc, p = kc & 1;
      if (k >= m) break;
      if (bj == kb) {
#pragma unroll
        for (int r = 0; r < 4; ++r) colA[p][r0 + r] = a[r][kc];
      }
      if (bi == kb) {
#pragma unroll
        for (int c = 0; c < 4; ++c) rowX[p][c0 + c] = x[kc][c];
      }
      __syncthreads();
      const double dk = colA[p][k].x;
      bad = bad || !(dk > th);
      const double lk = sqrt(fmax(dk, 1e-300)), inv = 1.0 / lk;
      cplx li[4], lj[4], xk[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const cplx vi = colA[p][r0 + r], vj = colA[p][c0 + r], vx = rowX[p][c0 + r];
        const double si = r0 + r > k ? inv : 0.0, sj = c0 + r > k ? inv : 0.0;
        li[r] = cscale(vi, si);
        lj[r] = cscale(vj, sj);
        xk[r] = cscale(vx, inv);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          a[r][c] = csub(a[r][c], cmul(li[r], cconj(lj[c])));
          x[r][c] = csub(x[r][c], cmul(li[r], xk[c]));
        }
      if (bj == kb) {  // column k of L final
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = r0 + r;
          a[r][kc] = i > k ? li[r] : (i == k ? cmk(lk, 0.0) : a[r][kc]);
        }
      }
      if (bi == kb) {  // row k of X final
#pragma unroll
        for (int c = 0; c < 4; ++c) x[kc][c] = xk[c];
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int i = r0 + r, j = c0 + c;
      if (i < m && j <= i) W[(long)(b0 + i) * n + b0 + j] = a[r][c];
      Linv[i * 64 + j] = (i < m && j < m) ? (j <= i ? x[r][c] : cmk(0, 0))
                                          : cmk(i == j ? 1.0 : 0.0, 0.0);
    }
  if (t == 0 && bad) fail[b] = 1;
}

__global__ void chol_finish_kernel(int n, int* __restrict__ piv, int* __restrict__ rank,
                                   const int* __restrict__ fail) {
  const int b = blockIdx.x;
  for (int i = threadIdx.x; i < n; i += blockDim.x) piv[(long)b * n + i] = i;
  if (threadIdx.x == 0) rank[b] = fail[b] ? 0 : n;
}

}  // namespace

// pivot values are kept in `dmax0 + batch` (caller allocates 2*batch + batch*rmax doubles: see api)
size_t pchol_trail_elems(int n, int batch) { return n <= PB_THREADS ? (size_t)n * n * batch : 0; }

int pchol(hipStream_t s, const cplx* A, long lda, long sA, int n, int batch, int rmax,
          double tol_rel, double tol_abs, cplx* L, int* piv, int* rank, double* d, int* flags,
          double* work, cplx* trail) {
  FISDF_CHECK(n > 0 && batch > 0 && rmax > 0 && rmax <= n, "pchol: bad sizes");
  FISDF_CHECK(batch < 65536, "pchol: batch too large");
  double* thr = work;                  // batch
  double* pval = work + batch;         // batch * rmax
  const int nt = 1024;
  hipLaunchKernelGGL(pchol_init, dim3(batch), dim3(nt), 0, s, A, lda, sA, n, rmax, tol_rel,
                     tol_abs, piv, pval, rank, d, flags, thr);
  FISDF_HIP(hipGetLastError());
  if (n <= PB_THREADS) {
    // blocked: trailing copy W of A, panels of NB pivots, batched ZGEMM trailing updates
    constexpr int NB = 32;
    const long nn = (long)n * n;
    cplx* W = trail;  // the caller's (pchol_trail_elems): no stream-ordered pool memory
    FISDF_CHECK(W != nullptr, "pchol: trailing-update workspace missing");
    FISDF_HIP(hipMemcpy2DAsync(W, sizeof(cplx) * n, A, sizeof(cplx) * lda, sizeof(cplx) * n,
                               (size_t)n * batch, hipMemcpyDeviceToDevice, s));
    if (sA != (long)n * lda) {  // batch stride differs from a packed copy: copy per matrix
      for (int bb = 0; bb < batch; ++bb)
        FISDF_HIP(hipMemcpy2DAsync(W + bb * nn, sizeof(cplx) * n, A + bb * sA, sizeof(cplx) * lda,
                                   sizeof(cplx) * n, n, hipMemcpyDeviceToDevice, s));
    }
    const cplx mone = cmk(-1, 0), one = cmk(1, 0);
    for (int j0 = 0; j0 < rmax; j0 += NB) {
      hipLaunchKernelGGL(pchol_panel<NB>, dim3(batch), dim3(PB_THREADS), 0, s, W, nn, n, rmax, j0,
                         L, piv, rank, d, flags, thr);
      FISDF_HIP(hipGetLastError());
      const int kc = std::min(NB, rmax - j0);
      if (j0 + kc < rmax)  // W -= L[:, j0:j0+kc] L[:, j0:j0+kc]^H
        FISDF_TRY(zgemm(s, OP_N, OP_C, n, n, kc, mone, L + j0, rmax, (long)n * rmax, L + j0, rmax,
                        (long)n * rmax, one, W, n, nn, batch));
    }
    return 0;
  }
  const int rows_per_block = 4;
  dim3 g((n + rows_per_block - 1) / rows_per_block, batch);
  for (int j = 0; j < rmax; ++j) {
    hipLaunchKernelGGL(pchol_step, g, dim3(64 * rows_per_block), 0, s, A, lda, sA, n, rmax, j,
                       piv, pval, L, d, flags);
    hipLaunchKernelGGL(pchol_pick, dim3(batch), dim3(nt), 0, s, n, rmax, j, piv, pval, rank, d,
                       flags, thr);
  }
  FISDF_HIP(hipGetLastError());
  return 0;
}

// Unpivoted blocked Cholesky of batch n x n Hermitian matrices W (in place, ld n, batch stride
// n*n; lower triangle = L on return).  fail[b] = 1 if a pivot <= tol_rel*max(diag) (the caller
// falls back to pchol); piv = identity, rank = n (0 if failed).  work: batch*(4096 cplx) +
// batch doubles.
int chol_unpivoted(hipStream_t s, cplx* W, int n, int batch, double tol_rel, int* piv, int* rank,
                   int* fail, cplx* work) {
  FISDF_CHECK(n > 0 && batch > 0, "chol_unpivoted: bad sizes");
  const long nn = (long)n * n;
  cplx* Linv = work;
  double* thr = (double*)(work + (long)batch * 4096);
  hipLaunchKernelGGL(diag_max_kernel, dim3(batch), dim3(256), 0, s, W, n, nn, tol_rel, thr, fail);
  FISDF_HIP(hipGetLastError());
  const cplx one = cmk(1, 0), zero = cmk(0, 0);
  for (int b0 = 0; b0 < n; b0 += 64) {
    const int m = std::min(64, n - b0), b1 = b0 + m;
    hipLaunchKernelGGL(chol_diag_kernel, dim3(batch), dim3(256), 0, s, W, n, nn, b0, m, thr, fail,
                       Linv);
    FISDF_HIP(hipGetLastError());
    if (b1 < n) {
      // panel: W[b1:, b0:b1] <- W[b1:, b0:b1] L_bb^{-H}  (in place: one N tile, rows per WG)
      FISDF_TRY(zgemm(s, OP_N, OP_C, n - b1, m, m, one, W + (long)b1 * n + b0, n, nn, Linv, 64,
                      4096, zero, W + (long)b1 * n + b0, n, nn, batch));
      // trailing: W[b1:, b1:] -= P P^H (Hermitian: lower tiles + mirror)
      FISDF_TRY(herk_batched(s, n - b1, m, -1.0, W + (long)b1 * n + b0, n, nn, 1.0,
                             W + (long)b1 * n + b1, n, nn, batch));
    }
  }
  hipLaunchKernelGGL(chol_finish_kernel, dim3(batch), dim3(256), 0, s, n, piv, rank, fail);
  FISDF_HIP(hipGetLastError());
  return 0;
}

// selection: pivots of the real Gram x4 = Re(X2)^2 * scale (n x n, X2 complex); piv/rank
// device; work = W (n*n doubles) + L panel (n*16) + d (n) + thr; flags (1 int).  Returns 1 in
// *handled when n fits the register panel (n <= 4096), else 0 (caller uses pchol).
// FISDF_SEL_COOP=0 selects the blocked single-CU path (read per call: tests compare the two)
bool select_coop_enabled() {
  const char* e = getenv("FISDF_SEL_COOP");
  return !(e && e[0] == '0');
}

// Launch of a grid whose workgroups wait on each other (the selection kernels): every workgroup
// must be resident at once.  Default (round 6) below the HIP 7.2 runtime (torch's bundled 7.0,
// the mirror and bench.py): a plain launch after the occupancy check (the same residency,
// MI355X_MICROARCH.md); from 7.2 on (the torch-free C-ABI) hipLaunchCooperativeKernel, which is
// faster there; FISDF_COOP_LAUNCH=0/1 forces either.  Why the plain launch where it is as fast
// (profiles/r05/rocprof_exit/README.txt, profiles/r06/lanes/README.txt):
//  * a process that made one cooperative launch SIGSEGVs in its exit handlers under rocprofv3
//    (ROCm 7.2; a one-kernel control program reproduces it); the plain launch exits cleanly;
//  * concurrent first cooperative launches from several host threads (fisdf_group's ranks) each
//    create the device's cooperative queue (three "cooperative: 1" queue creations in the
//    runtime log for three rank threads), which the runtime's exit handlers then tear down
//    badly (SIGSEGV in libhsa-runtime64 under libamdhip64's atexit, main thread);
//  * what made the plain launch slower (the two fit lanes serialised: C3 90 vs 81 ms/step) is
//    the order the runtime creates hardware queues in, not the launch: the cooperative queue is
//    created between the context stream's queue and the side / aux streams' ones, and one
//    padding stream in that place (ensure_side, api.hip) gives the plain launch the same step
//    time (80.6-80.7 ms either way, interleaved on one box).
bool coop_launch_enabled() {
  static const bool coop = [] {
    const char* e = getenv("FISDF_COOP_LAUNCH");
    if (e) return e[0] == '1';
    // the plain launch (+ padding stream) matches the cooperative one on the ROCm 7.0 runtime
    // torch bundles (C3 80.6-80.7 ms either way) but not on the system 7.2 runtime the torch-free
    // C-ABI runs on (83.3 vs 79.5 ms/step, padding 0-2 streams: 82.9-83.5; profiles/r06/capi/):
    // cooperative from 7.2 on
    int v = 0;
    if (hipRuntimeGetVersion(&v) != hipSuccess) return false;
    return v / 10000000 > 7 || (v / 10000000 == 7 && (v / 100000) % 100 >= 2);
  }();
  return coop;
}

hipError_t launch_coresident(const void* fn, int grid, int threads, void** args, size_t lds,
                             hipStream_t s, int ncu) {
  if (coop_launch_enabled()) {
    // one cooperative launch at a time in the process: concurrent ones from several host threads
    // (fisdf_group's ranks) left the runtime crashing in its exit handlers.  FISDF_COOP_MUTEX=0
    // (diagnosis only, tools/crash_probe.sh) drops the lock to reproduce that crash.
    static const bool serial = [] {
      const char* e = getenv("FISDF_COOP_MUTEX");
      return !(e && e[0] == '0');
    }();
    static std::mutex mu;
    if (!serial)
      return hipLaunchCooperativeKernel(fn, dim3(grid), dim3(threads), args, (unsigned)lds, s);
    std::lock_guard<std::mutex> lk(mu);
    return hipLaunchCooperativeKernel(fn, dim3(grid), dim3(threads), args, (unsigned)lds, s);
  }
  int per_cu = 0;
  const hipError_t oe = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, lds);
  if (oe != hipSuccess) return oe;
  if ((long)per_cu * ncu < grid) return hipErrorCooperativeLaunchTooLarge;
  return hipLaunchKernel(fn, dim3(grid), dim3(threads), args, lds, s);
}

// launches pchol_select_coop when the owned L rows fit the LDS of a co-resident grid;
// *handled = false (nothing enqueued that matters) otherwise or if the launch is refused.  No
// host synchronisation: *err_dev receives the device address of the kernel's error flag (a
// stalled step), which the caller reads back with the pivots and the rank in one copy.
int pchol_select_coop_launch(hipStream_t s, const cplx* X2, double scale, int n, int rmax,
                             double tol, int* piv, int* rank, double* work, bool* handled,
                             const int** err_dev, int* progress) {
  *handled = false;
  *err_dev = nullptr;
  if (!select_coop_enabled() || n < 64) return 0;
  static const int ncu = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return v;
  }();
  // read per call (the GPU tests force the split path on small cases): FISDF_SEL_LDS_COLS=k
  // keeps at most k columns of the owned L rows in LDS
  const char* ek = getenv("FISDF_SEL_LDS_COLS");
  const int kcap = ek ? atoi(ek) : 0;
  constexpr size_t kLds = 150 * 1024;
  // 128 workgroups: the per-pivot time is flat from 128 to 256 (cross-XCD round trips)
  // FISDF_SEL_WGS=g caps the grid (experiments: the exchange's cost against its poller count)
  const char* eg = getenv("FISDF_SEL_WGS");
  int G = std::min({eg ? std::max(1, atoi(eg)) : 128, ncu, (n + 7) / 8});
  if (G < 1) return 0;
  int RW = (n + G - 1) / G;
  G = (n + RW - 1) / RW;
  int K = rmax, tpr = 8;
  size_t lds = sizeof(double) * ((size_t)RW * rmax + rmax + 2 * (size_t)RW);
  if (lds > kLds || kcap > 0) {
    // the owned L rows do not fit: one workgroup per CU, the first K columns in LDS and the
    // rest read back (agent-coherent) from the global L
    G = std::min(ncu, (n + 7) / 8);
    RW = (n + G - 1) / G;
    G = (n + RW - 1) / RW;
    K = (int)(((long)(kLds / sizeof(double)) - rmax - 2L * RW) / RW);
    if (kcap > 0) K = std::min(K, kcap);
    if (K < 16) return 0;
    K = std::min(K, rmax);
    tpr = 8;
    lds = sizeof(double) * ((size_t)RW * K + rmax + 2 * (size_t)RW);
  }
  if (lds > kLds || RW > SC_MAXRW) return 0;
  // threads per owned row: the most (a power of two, <= 32) that the workgroup holds
  while (tpr < 32 && RW * tpr * 2 <= SC_THREADS) tpr *= 2;
  // scratch in the caller's work area (n*n doubles): records, global L, error flag
  u32x4* rec = (u32x4*)work;
  double* Lg = work + 4 * G;
  int* err = (int*)(Lg + (long)n * rmax);
  if ((long)(4 * G + (long)n * rmax + 2) > (long)n * n) return 0;
  FISDF_HIP(hipMemsetAsync(rec, 0, 2 * G * sizeof(u32x4), s));
  FISDF_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
  FISDF_HIP(hipMemsetAsync(rank, 0, sizeof(int), s));
  FISDF_TRY(func_max_lds((const void*)pchol_select_coop, (int)kLds));
  // FISDF_SEL_PROF=1: per-step phase timestamps of workgroup 0 (timing probe), printed below;
  // one 8192-step buffer per device, the probe off for longer selections
  constexpr int kProfSteps = 8192;
  static unsigned long long* prof[64] = {};
  int pdev = 0;
  FISDF_HIP(hipGetDevice(&pdev));
  const bool want_prof = getenv("FISDF_SEL_PROF") != nullptr && rmax <= kProfSteps && pdev < 64;
  if (want_prof && !prof[pdev])
    FISDF_HIP(hipMalloc(&prof[pdev], sizeof(unsigned long long) * 4 * kProfSteps));
  unsigned long long* profp = want_prof ? prof[pdev] : nullptr;
  if (profp) FISDF_HIP(hipMemsetAsync(profp, 0, sizeof(unsigned long long) * 4 * rmax, s));
  void* args[] = {(void*)&X2, (void*)&scale, (void*)&n,   (void*)&rmax, (void*)&tol, (void*)&RW,
                  (void*)&K,   (void*)&tpr,   (void*)&piv, (void*)&rank, (void*)&rec, (void*)&Lg,
                  (void*)&err, (void*)&profp, (void*)&progress};
  const hipError_t e =
      launch_coresident((const void*)pchol_select_coop, G, SC_THREADS, args, lds, s, ncu);
  if (e != hipSuccess) {  // refused (e.g. not co-resident): the caller's blocked path runs
    (void)hipGetLastError();
    return 0;
  }
  *err_dev = err;
  *handled = true;
  if (profp) {
    std::vector<unsigned long long> h(4 * (size_t)rmax);
    FISDF_HIP(hipMemcpyAsync(h.data(), profp, sizeof(unsigned long long) * h.size(),
                             hipMemcpyDeviceToHost, s));
    FISDF_HIP(hipStreamSynchronize(s));
    double ph[4] = {0, 0, 0, 0};
    int cnt = 0;
    for (int j = 1; j < rmax; ++j) {
      const unsigned long long* a = &h[4 * (size_t)j];
      const unsigned long long prev = h[4 * (size_t)(j - 1) + 3];
      if (!a[0] || !a[1] || !a[2] || !a[3] || !prev) continue;
      ph[0] += (double)(a[0] - prev);  // step start -> record posted (the post's reduction)
      ph[1] += (double)(a[1] - a[0]);  // posted -> winner known (poll + block arg-max)
      ph[2] += (double)(a[2] - a[1]);  // gather of L[p, :j] and x4[p, rows]
      ph[3] += (double)(a[3] - a[2]);  // column j
      ++cnt;
    }
    if (cnt)  // s_memrealtime: 100 MHz
      fprintf(stderr, "select coop G=%d RW=%d: per step (us) post %.2f, exchange %.2f, gather %.2f, column %.2f\n",
              G, RW, ph[0] / cnt / 100.0, ph[1] / cnt / 100.0, ph[2] / cnt / 100.0, ph[3] / cnt / 100.0);
  }
  return 0;
}

// FISDF_SEL_MODE (read per call: the GPU tests compare the paths): "batch" tries the
// batched-candidate kernel, then the cooperative one; "coop" starts at the cooperative kernel;
// "blocked" (or FISDF_SEL_COOP=0) runs the blocked single-CU path only.  Default: batch from
// 800 pivots on (C4, 1000 pivots: 5.3 vs 6.4 ms), coop below (C3, 600: 4.36 vs 4.41 ms, a tie;
// profiles/r05/selection/README.txt)
int select_mode(int rmax) {
  const char* e = getenv("FISDF_SEL_MODE");
  if (!select_coop_enabled()) return 2;
  if (!e) return rmax >= 800 ? 0 : 1;
  if (!strcmp(e, "coop")) return 1;
  if (!strcmp(e, "blocked")) return 2;
  return 0;
}

// launches pchol_select_batch when the owned rows fit (n <= 4096, 16 rows per workgroup on at
// most ncu - 1 workgroups, rmax <= 1024); *handled = false otherwise or if the launch is refused.
int pchol_select_batch_launch(hipStream_t s, const cplx* X2, double scale, int n, int rmax,
                              double tol, int* piv, int* rank, double* work, bool* handled,
                              const int** err_dev) {
  *handled = false;
  *err_dev = nullptr;
  if (n < 2 * SB_M || n > SB_GR * SB_THREADS || rmax > 4096) return 0;
  static const int ncu = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return v;
  }();
  const int RW = 16;
  const int G = (n + RW - 1) / RW;
  if (G + 1 > ncu) return 0;
  constexpr size_t kLds = 150 * 1024;
  const size_t owner = sizeof(double) * (8 * 256 + SB_M * SB_S + 2 * 16 * SB_S + (size_t)RW * rmax);
  const size_t leader = sizeof(double) * (3 * 8 * 256 + SB_M * SB_M + 64 + SB_M * SB_S + 16);
  const size_t lds = std::max(owner, leader);
  if (lds > kLds) return 0;
  // scratch in the caller's work area (n*n doubles): granules, publish area, global L, error flag
  u32x4* ddg = (u32x4*)work;
  const long pub_d = 2L * SB_NPUB;
  u32x4* pub = (u32x4*)(work + 2L * n);
  double* Lg = work + 2L * n + pub_d;
  int* err = (int*)(Lg + (long)n * rmax);
  if (2L * n + pub_d + (long)n * rmax + 2 > (long)n * n) return 0;
  FISDF_HIP(hipMemsetAsync(ddg, 0, sizeof(u32x4) * n, s));
  FISDF_HIP(hipMemsetAsync(pub, 0, sizeof(u32x4) * SB_NPUB, s));  // no stale batch words
  FISDF_HIP(hipMemsetAsync(err, 0, sizeof(int), s));
  FISDF_HIP(hipMemsetAsync(rank, 0, sizeof(int), s));
  FISDF_TRY(func_max_lds((const void*)pchol_select_batch, (int)kLds));
  // FISDF_SEL_PROF=1: per-batch phase timestamps of the leader (timing probe), printed below
  constexpr int kProfBatches = 8192;
  static unsigned long long* prof[64] = {};
  int pdev = 0;
  FISDF_HIP(hipGetDevice(&pdev));
  const bool want_prof = getenv("FISDF_SEL_PROF") != nullptr && pdev < 64;
  if (want_prof && !prof[pdev])
    FISDF_HIP(hipMalloc(&prof[pdev], sizeof(unsigned long long) * 4 * kProfBatches));
  unsigned long long* profp = want_prof ? prof[pdev] : nullptr;
  const int nb_cap = std::min(rmax, kProfBatches);
  if (profp) FISDF_HIP(hipMemsetAsync(profp, 0, sizeof(unsigned long long) * 4 * nb_cap, s));
  int rw = RW;
  void* args[] = {(void*)&X2,  (void*)&scale, (void*)&n,   (void*)&rmax, (void*)&tol,
                  (void*)&rw,  (void*)&piv,   (void*)&rank, (void*)&ddg, (void*)&pub,
                  (void*)&Lg,  (void*)&err,   (void*)&profp};
  const hipError_t e =
      launch_coresident((const void*)pchol_select_batch, G + 1, SB_THREADS, args, lds, s, ncu);
  if (e != hipSuccess) {  // refused (e.g. not co-resident): the caller's next path runs
    (void)hipGetLastError();
    return 0;
  }
  *err_dev = err;
  *handled = true;
  if (profp) {
    std::vector<unsigned long long> h(4 * (size_t)nb_cap);
    FISDF_HIP(hipMemcpyAsync(h.data(), profp, sizeof(unsigned long long) * h.size(),
                             hipMemcpyDeviceToHost, s));
    FISDF_HIP(hipStreamSynchronize(s));
    double ph[4] = {0, 0, 0, 0};
    int cnt = 0, nb = 0;
    for (int b = 0; b < nb_cap; ++b) {
      const unsigned long long* a = &h[4 * (size_t)b];
      if (!a[0]) break;
      ++nb;
      if (b == 0 || !a[1] || !a[2] || !a[3]) continue;
      const unsigned long long prev = h[4 * (size_t)(b - 1) + 3];
      ph[0] += (double)(a[0] - prev);  // published -> owners' update, gather, candidates
      ph[1] += (double)(a[1] - a[0]);  // candidates' residual block (MFMA Gram)
      ph[2] += (double)(a[2] - a[1]);  // greedy steps
      ph[3] += (double)(a[3] - a[2]);  // publish
      ++cnt;
    }
    if (cnt)  // s_memrealtime: 100 MHz
      fprintf(stderr, "select batch G=%d RW=%d: %d batches, per batch (us) owners+gather+select "
                      "%.2f, gram %.2f, steps %.2f, publish %.2f\n",
              G, RW, nb, ph[0] / cnt / 100.0, ph[1] / cnt / 100.0, ph[2] / cnt / 100.0,
              ph[3] / cnt / 100.0);
  }
  return 0;
}

int pchol_select_real(hipStream_t s, const cplx* X2, double scale, int n, int rmax, double tol,
                      int* piv, int* rank, double* work, int* flags, bool* handled,
                      bool allow_coop, const int** coop_err, int* progress, bool* publishes) {
  *handled = false;
  *coop_err = nullptr;
  if (publishes) *publishes = false;
  if (rmax <= 0) return 0;
  const int mode = select_mode(rmax);
  if (allow_coop && mode == 0) {
    FISDF_TRY(pchol_select_batch_launch(s, X2, scale, n, rmax, tol, piv, rank, work, handled,
                                        coop_err));
    if (*handled) return 0;
  }
  if (allow_coop && mode <= 1) {
    FISDF_TRY(pchol_select_coop_launch(s, X2, scale, n, rmax, tol, piv, rank, work, handled,
                                       coop_err, progress));
    if (*handled) {
      if (publishes) *publishes = progress != nullptr;
      return 0;
    }
  }
  if (n > 8 * PR_THREADS) return 0;
  double* W = work;
  double* Lpan = W + (long)n * n;
  double* d = Lpan + (long)n * 16;
  double* thr = d + n;
  FISDF_HIP(hipMemsetAsync(flags, 0, sizeof(int), s));
  FISDF_HIP(hipMemsetAsync(rank, 0, sizeof(int), s));
  const long n2 = (long)n * n;
  hipLaunchKernelGGL(real_square_scale_kernel, dim3((unsigned)std::min<long>((n2 + 255) / 256, 8192)),
                     dim3(256), 0, s, X2, scale, W, d, n2, n);
  FISDF_HIP(hipGetLastError());
  const int rpt = (n + PR_THREADS - 1) / PR_THREADS;
  const int nt = (n + 63) / 64;
  const dim3 ug(nt * (nt + 1) / 2);
#define FISDF_PR(R, NBv)                                                                         for (int j0 = 0; j0 < rmax; j0 += NBv) {                                                          hipLaunchKernelGGL((pchol_real_panel<R, NBv>), dim3(1), dim3(PR_THREADS), 0, s, W, n, rmax,                        j0, tol, Lpan, piv, rank, d, flags, thr);                                   if (j0 + NBv < rmax)                                                                             hipLaunchKernelGGL((syrk_real_update<NBv>), ug, dim3(256), 0, s, W, n, Lpan, flags);        }
  if (rpt <= 2) { FISDF_PR(2, 16) }
  else if (rpt <= 4) { FISDF_PR(4, 16) }
  else if (rpt <= 7) { FISDF_PR(7, 12) }
  else { FISDF_PR(8, 8) }
#undef FISDF_PR
  FISDF_HIP(hipGetLastError());
  *handled = true;
  return 0;
}

}  // namespace fisdf
