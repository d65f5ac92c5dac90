// Small device kernels around the GEMM / FFT / Cholesky engines:
// pivot-order factor gather, diagonal-block triangular inverses, blocked TRSM driver,
// Coulomb weights, the y-build square, scatter/gather and J/K element-wise steps.
#include "common.h"
#include "linalg.h"

#include <cmath>

namespace fisdf {

namespace {

// Lp[b][s][t] = L[b][piv[b][s]][t] (t <= s < r_b), zero above the diagonal; identity beyond
// the rank.  L: (batch, n, rmax), piv: (batch, rmax), Lp: (batch, rpad, rpad).
__global__ void gather_lp_kernel(const cplx* __restrict__ L, int n, int rmax,
                                 const int* __restrict__ piv, const int* __restrict__ rank,
                                 int rpad, cplx* __restrict__ Lp) {
  const int b = blockIdx.y;
  const int r = rank[b];
  L += (long)b * n * rmax;
  piv += (long)b * rmax;
  Lp += (long)b * rpad * rpad;
  long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= (long)rpad * rpad) return;
  int s = (int)(e / rpad), t = (int)(e % rpad);
  cplx v = cmk(0, 0);
  if (s < r && t < r) {
    if (t <= s) v = L[(long)piv[s] * rmax + t];
  } else if (s == t) {
    v = cmk(1, 0);
  }
  Lp[e] = v;
}

// inverse of each nb x nb lower-triangular diagonal block of Lp (r x r, ld = ldl)
__global__ __launch_bounds__(64) void trinv_blocks_kernel(const cplx* __restrict__ Lp, int r,
                                                          int ldl, long sL, int nb, long sLi,
                                                          cplx* __restrict__ Linv) {
  __shared__ cplx Ls[64][65];
  __shared__ cplx Xs[64][65];
  Lp += blockIdx.y * sL;
  Linv += blockIdx.y * sLi;
  const int blk = blockIdx.x;
  const int b0 = blk * nb;
  const int m = min(nb, r - b0);
  const int j = threadIdx.x;
  for (int i = 0; i < m; ++i)
    if (j < m) Ls[i][j] = Lp[(long)(b0 + i) * ldl + b0 + j];
  __syncthreads();
  if (j < m) {
    for (int i = 0; i < m; ++i) {
      cplx s = cmk(i == j ? 1.0 : 0.0, 0.0);
      for (int t = j; t < i; ++t) s = csub(s, cmul(Ls[i][t], Xs[t][j]));
      // divide by L_ii
      cplx d = Ls[i][i];
      double den = d.x * d.x + d.y * d.y;
      Xs[i][j] = i < j ? cmk(0, 0) : cmk((s.x * d.x + s.y * d.y) / den, (s.y * d.x - s.x * d.y) / den);
    }
  }
  __syncthreads();
  cplx* out = Linv + (long)blk * nb * nb;
  for (int i = 0; i < nb; ++i)
    if (j < nb) out[i * nb + j] = (i < m && j < m) ? Xs[i][j] : cmk(i == j ? 1.0 : 0.0, 0.0);
}

// Same inverses for the partition [0, s0), [s0, s0+64), ... written straight into the
// diagonal blocks of Q (ld = ldq) — the block-row operator of trsm_merged_batched.  Register-blocked
// like chol_diag_kernel's inverse phase: 256 threads, thread t owns the 4 x 4 block (rows
// 4 (t >> 4), cols 4 (t & 15)) of X = L_bb^{-1}, built by right-looking forward substitution
// on the identity (row k final once rows < k are subtracted, then scaled by 1 / L_kk) with one
// barrier per row.  (The one-wave column-serial version ran 6 ms at C3 beside the y build.)
__global__ __launch_bounds__(256) void trinv_into_kernel(const cplx* __restrict__ Lp, int r,
                                                         int ldl, long sL, int s0,
                                                         cplx* __restrict__ Q, int ldq, long sQ) {
  __shared__ cplx Ls[64][65];
  __shared__ cplx vec[2][64];
  Lp += blockIdx.y * sL;
  Q += blockIdx.y * sQ;
  const int blk = blockIdx.x;
  const int b0 = blk == 0 ? 0 : s0 + (blk - 1) * 64;
  const int m = blk == 0 ? s0 : min(64, r - b0);
  const int t = threadIdx.x, bi = t >> 4, bj = t & 15, r0 = bi * 4, c0 = bj * 4;
  for (int e = t; e < 64 * 64; e += 256) {
    const int i = e >> 6, j = e & 63;
    Ls[i][j] = (i < m && j <= i) ? Lp[(long)(b0 + i) * ldl + b0 + j] : cmk(0, 0);
  }
  __syncthreads();
  cplx x[4][4];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr)
#pragma unroll
    for (int c = 0; c < 4; ++c) x[rr][c] = cmk(r0 + rr == c0 + c ? 1.0 : 0.0, 0.0);
  // k = 4 kb + kr with kr unrolled: register arrays keep compile-time indices
  for (int kb = 0; 4 * kb < m; ++kb) {
#pragma unroll
    for (int kr = 0; kr < 4; ++kr) {
      const int k = 4 * kb + kr, p = kr & 1;
      if (k >= m) break;
      if (bi == kb) {
        const cplx d = Ls[k][k];
        const double den = d.x * d.x + d.y * d.y;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const cplx v = x[kr][c];
          x[kr][c] = cmk((v.x * d.x + v.y * d.y) / den, (v.y * d.x - v.x * d.y) / den);
          vec[p][c0 + c] = x[kr][c];
        }
      }
      __syncthreads();
      cplx xk[4], lik[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) xk[c] = vec[p][c0 + c];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) lik[rr] = (r0 + rr > k && r0 + rr < m) ? Ls[r0 + rr][k] : cmk(0, 0);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int c = 0; c < 4; ++c) x[rr][c] = csub(x[rr][c], cmul(lik[rr], xk[c]));
    }
  }
#pragma unroll
  for (int rr = 0; rr < 4; ++rr)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int i = r0 + rr, j = c0 + c;
      if (i < m && j < m) Q[(long)(b0 + i) * ldq + b0 + j] = x[rr][c];
    }
}

// W[b][piv[b][s]][piv[b][t]] = Wpp[b][s][t] for s,t < rank[b]   (W zeroed beforehand)
__global__ void scatter_w_kernel(const cplx* __restrict__ Wpp, int ldw, long sW,
                                 const int* __restrict__ piv, const int* __restrict__ rank,
                                 cplx* __restrict__ W, int nip) {
  const int b = blockIdx.y;
  const int r = rank[b];
  long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= (long)r * r) return;
  int s = (int)(e / r), t = (int)(e % r);
  const int* p = piv + (long)b * nip;
  W[(long)b * nip * nip + (long)p[s] * nip + p[t]] = Wpp[b * sW + (long)s * ldw + t];
}

__global__ void conj_transpose_kernel(const cplx* __restrict__ A, int n, long sA,
                                      cplx* __restrict__ B) {
  const int b = blockIdx.y;
  long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= (long)n * n) return;
  int i = (int)(e / n), j = (int)(e % n);
  B[b * sA + (long)j * n + i] = cconj(A[b * sA + e]);
}

// sqrt(coulG(k+G) * scale); PySCF get_coulG (exxdiv=None, wrap_around=True) restated
// omega != 0: PySCF's range-separated kernels, omega > 0 the long-range erf(w r)/r
// (x exp(-|k+G|^2 / 4w^2)), omega < 0 the short-range erfc(|w| r)/r (x (1 - exp(...)), and its
// finite |k+G| = 0 limit pi / w^2)
__global__ void coulg_weight_kernel(int n0, int n1, int n2, CellGeom g, double kx, double ky,
                                    double kz, double scale, int take_sqrt, double omega,
                                    double* __restrict__ w) {
  long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  long ngrid = (long)n0 * n1 * n2;
  if (e >= ngrid) return;
  int i2 = (int)(e % n2), i1 = (int)((e / n2) % n1), i0 = (int)(e / ((long)n1 * n2));
  int ns[3] = {n0, n1, n2};
  int is[3] = {i0, i1, i2};
  double G[3] = {0, 0, 0};
  for (int a = 0; a < 3; ++a) {
    int m = is[a] < (ns[a] + 1) / 2 ? is[a] : is[a] - ns[a];
    for (int c = 0; c < 3; ++c) G[c] += m * g.b[a][c];
  }
  double k[3] = {kx, ky, kz};
  bool nonzero_k = fabs(kx) + fabs(ky) + fabs(kz) > 1e-9;
  double kG[3];
  for (int c = 0; c < 3; ++c) kG[c] = nonzero_k ? k[c] + G[c] : G[c];
  bool boundary = false;
  if (nonzero_k) {
    const double twopi = 6.283185307179586;
    double red[3];
    int edge[3];
    for (int a = 0; a < 3; ++a) {
      double h = (double)(ns[a] / 2) + 0.5;
      double r = (kG[0] * g.a[a][0] + kG[1] * g.a[a][1] + kG[2] * g.a[a][2]) / (twopi * h);
      r = rint(r * 1e9) / 1e9;
      red[a] = r;
      edge[a] = (int)r;  // truncation, as numpy astype(int)
    }
    for (int a = 0; a < 3; ++a) {
      if (red[a] == 1.0 || red[a] == -1.0) boundary = true;
      double h = (double)(ns[a] / 2) + 0.5;
      for (int c = 0; c < 3; ++c) {
        if (edge[a] == 1) kG[c] -= 2 * h * g.b[a][c];
        if (edge[a] == -1) kG[c] += 2 * h * g.b[a][c];
      }
    }
  }
  double g2 = kG[0] * kG[0] + kG[1] * kG[1] + kG[2] * kG[2];
  double cg = (g2 == 0.0 || boundary) ? 0.0 : 4.0 * 3.141592653589793 / g2;
  if (omega != 0.0 && !boundary) {
    const double f = exp(-0.25 * g2 / (omega * omega));
    if (omega > 0.0)
      cg *= f;
    else
      cg = g2 == 0.0 ? 3.141592653589793 / (omega * omega) : cg * (1.0 - f);
  }
  double v = cg * scale;
  w[e] = take_sqrt ? sqrt(v) : v;
}

// out[e] = (Re in[e])^2 + 0i ; records max |Im in| (bit pattern of a non-negative double)
__global__ void square_real_kernel(const cplx* __restrict__ in, cplx* __restrict__ out, long n,
                                   unsigned long long* __restrict__ maximag) {
  double mi = 0.0;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    cplx v = in[e];
    out[e] = cmk(v.x * v.x, 0.0);
    mi = fmax(mi, fabs(v.y));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mi = fmax(mi, __shfl_xor(mi, o, 64));
  if ((threadIdx.x & 63) == 0 && maximag) atomicMax(maximag, (unsigned long long)__double_as_longlong(mi));
}

// out[R,I,J] = scale * Re(in[R,I,J]) (+0i);  records max |Im|
// rho[x, I] = scale * sum_{k,n} T[x,k,I,n] conj(X[k,I,n]): one wave per (x, I), lanes over the
// (k, n) pairs, fixed-order shuffle reduction (one thread per (x, I) left 10 waves on the chip)
__global__ __launch_bounds__(64) void rho_diag_kernel(const cplx* __restrict__ T,
                                                      const cplx* __restrict__ X, int nset, int nk,
                                                      int nip, int nao, double scale,
                                                      cplx* __restrict__ rho) {
  const long e = blockIdx.x;
  if (e >= (long)nset * nip) return;
  const int x = (int)(e / nip), I = (int)(e % nip), lane = threadIdx.x;
  double sr = 0, si = 0;
  for (int t = lane; t < nk * nao; t += 64) {
    const int k = t / nao, n = t - k * nao;
    const cplx a = T[(((long)x * nk + k) * nip + I) * nao + n], b = X[((long)k * nip + I) * nao + n];
    sr += a.x * b.x + a.y * b.y;
    si += a.y * b.x - a.x * b.y;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sr += __shfl_xor(sr, o, 64);
    si += __shfl_xor(si, o, 64);
  }
  if (lane == 0) rho[e] = cmk(sr * scale, si * scale);
}

// Xv[x,k,I,n] = v[x,I] * X[k,I,n]
// Xv[x][k][I][m] = v[x][I] * X[k][i0+I][m] for I < nb (X: nip rows per k)
__global__ void scale_rows_kernel(const cplx* __restrict__ X, const cplx* __restrict__ v, int nset,
                                  int nk, int nip, int i0, int nb, int nao, cplx* __restrict__ Xv) {
  long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  long per = (long)nk * nb * nao;
  if (e >= (long)nset * per) return;
  int x = (int)(e / per);
  long r = e % per;
  int k = (int)(r / ((long)nb * nao));
  int I = (int)((r / nao) % nb), m = (int)(r % nao);
  Xv[e] = cmul(v[(long)x * nb + I], X[((long)k * nip + i0 + I) * nao + m]);
}

// ---- y build, k-mesh part (fftisdf.py:79-85) -----------------------------------------
// Phi = exp(i T_R.k)/sqrt(nk) is separable over the k-mesh axes, so
// fx_s = Phi fx_k and y_k = Phi^T y_s are 3-D inverse-sign DFTs of length kmesh along the
// k index of every (I, g) column.  One workgroup takes CT columns: the nk x CT tile is
// staged in LDS (coalesced over columns), transformed axis by axis (direct n_a-point
// DFTs, n_a <= 16), squared (real part; max|Im| monitored = fftisdf.py:81), transformed
// again, and the q-shard rows are written straight into yT[q-q0][I][g] — one HBM pass
// instead of two dense nk x nk GEMMs with an intermediate.
constexpr int KM_MAXN = 16;

__device__ void kmesh_axis_dft(cplx* T, int CT, int ld, int nk, int na, int stride,
                               const cplx* __restrict__ w, int tid, int nthr) {
  // lines: all k with k_a == 0 along this axis, for each column
  const int nlines = nk / na;
  const int items = nlines * CT;
  for (int it = tid; it < items; it += nthr) {
    const int c = it % CT;
    const int line = it / CT;
    // base k index of the line: decompose line over the other axes (k = hi*na*stride + j*stride + lo)
    const int lo = line % stride;
    const int hi = line / stride;
    const int base = hi * na * stride + lo;
    cplx out[KM_MAXN];
#pragma unroll
    for (int x = 0; x < KM_MAXN; ++x) {
      cplx acc = cmk(0, 0);
      if (x < na) {
        for (int j = 0; j < na; ++j)
          acc = cadd(acc, cmul(T[(base + j * stride) * ld + c], w[(x * j) % na]));
      }
      out[x] = acc;
    }
#pragma unroll
    for (int x = 0; x < KM_MAXN; ++x)
      if (x < na) T[(base + x * stride) * ld + c] = out[x];
  }
}

// index of -k on the k-mesh (k = (a*n1 + b)*n2 + c, ascending cartesian order)
__host__ __device__ constexpr int kmesh_partner(int k, int n0, int n1, int n2) {
  return (((n0 - k / (n1 * n2)) % n0) * n1 + (n1 - (k / n2) % n1) % n1) * n2 + (n2 - k % n2) % n2;
}
// time reversal: fx is stored for the representatives k <= -k only (36 of 64 at 4x4x4), in
// ascending k; the slot of representative k is the number of representatives below it
__host__ __device__ constexpr bool kmesh_is_rep(int k, int n0, int n1, int n2) {
  return k <= kmesh_partner(k, n0, n1, n2);
}
__host__ __device__ constexpr int kmesh_rep_slot(int k, int n0, int n1, int n2) {
  int s = 0;
  for (int j = 0; j < k; ++j) s += kmesh_is_rep(j, n0, n1, n2) ? 1 : 0;
  return s;
}

__global__ __launch_bounds__(256) void kmesh_y_kernel(
    const cplx* __restrict__ FX, long ncol, int nk, int n0, int n1, int n2,
    const int* __restrict__ qlist, int nq, int m, cplx* __restrict__ yT, long qs, long Is,
    long goff, int CT, int half,
    unsigned long long* __restrict__ mon) {
  extern __shared__ cplx sm[];
  cplx* w0 = sm;
  cplx* w1 = sm + KM_MAXN;
  cplx* w2 = sm + 2 * KM_MAXN;
  cplx* T = sm + 3 * KM_MAXN;
  int* src = (int*)(T + (long)nk * (CT + 1));  // FX slot of k (negated - 1: conj of that slot)
  const int ld = CT + 1;
  const int tid = threadIdx.x, nthr = blockDim.x;
  for (int k = tid; k < nk; k += nthr) {
    if (!half) {
      src[k] = k;
    } else {
      const int p = kmesh_partner(k, n0, n1, n2);
      src[k] = k <= p ? kmesh_rep_slot(k, n0, n1, n2) : -1 - kmesh_rep_slot(p, n0, n1, n2);
    }
  }
  const int ns[3] = {n0, n1, n2};
  for (int a = 0; a < 3; ++a) {
    cplx* w = a == 0 ? w0 : (a == 1 ? w1 : w2);
    for (int t = tid; t < ns[a]; t += nthr) {
      double s, cc;
      sincospi(2.0 * t / ns[a], &s, &cc);  // exp(+2 pi i t / n_a)
      w[t] = cmk(cc, s);
    }
  }
  __syncthreads();  // src is read by every thread's first tile load
  const double sc = 1.0 / sqrt((double)nk);
  const long ntiles = (ncol + CT - 1) / CT;
  // persistent over column tiles: twiddles once, U loads in flight per thread
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
  const long c0 = tile * CT;
  constexpr int U = 8;
  const int tot = nk * CT;
  for (int e0 = 0; e0 < tot; e0 += U * nthr) {
    cplx v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * nthr + tid;
      const int c = e % CT;
      const long col = c0 + c;
      const bool ok = e < tot && col < ncol;
      int k = ok ? src[e / CT] : 0;
      const bool mirror = k < 0;  // time reversal: fx_{-k} = conj(fx_k) of its representative
      if (mirror) k = -1 - k;
      v[u] = FX[ok ? (long)k * ncol + col : 0];
      if (!ok) v[u] = cmk(0, 0);
      if (mirror) v[u] = cconj(v[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * nthr + tid;
      if (e < tot) T[(e / CT) * ld + (e % CT)] = v[u];
    }
  }
  __syncthreads();
  // fx_s = Phi fx_k
  kmesh_axis_dft(T, CT, ld, nk, n0, n1 * n2, w0, tid, nthr);
  __syncthreads();
  kmesh_axis_dft(T, CT, ld, nk, n1, n2, w1, tid, nthr);
  __syncthreads();
  kmesh_axis_dft(T, CT, ld, nk, n2, 1, w2, tid, nthr);
  __syncthreads();
  // y_s = Re(fx_s)^2  (fx_s is real: fftisdf.py:81)
  double mi = 0.0;
  for (int e = tid; e < nk * CT; e += nthr) {
    const int k = e / CT, c = e % CT;
    cplx v = T[k * ld + c];
    const double re = v.x * sc;
    mi = fmax(mi, fabs(v.y * sc));
    T[k * ld + c] = cmk(re * re, 0.0);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mi = fmax(mi, __shfl_xor(mi, o, 64));
  if ((tid & 63) == 0 && mon) atomicMax(mon, (unsigned long long)__double_as_longlong(mi));
  __syncthreads();
  // y_k = Phi^T y_s  (Phi symmetric in R <-> k)
  kmesh_axis_dft(T, CT, ld, nk, n0, n1 * n2, w0, tid, nthr);
  __syncthreads();
  kmesh_axis_dft(T, CT, ld, nk, n1, n2, w1, tid, nthr);
  __syncthreads();
  kmesh_axis_dft(T, CT, ld, nk, n2, 1, w2, tid, nthr);
  __syncthreads();
  for (int e = tid; e < nq * CT; e += nthr) {
    const int qq = e / CT, c = e % CT;
    const long col = c0 + c;
    if (col < ncol) {
      const long I = col / m, g = col % m;
      cplx v = T[qlist[qq] * ld + c];
      yT[qq * qs + I * Is + goff + g] = cmk(v.x * sc, v.y * sc);
    }
  }
  __syncthreads();  // T is reloaded by the next tile
  }
}

// Register variant for the common k-meshes (compile-time N0 x N1 x N2): one thread per
// column holds all NK k-values, so the NK loads of a column are in flight together and the
// separable DFTs are straight-line code with compile-time twiddle indices.
template <int N, int S, int NK>
__device__ __forceinline__ void reg_axis_dft(cplx* v, const cplx* tw) {
#pragma unroll
  for (int hi = 0; hi < NK / (N * S); ++hi)
#pragma unroll
    for (int lo = 0; lo < S; ++lo) {
      cplx* p = v + hi * N * S + lo;
      if constexpr (N == 2) {
        const cplx a = p[0], b = p[S];
        p[0] = cadd(a, b);
        p[S] = csub(a, b);
      } else if constexpr (N == 4) {  // exp(+2 pi i xj/4): multiplications by +-i are swaps
        const cplx a = p[0], b = p[S], c = p[2 * S], d = p[3 * S];
        const cplx s0 = cadd(a, c), d0 = csub(a, c), s1 = cadd(b, d), d1 = csub(b, d);
        const cplx id1 = cmk(-d1.y, d1.x);  // i * (b - d)
        p[0] = cadd(s0, s1);
        p[S] = cadd(d0, id1);
        p[2 * S] = csub(s0, s1);
        p[3 * S] = csub(d0, id1);
      } else if constexpr (N > 1) {
        cplx u[N];
#pragma unroll
        for (int j = 0; j < N; ++j) u[j] = p[j * S];
#pragma unroll
        for (int x = 0; x < N; ++x) {
          cplx acc = u[0];
#pragma unroll
          for (int j = 1; j < N; ++j) acc = cadd(acc, cmul(u[j], tw[(x * j) % N]));
          p[x * S] = acc;
        }
      }
    }
}

template <int N0, int N1, int N2, bool HALF>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 2))) void kmesh_y_reg_kernel(
    const cplx* __restrict__ FX, int ncol, unsigned long long qmask, int m, cplx* __restrict__ yT,
    long qs, long Is, long goff, unsigned long long* __restrict__ mon, double csign) {
  constexpr int NK = N0 * N1 * N2;
  cplx tw0[N0], tw1[N1], tw2[N2];
#pragma unroll
  for (int t = 0; t < N0; ++t) { double s, c; sincospi(2.0 * t / N0, &s, &c); tw0[t] = cmk(c, s); }
#pragma unroll
  for (int t = 0; t < N1; ++t) { double s, c; sincospi(2.0 * t / N1, &s, &c); tw1[t] = cmk(c, s); }
#pragma unroll
  for (int t = 0; t < N2; ++t) { double s, c; sincospi(2.0 * t / N2, &s, &c); tw2[t] = cmk(c, s); }
  const double sc = 1.0 / sqrt((double)NK);
  double mi = 0.0;
  for (int col = blockIdx.x * blockDim.x + threadIdx.x; col < ncol; col += gridDim.x * blockDim.x) {
    cplx v[NK];
    // HALF: only the representatives k <= -k are stored; fx_{-k} = conj(fx_k) (time reversal)
#pragma unroll
    for (int k = 0; k < NK; ++k)
      if (!HALF || kmesh_is_rep(k, N0, N1, N2))
        v[k] = FX[(long)(HALF ? kmesh_rep_slot(k, N0, N1, N2) : k) * ncol + col];
#pragma unroll
    for (int k = 0; k < NK; ++k)
      if (HALF && !kmesh_is_rep(k, N0, N1, N2)) v[k] = cconj(v[kmesh_partner(k, N0, N1, N2)]);
    // fx_s = Phi fx_k (fftisdf.py:79)
    reg_axis_dft<N0, N1 * N2, NK>(v, tw0);
    reg_axis_dft<N1, N2, NK>(v, tw1);
    reg_axis_dft<N2, 1, NK>(v, tw2);
    // y_s = fx_s^2, fx_s real (fftisdf.py:81,83)
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const double re = v[k].x * sc;
      mi = fmax(mi, fabs(v[k].y * sc));
      v[k] = cmk(re * re, 0.0);
    }
    // y_k = Phi^T y_s (fftisdf.py:84)
    reg_axis_dft<N0, N1 * N2, NK>(v, tw0);
    reg_axis_dft<N1, N2, NK>(v, tw1);
    reg_axis_dft<N2, 1, NK>(v, tw2);
    const unsigned I = (unsigned)col / (unsigned)m, g = (unsigned)col - I * (unsigned)m;
    cplx* out = yT + (long)I * Is + goff + g;
#pragma unroll
    for (int k = 0; k < NK; ++k)
      if ((qmask >> k) & 1ull)  // slot of q = k in the ascending q-list
        out[(long)__popcll(qmask & ((1ull << k) - 1ull)) * qs] = cmk(v[k].x * sc, csign * v[k].y * sc);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mi = fmax(mi, __shfl_xor(mi, o, 64));
  if ((threadIdx.x & 63) == 0 && mon) atomicMax(mon, (unsigned long long)__double_as_longlong(mi));
}

// get_k's k-mesh transform pair in registers (fftisdf.py:211-222), one thread per (I, J) column
// of the block rows, in place: rho_s = Phi rho_k (:215, real: max |Im| recorded, :216),
// V_s = W_s * Re(rho_s) (:219; W_s real, row s at Ws + s * ws_Rstride), V_k = Phi^T V_s (:222) —
// the separable DFTs of kmesh_y_reg_kernel (Phi[R][q] = e^{i T_R . k_q} / sqrt(nk) is symmetric,
// so Phi^T is the same transform) instead of two dense nk x nk GEMMs with the product in the
// first one's epilogue: one read of rho_k and W_s, one write of V_k.
template <int N0, int N1, int N2>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_wsrho_reg_kernel(
    cplx* __restrict__ B, long ncol, const double* __restrict__ Ws, long ws_Rstride,
    unsigned long long* __restrict__ mon) {
  constexpr int NK = N0 * N1 * N2;
  cplx tw0[N0], tw1[N1], tw2[N2];
#pragma unroll
  for (int t = 0; t < N0; ++t) { double s, c; sincospi(2.0 * t / N0, &s, &c); tw0[t] = cmk(c, s); }
#pragma unroll
  for (int t = 0; t < N1; ++t) { double s, c; sincospi(2.0 * t / N1, &s, &c); tw1[t] = cmk(c, s); }
#pragma unroll
  for (int t = 0; t < N2; ++t) { double s, c; sincospi(2.0 * t / N2, &s, &c); tw2[t] = cmk(c, s); }
  const double sc = 1.0 / sqrt((double)NK);
  double mi = 0.0;
  for (long col = blockIdx.x * (long)blockDim.x + threadIdx.x; col < ncol;
       col += (long)gridDim.x * blockDim.x) {
    cplx v[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) v[k] = B[(long)k * ncol + col];
    reg_axis_dft<N0, N1 * N2, NK>(v, tw0);
    reg_axis_dft<N1, N2, NK>(v, tw1);
    reg_axis_dft<N2, 1, NK>(v, tw2);
#pragma unroll
    for (int s = 0; s < NK; ++s) {
      mi = fmax(mi, fabs(v[s].y * sc));
      v[s] = cmk(Ws[(long)s * ws_Rstride + col] * (v[s].x * sc), 0.0);
    }
    reg_axis_dft<N0, N1 * N2, NK>(v, tw0);
    reg_axis_dft<N1, N2, NK>(v, tw1);
    reg_axis_dft<N2, 1, NK>(v, tw2);
#pragma unroll
    for (int k = 0; k < NK; ++k) B[(long)k * ncol + col] = cmk(v[k].x * sc, v[k].y * sc);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mi = fmax(mi, __shfl_xor(mi, o, 64));
  if ((threadIdx.x & 63) == 0 && mon) atomicMax(mon, (unsigned long long)__double_as_longlong(mi));
}

// Fused y build for the register k-meshes under time reversal (fftisdf.py:76-85).  One
// workgroup per 16 (I) x 16 (g) column tile; fx_k = X_k f_k^H is formed on FP64 MFMA for the
// representative k (K = nao, 3-multiplication complex form: t1 = Xr fr, t2 = Xi fi,
// t3 = (Xr + Xi)(fr - fi); Re = t1 + t2, Im = t3 - t1 + t2) and never reaches HBM (the
// unfused path writes and re-reads it: 2/3 of the y build's traffic).  The k-mesh DFTs are
// split by k-planes a (axis 0) so that only one chunk of fx is staged in LDS at a time and two
// workgroups fit a CU (one's MFMA phase overlaps the other's DFT phase):
//   t_a(s) = sum_{b,c} fx(a,b,c) e^{+2 pi i (b s_b/N1 + c s_c/N2)}    (2-D DFT per plane)
// with t_{-a} = conj(t_a) pointwise (fx_{-k} = conj(fx_k)), so only planes a <= -a are formed:
// chunk A = the complex planes 0 < a < N0/2 (every k a representative), chunk B = the
// self-paired planes a = 0, N0/2 (half their k; t_a real).  Then per s:
//   fx_s(a', s) = sum_a e^{+2 pi i a a'/N0} t_a(s),  y_s = fx_s^2 (fftisdf.py:81,83),
//   r_qa(s) = sum_a' e^{+2 pi i a' qa/N0} y_s(a', s),  y(qa, .) = 2-D DFT of r_qa (:84),
// and y_{-q} = conj(y_q).  Tile order: XCD-aware (workgroup id & 7 = XCD), an XCD's resident
// workgroups walk the I-tiles of one g-tile (the f tile stays in its L2).
// mode (debug timing, FISDF_YF_MODE): bit 0 skips the MFMA phase, bit 1 the DFT + stores.
constexpr int YF_MAXKS = 7;  // nao <= 28 per K chunk (larger nao loops over chunks)
struct YfPlan {
  int nA, nB;   // slots of chunk A (complex planes) and B (self-paired planes)
  int kA[16];   // k of each slot, in the kernel's slot order
  int kB[32];
};

template <int N1, int N2>
__host__ __device__ constexpr int yf_inplane_partner(int bc) {
  return ((N1 - bc / N2) % N1) * N2 + (N2 - bc % N2) % N2;
}
template <int N1, int N2>
__host__ __device__ constexpr int yf_inplane_rank(int bc) {
  int r = 0;
  for (int j = 0; j < bc; ++j) r += j <= yf_inplane_partner<N1, N2>(j) ? 1 : 0;
  return r;
}

// fx for the chunk's slots (wave w: slots w, w+4, ...) into buf[slot][256]
__device__ __forceinline__ void yf_mfma_chunk(const cplx* __restrict__ XT, int nip, int nao,
                                              const cplx* __restrict__ FT, int m, int sbase,
                                              int nslot, int Ia, bool okI,
                                              int ga, bool okg, int lane, int w,
                                              cplx* __restrict__ buf) {
  const int i16 = lane & 15, kq = lane >> 4;
  const int nkc = (nao + 4 * YF_MAXKS - 1) / (4 * YF_MAXKS);
  // explicit operand buffers (no register rotation between iterations)
  cplx a0[YF_MAXKS], b0[YF_MAXKS], a1[YF_MAXKS], b1[YF_MAXKS];
  // Branch-free operand loads: rows past nip / m are clamped to the last valid row (their
  // columns are never stored) and K past nao to its last element, with the A operand zeroed at
  // use (a select after the load made the compiler wait for the next slot's loads right after
  // issuing them, before this slot's MFMAs, exposing the full load latency every slot).  The
  // slot index is wave-uniform, so ks[s] is a scalar load.
  const int Ic = min(Ia, nip - 1), gc = min(ga, m - 1);
  (void)okI;
  (void)okg;
  // operands from the mu-major copies XT[slot][mu][I], FT[slot][mu][g] (yf_transpose_kernel):
  // at a fixed mu the 16 rows of a fragment are 256 contiguous bytes, so one load instruction
  // moves 4 x 256 B in full 128-B lines instead of 16 rows x 64 B (half lines) from the
  // [k][row][mu] layouts (which kept the L1/TA path busier than the MFMA pipe)
  auto load = [&](cplx (&a)[YF_MAXKS], cplx (&b)[YF_MAXKS], int s, int c) {
    const long sl = (long)(sbase + s) * nao;
    const cplx* xa = XT + sl * nip + Ic;
    const cplx* fb = FT + sl * m + gc;
#pragma unroll
    for (int kk = 0; kk < YF_MAXKS; ++kk) {
      const int mu = min(c * 4 * YF_MAXKS + kk * 4 + kq, nao - 1);
      a[kk] = xa[(long)mu * nip];
      b[kk] = fb[(long)mu * m];
    }
  };
  f64x4 t1 = {0, 0, 0, 0}, t2 = {0, 0, 0, 0}, t3 = {0, 0, 0, 0};
  auto mma = [&](const cplx (&a)[YF_MAXKS], const cplx (&b)[YF_MAXKS], int s, int c, int cn) {
#pragma unroll
    for (int kk = 0; kk < YF_MAXKS; ++kk) {
      if (c * 4 * YF_MAXKS + kk * 4 >= nao) break;  // wave-uniform: a K step past nao
      const bool ok = c * 4 * YF_MAXKS + kk * 4 + kq < nao;
      const double ar = ok ? a[kk].x : 0.0, ai = ok ? a[kk].y : 0.0, br = b[kk].x, bi = b[kk].y;
      t1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ar, br, t1, 0, 0, 0);
      t2 = __builtin_amdgcn_mfma_f64_16x16x4f64(ai, bi, t2, 0, 0, 0);
      t3 = __builtin_amdgcn_mfma_f64_16x16x4f64(ar + ai, br - bi, t3, 0, 0, 0);
    }
    if (cn == 0) {  // slot complete: C row = Il = kq + 4 r, col = gl = i16
#pragma unroll
      for (int r = 0; r < 4; ++r)
        buf[s * 256 + (kq + 4 * r) * 16 + i16] = cmk(t1[r] + t2[r], t3[r] - t1[r] + t2[r]);
      t1 = f64x4{0, 0, 0, 0};
      t2 = f64x4{0, 0, 0, 0};
      t3 = f64x4{0, 0, 0, 0};
    }
  };
  auto next = [&](int s, int c, int& sn, int& cn) {
    sn = s;
    cn = c + 1;
    if (cn == nkc) { sn = s + 4; cn = 0; }
  };
  // two operand buffers: the loads run one (slot, K-chunk) item ahead of the MFMAs (three, two
  // items ahead, spill 22 VGPRs at 256 and measured slower: 6.3 vs 5.1 ms MFMA phase; four
  // buffers of half-slot items (K chunks of 16) fit in 233 VGPRs and measured 5.7 ms).  The
  // loads are issued unconditionally (past the last slot they re-read a valid one and are never
  // used): a conditional load made the compiler's wait counts conservative on the path that
  // issued them, draining the next slot's loads before this slot's MFMAs
  int s = __builtin_amdgcn_readfirstlane(w), c = 0, sl, cl;
  if (s >= nslot) return;
  auto load_item = [&](cplx (&a)[YF_MAXKS], cplx (&b)[YF_MAXKS], int si, int ci) {
    load(a, b, min(si, nslot - 1), si < nslot ? ci : 0);
  };
  auto step = [&](cplx (&al)[YF_MAXKS], cplx (&bl)[YF_MAXKS], const cplx (&am)[YF_MAXKS],
                  const cplx (&bm)[YF_MAXKS]) {
    load_item(al, bl, sl, cl);
    next(sl, cl, sl, cl);
    int sn, cn;
    next(s, c, sn, cn);
    mma(am, bm, s, c, cn);
    s = sn;
    c = cn;
    return s < nslot;
  };
  load(a0, b0, s, 0);
  next(s, c, sl, cl);
  for (;;) {
    if (!step(a1, b1, a0, b0)) break;
    if (!step(a0, b0, a1, b1)) break;
  }
}

// dst[j][mu][r] = src[k_j * kstride + r * nao + mu] for r < nrow: the plan's k (slot j: chunk A's
// k, then chunk B's) in mu-major order for the fused kernel's fragment loads.  One workgroup per
// (64-row block, slot): the block's 64 x nao elements (contiguous) are read coalesced into LDS
// and written out row-contiguous per mu.
__global__ __launch_bounds__(256) void yf_transpose_kernel(const cplx* __restrict__ src,
                                                           long kstride, int nrow, int nao,
                                                           YfPlan plan, cplx* __restrict__ dst) {
  extern __shared__ cplx tile[];  // [64][nao + 1]
  const int j = blockIdx.y;
  const int k = j < plan.nA ? plan.kA[j] : plan.kB[j - plan.nA];
  const int r0 = blockIdx.x * 64, nr = min(64, nrow - r0), ld = nao + 1;
  const cplx* sp = src + (long)k * kstride + (long)r0 * nao;
  for (int e = threadIdx.x; e < nr * nao; e += 256) {
    const int r = e / nao, mu = e - r * nao;
    tile[r * ld + mu] = sp[e];
  }
  __syncthreads();
  cplx* dp = dst + (long)j * nao * nrow + r0;
  for (int e = threadIdx.x; e < nao * 64; e += 256) {
    const int mu = e >> 6, r = e & 63;
    if (r < nr) dp[(long)mu * nrow + r] = tile[r * ld + mu];
  }
}

// XT[j][mu][I] = x0[k_j][piv[I]][mu] for the rows [lo, hi) of a streamed y build
// (y_fused_stream): the pivots come from a selection still running on another stream, so one
// thread per workgroup first waits until the selection has published at least `hi` of them
// (pchol_select_coop's progress word, agent-coherent; kSelDone once it has ended, also written
// by the caller after the kernel whatever path ran).  The wait is bounded: past ~10 s it sets
// *err (the build then fails loudly) and goes on with whatever pivots are there; a pivot is
// clamped into [0, ng0) before it addresses x0.
constexpr long kXtSpinCap = 3000000;  // s_sleep(127) rounds: ~10 s
__global__ __launch_bounds__(256) void yf_xt_stream_kernel(const cplx* __restrict__ x0,
                                                           long kstride, int ng0, int nao,
                                                           const int* __restrict__ piv,
                                                           const int* __restrict__ progress,
                                                           int lo, int hi, int nip, YfPlan plan,
                                                           cplx* __restrict__ XT,
                                                           int* __restrict__ err) {
  extern __shared__ cplx tile[];  // [64][nao + 1]
  __shared__ int s_p[64];
  if (threadIdx.x == 0) {
    long spins = 0;
    while (__hip_atomic_load(progress, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < hi) {
      __builtin_amdgcn_s_sleep(127);
      if (++spins > kXtSpinCap) {
        atomicExch(err, 1);
        break;
      }
    }
  }
  __syncthreads();
  const int j = blockIdx.y;
  const int k = j < plan.nA ? plan.kA[j] : plan.kB[j - plan.nA];
  const int r0 = lo + blockIdx.x * 64, nr = min(64, hi - r0), ld = nao + 1;
  if (threadIdx.x < 64) {
    int p = 0;
    if ((int)threadIdx.x < nr)
      p = __hip_atomic_load(&piv[r0 + threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_p[threadIdx.x] = min(max(p, 0), ng0 - 1);
  }
  __syncthreads();
  const cplx* sp = x0 + (long)k * kstride;
  for (int e = threadIdx.x; e < nr * nao; e += 256) {
    const int r = e / nao, mu = e - r * nao;
    tile[r * ld + mu] = sp[(long)s_p[r] * nao + mu];
  }
  __syncthreads();
  cplx* dp = XT + (long)j * nao * nip + r0;
  for (int e = threadIdx.x; e < nao * 64; e += 256) {
    const int mu = e >> 6, r = e & 63;
    if (r < nr) dp[(long)mu * nip + r] = tile[r * ld + mu];
  }
}

template <int N0, int N1, int N2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void y_fused_kernel(
    const cplx* __restrict__ XT, int nip, int nao, const cplx* __restrict__ FT, int m,
    int nIt, int nGt, YfPlan plan, unsigned long long qmask, unsigned long long rmask,
    cplx* __restrict__ yT, long qs, long Is, long goff, int mode, int gpair, int it0) {
  constexpr int P = N1 * N2, NK = N0 * P;
  constexpr int R = yf_inplane_rank<N1, N2>(P);         // in-plane representatives
  constexpr int NC = (N0 - 1) / 2;                        // complex planes 1..NC (N0 <= 4: 0 or 1)
  constexpr int NR = (N0 % 2 == 0 && N0 > 1) ? 2 : 1;     // self-paired planes 0 (, N0/2)
  static_assert(N0 <= 4 && NC <= 1, "y_fused: k-mesh axis 0 must be <= 4");
  extern __shared__ cplx buf[];  // [slot][256]: column c = Il * 16 + gl
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // XCD x walks its g-tiles (gt = x mod 8) in groups of gpair: within a group the I-tiles go
  // slowest, so the workgroups of one I-tile (same X panels) run back to back
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int grp = j / (nIt * gpair), rem = j - grp * nIt * gpair;
  const int it = rem / gpair, gt = (grp * gpair + rem % gpair) * 8 + xcd;
  if (gt >= nGt) return;
  const int I0 = (it0 + it) * 16, g0 = gt * 16;  // it0: the launch's first I-tile (streamed y)
  const int Ia = I0 + (lane & 15), ga = g0 + (lane & 15);
  const bool okI = Ia < nip, okg = ga < m;
  cplx tw0[N0], tw1[N1], tw2[N2];
#pragma unroll
  for (int t = 0; t < N0; ++t) { double sn, cs; sincospi(2.0 * t / N0, &sn, &cs); tw0[t] = cmk(cs, sn); }
#pragma unroll
  for (int t = 0; t < N1; ++t) { double sn, cs; sincospi(2.0 * t / N1, &sn, &cs); tw1[t] = cmk(cs, sn); }
#pragma unroll
  for (int t = 0; t < N2; ++t) { double sn, cs; sincospi(2.0 * t / N2, &sn, &cs); tw2[t] = cmk(cs, sn); }
  cplx tc[NC > 0 ? P : 1];  // t_1 (complex plane)
  double tr[NR][P];         // t_0 (, t_{N0/2})
  // chunk B first: during the MFMA phase of chunk A only the real tr (NR x P doubles) is live,
  // not the complex tc (the registers the MFMA phase's operand prefetch needs)
  // ---- chunk B: the self-paired planes, half their k each ----
  if (!(mode & 1)) yf_mfma_chunk(XT, nip, nao, FT, m, plan.nA, plan.nB, Ia, okI, ga, okg, lane, w, buf);
  __syncthreads();
  if (!(mode & 2)) {
#pragma unroll
    for (int pi = 0; pi < NR; ++pi) {
      cplx u[P];
#pragma unroll
      for (int bc = 0; bc < P; ++bc)
        if (bc <= yf_inplane_partner<N1, N2>(bc))
          u[bc] = (mode & 1) ? cmk(0, 0) : buf[(pi * R + yf_inplane_rank<N1, N2>(bc)) * 256 + tid];
#pragma unroll
      for (int bc = 0; bc < P; ++bc)
        if (bc > yf_inplane_partner<N1, N2>(bc)) u[bc] = cconj(u[yf_inplane_partner<N1, N2>(bc)]);
      reg_axis_dft<N1, N2, P>(u, tw1);
      reg_axis_dft<N2, 1, P>(u, tw2);
#pragma unroll
      for (int bc = 0; bc < P; ++bc) tr[pi][bc] = u[bc].x;
    }
  }
  // ---- chunk A: the complex plane a = 1 ----
  if constexpr (NC > 0) {
    __syncthreads();  // buf is rewritten by chunk A
    if (!(mode & 1)) yf_mfma_chunk(XT, nip, nao, FT, m, 0, plan.nA, Ia, okI, ga, okg, lane, w, buf);
    __syncthreads();
    if (mode & 2) return;
#pragma unroll
    for (int bc = 0; bc < P; ++bc) tc[bc] = (mode & 1) ? cmk(0, 0) : buf[bc * 256 + tid];
    reg_axis_dft<N1, N2, P>(tc, tw1);
    reg_axis_dft<N2, 1, P>(tc, tw2);
  }
  if (mode & 2) return;
  // ---- per s: fx_s over axis 0, y_s = fx_s^2, r_qa = axis-0 DFT of y_s ----
  const double sc = 1.0 / sqrt((double)NK), sc2 = sc * sc;
  double rr[NR][P];
  cplx rc[NC > 0 ? P : 1];
#pragma unroll
  for (int s = 0; s < P; ++s) {
    double ys[N0];
#pragma unroll
    for (int a2 = 0; a2 < N0; ++a2) {
      double f = tr[0][s];
      if constexpr (NR == 2) f += (a2 & 1) ? -tr[1][s] : tr[1][s];
      if constexpr (NC > 0) {  // 2 Re(w^{a2} t_1)
        const cplx wv = tw0[a2 % N0];
        f += 2.0 * (wv.x * tc[s].x - wv.y * tc[s].y);
      }
      ys[a2] = f * f * sc2;
    }
    double r0 = 0.0, rh = 0.0;
    cplx r1 = cmk(0, 0);
#pragma unroll
    for (int a2 = 0; a2 < N0; ++a2) {
      r0 += ys[a2];
      if constexpr (NR == 2) rh += (a2 & 1) ? -ys[a2] : ys[a2];
      if constexpr (NC > 0) r1 = cadd(r1, cscale(tw0[a2 % N0], ys[a2]));
    }
    rr[0][s] = r0;
    if constexpr (NR == 2) rr[1][s] = rh;
    if constexpr (NC > 0) rc[s] = r1;
  }
  // ---- output planes: y(qa, .) = 2-D DFT of r_qa; y(-q) = conj(y(q)) ----
  const int I = I0 + (tid >> 4), g = g0 + (tid & 15);
  if (I >= nip || g >= m) return;
  cplx* out = yT + (long)I * Is + goff + g;
  auto put = [&](int q, cplx v) {
    if ((qmask >> q) & 1ull) {
      // non-temporal: y (GBs, read back by the fit's FFTs much later) streams past L2, so the
      // X / f operand lines of the MFMA phase stay cached (y -0.22 ms, the factor beside it
      // -0.4 ms at C3, profiles/r03_ab/gemm_pipe.log)
      const long so = (long)__popcll(qmask & ((1ull << q) - 1ull)) * qs;
      if ((rmask >> q) & 1ull) {
        // a self-conjugate q (rmask): y_q is real (its DFT twiddles at these frequencies are
        // +-1, so the imaginary part is exactly zero) and is stored as doubles in the first
        // half of its slot, [I][g] with the same strides: half the bytes (fft3d in_real)
        __builtin_nontemporal_store(v.x * sc, (double*)(yT + so) + ((long)I * Is + goff + g));
      } else {
        typedef double dv2 __attribute__((ext_vector_type(2)));
        __builtin_nontemporal_store(dv2{v.x * sc, v.y * sc}, (dv2*)(out + so));
      }
    }
  };
#pragma unroll
  for (int pi = 0; pi < NR; ++pi) {
    cplx u[P];
#pragma unroll
    for (int bc = 0; bc < P; ++bc) u[bc] = cmk(rr[pi][bc], 0.0);
    reg_axis_dft<N1, N2, P>(u, tw1);
    reg_axis_dft<N2, 1, P>(u, tw2);
    const int qa = pi == 0 ? 0 : N0 / 2;
#pragma unroll
    for (int bc = 0; bc < P; ++bc) put(qa * P + bc, u[bc]);
  }
  if constexpr (NC > 0) {
    reg_axis_dft<N1, N2, P>(rc, tw1);
    reg_axis_dft<N2, 1, P>(rc, tw2);
#pragma unroll
    for (int bc = 0; bc < P; ++bc) {
      put(P + bc, rc[bc]);
      put((N0 - 1) * P + yf_inplane_partner<N1, N2>(bc), cconj(rc[bc]));
    }
  }
}

// pair densities at the interpolation points: P[I][i*n2 + j] = conj(A[I][i]) * B[I][j]
__global__ void pair_product_kernel(const cplx* __restrict__ A, int n1, const cplx* __restrict__ B,
                                    int n2, int nip, cplx* __restrict__ P) {
  long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long tot = (long)nip * n1 * n2;
  if (e >= tot) return;
  const int j = (int)(e % n2);
  const int i = (int)((e / n2) % n1);
  const int I = (int)(e / ((long)n1 * n2));
  P[e] = cmul(cconj(A[(long)I * n1 + i]), B[(long)I * n2 + j]);
}

// out[g][q*nao + m] = x0[q][g][m]   (k-point axis folded into the GEMM K dimension)
__global__ void permute_kgm_kernel(const cplx* __restrict__ x0, int nq, int ng, int nao,
                                   cplx* __restrict__ out) {
  long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long tot = (long)nq * ng * nao;
  if (e >= tot) return;
  const int m = (int)(e % nao);
  const int g = (int)((e / nao) % ng);
  const int q = (int)(e / ((long)nao * ng));
  out[(long)g * nq * nao + (long)q * nao + m] = x0[e];
}

// X[k,I,:] = x0[k, perm[I], :]
__global__ void gather_points_kernel(const cplx* __restrict__ x0, int nk, int ng0, int nao,
                                     const int* __restrict__ perm, int nip, cplx* __restrict__ X) {
  long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= (long)nk * nip * nao) return;
  int m = (int)(e % nao);
  int I = (int)((e / nao) % nip);
  int k = (int)(e / ((long)nao * nip));
  X[e] = x0[((long)k * ng0 + perm[I]) * nao + m];
}

// x4[i,j] = Re(x2[i,j])^2 / nk  (fftisdf.py:379)  — stored as complex (+0i) for pchol
__global__ void square_scale_kernel(const cplx* __restrict__ in, double s, cplx* __restrict__ out,
                                    long n) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    double r = in[e].x;
    out[e] = cmk(r * r * s, 0.0);
  }
}

// y_s element-wise square in place, complex: x2_s -> x4_s (complex square, fftisdf.py:45)
__global__ void csquare_kernel(cplx* __restrict__ a, long n, unsigned long long* __restrict__ maximag) {
  double mi = 0.0;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    cplx v = a[e];
    mi = fmax(mi, fabs(v.y));
    a[e] = cmul(v, v);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mi = fmax(mi, __shfl_xor(mi, o, 64));
  if ((threadIdx.x & 63) == 0 && maximag) atomicMax(maximag, (unsigned long long)__double_as_longlong(mi));
}

inline int nblocks(long n, int bs = 256, long cap = 1L << 20) {
  long b = (n + bs - 1) / bs;
  return (int)std::max(1L, std::min(b, cap));
}

}  // namespace

int gather_lp(hipStream_t s, const cplx* L, int n, int rmax, const int* piv, const int* rank,
              int rpad, cplx* Lp, int batch) {
  long e = (long)rpad * rpad;
  if (e == 0 || batch == 0) return 0;
  hipLaunchKernelGGL(gather_lp_kernel, dim3(nblocks(e, 256, 1L << 30), batch), dim3(256), 0, s, L,
                     n, rmax, piv, rank, rpad, Lp);
  FISDF_HIP(hipGetLastError());
  return 0;
}

// Q (r x r, ld = r per batch entry): block rows of the merged forward substitution,
//   Q[b, b] = L_bb^{-1},  Q[b, :b0] = -L_bb^{-1} L[b, :b0]
// over the partition [0, s0), [s0, s0+64), ..., s0 = r - 64 (nblk - 1) (the partial block
// first, so every large-K step of trsm_merged_batched has a full 64-row tile).
int build_trsm_q(hipStream_t s, const cplx* Lp, int r, long sL, cplx* Q, int batch, int mode) {
  const int nblk = (r + 63) / 64;
  if (nblk == 0 || batch == 0) return 0;
  const int s0 = r - 64 * (nblk - 1);
  const long rr = (long)r * r;
  hipLaunchKernelGGL(trinv_into_kernel, dim3(nblk, batch), dim3(256), 0, s, Lp, r, r, sL, s0, Q, r,
                     rr);
  FISDF_HIP(hipGetLastError());
  const cplx mone = cmk(-1, 0), zero = cmk(0, 0);
  for (int b = 1; b < nblk; ++b) {
    const int b0 = s0 + (b - 1) * 64;
    FISDF_TRY(zgemm(s, OP_N, OP_N, 64, b0, 64, mone, Q + (long)b0 * r + b0, r, rr,
                    Lp + (long)b0 * r, r, sL, zero, Q + (long)b0 * r, r, rr, batch, 1, nullptr,
                    EPI_NONE, nullptr, mode));
  }
  return 0;
}

// X = L^{-1} X in place for a batch of X (r x ncol, ld; batch strides sQ, sX): one GEMM launch
// per block row with the Q of build_trsm_q, X[b] = Q[b, :b1] X[:b1] — each workgroup owns whole
// columns (M <= 64), so it reads all of X[:b1] for its columns before its epilogue overwrites
// X[b].
// lower_rhs: X is lower-triangular (the identity, for L^{-1}), so block row b only has
// columns < b1 to compute (the rest stay zero)
// work (work_elems cplx, may be null): split-K partials for long block rows (each 64 x 64 tile
// otherwise runs its whole K = b1 alone, which leaves most CUs idle for a small batch); the
// partials are reduced by a later kernel, so the in-place update stays safe.  The split of a
// block row depends on that row's shape only (trsm_split_k), never on the batch size, so a
// matrix gets the same summation order whichever other matrices share its batch (the 1-GPU and
// the k-sharded builds factor different batches and must agree bitwise); a batch whose partials
// exceed the workspace is processed in sub-batches.
int trsm_split_k(int nc, int b1) {
  if (b1 < 256) return 1;
  const int tiles = (nc + 63) / 64;
  return std::max(1, std::min({256 / std::max(tiles, 1), b1 / 128, 16}));
}

long trsm_split_work_elems(int r, int batch) {
  long mx = 0;
  const int nblk = (r + 63) / 64, s0 = r - 64 * (nblk - 1);
  for (int b = 0; b < nblk; ++b) {
    const int b0 = b == 0 ? 0 : s0 + (b - 1) * 64, m = std::min(b == 0 ? s0 : 64, r - b0);
    for (int nc : {r, b0 + m}) {  // a full right-hand side, or the lower-triangular identity
      const int ks = trsm_split_k(nc, b0 + m);
      if (ks > 1) mx = std::max(mx, (long)ks * m * nc);
    }
  }
  return mx * batch;
}

int trsm_merged_batched(hipStream_t s, const cplx* Q, long sQ, int r, cplx* X, long ld, long sX,
                        int ncol, int batch, bool lower_rhs, cplx* work, long work_elems) {
  const int nblk = (r + 63) / 64;
  if (nblk == 0 || batch == 0) return 0;
  const int s0 = r - 64 * (nblk - 1);
  const cplx one = cmk(1, 0), zero = cmk(0, 0);
  for (int b = 0; b < nblk; ++b) {
    const int b0 = b == 0 ? 0 : s0 + (b - 1) * 64;
    const int m = std::min(b == 0 ? s0 : 64, r - b0), b1 = b0 + m;
    const int nc = lower_rhs ? std::min(ncol, b1) : ncol;
    const int ks = work ? trsm_split_k(nc, b1) : 1;
    const long per = (long)ks * m * nc;  // partials of one matrix
    const int sub = ks > 1 ? (int)std::max(1L, std::min<long>(batch, work_elems / per)) : batch;
    FISDF_CHECK(ks == 1 || per <= work_elems, "trsm_merged_batched: split-K workspace too small");
    for (int z0 = 0; z0 < batch; z0 += sub) {
      const int nb = std::min(sub, batch - z0);
      FISDF_TRY(zgemm(s, OP_N, OP_N, m, nc, b1, one, Q + z0 * sQ + (long)b0 * r, r, sQ,
                      X + z0 * sX, ld, sX, zero, X + z0 * sX + (long)b0 * ld, ld, sX, nb, ks,
                      ks > 1 ? work : nullptr));
    }
  }
  return 0;
}

__global__ void set_identity_kernel(cplx* __restrict__ X, int n, int batch) {
  long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long nn = (long)n * n;
  if (e >= nn * batch) return;
  const long r = e % nn;
  X[e] = cmk(r / n == r % n ? 1.0 : 0.0, 0.0);
}

int set_identity(hipStream_t s, cplx* X, int n, int batch) {
  const long tot = (long)n * n * batch;
  if (tot == 0) return 0;
  hipLaunchKernelGGL(set_identity_kernel, dim3(nblocks(tot, 256, 1L << 30)), dim3(256), 0, s, X, n,
                     batch);
  FISDF_HIP(hipGetLastError());
  return 0;
}

int trinv_blocks(hipStream_t s, const cplx* Lp, int r, int ldl, long sL, int nb, long sLi,
                 cplx* Linv, int batch) {
  FISDF_CHECK(nb >= 1 && nb <= 64, "trinv_blocks: nb must be <= 64");
  int nblk = (r + nb - 1) / nb;
  if (nblk == 0 || batch == 0) return 0;
  hipLaunchKernelGGL(trinv_blocks_kernel, dim3(nblk, batch), dim3(64), 0, s, Lp, r, ldl, sL, nb,
                     sLi, Linv);
  FISDF_HIP(hipGetLastError());
  return 0;
}

// X = L^{-1} B  (lower=1) or X = L^{-H} B (lower=0, backward with L^H); B is overwritten.
// L: r x r lower (ld = ldl, batch stride sL); Linv: diagonal-block inverses (batch stride
// sLi); B, X: r x ncol (ld, batch strides given).  Blocked: one ZGEMM update + one
// ZGEMM with the block inverse per 64-row block (factored order, never an explicit inverse).
int trsm_blocked(hipStream_t s, int lower, const cplx* Lp, long ldl, long sL, int r,
                 const cplx* Linv, long sLi, int nb, cplx* B, long ldb, long sB, cplx* X, long ldx,
                 long sX, int ncol, int batch, int a_real) {
  const cplx one = cmk(1, 0), mone = cmk(-1, 0), zero = cmk(0, 0);
  // a_real: L (and hence its diagonal-block inverses) is real -> half the MFMA work
  const int md = a_real ? GEMM_A_REAL : GEMM_FULL;
  int nblk = (r + nb - 1) / nb;
  for (int bi = 0; bi < nblk; ++bi) {
    int blk = lower ? bi : nblk - 1 - bi;
    int b0 = blk * nb, b1 = std::min(r, b0 + nb), m = b1 - b0;
    if (lower) {
      if (b0 > 0)  // B_b -= L[b, :b] X[:b]
        FISDF_TRY(zgemm(s, OP_N, OP_N, m, ncol, b0, mone, Lp + (long)b0 * ldl, ldl, sL, X, ldx,
                        sX, one, B + (long)b0 * ldb, ldb, sB, batch, 1, nullptr, EPI_NONE, nullptr,
                        md));
      FISDF_TRY(zgemm(s, OP_N, OP_N, m, ncol, m, one, Linv + (long)blk * nb * nb, nb, sLi,
                      B + (long)b0 * ldb, ldb, sB, zero, X + (long)b0 * ldx, ldx, sX, batch, 1,
                      nullptr, EPI_NONE, nullptr, md));
    } else {
      if (b1 < r)  // B_b -= (L^H)[b, >b] X[>b] = conj(L[>b, b])^T X[>b]
        FISDF_TRY(zgemm(s, OP_C, OP_N, m, ncol, r - b1, mone, Lp + (long)b1 * ldl + b0, ldl, sL,
                        X + (long)b1 * ldx, ldx, sX, one, B + (long)b0 * ldb, ldb, sB, batch, 1,
                        nullptr, EPI_NONE, nullptr, md));
      FISDF_TRY(zgemm(s, OP_C, OP_N, m, ncol, m, one, Linv + (long)blk * nb * nb, nb, sLi,
                      B + (long)b0 * ldb, ldb, sB, zero, X + (long)b0 * ldx, ldx, sX, batch, 1,
                      nullptr, EPI_NONE, nullptr, md));
    }
  }
  return 0;
}

// Coulomb-weight asymmetry of a self-conjugate q (2 k_q = m . b): for real z_q,
// Zhat(G') = conj(Zhat(G)) with G' = -G - 2 k_q, so W_q = sum_G c_G Zhat_G Zhat_G^H is real
// except where c(k+G) != c(k+G') — the Nyquist planes of even meshes (fftfreq puts -N/2 in
// both members of a pair) and the box-edge wrap of get_coulG.  One workgroup lists those G
// (ascending, deterministic) so Im(W_q) can be formed from them alone.
__global__ __launch_bounds__(1024) void asym_list_kernel(const double* __restrict__ w, int n0,
                                                         int n1, int n2, int m0, int m1, int m2,
                                                         int* __restrict__ idx,
                                                         int* __restrict__ count) {
  __shared__ int base;
  __shared__ int warp_tot[16];
  const long ngrid = (long)n0 * n1 * n2;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (long e0 = 0; e0 < ngrid; e0 += blockDim.x) {
    const long e = e0 + threadIdx.x;
    bool flag = false;
    if (e < ngrid) {
      const int i2 = (int)(e % n2), i1 = (int)((e / n2) % n1), i0 = (int)(e / ((long)n1 * n2));
      const int p0 = ((-i0 - m0) % n0 + n0) % n0, p1 = ((-i1 - m1) % n1 + n1) % n1,
                p2 = ((-i2 - m2) % n2 + n2) % n2;
      const long pe = ((long)p0 * n1 + p1) * n2 + p2;
      // pairs whose weights differ only by rounding (|k+G| and |k+G'| evaluated from
      // different index vectors) contribute rounding-level Im parts: not listed
      flag = fabs(w[e] - w[pe]) > 1e-13 * fmax(fabs(w[e]), fabs(w[pe]));
    }
    const unsigned long long bal = __ballot(flag);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) warp_tot[wv] = __popcll(bal);
    __syncthreads();
    int off = base;
    for (int j = 0; j < wv; ++j) off += warp_tot[j];
    if (flag) idx[off + before] = (int)e;
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      for (int j = 0; j < (int)(blockDim.x >> 6); ++j) t += warp_tot[j];
      base += t;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *count = base;
}

// ---- self-conjugate q on half the G (the Hermitian pairing Zhat(G') = conj(Zhat(G)),
// G' = -G - m.b, of a real z_q): planes i0 of the prefix [0, nH) hold one member of every pair
// (both members of a pair inside a self-paired plane i0 == (-i0 - m0) mod n0) -----------------
__device__ __forceinline__ long partner_index(long e, int n0, int n1, int n2, int m0, int m1,
                                              int m2, int* i0p, int* p0p) {
  const int i2 = (int)(e % n2), i1 = (int)((e / n2) % n1), i0 = (int)(e / ((long)n1 * n2));
  const int p0 = ((-i0 - m0) % n0 + n0) % n0, p1 = ((-i1 - m1) % n1 + n1) % n1,
            p2 = ((-i2 - m2) % n2 + n2) % n2;
  *i0p = i0;
  *p0p = p0;
  return ((long)p0 * n1 + p1) * n2 + p2;
}

// w[e] <- sqrt(c[e] + c[e']) on strict prefix planes, sqrt(c[e]) on a self-paired plane, 0 beyond
// the prefix (c = coulG * scale, not square-rooted), in place
__global__ void half_weight_kernel(double* __restrict__ w, const double* __restrict__ c, int n0,
                                   int n1, int n2, int m0, int m1, int m2, int nH) {
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= (long)n0 * n1 * n2) return;
  int i0, p0;
  const long pe = partner_index(e, n0, n1, n2, m0, m1, m2, &i0, &p0);
  double v = 0.0;
  if (i0 < nH) v = (p0 == i0) ? c[e] : c[e] + c[pe];
  w[e] = sqrt(v);
}

// one workgroup lists the prefix G whose pair has unequal weights (ascending) with the factor
// f = (c - c') / (c + c') of Im(G) (strict planes; 1 on a self-paired plane, where both members
// are listed), so Im W = Im(U_A diag(f) U_A^H) over the half-grid U
__global__ __launch_bounds__(1024) void asym_half_kernel(const double* __restrict__ c, int n0,
                                                         int n1, int n2, int m0, int m1, int m2,
                                                         int nH, int* __restrict__ idx,
                                                         double* __restrict__ f,
                                                         int* __restrict__ count) {
  __shared__ int base;
  __shared__ int warp_tot[16];
  const long nprefix = (long)nH * n1 * n2;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (long e0 = 0; e0 < nprefix; e0 += blockDim.x) {
    const long e = e0 + threadIdx.x;
    bool flag = false;
    double fv = 1.0;
    if (e < nprefix) {
      int i0, p0;
      const long pe = partner_index(e, n0, n1, n2, m0, m1, m2, &i0, &p0);
      const double ce = c[e], cp = c[pe];
      flag = fabs(ce - cp) > 1e-13 * fmax(fabs(ce), fabs(cp));
      if (p0 != i0 && flag) fv = (ce - cp) / (ce + cp);
    }
    const unsigned long long bal = __ballot(flag);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) warp_tot[wv] = __popcll(bal);
    __syncthreads();
    int off = base;
    for (int j = 0; j < wv; ++j) off += warp_tot[j];
    if (flag) {
      idx[off + before] = (int)e;
      f[off + before] = fv;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      for (int j = 0; j < (int)(blockDim.x >> 6); ++j) t += warp_tot[j];
      base += t;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *count = base;
}

// out[i][j] = A[i][idx[j]] * (f ? f[j] : 1)
__global__ void gather_cols_scaled_kernel(const cplx* __restrict__ A, long ld, int r,
                                          const int* __restrict__ idx, const double* __restrict__ f,
                                          int n, cplx* __restrict__ out) {
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= (long)r * n) return;
  const int i = (int)(e / n), j = (int)(e % n);
  const cplx v = A[(long)i * ld + idx[j]];
  out[e] = f ? cscale(v, f[j]) : v;
}

// out[i][j] = A[i][idx[j]]  (r rows of ld, n listed columns)
__global__ void gather_cols_kernel(const cplx* __restrict__ A, long ld, int r,
                                   const int* __restrict__ idx, int n, cplx* __restrict__ out) {
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= (long)r * n) return;
  const int i = (int)(e / n), j = (int)(e % n);
  out[e] = A[(long)i * ld + idx[j]];
}

// G.y += H.y (n x n, leading dims ldg / ldh)
__global__ void add_imag_kernel(cplx* __restrict__ G, int ldg, const cplx* __restrict__ H, int ldh,
                                int n) {
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= (long)n * n) return;
  const int i = (int)(e / n), j = (int)(e % n);
  G[(long)i * ldg + j].y += H[(long)i * ldh + j].y;
}

__global__ void zero_imag_kernel(cplx* __restrict__ a, long n) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x)
    a[e].y = 0.0;
}

int asym_list(hipStream_t s, const double* w, const int mesh[3], const int m[3], int* idx,
              int* count) {
  hipLaunchKernelGGL(asym_list_kernel, dim3(1), dim3(1024), 0, s, w, mesh[0], mesh[1], mesh[2],
                     m[0], m[1], m[2], idx, count);
  FISDF_HIP(hipGetLastError());
  return 0;
}

int gather_cols(hipStream_t s, const cplx* A, long ld, int r, const int* idx, int n, cplx* out) {
  const long e = (long)r * n;
  if (e == 0) return 0;
  hipLaunchKernelGGL(gather_cols_kernel, dim3(nblocks(e, 256, 1L << 30)), dim3(256), 0, s, A, ld,
                     r, idx, n, out);
  FISDF_HIP(hipGetLastError());
  return 0;
}

int half_prefix_planes(int n0, int m0) {
  int nH = 0;
  for (int i0 = 0; i0 < n0; ++i0)
    if (i0 <= ((-i0 - m0) % n0 + n0) % n0) nH = i0 + 1;
  return nH;
}

int half_weight(hipStream_t s, double* w, const double* c, const int mesh[3], const int m[3]) {
  const long n = (long)mesh[0] * mesh[1] * mesh[2];
  hipLaunchKernelGGL(half_weight_kernel, dim3(nblocks(n, 256, 1L << 30)), dim3(256), 0, s, w, c,
                     mesh[0], mesh[1], mesh[2], m[0], m[1], m[2], half_prefix_planes(mesh[0], m[0]));
  FISDF_HIP(hipGetLastError());
  return 0;
}

int asym_half(hipStream_t s, const double* c, const int mesh[3], const int m[3], int* idx,
              double* f, int* count) {
  hipLaunchKernelGGL(asym_half_kernel, dim3(1), dim3(1024), 0, s, c, mesh[0], mesh[1], mesh[2],
                     m[0], m[1], m[2], half_prefix_planes(mesh[0], m[0]), idx, f, count);
  FISDF_HIP(hipGetLastError());
  return 0;
}

int gather_cols_scaled(hipStream_t s, const cplx* A, long ld, int r, const int* idx,
                       const double* f, int n, cplx* out) {
  const long e = (long)r * n;
  if (e == 0) return 0;
  hipLaunchKernelGGL(gather_cols_scaled_kernel, dim3(nblocks(e, 256, 1L << 30)), dim3(256), 0, s, A,
                     ld, r, idx, f, n, out);
  FISDF_HIP(hipGetLastError());
  return 0;
}

int add_imag(hipStream_t s, cplx* G, int ldg, const cplx* H, int ldh, int n) {
  const long e = (long)n * n;
  if (e == 0) return 0;
  hipLaunchKernelGGL(add_imag_kernel, dim3(nblocks(e, 256, 1L << 30)), dim3(256), 0, s, G, ldg, H,
                     ldh, n);
  FISDF_HIP(hipGetLastError());
  return 0;
}

int zero_imag(hipStream_t s, cplx* a, long n) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(zero_imag_kernel, dim3(nblocks(n, 256, 8192)), dim3(256), 0, s, a, n);
  FISDF_HIP(hipGetLastError());
  return 0;
}

// factor staging: x4s[i] = x4all[qs[i]] (imaginary part zeroed for a self-conjugate q, whose
// x4_q is real up to rounding) and, if L is given, the same into L (the in-place Cholesky's
// input) — one pass instead of a copy per q plus a bulk copy
__global__ void stage_x4_kernel(const cplx* __restrict__ x4all, const int* __restrict__ qr, int nq,
                                long nn, cplx* __restrict__ x4s, cplx* __restrict__ L) {
  const int i = blockIdx.y;
  const long q = qr[i];
  const bool re = qr[nq + i] != 0;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < nn; e += (long)gridDim.x * blockDim.x) {
    cplx v = x4all[q * nn + e];
    if (re) v.y = 0.0;
    x4s[(long)i * nn + e] = v;
    if (L) L[(long)i * nn + e] = v;
  }
}

int stage_x4(hipStream_t s, const cplx* x4all, const int* qr, int nq, long nn, cplx* x4s, cplx* L) {
  if (nq == 0 || nn == 0) return 0;
  hipLaunchKernelGGL(stage_x4_kernel, dim3(nblocks(nn, 256, 512), nq), dim3(256), 0, s, x4all, qr, nq,
                     nn, x4s, L);
  FISDF_HIP(hipGetLastError());
  return 0;
}

// ---- minimum-norm (complete orthogonal) operator of a rank-deficient x4_q ----------------
namespace {

// A[s][t] = L[piv[s]][t] for every row s < n (the rejected pivots' rows included), t < r
__global__ void gather_trapezoid_kernel(const cplx* __restrict__ L, int n, int rmax,
                                        const int* __restrict__ piv, int r, cplx* __restrict__ A) {
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= (long)n * r) return;
  const int s = (int)(e / r), t = (int)(e % r);
  A[e] = (t <= s) ? L[(long)piv[s] * rmax + t] : cmk(0, 0);
}

// S += shift I with shift = 11 (n r + r (r + 1)) eps tr(S): the first pass of shifted
// CholeskyQR3 (tr(A^H A) = |A|_F^2 >= |A|_2^2), so the Cholesky of a Gram with cond ~ 1/eps
// cannot break down; the two unshifted passes after it restore orthogonality
__global__ __launch_bounds__(256) void shift_gram_kernel(cplx* __restrict__ S, int r, int n) {
  __shared__ double part[256];
  double t = 0.0;
  for (int i = threadIdx.x; i < r; i += 256) t += S[(long)i * r + i].x;
  part[threadIdx.x] = t;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  const double shift = 11.0 * ((double)n * r + (double)r * (r + 1)) * 2.220446049250313e-16 * part[0];
  for (int i = threadIdx.x; i < r; i += 256) S[(long)i * r + i].x += shift;
}

// piv[r..n) = the rows not among the first r pivots, ascending (the pivoted Cholesky stops at
// its rank and leaves them unset): the minimum-norm operator uses every row of x4_q
__global__ __launch_bounds__(1024) void complete_perm_kernel(int* __restrict__ piv, int n, int r) {
  extern __shared__ int used[];
  for (int i = threadIdx.x; i < n; i += blockDim.x) used[i] = 0;
  __syncthreads();
  for (int s = threadIdx.x; s < r; s += blockDim.x) used[piv[s]] = 1;
  __syncthreads();
  if (threadIdx.x == 0) {
    int k = r;
    for (int i = 0; i < n; ++i)
      if (!used[i]) piv[k++] = i;
  }
}

// H = X^H (r x r, ld r)
__global__ void adjoint_kernel(const cplx* __restrict__ X, int r, cplx* __restrict__ H) {
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= (long)r * r) return;
  const int i = (int)(e / r), j = (int)(e % r);
  H[(long)j * r + i] = cconj(X[e]);
}

}  // namespace

int min_norm_operator(hipStream_t s, const cplx* L, int n, int rmax, int* piv, int r,
                      cplx* M, long ldm, void* work, int* fail, cplx* q_out, cplx* rinv_out) {
  FISDF_CHECK(r >= 1 && r <= n && n <= rmax, "min_norm_operator: bad sizes");
  const long rr = (long)r * r, nr = (long)n * r;
  cplx* A = (cplx*)work;            // n x r: A = P L, then Q
  cplx* A2 = A + nr;                // n x r
  cplx* S = A2 + nr;                // r x r Gram / its Cholesky factor
  cplx* Qop = S + rr;               // r x r block-row operator of the triangular inverse
  cplx* Li = Qop + rr;              // r x r inverse of the pass's factor
  cplx* Ri = Li + rr;               // r x r accumulated R^{-1}
  cplx* Rt = Ri + rr;               // r x r
  cplx* cw = Rt + rr;               // chol_unpivoted work: 4096 cplx + 1 double
  int* iw = (int*)(cw + 4096 + 1);  // piv (r), rank
  const cplx one = cmk(1, 0), zero = cmk(0, 0);
  if (r < n) {
    hipLaunchKernelGGL(complete_perm_kernel, dim3(1), dim3(1024), sizeof(int) * n, s,
                       piv, n, r);
    FISDF_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(gather_trapezoid_kernel, dim3(nblocks(nr, 256, 1L << 30)), dim3(256), 0, s, L,
                     n, rmax, piv, r, A);
  FISDF_HIP(hipGetLastError());
  for (int pass = 0; pass < 3; ++pass) {
    // S = A^H A = Lc Lc^H;  A <- A Lc^{-H};  R^{-1} <- R^{-1} Lc^{-H}
    FISDF_TRY(zgemm(s, OP_C, OP_N, r, r, n, one, A, r, 0, A, r, 0, zero, S, r, 0, 1));
    if (pass == 0) {
      hipLaunchKernelGGL(shift_gram_kernel, dim3(1), dim3(256), 0, s, S, r, n);
      FISDF_HIP(hipGetLastError());
    }
    FISDF_TRY(chol_unpivoted(s, S, r, 1, 0.0, iw, iw + r, fail + pass, cw));
    FISDF_TRY(build_trsm_q(s, S, r, rr, Qop, 1, GEMM_FULL));
    FISDF_TRY(set_identity(s, Li, r, 1));
    FISDF_TRY(trsm_merged_batched(s, Qop, rr, r, Li, r, rr, r, 1, true));
    FISDF_TRY(zgemm(s, OP_N, OP_C, n, r, r, one, A, r, 0, Li, r, 0, zero, A2, r, 0, 1));
    std::swap(A, A2);
    if (pass == 0) {
      hipLaunchKernelGGL(adjoint_kernel, dim3(nblocks(rr, 256, 1L << 30)), dim3(256), 0, s, Li, r, Ri);
      FISDF_HIP(hipGetLastError());
    } else {
      FISDF_TRY(zgemm(s, OP_N, OP_C, r, r, r, one, Ri, r, 0, Li, r, 0, zero, Rt, r, 0, 1));
      std::swap(Ri, Rt);
    }
  }
  // A^+ = R^{-1} Q^H  (r x n)
  FISDF_TRY(zgemm(s, OP_N, OP_C, r, n, r, one, Ri, r, 0, A, r, 0, zero, M, ldm, 0, 1));
  if (q_out) FISDF_HIP(hipMemcpyAsync(q_out, A, sizeof(cplx) * nr, hipMemcpyDeviceToDevice, s));
  if (rinv_out) FISDF_HIP(hipMemcpyAsync(rinv_out, Ri, sizeof(cplx) * rr, hipMemcpyDeviceToDevice, s));
  return 0;
}

size_t min_norm_work_bytes(int n, int r) {
  return sizeof(cplx) * (2 * (size_t)n * r + 5 * (size_t)r * r + 4097) + sizeof(int) * ((size_t)r + 1);
}

int scatter_w(hipStream_t s, const cplx* Wpp, int ldw, long sW, int rmax, const int* piv,
              const int* rank, cplx* W, int nip, int batch) {
  FISDF_HIP(hipMemsetAsync(W, 0, sizeof(cplx) * (size_t)nip * nip * batch, s));
  long n = (long)rmax * rmax;
  if (n == 0 || batch == 0) return 0;
  hipLaunchKernelGGL(scatter_w_kernel, dim3(nblocks(n, 256, 1L << 30), batch), dim3(256), 0, s,
                     Wpp, ldw, sW, piv, rank, W, nip);
  FISDF_HIP(hipGetLastError());
  return 0;
}

int conj_transpose(hipStream_t s, const cplx* A, int n, long sA, cplx* B, int batch) {
  long e = (long)n * n;
  if (e == 0 || batch == 0) return 0;
  hipLaunchKernelGGL(conj_transpose_kernel, dim3(nblocks(e, 256, 1L << 30), batch), dim3(256), 0,
                     s, A, n, sA, B);
  FISDF_HIP(hipGetLastError());
  return 0;
}

int coulg_weight(hipStream_t s, const int mesh[3], const CellGeom& g, const double k[3],
                 double scale, int take_sqrt, double* w, double omega) {
  long ngrid = (long)mesh[0] * mesh[1] * mesh[2];
  hipLaunchKernelGGL(coulg_weight_kernel, dim3(nblocks(ngrid, 256, 1L << 30)), dim3(256), 0, s,
                     mesh[0], mesh[1], mesh[2], g, k[0], k[1], k[2], scale, take_sqrt, omega, w);
  FISDF_HIP(hipGetLastError());
  return 0;
}

int square_real(hipStream_t s, const cplx* in, cplx* out, long n, unsigned long long* maximag) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(square_real_kernel, dim3(nblocks(n, 256, 8192)), dim3(256), 0, s, in, out, n,
                     maximag);
  FISDF_HIP(hipGetLastError());
  return 0;
}

int csquare(hipStream_t s, cplx* a, long n, unsigned long long* maximag) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(csquare_kernel, dim3(nblocks(n, 256, 8192)), dim3(256), 0, s, a, n, maximag);
  FISDF_HIP(hipGetLastError());
  return 0;
}

int rho_diag(hipStream_t s, const cplx* T, const cplx* X, int nset, int nk, int nip, int nao,
             double scale, cplx* rho) {
  long n = (long)nset * nip;
  if (n == 0) return 0;
  FISDF_CHECK(n < (1L << 31), "rho_diag: too many rows");
  hipLaunchKernelGGL(rho_diag_kernel, dim3((unsigned)n), dim3(64), 0, s, T, X, nset,
                     nk, nip, nao, scale, rho);
  FISDF_HIP(hipGetLastError());
  return 0;
}

int scale_rows(hipStream_t s, const cplx* X, const cplx* v, int nset, int nk, int nip, int i0,
               int nb, int nao, cplx* Xv) {
  long n = (long)nset * nk * nb * nao;
  if (n == 0) return 0;
  hipLaunchKernelGGL(scale_rows_kernel, dim3(nblocks(n, 256, 1L << 30)), dim3(256), 0, s, X, v,
                     nset, nk, nip, i0, nb, nao, Xv);
  FISDF_HIP(hipGetLastError());
  return 0;
}

int kmesh_half_count(const int kmesh[3]) {
  const int nk = kmesh[0] * kmesh[1] * kmesh[2];
  return nk == 0 ? 0 : kmesh_rep_slot(nk, kmesh[0], kmesh[1], kmesh[2]);
}

int kmesh_rep_runs(const int kmesh[3], std::vector<int>* runs) {
  const int nk = kmesh[0] * kmesh[1] * kmesh[2];
  runs->clear();
  for (int k = 0; k < nk;) {
    if (!kmesh_is_rep(k, kmesh[0], kmesh[1], kmesh[2])) { ++k; continue; }
    int e = k;
    while (e < nk && kmesh_is_rep(e, kmesh[0], kmesh[1], kmesh[2])) ++e;
    runs->push_back(k);
    runs->push_back(e);
    k = e;
  }
  return 0;
}

#define FISDF_KM_REG_MESHES(X)                                                                 \
  X(1, 1, 1) X(1, 1, 2) X(2, 2, 2) X(3, 3, 1) X(3, 3, 3) X(4, 4, 4) X(2, 2, 1) X(1, 2, 2)       \
  X(4, 4, 1) X(2, 2, 4)

int k_wsrho_reg(hipStream_t s, cplx* B, long ncol, const int kmesh[3], const double* Ws,
                long ws_Rstride, unsigned long long* mon, bool* handled) {
  *handled = false;
  if (ncol <= 0) return 0;
  const unsigned grid = (unsigned)std::max<long>(1, std::min<long>((ncol + 63) / 64, 32768));
#define FISDF_KW(a, b, c)                                                                      \
  if (kmesh[0] == a && kmesh[1] == b && kmesh[2] == c) {                                       \
    hipLaunchKernelGGL((k_wsrho_reg_kernel<a, b, c>), dim3(grid), dim3(64), 0, s, B, ncol, Ws,  \
                       ws_Rstride, mon);                                                       \
    FISDF_HIP(hipGetLastError());                                                              \
    *handled = true;                                                                           \
    return 0;                                                                                  \
  }
  FISDF_KM_REG_MESHES(FISDF_KW)
#undef FISDF_KW
  return 0;
}

bool kmesh_y_reg_applies(const int kmesh[3], long ncol) {
  bool on = false;
#define FISDF_KM_HAS(a, b, c) on = on || (kmesh[0] == a && kmesh[1] == b && kmesh[2] == c);
  FISDF_KM_REG_MESHES(FISDF_KM_HAS)
#undef FISDF_KM_HAS
  return on && ncol < (1L << 31);
}

int kmesh_y(hipStream_t s, const cplx* FX, long ncol, const int kmesh[3], const int* h_qs,
            const int* d_qs, int nq, int m, cplx* yT, long qs, long Is, long goff,
            bool half, unsigned long long* mon, bool conj_out) {
  const int nk = kmesh[0] * kmesh[1] * kmesh[2];
  for (int i = 0; i < nq; ++i)
    FISDF_CHECK(h_qs[i] >= 0 && h_qs[i] < nk && (i == 0 || h_qs[i] > h_qs[i - 1]),
                "kmesh_y: q-list must be ascending and inside the k-mesh");
  FISDF_CHECK(kmesh[0] <= KM_MAXN && kmesh[1] <= KM_MAXN && kmesh[2] <= KM_MAXN,
              "kmesh_y: k-mesh axes must be <= 16");
  if (ncol < (1L << 31) && nk <= 64) {
    const int nc = (int)ncol;
    unsigned long long qmask = 0;
    for (int i = 0; i < nq; ++i) qmask |= 1ull << h_qs[i];
    const unsigned grid = (unsigned)std::max<long>(1, std::min<long>((ncol + 63) / 64, 32768));
    const double csign = conj_out ? -1.0 : 1.0;
#define FISDF_KM(a, b, c)                                                                      \
  if (kmesh[0] == a && kmesh[1] == b && kmesh[2] == c) {                                       \
    if (half)                                                                                  \
      hipLaunchKernelGGL((kmesh_y_reg_kernel<a, b, c, true>), dim3(grid), dim3(64), 0, s, FX,   \
                         nc, qmask, m, yT, qs, Is, goff, mon, csign);                          \
    else                                                                                       \
      hipLaunchKernelGGL((kmesh_y_reg_kernel<a, b, c, false>), dim3(grid), dim3(64), 0, s, FX,  \
                         nc, qmask, m, yT, qs, Is, goff, mon, csign);                          \
    FISDF_HIP(hipGetLastError());                                                              \
    return 0;                                                                                  \
  }
    FISDF_KM_REG_MESHES(FISDF_KM)
#undef FISDF_KM
  }
  FISDF_CHECK(!conj_out, "kmesh_y: conj_out needs the register kernel's k-mesh");
  int CT = 64;
  while (CT > 8 && sizeof(cplx) * ((size_t)nk * (CT + 1) + 3 * KM_MAXN) > 64 * 1024) CT /= 2;
  const size_t lds = sizeof(cplx) * ((size_t)nk * (CT + 1) + 3 * KM_MAXN) + sizeof(int) * nk;
  FISDF_CHECK(lds <= 160 * 1024, "kmesh_y: k-mesh too large for the LDS tile");
  FISDF_CHECK(d_qs != nullptr, "kmesh_y: device q-list required for this k-mesh");
  const long tiles = (ncol + CT - 1) / CT;
  FISDF_CHECK(tiles < (1L << 31), "kmesh_y: too many columns");
  if (tiles == 0) return 0;
  const unsigned grid = (unsigned)std::min<long>(tiles, 4096);
  hipLaunchKernelGGL(kmesh_y_kernel, dim3(grid), dim3(256), lds, s, FX, ncol, nk,
                     kmesh[0], kmesh[1], kmesh[2], d_qs, nq, m, yT, qs, Is, goff, CT, half ? 1 : 0, mon);
  FISDF_HIP(hipGetLastError());
  return 0;
}

size_t y_fused_workspace(const int kmesh[3], int nip, int nao, int m) {
  const int n0 = kmesh[0], P = kmesh[1] * kmesh[2];
  if (n0 * P > 64 || n0 > 4 || P > 16 || m <= 0 || nip <= 0 || nao > 128)
    return 0;
  const int nr = (n0 % 2 == 0 && n0 > 1) ? 2 : 1;
  int nslot = n0 >= 3 ? P : 0;  // chunk A + chunk B (in-plane representatives), upper bound
  nslot += nr * P;
  return sizeof(cplx) * (size_t)nslot * nao * ((size_t)nip + m);
}

// the fused kernel's slot plan and q mask for this k-mesh / q-list; false: the fused kernel
// does not apply (the caller's two-kernel path runs)
static int yf_setup(const int kmesh[3], int nao, const int* h_qs, int nq, YfPlan* plan,
                    unsigned long long* qmask, size_t* lds, bool* ok) {
  *ok = false;
  const int n0 = kmesh[0], n1 = kmesh[1], n2 = kmesh[2];
  const int nk = n0 * n1 * n2, P = n1 * n2;
  if (nk > 64 || n0 > 4 || P > 16 || nao > 128) return 0;
  for (int i = 0; i < nq; ++i)
    FISDF_CHECK(h_qs[i] >= 0 && h_qs[i] < nk && (i == 0 || h_qs[i] > h_qs[i - 1]),
                "y_fused: q-list must be ascending and inside the k-mesh");
  *qmask = 0;
  for (int i = 0; i < nq; ++i) *qmask |= 1ull << h_qs[i];
  // slot order of the kernel: chunk A = plane 1 (if 1 < N0 - 1), all P; chunk B = planes
  // 0 (and N0/2 if even) at their in-plane representatives bc <= -bc, ascending
  *plan = YfPlan{};
  if (n0 >= 3)
    for (int bc = 0; bc < P; ++bc) plan->kA[plan->nA++] = P + bc;
  const int nr = (n0 % 2 == 0 && n0 > 1) ? 2 : 1;
  for (int pi = 0; pi < nr; ++pi) {
    const int a = pi == 0 ? 0 : n0 / 2;
    for (int bc = 0; bc < P; ++bc) {
      const int b = bc / n2, c = bc % n2;
      if (bc <= ((n1 - b) % n1) * n2 + (n2 - c) % n2) plan->kB[plan->nB++] = a * P + bc;
    }
  }
  *lds = sizeof(cplx) * 256 * (size_t)std::max(plan->nA, plan->nB);
  *ok = *lds <= 80 * 1024;
  return 0;
}

// y_fused_kernel over the I-tiles [it0, it0 + nIt) of a (nip, m) column grid
static int yf_launch(hipStream_t s, const int kmesh[3], const cplx* XT, int nip, int nao,
                     const cplx* FT, int m, int it0, int nIt, const YfPlan& plan,
                     unsigned long long qmask, unsigned long long rmask, cplx* yT, long qs,
                     long Is, long goff, size_t lds, bool* handled) {
  const int n0 = kmesh[0], n1 = kmesh[1], n2 = kmesh[2];
  const int nGt = (m + 15) / 16;
  constexpr int gpair = 4;  // g-tiles per group of the XCD walk (2 / 8 measured no better)
  const long grid = (long)nIt * ((nGt + 8 * gpair - 1) / (8 * gpair)) * gpair * 8;
  FISDF_CHECK(grid < (1L << 31), "y_fused: grid too large");
  FISDF_CHECK(it0 >= 0 && nIt >= 1 && (it0 + nIt - 1) * 16 < nip, "y_fused: I-tiles out of range");
  static const int mode = getenv("FISDF_YF_MODE") ? atoi(getenv("FISDF_YF_MODE")) : 0;
#define FISDF_YF(a, b, c)                                                                      \
  if (n0 == a && n1 == b && n2 == c) {                                                         \
    FISDF_TRY(func_max_lds((const void*)y_fused_kernel<a, b, c>, 80 * 1024));                \
    hipLaunchKernelGGL((y_fused_kernel<a, b, c>), dim3((unsigned)grid), dim3(256), lds, s, XT,  \
                       nip, nao, FT, m, nIt, nGt, plan, qmask, rmask & qmask, yT, qs, Is, goff, \
                       mode, gpair, it0);                                                     \
    FISDF_HIP(hipGetLastError());                                                              \
    *handled = true;                                                                           \
    return 0;                                                                                  \
  }
  FISDF_YF(1, 1, 1) FISDF_YF(1, 1, 2) FISDF_YF(2, 2, 2) FISDF_YF(3, 3, 1) FISDF_YF(3, 3, 3)
  FISDF_YF(4, 4, 4) FISDF_YF(2, 2, 1) FISDF_YF(1, 2, 2) FISDF_YF(4, 4, 1) FISDF_YF(2, 2, 4)
#undef FISDF_YF
  return 0;
}

int y_fused(hipStream_t s, const cplx* X, int nip, int nao, const cplx* F, long fks, int m,
            const int kmesh[3], const int* h_qs, int nq, cplx* yT, long qs, long Is, long goff,
            unsigned long long* mon, cplx* work, size_t work_bytes, unsigned long long rmask,
            bool* handled) {
  (void)mon;  // fx_s is real by construction here (t_{-a} = conj(t_a)); nothing to monitor
  *handled = false;
  if (m <= 0 || nip <= 0) return 0;
  YfPlan plan;
  unsigned long long qmask = 0;
  size_t lds = 0;
  bool ok = false;
  FISDF_TRY(yf_setup(kmesh, nao, h_qs, nq, &plan, &qmask, &lds, &ok));
  if (!ok) return 0;
  // mu-major copies of the plan's k: XT [slot][mu][I], FT [slot][mu][g]
  const int nsl = plan.nA + plan.nB;
  FISDF_CHECK(work && work_bytes >= sizeof(cplx) * (size_t)nsl * nao * ((size_t)nip + m),
              "y_fused: workspace too small");
  cplx* XT = work;
  cplx* FT = work + (size_t)nsl * nao * nip;
  const size_t tl = sizeof(cplx) * 64 * (size_t)(nao + 1);
  // nao up to 128: 64 x 129 x 16 B of LDS
  FISDF_TRY(func_max_lds((const void*)yf_transpose_kernel, 132 * 1024));
  hipLaunchKernelGGL(yf_transpose_kernel, dim3((nip + 63) / 64, nsl), dim3(256), tl, s, X,
                     (long)nip * nao, nip, nao, plan, XT);
  FISDF_HIP(hipGetLastError());
  hipLaunchKernelGGL(yf_transpose_kernel, dim3((m + 63) / 64, nsl), dim3(256), tl, s, F, fks, m,
                     nao, plan, FT);
  FISDF_HIP(hipGetLastError());
  return yf_launch(s, kmesh, XT, nip, nao, FT, m, 0, (nip + 15) / 16, plan, qmask, rmask, yT, qs,
                   Is, goff, lds, handled);
}

bool y_fused_applies(const int kmesh[3], int nao) {
  static const int inst[][3] = {{1, 1, 1}, {1, 1, 2}, {2, 2, 2}, {3, 3, 1}, {3, 3, 3},
                                {4, 4, 4}, {2, 2, 1}, {1, 2, 2}, {4, 4, 1}, {2, 2, 4}};
  bool have = false;  // the instantiations yf_launch dispatches to
  for (const auto& k : inst) have |= k[0] == kmesh[0] && k[1] == kmesh[1] && k[2] == kmesh[2];
  if (!have) return false;
  YfPlan plan;
  unsigned long long qmask = 0;
  size_t lds = 0;
  bool ok = false;
  const int q0 = 0;
  if (yf_setup(kmesh, nao, &q0, 1, &plan, &qmask, &lds, &ok) != 0) return false;
  return ok;
}

int y_fused_stream(hipStream_t s, const cplx* x0, int ng0, int nao, const int* piv,
                   const int* progress, int* err, int nip, int rows, const cplx* F, long fks,
                   int m, const int kmesh[3], const int* h_qs, int nq, cplx* yT, long qs, long Is,
                   long goff, cplx* work, size_t work_bytes, unsigned long long rmask,
                   bool* handled, hipStream_t s2, hipEvent_t ev_a, hipEvent_t ev_b) {
  *handled = false;
  if (m <= 0 || nip <= 0) return 0;
  FISDF_CHECK(rows >= 16 && rows % 16 == 0 && rows <= 64 * 16, "y_fused_stream: bad row block");
  FISDF_CHECK(!s2 || (ev_a && ev_b), "y_fused_stream: a second stream needs two events");
  YfPlan plan;
  unsigned long long qmask = 0;
  size_t lds = 0;
  bool ok = false;
  FISDF_TRY(yf_setup(kmesh, nao, h_qs, nq, &plan, &qmask, &lds, &ok));
  if (!ok) return 0;
  const int nsl = plan.nA + plan.nB;
  FISDF_CHECK(work && work_bytes >= sizeof(cplx) * (size_t)nsl * nao * ((size_t)nip + m),
              "y_fused_stream: workspace too small");
  cplx* XT = work;
  cplx* FT = work + (size_t)nsl * nao * nip;
  const size_t tl = sizeof(cplx) * 64 * (size_t)(nao + 1);
  FISDF_TRY(func_max_lds((const void*)yf_transpose_kernel, 132 * 1024));
  FISDF_TRY(func_max_lds((const void*)yf_xt_stream_kernel, 132 * 1024));
  // f's copy needs no pivot: it runs while the selection finds the first block
  hipLaunchKernelGGL(yf_transpose_kernel, dim3((m + 63) / 64, nsl), dim3(256), tl, s, F, fks, m,
                     nao, plan, FT);
  FISDF_HIP(hipGetLastError());
  // s2 (optional): odd blocks on a second stream, so one block's tail overlaps the next one's
  // start; s waits for s2 at the end (everything after the call on s sees the whole y)
  if (s2) {
    FISDF_HIP(hipEventRecord(ev_a, s));
    FISDF_HIP(hipStreamWaitEvent(s2, ev_a, 0));
  }
  for (int lo = 0, b = 0; lo < nip; lo += rows, ++b) {
    const int hi = std::min(nip, lo + rows);
    hipStream_t sb = (s2 && (b & 1)) ? s2 : s;
    hipLaunchKernelGGL(yf_xt_stream_kernel, dim3((hi - lo + 63) / 64, nsl), dim3(256), tl, sb, x0,
                       (long)ng0 * nao, ng0, nao, piv, progress, lo, hi, nip, plan, XT, err);
    FISDF_HIP(hipGetLastError());
    bool h = false;
    FISDF_TRY(yf_launch(sb, kmesh, XT, nip, nao, FT, m, lo / 16, (hi - lo + 15) / 16, plan, qmask,
                        rmask, yT, qs, Is, goff, lds, &h));
    FISDF_CHECK(h, "y_fused_stream: no kernel for this k-mesh");
  }
  if (s2) {
    FISDF_HIP(hipEventRecord(ev_b, s2));
    FISDF_HIP(hipStreamWaitEvent(s, ev_b, 0));
  }
  *handled = true;
  return 0;
}

int pair_product(hipStream_t s, const cplx* A, int n1, const cplx* B, int n2, int nip, cplx* P) {
  long n = (long)nip * n1 * n2;
  if (n == 0) return 0;
  hipLaunchKernelGGL(pair_product_kernel, dim3(nblocks(n, 256, 1L << 30)), dim3(256), 0, s, A, n1,
                     B, n2, nip, P);
  FISDF_HIP(hipGetLastError());
  return 0;
}

// out[g][j*nao + m] = scale_j * x0[k_j][g][m] for the listed k (the time-reversal-folded Gram);
// the k list travels in the kernel argument block, 64 entries per launch: a longer list (more
// than 64 representatives, e.g. 112 at 6x6x6) runs as several launches over column ranges
struct KgmSel {
  int k[64];
  double sc[64];
};
__global__ void permute_kgm_sel_kernel(const cplx* __restrict__ x0, KgmSel sel, int j0, int nchunk,
                                       int nsel, int ng, int nao, cplx* __restrict__ out) {
  long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long tot = (long)nchunk * ng * nao;
  if (e >= tot) return;
  const int m = (int)(e % nao);
  const int g = (int)((e / nao) % ng);
  const int j = (int)(e / ((long)nao * ng));
  out[(long)g * nsel * nao + (long)(j0 + j) * nao + m] =
      cscale(x0[((long)sel.k[j] * ng + g) * nao + m], sel.sc[j]);
}

int permute_kgm_sel(hipStream_t s, const cplx* x0, const int* h_k, const double* h_sc, int nsel,
                    int ng, int nao, cplx* out) {
  FISDF_CHECK(nsel >= 1, "permute_kgm_sel: no k-points");
  for (int j0 = 0; j0 < nsel; j0 += 64) {
    const int nc = std::min(64, nsel - j0);
    KgmSel sel;
    for (int j = 0; j < nc; ++j) {
      sel.k[j] = h_k[j0 + j];
      sel.sc[j] = h_sc[j0 + j];
    }
    const long n = (long)nc * ng * nao;
    hipLaunchKernelGGL(permute_kgm_sel_kernel, dim3(nblocks(n, 256, 1L << 30)), dim3(256), 0, s,
                       x0, sel, j0, nc, nsel, ng, nao, out);
    FISDF_HIP(hipGetLastError());
  }
  return 0;
}

// the time-reversal representatives k <= -k of the k-mesh and whether each is its own partner
void kmesh_reps(const int kmesh[3], std::vector<int>* reps, std::vector<char>* self) {
  const int nk = kmesh[0] * kmesh[1] * kmesh[2];
  reps->clear();
  self->clear();
  for (int k = 0; k < nk; ++k) {
    const int p = kmesh_partner(k, kmesh[0], kmesh[1], kmesh[2]);
    if (k <= p) {
      reps->push_back(k);
      self->push_back(k == p ? 1 : 0);
    }
  }
}

// time-reversal check of Bloch AO values a[k][r][m] (k stride ks): mon[0] = max over the
// representatives k <= -k of |a[-k] - conj(a[k])| (2 |Im a[k]| on a self-paired k), mon[1] = max
// |a[k]|, both as the ordered bit patterns of non-negative doubles.  Every pair is read once.
__global__ void tr_check_kernel(const cplx* __restrict__ a, long ks, long per_k, int nao,
                                long rstride, int n0, int n1, int n2,
                                unsigned long long* __restrict__ mon) {
  const int nk = n0 * n1 * n2;
  double dev = 0.0, mag = 0.0;
  const long tot = (long)nk * per_k;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < tot;
       e += (long)gridDim.x * blockDim.x) {
    const int k = (int)(e / per_k);
    const long i = e - (long)k * per_k;  // sampled row i / nao (every rstride-th row), AO i % nao
    const long r = (i / nao) * rstride * nao + i % nao;
    const int p = kmesh_partner(k, n0, n1, n2);
    if (p < k) continue;
    const cplx u = a[k * ks + r];
    const cplx v = p == k ? u : a[p * ks + r];
    dev = fmax(dev, fmax(fabs(v.x - u.x), fabs(v.y + u.y)));
    mag = fmax(mag, fmax(fabs(u.x), fabs(u.y)));
  }
  for (int o = 32; o > 0; o >>= 1) {
    dev = fmax(dev, __shfl_xor(dev, o, 64));
    mag = fmax(mag, __shfl_xor(mag, o, 64));
  }
  // one pair of device atomics per workgroup: the per-wave atomics (32 k of them on two words,
  // serialised in the memory fabric) cost ~0.9 ms per build at C3
  __shared__ double red[2][4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = dev;
    red[1][w] = mag;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) {
      dev = fmax(dev, red[0][i]);
      mag = fmax(mag, red[1][i]);
    }
    atomicMax(mon, (unsigned long long)__double_as_longlong(dev));
    atomicMax(mon + 1, (unsigned long long)__double_as_longlong(mag));
  }
}

int tr_check(hipStream_t s, const cplx* a, long ks, long rows, int nao, long rstride,
             const int kmesh[3], unsigned long long* mon) {
  FISDF_CHECK(rows > 0 && nao > 0 && rstride > 0 && ks >= rows * nao && kmesh[0] > 0 &&
                  kmesh[1] > 0 && kmesh[2] > 0,
              "tr_check: bad sizes");
  const long per_k = ((rows + rstride - 1) / rstride) * nao;
  const long n = (long)kmesh[0] * kmesh[1] * kmesh[2] * per_k;
  hipLaunchKernelGGL(tr_check_kernel, dim3(nblocks(n, 256, 1024)), dim3(256), 0, s, a, ks, per_k,
                     nao, rstride, kmesh[0], kmesh[1], kmesh[2], mon);
  FISDF_HIP(hipGetLastError());
  return 0;
}

int permute_kgm(hipStream_t s, const cplx* x0, int nq, int ng, int nao, cplx* out) {
  long n = (long)nq * ng * nao;
  if (n == 0) return 0;
  hipLaunchKernelGGL(permute_kgm_kernel, dim3(nblocks(n, 256, 1L << 30)), dim3(256), 0, s, x0, nq,
                     ng, nao, out);
  FISDF_HIP(hipGetLastError());
  return 0;
}

int gather_points(hipStream_t s, const cplx* x0, int nk, int ng0, int nao, const int* perm,
                  int nip, cplx* X) {
  long n = (long)nk * nip * nao;
  if (n == 0) return 0;
  hipLaunchKernelGGL(gather_points_kernel, dim3(nblocks(n, 256, 1L << 30)), dim3(256), 0, s, x0,
                     nk, ng0, nao, perm, nip, X);
  FISDF_HIP(hipGetLastError());
  return 0;
}

int square_scale(hipStream_t s, const cplx* in, double sc, cplx* out, long n) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(square_scale_kernel, dim3(nblocks(n, 256, 8192)), dim3(256), 0, s, in, sc,
                     out, n);
  FISDF_HIP(hipGetLastError());
  return 0;
}

}  // namespace fisdf
