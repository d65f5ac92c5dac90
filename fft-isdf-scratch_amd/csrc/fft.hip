// Batched 3-D complex FFT over the plane-wave mesh (forward, unnormalised, numpy sign).
//
// Replaces pbctools.fft(z_q * fq, mesh) of fftisdf.py:113 (and the fq = exp(-i k_q.r)
// of :99, the coulG weight of :114-115).  Only the FORWARD transform is needed: the
// inverse FFT + zeta z^H of :118-121 is folded into a Coulomb-weighted HERK by
// Parseval, so `weight` carries sqrt(coulG(k_q+G) * vol/ngrid^2).
//
// One kernel per axis.  A workgroup stages a tile of TL lines x n points
// (n = mesh[axis] <= 64) in LDS with coalesced loads (the TL lines are the
// contiguous inner index for the strided axes), runs a mixed-radix Stockham FFT
// (radix 4/2/3/5/7/11/13, twiddles from an n-th-root table in LDS) ping-ponging
// between two LDS buffers, and writes the tile back.  The first pass (axis 2)
// fuses the row gather (interpolation-point pivots) and the exp(-i k.r) phase,
// the last pass (axis 0) fuses the Coulomb weight.
#include <type_traits>

#include "common.h"

typedef double fft_dv2 __attribute__((ext_vector_type(2)));


#include <map>
#include <mutex>
#include <vector>
#include <cmath>

namespace fisdf {

namespace {

constexpr int MAXN = 64;
constexpr int MAXST = 8;

struct Stages {
  int nst;
  int radix[MAXST];
};

template <int R>
__device__ __forceinline__ void dft_small(cplx* v, const cplx* __restrict__ tw, int n) {
  // out[k] = sum_r v[r] * exp(-2 pi i r k / R);  exp(-2 pi i x / R) = tw[x * n / R]
  if constexpr (R == 2) {
    cplx a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
  } else if constexpr (R == 4) {
    cplx a0 = cadd(v[0], v[2]), a1 = csub(v[0], v[2]);
    cplx b0 = cadd(v[1], v[3]), b1 = csub(v[1], v[3]);
    // b1 * (-i)
    cplx b1m = cmk(b1.y, -b1.x);
    v[0] = cadd(a0, b0);
    v[2] = csub(a0, b0);
    v[1] = cadd(a1, b1m);
    v[3] = csub(a1, b1m);
  } else {
    cplx o[R];
    const int step = n / R;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      cplx acc = v[0];
#pragma unroll
      for (int r = 1; r < R; ++r) acc = cadd(acc, cmul(v[r], tw[((r * k) % R) * step]));
      o[k] = acc;
    }
#pragma unroll
    for (int k = 0; k < R; ++k) v[k] = o[k];
  }
}

// one Stockham radix-R stage over TL lines held in LDS; element p of line l at p*ps + l*ls
template <int R>
__device__ __forceinline__ void stockham_stage(const cplx* __restrict__ src, cplx* __restrict__ dst,
                                               const cplx* __restrict__ tw, int n, int Ns, int TL,
                                               int ps, int ls, int tid, int nthr) {
  const int nb = n / R;
  const int total = nb * TL;
  const int twstep = n / (Ns * R);
  for (int bf = tid; bf < total; bf += nthr) {
    const int l = bf % TL, j = bf / TL;
    cplx v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = src[(j + r * nb) * ps + l * ls];
    const int k = j % Ns;
    if (Ns > 1) {
#pragma unroll
      for (int r = 1; r < R; ++r) v[r] = cmul(v[r], tw[(k * r * twstep) % n]);
    }
    dft_small<R>(v, tw, n);
    const int idx = (j / Ns) * Ns * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) dst[(idx + r * Ns) * ps + l * ls] = v[r];
  }
}

// full line FFT of TL lines (all stages), ping-pong a <-> b; returns the buffer holding the result.
// BIG instantiates the generic radix 7/11/13 butterflies (register-hungry: only for meshes
// that need them, so the common 2/3/4/5 meshes keep occupancy).
template <bool BIG>
__device__ cplx* lds_fft_lines(cplx* a, cplx* b, const cplx* tw, int n, const int* radix, int nst,
                               int TL, int ps, int ls, int tid, int nthr) {
  int Ns = 1;
  for (int s = 0; s < nst; ++s) {
    const int R = radix[s];
    switch (R) {
      case 2: stockham_stage<2>(a, b, tw, n, Ns, TL, ps, ls, tid, nthr); break;
      case 3: stockham_stage<3>(a, b, tw, n, Ns, TL, ps, ls, tid, nthr); break;
      case 4: stockham_stage<4>(a, b, tw, n, Ns, TL, ps, ls, tid, nthr); break;
      case 5: stockham_stage<5>(a, b, tw, n, Ns, TL, ps, ls, tid, nthr); break;
      case 7: if constexpr (BIG) stockham_stage<7>(a, b, tw, n, Ns, TL, ps, ls, tid, nthr); break;
      case 11: if constexpr (BIG) stockham_stage<11>(a, b, tw, n, Ns, TL, ps, ls, tid, nthr); break;
      case 13: if constexpr (BIG) stockham_stage<13>(a, b, tw, n, Ns, TL, ps, ls, tid, nthr); break;
    }
    Ns *= R;
    __syncthreads();
    cplx* t = a;
    a = b;
    b = t;
  }
  return a;
}

__device__ __forceinline__ double fftfreq(int i, int n) {
  return (double)(i < (n + 1) / 2 ? i : i - n) / (double)n;
}

// axis pass. contiguous=1: lines are `n` contiguous elements (axis 2); tiles = TL consecutive lines.
// contiguous=0: element p of line (o, ii) at o*n*inner + p*inner + ii; tile = TL consecutive ii.
template <bool BIG>
__global__ __launch_bounds__(256) void fft_axis_kernel(
    const cplx* __restrict__ in, long in_ld, const int* __restrict__ rowidx, cplx* out, long out_ld,
    int rows, int n, int inner, int outer, int TL, int contiguous, Stages st,
    const cplx* __restrict__ twg, int n0, int n1, int n2, double kd0, double kd1, double kd2,
    int use_phase, const double* __restrict__ weight) {
  extern __shared__ cplx smem[];
  cplx* tw = smem;                 // n roots
  cplx* buf0 = smem + MAXN;        // TL*n
  cplx* buf1 = buf0 + TL * n;      // TL*n
  const int tid = threadIdx.x, nthr = blockDim.x;
  for (int t = tid; t < n; t += nthr) tw[t] = twg[t];

  // tile -> (row, line block)
  long tile = blockIdx.x;
  int tiles_per_row = contiguous ? (outer + TL - 1) / TL : outer * (inner / TL);
  int row = (int)(tile / tiles_per_row);
  int trow = (int)(tile % tiles_per_row);
  if (row >= rows) return;
  const cplx* src = in + (long)(rowidx ? rowidx[row] : row) * in_ld;
  cplx* dstp = out + (long)row * out_ld;
  const int ngrid = n0 * n1 * n2;

  long base;       // element offset of (line 0, p 0) of the tile inside the row
  int nlines = TL;
  if (contiguous) {
    int o0 = trow * TL;
    nlines = min(TL, outer - o0);
    base = (long)o0 * n;
  } else {
    int o = trow / (inner / TL), ib = trow % (inner / TL);
    base = (long)o * n * inner + (long)ib * TL;
  }
  auto gidx = [&](int l, int p) -> long {
    return contiguous ? base + (long)l * n + p : base + (long)p * inner + l;
  };

  const int tot = TL * n;
  // first U elements per thread: loads issued together (branch-free, clamped address)
  constexpr int U = 8;
  cplx pre[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = tid + u * nthr;
    int l, p;
    if (contiguous) { l = e / n; p = e % n; } else { l = e % TL; p = e / TL; }
    const bool ok = e < tot && l < nlines;
    pre[u] = src[ok ? gidx(l, p) : 0];
  }
  __syncthreads();
  auto put = [&](int e, cplx v) {
    int l, p;
    if (contiguous) { l = e / n; p = e % n; } else { l = e % TL; p = e / TL; }
    if (l < nlines) {
      if (use_phase) {
        long g = gidx(l, p);
        int i2 = (int)(g % n2);
        int i1 = (int)((g / n2) % n1);
        int i0 = (int)(g / ((long)n1 * n2));
        double th = -(fftfreq(i0, n0) * kd0 + fftfreq(i1, n1) * kd1 + fftfreq(i2, n2) * kd2);
        double s, c;
        sincos(th, &s, &c);
        v = cmul(v, cmk(c, s));
      }
    } else {
      v = cmk(0, 0);
    }
    buf0[p * TL + l] = v;
  };
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = tid + u * nthr;
    if (e < tot) put(e, pre[u]);
  }
  for (int e = tid + U * nthr; e < tot; e += nthr) {
    int l, p;
    if (contiguous) { l = e / n; p = e % n; } else { l = e % TL; p = e / TL; }
    put(e, l < nlines ? src[gidx(l, p)] : cmk(0, 0));
  }
  __syncthreads();
  cplx* a = lds_fft_lines<BIG>(buf0, buf1, tw, n, st.radix, st.nst, TL, TL, 1, tid, nthr);
  for (int e = tid; e < tot; e += nthr) {
    int l, p;
    if (contiguous) { l = e / n; p = e % n; } else { l = e % TL; p = e / TL; }
    if (l < nlines) {
      long g = gidx(l, p);
      cplx v = a[p * TL + l];
      if (weight) v = cscale(v, weight[g % ngrid]);
      dstp[g] = v;
    }
  }
}

// 2-D FFT of one (i1, i2) plane (n1*n2 contiguous points) per workgroup: axes 2 and 1 in
// LDS, one HBM round trip instead of two.  Fuses the row gather and exp(-i k.r).
template <bool BIG>
__global__ __launch_bounds__(256) void fft_plane_kernel(
    const cplx* __restrict__ in, long in_ld, const int* __restrict__ rowidx, cplx* out, long out_ld,
    int rows, Stages st1, Stages st2, const cplx* __restrict__ tw1g, const cplx* __restrict__ tw2g,
    int n0, int n1, int n2, double kd0, double kd1, double kd2, int use_phase,
    const PlaneRef* __restrict__ planes) {
  extern __shared__ cplx smem[];
  cplx* tw1 = smem;
  cplx* tw2 = smem + MAXN;
  cplx* ph1 = smem + 2 * MAXN;  // exp(-i f(i1) kd1) * exp(-i f(i0) kd0)
  cplx* ph2 = smem + 3 * MAXN;  // exp(-i f(i2) kd2)
  const int P = n1 * n2;
  cplx* buf0 = smem + 4 * MAXN;
  cplx* buf1 = buf0 + P;
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int row = blockIdx.x / n0, i0 = blockIdx.x % n0;
  if (row >= rows) return;
  const long r = rowidx ? rowidx[row] : row;
  const cplx* src = planes ? in + planes[i0].base + r * planes[i0].ld : in + r * in_ld + (long)i0 * P;
  cplx* dstp = out + (long)row * out_ld + (long)i0 * P;
  // issue this plane's loads first (branch-free, up to 8 per thread in flight)
  constexpr int U = 8;
  cplx v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = tid + u * nthr;
    v[u] = src[e < P ? e : 0];
  }
  for (int t = tid; t < n1; t += nthr) tw1[t] = tw1g[t];
  for (int t = tid; t < n2; t += nthr) tw2[t] = tw2g[t];
  if (use_phase) {
    // separable phase exp(-i k.r) = e0(i0) e1(i1) e2(i2): one sincos per axis entry
    double s0, c0;
    sincos(-fftfreq(i0, n0) * kd0, &s0, &c0);
    for (int t = tid; t < n1; t += nthr) {
      double s, c;
      sincos(-fftfreq(t, n1) * kd1, &s, &c);
      ph1[t] = cmul(cmk(c, s), cmk(c0, s0));
    }
    for (int t = tid; t < n2; t += nthr) {
      double s, c;
      sincos(-fftfreq(t, n2) * kd2, &s, &c);
      ph2[t] = cmk(c, s);
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = tid + u * nthr;
    if (e < P) {
      cplx x = v[u];
      if (use_phase) x = cmul(x, cmul(ph1[e / n2], ph2[e % n2]));
      buf0[e] = x;
    }
  }
  for (int e = tid + U * nthr; e < P; e += nthr) {  // planes larger than U*256 points
    cplx x = src[e];
    if (use_phase) x = cmul(x, cmul(ph1[e / n2], ph2[e % n2]));
    buf0[e] = x;
  }
  __syncthreads();
  // axis 2: n1 lines of n2 contiguous points (p stride 1, line stride n2)
  cplx* a = lds_fft_lines<BIG>(buf0, buf1, tw2, n2, st2.radix, st2.nst, n1, 1, n2, tid, nthr);
  cplx* b = a == buf0 ? buf1 : buf0;
  // axis 1: n2 lines of n1 points (p stride n2, line stride 1)
  a = lds_fft_lines<BIG>(a, b, tw1, n1, st1.radix, st1.nst, n2, n2, 1, tid, nthr);
  for (int e = tid; e < P; e += nthr) dstp[e] = a[e];
}

// ---- register FFT kernels for the common meshes (compile-time line length) -------------
// A line of N points lives in one lane's registers and is transformed by a fully unrolled
// mixed-radix Cooley-Tukey recursion (radix 4/2/3/5, prime lengths by direct DFT) with
// compile-time twiddle indices: trivial twiddles (+-1, +-i) cost nothing and the rest are
// wave-uniform loads from the n-th-root table.  The plane kernel does axes 2 and 1 of one
// (i0) plane per wave through a padded LDS image; the axis-0 kernel needs no LDS at all:
// lane = consecutive (i1, i2) column, so every one of its N0 loads/stores is a contiguous
// 16*64-byte wave access.
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

constexpr int first_factor(int n) {
  return (n % 4 == 0 && n > 4) ? 4 : (n % 2 == 0 && n > 2) ? 2 : (n % 3 == 0 && n > 3) ? 3
       : (n % 5 == 0 && n > 5) ? 5 : n;
}

// v * W_NT^E (W_NT^t = exp(-2 pi i t / NT) = W[t])
template <int NT, int E>
__device__ __forceinline__ cplx twmul(cplx v, const cplx* __restrict__ W) {
  constexpr int e = E % NT;
  if constexpr (e == 0) return v;
  else if constexpr (4 * e == NT) return cmk(v.y, -v.x);       // * (-i)
  else if constexpr (2 * e == NT) return cmk(-v.x, -v.y);      // * (-1)
  else if constexpr (4 * e == 3 * NT) return cmk(-v.y, v.x);   // * (+i)
  else return cmul(v, W[e]);
}

template <int N, int NT>
__device__ __forceinline__ void fft_rec(cplx* x, const cplx* __restrict__ W) {
  if constexpr (N == 1) {
  } else if constexpr (N == 2) {
    const cplx a = x[0], b = x[1];
    x[0] = cadd(a, b);
    x[1] = csub(a, b);
  } else if constexpr (N == 4) {
    const cplx a0 = cadd(x[0], x[2]), a1 = csub(x[0], x[2]);
    const cplx b0 = cadd(x[1], x[3]), b1 = csub(x[1], x[3]);
    const cplx b1m = cmk(b1.y, -b1.x);  // b1 * (-i)
    x[0] = cadd(a0, b0);
    x[2] = csub(a0, b0);
    x[1] = cadd(a1, b1m);
    x[3] = csub(a1, b1m);
  } else if constexpr (first_factor(N) == N) {  // prime: direct DFT
    cplx o[N];
    static_for<0, N>([&](auto kc) {
      constexpr int K = decltype(kc)::value;
      cplx acc = x[0];
      static_for<1, N>([&](auto jc) {
        constexpr int J = decltype(jc)::value;
        acc = cadd(acc, twmul<NT, ((J * K) % N) * (NT / N)>(x[J], W));
      });
      o[K] = acc;
    });
    static_for<0, N>([&](auto kc) { x[decltype(kc)::value] = o[decltype(kc)::value]; });
  } else {
    // n = B n1 + n2, k = k1 + A k2:  X = DFT_B_n2[ W_N^(n2 k1) DFT_A_n1[x] ]
    constexpr int A = first_factor(N), B = N / A;
    cplx y[N];
    static_for<0, B>([&](auto n2c) {
      constexpr int N2 = decltype(n2c)::value;
      cplx t[A];
      static_for<0, A>([&](auto c) { t[decltype(c)::value] = x[B * decltype(c)::value + N2]; });
      fft_rec<A, NT>(t, W);
      static_for<0, A>([&](auto c) {
        constexpr int K1 = decltype(c)::value;
        y[K1 * B + N2] = twmul<NT, (N2 * K1) * (NT / N)>(t[K1], W);
      });
    });
    static_for<0, A>([&](auto k1c) {
      constexpr int K1 = decltype(k1c)::value;
      cplx t[B];
      static_for<0, B>([&](auto c) { t[decltype(c)::value] = y[K1 * B + decltype(c)::value]; });
      fft_rec<B, NT>(t, W);
      static_for<0, B>([&](auto c) { x[K1 + A * decltype(c)::value] = t[decltype(c)::value]; });
    });
  }
}

// axes 2 and 1 of one (row, i0) plane per 64-lane workgroup; fuses the row gather and the
// separable phase exp(-i k.r) = e0(i0) e1(i1) e2(i2)
template <int NN>
__global__ __launch_bounds__(64) void fft_plane_reg(const cplx* __restrict__ in, long in_ld,
                                                    const int* __restrict__ rowidx, cplx* out,
                                                    long out_ld, int rows, int n0,
                                                    const cplx* __restrict__ W, double kd0,
                                                    double kd1, double kd2, int use_phase,
                                                    const PlaneRef* __restrict__ planes,
                                                    int nrow_out, int in_real) {
  constexpr int P = NN * NN, LD = NN + 1;
  __shared__ cplx img[NN * LD];
  __shared__ cplx ph1[NN], ph2[NN];
  const int lane = threadIdx.x;
  const int row = blockIdx.x / n0, i0 = blockIdx.x % n0;
  if (row >= rows) return;
  const long r = rowidx ? rowidx[row] : row;
  const cplx* src = planes ? in + planes[i0].base + r * planes[i0].ld : in + r * in_ld + (long)i0 * P;
  cplx* dst = out + (long)row * out_ld + (long)i0 * P;
  constexpr int U = (P + 63) / 64;
  cplx v[U];
  if (in_real) {  // real rows (a self-conjugate q's y): doubles at the same offsets
    const double* srr = (const double*)in + r * in_ld + (long)i0 * P;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = lane + 64 * u;
      v[u] = cmk(srr[e < P ? e : 0], 0.0);
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = lane + 64 * u;
      v[u] = src[e < P ? e : 0];
    }
  }
  if (use_phase && lane < NN) {
    double s0, c0, s, c;
    sincos(-fftfreq(i0, n0) * kd0, &s0, &c0);
    sincos(-fftfreq(lane, NN) * kd1, &s, &c);
    ph1[lane] = cmul(cmk(c, s), cmk(c0, s0));
    sincos(-fftfreq(lane, NN) * kd2, &s, &c);
    ph2[lane] = cmk(c, s);
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = lane + 64 * u;
    if (e < P) {
      const int i1 = e / NN, i2 = e - i1 * NN;
      cplx x = v[u];
      if (use_phase) x = cmul(x, cmul(ph1[i1], ph2[i2]));
      img[i1 * LD + i2] = x;
    }
  }
  __syncthreads();
  if (lane < NN) {  // axis 2: line i1 = lane
    cplx x[NN];
#pragma unroll
    for (int p = 0; p < NN; ++p) x[p] = img[lane * LD + p];
    fft_rec<NN, NN>(x, W);
#pragma unroll
    for (int p = 0; p < NN; ++p) img[lane * LD + p] = x[p];
  }
  __syncthreads();
  if (lane < NN) {  // axis 1: line i2 = lane
    cplx x[NN];
#pragma unroll
    for (int p = 0; p < NN; ++p) x[p] = img[p * LD + lane];
    fft_rec<NN, NN>(x, W);
#pragma unroll
    for (int p = 0; p < NN; ++p) img[p * LD + lane] = x[p];
  }
  __syncthreads();
  // lines j1 < nrow_out only (all of them, or the Hermitian prefix: fft_axis0_herm)
  const int Pout = nrow_out * NN;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = lane + 64 * u;
    if (e < Pout) {
      const int i1 = e / NN, i2 = e - i1 * NN;
      dst[e] = img[i1 * LD + i2];
    }
  }
}

// axis 0: one line (row, column l = i1*n1n2... ) per lane, N0 strided loads, in registers
template <int N0>
__global__ __launch_bounds__(256) void fft_axis0_reg(const cplx* in, long in_ld, cplx* out,
                                                     long out_ld, int rows, int P,
                                                     const cplx* __restrict__ W,
                                                     const double* __restrict__ weight) {
  const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (t >= (long)rows * P) return;
  const int row = (int)(t / P), l = (int)(t - (long)row * P);
  const cplx* src = in + (long)row * in_ld + l;
  cplx* dst = out + (long)row * out_ld + l;
  cplx x[N0];
#pragma unroll
  for (int p = 0; p < N0; ++p) x[p] = src[(long)p * P];
  fft_rec<N0, N0>(x, W);
  if (weight) {
#pragma unroll
    for (int p = 0; p < N0; ++p) x[p] = cscale(x[p], weight[(long)p * P + l]);
  }
#pragma unroll
  // the final pass's output (Yhat, 0.45 GB per q at C3, read by the fit's triangular GEMM once its
  // lane gets there) is stored non-temporally: it streams past the L2s the MFMA lanes' operands
  // live in (C3 -1.1 ms/step; the first pass's output, re-read at once, keeps plain stores:
  // profiles/r03_ab/gemm_pipe.log)
  for (int p = 0; p < N0; ++p)
    __builtin_nontemporal_store(fft_dv2{x[p].x, x[p].y}, (fft_dv2*)(dst + (long)p * P));
}

constexpr int herm_prefix(int n, int m) {
  int nH = 0;
  for (int i = 0; i < n; ++i)
    if (i <= ((-i - m) % n + n) % n) nH = i + 1;
  return nH;
}

// axis 0 of a Hermitian-paired transform (a self-conjugate q: out(j') = conj(out(j)),
// j' = -j - m): the plane pass wrote only the lines j1 < n1H.  A column (j1', j2') on a line it
// skipped is the partner of a stored column (j1, j2) = (-j1' - m1, -j2' - m2), and
//   T(i0, j1', j2') = e^{-2 pi i m0 i0 / n0} conj(T(i0, j1, j2))
// (the axis-0 phase squared).  Lanes l and l + 32 of a wave take one stored column and its
// partner: both read the stored column (the same addresses, one fetch), the partner lane
// conjugates and twiddles, each transforms its column and stores its prefix planes j0 < NH.
// The transform is in place: the wave's loads all complete before its first store, and no other
// wave touches the pair, so reading a column another lane overwrites is race-free.  Columns of
// the self-paired lines (both members stored) take one lane each (blocks past npb).  Per lane
// the same registers as fft_axis0_reg; moves n1H / n1 of its intermediate and NH / n0 of its
// output.
template <int N0, int M0>
__global__ __launch_bounds__(256) void fft_axis0_herm(const cplx* in, long in_ld, cplx* out,
                                                      long out_ld, int rows, int n1, int n2,
                                                      int m1, int m2, int lo, int hi, int sl0,
                                                      int sl1, int npb,
                                                      const cplx* __restrict__ W,
                                                      const double* __restrict__ weight) {
  constexpr int NH = herm_prefix(N0, M0);
  const int P = n1 * n2;
  const int lane = threadIdx.x & 63;
  int row, c, d;
  bool flip = false;
  if ((int)blockIdx.x < npb) {  // pair region: 32 stored columns and their partners per wave
    const long npr = (long)(hi - lo) * n2;
    const long k = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * 32 + (lane & 31);
    if (k >= (long)rows * npr) return;
    row = (int)(k / npr);
    const int kk = (int)(k - (long)row * npr);
    const int j1 = lo + kk / n2, j2 = kk - (kk / n2) * n2;
    c = j1 * n2 + j2;
    flip = lane >= 32;
    d = flip ? (((-j1 - m1) % n1 + n1) % n1) * n2 + ((-j2 - m2) % n2 + n2) % n2 : c;
  } else {  // self-paired lines sl0, sl1 (-1: none)
    const int nsl = (sl0 >= 0) + (sl1 >= 0);
    const long nsr = (long)nsl * n2;
    const long s = (long)(blockIdx.x - npb) * 256 + threadIdx.x;
    if (s >= (long)rows * nsr) return;
    row = (int)(s / nsr);
    const int ss = (int)(s - (long)row * nsr);
    const int li = ss / n2;
    const int j1 = (li == 0 && sl0 >= 0) ? sl0 : sl1;
    c = d = j1 * n2 + (ss - li * n2);
  }
  const cplx* src = in + (long)row * in_ld + c;
  cplx* dst = out + (long)row * out_ld + d;
  cplx x[N0];
#pragma unroll
  for (int p = 0; p < N0; ++p) x[p] = src[(long)p * P];
  if (flip) {
#pragma unroll
    for (int p = 0; p < N0; ++p) {
      x[p].y = -x[p].y;
      if constexpr (M0 != 0) x[p] = cmul(x[p], W[(p * M0) % N0]);
    }
  }
  fft_rec<N0, N0>(x, W);
  if (weight) {
#pragma unroll
    for (int p = 0; p < NH; ++p) x[p] = cscale(x[p], weight[(long)p * P + d]);
  }
  // same non-temporal stores as fft_axis0_reg
#pragma unroll
  for (int p = 0; p < NH; ++p)
    __builtin_nontemporal_store(fft_dv2{x[p].x, x[p].y}, (fft_dv2*)(dst + (long)p * P));
}

// meshes with register kernels (cubic n^3 for the plane kernel; any n0 for axis 0)
#define FISDF_REG_SIZES(X) X(8) X(12) X(13) X(15) X(16) X(18) X(20) X(24) X(25) X(27) X(30) X(32) X(36) X(40) X(45) X(48)

int fft_plane_reg_launch(hipStream_t s, int n, const cplx* in, long in_ld, const int* rowidx,
                         cplx* out, long out_ld, int rows, int n0, const cplx* W, const double* kd,
                         const PlaneRef* planes, int nrow_out, bool in_real, bool* done) {
  *done = false;
  const double k0 = kd ? kd[0] : 0, k1 = kd ? kd[1] : 0, k2 = kd ? kd[2] : 0;
  const long nplanes = (long)rows * n0;
#define FISDF_PL(N)                                                                            \
  if (n == N) {                                                                                \
    hipLaunchKernelGGL(fft_plane_reg<N>, dim3((unsigned)nplanes), dim3(64), 0, s, in, in_ld,    \
                       rowidx, out, out_ld, rows, n0, W, k0, k1, k2, kd ? 1 : 0, planes,        \
                       nrow_out, in_real ? 1 : 0);                                            \
    *done = true;                                                                              \
  }
  FISDF_REG_SIZES(FISDF_PL)
#undef FISDF_PL
  if (*done) FISDF_HIP(hipGetLastError());
  return 0;
}

int fft_axis0_reg_launch(hipStream_t s, int n0, const cplx* in, long in_ld, cplx* out, long out_ld,
                         int rows, int P, const cplx* W, const double* weight, bool* done) {
  *done = false;
  const long threads = (long)rows * P;
  const unsigned blocks = (unsigned)((threads + 255) / 256);
#define FISDF_AX(N)                                                                            \
  if (n0 == N) {                                                                               \
    hipLaunchKernelGGL(fft_axis0_reg<N>, dim3(blocks), dim3(256), 0, s, in, in_ld, out, out_ld, \
                       rows, P, W, weight);                                                    \
    *done = true;                                                                              \
  }
  FISDF_REG_SIZES(FISDF_AX)
#undef FISDF_AX
  if (*done) FISDF_HIP(hipGetLastError());
  return 0;
}

int fft_axis0_herm_launch(hipStream_t s, int n0, const cplx* in, long in_ld, cplx* out,
                          long out_ld, int rows, int n1, int n2, int n1H, const int m[3],
                          const cplx* W, const double* weight, bool* done) {
  *done = false;
  auto partner1 = [&](int j) { return ((-j - m[1]) % n1 + n1) % n1; };
  // stored lines: [lo, hi) pair with skipped lines; sl0 / sl1 are self-paired (or -1)
  const int sl0 = partner1(0) == 0 ? 0 : -1;
  const int sl1 = (n1H - 1 > 0 && partner1(n1H - 1) == n1H - 1) ? n1H - 1 : -1;
  const int lo = sl0 >= 0 ? 1 : 0, hi = sl1 >= 0 ? n1H - 1 : n1H;
  for (int j = lo; j < hi; ++j)
    FISDF_CHECK(partner1(j) >= n1H, "fft: Hermitian line pairing");
  const long pairs = (long)rows * (hi - lo) * n2;
  const long npb = (pairs + 127) / 128;  // 4 waves x 32 pairs per block
  const long nself = (long)rows * ((sl0 >= 0) + (sl1 >= 0)) * n2;
  const long blocks = npb + (nself + 255) / 256;
  FISDF_CHECK(blocks < (1L << 31), "fft: too many blocks");
#define FISDF_AXH(N)                                                                           \
  if (n0 == N) {                                                                               \
    if (m[0] == 0)                                                                             \
      hipLaunchKernelGGL((fft_axis0_herm<N, 0>), dim3((unsigned)blocks), dim3(256), 0, s, in,    \
                         in_ld, out, out_ld, rows, n1, n2, m[1], m[2], lo, hi, sl0, sl1,       \
                         (int)npb, W, weight);                                                 \
    else                                                                                       \
      hipLaunchKernelGGL((fft_axis0_herm<N, 1>), dim3((unsigned)blocks), dim3(256), 0, s, in,    \
                         in_ld, out, out_ld, rows, n1, n2, m[1], m[2], lo, hi, sl0, sl1,       \
                         (int)npb, W, weight);                                                 \
    *done = true;                                                                              \
  }
  FISDF_REG_SIZES(FISDF_AXH)
#undef FISDF_AXH
  if (*done) FISDF_HIP(hipGetLastError());
  return 0;
}

bool needs_big(const Stages& st) {
  for (int i = 0; i < st.nst; ++i)
    if (st.radix[i] > 5) return true;
  return false;
}

bool factorize(int n, Stages& st) {
  st.nst = 0;
  const int rs[] = {4, 2, 3, 5, 7, 11, 13};
  for (int r : rs)
    while (n % r == 0) {
      if (st.nst >= MAXST) return false;
      st.radix[st.nst++] = r;
      n /= r;
    }
  return n == 1;
}

struct TwTable {
  cplx* dev = nullptr;
};
std::mutex g_tw_mu;
std::map<std::pair<int, int>, TwTable> g_tw;  // (device, n) -> roots

int get_twiddles(int n, const cplx** out) {
  int dev = 0;
  FISDF_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_tw_mu);
  auto key = std::make_pair(dev, n);
  auto it = g_tw.find(key);
  if (it == g_tw.end()) {
    std::vector<cplx> h(n);
    for (int t = 0; t < n; ++t) {
      // exp(-2 pi i t / n), exact for the quarter points
      long double ang = -2.0L * 3.14159265358979323846264338327950288L * t / n;
      h[t] = cmk((double)cosl(ang), (double)sinl(ang));
      if ((4 * t) % n == 0) {
        int q = (4 * t) / n;
        const double re[4] = {1, 0, -1, 0}, im[4] = {0, -1, 0, 1};
        h[t] = cmk(re[q], im[q]);
      }
    }
    TwTable tt;
    FISDF_HIP(hipMalloc(&tt.dev, sizeof(cplx) * n));
    FISDF_HIP(hipMemcpy(tt.dev, h.data(), sizeof(cplx) * n, hipMemcpyHostToDevice));
    it = g_tw.emplace(key, tt).first;
  }
  *out = it->second.dev;
  return 0;
}

int largest_divisor_le(int x, int cap) {
  for (int d = std::min(x, cap); d >= 1; --d)
    if (x % d == 0) return d;
  return 1;
}

int axis_pass(hipStream_t s, const cplx* in, long in_ld, const int* rowidx, cplx* out, long out_ld,
              int rows, int axis, int n0, int n1, int n2, const double* kd, const double* weight) {
  const int dims[3] = {n0, n1, n2};
  const int n = dims[axis];
  Stages st;
  FISDF_CHECK(n >= 1 && n <= MAXN, "fft: mesh dimension must be in [1, 64]");
  FISDF_CHECK(factorize(n, st), "fft: mesh dimension must factor into 2,3,5,7,11,13");
  const cplx* tw = nullptr;
  FISDF_TRY(get_twiddles(n, &tw));
  int inner = 1, outer = 1;
  for (int a = axis + 1; a < 3; ++a) inner *= dims[a];
  for (int a = 0; a < axis; ++a) outer *= dims[a];
  int contiguous = (axis == 2);
  int TL;
  long tiles;
  if (contiguous) {
    TL = std::max(1, std::min(64, 2048 / n));
    tiles = (long)rows * ((outer + TL - 1) / TL);
  } else {
    TL = largest_divisor_le(inner, 64);
    if (TL < 16 && inner > 64) TL = largest_divisor_le(inner, 128);  // keep tiles wide
    FISDF_CHECK(TL <= 128, "fft: tile too wide");
    tiles = (long)rows * outer * (inner / TL);
  }
  FISDF_CHECK(tiles < (1L << 31), "fft: too many tiles");
  size_t lds = sizeof(cplx) * (MAXN + 2 * (size_t)TL * n);
  FISDF_CHECK(lds <= 160 * 1024, "fft: LDS tile too large");
  double k0 = 0, k1 = 0, k2 = 0;
  int use_phase = kd != nullptr;
  if (kd) { k0 = kd[0]; k1 = kd[1]; k2 = kd[2]; }
  if (needs_big(st))
    hipLaunchKernelGGL(fft_axis_kernel<true>, dim3((unsigned)tiles), dim3(256), lds, s, in, in_ld,
                       rowidx, out, out_ld, rows, n, inner, outer, TL, contiguous, st, tw, n0, n1,
                       n2, k0, k1, k2, use_phase, weight);
  else
    hipLaunchKernelGGL(fft_axis_kernel<false>, dim3((unsigned)tiles), dim3(256), lds, s, in, in_ld,
                       rowidx, out, out_ld, rows, n, inner, outer, TL, contiguous, st, tw, n0, n1,
                       n2, k0, k1, k2, use_phase, weight);
  FISDF_HIP(hipGetLastError());
  return 0;
}

}  // namespace

// the register path's mesh test (square (i1, i2) planes of a listed size, listed n0)
bool reg_mesh(int n0, int n1, int n2) {
  if (n1 != n2) return false;
  int a = 0, b = 0;
#define FISDF_HAS(N) if (n1 == N) a = 1; if (n0 == N) b = 1;
  FISDF_REG_SIZES(FISDF_HAS)
#undef FISDF_HAS
  return a && b;
}

size_t plane_kernel_lds(int n1, int n2) { return sizeof(cplx) * (4 * MAXN + 2 * (size_t)n1 * n2); }

bool fft3d_reads_real(int n0, int n1, int n2) { return reg_mesh(n0, n1, n2); }

bool fft3d_reads_slices(int n0, int n1, int n2) {
  return reg_mesh(n0, n1, n2) || plane_kernel_lds(n1, n2) <= 96 * 1024;
}

// FISDF_FFT_HERM=0: the self-conjugate q's transform runs the full two passes (A/B)
bool fft_herm_enabled() {
  static const bool on = [] {
    const char* e = getenv("FISDF_FFT_HERM");
    return !(e && e[0] == '0');
  }();
  return on;
}

int fft3d(hipStream_t s, const cplx* in, long in_ld, const int* rowidx, cplx* out, long out_ld,
          int rows, int n0, int n1, int n2, const double* kd, const double* weight, cplx* /*work*/,
          const PlaneRef* planes, const int* herm, bool in_real) {
  if (rows == 0) return 0;
  FISDF_CHECK(!in_real || (reg_mesh(n0, n1, n2) && !planes && in != out),
              "fft: real input needs the register path and unsliced, out-of-place rows");
  FISDF_CHECK(in != out || rowidx == nullptr, "fft: in-place pass cannot gather rows");
  FISDF_CHECK(!planes || fft3d_reads_slices(n0, n1, n2), "fft: sliced input needs a plane kernel");
  if (reg_mesh(n0, n1, n2)) {  // register kernels: square (i1, i2) planes of a listed size, listed n0
    const cplx *W12 = nullptr, *W0 = nullptr;
    FISDF_TRY(get_twiddles(n1, &W12));
    FISDF_TRY(get_twiddles(n0, &W0));
    bool ok1 = false, ok0 = false;
    FISDF_CHECK((long)rows * n0 < (1L << 31) && (long)rows * n1 * n2 < (1L << 38), "fft: too large");
    if (herm && (herm[0] == 0 || herm[0] == 1) && fft_herm_enabled()) {
      // Hermitian-paired input: the plane pass stores the lines j1 < n1H, the axis-0 pass
      // completes their partners and writes the prefix planes only
      const int m[3] = {herm[0], ((herm[1] % n1) + n1) % n1, ((herm[2] % n2) + n2) % n2};
      const int n1H = herm_prefix(n1, m[1]);
      FISDF_TRY(fft_plane_reg_launch(s, n1, in, in_ld, rowidx, out, out_ld, rows, n0, W12, kd,
                                     planes, n1H, in_real, &ok1));
      FISDF_TRY(fft_axis0_herm_launch(s, n0, out, out_ld, out, out_ld, rows, n1, n2, n1H, m, W0,
                                      weight, &ok0));
      FISDF_CHECK(ok1 && ok0, "fft: register kernel dispatch failed");
      return 0;
    }
    {
      FISDF_TRY(fft_plane_reg_launch(s, n1, in, in_ld, rowidx, out, out_ld, rows, n0, W12, kd,
                                     planes, n1, in_real, &ok1));
      FISDF_TRY(fft_axis0_reg_launch(s, n0, out, out_ld, out, out_ld, rows, n1 * n2, W0, weight, &ok0));
      FISDF_CHECK(ok1 && ok0, "fft: register kernel dispatch failed");
      return 0;
    }
  }
  const size_t plane_lds = plane_kernel_lds(n1, n2);
  if (plane_lds <= 96 * 1024) {
    // axes 2+1 fused per (i1,i2) plane, then axis 0 with the Coulomb weight: 2 HBM passes
    Stages st1, st2;
    FISDF_CHECK(n1 <= MAXN && n2 <= MAXN && factorize(n1, st1) && factorize(n2, st2),
                "fft: mesh dimension must be <= 64 and factor into 2,3,5,7,11,13");
    const cplx *tw1 = nullptr, *tw2 = nullptr;
    FISDF_TRY(get_twiddles(n1, &tw1));
    FISDF_TRY(get_twiddles(n2, &tw2));
    const long nplanes = (long)rows * n0;
    FISDF_CHECK(nplanes < (1L << 31), "fft: too many planes");
    double k0 = 0, k1 = 0, k2 = 0;
    if (kd) { k0 = kd[0]; k1 = kd[1]; k2 = kd[2]; }
    if (needs_big(st1) || needs_big(st2))
      hipLaunchKernelGGL(fft_plane_kernel<true>, dim3((unsigned)nplanes), dim3(256), plane_lds, s,
                         in, in_ld, rowidx, out, out_ld, rows, st1, st2, tw1, tw2, n0, n1, n2, k0,
                         k1, k2, kd != nullptr ? 1 : 0, planes);
    else
      hipLaunchKernelGGL(fft_plane_kernel<false>, dim3((unsigned)nplanes), dim3(256), plane_lds, s,
                         in, in_ld, rowidx, out, out_ld, rows, st1, st2, tw1, tw2, n0, n1, n2, k0,
                         k1, k2, kd != nullptr ? 1 : 0, planes);
    FISDF_HIP(hipGetLastError());
  } else {
    FISDF_TRY(axis_pass(s, in, in_ld, rowidx, out, out_ld, rows, 2, n0, n1, n2, kd, nullptr));
    FISDF_TRY(axis_pass(s, out, out_ld, nullptr, out, out_ld, rows, 1, n0, n1, n2, nullptr, nullptr));
  }
  FISDF_TRY(axis_pass(s, out, out_ld, nullptr, out, out_ld, rows, 0, n0, n1, n2, nullptr, weight));
  return 0;
}

}  // namespace fisdf
