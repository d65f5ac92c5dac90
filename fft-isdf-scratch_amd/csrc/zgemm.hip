// Batched complex128 GEMM / HERK on CDNA4 FP64 matrix cores (v_mfma_f64_16x16x4_f64).
//
// Replaces every BLAS zgemm the reference issues through NumPy `@` on the hot path
// (fftisdf.py:38,41,46,76,79,84,121,205,211,215,222,225; einsums :155,159,166) and the
// HERK that W_q = zeta_q z_q^H (fftisdf.py:121) becomes after the Parseval rewrite.
//
// Tile: 64x64 complex per 256-thread workgroup (4 waves, each 32x32 = 2x2 MFMA blocks of
// 16x16).  K advances BK complex per step; the operand tiles go global -> LDS by LDS-DMA
// through an NS-deep ring (zgemm_glds_kernel below).  LDS holds interleaved complex (16 B), so
// each MFMA operand pair (re, im) is one ds_read_b128.  Layout per operand:
//   * M/N-contiguous operand: LDS [k][m] plain (64 complex rows = 256 dwords: the
//     ds_read_b128 lane groups hit disjoint banks);
//   * K-contiguous operand:   LDS [m][k ^ (m & 15)] (XOR swizzle on the 16-complex row).
// f64 MFMA fragment maps (cdna_hip_programming.md §3):
//   A: lane l holds A[i=l&15][k=l>>4];  B: B[k=l>>4][j=l&15];
//   C/D: 4 f64 per lane, col = l&15, row = (l>>4) + 4*r.
//
// HERK=true: C = alpha A A^H (OPA = N, OPB = C, B == A, M == N); only lower-triangle tiles
// (ti >= tj) are launched and the epilogue mirrors the conjugate into the upper triangle —
// half the MFMA work of the GEMM.
//
// XCD-aware tile order.  The grid is 1-D, padded to a multiple of 8: workgroup b runs on
// XCD b % 8 (the dispatcher's round-robin; used for speed only, never for correctness) and
// XCD x owns the contiguous chunk [x*per, (x+1)*per) of the tile order (z-slice major, then
// M-tile fastest).  The workgroups resident on one XCD at a time are therefore neighbours
// in that order: the M-tiles of one N-panel (GEMM), or all tiles of one K-split (HERK),
// which read the same operand panels — served by that XCD's own 4 MB L2 instead of
// each XCD re-fetching them from HBM / Infinity Cache.
#include "common.h"

namespace fisdf {

namespace {

constexpr int BM = 64, BN = 64, BK = 8;  // BK = 8: 16 KB per ring slot (BK = 16 measured slower)
constexpr int TILE = 64 * BK;   // complex elements per operand tile

// Operand staging. ROW_IS_K: the tile's "outer" index is the M (or N) index and k is
// contiguous in global memory (A op N/conj, B op T/conj-T).
template <bool KCONTIG>
struct Stage {
  // thread-element e -> (outer index x in [0,64), k in [0,BK)) chosen for coalesced loads
  __device__ static __forceinline__ void coord(int e, int& x, int& k) {
    if (KCONTIG) { x = e / BK; k = e % BK; }
    else { x = e % 64; k = e / 64; }
  }
  // LDS slot of (x, k)
  __device__ static __forceinline__ int slot(int x, int k) {
    if (KCONTIG) return x * BK + (k ^ (x & (BK - 1)));
    else return k * 64 + x;
  }
};

// Epilogue shared by both kernels: split-K partials, the fused y-square epilogue, or
// C = alpha acc + beta C; HERK blocks strictly below the diagonal are mirrored.
template <bool HERK>
__device__ __forceinline__ void zgemm_epilogue(int M, int N, cplx alpha, cplx beta,
                                               cplx* __restrict__ C, long ldc, long sC, int ksplit,
                                               int split, int bz, cplx* __restrict__ work, int epi,
                                               unsigned long long* __restrict__ mon, long ldaux,
                                               int m0, int n0,
                                               int wm, int wn, int lane, int mask,
                                               const f64x4 (&accR)[2][2], const f64x4 (&accI)[2][2]) {
  if (ksplit > 1) {
    cplx* Wp = work + ((long)bz * ksplit + split) * (long)M * N;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int row = m0 + wm + mi * 16 + (lane >> 4) + 4 * r;
          int col = n0 + wn + ni * 16 + (lane & 15);
          // HERK partials keep only the computed (lower) 16x16 blocks: herk_reduce_kernel
          // writes their conjugate mirrors once, after the sum
          if (((mask >> (mi * 2 + ni)) & 1) && row < M && col < N)
            Wp[(long)row * N + col] = cmk(accR[mi][ni][r], accI[mi][ni][r]);
        }
    return;
  }
  C += (long)bz * sC;
  if (epi == EPI_STREAM) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int row = m0 + wm + mi * 16 + (lane >> 4) + 4 * r;
          int col = n0 + wn + ni * 16 + (lane & 15);
          if (((mask >> (mi * 2 + ni)) & 1) && row < M && col < N) {
            const cplx v = cmul(alpha, cmk(accR[mi][ni][r], accI[mi][ni][r]));
            double* cp = (double*)(C + (long)row * ldc + col);
            __builtin_nontemporal_store(v.x, cp);
            __builtin_nontemporal_store(v.y, cp + 1);
          }
        }
    return;
  }
  if (epi == EPI_REAL || epi == EPI_WSRHO) {
    // EPI_REAL: C (REAL: double*, row stride ldc doubles; batch 1) = Re(alpha acc);
    // EPI_WSRHO: C = aux[row][col] Re(alpha acc) + 0i with aux real (double*, row stride
    // ldaux doubles, passed as work); both record max |Im(alpha acc)| in *mon
    double* Cd = (double*)(C - (long)bz * sC);
    const double* auxd = (const double*)work;
    double mx = 0.0;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int row = m0 + wm + mi * 16 + (lane >> 4) + 4 * r;
          int col = n0 + wn + ni * 16 + (lane & 15);
          if (((mask >> (mi * 2 + ni)) & 1) && row < M && col < N) {
            const cplx v = cmul(alpha, cmk(accR[mi][ni][r], accI[mi][ni][r]));
            mx = fmax(mx, fabs(v.y));
            if (epi == EPI_WSRHO)
              C[(long)row * ldc + col] = cmk(auxd[(long)row * ldaux + col] * v.x, 0.0);
            else
              Cd[(long)row * ldc + col] = v.x;
          }
        }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
    if (lane == 0 && mon) atomicMax(mon, (unsigned long long)__double_as_longlong(mx));
    return;
  }
  if (epi == EPI_CSQUARE) {  // C = (alpha acc)^2 elementwise; max |Im(alpha acc)| -> *mon
    double mx = 0.0;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int row = m0 + wm + mi * 16 + (lane >> 4) + 4 * r;
          int col = n0 + wn + ni * 16 + (lane & 15);
          if (((mask >> (mi * 2 + ni)) & 1) && row < M && col < N) {
            const cplx v = cmul(alpha, cmk(accR[mi][ni][r], accI[mi][ni][r]));
            mx = fmax(mx, fabs(v.y));
            C[(long)row * ldc + col] = cmul(v, v);
          }
        }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
    if (lane == 0 && mon) atomicMax(mon, (unsigned long long)__double_as_longlong(mx));
    return;
  }
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int row = m0 + wm + mi * 16 + (lane >> 4) + 4 * r;
        int col = n0 + wn + ni * 16 + (lane & 15);
        const bool mirror = HERK && (m0 + wm + mi * 16 > n0 + wn + ni * 16);
        if (((mask >> (mi * 2 + ni)) & 1) && row < M && col < N) {
          cplx v = cmul(alpha, cmk(accR[mi][ni][r], accI[mi][ni][r]));
          cplx* cp = C + (long)row * ldc + col;
          if (beta.x != 0.0 || beta.y != 0.0) v = cadd(v, cmul(beta, *cp));
          *cp = v;
          if (mirror) C[(long)col * ldc + row] = cconj(v);
        }
      }
}

// ---- the GEMM kernel -------------------------------------------------------------------
// The operand tiles go global -> LDS directly (global_load_lds_dwordx4, no staging registers) through a THREE-deep
// LDS ring: the loads of K-step s+2 are issued at step s, so each has two full steps to land
// (the register-staged kernel waited on its loads one step after issue: at 3 workgroups/CU
// its per-step time was set by L2/HBM latency, not by the MFMA pipe).  The LDS image is
// lane-linear per wave-instruction (dest = base + lane*16); the K-contiguous operands keep
// their XOR swizzle by permuting the per-lane SOURCE address instead.  Out-of-range lanes
// read a zero page; conjugation is folded into the MFMA operand signs.
#ifndef FISDF_GEMM_3M
#define FISDF_GEMM_3M 1  // 3 real MFMAs per complex block in FULL mode (0: the 4-product form)
#endif
#ifndef FISDF_NST
#define FISDF_NST 3
#endif
constexpr int NST = FISDF_NST;  // LDS ring depth; loads run NST-1 K-steps ahead
constexpr int LPW = TILE / (64 * 4);  // glds wave-instructions per operand per step per wave
__device__ cplx g_zero_page[64];      // zero-initialised device global

template <int OPA, int OPB, bool HERK, int MODE, int NS, bool PIPE = false>
__global__ __launch_bounds__(256) void zgemm_glds_kernel(int M, int N, int K, cplx alpha,
                                                         const cplx* __restrict__ A, long lda, long sA,
                                                         const cplx* __restrict__ B, long ldb, long sB,
                                                         cplx beta, cplx* __restrict__ C, long ldc, long sC,
                                                         int ksplit, int kchunk, cplx* __restrict__ work,
                                                         int epi, unsigned long long* __restrict__ mon, long ldaux,
                                                         int nMt, int ntile, int ntot,
                                                         unsigned long long* __restrict__ span) {
  constexpr bool AK = !(OPA & 1);  // A stored [m][k]
  constexpr bool BKc = (OPB & 1);  // B stored [n][k]
  constexpr bool CA = (OPA & 2) != 0, CB = (OPB & 2) != 0;
  typedef Stage<AK> SA;
  typedef Stage<BKc> SB;
  // [stage][A|B][TILE], one object (48 KB at BK = 8, NS = 3; NS = 2 for short K loops)
  __shared__ cplx sm[NS * 2 * TILE];

  const int per = (int)(gridDim.x >> 3);
  const int order = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (order >= ntot) return;
  span_begin(span);
  const int zz = order / ntile, t = order - zz * ntile;
  const int split = zz % ksplit;
  const int bz = zz / ksplit;
  A += (long)bz * sA;
  B += (long)bz * sB;
  int ti = t % nMt, tj = t / nMt;
  // GEMM_A_LOWER: M-tile i runs K = 64 (i + 1); the longest tiles of each N-panel go first so
  // the short ones fill the end of the launch (longest-processing-time order)
  if constexpr ((MODE & GEMM_A_LOWER) != 0) ti = nMt - 1 - ti;
  if (HERK) {
    ti = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
    while (ti * (ti + 1) / 2 > t) --ti;
    tj = t - ti * (ti + 1) / 2;
  }
  const int m0 = ti * BM, n0 = tj * BN;
  int kbeg = split * kchunk;
  int kend = min(K, kbeg + kchunk);
  if constexpr ((MODE & GEMM_A_LOWER) != 0) kend = min(kend, m0 + BM);  // A[m][k] = 0 for k > m
  if constexpr ((MODE & GEMM_A_UPPER) != 0) kbeg = max(kbeg, m0);        // A[m][k] = 0 for k < m

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // wave -> sub-tile: the role rotates with the tile so idle roles spread over the SIMDs.
  // Default 2x2 quadrants of 32x32; tiles whose valid 16x16 blocks would leave waves idle get
  // another split so the 4 waves share the valid blocks: an edge row of tiles with <= 32
  // valid rows splits by 16-column blocks (and an edge column by 16-row blocks), a full HERK
  // diagonal tile gives its 10 lower blocks out as 3 + 3 + 2 + 2.  `own` = the blocks of the
  // wave's nominal 2x2 (bit mi*2+ni) it is responsible for.
  const int role = (w + ti + tj) & 3;
  const int vr = min(4, max(0, (M - m0 + 15) / 16)), vc = min(4, max(0, (N - n0 + 15) / 16));
  int wm, wn, own;
  if (HERK && ti == tj && vr == 4) {
    wm = role == 0 ? 0 : (role == 1 ? 32 : (role == 2 ? 32 : 48));
    wn = role == 1 ? 32 : 0;
    own = role < 2 ? 15 : 3;
  } else if (vr <= 2 && vc > 2) {
    wm = 0; wn = 16 * role; own = 5;
  } else if (vc <= 2 && vr > 2) {
    wm = 16 * role; wn = 0; own = 3;
  } else {
    wm = (role >> 1) * 32; wn = (role & 1) * 32; own = 15;
  }

  // per-lane source of each glds: slot s = (w*LPW + j)*64 + lane of the operand tile
  const cplx* srcA[LPW];
  const cplx* srcB[LPW];
  int kA[LPW], kB[LPW];
  bool rowA[LPW], rowB[LPW];
  long stepA, stepB;  // element advance of the source per K-step
#pragma unroll
  for (int j = 0; j < LPW; ++j) {
    const int sl = (w * LPW + j) * 64 + lane;
    int x, k;
    if (AK) { x = sl / BK; k = (sl % BK) ^ (x & (BK - 1)); }
    else { x = sl % 64; k = sl / 64; }
    rowA[j] = m0 + x < M;
    kA[j] = k;
    srcA[j] = A + (AK ? (long)(m0 + x) * lda + (kbeg + k) : (long)(kbeg + k) * lda + (m0 + x));
    if (BKc) { x = sl / BK; k = (sl % BK) ^ (x & (BK - 1)); }
    else { x = sl % 64; k = sl / 64; }
    rowB[j] = n0 + x < N;
    kB[j] = k;
    srcB[j] = B + (BKc ? (long)(n0 + x) * ldb + (kbeg + k) : (long)(kbeg + k) * ldb + (n0 + x));
  }
  stepA = AK ? (long)BK : (long)BK * lda;
  stepB = BKc ? (long)BK : (long)BK * ldb;

  // The LDS-DMA is issued from inline asm so that hipcc's waitcnt pass does not see it (it
  // would drain vmcnt(0) before the next ds_read); its completion is counted by hand below.
  const cplx* zp = g_zero_page;
  const unsigned lds0 = (unsigned)(uintptr_t)sm;
  auto glds = [&](const cplx* src, unsigned lds_byte) {
    unsigned keep;
    const unsigned dst = __builtin_amdgcn_readfirstlane(lds_byte);
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
  };
  auto issue = [&](int st) {  // K-step st -> ring slot st % NS
    const int buf = st % NS;
    const int k0 = kbeg + st * BK;
    const unsigned la = lds0 + (unsigned)((buf * 2 + 0) * TILE) * 16u;
    const unsigned lb = lds0 + (unsigned)((buf * 2 + 1) * TILE) * 16u;
#pragma unroll
    for (int j = 0; j < LPW; ++j) {
      const cplx* pa = (rowA[j] && k0 + kA[j] < kend) ? srcA[j] + st * stepA : zp;
      glds(pa, la + (unsigned)((w * LPW + j) * 64) * 16u);
      const cplx* pb = (rowB[j] && k0 + kB[j] < kend) ? srcB[j] + st * stepB : zp;
      glds(pb, lb + (unsigned)((w * LPW + j) * 64) * 16u);
    }
  };

  // FULL mode, 3 real products per complex block (FISDF_GEMM_3M): accR = P1 = ar br,
  // accI = P2 = ai' bi', acc3 = P3 = (ar + ai')(br + bi'); Re = P1 - P2, Im = P3 - P1 - P2
  // after the K loop (tests/experiments/three_mult.py: J/K unchanged to the last digit shown)
  constexpr bool M3 = FISDF_GEMM_3M && (MODE & (GEMM_A_REAL | GEMM_RE_ONLY)) == 0;
  f64x4 accR[2][2], accI[2][2], acc3[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      accR[i][j] = f64x4{0, 0, 0, 0};
      accI[i][j] = f64x4{0, 0, 0, 0};
      acc3[i][j] = f64x4{0, 0, 0, 0};
    }

  int mask = 0;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int r0 = m0 + wm + mi * 16, c0 = n0 + wn + ni * 16;
      const bool live = ((own >> (mi * 2 + ni)) & 1) && r0 < M && c0 < N && !(HERK && c0 > r0);
      mask |= (live ? 1 : 0) << (mi * 2 + ni);
    }

  const int nsteps = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  const int i16 = lane & 15, kq = lane >> 4;
  if constexpr (PIPE && M3) {
    // Software-pipelined 3-multiplication loop (host-checked: K and the K-chunk multiples of BK,
    // operand extents < 4 GB).  The next K-substep's LDS fragments are read while the current
    // substep's P3 = (ar + ai')(br + bi') group runs (P1 and P2 are the last uses of the raw
    // fragments, so the reads reuse their registers); the next K-step's barrier sits between
    // the last substep's P1/P2 and P3 groups.  Rows / columns outside the matrix read a clamped
    // in-range row / column (they only feed C entries that are never stored), so every lane
    // advances by one uniform stride: per-lane 32-bit byte offsets from a wave-uniform base
    // (the SADDR form of the LDS-DMA load).  No loads past the last K-step.
    (void)rowA;
    (void)rowB;
    unsigned oA[LPW], oB[LPW];
#pragma unroll
    for (int j = 0; j < LPW; ++j) {
      const int sl = (w * LPW + j) * 64 + lane;
      int x, k;
      if (AK) { x = sl / BK; k = (sl % BK) ^ (x & (BK - 1)); }
      else { x = sl % 64; k = sl / 64; }
      const long xa = min(m0 + x, M - 1);
      oA[j] = (unsigned)((AK ? xa * lda + k : (long)k * lda + xa) * 16);
      if (BKc) { x = sl / BK; k = (sl % BK) ^ (x & (BK - 1)); }
      else { x = sl % 64; k = sl / 64; }
      const long xb = min(n0 + x, N - 1);
      oB[j] = (unsigned)((BKc ? xb * ldb + k : (long)k * ldb + xb) * 16);
    }
    const cplx* baseA = A + (AK ? (long)kbeg : (long)kbeg * lda);
    const cplx* baseB = B + (BKc ? (long)kbeg : (long)kbeg * ldb);
    const int wu = __builtin_amdgcn_readfirstlane(w);
    auto gldss = [&](const cplx* base, unsigned off, unsigned lds_byte) {
      unsigned keep;
      const unsigned dst = __builtin_amdgcn_readfirstlane(lds_byte);
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(off), "s"(base), "s"(dst) : "memory");
    };
    auto issue_p = [&](int st) {
      const int buf = st % NS;
      const unsigned la = lds0 + (unsigned)((buf * 2 + 0) * TILE) * 16u;
      const unsigned lb = lds0 + (unsigned)((buf * 2 + 1) * TILE) * 16u;
      const cplx* ba = baseA + st * stepA;
      const cplx* bb = baseB + st * stepB;
#pragma unroll
      for (int j = 0; j < LPW; ++j) {
        gldss(ba, oA[j], la + (unsigned)((wu * LPW + j) * 64) * 16u);
        gldss(bb, oB[j], lb + (unsigned)((wu * LPW + j) * 64) * 16u);
      }
    };
    auto pipeloop = [&](auto maskc) {
      constexpr int MASK = decltype(maskc)::value;
      if (nsteps == 0) return;
#pragma unroll
      for (int st = 0; st < NS - 1; ++st)
        if (st < nsteps) issue_p(st);
      if (nsteps > 1)
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * LPW * (NS - 2)) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      cplx fa[2], fb[2];
      auto rd = [&](int slot, int kk) {
        const cplx* as = sm + (long)(slot * 2 + 0) * TILE;
        const cplx* bs = sm + (long)(slot * 2 + 1) * TILE;
        const int k = kk + kq;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          fa[u] = as[SA::slot((wm + u * 16 + i16) & 63, k)];
          fb[u] = bs[SB::slot((wn + u * 16 + i16) & 63, k)];
        }
      };
      rd(0, 0);
      if (NS - 1 < nsteps) issue_p(NS - 1);
      double sa[2], sb[2];
      auto p12 = [&]() {
        double ar[2], ai[2], br[2], bi[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          ar[u] = fa[u].x;
          ai[u] = CA ? -fa[u].y : fa[u].y;
          br[u] = fb[u].x;
          bi[u] = CB ? -fb[u].y : fb[u].y;
          sa[u] = ar[u] + ai[u];
          sb[u] = br[u] + bi[u];
        }
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            if ((MASK >> (mi * 2 + ni)) & 1)
              accR[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[mi], br[ni], accR[mi][ni], 0, 0, 0);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            if ((MASK >> (mi * 2 + ni)) & 1)
              accI[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai[mi], bi[ni], accI[mi][ni], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      };
      auto p3 = [&]() {
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            if ((MASK >> (mi * 2 + ni)) & 1)
              acc3[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(sa[mi], sb[ni], acc3[mi][ni], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      };
      for (int s = 0; s < nsteps; ++s) {
        const int cur = s % NS;
        p12();
        rd(cur, 4);
        __builtin_amdgcn_sched_barrier(0);
        p3();
        p12();
        if (s + 1 < nsteps) {
          if (s + 2 < nsteps)
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * LPW * (NS - 2)) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          rd((s + 1) % NS, 0);
          if (s + NS < nsteps) issue_p(s + NS);
          __builtin_amdgcn_sched_barrier(0);
        }
        p3();
      }
    };
    switch (mask) {
      case 13: pipeloop(std::integral_constant<int, 13>{}); break;
      case 5: pipeloop(std::integral_constant<int, 5>{}); break;
      case 3: pipeloop(std::integral_constant<int, 3>{}); break;
      case 1: pipeloop(std::integral_constant<int, 1>{}); break;
      case 0: pipeloop(std::integral_constant<int, 0>{}); break;
      default: pipeloop(std::integral_constant<int, 15>{}); break;
    }
  } else {
  // (steps past the end load the zero page: the counted waits assume NST-1 steps in flight)
  if (nsteps > 0) {
#pragma unroll
    for (int st = 0; st < NS - 1; ++st) issue(st);
  }
  auto mainloop = [&](auto maskc) {
    constexpr int MASK = decltype(maskc)::value;
    for (int s = 0; s < nsteps; ++s) {
      // own loads of step s retired (step s+1's 2*LPW stay in flight), then every wave's:
      // the barrier also retires all reads of the slot step s+2 is about to overwrite
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * LPW * (NS - 2)) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      const int cur = s % NS;
      const cplx* as = sm + (long)(cur * 2 + 0) * TILE;
      const cplx* bs = sm + (long)(cur * 2 + 1) * TILE;
      const int kleft = kend - kbeg - s * BK;  // K-substeps past the end hold only zeros
      issue(s + NS - 1);
#pragma unroll
      for (int kk = 0; kk < BK; kk += 4) {
        if (kk > 0 && kk >= kleft) break;
        cplx a[2], b[2];
        const int k = kk + kq;
#pragma unroll
        for (int u = 0; u < 2; ++u) {  // & 63: a masked block past the tile reads in-tile rows
          a[u] = as[SA::slot((wm + u * 16 + i16) & 63, k)];
          b[u] = bs[SB::slot((wn + u * 16 + i16) & 63, k)];
        }
        // op(A) = a (or conj a), op(B) = b (or conj b):
        //   Re += ar br - ai' bi' ;  Im += ar bi' + ai' br   (ai' = +-ai, bi' = +-bi)
        double ar[2], ai[2], nai[2], br[2], bi[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          ar[u] = a[u].x;
          ai[u] = CA ? -a[u].y : a[u].y;
          nai[u] = -ai[u];
          br[u] = b[u].x;
          bi[u] = CB ? -b[u].y : b[u].y;
        }
        constexpr bool AREAL = (MODE & GEMM_A_REAL) != 0, REONLY = (MODE & GEMM_RE_ONLY) != 0;
        if constexpr (M3) {
          double as[2], bs[2];
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            as[u] = ar[u] + ai[u];
            bs[u] = br[u] + bi[u];
          }
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              if (((MASK >> (mi * 2 + ni)) & 1) )
                accR[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[mi], br[ni], accR[mi][ni], 0, 0, 0);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              if (((MASK >> (mi * 2 + ni)) & 1) )
                accI[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai[mi], bi[ni], accI[mi][ni], 0, 0, 0);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              if (((MASK >> (mi * 2 + ni)) & 1) )
                acc3[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(as[mi], bs[ni], acc3[mi][ni], 0, 0, 0);
          continue;
        }
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            if (((MASK >> (mi * 2 + ni)) & 1) )
              accR[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[mi], br[ni], accR[mi][ni], 0, 0, 0);
        if constexpr (!REONLY) {
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              if (((MASK >> (mi * 2 + ni)) & 1) )
                accI[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[mi], bi[ni], accI[mi][ni], 0, 0, 0);
        }
        if constexpr (!AREAL) {
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              if (((MASK >> (mi * 2 + ni)) & 1) )
                accR[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(nai[mi], bi[ni], accR[mi][ni], 0, 0, 0);
        }
        if constexpr (!AREAL && !REONLY) {
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              if (((MASK >> (mi * 2 + ni)) & 1) )
                accI[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai[mi], br[ni], accI[mi][ni], 0, 0, 0);
        }
      }
    }
  };
  switch (mask) {
    case 13: mainloop(std::integral_constant<int, 13>{}); break;
    case 5: mainloop(std::integral_constant<int, 5>{}); break;
    case 3: mainloop(std::integral_constant<int, 3>{}); break;
    case 1: mainloop(std::integral_constant<int, 1>{}); break;
    case 0: mainloop(std::integral_constant<int, 0>{}); break;
    default: mainloop(std::integral_constant<int, 15>{}); break;
  }
  }
  // drain the (zero-page / unused) loads still in flight before the workgroup exits
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (M3) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double p1 = accR[mi][ni][r], p2 = accI[mi][ni][r], p3 = acc3[mi][ni][r];
          accR[mi][ni][r] = p1 - p2;
          accI[mi][ni][r] = p3 - p1 - p2;
        }
  }

  zgemm_epilogue<HERK>(M, N, alpha, beta, C, ldc, sC, ksplit, split, bz, work, epi, mon, ldaux, m0, n0, wm,
                       wn, lane, mask, accR, accI);
  span_end(span);
}

// C = alpha * sum_s work[s] + beta * C  (deterministic split-K reduction)
__global__ void ksplit_reduce(int M, int N, int ksplit, const cplx* __restrict__ work, cplx alpha,
                              cplx beta, cplx* __restrict__ C, long ldc, long sC,
                              unsigned long long* __restrict__ span) {
  span_begin(span);
  const int bz = blockIdx.y;
  const long MN = (long)M * N;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < MN; e += (long)gridDim.x * blockDim.x) {
    cplx acc = cmk(0, 0);
    for (int s = 0; s < ksplit; ++s) acc = cadd(acc, work[((long)bz * ksplit + s) * MN + e]);
    int row = (int)(e / N), col = (int)(e % N);
    cplx* cp = C + (long)bz * sC + (long)row * ldc + col;
    cplx v = cmul(alpha, acc);
    if (beta.x != 0.0 || beta.y != 0.0) v = cadd(v, cmul(beta, *cp));
    *cp = v;
  }
  span_end(span);
}

// HERK split-K reduction: C = alpha sum_s work[s] over the lower 16x16 blocks the HERK kernel
// computed (the partials hold nothing else), and C[c][r] = conj(C[r][c]) for the strictly-lower
// blocks — one 32x32 tile of the lower triangle per workgroup, the mirror through LDS so both
// the partial reads and the C writes stay coalesced
__global__ __launch_bounds__(256) void herk_reduce_kernel(int n, int ksplit,
                                                          const cplx* __restrict__ work, double alpha,
                                                          cplx* __restrict__ C, long ldc,
                                                          unsigned long long* __restrict__ span) {
  // one 16 x 16 lower block per workgroup (the partials hold exactly those: the HERK computes the
  // lower 16 x 16 blocks), one element per thread, 8 partials in flight per thread; every
  // element sums its partials in ascending s.  (32 x 32 tiles with one load in flight per thread
  // gave ~190 workgroups at 0.7 TB/s: latency-bound.)
  span_begin(span);
  __shared__ cplx tile[16][17];
  int t = blockIdx.x, ti = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
  while (ti * (ti + 1) / 2 > t) --ti;
  const int tj = t - ti * (ti + 1) / 2;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const long nn = (long)n * n;
  const int r = ti * 16 + ty, c = tj * 16 + tx;
  const bool valid = r < n && c < n;
  const cplx* w = work + (valid ? (long)r * n + c : 0);
  cplx acc = cmk(0, 0);
  for (int s0 = 0; s0 < ksplit; s0 += 8) {
    cplx v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = (s0 + u < ksplit && valid) ? w[(long)(s0 + u) * nn] : cmk(0, 0);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (s0 + u < ksplit) acc = cadd(acc, v[u]);
  }
  cplx a = cmk(0, 0);
  if (valid) {
    a = cscale(acc, alpha);
    C[(long)r * ldc + c] = a;
  }
  tile[ty][tx] = a;
  __syncthreads();
  if (ti > tj) {  // C[tj*16 + ty][ti*16 + tx] = conj(C[ti*16 + tx][tj*16 + ty])
    const int sr = tj * 16 + ty, sc = ti * 16 + tx;
    if (sr < n && sc < n) C[(long)sr * ldc + sc] = cconj(tile[tx][ty]);
  }
  span_end(span);
}

// the kernel-exact timing events of the current zgemm()/herk() call (taken from launch_events()
// at its entry): the main kernel records `start`, the call's last kernel `stop`
struct CallEvents {
  unsigned long long* span = nullptr;
  CallEvents() {
    LaunchEvents& le = launch_events();
    span = le.span;
    le = LaunchEvents();
  }
};

// FISDF_GEMM_PIPE=0: the unpipelined main loop for every launch (A/B on one box)
bool pipe_enabled() {
  static const bool on = [] {
    const char* e = getenv("FISDF_GEMM_PIPE");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <int OPA, int OPB, bool HERK = false, int MODE = GEMM_FULL>
void launch(hipStream_t s, dim3 grid, int M, int N, int K, cplx alpha, const cplx* A, long lda,
            long sA, const cplx* B, long ldb, long sB, cplx beta, cplx* C, long ldc, long sC,
            int ksplit, int kchunk, cplx* work, int epi, unsigned long long* mon, long ldaux,
            unsigned long long* span = nullptr) {
  // grid = (N-tiles or triangle tiles, M-tiles, z-slices) -> padded 1-D XCD-aware order
  const int nMt = HERK ? 1 : (int)grid.y;
  const int ntile = (int)(grid.x * (HERK ? 1 : grid.y));
  const long ntot = (long)ntile * grid.z;
  const long per = (ntot + 7) / 8;
  const dim3 g((unsigned)(8 * per));
  // short K loops (<= 4 steps per workgroup, e.g. the y build's K = nao): a 2-deep ring
  // (32 KB of LDS) lets more workgroups share a CU, overlapping their load and store phases
  // the software-pipelined 3-multiplication loop: every workgroup's K range a whole number of
  // K-steps, per-lane operand offsets within 32 bits
  constexpr bool M3 = FISDF_GEMM_3M && (MODE & (GEMM_A_REAL | GEMM_RE_ONLY)) == 0;
  auto fits32 = [](long rows, long ld) { return rows * ld * 16 < (1L << 32); };
  const bool pipe = M3 && pipe_enabled() && K % BK == 0 && kchunk % BK == 0 &&
                    fits32(!(OPA & 1) ? M : K, lda) && fits32((OPB & 1) ? N : K, ldb);
  if (kchunk <= 4 * BK)
    hipLaunchKernelGGL((zgemm_glds_kernel<OPA, OPB, HERK, MODE, 2>), g, dim3(256), 0, s, M, N, K,
                       alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, ksplit, kchunk, work, epi,
                       mon, ldaux, nMt, ntile, (int)ntot, span);
  else if (pipe)
    hipLaunchKernelGGL((zgemm_glds_kernel<OPA, OPB, HERK, MODE, NST, M3>), g, dim3(256), 0, s, M, N,
                       K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, ksplit, kchunk, work, epi,
                       mon, ldaux, nMt, ntile, (int)ntot, span);
  else
    hipLaunchKernelGGL((zgemm_glds_kernel<OPA, OPB, HERK, MODE, NST>), g, dim3(256), 0, s, M, N, K,
                       alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, ksplit, kchunk, work, epi,
                       mon, ldaux, nMt, ntile, (int)ntot, span);
}

}  // namespace

int zgemm(hipStream_t s, int opA, int opB, int M, int N, int K, cplx alpha, const cplx* A,
          long lda, long sA, const cplx* B, long ldb, long sB, cplx beta, cplx* C, long ldc,
          long sC, int batch, int ksplit, cplx* work, int epi, unsigned long long* mon, int mode,
          long ldaux) {
  FISDF_CHECK(M >= 0 && N >= 0 && K >= 0 && batch >= 0, "zgemm: negative size");
  FISDF_CHECK(opA >= 0 && opA < 4 && opB >= 0 && opB < 4, "zgemm: bad op");
  FISDF_CHECK(mode >= 0 && mode <= 8, "zgemm: bad mode");
  FISDF_CHECK(mode == GEMM_FULL || mode == GEMM_A_UPPER ||
                  (opB == OP_N && (opA == OP_N || opA == OP_C)),
              "zgemm: real modes are implemented for (N,N) and (C,N) only");
  // GEMM_A_UPPER with split-K: a split whose K range lies wholly left of an M-tile's first row
  // runs no K-step and writes a zero partial (the reduce sums every split)
  FISDF_CHECK(mode != GEMM_A_UPPER || opA == OP_C,
              "zgemm: GEMM_A_UPPER is implemented for op(A) = A^H");
  FISDF_CHECK(!(mode & GEMM_A_LOWER) || (opA == OP_N && opB == OP_N && !(mode & GEMM_RE_ONLY)),
              "zgemm: GEMM_A_LOWER is implemented for (N,N), optionally with GEMM_A_REAL");
  if (M == 0 || N == 0 || batch == 0) return 0;
  if (ksplit < 1) ksplit = 1;
  if (epi != EPI_NONE) ksplit = 1;
  if (zgemm_wide_applies(opA, opB, M, N, K, lda, ldb, batch, ksplit, epi, mode)) {
    const CallEvents ev;
    return zgemm_nn_wide(s, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, mode, ev.span);
  }
  if (ksplit > 1) FISDF_CHECK(work != nullptr, "zgemm: split-K needs a workspace");
  int kchunk = (K + ksplit - 1) / ksplit;
  kchunk = ((kchunk + BK - 1) / BK) * BK;
  if (kchunk == 0) kchunk = BK;
  ksplit = std::max(1, (K + kchunk - 1) / kchunk);
  FISDF_CHECK((long)((N + BN - 1) / BN) * ((M + BM - 1) / BM) * batch * ksplit < (1L << 31),
              "zgemm: too many tiles");
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, batch * ksplit);
  const CallEvents ev;
#define FISDF_CASE(a, b)                                                                      \
  case a * 4 + b:                                                                             \
    launch<a, b>(s, grid, M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, ksplit,   \
                 kchunk, work, epi, mon, ldaux, ev.span);                           \
    break;
#define FISDF_MCASE(a, b, m)                                                                  \
  if (opA == a && opB == b && mode == m) {                                                    \
    launch<a, b, false, m>(s, grid, M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, \
                           ksplit, kchunk, work, epi, mon, ldaux, ev.span);         \
  }
  FISDF_MCASE(0, 0, 1) FISDF_MCASE(0, 0, 2) FISDF_MCASE(0, 0, 3)
  FISDF_MCASE(0, 0, 4) FISDF_MCASE(0, 0, 5)
  FISDF_MCASE(3, 0, 1) FISDF_MCASE(3, 0, 2) FISDF_MCASE(3, 0, 3)
  FISDF_MCASE(3, 0, 8) FISDF_MCASE(3, 3, 8)
#undef FISDF_MCASE
  if (mode == GEMM_FULL) switch (opA * 4 + opB) {
    FISDF_CASE(0, 0) FISDF_CASE(0, 1) FISDF_CASE(0, 2) FISDF_CASE(0, 3)
    FISDF_CASE(1, 0) FISDF_CASE(1, 1) FISDF_CASE(1, 2) FISDF_CASE(1, 3)
    FISDF_CASE(2, 0) FISDF_CASE(2, 1) FISDF_CASE(2, 2) FISDF_CASE(2, 3)
    FISDF_CASE(3, 0) FISDF_CASE(3, 1) FISDF_CASE(3, 2) FISDF_CASE(3, 3)
  }
#undef FISDF_CASE
  FISDF_HIP(hipGetLastError());
  if (ksplit > 1) {
    long MN = (long)M * N;
    int blocks = (int)std::min<long>((MN + 255) / 256, 4096);
    hipLaunchKernelGGL(ksplit_reduce, dim3(blocks, batch), dim3(256), 0, s, M, N, ksplit,
                       (const cplx*)work, alpha, beta, C, ldc, sC, ev.span);
    FISDF_HIP(hipGetLastError());
  }
  return 0;
}

// C = alpha A A^H, A: n x K (row-major, lda), C: n x n (ldc) Hermitian, lower tiles + mirror.
int herk(hipStream_t s, int n, int K, double alpha, const cplx* A, long lda, cplx* C, long ldc,
         int ksplit, cplx* work, int mode) {
  FISDF_CHECK(mode == GEMM_FULL || mode == GEMM_RE_ONLY, "herk: mode must be FULL or RE_ONLY");
  FISDF_CHECK(n >= 0 && K >= 0, "herk: negative size");
  if (n == 0) return 0;
  if (ksplit < 1) ksplit = 1;
  if (ksplit > 1) FISDF_CHECK(work != nullptr, "herk: split-K needs a workspace");
  int kchunk = (K + ksplit - 1) / ksplit;
  kchunk = std::max(BK, ((kchunk + BK - 1) / BK) * BK);
  ksplit = std::max(1, (K + kchunk - 1) / kchunk);
  const int nt = (n + BM - 1) / BM;
  dim3 grid(nt * (nt + 1) / 2, 1, ksplit);
  const CallEvents ev;
  if (mode == GEMM_RE_ONLY)  // C = Re(A A^H): 2 of the 4 MFMAs per complex block
    launch<OP_N, OP_C, true, GEMM_RE_ONLY>(s, grid, n, n, K, cmk(alpha, 0), A, lda, 0, A, lda, 0,
                                           cmk(0, 0), C, ldc, 0, ksplit, kchunk, work, EPI_NONE,
                                           nullptr, 0, ev.span);
  else
    launch<OP_N, OP_C, true>(s, grid, n, n, K, cmk(alpha, 0), A, lda, 0, A, lda, 0, cmk(0, 0), C,
                             ldc, 0, ksplit, kchunk, work, EPI_NONE, nullptr, 0, ev.span);
  FISDF_HIP(hipGetLastError());
#ifdef FISDF_EXP_NOREDUCE  // timing experiment only (wrong results): no split-K reduction
  ksplit = 1;
#endif
  if (ksplit > 1) {
    const int t16 = (n + 15) / 16;
    hipLaunchKernelGGL(herk_reduce_kernel, dim3(t16 * (t16 + 1) / 2), dim3(256), 0, s, n, ksplit,
                       (const cplx*)work, alpha, C, ldc, ev.span);
    FISDF_HIP(hipGetLastError());
  }
  return 0;
}

// C[b] = alpha A[b] A[b]^H + beta C[b] for a batch (A: n x K, lda, batch stride sA; C: n x n,
// ldc, stride sC): lower tiles computed, upper mirrored — the blocked Cholesky's trailing
// update (beta = 1, alpha = -1) at half the tiles of the full GEMM
int herk_batched(hipStream_t s, int n, int K, double alpha, const cplx* A, long lda, long sA,
                 double beta, cplx* C, long ldc, long sC, int batch) {
  FISDF_CHECK(n >= 0 && K >= 0 && batch >= 0, "herk_batched: negative size");
  if (n == 0 || batch == 0) return 0;
  const int kchunk = std::max(BK, ((K + BK - 1) / BK) * BK);
  const int nt = (n + BM - 1) / BM;
  dim3 grid(nt * (nt + 1) / 2, 1, batch);
  launch<OP_N, OP_C, true>(s, grid, n, n, K, cmk(alpha, 0), A, lda, sA, A, lda, sA, cmk(beta, 0), C,
                           ldc, sC, 1, kchunk, nullptr, EPI_NONE, nullptr, 0);
  FISDF_HIP(hipGetLastError());
  return 0;
}

}  // namespace fisdf
