// Wide-tile complex128 GEMM for the fit's big NN products (U = L^{-1} Yhat, the minimum-norm
// U = M Yhat; fftisdf.py:108 in factored order) on CDNA4 FP64 matrix cores.
//
// Same operand path as zgemm_glds_kernel (global_load_lds_dwordx4 into an NS-deep LDS ring,
// counted vmcnt waits, one barrier per K-step, 3 real MFMAs per complex 16x16x4 block in FULL
// mode), but each wave owns 32 x 64 of C (2 x 4 blocks of v_mfma_f64_16x16x4_f64) instead of
// 32 x 32, so the workgroup tile is 64 x 128: per K-substep a wave issues 24 MFMAs against 6 LDS
// fragment reads and 6 operand additions (12 / 4 / 4 in the 64 x 64 kernel), and per K-step 6
// LDS-DMA pieces (4 per 24 MFMAs there) — the per-MFMA overheads that held the 64 x 64 kernel
// at ~75 % of the FP64 MFMA pipe (profiles/r02_pmc_gemm_summary.txt) are halved or better.
// op(A) = A (N, [m][k], K-contiguous: XOR-swizzled LDS image), op(B) = B (N, [k][n]).
// MODE: GEMM_FULL, GEMM_A_REAL (Im A = 0: 2 MFMAs per block), GEMM_A_LOWER (A lower
// triangular: each M-tile stops its K loop at its last row; longest tiles dispatched first).
// XCD-aware order as in zgemm.hip: XCD x owns a contiguous chunk of (M-tile fastest, N-panel)
// order, so the M-tiles sharing one 128-column panel of B read it from that XCD's L2.
#include "common.h"

namespace fisdf {

namespace {

#ifndef FISDF_WIDE_PIPE
#define FISDF_WIDE_PIPE 1
#endif

constexpr int WBM = 64, WBN = 128, WBK = 8;
constexpr int TA = WBM * WBK;   // complex elements of one A stage (8 KB)
constexpr int TB = WBN * WBK;   // one B stage (16 KB)
constexpr int LPA = TA / 256;   // LDS-DMA pieces per wave per K-step: A
constexpr int LPB = TB / 256;   //                                      B
__device__ cplx g_wide_zero[64];

template <int MODE, int NS>
__global__ __launch_bounds__(256, 2) void zgemm_nn_wide_kernel(
    int M, int N, int K, cplx alpha, const cplx* __restrict__ A, long lda,
    const cplx* __restrict__ B, long ldb, cplx beta, cplx* __restrict__ C, long ldc, int nMt,
    int ntot, unsigned long long* __restrict__ span) {
  __shared__ cplx sm[NS * (TA + TB)];
  const int per = (int)(gridDim.x >> 3);
  const int order = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (order >= ntot) return;
  span_begin(span);
  int ti = order % nMt;
  const int tj = order / nMt;
  if constexpr ((MODE & GEMM_A_LOWER) != 0) ti = nMt - 1 - ti;  // longest K first
  const int m0 = ti * WBM, n0 = tj * WBN;
  int kend = K;
  if constexpr ((MODE & GEMM_A_LOWER) != 0) kend = min(kend, m0 + WBM);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // an M-edge tile with <= 32 valid rows gives every wave 32 rows x 32 columns (2 x 2 blocks)
  // instead of leaving the lower two waves idle
  const int vr = min(4, max(0, (M - m0 + 15) / 16));
  const bool edge = vr <= 2;
  const int wm = edge ? 0 : (w >> 1) * 32;
  const int wn = edge ? 32 * w : (w & 1) * 64;

  // LDS-DMA sources.  A stage: slot sl = row x * 8 + k' holds A[m0 + x][k0 + (k' ^ (x & 7))];
  // B stage: slot sl = k * 128 + x holds B[k0 + k][n0 + x].  Rows / columns outside the matrix
  // read a zero page (step 0 then: they never advance).
  const cplx* zp = g_wide_zero;
  const cplx* srcA[LPA];
  const cplx* srcB[LPB];
  int kA[LPA], kB[LPB];
#pragma unroll
  for (int j = 0; j < LPA; ++j) {
    const int sl = (w * LPA + j) * 64 + lane;
    const int x = sl / WBK, k = (sl % WBK) ^ (x & (WBK - 1));
    kA[j] = k;
    srcA[j] = m0 + x < M ? A + (long)(m0 + x) * lda + k : nullptr;
  }
#pragma unroll
  for (int j = 0; j < LPB; ++j) {
    const int sl = (w * LPB + j) * 64 + lane;
    const int x = sl % WBN, k = sl / WBN;
    kB[j] = k;
    srcB[j] = n0 + x < N ? B + (long)k * ldb + (n0 + x) : nullptr;
  }
  const unsigned lds0 = (unsigned)(uintptr_t)sm;
  auto glds = [&](const cplx* src, unsigned lds_byte) {
    unsigned keep;
    const unsigned dst = __builtin_amdgcn_readfirstlane(lds_byte);
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
  };
  auto issue = [&](int st) {  // K-step st -> ring slot st % NS
    const int buf = st % NS;
    const int k0 = st * WBK;
    const unsigned la = lds0 + (unsigned)(buf * (TA + TB)) * 16u;
    const unsigned lb = la + (unsigned)TA * 16u;
#pragma unroll
    for (int j = 0; j < LPA; ++j) {
      const cplx* pa = (srcA[j] && k0 + kA[j] < kend) ? srcA[j] + k0 : zp;
      glds(pa, la + (unsigned)((w * LPA + j) * 64) * 16u);
    }
#pragma unroll
    for (int j = 0; j < LPB; ++j) {
      const cplx* pb = (srcB[j] && k0 + kB[j] < kend) ? srcB[j] + (long)k0 * ldb : zp;
      glds(pb, lb + (unsigned)((w * LPB + j) * 64) * 16u);
    }
  };

  constexpr bool AREAL = (MODE & GEMM_A_REAL) != 0;
  // FULL: accR = P1 = ar br, accI = P2 = ai bi, acc3 = P3 = (ar + ai)(br + bi); after the K loop
  // Re = P1 - P2, Im = P3 - P1 - P2.  A_REAL: accR = ar br, accI = ar bi.
  f64x4 accR[2][4], accI[2][4], acc3[AREAL ? 1 : 2][AREAL ? 1 : 4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      accR[i][j] = f64x4{0, 0, 0, 0};
      accI[i][j] = f64x4{0, 0, 0, 0};
      if constexpr (!AREAL) acc3[i][j] = f64x4{0, 0, 0, 0};
    }

  const int nsteps = kend > 0 ? (kend + WBK - 1) / WBK : 0;
  const int i16 = lane & 15, kq = lane >> 4;
#if FISDF_WIDE_PIPE
  // Software-pipelined main loop (kend % WBK == 0, checked by zgemm_wide_applies): the LDS
  // fragments of the next K-substep are read while the current substep's third MFMA group
  // (P3 = (ar + ai)(br + bi)) runs — after P1 and P2 the raw fragments are dead, so the reads
  // reuse their registers — and the barrier of the next K-step sits inside the last substep,
  // between its P1/P2 and P3 groups.  Per-lane operand pointers advance by a fixed stride (the
  // zero page at stride 0 for rows / columns outside the matrix); no loads past the last step.
  // rows / columns outside the matrix read a clamped in-range row / column instead of the zero
  // page: they only feed C rows / columns that are never stored, and every lane then advances
  // by the same (scalar) stride
  (void)kA;
  (void)kB;
  // per-lane 32-bit byte offsets from a wave-uniform base (the SADDR form of the LDS-DMA load):
  // one VGPR per piece, the K advance in scalar registers
  unsigned oA[LPA], oB[LPB];
#pragma unroll
  for (int j = 0; j < LPA; ++j) {
    const int sl = (w * LPA + j) * 64 + lane;
    const int x = sl / WBK, k = (sl % WBK) ^ (x & (WBK - 1));
    oA[j] = (unsigned)(((long)min(m0 + x, M - 1) * lda + k) * 16);
  }
#pragma unroll
  for (int j = 0; j < LPB; ++j) {
    const int sl = (w * LPB + j) * 64 + lane;
    const int x = sl % WBN, k = sl / WBN;
    oB[j] = (unsigned)(((long)k * ldb + min(n0 + x, N - 1)) * 16);
  }
  const long dBs = (long)WBK * ldb;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  auto gldss = [&](const cplx* base, unsigned off, unsigned lds_byte) {
    unsigned keep;
    const unsigned dst = __builtin_amdgcn_readfirstlane(lds_byte);
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(off), "s"(base), "s"(dst) : "memory");
  };
  auto issue_p = [&](int st) {  // K-step st -> ring slot st % NS
    const int buf = st % NS;
    const unsigned la = lds0 + (unsigned)(buf * (TA + TB)) * 16u;
    const unsigned lb = la + (unsigned)TA * 16u;
    const cplx* ba = A + (long)st * WBK;
    const cplx* bb = B + st * dBs;
#pragma unroll
    for (int j = 0; j < LPA; ++j) gldss(ba, oA[j], la + (unsigned)((wu * LPA + j) * 64) * 16u);
#pragma unroll
    for (int j = 0; j < LPB; ++j) gldss(bb, oB[j], lb + (unsigned)((wu * LPB + j) * 64) * 16u);
  };
  auto pipeloop = [&](auto nbc) {
    constexpr int NB = decltype(nbc)::value;
    if (nsteps == 0) return;
#pragma unroll
    for (int st = 0; st < NS - 1; ++st)
      if (st < nsteps) issue_p(st);
    if (nsteps > 1)
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((LPA + LPB) * (NS - 2)) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    cplx fa[2], fb[NB];
    auto rd = [&](int slot, int kk) {
      const cplx* as = sm + (long)slot * (TA + TB);
      const cplx* bs = as + TA;
      const int k = kk + kq;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int x = wm + u * 16 + i16;
        fa[u] = as[x * WBK + (k ^ (x & (WBK - 1)))];
      }
#pragma unroll
      for (int u = 0; u < NB; ++u) fb[u] = bs[k * WBN + wn + u * 16 + i16];
    };
    rd(0, 0);
    if (NS - 1 < nsteps) issue_p(NS - 1);
    double sa[2], sb[NB];
    auto p12 = [&]() {
#pragma unroll
      for (int u = 0; u < 2; ++u) sa[u] = fa[u].x + fa[u].y;
#pragma unroll
      for (int u = 0; u < NB; ++u) sb[u] = fb[u].x + fb[u].y;
      if constexpr (AREAL) {
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < NB; ++ni)
            accR[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[mi].x, fb[ni].x, accR[mi][ni], 0, 0, 0);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < NB; ++ni)
            accI[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[mi].x, fb[ni].y, accI[mi][ni], 0, 0, 0);
      } else {
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < NB; ++ni)
            accR[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[mi].x, fb[ni].x, accR[mi][ni], 0, 0, 0);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < NB; ++ni)
            accI[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[mi].y, fb[ni].y, accI[mi][ni], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    auto p3 = [&]() {
      if constexpr (!AREAL) {
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < NB; ++ni)
            acc3[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(sa[mi], sb[ni], acc3[mi][ni], 0, 0, 0);
      }
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
        // step s+1 landed (step s+2's pieces may stay in flight) and every wave is done with
        // step s's slot, which issue_p(s + NS) refills
        if (s + 2 < nsteps)
          asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((LPA + LPB) * (NS - 2)) : "memory");
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
  if (edge)
    pipeloop(std::integral_constant<int, 2>{});
  else
    pipeloop(std::integral_constant<int, 4>{});
#else
  if (nsteps > 0) {
#pragma unroll
    for (int st = 0; st < NS - 1; ++st) issue(st);
  }
  auto mainloop = [&](auto nbc) {
    constexpr int NB = decltype(nbc)::value;  // column blocks per wave (4, or 2 on an edge tile)
    for (int s = 0; s < nsteps; ++s) {
      // own pieces of step s landed (the NS-2 later steps' stay in flight), then every wave's:
      // the barrier also retires all reads of the slot step s+NS-1 is about to overwrite
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((LPA + LPB) * (NS - 2)) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      const int cur = s % NS;
      const cplx* as = sm + (long)cur * (TA + TB);
      const cplx* bs = as + TA;
      const int kleft = kend - s * WBK;  // K-substeps past the end hold only zeros
      issue(s + NS - 1);
#pragma unroll
      for (int kk = 0; kk < WBK; kk += 4) {
        if (kk > 0 && kk >= kleft) break;
        const int k = kk + kq;
        double ar[2], ai[2], br[NB], bi[NB];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int x = wm + u * 16 + i16;
          const cplx a = as[x * WBK + (k ^ (x & (WBK - 1)))];
          ar[u] = a.x;
          ai[u] = a.y;
        }
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          const cplx b = bs[k * WBN + wn + u * 16 + i16];
          br[u] = b.x;
          bi[u] = b.y;
        }
        if constexpr (AREAL) {
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < NB; ++ni)
              accR[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[mi], br[ni], accR[mi][ni], 0, 0, 0);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < NB; ++ni)
              accI[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[mi], bi[ni], accI[mi][ni], 0, 0, 0);
        } else {
          double sa[2], sb[NB];
#pragma unroll
          for (int u = 0; u < 2; ++u) sa[u] = ar[u] + ai[u];
#pragma unroll
          for (int u = 0; u < NB; ++u) sb[u] = br[u] + bi[u];
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < NB; ++ni)
              accR[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[mi], br[ni], accR[mi][ni], 0, 0, 0);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < NB; ++ni)
              accI[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai[mi], bi[ni], accI[mi][ni], 0, 0, 0);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < NB; ++ni)
              acc3[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(sa[mi], sb[ni], acc3[mi][ni], 0, 0, 0);
        }
      }
    }
  };
  if (edge)
    mainloop(std::integral_constant<int, 2>{});
  else
    mainloop(std::integral_constant<int, 4>{});
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the zero-page pieces in flight

  const int nb = edge ? 2 : 4;
  const bool use_beta = beta.x != 0.0 || beta.y != 0.0;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      if (ni >= nb) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + mi * 16 + (lane >> 4) + 4 * r;
        const int col = n0 + wn + ni * 16 + (lane & 15);
        if (row < M && col < N) {
          double re, im;
          if constexpr (AREAL) {
            re = accR[mi][ni][r];
            im = accI[mi][ni][r];
          } else {
            const double p1 = accR[mi][ni][r], p2 = accI[mi][ni][r], p3 = acc3[mi][ni][r];
            re = p1 - p2;
            im = p3 - p1 - p2;
          }
          cplx v = cmul(alpha, cmk(re, im));
          cplx* cp = C + (long)row * ldc + col;
          if (use_beta) v = cadd(v, cmul(beta, *cp));
          // non-temporal: U (0.45 GB per q at C3) is read next by the HERK, long after the L2
          // could hold it; streaming it past L2 keeps the L^-1 bands and Yhat panels the other
          // tiles re-read (interleaved A/B, three pairs: 81.09 vs 81.27 ms/step)
          typedef double dv2 __attribute__((ext_vector_type(2)));
          __builtin_nontemporal_store(dv2{v.x, v.y}, (dv2*)cp);
        }
      }
    }
  span_end(span);
}

template <int MODE>
void launch_wide(hipStream_t s, int M, int N, int K, cplx alpha, const cplx* A, long lda,
                 const cplx* B, long ldb, cplx beta, cplx* C, long ldc, unsigned long long* span) {
  const int nMt = (M + WBM - 1) / WBM, nNt = (N + WBN - 1) / WBN;
  const long ntot = (long)nMt * nNt;
  const long per = (ntot + 7) / 8;
  hipLaunchKernelGGL((zgemm_nn_wide_kernel<MODE, 3>), dim3((unsigned)(8 * per)), dim3(256), 0, s, M,
                     N, K, alpha, A, lda, B, ldb, beta, C, ldc, nMt, (int)ntot, span);
}

}  // namespace

// FISDF_GEMM_WIDE=0 routes these products through the 64 x 64 kernel (A/B on one box)
bool wide_gemm_enabled() {
  static const bool on = [] {
    const char* e = getenv("FISDF_GEMM_WIDE");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool zgemm_wide_applies(int opA, int opB, int M, int N, int K, long lda, long ldb, int batch,
                        int ksplit, int epi,
                        int mode) {
  // the pipelined loop addresses each lane's operand piece by a 32-bit byte offset from a
  // wave-uniform base: A's last row up to column K, B's first WBK rows
  const long lim = 1L << 32;
  const bool off32 = ((long)std::max(M - 1, 0) * lda + K) * 16 < lim &&
                     ((long)WBK * ldb + N) * 16 < lim;
  return opA == OP_N && opB == OP_N && batch == 1 && ksplit <= 1 && epi == EPI_NONE &&
         K % WBK == 0 && off32 &&
         (mode & ~(GEMM_A_REAL | GEMM_A_LOWER)) == 0 && N >= 4 * WBN && wide_gemm_enabled();
}

int zgemm_nn_wide(hipStream_t s, int M, int N, int K, cplx alpha, const cplx* A, long lda,
                  const cplx* B, long ldb, cplx beta, cplx* C, long ldc, int mode,
                  unsigned long long* span) {
  FISDF_CHECK((long)((M + WBM - 1) / WBM) * ((N + WBN - 1) / WBN) < (1L << 31),
              "zgemm_nn_wide: too many tiles");
  switch (mode) {
    case GEMM_FULL: launch_wide<GEMM_FULL>(s, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, span); break;
    case GEMM_A_REAL: launch_wide<GEMM_A_REAL>(s, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, span); break;
    case GEMM_A_LOWER: launch_wide<GEMM_A_LOWER>(s, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, span); break;
    case GEMM_A_LOWER | GEMM_A_REAL:
      launch_wide<GEMM_A_LOWER | GEMM_A_REAL>(s, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, span);
      break;
    default: FISDF_CHECK(false, "zgemm_nn_wide: unsupported mode");
  }
  FISDF_HIP(hipGetLastError());
  return 0;
}

}  // namespace fisdf
