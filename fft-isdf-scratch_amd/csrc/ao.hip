// Bloch AO values on a uniform grid: the input layer PySCF's
// pbc_eval_gto('GTOval') / KNumInt.block_loop provides to fftisdf.py:72,327-355,367-370,
// restated on the host as fisdf/cell.py (eval_ao_folded + eval_ao_kpts) and moved here.
//
//   F_R(r)   = sum_{T = n.a, n = R mod kmesh} phi(r - T)          (real, image-folded)
//   chi_k(r) = sum_R exp(i T_R . k) F_R(r)                         (k-mesh inverse DFT)
//
// ao_folded_kernel: one thread per (grid point, AO), translations grouped by image R in the
// host list's order (the same summation order as cell.py); bloch_dft_reg_kernel: one thread
// per (g, AO) column, the separable k-mesh DFT in registers (as the y build's).
#include <vector>

#include "common.h"
#include "linalg.h"

namespace fisdf {

namespace {

struct AoShell {
  int atom, l, nprim, p0;  // p0: first primitive in the exponent / coefficient arrays
};

// real solid harmonics r^l Y_lm, cell.py::_real_sph order and constants
__device__ __forceinline__ double real_sph(int l, int m, double x, double y, double z) {
  if (l == 0) return 0.28209479177387814;
  if (l == 1) return 0.4886025119029199 * (m == 0 ? x : (m == 1 ? y : z));
  const double r2 = x * x + y * y + z * z;
  if (l == 2) {
    switch (m) {
      case 0: return 1.0925484305920792 * x * y;
      case 1: return 1.0925484305920792 * y * z;
      case 2: return 0.31539156525252005 * (3 * z * z - r2);
      case 3: return 1.0925484305920792 * x * z;
      default: return 0.5462742152960396 * (x * x - y * y);
    }
  }
  switch (m) {  // l == 3
    case 0: return 0.5900435899266435 * y * (3 * x * x - y * y);
    case 1: return 2.890611442640554 * x * y * z;
    case 2: return 0.4570457994644658 * y * (5 * z * z - r2);
    case 3: return 0.3731763325901154 * z * (5 * z * z - 3 * r2);
    case 4: return 0.4570457994644658 * x * (5 * z * z - r2);
    case 5: return 1.445305721320277 * z * (x * x - y * y);
    default: return 0.5900435899266435 * x * (x * x - 3 * y * y);
  }
}

__global__ __launch_bounds__(256) void ao_folded_kernel(
    const double* __restrict__ coords, int ng, int nao, const int* __restrict__ ao_shell,
    const int* __restrict__ ao_m, const AoShell* __restrict__ sh, const double* __restrict__ pexp,
    const double* __restrict__ pcoef, const double* __restrict__ atoms,
    const double* __restrict__ Tvec, const int* __restrict__ Toff, int nimg, double rc2,
    double* __restrict__ F) {
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= (long)ng * nao) return;
  const int g = (int)(e / nao), nu = (int)(e % nao);
  const AoShell s = sh[ao_shell[nu]];
  const int m = ao_m[nu];
  const double gx = coords[3L * g] - atoms[3 * s.atom];
  const double gy = coords[3L * g + 1] - atoms[3 * s.atom + 1];
  const double gz = coords[3L * g + 2] - atoms[3 * s.atom + 2];
  for (int R = 0; R < nimg; ++R) {
    double acc = 0.0;
    for (int t = Toff[R]; t < Toff[R + 1]; ++t) {
      const double dx = gx - Tvec[3 * t], dy = gy - Tvec[3 * t + 1], dz = gz - Tvec[3 * t + 2];
      const double r2 = dx * dx + dy * dy + dz * dz;
      if (r2 < rc2) {
        double rad = 0.0;
        for (int p = 0; p < s.nprim; ++p) rad += exp(-pexp[s.p0 + p] * r2) * pcoef[s.p0 + p];
        acc += rad * real_sph(s.l, m, dx, dy, dz);
      }
    }
    F[((long)R * ng + g) * nao + nu] = acc;
  }
}

template <int N, int S, int NK>
__device__ __forceinline__ void ao_axis_dft(cplx* v, const cplx* tw) {
#pragma unroll
  for (int hi = 0; hi < NK / (N * S); ++hi)
#pragma unroll
    for (int lo = 0; lo < S; ++lo) {
      cplx* p = v + hi * N * S + lo;
      if constexpr (N > 1) {
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

// chi[k][c] = sum_R exp(+2 pi i sum_a r_a k_a / n_a) F[R][c]   (c = g*nao + nu)
template <int N0, int N1, int N2>
__global__ __launch_bounds__(64) void bloch_dft_reg_kernel(const double* __restrict__ F, long ncol,
                                                           cplx* __restrict__ chi) {
  constexpr int NK = N0 * N1 * N2;
  cplx tw0[N0], tw1[N1], tw2[N2];
#pragma unroll
  for (int t = 0; t < N0; ++t) { double s, c; sincospi(2.0 * t / N0, &s, &c); tw0[t] = cmk(c, s); }
#pragma unroll
  for (int t = 0; t < N1; ++t) { double s, c; sincospi(2.0 * t / N1, &s, &c); tw1[t] = cmk(c, s); }
#pragma unroll
  for (int t = 0; t < N2; ++t) { double s, c; sincospi(2.0 * t / N2, &s, &c); tw2[t] = cmk(c, s); }
  for (long col = blockIdx.x * (long)blockDim.x + threadIdx.x; col < ncol;
       col += (long)gridDim.x * blockDim.x) {
    cplx v[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) v[k] = cmk(F[(long)k * ncol + col], 0.0);
    ao_axis_dft<N0, N1 * N2, NK>(v, tw0);
    ao_axis_dft<N1, N2, NK>(v, tw1);
    ao_axis_dft<N2, 1, NK>(v, tw2);
#pragma unroll
    for (int k = 0; k < NK; ++k) chi[(long)k * ncol + col] = v[k];
  }
}

// any k-mesh: one thread per (k, column), direct sum over the images
__global__ void bloch_dft_kernel(const double* __restrict__ F, long ncol, int n0, int n1, int n2,
                                 cplx* __restrict__ chi) {
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int nk = n0 * n1 * n2;
  if (e >= ncol * nk) return;
  const int k = (int)(e / ncol);
  const long col = e % ncol;
  const int k2 = k % n2, k1 = (k / n2) % n1, k0 = k / (n1 * n2);
  cplx acc = cmk(0, 0);
  for (int R = 0; R < nk; ++R) {
    const int r2 = R % n2, r1 = (R / n2) % n1, r0 = R / (n1 * n2);
    // exp(2 pi i (r0 k0 / n0 + r1 k1 / n1 + r2 k2 / n2)), each term reduced mod 1 exactly
    const double f = (double)((r0 * k0) % n0) / n0 + (double)((r1 * k1) % n1) / n1 +
                     (double)((r2 * k2) % n2) / n2;
    double s, c;
    sincospi(2.0 * f, &s, &c);
    const double x = F[(long)R * ncol + col];
    acc = cadd(acc, cmk(c * x, s * x));
  }
  chi[(long)k * ncol + col] = acc;
}

// band k-points (any k, kpts_band of get_jk): chi[k][col] = sum_t exp(i k . T_t) F[t][col], one
// thread per (k, column), F holding one image per lattice translation
__global__ void bloch_band_kernel(const double* __restrict__ F, long ncol, int nT,
                                  const cplx* __restrict__ ph, int nkb, cplx* __restrict__ chi) {
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= ncol * nkb) return;
  const int k = (int)(e / ncol);
  const long col = e % ncol;
  cplx acc = cmk(0, 0);
  for (int t = 0; t < nT; ++t) {
    const double x = F[(long)t * ncol + col];
    const cplx p = ph[(long)t * nkb + k];
    acc = cadd(acc, cmk(p.x * x, p.y * x));
  }
  chi[(long)k * ncol + col] = acc;
}

}  // namespace

int eval_ao(hipStream_t s, const double* d_coords, int ng, int natm, const double* h_atoms, int nsh,
            const int* h_sh_atom, const int* h_sh_l, const int* h_sh_nprim, const double* h_exps,
            const double* h_coefs, int nT, const int* h_tn, const int kmesh[3], const double a[9],
            double rcut, double* F, void* scratch, size_t scratch_size, cplx* chi, int* h_nao,
            int nkb, const double* h_kband) {
  FISDF_CHECK(ng >= 0 && natm > 0 && nsh > 0 && nT >= 0, "eval_ao: bad sizes");
  // band mode (nkb > 0): every translation is its own image, phases exp(i k.T) per band k
  const bool band = nkb > 0;
  const int nimg = band ? std::max(nT, 1) : kmesh[0] * kmesh[1] * kmesh[2];
  // shells, AO -> (shell, m) maps
  std::vector<AoShell> sh(nsh);
  std::vector<int> ao_shell, ao_m;
  int p0 = 0;
  for (int i = 0; i < nsh; ++i) {
    FISDF_CHECK(h_sh_l[i] >= 0 && h_sh_l[i] <= 3, "eval_ao: angular momentum must be <= 3");
    FISDF_CHECK(h_sh_atom[i] >= 0 && h_sh_atom[i] < natm, "eval_ao: shell atom out of range");
    sh[i] = AoShell{h_sh_atom[i], h_sh_l[i], h_sh_nprim[i], p0};
    p0 += h_sh_nprim[i];
    for (int m = 0; m < 2 * h_sh_l[i] + 1; ++m) {
      ao_shell.push_back(i);
      ao_m.push_back(m);
    }
  }
  const int nao = (int)ao_shell.size();
  if (h_nao) *h_nao = nao;
  // translations T = n . a grouped by image R = n mod kmesh, list order kept within R
  std::vector<std::vector<double>> byR(nimg);
  for (int t = 0; t < nT; ++t) {
    const int* n = h_tn + 3 * t;
    int r[3];
    for (int d = 0; d < 3 && !band; ++d) r[d] = ((n[d] % kmesh[d]) + kmesh[d]) % kmesh[d];
    const int R = band ? t : (r[0] * kmesh[1] + r[1]) * kmesh[2] + r[2];
    for (int d = 0; d < 3; ++d)
      byR[R].push_back(n[0] * a[0 * 3 + d] + n[1] * a[1 * 3 + d] + n[2] * a[2 * 3 + d]);
  }
  std::vector<double> Tvec;
  std::vector<int> Toff(nimg + 1, 0);
  for (int R = 0; R < nimg; ++R) {
    Tvec.insert(Tvec.end(), byR[R].begin(), byR[R].end());
    Toff[R + 1] = (int)(Tvec.size() / 3);
  }
  // device copies of the small tables, carved from the scratch buffer
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  };
  const size_t oS = take(sizeof(AoShell) * nsh), oAS = take(sizeof(int) * nao),
               oAM = take(sizeof(int) * nao), oE = take(sizeof(double) * p0),
               oC = take(sizeof(double) * p0), oA = take(sizeof(double) * 3 * natm),
               oT = take(sizeof(double) * std::max<size_t>(Tvec.size(), 1)),
               oO = take(sizeof(int) * (nimg + 1)),
               oP = take(sizeof(cplx) * (band ? (size_t)nimg * nkb : 1));
  FISDF_CHECK(off <= scratch_size, "eval_ao: scratch too small");
  std::vector<cplx> ph;
  if (band) {  // exp(i k . T_t), T_t = n_t . a in the translation order (one image each)
    ph.resize((size_t)nimg * nkb, cmk(0, 0));
    for (int t = 0; t < nT; ++t)
      for (int k = 0; k < nkb; ++k) {
        double th = 0;
        for (int d = 0; d < 3; ++d) th += Tvec[3 * t + d] * h_kband[3 * k + d];
        ph[(size_t)t * nkb + k] = cmk(std::cos(th), std::sin(th));
      }
  }
  char* b = (char*)scratch;
  FISDF_HIP(hipMemcpyAsync(b + oS, sh.data(), sizeof(AoShell) * nsh, hipMemcpyHostToDevice, s));
  FISDF_HIP(hipMemcpyAsync(b + oAS, ao_shell.data(), sizeof(int) * nao, hipMemcpyHostToDevice, s));
  FISDF_HIP(hipMemcpyAsync(b + oAM, ao_m.data(), sizeof(int) * nao, hipMemcpyHostToDevice, s));
  FISDF_HIP(hipMemcpyAsync(b + oE, h_exps, sizeof(double) * p0, hipMemcpyHostToDevice, s));
  FISDF_HIP(hipMemcpyAsync(b + oC, h_coefs, sizeof(double) * p0, hipMemcpyHostToDevice, s));
  FISDF_HIP(hipMemcpyAsync(b + oA, h_atoms, sizeof(double) * 3 * natm, hipMemcpyHostToDevice, s));
  if (!Tvec.empty())
    FISDF_HIP(hipMemcpyAsync(b + oT, Tvec.data(), sizeof(double) * Tvec.size(),
                             hipMemcpyHostToDevice, s));
  FISDF_HIP(hipMemcpyAsync(b + oO, Toff.data(), sizeof(int) * (nimg + 1), hipMemcpyHostToDevice, s));
  if (band)
    FISDF_HIP(hipMemcpyAsync(b + oP, ph.data(), sizeof(cplx) * ph.size(), hipMemcpyHostToDevice, s));
  if (ng == 0) {
    FISDF_HIP(hipStreamSynchronize(s));  // the host tables must outlive the asynchronous copies
    return 0;
  }
  const long nth = (long)ng * nao;
  hipLaunchKernelGGL(ao_folded_kernel, dim3((unsigned)((nth + 255) / 256)), dim3(256), 0, s,
                     d_coords, ng, nao, (const int*)(b + oAS), (const int*)(b + oAM),
                     (const AoShell*)(b + oS), (const double*)(b + oE), (const double*)(b + oC),
                     (const double*)(b + oA), (const double*)(b + oT), (const int*)(b + oO), nimg,
                     rcut * rcut, F);
  FISDF_HIP(hipGetLastError());
  // the host tables must outlive the asynchronous copies
  FISDF_HIP(hipStreamSynchronize(s));
  const long ncol = nth;
  if (band) {
    const long tot = ncol * nkb;
    hipLaunchKernelGGL(bloch_band_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, F,
                       ncol, nT, (const cplx*)(b + oP), nkb, chi);
    FISDF_HIP(hipGetLastError());
    return 0;
  }
#define FISDF_BD(x, y, z)                                                                      \
  if (kmesh[0] == x && kmesh[1] == y && kmesh[2] == z) {                                       \
    hipLaunchKernelGGL((bloch_dft_reg_kernel<x, y, z>),                                         \
                       dim3((unsigned)std::min<long>((ncol + 63) / 64, 65536)), dim3(64), 0, s, F, \
                       ncol, chi);                                                             \
    FISDF_HIP(hipGetLastError());                                                              \
    return 0;                                                                                  \
  }
  FISDF_BD(1, 1, 1) FISDF_BD(1, 1, 2) FISDF_BD(2, 2, 2) FISDF_BD(3, 3, 1) FISDF_BD(3, 3, 3)
  FISDF_BD(4, 4, 4) FISDF_BD(2, 2, 1) FISDF_BD(1, 2, 2) FISDF_BD(4, 4, 1) FISDF_BD(2, 2, 4)
#undef FISDF_BD
  const long tot = ncol * nimg;
  hipLaunchKernelGGL(bloch_dft_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, F,
                     ncol, kmesh[0], kmesh[1], kmesh[2], chi);
  FISDF_HIP(hipGetLastError());
  return 0;
}

}  // namespace fisdf
