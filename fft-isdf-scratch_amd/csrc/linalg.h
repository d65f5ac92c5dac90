#pragma once
#include "common.h"

#include <vector>

namespace fisdf {

struct CellGeom {
  double a[3][3];  // lattice vectors (rows), bohr
  double b[3][3];  // reciprocal vectors (rows), 2*pi*inv(a)^T
};

int gather_lp(hipStream_t s, const cplx* L, int n, int rmax, const int* piv, const int* rank,
              int rpad, cplx* Lp, int batch);
int trinv_blocks(hipStream_t s, const cplx* Lp, int r, int ldl, long sL, int nb, long sLi,
                 cplx* Linv, int batch);
int build_trsm_q(hipStream_t s, const cplx* Lp, int r, long sL, cplx* Q, int batch, int mode);
int trsm_merged_batched(hipStream_t s, const cplx* Q, long sQ, int r, cplx* X, long ld, long sX,
                        int ncol, int batch, bool lower_rhs = false, cplx* work = nullptr,
                        long work_elems = 0);
// split-K of one block row of trsm_merged_batched (from its shape only) and the workspace
// (complex elements) that lets a batch of `batch` r x r matrices run in one launch per row
int trsm_split_k(int nc, int b1);
long trsm_split_work_elems(int r, int batch);
int set_identity(hipStream_t s, cplx* X, int n, int batch);
// out[g][j*nao + m] = h_sc[j] * x0[h_k[j]][g][m] for the nsel listed k (any nsel)
int permute_kgm_sel(hipStream_t s, const cplx* x0, const int* h_k, const double* h_sc, int nsel,
                    int ng, int nao, cplx* out);
// time-reversal check of Bloch AO values a[k][row][nao] (k stride ks elements, get_kpts order) on
// every rstride-th row: atomically maxes mon[0] with max |a[-k] - conj(a[k])| and mon[1] with
// max |a[k]| (double bits)
int tr_check(hipStream_t s, const cplx* a, long ks, long rows, int nao, long rstride,
             const int kmesh[3], unsigned long long* mon);
// the time-reversal representatives k <= -k (ascending) and whether each is self-paired
void kmesh_reps(const int kmesh[3], std::vector<int>* reps, std::vector<char>* self);
int trsm_blocked(hipStream_t s, int lower, const cplx* Lp, long ldl, long sL, int r,
                 const cplx* Linv, long sLi, int nb, cplx* B, long ldb, long sB, cplx* X, long ldx,
                 long sX, int ncol, int batch, int a_real = 0);
// G indices whose Coulomb weight differs from that of G' = -G - m.b (ascending) -> idx, *count
int asym_list(hipStream_t s, const double* w, const int mesh[3], const int m[3], int* idx,
              int* count);
int gather_cols(hipStream_t s, const cplx* A, long ld, int r, const int* idx, int n, cplx* out);
// self-conjugate q on half the G: the prefix planes i0 < nH hold one member of every Hermitian
// pair G' = -G - m.b (both members on a self-paired plane); half_weight: w = sqrt of the pair's
// combined weight (c = coulG*scale, not rooted) on the prefix, 0 beyond; asym_half: the prefix G
// of unequal pair weights with f = (c - c')/(c + c') (1 on a self-paired plane), ascending
int half_prefix_planes(int n0, int m0);
int half_weight(hipStream_t s, double* w, const double* c, const int mesh[3], const int m[3]);
int asym_half(hipStream_t s, const double* c, const int mesh[3], const int m[3], int* idx,
              double* f, int* count);
int gather_cols_scaled(hipStream_t s, const cplx* A, long ld, int r, const int* idx,
                       const double* f, int n, cplx* out);
int add_imag(hipStream_t s, cplx* G, int ldg, const cplx* H, int ldh, int n);
// zero the imaginary parts of n complex elements
int zero_imag(hipStream_t s, cplx* a, long n);
// x4s[i] = x4all[qr[i]] (imag zeroed where qr[nq + i] != 0), also into L if not null
int stage_x4(hipStream_t s, const cplx* x4all, const int* qr, int nq, long nn, cplx* x4s, cplx* L);
// Minimum-norm operator of a rank-deficient x4_q from its rank-revealing pivoted Cholesky
// x4[P,P] ~ L L^H (L: rows of f_L, row order; piv: the pivot order; r = rank): A = P L (n x r),
// thin QR A = Q R by shifted CholeskyQR3, M = A^+ = R^{-1} Q^H (r x n, ld ldm; columns in pivot
// order) so that z[P] = M^H M y[P] is the minimum-norm solution (gelsy's complete orthogonal
// step).  Completes piv[r..n) with the rows outside the first r pivots (ascending).
// q_out (n x r) / rinv_out (r x r), if given, receive Q and R^{-1}.  work: min_norm_work_bytes(n, r); fail: 3 device ints (Cholesky breakdown per pass).
int min_norm_operator(hipStream_t s, const cplx* L, int n, int rmax, int* piv, int r,
                      cplx* M, long ldm, void* work, int* fail, cplx* q_out = nullptr,
                      cplx* rinv_out = nullptr);
size_t min_norm_work_bytes(int n, int r);
int scatter_w(hipStream_t s, const cplx* Wpp, int ldw, long sW, int rmax, const int* piv,
              const int* rank, cplx* W, int nip, int batch);
int conj_transpose(hipStream_t s, const cplx* A, int n, long sA, cplx* B, int batch);
int coulg_weight(hipStream_t s, const int mesh[3], const CellGeom& g, const double k[3],
                 double scale, int take_sqrt, double* w, double omega = 0.0);
int square_real(hipStream_t s, const cplx* in, cplx* out, long n, unsigned long long* maximag);
int csquare(hipStream_t s, cplx* a, long n, unsigned long long* maximag);
int rho_diag(hipStream_t s, const cplx* T, const cplx* X, int nset, int nk, int nip, int nao,
             double scale, cplx* rho);
int scale_rows(hipStream_t s, const cplx* X, const cplx* v, int nset, int nk, int nip, int i0,
               int nb, int nao, cplx* Xv);
int gather_points(hipStream_t s, const cplx* x0, int nk, int ng0, int nao, const int* perm,
                  int nip, cplx* X);
int square_scale(hipStream_t s, const cplx* in, double sc, cplx* out, long n);
int permute_kgm(hipStream_t s, const cplx* x0, int nq, int ng, int nao, cplx* out);
int pair_product(hipStream_t s, const cplx* A, int n1, const cplx* B, int n2, int nip, cplx* P);
// y_q = Phi^T (Re(Phi FX))^2 for the ascending q-list (h_qs on the host; d_qs a device copy,
// needed only when the k-mesh has more than 64 points), written to yT[slot][I][goff + g].
// half: FX holds only the kmesh_half_count(kmesh) representatives k <= -k (ascending k, 36 of
// 64 at 4x4x4); the others are conj(FX[-k]) (time reversal).  kmesh_rep_runs: the
// representatives as [begin, end) runs of consecutive k (pairs appended to runs)
int kmesh_half_count(const int kmesh[3]);
// Fused y build (time reversal, register k-meshes): fx_k = X_k f_k^H on MFMA for the
// representative k, staged per 16 x 16 (I, g) tile in LDS, then the kmesh_y DFTs — no fx in
// HBM.  X (nk, nip, nao); F = f + g0*nao with k stride fks (g rows of nao); writes
// yT[slot][I][goff + g] for g < m.  *handled = false (nothing enqueued) for other k-meshes
// or nk > 64 (the two-kernel path then runs).
// workspace bytes of y_fused for this shape (0: the fused kernel does not apply)
size_t y_fused_workspace(const int kmesh[3], int nip, int nao, int m);
// rmask: q (bits) stored real, as doubles in the first half of their slot (self-conjugate q)
int y_fused(hipStream_t s, const cplx* X, int nip, int nao, const cplx* F, long fks, int m,
            const int kmesh[3], const int* h_qs, int nq, cplx* yT, long qs, long Is, long goff,
            unsigned long long* mon, cplx* work, size_t work_bytes, unsigned long long rmask,
            bool* handled);
// whether the fused kernel covers this k-mesh (time reversal assumed)
bool y_fused_applies(const int kmesh[3], int nao);
// The same y build streamed behind a running selection (api.hip build_impl): rows [0, nip) of
// y in blocks of `rows` (a multiple of 16); block [lo, hi) forms its XT rows straight from x0
// through piv[lo..hi) once the selection's progress word (device) reaches hi, then runs the
// fused kernel on its I-tiles.  X is never read; work holds XT (nip rows) and FT as for
// y_fused.  *err (device) is set if a block waited past the bound.  *handled as for y_fused.
int y_fused_stream(hipStream_t s, const cplx* x0, int ng0, int nao, const int* piv,
                   const int* progress, int* err, int nip, int rows, const cplx* F, long fks,
                   int m, const int kmesh[3], const int* h_qs, int nq, cplx* yT, long qs, long Is,
                   long goff, cplx* work, size_t work_bytes, unsigned long long rmask,
                   bool* handled, hipStream_t s2 = nullptr, hipEvent_t ev_a = nullptr,
                   hipEvent_t ev_b = nullptr);
int kmesh_rep_runs(const int kmesh[3], std::vector<int>* runs);
// Bloch AO values (ao.hip): F (nimg, ng, nao) f64 workspace, scratch for the small tables;
// nkb > 0: at the nkb band k-points h_kband (any k) instead of the k-mesh, F (nT, ng, nao)
int eval_ao(hipStream_t s, const double* d_coords, int ng, int natm, const double* h_atoms, int nsh,
            const int* h_sh_atom, const int* h_sh_l, const int* h_sh_nprim, const double* h_exps,
            const double* h_coefs, int nT, const int* h_tn, const int kmesh[3], const double a[9],
            double rcut, double* F, void* scratch, size_t scratch_size, cplx* chi, int* h_nao,
            int nkb = 0, const double* h_kband = nullptr);
// conj_out: store conj(y_q) — the x4 build's Phi^H x4_s (fftisdf.py:46; x4_s real) where the y
// build has Phi^T y_s (:84)
int kmesh_y(hipStream_t s, const cplx* FX, long ncol, const int kmesh[3], const int* h_qs,
            const int* d_qs, int nq, int m, cplx* yT, long qs, long Is, long goff, bool half,
            unsigned long long* mon, bool conj_out = false);
// whether kmesh_y runs its register kernel for this k-mesh and column count (no device q-list)
bool kmesh_y_reg_applies(const int kmesh[3], long ncol);
// get_k's rho_s = Phi rho_k, V_s = W_s * Re(rho_s), V_k = Phi^T V_s in place on B (nk rows of
// ncol columns; W_s row s at Ws + s * ws_Rstride) for the register k-meshes; *handled = false
// (nothing enqueued) otherwise.  max |Im rho_s| into *mon
int k_wsrho_reg(hipStream_t s, cplx* B, long ncol, const int kmesh[3], const double* Ws,
                long ws_Rstride, unsigned long long* mon, bool* handled);

}  // namespace fisdf
