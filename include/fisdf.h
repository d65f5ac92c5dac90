/*
 * fisdf — MI355X-native FFT-ISDF kernel library: the C-ABI drop-in boundary.
 *
 * The reference (yangjunjie0320/fft-isdf-scratch) has no native boundary: its hot
 * path is the Python module fftisdf.py calling NumPy/SciPy/PySCF.  Each entry point
 * below replaces one stage of that path; the Python mirror of the reference's
 * `ISDF` class (fft-isdf-scratch_amd/fisdf/isdf.py) binds them with ctypes
 * (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - complex arrays are complex128 (interleaved double re/im), C-contiguous.
 *  - pointers named d_* are DEVICE pointers (hipMalloc'ed, or from fisdf_malloc);
 *    pointers named h_* are host pointers.  Work is enqueued on the context's stream
 *    and is asynchronous unless the function says "synchronous".
 *  - every function returns 0 on success or a negative code; fisdf_last_error(ctx)
 *    returns the message of that context's last failure (fisdf_last_error(NULL): the last
 *    failure on the calling thread, e.g. of fisdf_create).
 *  - a context is not thread-safe; several contexts (devices) may be driven from one thread.
 *
 * Two layers: the composite entries (fisdf_build / fisdf_get_jk / fisdf_get_wq, the reference's
 * ISDF.build() and ISDF.get_jk(), fftisdf.py:308-325,390-408) drive the whole 1-GPU path; the
 * stage entries below them are what the composite entries run, exported for k-sharded callers
 * (which interleave collectives between the stages, fisdf/isdf.py) and for the tests.
 */
#ifndef FISDF_H
#define FISDF_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FISDF_ABI_VERSION 4

typedef struct fisdf_ctx fisdf_ctx;

/* stage ids for fisdf_timings */
enum {
  FISDF_ST_SELECT = 0, /* Gram + pivoted Cholesky (fftisdf.py:357-388)          */
  FISDF_ST_X4 = 1,     /* x2_k, x2_s, x4_s, x4_k (fftisdf.py:38-48)               */
  FISDF_ST_Y = 2,      /* y build (fftisdf.py:67-87)                              */
  FISDF_ST_FACTOR = 3, /* per-q factorisation of x4_q (replaces zgelsy QRCP :108) */
  FISDF_ST_FFT = 4,    /* fft(z_q * f_q) * coulG weight (fftisdf.py:113-115)      */
  FISDF_ST_TRSM = 5,   /* factored fit application (fftisdf.py:108)               */
  FISDF_ST_HERK = 6,   /* W_q = zeta z_q^H (fftisdf.py:118-121, Parseval HERK)   */
  FISDF_ST_SMALL = 7,  /* nip x nip back-substitutions + scatter                  */
  FISDF_ST_J = 8,      /* get_j_kpts (fftisdf.py:133-171)                         */
  FISDF_ST_K = 9,      /* get_k_kpts (fftisdf.py:173-228)                         */
  FISDF_ST_WS = 10,    /* W_s = Re(Phi W) sqrt(nk) (fftisdf.py:204-207)           */
  FISDF_ST_AO = 11,    /* Bloch AO values (input layer, fftisdf.py:72,367-370)    */
  FISDF_NSTAGES = 12
};

/* ---- context / memory ---------------------------------------------------- */
int fisdf_abi_version(void);
int fisdf_create(int device, void* hip_stream /* NULL: default (null) stream */, fisdf_ctx** out);
int fisdf_destroy(fisdf_ctx* ctx);
const char* fisdf_last_error(const fisdf_ctx* ctx /* NULL: the calling thread's last failure */);
int fisdf_sync(fisdf_ctx* ctx);
int fisdf_malloc(fisdf_ctx* ctx, size_t bytes, void** d_ptr);
int fisdf_free(fisdf_ctx* ctx, void* d_ptr);
int fisdf_memcpy_htod(fisdf_ctx* ctx, void* d_dst, const void* h_src, size_t bytes); /* synchronous */
int fisdf_memcpy_dtoh(fisdf_ctx* ctx, void* h_dst, const void* d_src, size_t bytes); /* synchronous */
int fisdf_set_timing(fisdf_ctx* ctx, int enable);
int fisdf_timings(fisdf_ctx* ctx, double* h_ms /* FISDF_NSTAGES */, int* h_calls); /* synchronous; resets */
/* reality invariants, max |Im| seen since the last call: [0] x2_s (fftisdf.py:43),
 * [1] fx_s (fftisdf.py:81), [2] rho_s (fftisdf.py:216).  synchronous; resets. */
int fisdf_max_imag(fisdf_ctx* ctx, double* h_out /* 3 */);

/* ---- composite entries: the whole 1-GPU build and get_jk ----------------
 * Replace InterpolativeSeparableDensityFitting.build() + get_jk() (fftisdf.py:308-325, 22-128,
 * 390-408): selection (:357-388), x4 (:38-48), y (:67-87), per-q fit + FFT Coulomb (:97-121),
 * W_s (:204-207) in one call, the results left resident on the device for fisdf_get_jk. */
typedef struct fisdf_build_opts {
  int nip_max;             /* cap on interpolation points, int(nao * c0) (fftisdf.py:383); <= 0: ng0 */
  double select_tol;       /* dpstrf tolerance of the selection; <= 0: ng0 * eps * max diag */
  const int* perm;         /* host, n_perm parent-grid indices: use these points, no selection */
  int n_perm;              /*   (ISDF.set_interpolation_points / a refit on the same points)     */
  int fit_mode;            /* FISDF_FIT_LSTSQ (gelsy semantics, default), _SVD, _BASIC */
  double fit_tol;          /* relative pivot cut of the x4_q factorisation (4.2e-15: gelsy's rank
                              decision at rcond = eps, fftisdf.py:108) */
  int pivoted_fit;         /* -1 default (fisdf_set_pivoted_fit), 0, 1 */
  int half_grid;           /* -1 default (fisdf_set_half_grid), 0, 1 */
  int time_reversal;       /* 1: fit one q of each (q, -q) pair, W_{-q} = conj(W_q) (default);
                              the build checks x0_{-k} = conj(x0_k), f_{-k} = conj(f_k) on the device
                              (relative 1e-9) and fits every q when they do not hold */
  int real_self_conjugate; /* 1: q with 2 k_q in the reciprocal lattice fitted in real arithmetic */
  double omega;            /* Coulomb kernel (fisdf_set_omega); 0 = 1/r */
} fisdf_build_opts;
void fisdf_build_opts_default(fisdf_build_opts* opts);

/* The build.  d_x0 (nk, ng0, nao) c128: Bloch AOs on the parent grid (:367-370); d_f (nk,
 * ngrid, nao): Bloch AOs on the FFT grid (:72); kmesh, mesh, a: k-mesh, FFT mesh, lattice rows
 * (bohr); opts may be NULL (defaults).  *h_nip = interpolation points.  Synchronous (returns
 * with the device work enqueued; the host waits only where the stages read ranks back).
 * Replaces the previous build's results; its buffers are released first. */
int fisdf_build(fisdf_ctx* ctx, const void* d_x0, int ng0, const void* d_f, int nao,
                const int kmesh[3], const int mesh[3], const double a[9],
                const fisdf_build_opts* opts, int* h_nip);
/* 1 in *h_streamed if the last fisdf_build formed y (:67-87) behind the selection: its fused y
 * kernel started on the first pivots the cooperative selection kernel published, on a second
 * stream, instead of after the selection (the selection's own points, time reversal, a k-mesh the
 * fused kernel covers; environment FISDF_Y_STREAM=0, read per build, turns it off).  The y,
 * hence every result, is the same either way. */
int fisdf_build_y_streamed(fisdf_ctx* ctx, int* h_streamed);
/* The same streamed y for a caller that drives the stages itself (the k-sharded mirror, one
 * process per GPU).  arm, before fisdf_select_points(_km) / fisdf_select_pivots: the arguments of
 * fisdf_build_y_qs (d_f at the first grid point of the m-point block, k stride f_kstride; y_q of
 * the ascending q-list h_qs into d_yT[slot][I][g], slot stride nip_max * m) with the point cap
 * nip_max in place of nip and d_x0 (nk, ng0, nao) in place of X; time reversal must be on
 * (fisdf_set_time_reversal) and the k-mesh one the fused y kernel covers, else *h_armed = 0 and
 * nothing streams.  The next selection then forms y on a second stream as its pivots appear.
 * finish, after the selection, with the nip it returned: *h_streamed = 1 if d_yT holds
 * fisdf_build_y_qs's result for those points (the caller skips it), 0 if not (the caller builds
 * y as usual, e.g. the selection stopped below the cap); either way the context stream is
 * ordered after the y stream.  Not synchronous for the device; finish waits for the y stream's
 * host-visible completion flag. */
int fisdf_y_stream_arm(fisdf_ctx* ctx, const void* d_x0, int ng0, const void* d_f, long f_kstride,
                       int m, int nao, int nip_max, const int kmesh[3], const int* h_qs, int nq,
                       void* d_yT, int* h_armed);
int fisdf_y_stream_finish(fisdf_ctx* ctx, int nip, int* h_streamed);

/* What the last build left resident.  Pointers stay valid until the next fisdf_build,
 * fisdf_build_release or fisdf_destroy on the context.  fisdf_build restores the context's stage
 * settings (time reversal, fit mode, pivoted fit, half grid, omega, factor priority) on return. */
typedef struct fisdf_build_result {
  int nk, nip, nao, nfit;     /* k-points, interpolation points, AOs, fitted q */
  int used_pivoted_fit;       /* 1: some x4_q needed the pivoted (rank-revealing) factorisation */
  int min_norm_slots;         /* q fitted through the minimum-norm operator */
  const int* perm;            /* host (nip): the interpolation points, parent-grid indices */
  const int* fit_qs;          /* host (nfit): fitted q, ascending (W_q slot i <-> q = fit_qs[i]) */
  const int* ranks;           /* host (nfit): numerical rank of each fitted x4_q (:122) */
  const int* partner;         /* host (nk): index of -q; W_q = conj(W_{partner[q]}) if not fitted */
  const void* d_X;            /* (nk, nip, nao) c128: x0 at the points (fftisdf.py:125, _x) */
  const void* d_x4;           /* (nk, nip, nip) c128 */
  const void* d_Wq;           /* (nfit, nip, nip) c128 */
  const void* d_Ws;           /* (nk, nip, nip) float64: W_s = Re(...) (fftisdf.py:207) */
  int time_reversal;          /* 1: one q of each (q, -q) pair fitted, W_{-q} = conj(W_q); 0: every
                                 q fitted (asked for, or the inputs failed the check below) */
  double tr_deviation;        /* max |a[-k] - conj(a[k])| / max |a| over x0 and f (0 unchecked) */
  /* k-sharded build (fisdf_build_sharded): this rank's share.  nfit / fit_qs / ranks / d_Wq are
   * the rank's own q; d_Ws holds only interpolation-point rows [row0, row1) of every W_s[R],
   * (nk, row1 - row0, nip) float64; d_W0 is W_0 (broadcast from its owner).  One GPU: rank 0 of
   * 1, rows [0, nip), d_W0 = slot 0 of d_Wq. */
  int shard_rank, shard_size;
  int row0, row1;
  const void* d_W0;           /* (nip, nip) c128 */
} fisdf_build_result;
int fisdf_build_get(fisdf_ctx* ctx, fisdf_build_result* out);
/* Time-reversal check of Bloch AO values d_a[k][per_k] (k stride k_stride elements, get_kpts
 * order over kmesh): h_out[0] = max |a[-k] - conj(a[k])| (2 |Im a| on a self-paired k), h_out[1] =
 * max |a|.  What the fold over k <= -k relies on (fisdf_set_time_reversal).  synchronous. */
int fisdf_check_time_reversal(fisdf_ctx* ctx, const void* d_a, long k_stride, long per_k,
                              const int kmesh[3], double* h_out);
int fisdf_build_release(fisdf_ctx* ctx);

/* ---- k-sharded composite build over several GPUs -----------------------------
 * One process (or thread) per GPU, each with its own context, all calling fisdf_build_sharded
 * with the same inputs and options (the Python mirror's torch.distributed build, fisdf/isdf.py
 * build(), in C).  The fitted q are shared by cost, longest first (a self-conjugate q 0.6 of a
 * complex one); the selection and x4 are replicated (identical pivots on every rank, no
 * collective); y is built on the rank's plane-aligned grid slice for every fitted q and
 * exchanged with one all-to-all per local q (each q's fit starts when its piece has landed);
 * W_s row blocks are reduce-scattered; W_0 is broadcast from the rank fitting q = 0.  W_q of a
 * rank equals the 1-GPU build's bit for bit.  fisdf_get_jk on a sharded build contracts the
 * rank's interpolation-point rows and all-reduces J and K (every rank gets the whole result).
 *
 * The collectives come from the caller (MPI, RCCL, a framework's process group) through
 * fisdf_comm; each is enqueued stream-ordered on `stream` (a hipStream_t): it may return before
 * the transfer is done, as long as work enqueued on `stream` afterwards sees the result.  Device
 * pointers throughout; zero-byte entries are allowed.  Return 0, or non-zero on failure. */
typedef struct fisdf_comm {
  int rank, size;
  void* user;
  /* send d_send[r] (send_bytes[r]) to rank r and receive d_recv[r] (recv_bytes[r]) from rank r,
   * for every r (self included) */
  int (*all_to_all)(void* user, const void* const* d_send, const size_t* send_bytes,
                    void* const* d_recv, const size_t* recv_bytes, void* stream);
  /* d_recv[i] = sum over ranks of d_send[rank * count + i], i < count */
  int (*reduce_scatter_f64)(void* user, const double* d_send, double* d_recv, size_t count,
                            void* stream);
  /* in place: d_buf[i] = sum over ranks of d_buf[i] */
  int (*allreduce_f64)(void* user, double* d_buf, size_t count, void* stream);
  /* in place: d_buf of rank `root` to every rank */
  int (*broadcast)(void* user, void* d_buf, size_t bytes, int root, void* stream);
} fisdf_comm;
/* The build of one rank.  `comm` must stay valid while the build's results are used
 * (fisdf_get_jk all-reduces through it).  Arguments otherwise as fisdf_build. */
int fisdf_build_sharded(fisdf_ctx* ctx, const fisdf_comm* comm, const void* d_x0, int ng0,
                        const void* d_f, int nao, const int kmesh[3], const int mesh[3],
                        const double a[9], const fisdf_build_opts* opts, int* h_nip);
/* A fisdf_comm over RCCL (librccl, loaded at run time): rank 0 makes the id, the caller hands it
 * to every rank (MPI_Bcast, a file, a TCP store), each rank then joins on its own GPU.  The
 * collectives run on the stream they are given, over xGMI within a node. */
#define FISDF_COMM_ID_BYTES 128
int fisdf_comm_rccl_unique_id(unsigned char h_id[FISDF_COMM_ID_BYTES]);
int fisdf_comm_rccl_init(const unsigned char h_id[FISDF_COMM_ID_BYTES], int rank, int size,
                         int device, fisdf_comm* out);
int fisdf_comm_rccl_destroy(fisdf_comm* comm);

/* ---- one process, several GPUs (SURVEY §8(b)'s fisdf_create(ndev, dev_ids)) -----------------
 * A group of n ranks, rank r on devices[r] with a context and a stream of its own, joined by
 * RCCL (FISDF_GROUP_RCCL: distinct devices) or by device copies between the ranks' buffers
 * (FISDF_GROUP_COPY: any devices, a device may repeat).  fisdf_group_build / _get_jk run
 * fisdf_build_sharded / fisdf_get_jk on every rank at once, one host thread per rank; the per-rank
 * arrays hold each rank's device pointers (the same AO values on every rank).  Results: through
 * fisdf_group_ctx(g, r) and the single-rank entries (fisdf_build_get, ...); every rank's J/K are
 * the full, all-reduced matrices.  On failure the message is fisdf_group_last_error(g). */
#define FISDF_GROUP_COPY 0
#define FISDF_GROUP_RCCL 1
typedef struct fisdf_group fisdf_group;
int fisdf_group_create(int n, const int* devices, int kind, fisdf_group** out);
int fisdf_group_destroy(fisdf_group* g);
fisdf_ctx* fisdf_group_ctx(fisdf_group* g, int rank);
const char* fisdf_group_last_error(fisdf_group* g);
int fisdf_group_build(fisdf_group* g, const void* const* d_x0, int ng0, const void* const* d_f,
                      int nao, const int kmesh[3], const int mesh[3], const double a[9],
                      const fisdf_build_opts* opts, int* h_nip);
int fisdf_group_get_jk(fisdf_group* g, const void* const* d_dms, int nset, int with_j,
                       int with_k, void* const* d_vj, void* const* d_vk);

/* Host copies of the reference's attributes (fftisdf.py:125-128): h_x (nk, nip, nao) = _x,
 * h_w0 (nip, nip) = _w0, h_wq (nk, nip, nip) = _wq (unfitted q filled as conj(W_{-q}); not on a
 * sharded build of several ranks, whose W_q are distributed: fisdf_build_get per rank).
 * synchronous. */
int fisdf_get_x(fisdf_ctx* ctx, void* h_x);
int fisdf_get_w0(fisdf_ctx* ctx, void* h_w0);
int fisdf_get_wq(fisdf_ctx* ctx, void* h_wq);

/* get_jk of the last build (fftisdf.py:390-408 -> get_k_kpts :173-228, then get_j_kpts
 * :133-171): d_dms (nset, nk, nao, nao) c128 device; d_vj / d_vk same shape (either may be NULL
 * when with_j / with_k is 0).  J is complex: a Gamma-only caller takes .real (:169-170).
 * After fisdf_build_sharded every rank calls it with the same d_dms: each contracts its own
 * interpolation-point rows and J / K are all-reduced through the build's fisdf_comm.
 * asynchronous. */
int fisdf_get_jk(fisdf_ctx* ctx, const void* d_dms, int nset, int with_j, int with_k, void* d_vj,
                 void* d_vk);

/* Device memory of the composite build's buffers (X, x4, y, W_q, W_s) from the caller, e.g. a
 * framework's caching allocator; alloc(NULL-safe) returns a device pointer of >= bytes or NULL.
 * The library returns each buffer through free_fn once it no longer uses it — the y buffer right
 * after the fit is enqueued, so free_fn must be stream-ordered on the context's stream (like
 * hipFreeAsync / a caching allocator bound to that stream); the rest at the next build or
 * fisdf_build_release (not at fisdf_destroy: the caller owns what it allocated).  NULL: library-
 * owned buffers, kept between builds of the same size (fisdf_build_release frees them). */
typedef void* (*fisdf_alloc_fn)(size_t bytes, void* user);
typedef void (*fisdf_free_fn)(void* d_ptr, void* user);
int fisdf_set_allocator(fisdf_ctx* ctx, fisdf_alloc_fn alloc, fisdf_free_fn release, void* user);

/* ---- input layer: Bloch AO values ------------------------
 * Replaces PySCF pbc_eval_gto('GTOval', coords, kpts) / KNumInt.block_loop as called at
 * fftisdf.py:72,327-355,367-370 (restated on the host by fisdf/cell.py eval_ao_kpts):
 *   chi_k(r_g)[nu] = sum_{T = n.a} exp(i k.T) phi_nu(r_g - T)
 * for contracted real-spherical Gaussian shells (l <= 3, cell.py's harmonics and order).
 * d_coords (ng, 3) f64 device; h_atoms (natm, 3); shells: atom, l, nprim, then the nprim
 * exponents / normalised coefficients of each shell in order; h_tn (nT, 3) the lattice
 * translations n to sum (T = n @ a, image R = n mod kmesh); terms with |r - T - atom| >= rcut
 * are dropped.  d_out (nk, ng, nao) c128, nk = prod(kmesh), kpts = make_kpts order. */
int fisdf_eval_ao(fisdf_ctx* ctx, const void* d_coords, int ng, int natm, const double* h_atoms,
                  int nsh, const int* h_sh_atom, const int* h_sh_l, const int* h_sh_nprim,
                  const double* h_exps, const double* h_coefs, int nT, const int* h_tn,
                  const int kmesh[3], const double a[9], double rcut, int nao, void* d_out);

/* Same Bloch AO values at nkb arbitrary (band) k-points h_kpts (nkb, 3), cartesian 1/bohr —
 * the AOs at the interpolation points that get_jk(kpts_band=...) contracts.  d_out (nkb, ng, nao). */
int fisdf_eval_ao_band(fisdf_ctx* ctx, const void* d_coords, int ng, int natm, const double* h_atoms,
                       int nsh, const int* h_sh_atom, const int* h_sh_l, const int* h_sh_nprim,
                       const double* h_exps, const double* h_coefs, int nT, const int* h_tn,
                       int nkb, const double* h_kpts, const double a[9], double rcut, int nao,
                       void* d_out);

/* ---- A1: interpolation-point selection ------------------------------------
 * Replaces InterpolativeSeparableDensityFitting.select_interpolation_points
 * (fftisdf.py:357-388): x2 = sum_q Re(x0_q^* x0_q^T); x4 = x2*x2/nk; greedy pivoted
 * Cholesky of x4 (LAPACK dpstrf semantics, tol <= 0 -> ng0*eps*max(diag)).
 * Produces the first min(nip_max, rank) pivots.  synchronous.
 *   d_x0 (nk, ng0, nao) c128;  h_perm (nip_max) int;  *h_npiv = pivots produced;
 *   *h_full_rank = 1 if the tolerance (not nip_max) stopped the factorisation. */
int fisdf_select_points(fisdf_ctx* ctx, const void* d_x0, int nk, int ng0, int nao, int nip_max,
                        double tol, int* h_perm, int* h_npiv, int* h_full_rank);
/* The same for a k-mesh (x0 in get_kpts order over kmesh[0]*kmesh[1]*kmesh[2] k-points): with
 * fisdf_set_time_reversal on (real AOs, x0_{-k} = conj(x0_k)) the Gram sums the representatives
 * k <= -k only, a paired one counted twice (36 of 64 k at 4x4x4). */
int fisdf_select_points_km(fisdf_ctx* ctx, const void* d_x0, const int kmesh[3], int ng0, int nao,
                           int nip_max, double tol, int* h_perm, int* h_npiv, int* h_full_rank);

/* The two halves of fisdf_select_points, for a k-point-sharded selection:
 * fisdf_select_gram: d_x2 (ng0, ng0) c128 = Re(sum_{q in [q0,q1)} x0_q x0_q^H) + 0i (the real
 *   part is fftisdf.py:376-378's x2, the only part :379 uses; shards are summed with an
 *   all-reduce);
 * fisdf_select_pivots: x4 = Re(x2)^2/nk and the greedy pivoted Cholesky (fftisdf.py:379-384);
 *   synchronous. */
int fisdf_select_gram(fisdf_ctx* ctx, const void* d_x0, int nk, int q0, int q1, int ng0, int nao,
                      void* d_x2);
int fisdf_select_pivots(fisdf_ctx* ctx, const void* d_x2, int nk, int ng0, int nip_max, double tol,
                        int* h_perm, int* h_npiv, int* h_full_rank);

/* Reassemble a k-shard's y after the grid-slice all-to-all: d_recv holds, for p = 0..nparts-1,
 * a (nrows, h_ng[p]) block of grid points [h_g0[p], h_g0[p]+h_ng[p]); d_yT is (nrows, ngrid). */
int fisdf_unpack_slices(fisdf_ctx* ctx, const void* d_recv, int nrows, int nparts,
                        const long* h_g0, const long* h_ng, long ngrid, void* d_yT);

/* X[k, I, :] = x0[k, perm[I], :]  (fftisdf.py:388) */
int fisdf_gather_points(fisdf_ctx* ctx, const void* d_x0, int nk, int ng0, int nao,
                        const int* h_perm, int nip, void* d_X);

/* ---- A2: x4_k = Phi^H ((Phi x2_k)^2), x2_k = X_k^* X_k^T  (fftisdf.py:38-48) ----
 *   d_X (nk, nip, nao); d_x4 (nk, nip, nip); a: lattice (3x3 rows, bohr) */
int fisdf_build_x4(fisdf_ctx* ctx, const void* d_X, int nip, int nao, const int kmesh[3],
                   const double a[9], void* d_x4);

/* ---- A3: y build for one grid block (fftisdf.py:67-87) ---------------------
 * d_f: Bloch AOs of the block, element (k, g, m) at d_f[k*f_kstride + g*nao + m],
 * g in [0, nblk); writes y_q, q in [q0, q1) (a k-point shard), for grid points
 * [g0, g0+nblk) into the library's transposed layout d_yT[q-q0][I][g]
 * (q1-q0, nip, ngrid). */
int fisdf_build_y(fisdf_ctx* ctx, const void* d_f, long f_kstride, int g0, int nblk, int ngrid,
                  const void* d_X, int nip, int nao, const int kmesh[3], const double a[9],
                  int q0, int q1, void* d_yT);

/* Same for an explicit ascending q-list h_qs[0..nq) (e.g. the time-reversal representatives
 * of this rank, see fisdf_fit_coulomb_qs): y_q is written to d_yT[i] for q = h_qs[i]. */
int fisdf_build_y_qs(fisdf_ctx* ctx, const void* d_f, long f_kstride, int g0, int nblk, int ngrid,
                     const void* d_X, int nip, int nao, const int kmesh[3], const double a[9],
                     const int* h_qs, int nq, void* d_yT);

/* ---- A4: per-q factorisation of x4_q, q in [q0, q1) (replaces zgelsy's QRCP,
 * fftisdf.py:108).  Pivoted Cholesky with rank cut tol_rel*max(diag); factors stay in
 * the context.  d_x4: (nk, nip, nip) (all q).  synchronous: h_ranks (q1-q0) receives
 * the numerical ranks (logged at fftisdf.py:122). */
int fisdf_factor_x4(fisdf_ctx* ctx, const void* d_x4, int q0, int q1, int nip, double tol_rel,
                    int* h_ranks);
/* q-list form: factors x4_q for q = h_qs[i] (ascending); h_ranks (nq).  kmesh (may be NULL):
 * q that are their own time-reversal partner (2 k_q a reciprocal-lattice vector) have real
 * x4_q, y_q, z_q and W_q; with kmesh given they are factored as real and fitted with real-
 * factor / real-part GEMMs (half the MFMA work). */
int fisdf_factor_x4_qs(fisdf_ctx* ctx, const void* d_x4, const int* h_qs, int nq, int nip,
                       double tol_rel, const int* kmesh, int* h_ranks);
/* Asynchronous form: enqueues the factorisation on the context's side stream (after the work
 * already enqueued on the main stream, i.e. x4) and returns at once, so the y build enqueued
 * next overlaps it.  fisdf_factor_x4_wait (synchronous on the side stream) returns the ranks;
 * fisdf_fit_coulomb_qs waits by itself. */
int fisdf_factor_x4_async(fisdf_ctx* ctx, const void* d_x4, const int* h_qs, int nq, int nip,
                          double tol_rel, const int* kmesh);
int fisdf_factor_x4_wait(fisdf_ctx* ctx, int* h_ranks /* nq, may be NULL */);
/* Record the point on the main stream (x4 built) the next fisdf_factor_x4_async starts from, so
 * that the y build can be enqueued between the two calls: the factorisation reads its ranks back
 * to the host mid-chain, which can block the enqueueing thread until the side stream gets there. */
int fisdf_factor_x4_mark(fisdf_ctx* ctx);
/* Factorisation path.  Default (mode -1: unless FISDF_PIVOTED_FIT=1 in the environment): an
 * unpivoted blocked Cholesky, kept when every pivot exceeds tol_rel * max(diag) (the full-rank
 * verdict of the rank-revealing factorisation) and otherwise redone — for the whole batch —
 * by the greedy pivoted Cholesky; mode 1 forces the pivoted one, mode 0 the default.
 * fisdf_factor_info: 1 if the last factorisation used the pivoted path. */
int fisdf_set_pivoted_fit(fisdf_ctx* ctx, int mode);
int fisdf_factor_info(fisdf_ctx* ctx, int* h_used_pivoted);
/* Solution the fit applies (replaces scipy lstsq/gelsy, fftisdf.py:108, and the SVD
 * pseudo-solve of fftdf-with-k-svd.py:158-164):
 *  FISDF_FIT_LSTSQ (default): gelsy's semantics — the unique solution of a full-rank x4_q
 *    (blocked Cholesky, TRSM-first factored order) and, when the rank-revealing factor finds
 *    rank r < nip, the MINIMUM-NORM solution z = x4_r^+ y: A = P L (nip x r), thin QR A = Q R
 *    (shifted CholeskyQR3 on the device), z[P] = M^H M y[P] with M = A^+ = R^{-1} Q^H — the
 *    complete orthogonal step gelsy takes after its QRCP;
 *  FISDF_FIT_SVD: the truncated pseudo-solve on every q (rank-revealing factor with the
 *    relative cut tol_rel, then the same minimum-norm operator), the "SVD fit" configuration;
 *  FISDF_FIT_BASIC: the basic solution z[P1] = L11^-H L11^-1 y[P1] (round-1 behaviour).
 * fisdf_min_norm_info: number of q of the last factorisation fitted through M. */
#define FISDF_FIT_LSTSQ 0
#define FISDF_FIT_SVD 1
#define FISDF_FIT_BASIC 2
int fisdf_set_fit_mode(fisdf_ctx* ctx, int mode);
/* A self-conjugate q (real z_q: Zhat(G') = conj(Zhat(G)), G' = -G - 2 k_q) is fitted on half the
 * grid — one member of each pair G, G' with the pair's combined Coulomb weight, the asymmetric
 * pairs' Im(W) from a signed-weight GEMM — so its TRSM and HERK run over ~N/2 columns.
 * mode -1: environment FISDF_HALF_G (default on), 0 off (full grid), 1 on. */
int fisdf_set_half_grid(fisdf_ctx* ctx, int mode);
int fisdf_min_norm_info(fisdf_ctx* ctx, int* h_nslots);

/* ---- A4+A5: fit + FFT Coulomb for the factored shard q in [q0, q1) (fftisdf.py:97-121)
 * Needs fisdf_factor_x4 on the same range.  W_q = zeta_q z_q^H computed as
 * (vol/N^2) Zhat diag(coulG(k_q+G)) Zhat^H with Zhat = FFT(z_q * f_q), the
 * fit applied in factored order.  d_yT: (q1-q0, nip, ngrid) from fisdf_build_y;
 * d_Wq: (q1-q0, nip, nip). */
int fisdf_fit_coulomb(fisdf_ctx* ctx, int q0, int q1, const void* d_yT, int nip,
                      const int mesh[3], const int kmesh[3], const double a[9], void* d_Wq);
/* q-list form (the list given to fisdf_factor_x4_qs).  Time reversal: y_s and x4_s are real
 * (fftisdf.py:43,81), so y_{-q} = conj(y_q), x4_{-q} = conj(x4_q) and W_{-q} = conj(W_q);
 * callers may fit only one q of each (q, -q) pair and weight it 2 in fisdf_build_ws_qs. */
int fisdf_fit_coulomb_qs(fisdf_ctx* ctx, const int* h_qs, int nq, const void* d_yT, int nip,
                         const int mesh[3], const int kmesh[3], const double a[9], void* d_Wq);
/* Fit lanes: the q of one fisdf_fit_coulomb_qs call are spread round-robin over `lanes`
 * streams with private workspaces (one q's memory-bound FFT/HERK overlaps another's
 * MFMA-bound TRSM); 0 (default): FISDF_FIT_LANES from the environment, else 2.  Results do
 * not depend on it (same kernels, same per-q arithmetic). */
int fisdf_set_fit_lanes(fisdf_ctx* ctx, int lanes);
/* Stream priority of the x4_q factorisation chain (fisdf_factor_x4_async): 0 (default) = the
 * device's least priority (the 1-GPU build, where the chain hides behind the y build), 1 = the
 * greatest (a k-shard, whose 1/N-grid y build leaves the chain on the critical path). */
int fisdf_set_factor_priority(fisdf_ctx* ctx, int high);
/* Pipelined FFT stream of the fit (with >= 2 lanes): mode -1 = FISDF_FIT_PIPE from the
 * environment (default on), 0 off (the FFT runs in its lane), 1 on; the FFTs run ahead of the
 * lanes into a ring of `depth` Yhat slots (0: FISDF_PIPE_DEPTH or lanes + 2), i.e.
 * depth x rank x ngrid complex of workspace (C3: 448 MB per slot), whatever the number of q.
 * Falls back to the in-lane FFT when the device lacks the memory.  Results do not depend on it. */
int fisdf_set_fit_pipe(fisdf_ctx* ctx, int mode, int depth);
/* What the last fisdf_fit_coulomb_qs ran with: MFMA lanes and ring depth (0 = not pipelined). */
int fisdf_fit_info(fisdf_ctx* ctx, int* h_lanes, int* h_pipe_depth);
/* Sharded build: record, on the context's stream, that y of the j-th q of the NEXT
 * fisdf_fit_coulomb_qs call has landed in d_yT (after its all-to-all piece is unpacked).  When
 * every q of that call is marked, the call runs its lanes on side streams and starts each q's
 * FFT as soon as its own piece is there (one call for the whole shard keeps the lanes and the
 * pipelined FFT stream; replaces one call per q).  Marks are consumed by the call. */
int fisdf_mark_y_ready(fisdf_ctx* ctx, int j);
/* The same, with the j-th q's y read IN PLACE from its all-to-all piece d_recv (replaces
 * fisdf_unpack_slices + fisdf_mark_y_ready): d_recv holds, for p = 0..nparts-1, the (nip,
 * h_ng[p]) block of grid points [h_g0[p], h_g0[p] + h_ng[p]), whole planes of the mesh; the fit's
 * FFT reads each plane where it lies.  Every piece of one call has the same layout; d_yT of that
 * call may then be NULL.  The piece must stay alive until the call's work is done. */
int fisdf_set_y_slices(fisdf_ctx* ctx, int j, const void* d_recv, int nparts, const long* h_g0,
                       const long* h_ng);
/* Grow the context's scratch arena to at least `bytes` now (pre-allocation; a failed growth
 * leaves an empty arena, never a stale one). */
int fisdf_reserve_workspace(fisdf_ctx* ctx, size_t bytes);
/* Coulomb kernel of the fit (and of fisdf_coulg): 0 = 1/r (default, fftisdf.py:114); omega > 0 the
 * long-range erf(omega r)/r, omega < 0 the short-range erfc(|omega| r)/r (PySCF get_coulG's
 * omega; the reference's get_jk raises for omega, fftisdf.py:392-393). */
int fisdf_set_omega(fisdf_ctx* ctx, double omega);
/* Time reversal of the inputs (real AOs, k-mesh closed under k -> -k): f_{-k} = conj(f_k)
 * and x_{-k} = conj(x_k), so fx_{-k} = conj(fx_k) (fftisdf.py:76) and fisdf_build_y(_qs)
 * computes fx_k only for the k-planes a <= kmesh[0]/2.  Default 0 (every k computed). */
int fisdf_set_time_reversal(fisdf_ctx* ctx, int on);

/* ---- A8 prep: W_s[R] = sqrt(nk) Re(sum_{q in [q0,q1)} Phi[R,q] W_q) (fftisdf.py:204-207)
 * d_Wq: (q1-q0, nip, nip) shard; d_Ws: (nimg, nip, nip) REAL float64 (the reference keeps
 * W_s = ws.real, :207; a partial sum for a q-shard, summed over the shards). */
int fisdf_build_ws(fisdf_ctx* ctx, const void* d_Wq, int q0, int q1, int nip,
                   const int kmesh[3], const double a[9], void* d_Ws);
/* q-list form: W_s[R] = sqrt(nk) Re(sum_i h_wt[i] Phi[R,q_i] W_{q_i}) (h_wt NULL: all 1;
 * 2 for a time-reversal representative whose partner -q is not listed).  synchronous. */
int fisdf_build_ws_qs(fisdf_ctx* ctx, const void* d_Wq, const int* h_qs, const double* h_wt,
                      int nq, int nip, const int kmesh[3], const double a[9], void* d_Ws);

/* Row block [i0, i1) of W_s for a q-list: d_Ws (nk, i1-i0, nip) float64 = rows i0..i1 of every W_s[R] of
 * fisdf_build_ws_qs.  A k-sharded build forms every rank's block of its partial sum and
 * REDUCE-SCATTERS them (each rank then holds the rows its get_k contracts, half the bytes of the
 * all-reduce of the whole W_s).  asynchronous. */
int fisdf_build_ws_rows(fisdf_ctx* ctx, const void* d_Wq, const int* h_qs, const double* h_wt,
                        int nq, int nip, const int kmesh[3], const double a[9], int i0, int i1,
                        void* d_Ws);
/* Every rank's row block in one call (the reduce-scatter input): block b = rows
 * [h_rows[b], h_rows[b+1]) written as (nk, rows, nip) float64 at d_Wsb + b * chunk doubles.
 * asynchronous. */
int fisdf_build_ws_blocks(fisdf_ctx* ctx, const void* d_Wq, const int* h_qs, const double* h_wt,
                          int nq, int nip, const int kmesh[3], const double a[9], int nblk,
                          const int* h_rows, long chunk, void* d_Wsb);

/* ---- A7: get_j_kpts (fftisdf.py:133-171) ------------------------------------
 * d_dms (nset, nk, nao, nao); d_vj same shape (complex; caller takes .real for Gamma). */
int fisdf_get_j(fisdf_ctx* ctx, const void* d_X, const void* d_W0, const void* d_dms, int nset,
                int nk, int nip, int nao, void* d_vj);

/* ---- A8: get_k_kpts (fftisdf.py:173-228) ------------------------------------ */
int fisdf_get_k(fisdf_ctx* ctx, const void* d_X, const void* d_Ws, const void* d_dms, int nset,
                int nip, int nao, const int kmesh[3], const double a[9], void* d_vk);

/* Row-block forms: the contribution of the interpolation points I in [i0, i1) to J / K
 * (J_k = sum_I X_k[I]^H v_I X_k[I], K_k = sum_I X_k[I]^H (V_k[I,:] X_k)); the full result is
 * the sum over a partition of [0, nip) — a sharded caller all-reduces nset*nk*nao^2 values.
 * fisdf_get_j / fisdf_get_k are the [0, nip) cases. */
int fisdf_get_j_rows(fisdf_ctx* ctx, const void* d_X, const void* d_W0, const void* d_dms,
                     int nset, int nk, int nip, int nao, int i0, int i1, void* d_vj);
int fisdf_get_k_rows(fisdf_ctx* ctx, const void* d_X, const void* d_Ws, const void* d_dms,
                     int nset, int nip, int nao, const int kmesh[3], const double a[9], int i0,
                     int i1, void* d_vk);
/* the same with only this block's W_s rows at hand: d_Ws_rows (nk, i1-i0, nip) float64.  d_Ws
 * of fisdf_get_k / fisdf_get_k_rows is the real (nk, nip, nip) array of fisdf_build_ws_qs. */
int fisdf_get_k_rows_local(fisdf_ctx* ctx, const void* d_X, const void* d_Ws_rows,
                           const void* d_dms, int nset, int nip, int nao, const int kmesh[3],
                           const double a[9], int i0, int i1, void* d_vk);
/* J at band k-points (get_jk kpts_band; the reference asserts nband == nkpt, fftisdf.py:164):
 * rho and v = W0 rho from the k-mesh dms as fisdf_get_j, then J_k' = Xb_k'^H diag(v) Xb_k' with
 * d_Xb (nkb, nip, nao) the AOs at the interpolation points for the band k-points (the q = 0 pair
 * fit serves any k' on both sides).  d_vj (nset, nkb, nao, nao); rows [i0, i1) as above. */
int fisdf_get_j_band_rows(fisdf_ctx* ctx, const void* d_X, const void* d_W0, const void* d_dms,
                          int nset, int nk, int nip, int nao, const void* d_Xb, int nkb, int i0,
                          int i1, void* d_vj);

/* ---- ISDF 4-index integrals (get_eri / ao2mo surface) --------------------------
 * eri[i*n2+j][k*n4+l] = sum_IJ W_q[I,J] conj(A1[I,i]) A2[I,j] conj(A3[J,k]) A4[J,l] with
 * A_s = X_{kidx[s]} C_s, q = k2 - k1 (fftdf-with-k-lstsq.py:221-232).  d_Wq: the (nip,nip)
 * W of that q; h_dC: host array of 4 DEVICE pointers to (nao, nmo[s]) MO coefficients, or
 * NULL (or NULL entries) for AO integrals.  d_out: (n1*n2, n3*n4) c128. */
int fisdf_get_eri(fisdf_ctx* ctx, const void* d_X, int nip, int nao, const int kidx[4],
                  const void* d_Wq, const void* const* h_dC, const int nmo[4], void* d_out);

/* ---- building blocks exported for tests / other callers -------------------- */
/* C[b] = alpha op(A[b]) op(B[b]) + beta C[b]; op: 0 N, 1 T, 2 conj, 3 conj-transpose */
int fisdf_zgemm(fisdf_ctx* ctx, int opA, int opB, int M, int N, int K, const double alpha[2],
                const void* d_A, long lda, long strideA, const void* d_B, long ldb, long strideB,
                const double beta[2], void* d_C, long ldc, long strideC, int batch, int ksplit);
/* the same with the fit's arithmetic modes (no split-K): 1 = Im op(A) taken as zero, 2 = only
 * Re C formed, 4 = op(A) lower triangular (op N), 8 = op(A) = A^H upper triangular (op C), 5 =
 * 4 | 1; NN products with N >= 512 run on the 64 x 128-tile kernel */
int fisdf_zgemm_mode(fisdf_ctx* ctx, int opA, int opB, int M, int N, int K, const double alpha[2],
                     const void* d_A, long lda, long strideA, const void* d_B, long ldb,
                     long strideB, const double beta[2], void* d_C, long ldc, long strideC,
                     int batch, int mode);
/* C = alpha A A^H (A: n x K, lda; C: n x n, ldc), Hermitian: lower tiles + mirror */
int fisdf_herk(fisdf_ctx* ctx, int n, int K, double alpha, const void* d_A, long lda, void* d_C,
               long ldc, int ksplit);
/* forward 3-D FFT (numpy fftn sign, unnormalised) of `rows` rows of n0*n1*n2 points */
int fisdf_fft3d(fisdf_ctx* ctx, const void* d_in, void* d_out, int rows, const int mesh[3]);
/* the fit's transform of a self-conjugate q: rows pre-multiplied by exp(-i f.kd) (f: fftfreq
 * fractions; kd may be NULL), m (or NULL) = 2 k_q in mesh units: the input is real up to that
 * phase, out(j') = conj(out(j)) for j' = -j - m, and only the prefix planes
 * j0 < #{i0 : i0 <= (-i0 - m0) mod n0} of d_out are written (register meshes; other meshes
 * write every plane).  in_real: d_in holds rows of doubles (same strides), d_in != d_out,
 * register meshes only (an error otherwise) */
int fisdf_fft3d_paired(fisdf_ctx* ctx, const void* d_in, void* d_out, int rows, const int mesh[3],
                       const double kd[3], const int m[3], int in_real);
/* sqrt(coulG(k+G) * scale) (or without sqrt), PySCF get_coulG(exxdiv=None) restated */
int fisdf_coulg(fisdf_ctx* ctx, const int mesh[3], const double a[9], const double k[3],
                double scale, int take_sqrt, double* d_w);
/* minimum-norm operator of one Hermitian PSD n x n matrix (the fit's FISDF_FIT_LSTSQ/SVD path):
 * rank-revealing pivoted Cholesky (cut tol_rel * max diag) then M = (P L)^+ (n x n, rows < rank
 * valid, columns in pivot order h_piv), so x4^+ ~ P M^H M P^T; d_Q (n x rank) and d_Rinv
 * (rank x rank), if not NULL, receive the thin QR factors P L = Q R; synchronous */
int fisdf_min_norm_operator(fisdf_ctx* ctx, const void* d_A, int n, double tol_rel, void* d_M,
                            void* d_Q, void* d_Rinv, int* h_piv /* n */, int* h_rank);
/* batched pivoted Cholesky (pivots + ranks to host; synchronous) */
int fisdf_pivoted_cholesky(fisdf_ctx* ctx, const void* d_A, int n, int batch, int rmax,
                           double tol_rel, int* h_piv /* batch*rmax */, int* h_rank /* batch */);
/* the fit's unpivoted blocked Cholesky of batch Hermitian PD n x n matrices, in place (lower
 * triangle = L on return; 64-column blocks, the diagonal blocks factored and inverted in LDS);
 * h_fail[b] = 1 when a pivot fell below tol_rel * max(diag) (the fit then refactors with
 * pivoting).  synchronous */
int fisdf_cholesky(fisdf_ctx* ctx, void* d_A, int n, int batch, double tol_rel, int* h_fail);
/* L^{-1} of batch lower-triangular n x n matrices by the factor stage's block-row substitution
 * (the operator the fit's triangular GEMM applies); a matrix's result does not depend on the
 * batch it is computed in */
int fisdf_tri_inverse(fisdf_ctx* ctx, const void* d_L, int n, int batch, void* d_Linv);

#ifdef __cplusplus
}
#endif

#endif /* FISDF_H */
