// C-ABI of libfisdf.so (include/fisdf.h): orchestration of the HIP kernels that
// replace the reference's fftisdf.py hot path.  Each entry cites the reference lines
// it stands in for.
#include "../../include/fisdf.h"

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "common.h"
#include "linalg.h"

namespace fisdf {

static thread_local std::string g_last_error;
// the context the calling thread is working on (set by the entry points' guards): a failure is
// recorded in it too, so fisdf_last_error(ctx) reports that context's own last failure.  Only a
// context that is still alive is written (one destroyed on another thread must not
// be), and fisdf_create clears it, so its failures go to fisdf_last_error(NULL) only
static thread_local fisdf_ctx* t_cur_ctx = nullptr;
static std::mutex g_live_mu;
static std::set<const fisdf_ctx*> g_live;
void set_ctx_error(fisdf_ctx* c, const std::string& msg);
void set_error(const std::string& msg) {
  g_last_error = msg;
  if (!t_cur_ctx) return;
  std::lock_guard<std::mutex> lk(g_live_mu);
  if (g_live.count(t_cur_ctx)) set_ctx_error(t_cur_ctx, msg);
}

LaunchEvents& launch_events() {
  static thread_local LaunchEvents ev;
  return ev;
}

}  // namespace fisdf

using namespace fisdf;

// default relative pivot cut of the x4_q factorisation (fisdf_build_opts.fit_tol, the rank of a
// rank-deficient x4_q): 4.2e-15 ~ 19 eps is where the pivoted Cholesky's ranks reproduce gelsy's
// (fftisdf.py:108: QRCP + incremental condition estimate at rcond = eps) in the reference demo's
// regime (C2 at c0 = 1e4, every x4_q rank-deficient): per-q ranks 0-13 from gelsy's, J/K within
// 0.78 / 0.71 of gelsy's own rcond band; the round-4 cut 1e-14 sat 27-37 ranks below it, at
// 1.38 / 0.97 of the band (tests/experiments/rank_rule_c2.py, profiles/r05/rank_regime/)
constexpr double kFitTolDefault = 4.2e-15;

struct fisdf_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  // grow-only scratch arena (sequential use on `stream`)
  void* arena = nullptr;
  size_t arena_size = 0;
  // phase matrices Phi (nimg x nk) keyed by kmesh + lattice
  std::map<std::vector<double>, cplx*> phase_cache;
  // per-q factors of x4_q (fisdf_factor_x4)
  std::vector<int> f_qs;  // the factored q (ascending), slot i <-> q = f_qs[i]
  std::vector<char> f_real;  // slot factored as real (self-conjugate q, kmesh given)
  // per (mesh, lattice, k_q): device list of G with asymmetric Coulomb weight (asym_list)
  struct Asym { int* idx = nullptr; int n = 0; double* f = nullptr; };
  std::map<std::vector<double>, Asym> asym_cache;
  // fisdf_set_half_grid: a self-conjugate q is fitted on half the G (its Hermitian pairs), -1:
  // environment FISDF_HALF_G (default on)
  int half_grid = -1;
  // per (mesh, k-mesh, lattice, q, omega): sqrt(coulG(k_q + G) vol / N^2) of the fit, computed
  // once (the timed steps of a repeated build reuse them)
  std::map<std::vector<double>, double*> wt_cache;
  int f_nk = 0, f_nip = 0, f_nb = 64;
  cplx* f_L = nullptr;      // (nk, nip, nip) raw left-looking factor (row order)
  cplx* f_Lp = nullptr;     // (nk, nip*nip) pivot-order factor, ld = rank_q
  cplx* f_Linv = nullptr;   // (nk, nblk*nb*nb)
  cplx* f_Q = nullptr;      // (nk, nip, nip) block-row operator of trsm_merged_batched (build_trsm_q)
  cplx* f_Li = nullptr;     // (nk, nip, nip) L^{-1} (pivot order) = trsm_merged_batched on the identity
  cplx* f_ksw = nullptr;    // split-K partials of that substitution (trsm_split_work_elems)
  long f_ksw_elems = 0;
  cplx* f_x4s = nullptr;    // (nk, nip, nip) staged x4_q of the factored slots
  int* f_fail_pinned = nullptr;  // unpivoted path: per-slot failure flags (host, pinned)
  int* f_qr_pinned = nullptr;    // factored q-list + real flags (2 nk ints, pinned) and device copy
  int* f_qr_dev = nullptr;
  double f_tol = kFitTolDefault;
  bool f_check_fail = false, f_used_pivoted = false;
  int f_cap_nk = 0, f_cap_nip = 0;  // shape the factor buffers were allocated for
  int force_pivoted = -1;  // fisdf_set_pivoted_fit; -1: environment FISDF_PIVOTED_FIT
  // fisdf_set_fit_mode: FISDF_FIT_LSTSQ (gelsy semantics: the unique solution of a full-rank
  // x4_q, the minimum-norm one of a rank-deficient x4_q), FISDF_FIT_SVD (rank-revealing factor
  // and the minimum-norm operator on every q), FISDF_FIT_BASIC (basic solution, round-1 path)
  int fit_mode = 0;
  cplx* f_M = nullptr;          // (nk, nip, nip) minimum-norm operators A^+ (rows < rank)
  std::vector<char> f_cod;      // slot fitted through its minimum-norm operator
  // the fit's pipelined-FFT ring (Yhat slots, nip rows each), a grow-only buffer of its own
  cplx* f_ring = nullptr;
  size_t f_ring_bytes = 0;
  // grow-only temporaries instead of the stream-ordered pool (hipMallocAsync): on the HIP 7.2
  // runtime a block freed on one stream was handed to another stream's allocation while the
  // first still used it (torch-free C-ABI build: the pivoted factor's ranks corrupted by the
  // Coulomb weights computed beside it on the FFT stream).  ws_main: the main stream's;
  // ws_side_a / ws_side_b: the factorisation's (side stream)
  struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
  } ws_main, ws_side_a, ws_side_b, ws_x4;  // ws_x4: x2_k of an x4 built on the side stream
  int* f_nip_dev = nullptr;     // device copy of nip (scatter of a full W_PP)
  int lanes = 0;           // fisdf_set_fit_lanes; 0: environment FISDF_FIT_LANES / default
  bool time_reversal = false;  // fisdf_set_time_reversal: fx_{-k} = conj(fx_k) in build_y
  double omega = 0.0;          // fisdf_set_omega: range-separated Coulomb kernel of the fit
  // extra streams of the fit lanes (fisdf_fit_coulomb_qs)
  hipStream_t aux[3] = {nullptr, nullptr, nullptr};
  hipEvent_t ev_fork = nullptr, ev_join[3] = {nullptr, nullptr, nullptr};
  // cross-stream ordering of buffers handed back to the caller's allocator: a
  // call that gives aux[i] work bumps aux_use[i]; joining aux[i] into `stream` (aux_join) sets
  // aux_joined[i] = aux_use[i].  build_return asserts every aux stream is joined, so a buffer
  // freed stream-ordered on `stream` has no reader left on another stream
  unsigned aux_use[3] = {0, 0, 0}, aux_joined[3] = {0, 0, 0};
  hipEvent_t ev_ybuf[4] = {nullptr, nullptr, nullptr, nullptr};  // y pipeline: fx ready / free
  std::vector<hipEvent_t> ev_q;  // FISDF_FIT_PIPE: Yhat of fitted q ready (FFT stream)
  std::vector<hipEvent_t> ev_free;  // FISDF_FIT_PIPE: Yhat ring slot read by its lane
  int pipe_mode = -1;   // fisdf_set_fit_pipe; -1: environment FISDF_FIT_PIPE (default on)
  int pipe_depth = 0;   // ring slots; 0: lanes + 2
  int last_fit_lanes = 0, last_fit_pipe = 0;  // what the last fisdf_fit_coulomb_qs ran with
  std::vector<hipEvent_t> ev_ready;  // fisdf_mark_y_ready: y of local q j landed (sharded fit)
  std::vector<char> ready_marked;
  // fisdf_set_y_slices: y of local q j read in place from its all-to-all piece (grid slices)
  std::vector<const cplx*> y_piece;
  // the composite 1-GPU build stores the self-conjugate q's y real (y_real_store, set around
  // its y build and fit); y_real_slot[i]: slot i of the last fisdf_build_y_qs holds doubles
  bool y_real_store = false;
  std::vector<char> y_real_slot;
  std::vector<long> y_slices;  // (g0, ng) pairs of the pieces' layout, shared by every piece
  std::map<std::vector<long>, PlaneRef*> plane_cache;  // device plane tables per (slices, mesh, rows)
  int* f_piv = nullptr;     // (nk, nip)
  int* f_rank_dev = nullptr;
  std::vector<int> f_rank;  // host copy
  // the factorisation runs on a side stream, overlapped with the y build on `stream`, at the
  // priority fisdf_set_factor_priority asked for (side_hi: the priority it was created with)
  hipStream_t side = nullptr;
  int factor_hi = 0, side_hi = -1;
  std::vector<hipStream_t> pad;  // FISDF_PAD_QUEUES (ensure_side)
  void* pad_buf = nullptr;
  hipEvent_t ev_x4 = nullptr, ev_fac = nullptr, ev_chol = nullptr;
  hipEvent_t ev_fac_early = nullptr;  // the first f_early slots' operators (factor_finish)
  int f_early = 0;
  bool f_fac_unjoined = false;  // ev_fac not yet waited on by the main stream (fit lanes do)
  bool f_pending = false;
  bool x4_marked = false;  // fisdf_factor_x4_mark recorded ev_x4 for the next factor_x4_async
  int* f_rank_pinned = nullptr;  // host (pinned) copy target, f_nk ints
  void* f_scratch = nullptr;     // device scratch of the factorisation
  size_t f_scratch_size = 0;
  // pinned staging of small host arrays copied asynchronously (q-lists)
  int* stage_pinned = nullptr;
  int* sel_pinned = nullptr;  // selection read-back {error flag, rank, pivots} (pinned)
  size_t sel_cap = 0;
  size_t stage_cap = 0;
  hipEvent_t ev_stage = nullptr;
  // reality-invariant monitors
  unsigned long long* maximag = nullptr;  // 3 slots
  // time-reversal check of the build's AO inputs (x0, f): {max dev, max |a|} x 2 on the device,
  // read back through tr_pinned when ev_tr completes
  unsigned long long* trmon = nullptr;
  unsigned long long* tr_pinned = nullptr;
  hipEvent_t ev_tr = nullptr;
  // timing
  bool timing = false;
  struct Ev { int stage; hipEvent_t a, b; int span; };
  std::vector<Ev> events;
  // kernel execution spans of the kernel-exact stages (StageTimer): 2 u64 per slot, all-ones
  // initialised, read and refilled by fisdf_timings
  unsigned long long* spans = nullptr;
  int span_used = 0;
  static constexpr int kSpanCap = 16384;
  std::string last_error;  // fisdf_last_error(ctx)
  // fisdf_build: the resident result of the last composite build (W_q, W_s, X, ... on the device)
  struct Build {
    bool valid = false;
    int nk = 0, nip = 0, nao = 0, ng0 = 0, nfit = 0, used_pivoted = 0, min_norm = 0;
    int time_reversal = 0;  // 1: one q of each (q, -q) pair fitted (the inputs passed the check)
    double tr_deviation = 0.0;
    int kmesh[3] = {0, 0, 0}, mesh[3] = {0, 0, 0};
    double a[9] = {0};
    std::vector<int> perm, fit_qs, partner, ranks;
    std::vector<double> wt;
    void *X = nullptr, *x4 = nullptr, *Wq = nullptr, *Ws = nullptr;
    // fisdf_build_sharded: this rank's share (W_s rows [row0, row1), W_0 broadcast) and the
    // caller's collectives (get_jk all-reduces through them)
    int shard_rank = 0, shard_size = 1, row0 = 0, row1 = 0;
    void* W0 = nullptr;
    bool sharded = false;
    bool y_streamed = false;  // y formed behind the selection (fisdf_build_y_streamed)
    fisdf_comm comm{};
  } bld;
  // stream of the sharded build's all-to-all (fisdf_build_sharded), forked from `stream`
  hipStream_t comm_stream = nullptr;
  hipEvent_t ev_comm = nullptr;
  // fisdf_set_allocator: device memory of the composite build's buffers from the caller (e.g. a
  // framework's caching allocator), else library-owned grow-only buffers
  fisdf_alloc_fn alloc_fn = nullptr;
  fisdf_free_fn free_fn = nullptr;
  void* alloc_user = nullptr;
  std::map<int, std::pair<void*, size_t>> owned;  // role -> library-owned buffer
  std::vector<void*> lent;                        // buffers from alloc_fn not yet returned
  // The y build streamed behind the selection (build_impl, FISDF_Y_STREAM): while the
  // cooperative selection runs on `stream`, aux[2] and aux[0] form y in blocks of pivots as the
  // kernel publishes them (pchol_select_coop's progress word).  ys_dev: {progress, spin error}
  // (device ints); ws_ypiv: the pivots, context-owned so that no later arena user
  // overwrites them under the y stream; ws_ystream: XT / FT of the fused kernel.  `ys` is the
  // build's request, armed around the first selection only; enqueued: the y stream received the
  // work.
  int* ys_dev = nullptr;
  int* ys_err_pinned = nullptr;
  hipEvent_t ev_yerr = nullptr;
  hipEvent_t ev_ysfork = nullptr;  // `stream` just before the selection kernel: the y stream's start
  hipEvent_t ev_ys2[2] = {nullptr, nullptr};  // the streamed y's second stream (FISDF_Y_STREAM_2S)
  DevBuf ws_ypiv, ws_ystream;
  struct YStream {
    bool armed = false, enqueued = false;
    bool stale = false;  // the kernel it followed failed (a stalled step): its pivots were redone
    int aux = 2;         // the aux stream it runs on
    const cplx* x0 = nullptr;
    const cplx* f = nullptr;
    int ng0 = 0, nao = 0, nip = 0, rows = 128;
    long m = 0, fks = 0;  // grid points of the y build (columns of yT), k stride of f
    int kmesh[3] = {0, 0, 0};
    std::vector<int> qs;
    cplx* yT = nullptr;
    unsigned long long rmask = 0;
  } ys;
};

namespace fisdf {
void set_ctx_error(fisdf_ctx* c, const std::string& msg) { c->last_error = msg; }
}  // namespace fisdf

namespace {

// a grow-only temporary (growth waits for the device: the old block may be in use on any stream)
static int devbuf_get(fisdf_ctx::DevBuf& w, size_t bytes, void** out) {
  bytes = std::max<size_t>(bytes, 256);
  if (bytes > w.n) {
    if (w.p) {
      FISDF_HIP(hipDeviceSynchronize());
      FISDF_HIP(hipFree(w.p));
    }
    w.p = nullptr;
    w.n = 0;
    FISDF_HIP(hipMalloc(&w.p, bytes));
    w.n = bytes;
  }
  *out = w.p;
  return 0;
}

int arena_get(fisdf_ctx* c, size_t bytes, void** out) {
  bytes = std::max<size_t>(bytes, 256);
  if (bytes > c->arena_size) {
    FISDF_HIP(hipStreamSynchronize(c->stream));
    if (c->arena) FISDF_HIP(hipFree(c->arena));
    c->arena = nullptr;
    c->arena_size = 0;  // a failed growth below must not leave a stale size behind a null base
    size_t sz = bytes + bytes / 8;
    if (hipMalloc(&c->arena, sz) != hipSuccess) {
      (void)hipGetLastError();
      c->arena = nullptr;
      FISDF_HIP(hipMalloc(&c->arena, bytes));  // without the growth slack, then give up
      sz = bytes;
    }
    c->arena_size = sz;
  }
  *out = c->arena;
  return 0;
}

// carve aligned sub-buffers from one arena request
struct Carver {
  size_t off = 0;
  size_t take(size_t bytes) {
    size_t o = off;
    off += (bytes + 255) / 256 * 256;
    return o;
  }
};

// Asynchronous upload of a small host int array: staged through a pinned buffer whose reuse
// waits for the previous copy (no host sync on the stream).
// host -> device through the context's pinned staging buffer, asynchronous on the main stream;
// the buffer is reused once the previous staged copy has completed (ev_stage)
int upload_bytes(fisdf_ctx* c, const void* h, size_t bytes, void* d) {
  if (bytes == 0) return 0;
  if (!c->ev_stage) FISDF_HIP(hipEventCreateWithFlags(&c->ev_stage, hipEventDisableTiming));
  FISDF_HIP(hipEventSynchronize(c->ev_stage));
  if (bytes > c->stage_cap) {
    if (c->stage_pinned) FISDF_HIP(hipHostFree(c->stage_pinned));
    c->stage_pinned = nullptr;
    c->stage_cap = 0;
    FISDF_HIP(hipHostMalloc((void**)&c->stage_pinned, bytes, hipHostMallocDefault));
    c->stage_cap = bytes;
  }
  std::memcpy(c->stage_pinned, h, bytes);
  FISDF_HIP(hipMemcpyAsync(d, c->stage_pinned, bytes, hipMemcpyHostToDevice, c->stream));
  FISDF_HIP(hipEventRecord(c->ev_stage, c->stream));
  return 0;
}

int upload_ints(fisdf_ctx* c, const int* h, int n, int* d) {
  return n <= 0 ? 0 : upload_bytes(c, h, sizeof(int) * (size_t)n, d);
}

// Stage timer on stream `st`: events recorded on the stream around the stage.  kernel_exact: the
// stage is ONE zgemm()/herk() call whose kernels also record their execution span on the device
// (launch_events); fisdf_timings then reports that span — the kernels' own begin to end, as
// rocprofv3's kernel trace times them — instead of the event interval, which beside the other fit
// lanes also counts the time the stream waits for free CUs (r02: ~10 % more than the trace).
struct StageTimer {
  fisdf_ctx* c;
  int stage;
  hipStream_t st;
  bool exact;
  hipEvent_t a = nullptr, b = nullptr;
  int span = -1;
  StageTimer(fisdf_ctx* c_, int stg, hipStream_t on = nullptr, bool kernel_exact = false)
      : c(c_), stage(stg), st(on ? on : c_->stream), exact(kernel_exact) {
    if (c->timing) {
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      (void)hipEventRecord(a, st);
      if (exact && c->spans && c->span_used < fisdf_ctx::kSpanCap) {
        span = c->span_used++;
        LaunchEvents le;
        le.span = c->spans + 2 * span;
        launch_events() = le;
      }
    }
  }
  ~StageTimer() {
    if (c->timing) {
      (void)hipEventRecord(b, st);
      if (span >= 0) launch_events() = LaunchEvents();
      c->events.push_back({stage, a, b, span});
    }
  }
};

void lattice(const double a[9], CellGeom& g) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) g.a[i][j] = a[3 * i + j];
  // b = 2 pi inv(a)^T
  const double(*A)[3] = g.a;
  double det = A[0][0] * (A[1][1] * A[2][2] - A[1][2] * A[2][1]) -
               A[0][1] * (A[1][0] * A[2][2] - A[1][2] * A[2][0]) +
               A[0][2] * (A[1][0] * A[2][1] - A[1][1] * A[2][0]);
  double inv[3][3];
  inv[0][0] = (A[1][1] * A[2][2] - A[1][2] * A[2][1]) / det;
  inv[0][1] = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) / det;
  inv[0][2] = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) / det;
  inv[1][0] = (A[1][2] * A[2][0] - A[1][0] * A[2][2]) / det;
  inv[1][1] = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) / det;
  inv[1][2] = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) / det;
  inv[2][0] = (A[1][0] * A[2][1] - A[1][1] * A[2][0]) / det;
  inv[2][1] = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) / det;
  inv[2][2] = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) / det;
  const double twopi = 6.283185307179586;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) g.b[i][j] = twopi * inv[j][i];
}

double cell_volume(const double a[9]) {
  return std::fabs(a[0] * (a[4] * a[8] - a[5] * a[7]) - a[1] * (a[3] * a[8] - a[5] * a[6]) +
                   a[2] * (a[3] * a[7] - a[4] * a[6]));
}

// k-point q of the mesh (get_kpts order, wrap_around=False): k = (i/n) . b
void kpoint(const int kmesh[3], const CellGeom& g, int q, double k[3]) {
  int i2 = q % kmesh[2], i1 = (q / kmesh[2]) % kmesh[1], i0 = q / (kmesh[1] * kmesh[2]);
  double f[3] = {(double)i0 / kmesh[0], (double)i1 / kmesh[1], (double)i2 / kmesh[2]};
  for (int c = 0; c < 3; ++c) k[c] = f[0] * g.b[0][c] + f[1] * g.b[1][c] + f[2] * g.b[2][c];
}

// Phi[R,k] = exp(i T_R . k)/sqrt(nk)  (k2gamma.get_phase, wrap_around=False)
int get_phase(fisdf_ctx* c, const int kmesh[3], const double a[9], const cplx** out) {
  std::vector<double> key = {(double)kmesh[0], (double)kmesh[1], (double)kmesh[2]};
  for (int i = 0; i < 9; ++i) key.push_back(a[i]);
  auto it = c->phase_cache.find(key);
  if (it != c->phase_cache.end()) { *out = it->second; return 0; }
  CellGeom g;
  lattice(a, g);
  int nk = kmesh[0] * kmesh[1] * kmesh[2];
  std::vector<cplx> h((size_t)nk * nk);
  for (int R = 0; R < nk; ++R) {
    int r2 = R % kmesh[2], r1 = (R / kmesh[2]) % kmesh[1], r0 = R / (kmesh[1] * kmesh[2]);
    double T[3];
    for (int cc = 0; cc < 3; ++cc) T[cc] = r0 * g.a[0][cc] + r1 * g.a[1][cc] + r2 * g.a[2][cc];
    for (int q = 0; q < nk; ++q) {
      double k[3];
      kpoint(kmesh, g, q, k);
      double th = T[0] * k[0] + T[1] * k[1] + T[2] * k[2];
      h[(size_t)R * nk + q] = cmk(std::cos(th) / std::sqrt((double)nk), std::sin(th) / std::sqrt((double)nk));
    }
  }
  cplx* d = nullptr;
  FISDF_HIP(hipMalloc(&d, sizeof(cplx) * h.size()));
  FISDF_HIP(hipMemcpy(d, h.data(), sizeof(cplx) * h.size(), hipMemcpyHostToDevice));
  c->phase_cache[key] = d;
  *out = d;
  return 0;
}

int device_guard(fisdf_ctx* c) {
  t_cur_ctx = c;
  FISDF_CHECK(c != nullptr, "null context");
  FISDF_HIP(hipSetDevice(c->device));
  return 0;
}

// the entry points that touch no device state: failures still go to the context's own message
int ctx_guard(fisdf_ctx* c) {
  t_cur_ctx = c;
  FISDF_CHECK(c != nullptr, "null context");
  return 0;
}

const cplx ONE = {1.0, 0.0}, ZERO = {0.0, 0.0};

int free_factors(fisdf_ctx* c) {
  if (c->f_L) FISDF_HIP(hipFree(c->f_L));
  if (c->f_Lp) FISDF_HIP(hipFree(c->f_Lp));
  if (c->f_Linv) FISDF_HIP(hipFree(c->f_Linv));
  if (c->f_Q) FISDF_HIP(hipFree(c->f_Q));
  c->f_Q = nullptr;
  if (c->f_Li) FISDF_HIP(hipFree(c->f_Li));
  c->f_Li = nullptr;
  if (c->f_ksw) FISDF_HIP(hipFree(c->f_ksw));
  c->f_ksw = nullptr;
  c->f_ksw_elems = 0;
  if (c->f_x4s) FISDF_HIP(hipFree(c->f_x4s));
  c->f_x4s = nullptr;
  if (c->f_M) FISDF_HIP(hipFree(c->f_M));
  c->f_M = nullptr;
  if (c->f_nip_dev) FISDF_HIP(hipFree(c->f_nip_dev));
  c->f_nip_dev = nullptr;
  c->f_cod.clear();
  if (c->f_fail_pinned) FISDF_HIP(hipHostFree(c->f_fail_pinned));
  c->f_fail_pinned = nullptr;
  if (c->f_qr_pinned) FISDF_HIP(hipHostFree(c->f_qr_pinned));
  c->f_qr_pinned = nullptr;
  if (c->f_qr_dev) FISDF_HIP(hipFree(c->f_qr_dev));
  c->f_qr_dev = nullptr;
  if (c->f_piv) FISDF_HIP(hipFree(c->f_piv));
  if (c->f_rank_dev) FISDF_HIP(hipFree(c->f_rank_dev));
  if (c->f_rank_pinned) FISDF_HIP(hipHostFree(c->f_rank_pinned));
  c->f_rank_pinned = nullptr;
  c->f_L = c->f_Lp = c->f_Linv = nullptr;
  c->f_piv = c->f_rank_dev = nullptr;
  c->f_rank.clear();
  c->f_qs.clear();
  c->f_real.clear();
  c->f_nk = c->f_nip = 0;
  c->f_cap_nk = c->f_cap_nip = 0;
  return 0;
}

// x2 = sum_{q in [q0,q1)} conj(x0_q) x0_q^T, via P = x0 permuted to (ng0, nq*nao) and the
// Hermitian update P P^H (only its real part is used: Re(P P^H) = Re(conj(P) P^T)).
// `tmp` must hold ng0*nq*nao complex.
int select_gram(fisdf_ctx* c, const cplx* x0, int nk, int q0, int q1, int ng0, int nao, cplx* x2,
                cplx* tmp, const int* kmesh) {
  int nq = q1 - q0;
  if (kmesh && c->time_reversal && q0 == 0 && q1 == nk) {
    // time reversal (x0_{-q} = conj(x0_q)): Re(x0_{-q} x0_{-q}^H) = Re(x0_q x0_q^H), so the sum
    // over the k-mesh is the sum over the representatives q <= -q with a paired one counted
    // twice — its copy scaled by sqrt(2): 36 of 64 k at 4x4x4
    std::vector<int> reps;
    std::vector<char> self;
    kmesh_reps(kmesh, &reps, &self);
    std::vector<double> sc(reps.size());
    for (size_t j = 0; j < reps.size(); ++j) sc[j] = self[j] ? 1.0 : std::sqrt(2.0);
    nq = (int)reps.size();
    FISDF_TRY(permute_kgm_sel(c->stream, x0, reps.data(), sc.data(), nq, ng0, nao, tmp));
  } else {
    FISDF_TRY(permute_kgm(c->stream, x0 + (long)q0 * ng0 * nao, nq, ng0, nao, tmp));
  }
  const int K = nq * nao;
  int ks = 1;
  const long tiles = (long)((ng0 + 63) / 64) * ((ng0 + 63) / 64 + 1) / 2;
  while (tiles * ks < 512 && K / (ks * 2) >= 256) ks *= 2;
  void* work = nullptr;
  if (ks > 1) FISDF_TRY(devbuf_get(c->ws_main, sizeof(cplx) * (size_t)ks * ng0 * ng0, &work));
  // only Re(x2) enters the selection (fftisdf.py:379): real-part HERK, imaginary part zero
  FISDF_TRY(herk(c->stream, ng0, K, 1.0, tmp, K, x2, ng0, ks, (cplx*)work, GEMM_RE_ONLY));
  (void)nk;
  return 0;
}

// q is its own time-reversal partner (2 k_q in the reciprocal lattice): Phi[:, q] is real, so
// x4_q, y_q and z_q are real and W_q = Zhat diag(c) Zhat^H is real (Hermitian-symmetric
// spectrum) — the fit runs with a real factor (GEMM_A_REAL) and a real-part HERK
bool self_conjugate(const int kmesh[3], int q) {
  const int i2 = q % kmesh[2], i1 = (q / kmesh[2]) % kmesh[1], i0 = q / (kmesh[1] * kmesh[2]);
  return (2 * i0) % kmesh[0] == 0 && (2 * i1) % kmesh[1] == 0 && (2 * i2) % kmesh[2] == 0;
}

// cached Coulomb weight of the fit for q (computed on `st` and waited for the first time, so
// every stream may read it afterwards)
// the reciprocal-lattice vector m.b = 2 k_q of a self-conjugate q
void self_conjugate_m(const int kmesh[3], int q, int m[3]) {
  const int i2 = q % kmesh[2], i1 = (q / kmesh[2]) % kmesh[1], i0 = q / (kmesh[1] * kmesh[2]);
  m[0] = 2 * i0 / kmesh[0];
  m[1] = 2 * i1 / kmesh[1];
  m[2] = 2 * i2 / kmesh[2];
}

// half: the self-conjugate q's half-grid weight sqrt(c_G + c_G') (sqrt(c_G) on a self-paired
// plane, 0 beyond the prefix planes), see linalg.h half_weight
int get_weight(fisdf_ctx* c, hipStream_t st, const int mesh[3], const int kmesh[3],
               const double a[9], int q, double scale, bool half, const double** out) {
  std::vector<double> key = {(double)mesh[0], (double)mesh[1], (double)mesh[2], (double)kmesh[0],
                             (double)kmesh[1], (double)kmesh[2], (double)q, c->omega, scale,
                             half ? 1.0 : 0.0};
  for (int i = 0; i < 9; ++i) key.push_back(a[i]);
  auto it = c->wt_cache.find(key);
  if (it == c->wt_cache.end()) {
    CellGeom g;
    lattice(a, g);
    double kq[3];
    kpoint(kmesh, g, q, kq);
    const size_t ng = (size_t)mesh[0] * mesh[1] * mesh[2];
    double* w = nullptr;
    FISDF_HIP(hipMalloc(&w, sizeof(double) * ng));
    if (!half) {
      FISDF_TRY(coulg_weight(st, mesh, g, kq, scale, 1, w, c->omega));
    } else {
      // a cache fill: plain allocations (no stream-ordered pool memory shared with other streams)
      double* cw = nullptr;
      FISDF_HIP(hipMalloc((void**)&cw, sizeof(double) * ng));
      FISDF_TRY(coulg_weight(st, mesh, g, kq, scale, 0, cw, c->omega));
      int m[3];
      self_conjugate_m(kmesh, q, m);
      FISDF_TRY(half_weight(st, w, cw, mesh, m));
      FISDF_HIP(hipStreamSynchronize(st));
      FISDF_HIP(hipFree(cw));
    }
    FISDF_HIP(hipStreamSynchronize(st));
    it = c->wt_cache.emplace(key, w).first;
  }
  *out = it->second;
  return 0;
}

// the half-grid asymmetric-weight list of a self-conjugate q with its Im factors (cached)
int get_asym_half(fisdf_ctx* c, hipStream_t st, const int mesh[3], const int kmesh[3],
                  const double a[9], int q, double scale, const fisdf_ctx::Asym** out) {
  std::vector<double> key = {(double)mesh[0], (double)mesh[1], (double)mesh[2], (double)kmesh[0],
                             (double)kmesh[1], (double)kmesh[2], (double)q, c->omega, scale, 1.0};
  for (int i = 0; i < 9; ++i) key.push_back(a[i]);
  auto it = c->asym_cache.find(key);
  if (it == c->asym_cache.end()) {
    CellGeom g;
    lattice(a, g);
    double kq[3];
    kpoint(kmesh, g, q, kq);
    const long ngrid = (long)mesh[0] * mesh[1] * mesh[2];
    fisdf_ctx::Asym as;
    double* cw = nullptr;
    FISDF_HIP(hipMalloc(&as.idx, sizeof(int) * (ngrid + 1)));
    FISDF_HIP(hipMalloc(&as.f, sizeof(double) * ngrid));
    FISDF_HIP(hipMalloc((void**)&cw, sizeof(double) * ngrid));  // a cache fill (see get_weight)
    FISDF_TRY(coulg_weight(st, mesh, g, kq, scale, 0, cw, c->omega));
    int m[3];
    self_conjugate_m(kmesh, q, m);
    FISDF_TRY(asym_half(st, cw, mesh, m, as.idx, as.f, as.idx + ngrid));
    FISDF_HIP(hipMemcpyAsync(&as.n, as.idx + ngrid, sizeof(int), hipMemcpyDeviceToHost, st));
    FISDF_HIP(hipStreamSynchronize(st));
    FISDF_HIP(hipFree(cw));
    it = c->asym_cache.emplace(key, as).first;
  }
  *out = &it->second;
  return 0;
}

// cached asym_list of a self-conjugate q (one synchronous count read the first time)
int get_asym(fisdf_ctx* c, hipStream_t st, const int mesh[3], const int kmesh[3],
             const double a[9], int q, const double* wt, const fisdf_ctx::Asym** out) {
  std::vector<double> key = {(double)mesh[0], (double)mesh[1], (double)mesh[2], (double)kmesh[0],
                             (double)kmesh[1], (double)kmesh[2], (double)q, c->omega};
  for (int i = 0; i < 9; ++i) key.push_back(a[i]);
  auto it = c->asym_cache.find(key);
  if (it == c->asym_cache.end()) {
    const int i2 = q % kmesh[2], i1 = (q / kmesh[2]) % kmesh[1], i0 = q / (kmesh[1] * kmesh[2]);
    const int m[3] = {2 * i0 / kmesh[0], 2 * i1 / kmesh[1], 2 * i2 / kmesh[2]};
    const long ngrid = (long)mesh[0] * mesh[1] * mesh[2];
    fisdf_ctx::Asym as;
    int* cnt = nullptr;
    FISDF_HIP(hipMalloc(&as.idx, sizeof(int) * (ngrid + 1)));
    cnt = as.idx + ngrid;
    FISDF_TRY(asym_list(st, wt, mesh, m, as.idx, cnt));
    FISDF_HIP(hipMemcpyAsync(&as.n, cnt, sizeof(int), hipMemcpyDeviceToHost, st));
    FISDF_HIP(hipStreamSynchronize(st));
    if (getenv("FISDF_VERBOSE")) fprintf(stderr, "fisdf: q %d: %d of %ld G with asymmetric weight\n", q, as.n, ngrid);
    it = c->asym_cache.emplace(key, as).first;
  }
  *out = &it->second;
  return 0;
}

int env_fit_lanes() {
  static const int n = [] {
    const char* e = getenv("FISDF_FIT_LANES");
    const int v = e ? atoi(e) : 2;
    return std::max(1, std::min(4, v));
  }();
  return n;
}

int env_fit_pipe() {
  static const int v = [] {
    const char* e = getenv("FISDF_FIT_PIPE");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return v;
}

// the FFT ring's depth when fisdf_set_fit_pipe gave none: FISDF_PIPE_DEPTH, else lanes + 2
int default_pipe_depth(int lanes) {
  static const int env = [] {
    const char* e = getenv("FISDF_PIPE_DEPTH");
    return e ? std::max(0, std::min(64, atoi(e))) : 0;
  }();
  return env > 0 ? env : lanes + 2;
}

int num_cus(int device) {
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n <= 0)
    n = 256;
  return n;
}

// The fit's extra streams: aux[0] and aux[1] are MFMA lanes, aux[2] the pipelined FFT stream (its
// priority below).  All three are created
// together and in this order: HIP maps a process's streams onto hardware queues by creation
// order, and leaving aux[1] uncreated when unused measured +4.5 ms/step (even with 8 queues).
int ensure_aux(fisdf_ctx* c) {
  if (c->ev_fork) return 0;
  FISDF_HIP(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
  int least = 0, greatest = 0;
  FISDF_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
  // The FFT stream's priority depends on the HIP runtime the process runs: on the ROCm 7.0
  // runtime torch bundles the least priority is -0.45 ms/step (the lanes' MFMA kernels take the
  // CU slots first, r03), but the 7.2 runtime honours it more strictly and starves the FFTs the
  // lanes wait on: +4.2 ms/step (tools/capi_bench.py, profiles/r04/capi_vs_torch).  So: least
  // below 7.2, the default priority from 7.2 on.  FISDF_FFT_PRIO: 0 least, 1 default, 2 greatest.
  static const int fft_prio = [] {
    const char* e = getenv("FISDF_FFT_PRIO");
    if (e) return atoi(e);
    int v = 0;
    if (hipRuntimeGetVersion(&v) != hipSuccess) return 1;
    return (v / 10000000 > 7 || (v / 10000000 == 7 && (v / 100000) % 100 >= 2)) ? 1 : 0;
  }();
  // FISDF_FFT_CUS=n (experiment): the FFT stream confined to n CUs spread evenly over the device
  // (hipExtStreamCreateWithCUMask), so the HBM-bound FFTs stop taking workgroup slots on every CU
  static const int fft_cus = getenv("FISDF_FFT_CUS") ? atoi(getenv("FISDF_FFT_CUS")) : 0;
  for (int l = 0; l < 3; ++l) {
    if (l == 2 && fft_cus > 0) {
      const int ncu = num_cus(c->device);
      std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
      const int n = std::min(fft_cus, ncu);
      for (int i = 0; i < n; ++i) {
        const int cu = (int)((long)i * ncu / n);
        mask[cu / 32] |= 1u << (cu % 32);
      }
      FISDF_HIP(hipExtStreamCreateWithCUMask(&c->aux[l], (uint32_t)mask.size(), mask.data()));
    } else if (l == 2 && fft_prio != 1)
      FISDF_HIP(hipStreamCreateWithPriority(&c->aux[l], hipStreamNonBlocking,
                                            fft_prio == 2 ? greatest : least));
    else
      FISDF_HIP(hipStreamCreateWithFlags(&c->aux[l], hipStreamNonBlocking));
    FISDF_HIP(hipEventCreateWithFlags(&c->ev_join[l], hipEventDisableTiming));
  }
  for (int l = 0; l < 4; ++l) FISDF_HIP(hipEventCreateWithFlags(&c->ev_ybuf[l], hipEventDisableTiming));
  return 0;
}


std::vector<int> q_range(int q0, int q1) {
  std::vector<int> v;
  for (int q = q0; q < q1; ++q) v.push_back(q);
  return v;
}

// aux[i] is given work that may read a build buffer (fork side of the invariant above)
void aux_fork(fisdf_ctx* c, int i) { ++c->aux_use[i]; }

// join aux[i] into the main stream: later work (and frees) on `stream` are ordered after it
int aux_join(fisdf_ctx* c, int i) {
  FISDF_HIP(hipEventRecord(c->ev_join[i], c->aux[i]));
  FISDF_HIP(hipStreamWaitEvent(c->stream, c->ev_join[i], 0));
  c->aux_joined[i] = c->aux_use[i];
  return 0;
}

int check_aux_joined(fisdf_ctx* c, const char* what) {
  for (int i = 0; i < 3; ++i)
    FISDF_CHECK(c->aux_joined[i] == c->aux_use[i],
                std::string(what) + ": aux stream " + std::to_string(i) +
                    " not joined into the context stream (a buffer would be freed under a reader)");
  return 0;
}

int check_qlist(const int* qs, int nq, int nk, const char* who) {
  FISDF_CHECK(nq >= 0 && (nq == 0 || qs != nullptr), std::string(who) + ": bad q-list");
  for (int i = 0; i < nq; ++i)
    FISDF_CHECK(qs[i] >= 0 && qs[i] < nk && (i == 0 || qs[i] > qs[i - 1]),
                std::string(who) + ": q-list must be ascending and inside the k-mesh");
  return 0;
}

// K-split for a HERK of n x n over K: the lower-triangle tile count times ks is chosen just
// below a whole number of rounds of resident workgroups (3 per CU for the 64x64 ZGEMM tile),
// so the last round is not a nearly empty tail; each split keeps >= 2048 of K (the split
// partials cost 2 ks n^2 x 16 B of extra traffic).
int pick_ksplit_herk(int n, int K, int ncu) {
  const long nt = (n + 63) / 64, tiles = nt * (nt + 1) / 2;
  const long slots = 3L * ncu;
  int best = 1;
  double best_eff = 0;
  for (int m = 1; m <= 4; ++m) {
    long ks = std::max(1L, (m * slots) / tiles);
    ks = std::min<long>(ks, std::max(1, K / 1024));  // C3 sweep (3M): ks 13 -> 41 is -5% HERK time
    const long T = tiles * ks;
    const double eff = (double)T / ((double)((T + slots - 1) / slots) * slots);
    if (eff > best_eff + 0.01 || (eff > best_eff - 0.01 && ks > best)) {
      if (eff > best_eff) best_eff = eff;
      best = (int)ks;
    }
  }
  return best;
}


int pick_ksplit(int M, int N, int K) {
  long tiles = (long)((M + 63) / 64) * ((N + 63) / 64);
  int ks = 1;
  while (tiles * ks < 1024 && K / (ks * 2) >= 512) ks *= 2;
  return ks;
}

}  // namespace

// ---------------------------------------------------------------------------
extern "C" {

int fisdf_abi_version(void) { return FISDF_ABI_VERSION; }

const char* fisdf_last_error(const fisdf_ctx* c) {
  return c ? c->last_error.c_str() : g_last_error.c_str();
}

int fisdf_create(int device, void* stream, fisdf_ctx** out) {
  t_cur_ctx = nullptr;
  FISDF_CHECK(out != nullptr, "out is null");
  int ndev = 0;
  FISDF_HIP(hipGetDeviceCount(&ndev));
  FISDF_CHECK(device >= 0 && device < ndev, "device id out of range (no GPU visible?)");
  FISDF_HIP(hipSetDevice(device));
  fisdf_ctx* c = new fisdf_ctx();
  c->device = device;
  // NULL = the device's default (null) stream, which orders with torch's default stream
  c->stream = (hipStream_t)stream;
  c->own_stream = false;
  FISDF_HIP(hipMalloc(&c->maximag, 4 * sizeof(unsigned long long)));
  FISDF_HIP(hipMemsetAsync(c->maximag, 0, 4 * sizeof(unsigned long long), c->stream));
  {
    std::lock_guard<std::mutex> lk(g_live_mu);
    g_live.insert(c);
  }
  *out = c;
  return 0;
}

int fisdf_destroy(fisdf_ctx* c) {
  if (!c) return 0;
  {
    std::lock_guard<std::mutex> lk(g_live_mu);
    g_live.erase(c);
  }
  if (t_cur_ctx == c) t_cur_ctx = nullptr;
  FISDF_HIP(hipSetDevice(c->device));
  FISDF_HIP(hipStreamSynchronize(c->stream));
  // buffers lent by the caller's allocator stay the caller's (fisdf_set_allocator)
  c->lent.clear();
  for (auto& kv : c->owned)
    if (kv.second.first) (void)hipFree(kv.second.first);
  c->owned.clear();
  for (auto& e : c->events) { (void)hipEventDestroy(e.a); (void)hipEventDestroy(e.b); }
  for (auto& kv : c->phase_cache) (void)hipFree(kv.second);
  for (auto& kv : c->asym_cache) {
    (void)hipFree(kv.second.idx);
    if (kv.second.f) (void)hipFree(kv.second.f);
  }
  for (auto& kv : c->wt_cache) (void)hipFree(kv.second);
  if (c->f_pending) (void)hipEventSynchronize(c->ev_fac);
  free_factors(c);
  if (c->f_scratch) (void)hipFree(c->f_scratch);
  if (c->f_ring) (void)hipFree(c->f_ring);
  for (int l = 0; l < 3; ++l)  // the streamed y build's workspaces may still be in use there
    if (c->aux[l]) (void)hipStreamSynchronize(c->aux[l]);
  if (c->ys_dev) (void)hipFree(c->ys_dev);
  if (c->ys_err_pinned) (void)hipHostFree(c->ys_err_pinned);
  if (c->ev_yerr) (void)hipEventDestroy(c->ev_yerr);
  if (c->ev_ysfork) (void)hipEventDestroy(c->ev_ysfork);
  for (hipEvent_t e : c->ev_ys2)
    if (e) (void)hipEventDestroy(e);
  for (auto* w : {&c->ws_main, &c->ws_side_a, &c->ws_side_b, &c->ws_x4, &c->ws_ypiv, &c->ws_ystream})
    if (w->p) (void)hipFree(w->p);
  for (hipStream_t p : c->pad) (void)hipStreamDestroy(p);
  if (c->pad_buf) (void)hipFree(c->pad_buf);
  if (c->side) {
    (void)hipStreamSynchronize(c->side);
    (void)hipStreamDestroy(c->side);
    (void)hipEventDestroy(c->ev_x4);
    (void)hipEventDestroy(c->ev_fac);
    (void)hipEventDestroy(c->ev_fac_early);
    (void)hipEventDestroy(c->ev_chol);
  }
  if (c->ev_fork) {
    (void)hipEventDestroy(c->ev_fork);
    for (int l = 0; l < 3; ++l) {
      if (c->aux[l]) {
        (void)hipStreamSynchronize(c->aux[l]);
        (void)hipStreamDestroy(c->aux[l]);
        c->aux[l] = nullptr;
      }
      (void)hipEventDestroy(c->ev_join[l]);
    }
    for (int l = 0; l < 4; ++l) (void)hipEventDestroy(c->ev_ybuf[l]);
  }
  for (hipEvent_t e : c->ev_q) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->ev_free) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->ev_ready) (void)hipEventDestroy(e);
  if (c->comm_stream) {
    (void)hipStreamSynchronize(c->comm_stream);
    (void)hipStreamDestroy(c->comm_stream);
    (void)hipEventDestroy(c->ev_comm);
  }
  for (auto& kv : c->plane_cache) (void)hipFree(kv.second);
  if (c->arena) (void)hipFree(c->arena);
  if (c->ev_stage) (void)hipEventSynchronize(c->ev_stage), (void)hipEventDestroy(c->ev_stage);
  if (c->stage_pinned) (void)hipHostFree(c->stage_pinned);
  if (c->sel_pinned) (void)hipHostFree(c->sel_pinned);
  if (c->maximag) (void)hipFree(c->maximag);
  if (c->ev_tr) (void)hipEventSynchronize(c->ev_tr), (void)hipEventDestroy(c->ev_tr);
  if (c->trmon) (void)hipFree(c->trmon);
  if (c->tr_pinned) (void)hipHostFree(c->tr_pinned);
  if (c->spans) (void)hipFree(c->spans);
  if (c->own_stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

int fisdf_sync(fisdf_ctx* c) {
  FISDF_TRY(device_guard(c));
  FISDF_HIP(hipStreamSynchronize(c->stream));
  return 0;
}

int fisdf_malloc(fisdf_ctx* c, size_t bytes, void** p) {
  FISDF_TRY(device_guard(c));
  FISDF_HIP(hipMalloc(p, std::max<size_t>(bytes, 1)));
  return 0;
}

int fisdf_free(fisdf_ctx* c, void* p) {
  FISDF_TRY(device_guard(c));
  FISDF_HIP(hipStreamSynchronize(c->stream));
  FISDF_HIP(hipFree(p));
  return 0;
}

int fisdf_memcpy_htod(fisdf_ctx* c, void* d, const void* h, size_t bytes) {
  FISDF_TRY(device_guard(c));
  FISDF_HIP(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, c->stream));
  FISDF_HIP(hipStreamSynchronize(c->stream));
  return 0;
}

int fisdf_memcpy_dtoh(fisdf_ctx* c, void* h, const void* d, size_t bytes) {
  FISDF_TRY(device_guard(c));
  FISDF_HIP(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, c->stream));
  FISDF_HIP(hipStreamSynchronize(c->stream));
  return 0;
}

int fisdf_set_timing(fisdf_ctx* c, int enable) {
  FISDF_TRY(device_guard(c));
  c->timing = enable != 0;
  if (c->timing && !c->spans) {
    FISDF_HIP(hipMalloc(&c->spans, sizeof(unsigned long long) * 2 * fisdf_ctx::kSpanCap));
    FISDF_HIP(hipMemsetAsync(c->spans, 0xff, sizeof(unsigned long long) * 2 * fisdf_ctx::kSpanCap,
                             c->stream));
    FISDF_HIP(hipStreamSynchronize(c->stream));
    c->span_used = 0;
  }
  return 0;
}

int fisdf_timings(fisdf_ctx* c, double* ms, int* calls) {
  FISDF_TRY(device_guard(c));
  FISDF_HIP(hipStreamSynchronize(c->stream));
  for (int i = 0; i < FISDF_NSTAGES; ++i) {
    if (ms) ms[i] = 0;
    if (calls) calls[i] = 0;
  }
  std::vector<unsigned long long> sp(2 * (size_t)c->span_used);
  if (c->span_used) {
    FISDF_HIP(hipDeviceSynchronize());  // the lanes' kernels too
    FISDF_HIP(hipMemcpy(sp.data(), c->spans, sizeof(unsigned long long) * sp.size(),
                        hipMemcpyDeviceToHost));
  }
  for (auto& e : c->events) {
    float t = 0;
    if (e.span >= 0) {
      // the kernels' own execution span: s_memrealtime runs at 100 MHz
      const unsigned long long t0 = sp[2 * e.span], t1 = ~sp[2 * e.span + 1];
      t = (t0 != ~0ull && sp[2 * e.span + 1] != ~0ull && t1 >= t0) ? (float)((t1 - t0) * 1e-5) : 0.f;
    } else {
      FISDF_HIP(hipEventElapsedTime(&t, e.a, e.b));
    }
    if (ms) ms[e.stage] += t;
    if (calls) calls[e.stage] += 1;
    (void)hipEventDestroy(e.a);
    (void)hipEventDestroy(e.b);
  }
  c->events.clear();
  if (c->span_used) {
    FISDF_HIP(hipMemsetAsync(c->spans, 0xff, sizeof(unsigned long long) * 2 * c->span_used, c->stream));
    FISDF_HIP(hipStreamSynchronize(c->stream));
    c->span_used = 0;
  }
  return 0;
}

int fisdf_max_imag(fisdf_ctx* c, double* out) {
  FISDF_TRY(device_guard(c));
  unsigned long long h[4];
  FISDF_HIP(hipMemcpyAsync(h, c->maximag, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  FISDF_HIP(hipStreamSynchronize(c->stream));
  for (int i = 0; i < 3; ++i) {
    double v;
    std::memcpy(&v, &h[i], sizeof(double));
    out[i] = v;
  }
  FISDF_HIP(hipMemsetAsync(c->maximag, 0, 4 * sizeof(unsigned long long), c->stream));
  return 0;
}

// ---- building blocks -------------------------------------------------------
int fisdf_zgemm(fisdf_ctx* c, int opA, int opB, int M, int N, int K, const double alpha[2],
                const void* A, long lda, long sA, const void* B, long ldb, long sB,
                const double beta[2], void* C, long ldc, long sC, int batch, int ksplit) {
  FISDF_TRY(device_guard(c));
  cplx* work = nullptr;
  if (ksplit > 1) {
    void* w;
    FISDF_TRY(arena_get(c, sizeof(cplx) * (size_t)ksplit * M * N * batch, &w));
    work = (cplx*)w;
  }
  return zgemm(c->stream, opA, opB, M, N, K, cmk(alpha[0], alpha[1]), (const cplx*)A, lda, sA,
               (const cplx*)B, ldb, sB, cmk(beta[0], beta[1]), (cplx*)C, ldc, sC, batch,
               ksplit, work);
}

int fisdf_zgemm_mode(fisdf_ctx* c, int opA, int opB, int M, int N, int K, const double alpha[2],
                     const void* A, long lda, long sA, const void* B, long ldb, long sB,
                     const double beta[2], void* C, long ldc, long sC, int batch, int mode) {
  FISDF_TRY(device_guard(c));
  return zgemm(c->stream, opA, opB, M, N, K, cmk(alpha[0], alpha[1]), (const cplx*)A, lda, sA,
               (const cplx*)B, ldb, sB, cmk(beta[0], beta[1]), (cplx*)C, ldc, sC, batch, 1,
               nullptr, EPI_NONE, nullptr, mode);
}

int fisdf_herk(fisdf_ctx* c, int n, int K, double alpha, const void* A, long lda, void* Cm,
               long ldc, int ksplit) {
  FISDF_TRY(device_guard(c));
  cplx* work = nullptr;
  if (ksplit > 1) {
    void* w;
    FISDF_TRY(arena_get(c, sizeof(cplx) * (size_t)ksplit * n * n, &w));
    work = (cplx*)w;
  }
  return herk(c->stream, n, K, alpha, (const cplx*)A, lda, (cplx*)Cm, ldc, ksplit, work);
}

int fisdf_fft3d(fisdf_ctx* c, const void* in, void* out, int rows, const int mesh[3]) {
  FISDF_TRY(device_guard(c));
  long ng = (long)mesh[0] * mesh[1] * mesh[2];
  return fft3d(c->stream, (const cplx*)in, ng, nullptr, (cplx*)out, ng, rows, mesh[0], mesh[1],
               mesh[2], nullptr, nullptr, nullptr);
}

int fisdf_fft3d_paired(fisdf_ctx* c, const void* in, void* out, int rows, const int mesh[3],
                       const double kd[3], const int m[3], int in_real) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(in && out && mesh && rows >= 0, "fft3d_paired: bad arguments");
  FISDF_CHECK(!in_real || in != out, "fft3d_paired: real input needs an output buffer of its own");
  long ng = (long)mesh[0] * mesh[1] * mesh[2];
  return fft3d(c->stream, (const cplx*)in, ng, nullptr, (cplx*)out, ng, rows, mesh[0], mesh[1],
               mesh[2], kd, nullptr, nullptr, nullptr, m, in_real != 0);
}

int fisdf_coulg(fisdf_ctx* c, const int mesh[3], const double a[9], const double k[3],
                double scale, int take_sqrt, double* w) {
  FISDF_TRY(device_guard(c));
  CellGeom g;
  lattice(a, g);
  return coulg_weight(c->stream, mesh, g, k, scale, take_sqrt, w, c->omega);
}

int fisdf_min_norm_operator(fisdf_ctx* c, const void* A, int n, double tol_rel, void* M,
                            void* Qo, void* Rio, int* h_piv, int* h_rank) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(n >= 1, "min_norm_operator: bad size");
  Carver cv;
  size_t oL = cv.take(sizeof(cplx) * (size_t)n * n);
  size_t oP = cv.take(sizeof(int) * (size_t)n);
  size_t oR = cv.take(sizeof(int));
  size_t oD = cv.take(sizeof(double) * (size_t)n);
  size_t oF = cv.take(sizeof(int) * 4);
  size_t oW = cv.take(sizeof(double) * (size_t)(1 + n));
  size_t oM = cv.take(min_norm_work_bytes(n, n));
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  char* b = (char*)base;
  void* trail = nullptr;
  FISDF_TRY(devbuf_get(c->ws_main, sizeof(cplx) * pchol_trail_elems(n, 1), &trail));
  FISDF_TRY(pchol(c->stream, (const cplx*)A, n, (long)n * n, n, 1, n, tol_rel, 0.0, (cplx*)(b + oL),
                  (int*)(b + oP), (int*)(b + oR), (double*)(b + oD), (int*)(b + oF),
                  (double*)(b + oW), (cplx*)trail));
  int r = 0;
  FISDF_HIP(hipMemcpyAsync(&r, b + oR, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  FISDF_HIP(hipStreamSynchronize(c->stream));
  FISDF_CHECK(r >= 1, "min_norm_operator: zero matrix");
  FISDF_HIP(hipMemsetAsync(M, 0, sizeof(cplx) * (size_t)n * n, c->stream));
  FISDF_TRY(min_norm_operator(c->stream, (const cplx*)(b + oL), n, n, (int*)(b + oP), r, (cplx*)M, n,
                              b + oM, (int*)(b + oF), (cplx*)Qo, (cplx*)Rio));
  int fl[3] = {0, 0, 0};
  FISDF_HIP(hipMemcpyAsync(fl, b + oF, sizeof(fl), hipMemcpyDeviceToHost, c->stream));
  FISDF_HIP(hipMemcpyAsync(h_piv, b + oP, sizeof(int) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
  FISDF_HIP(hipStreamSynchronize(c->stream));
  FISDF_CHECK(fl[0] == 0 && fl[1] == 0 && fl[2] == 0, "min_norm_operator: CholeskyQR breakdown");
  *h_rank = r;
  return 0;
}

int fisdf_pivoted_cholesky(fisdf_ctx* c, const void* A, int n, int batch, int rmax,
                           double tol_rel, int* h_piv, int* h_rank) {
  FISDF_TRY(device_guard(c));
  Carver cv;
  size_t oL = cv.take(sizeof(cplx) * (size_t)batch * n * rmax);
  size_t oP = cv.take(sizeof(int) * (size_t)batch * rmax);
  size_t oR = cv.take(sizeof(int) * batch);
  size_t oD = cv.take(sizeof(double) * (size_t)batch * n);
  size_t oF = cv.take(sizeof(int) * batch);
  size_t oW = cv.take(sizeof(double) * (size_t)batch * (1 + rmax));
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  char* b = (char*)base;
  void* trail = nullptr;
  FISDF_TRY(devbuf_get(c->ws_main, sizeof(cplx) * pchol_trail_elems(n, batch), &trail));
  FISDF_TRY(pchol(c->stream, (const cplx*)A, n, (long)n * n, n, batch, rmax, tol_rel, 0.0,
                  (cplx*)(b + oL), (int*)(b + oP), (int*)(b + oR), (double*)(b + oD),
                  (int*)(b + oF), (double*)(b + oW), (cplx*)trail));
  FISDF_HIP(hipMemcpyAsync(h_piv, b + oP, sizeof(int) * (size_t)batch * rmax,
                           hipMemcpyDeviceToHost, c->stream));
  FISDF_HIP(hipMemcpyAsync(h_rank, b + oR, sizeof(int) * batch, hipMemcpyDeviceToHost, c->stream));
  FISDF_HIP(hipStreamSynchronize(c->stream));
  return 0;
}

int fisdf_cholesky(fisdf_ctx* c, void* A, int n, int batch, double tol_rel, int* h_fail) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(n >= 1 && batch >= 1, "cholesky: bad sizes");
  Carver cv;
  size_t oW = cv.take(sizeof(cplx) * (size_t)batch * 4096 + sizeof(double) * batch);
  size_t oP = cv.take(sizeof(int) * (size_t)batch * n);
  size_t oR = cv.take(sizeof(int) * batch);
  size_t oF = cv.take(sizeof(int) * batch);
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  char* b = (char*)base;
  FISDF_TRY(chol_unpivoted(c->stream, (cplx*)A, n, batch, tol_rel, (int*)(b + oP), (int*)(b + oR),
                           (int*)(b + oF), (cplx*)(b + oW)));
  FISDF_HIP(hipMemcpyAsync(h_fail, b + oF, sizeof(int) * batch, hipMemcpyDeviceToHost, c->stream));
  FISDF_HIP(hipStreamSynchronize(c->stream));
  return 0;
}

int fisdf_tri_inverse(fisdf_ctx* c, const void* L, int n, int batch, void* Linv) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(n >= 1 && batch >= 1, "tri_inverse: bad sizes");
  const long nn = (long)n * n, we = std::max(1L, trsm_split_work_elems(n, batch));
  Carver cv;
  size_t oQ = cv.take(sizeof(cplx) * (size_t)batch * nn);
  size_t oK = cv.take(sizeof(cplx) * (size_t)we);
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  cplx* Q = (cplx*)((char*)base + oQ);
  // the factor stage's own sequence (factor_finish): block-row operator, then the merged
  // substitution applied to the identity
  FISDF_TRY(build_trsm_q(c->stream, (const cplx*)L, n, nn, Q, batch, GEMM_FULL));
  FISDF_TRY(set_identity(c->stream, (cplx*)Linv, n, batch));
  FISDF_TRY(trsm_merged_batched(c->stream, Q, nn, n, (cplx*)Linv, n, nn, n, batch, true,
                                (cplx*)((char*)base + oK), we));
  return 0;
}

// ---- A1 ---------------------------------------------------------------------
// The streamed y build's work on aux[2] and aux[0], enqueued right after the selection kernel (so
// it never precedes it on any queue): the fused y kernel block by block, each block's XT rows
// waiting on the kernel's progress word (y_fused_stream).  Ordered after everything on `stream`
// before the selection (the previous build's readers of the y buffer and workspaces included).
static int ensure_side(fisdf_ctx* c);

static int ystream_enqueue(fisdf_ctx* c, const int* piv) {
  fisdf_ctx::YStream& Y = c->ys;
  // the side stream first, then the aux streams: the order the unstreamed build creates them in
  // (the runtime places a process's streams on hardware queues in creation order, and the fit's
  // two lanes serialise when aux[0] lands elsewhere: C3 89 vs 81 ms/step, profiles/r06/lanes/)
  FISDF_TRY(ensure_side(c));
  FISDF_TRY(ensure_aux(c));
  const int nq = (int)Y.qs.size();
  const size_t yw = y_fused_workspace(Y.kmesh, Y.nip, Y.nao, (int)Y.m);
  FISDF_CHECK(yw > 0 && nq > 0, "streamed y: the fused kernel does not apply");
  void* wb = nullptr;
  FISDF_TRY(devbuf_get(c->ws_ystream, yw, &wb));
  // the aux stream that carries the streamed y: aux[2], the fit's FFT stream, whose FFTs then
  // follow y in stream order (C3 79.8 / 79.4 ms/step against 81.6 / 81.2 on aux[1] and 79.9 on
  // aux[0], profiles/r06/lanes2-3); FISDF_Y_STREAM_AUX (read per build) for A/B
  const int ia = [] {
    const char* e = getenv("FISDF_Y_STREAM_AUX");
    const int v = e ? atoi(e) : 2;
    return (v >= 0 && v <= 2) ? v : 2;
  }();
  c->ys.aux = ia;
  hipStream_t ys = c->aux[ia];
  aux_fork(c, ia);
  FISDF_HIP(hipStreamWaitEvent(ys, c->ev_ysfork, 0));
  // blocks alternate over aux[ia] and a second aux stream (one block's tail overlaps the next
  // one's start), ordered back into aux[ia] at the end, so joining aux[ia] joins both: C3 in one
  // process 79.05 / 79.30 against 79.52 / 79.59 ms/step on one stream (profiles/r06/ab11-12);
  // FISDF_Y_STREAM_2S=0 (read per build) keeps one stream
  const char* e2 = getenv("FISDF_Y_STREAM_2S");
  const int i2 = (e2 && e2[0] == '0') ? -1 : (ia == 0 ? 1 : 0);
  if (i2 >= 0 && !c->ev_ys2[0]) {
    FISDF_HIP(hipEventCreateWithFlags(&c->ev_ys2[0], hipEventDisableTiming));
    FISDF_HIP(hipEventCreateWithFlags(&c->ev_ys2[1], hipEventDisableTiming));
  }
  // (a round-6 experiment held the blocks after the first until x4 was done, on a device flag the
  // build set: x4 1.3 ms instead of 3.0, but the factor chain after it 5.2 instead of 4.1 ms and
  // the step 0.5-1 ms slower, profiles/r06/r06_gate.  Removed: a host-side device synchronisation
  // before the flag was set — a workspace growth, a hipFree — waited for the held blocks until
  // their bounded wait expired)
  bool handled = false;
  {
    StageTimer tm(c, FISDF_ST_Y, ys);
    FISDF_TRY(y_fused_stream(ys, Y.x0, Y.ng0, Y.nao, piv, c->ys_dev, c->ys_dev + 1, Y.nip, Y.rows,
                             Y.f, Y.fks, (int)Y.m, Y.kmesh, Y.qs.data(), nq, Y.yT,
                             (long)Y.nip * Y.m, Y.m, 0, (cplx*)wb, yw, Y.rmask, &handled,
                             i2 >= 0 ? c->aux[i2] : nullptr, c->ev_ys2[0], c->ev_ys2[1]));
  }
  // aux[i2]'s work is ordered before aux[ia]'s last command: joined with it (buffer-return
  // bookkeeping, check_aux_joined)
  if (i2 >= 0) {
    aux_fork(c, i2);
    c->aux_joined[i2] = c->aux_use[i2];
  }
  FISDF_CHECK(handled, "streamed y: nothing enqueued");
  Y.enqueued = true;
  return 0;
}

// after the selection: whether yT holds the y build of the selected points (the selection gave
// the cap's points, its first pass did not fail, the q-list is the armed one); the y stream's
// spin-error flag is queued for read-back (ev_yerr).  The caller joins the y stream (ystream_join).
static bool ystream_valid(fisdf_ctx* c, int nip, const int* qs, int nq) {
  const fisdf_ctx::YStream& Y = c->ys;
  return Y.enqueued && !Y.stale && nip == Y.nip && (int)Y.qs.size() == nq &&
         std::equal(Y.qs.begin(), Y.qs.end(), qs);
}

static int ystream_join(fisdf_ctx* c) {
  const int ia = c->ys.aux;
  if (!c->ys.enqueued || c->aux_joined[ia] == c->aux_use[ia]) return 0;
  FISDF_TRY(aux_join(c, ia));
  FISDF_HIP(hipMemcpyAsync(c->ys_err_pinned, c->ys_dev + 1, sizeof(int), hipMemcpyDeviceToHost,
                           c->stream));
  FISDF_HIP(hipEventRecord(c->ev_yerr, c->stream));
  return 0;
}

// the streamed y's bounded waits all met their pivots (call after ystream_join)
static int ystream_check(fisdf_ctx* c) {
  FISDF_HIP(hipEventSynchronize(c->ev_yerr));
  FISDF_CHECK(*c->ys_err_pinned == 0, "streamed y: the selection's progress never arrived");
  return 0;
}

// arm the streamed y for the next selection: y_q (q in qs, ascending) of rows [0, nip_max) on m
// grid points (f: k stride fks) into yT[slot][I][g], self-conjugate q in rmask stored real.
// *armed = false when the fused kernel does not cover the k-mesh (nothing will stream).
static int ystream_arm(fisdf_ctx* c, const void* x0, int ng0, const void* f, long fks, long m,
                       int nao, int nip_max, const int kmesh[3], const int* qs, int nq, void* yT,
                       unsigned long long rmask, bool* armed) {
  *armed = false;
  FISDF_TRY(ystream_join(c));  // a streamed y never finished (an error in between) is joined
  c->ys = fisdf_ctx::YStream();
  if (nip_max <= 0 || m <= 0 || nq <= 0 || !y_fused_applies(kmesh, nao)) return 0;
  FISDF_CHECK(x0 && f && yT && qs, "y_stream_arm: null argument");
  if (!c->ys_dev) {
    FISDF_HIP(hipMalloc((void**)&c->ys_dev, 4 * sizeof(int)));
    FISDF_HIP(hipHostMalloc((void**)&c->ys_err_pinned, sizeof(int), hipHostMallocDefault));
    FISDF_HIP(hipEventCreateWithFlags(&c->ev_yerr, hipEventDisableTiming));
    FISDF_HIP(hipEventCreateWithFlags(&c->ev_ysfork, hipEventDisableTiming));
  }
  fisdf_ctx::YStream& Y = c->ys;
  Y.x0 = (const cplx*)x0;
  Y.f = (const cplx*)f;
  Y.fks = fks;
  Y.m = m;
  Y.ng0 = ng0;
  Y.nao = nao;
  Y.nip = std::min(nip_max, ng0);
  for (int i = 0; i < 3; ++i) Y.kmesh[i] = kmesh[i];
  Y.qs.assign(qs, qs + nq);
  Y.yT = (cplx*)yT;
  Y.rmask = rmask;
  // pivots per block, FISDF_Y_STREAM_ROWS (a multiple of 16; read per build): 128 — C3 in one
  // process, 4 interleaved rounds: 64 rows 78.77, 128 78.29, 192 78.23, 256 78.45, unstreamed
  // 79.96 ms/step (profiles/r06/ab9_inproc.json); fewer, larger launches beat an earlier start
  const int rows_env = [] {
    const char* e = getenv("FISDF_Y_STREAM_ROWS");
    const int v = e ? atoi(e) : 128;
    return (v >= 16 && v % 16 == 0 && v <= 1024) ? v : 128;
  }();
  Y.rows = rows_env;
  Y.armed = true;
  *armed = true;
  return 0;
}

// The selection's pivots on the device: the cooperative kernel, the blocked or the generic pivoted
// Cholesky (in that order of preference), then ONE pinned read-back of {error flag, rank, pivots}
// and one stream synchronisation (round 2 synchronised twice through pageable copies); a
// cooperative run that reports a stalled step is redone on the non-cooperative paths.
static int select_pivots_dev(fisdf_ctx* c, const cplx* X2, double scale, int ng0, int nip_max,
                             double tol, cplx* X4, int* piv, int* rank, cplx* L, double* d,
                             int* flags, double* w, int* h_perm, int* h_rank) {
  const size_t nint = 2 + (size_t)nip_max;
  if (c->sel_cap < nint) {
    if (c->sel_pinned) FISDF_HIP(hipHostFree(c->sel_pinned));
    c->sel_pinned = nullptr;
    c->sel_cap = 0;
    FISDF_HIP(hipHostMalloc((void**)&c->sel_pinned, sizeof(int) * nint, hipHostMallocDefault));
    c->sel_cap = nint;
  }
  // an armed streamed y (build_impl, fisdf_y_stream_arm) is for this selection only
  const bool armed = c->ys.armed;
  c->ys.armed = false;
  for (int pass = 0; pass < 2; ++pass) {
    bool handled = false;
    const int* coop_err = nullptr;
    // a streamed y build reads the pivots while the kernel runs: the selection then writes them
    // to the context's own buffer and publishes its progress
    const bool stream_y = armed && pass == 0 && c->ys.nip == nip_max;
    int* progress = nullptr;
    if (stream_y) {
      void* pp = nullptr;
      FISDF_TRY(devbuf_get(c->ws_ypiv, sizeof(int) * (size_t)nip_max, &pp));
      piv = (int*)pp;
      progress = c->ys_dev;
      FISDF_HIP(hipMemsetAsync(c->ys_dev, 0, 2 * sizeof(int), c->stream));
      // the y stream starts from here, beside the kernel (not after it)
      FISDF_HIP(hipEventRecord(c->ev_ysfork, c->stream));
    }
    bool publishes = false;
    FISDF_TRY(pchol_select_real(c->stream, X2, scale, ng0, nip_max, tol, piv, rank, (double*)X4,
                                flags, &handled, pass == 0, &coop_err, progress, &publishes));
    if (stream_y) {
      // whatever ran, consumers waiting on the progress word are released when it has ended
      FISDF_HIP(hipMemsetD32Async(c->ys_dev, kSelDone, 1, c->stream));
      if (handled && publishes) FISDF_TRY(ystream_enqueue(c, piv));
    }
    if (!handled) {
      FISDF_TRY(square_scale(c->stream, X2, scale, X4, (long)ng0 * ng0));
      void* trail = nullptr;
      FISDF_TRY(devbuf_get(c->ws_main, sizeof(cplx) * pchol_trail_elems(ng0, 1), &trail));
      FISDF_TRY(pchol(c->stream, X4, ng0, 0, ng0, 1, nip_max, tol, 0.0, L, piv, rank, d, flags, w,
                      (cplx*)trail));
    }
    int* hp = c->sel_pinned;
    hp[0] = 0;
    if (coop_err)
      FISDF_HIP(hipMemcpyAsync(hp, coop_err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    FISDF_HIP(hipMemcpyAsync(hp + 1, rank, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    FISDF_HIP(hipMemcpyAsync(hp + 2, piv, sizeof(int) * nip_max, hipMemcpyDeviceToHost, c->stream));
    FISDF_HIP(hipStreamSynchronize(c->stream));
    if (stream_y && hp[0] != 0) c->ys.stale = true;
    if (hp[0] == 0) {
      *h_rank = hp[1];
      std::memcpy(h_perm, hp + 2, sizeof(int) * nip_max);
      return 0;
    }
  }
  FISDF_CHECK(false, "select: pivoted Cholesky failed on every path");
  return 0;
}

static int select_points_impl(fisdf_ctx* c, const void* x0v, int nk, const int* kmesh, int ng0,
                              int nao, int nip_max, double tol, int* h_perm, int* h_npiv,
                              int* h_full_rank);

int fisdf_select_points(fisdf_ctx* c, const void* x0v, int nk, int ng0, int nao, int nip_max,
                        double tol, int* h_perm, int* h_npiv, int* h_full_rank) {
  FISDF_TRY(device_guard(c));
  return select_points_impl(c, x0v, nk, nullptr, ng0, nao, nip_max, tol, h_perm, h_npiv,
                            h_full_rank);
}

int fisdf_select_points_km(fisdf_ctx* c, const void* x0v, const int kmesh[3], int ng0, int nao,
                           int nip_max, double tol, int* h_perm, int* h_npiv, int* h_full_rank) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(kmesh && kmesh[0] > 0 && kmesh[1] > 0 && kmesh[2] > 0, "select_points: bad k-mesh");
  return select_points_impl(c, x0v, kmesh[0] * kmesh[1] * kmesh[2], kmesh, ng0, nao, nip_max, tol,
                            h_perm, h_npiv, h_full_rank);
}

static int select_points_impl(fisdf_ctx* c, const void* x0v, int nk, const int* kmesh, int ng0,
                              int nao, int nip_max, double tol, int* h_perm, int* h_npiv,
                              int* h_full_rank) {
  FISDF_CHECK(nk > 0 && ng0 > 0 && nao > 0 && nip_max > 0, "select_points: bad sizes");
  nip_max = std::min(nip_max, ng0);
  StageTimer tm(c, FISDF_ST_SELECT);
  const cplx* x0 = (const cplx*)x0v;
  Carver cv;
  size_t oX2 = cv.take(sizeof(cplx) * (size_t)ng0 * ng0);
  size_t oX4 = cv.take(sizeof(cplx) * (size_t)ng0 * ng0);
  size_t oPm = cv.take(sizeof(cplx) * (size_t)ng0 * nk * nao);
  size_t oL = cv.take(sizeof(cplx) * (size_t)ng0 * nip_max);
  size_t oP = cv.take(sizeof(int) * nip_max);
  size_t oR = cv.take(sizeof(int) * 4);
  size_t oD = cv.take(sizeof(double) * ng0);
  size_t oF = cv.take(sizeof(int) * 4);
  size_t oW = cv.take(sizeof(double) * (1 + nip_max));
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  char* b = (char*)base;
  cplx* X2 = (cplx*)(b + oX2);
  cplx* X4 = (cplx*)(b + oX4);
  // x2 = sum_q conj(x0_q) x0_q^T   (fftisdf.py:376-378; real part taken below) as one
  // K = nk*nao Hermitian rank-K update of the permuted x0
  FISDF_TRY(select_gram(c, x0, nk, 0, nk, ng0, nao, X2, (cplx*)(b + oPm), kmesh));
  // x4 = Re(x2)^2 / nk (:379) and the greedy pivoted Cholesky (:381-384), first nip_max
  // pivots: real blocked panels (X4's storage holds the real trailing matrix)
  int rank = 0;
  FISDF_TRY(select_pivots_dev(c, X2, 1.0 / nk, ng0, nip_max, tol, X4, (int*)(b + oP),
                              (int*)(b + oR), (cplx*)(b + oL), (double*)(b + oD), (int*)(b + oF),
                              (double*)(b + oW), h_perm, &rank));
  *h_npiv = rank;
  if (h_full_rank) *h_full_rank = rank < nip_max ? 1 : 0;
  return 0;
}

int fisdf_select_gram(fisdf_ctx* c, const void* x0, int nk, int q0, int q1, int ng0, int nao,
                      void* x2) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(0 <= q0 && q0 <= q1 && q1 <= nk && ng0 > 0 && nao > 0, "select_gram: bad sizes");
  StageTimer tm(c, FISDF_ST_SELECT);
  if (q1 == q0) {
    FISDF_HIP(hipMemsetAsync(x2, 0, sizeof(cplx) * (size_t)ng0 * ng0, c->stream));
    return 0;
  }
  void* base;
  FISDF_TRY(arena_get(c, sizeof(cplx) * (size_t)ng0 * (q1 - q0) * nao, &base));
  return select_gram(c, (const cplx*)x0, nk, q0, q1, ng0, nao, (cplx*)x2, (cplx*)base, nullptr);
}

int fisdf_select_pivots(fisdf_ctx* c, const void* x2, int nk, int ng0, int nip_max, double tol,
                        int* h_perm, int* h_npiv, int* h_full_rank) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(nk > 0 && ng0 > 0 && nip_max > 0, "select_pivots: bad sizes");
  nip_max = std::min(nip_max, ng0);
  StageTimer tm(c, FISDF_ST_SELECT);
  Carver cv;
  size_t oX4 = cv.take(sizeof(cplx) * (size_t)ng0 * ng0);
  size_t oL = cv.take(sizeof(cplx) * (size_t)ng0 * nip_max);
  size_t oP = cv.take(sizeof(int) * nip_max);
  size_t oR = cv.take(sizeof(int) * 4);
  size_t oD = cv.take(sizeof(double) * ng0);
  size_t oF = cv.take(sizeof(int) * 4);
  size_t oW = cv.take(sizeof(double) * (1 + nip_max));
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  char* b = (char*)base;
  cplx* X4 = (cplx*)(b + oX4);
  int rank = 0;  // x4 = Re(x2)^2/nk (:379) + pivoted Cholesky (:381-384)
  FISDF_TRY(select_pivots_dev(c, (const cplx*)x2, 1.0 / nk, ng0, nip_max, tol, X4, (int*)(b + oP),
                              (int*)(b + oR), (cplx*)(b + oL), (double*)(b + oD), (int*)(b + oF),
                              (double*)(b + oW), h_perm, &rank));
  *h_npiv = rank;
  if (h_full_rank) *h_full_rank = rank < nip_max ? 1 : 0;
  return 0;
}

int fisdf_unpack_slices(fisdf_ctx* c, const void* recv, int nrows, int nparts, const long* h_g0,
                        const long* h_ng, long ngrid, void* yT) {
  FISDF_TRY(device_guard(c));
  StageTimer tm(c, FISDF_ST_Y);
  const char* src = (const char*)recv;
  for (int p = 0; p < nparts; ++p) {
    FISDF_CHECK(h_g0[p] >= 0 && h_ng[p] >= 0 && h_g0[p] + h_ng[p] <= ngrid, "unpack: bad slice");
    if (h_ng[p] == 0 || nrows == 0) continue;
    FISDF_HIP(hipMemcpy2DAsync((char*)yT + sizeof(cplx) * h_g0[p], sizeof(cplx) * ngrid, src,
                               sizeof(cplx) * h_ng[p], sizeof(cplx) * h_ng[p], nrows,
                               hipMemcpyDeviceToDevice, c->stream));
    src += sizeof(cplx) * (size_t)h_ng[p] * nrows;
  }
  return 0;
}

// ---- input layer: Bloch AO values -------------------------------------
int fisdf_eval_ao(fisdf_ctx* c, const void* d_coords, int ng, int natm, const double* h_atoms,
                  int nsh, const int* h_sh_atom, const int* h_sh_l, const int* h_sh_nprim,
                  const double* h_exps, const double* h_coefs, int nT, const int* h_tn,
                  const int* kmesh, const double* a, double rcut, int nao, void* d_out) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(kmesh && kmesh[0] > 0 && kmesh[1] > 0 && kmesh[2] > 0, "eval_ao: bad k-mesh");
  StageTimer tm(c, FISDF_ST_AO);
  int nao_sh = 0;
  for (int i = 0; i < nsh; ++i) nao_sh += 2 * h_sh_l[i] + 1;
  FISDF_CHECK(nao_sh == nao, "eval_ao: nao does not match the shells");
  const int nimg = kmesh[0] * kmesh[1] * kmesh[2];
  Carver cv;
  const size_t oF = cv.take(sizeof(double) * (size_t)nimg * ng * nao);
  const size_t tables = 1 << 20;
  const size_t oT = cv.take(tables + sizeof(double) * 3 * (size_t)std::max(nT, 1));
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  char* b = (char*)base;
  int nao_out = 0;
  FISDF_TRY(eval_ao(c->stream, (const double*)d_coords, ng, natm, h_atoms, nsh, h_sh_atom,
                    h_sh_l, h_sh_nprim, h_exps, h_coefs, nT, h_tn, kmesh, a, rcut,
                    (double*)(b + oF), b + oT, tables + sizeof(double) * 3 * (size_t)std::max(nT, 1),
                    (cplx*)d_out, &nao_out));
  return 0;
}

int fisdf_eval_ao_band(fisdf_ctx* c, const void* d_coords, int ng, int natm, const double* h_atoms,
                       int nsh, const int* h_sh_atom, const int* h_sh_l, const int* h_sh_nprim,
                       const double* h_exps, const double* h_coefs, int nT, const int* h_tn,
                       int nkb, const double* h_kpts, const double* a, double rcut, int nao,
                       void* d_out) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(nkb > 0 && h_kpts != nullptr, "eval_ao_band: no band k-points");
  StageTimer tm(c, FISDF_ST_AO);
  int nao_sh = 0;
  for (int i = 0; i < nsh; ++i) nao_sh += 2 * h_sh_l[i] + 1;
  FISDF_CHECK(nao_sh == nao, "eval_ao_band: nao does not match the shells");
  const int one[3] = {1, 1, 1};
  Carver cv;
  const size_t oF = cv.take(sizeof(double) * (size_t)std::max(nT, 1) * ng * nao);
  const size_t tables = (1 << 20) + sizeof(double) * 3 * (size_t)std::max(nT, 1) +
                        sizeof(cplx) * (size_t)std::max(nT, 1) * nkb + sizeof(int) * (nT + 2);
  const size_t oT = cv.take(tables);
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  char* b = (char*)base;
  int nao_out = 0;
  FISDF_TRY(eval_ao(c->stream, (const double*)d_coords, ng, natm, h_atoms, nsh, h_sh_atom, h_sh_l,
                    h_sh_nprim, h_exps, h_coefs, nT, h_tn, one, a, rcut, (double*)(b + oF), b + oT,
                    tables, (cplx*)d_out, &nao_out, nkb, h_kpts));
  return 0;
}

int fisdf_gather_points(fisdf_ctx* c, const void* x0, int nk, int ng0, int nao, const int* h_perm,
                        int nip, void* X) {
  FISDF_TRY(device_guard(c));
  void* base;
  FISDF_TRY(arena_get(c, sizeof(int) * (size_t)nip, &base));
  for (int i = 0; i < nip; ++i) FISDF_CHECK(h_perm[i] >= 0 && h_perm[i] < ng0, "perm out of range");
  // through the pinned staging buffer, stream-ordered (the arena's next user is enqueued after
  // the gather on the same stream): no host synchronisation
  FISDF_TRY(upload_ints(c, h_perm, nip, (int*)base));
  FISDF_TRY(gather_points(c->stream, (const cplx*)x0, nk, ng0, nao, (const int*)base, nip, (cplx*)X));
  return 0;
}

// ---- A2 ---------------------------------------------------------------------
// FISDF_X4_DFT=0: the x4 build through the two dense Phi GEMMs (A/B on one box)
static bool x4_dft_enabled() {  // read per call (A/B in one process)
  const char* e = getenv("FISDF_X4_DFT");
  return !(e && e[0] == '0');
}

static int build_x4_on(fisdf_ctx* c, hipStream_t st, fisdf_ctx::DevBuf* wsb, const void* Xv,
                       int nip, int nao, const int kmesh[3], const double a[9], void* x4v);

int fisdf_build_x4(fisdf_ctx* c, const void* Xv, int nip, int nao, const int kmesh[3],
                   const double a[9], void* x4v) {
  FISDF_TRY(device_guard(c));
  return build_x4_on(c, c->stream, nullptr, Xv, nip, nao, kmesh, a, x4v);
}

// x4 on stream st; wsb (optional): the x2_k workspace of the register path from this grow-only
// buffer instead of the arena (whose users are ordered on c->stream only)
static int build_x4_on(fisdf_ctx* c, hipStream_t st, fisdf_ctx::DevBuf* wsb, const void* Xv,
                       int nip, int nao, const int kmesh[3], const double a[9], void* x4v) {
  StageTimer tm(c, FISDF_ST_X4, st);
  const int nk = kmesh[0] * kmesh[1] * kmesh[2];
  const cplx* phase;
  FISDF_TRY(get_phase(c, kmesh, a, &phase));
  const cplx* X = (const cplx*)Xv;
  const long nn = (long)nip * nip;
  if (nk == 1) {
    // Gamma only: Phi = 1, so x2_s = x2_k and x4 = x2_s^2 (:45) straight from the x2 GEMM's
    // epilogue with the reality monitor of :43 (the two Phi GEMMs would run with M = 1)
    FISDF_TRY(zgemm(st, OP_R, OP_T, nip, nip, nao, ONE, X, nao, 0, X, nao, 0, ZERO,
                    (cplx*)x4v, nip, 0, 1, 1, nullptr, EPI_CSQUARE, c->maximag + 0));
    return 0;
  }
  if (x4_dft_enabled() && kmesh_y_reg_applies(kmesh, nn)) {
    // the k-mesh DFT pair of :41-46 per (I, J) column in registers (the y build's kmesh_y with
    // conj output: x4_k = Phi^H x4_s, x4_s real) instead of two dense nk x nk Phi GEMMs; under
    // time reversal (X_{-k} = conj(X_k), so x2_{-k} = conj(x2_k)) x2_k only for the
    // representatives k <= -k
    const bool half = c->time_reversal;
    const int nks = half ? kmesh_half_count(kmesh) : nk;
    void* base;
    if (wsb)
      FISDF_TRY(devbuf_get(*wsb, sizeof(cplx) * (size_t)nks * nn, &base));
    else
      FISDF_TRY(arena_get(c, sizeof(cplx) * (size_t)nks * nn, &base));
    cplx* X2k = (cplx*)base;
    std::vector<int> runs = {0, nk};
    if (half) FISDF_TRY(kmesh_rep_runs(kmesh, &runs));
    // x2_k = X_k^* X_k^T  (:38), one batched GEMM per run of stored k
    for (size_t r = 0, slot = 0; r < runs.size(); r += 2) {
      const int k0 = runs[r], nb = runs[r + 1] - runs[r];
      FISDF_TRY(zgemm(st, OP_R, OP_T, nip, nip, nao, ONE, X + (long)k0 * nip * nao, nao,
                      (long)nip * nao, X + (long)k0 * nip * nao, nao, (long)nip * nao, ZERO,
                      X2k + (long)slot * nn, nip, nn, nb));
      slot += nb;
    }
    // x2_s = Phi x2_k (:41, real: max|Im| monitored, :43), x4_s = x2_s^2 (:45),
    // x4_k = Phi^H x4_s (:46) for every k
    std::vector<int> all(nk);
    for (int q = 0; q < nk; ++q) all[q] = q;
    FISDF_TRY(kmesh_y(st, X2k, nn, kmesh, all.data(), nullptr, nk, nip, (cplx*)x4v, nn, nip,
                      0, half, c->maximag + 0, true));
    return 0;
  }
  FISDF_CHECK(st == c->stream, "build_x4: the dense path runs on the context stream only");
  Carver cv;
  size_t o1 = cv.take(sizeof(cplx) * nk * nn);
  size_t o2 = cv.take(sizeof(cplx) * nk * nn);
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  cplx* X2k = (cplx*)((char*)base + o1);
  cplx* X2s = (cplx*)((char*)base + o2);
  // x2_k = X_k^* X_k^T  (:38)
  FISDF_TRY(zgemm(st, OP_R, OP_T, nip, nip, nao, ONE, X, nao, (long)nip * nao, X, nao,
                  (long)nip * nao, ZERO, X2k, nip, nn, nk));
  // x2_s = Phi x2_k  (:41), must be real (:43), squared in the GEMM's epilogue:
  // x4_s = x2_s * x2_s (:45), recording max|Im x2_s|
  FISDF_TRY(zgemm(st, OP_N, OP_N, nk, nn, nk, ONE, phase, nk, 0, X2k, nn, 0, ZERO, X2s, nn,
                  0, 1, 1, nullptr, EPI_CSQUARE, c->maximag + 0));
  // x4_k = Phi^H x4_s (:46)
  FISDF_TRY(zgemm(st, OP_C, OP_N, nk, nn, nk, ONE, phase, nk, 0, X2s, nn, 0, ZERO,
                  (cplx*)x4v, nn, 0, 1));
  return 0;
}

// ---- A3 ---------------------------------------------------------------------
int fisdf_build_y_qs(fisdf_ctx* c, const void* fv, long f_kstride, int g0, int nblk, int ngrid,
                     const void* Xv, int nip, int nao, const int kmesh[3], const double a[9],
                     const int* h_qs, int nq, void* yTv) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(g0 >= 0 && nblk >= 0 && g0 + nblk <= ngrid, "build_y: block out of range");
  StageTimer tm(c, FISDF_ST_Y);
  const int nk = kmesh[0] * kmesh[1] * kmesh[2];
  FISDF_TRY(check_qlist(h_qs, nq, nk, "build_y"));
  FISDF_CHECK(nq > 0, "build_y: empty q-list");
  const cplx* f = (const cplx*)fv;
  const cplx* X = (const cplx*)Xv;
  cplx* yT = (cplx*)yTv;
  // grid sub-blocks of ~2 GB of FX temporary (swept on MI355X at C3 after the half-k /
  // short-K changes: y 28.1 / 22.7 / 20.9 / 18.4 / 16.7 ms for 128 MB / 256 MB / 512 MB /
  // 1 GB / 2 GB — cache-sized blocks lose more to the smaller GEMM/DFT launches than they
  // gain from Infinity-Cache residency; bigger blocks slow the side-stream factorisation)
  constexpr long yblk_bytes = 2048L << 20;
  // time reversal (fisdf_set_time_reversal): fx_k only for the representatives k <= -k, the
  // others are conj(fx_{-k}) inside kmesh_y — 36 of 64 k at 4x4x4
  const bool half = c->time_reversal;
  c->y_real_slot.assign(nq, 0);
#ifdef FISDF_EXP_NOY  // timing experiment only (wrong results)
  return 0;
#endif
  if (half && nblk > 0) {
    // fused fx + k-mesh DFT where the k-mesh allows it: no fx round trip through HBM
    bool done = false;
    const size_t yw = y_fused_workspace(kmesh, nip, nao, nblk);
    // self-conjugate q stored real (half their bytes) when the caller's fit reads them so:
    // the composite build on the whole grid (c->y_real_store)
    // (a 64-bit mask of q: the fused kernel runs only for nk <= 64, so larger meshes keep it 0)
    unsigned long long rmask = 0;
    if (c->y_real_store && g0 == 0 && nblk == ngrid && nk <= 64)
      for (int i = 0; i < nq; ++i) {
        const int q = h_qs[i];
        const int i2 = q % kmesh[2], i1 = (q / kmesh[2]) % kmesh[1], i0 = q / (kmesh[1] * kmesh[2]);
        if ((2 * i0) % kmesh[0] == 0 && (2 * i1) % kmesh[1] == 0 && (2 * i2) % kmesh[2] == 0)
          rmask |= 1ull << q;
      }
    if (yw) {
      void* wb = nullptr;
      FISDF_TRY(arena_get(c, yw, &wb));
      FISDF_TRY(y_fused(c->stream, X, nip, nao, f, f_kstride, nblk, kmesh, h_qs, nq, yT,
                        (long)nip * ngrid, ngrid, g0, c->maximag + 1, (cplx*)wb, yw, rmask, &done));
    }
    if (done) {
      for (int i = 0; i < nq; ++i) c->y_real_slot[i] = (rmask >> h_qs[i]) & 1ull ? 1 : 0;
      return 0;
    }
  }
  const int nks = half ? kmesh_half_count(kmesh) : nk;
  std::vector<int> runs = {0, nk};
  if (half) FISDF_TRY(kmesh_rep_runs(kmesh, &runs));
  const long per_g = (long)nks * nip * sizeof(cplx);
  int gb = (int)std::max(64L, std::min<long>(nblk, yblk_bytes / std::max(per_g, 1L)));
  gb = std::min(gb, std::max(nblk, 1));
  // pipelined: the fx GEMM of block i+1 (main stream) runs beside the k-mesh DFT of block i
  // (aux stream) on two fx buffers — the GEMM is write/compute bound, the DFT read/write bound,
  // and neither alone saturates HBM
  const int nbuf = gb < nblk ? 2 : 1;
  Carver cv;
  size_t o1[2];
  for (int i = 0; i < nbuf; ++i) o1[i] = cv.take((size_t)per_g * gb);
  size_t oq = cv.take(sizeof(int) * (size_t)nq);
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  int* dq = (int*)((char*)base + oq);
  FISDF_TRY(upload_ints(c, h_qs, nq, dq));
  hipStream_t sk = c->stream;
  if (nbuf == 2) {
    FISDF_TRY(ensure_aux(c));
    sk = c->aux[0];
    aux_fork(c, 0);
    FISDF_HIP(hipEventRecord(c->ev_fork, c->stream));
    FISDF_HIP(hipStreamWaitEvent(sk, c->ev_fork, 0));
  }
  const int fx_epi = EPI_STREAM;  // fx is read back by the DFT only a block later
  int blk = 0;
  for (int s0 = 0; s0 < nblk; s0 += gb, ++blk) {
    const int m = std::min(gb, nblk - s0);
    const long nm = (long)nip * m;
    const int bi = blk % nbuf;
    cplx* FX = (cplx*)((char*)base + o1[bi]);
    // buffer bi is free once the DFT of block blk-2 has read it
    if (nbuf == 2 && blk >= 2) FISDF_HIP(hipStreamWaitEvent(c->stream, c->ev_ybuf[2 + bi], 0));
    // fx_k^T = X_k f_k^H  -> FX[slot(k)][I][g]   (:76, transposed layout), one batched GEMM
    // per run of consecutive stored k
    for (size_t r = 0, slot = 0; r < runs.size(); r += 2) {
      const int k0 = runs[r], nb = runs[r + 1] - runs[r];
      FISDF_TRY(zgemm(c->stream, OP_N, OP_C, nip, m, nao, ONE, X + (long)k0 * nip * nao, nao,
                      (long)nip * nao, f + (long)k0 * f_kstride + (long)s0 * nao, nao, f_kstride,
                      ZERO, FX + (long)slot * nm, m, nm, nb, 1, nullptr, fx_epi));
      slot += nb;
    }
    if (nbuf == 2) {
      FISDF_HIP(hipEventRecord(c->ev_ybuf[bi], c->stream));
      FISDF_HIP(hipStreamWaitEvent(sk, c->ev_ybuf[bi], 0));
    }
    // fx_s = Phi fx_k (:79, real :81), y_s = fx_s^2 (:83), y_k = Phi^T y_s (:84) for the
    // listed q, written into yT[slot][I][g0+s0+g] (:85): separable k-mesh DFTs
    FISDF_TRY(kmesh_y(sk, FX, nm, kmesh, h_qs, dq, nq, m, yT, (long)nip * ngrid, ngrid,
                      (long)g0 + s0, half, c->maximag + 1));
    if (nbuf == 2) FISDF_HIP(hipEventRecord(c->ev_ybuf[2 + bi], sk));
  }
  if (nbuf == 2) FISDF_TRY(aux_join(c, 0));  // later work on the main stream (the fit, the
                                             // arena's next user) sees y
  return 0;
}

int fisdf_build_y(fisdf_ctx* c, const void* fv, long f_kstride, int g0, int nblk, int ngrid,
                  const void* Xv, int nip, int nao, const int kmesh[3], const double a[9],
                  int q0, int q1, void* yTv) {
  const int nk = kmesh[0] * kmesh[1] * kmesh[2];
  FISDF_CHECK(0 <= q0 && q0 < q1 && q1 <= nk, "build_y: bad q range");
  std::vector<int> qs = q_range(q0, q1);
  return fisdf_build_y_qs(c, fv, f_kstride, g0, nblk, ngrid, Xv, nip, nao, kmesh, a, qs.data(),
                          (int)qs.size(), yTv);
}

// ---- A4 ---------------------------------------------------------------------
// rank copies, pivot-order factor (identity-padded to nip so the small back-substitutions of
// all q run as one batch), diagonal-block inverses and the merged TRSM operator, on stream s
// need_linv: the diagonal-block inverses of Lp (trsm_blocked, used only when some rank < nip;
// the unpivoted path is full-rank by construction — a failing slot is refactored, and this
// rerun, by factor_pivoted_slots)
int factor_finish(fisdf_ctx* c, hipStream_t s, const int* rank_dev_src, bool need_linv) {
  const int nk = c->f_nk, nip = c->f_nip, nb = c->f_nb, nblk = (nip + nb - 1) / nb;
  const long nn = (long)nip * nip;
  FISDF_HIP(hipMemcpyAsync(c->f_rank_pinned, rank_dev_src, sizeof(int) * nk, hipMemcpyDeviceToHost, s));
  FISDF_HIP(hipMemcpyAsync(c->f_rank_dev, rank_dev_src, sizeof(int) * nk, hipMemcpyDeviceToDevice, s));
  // ranks and pivots are known here: fisdf_factor_x4_wait returns on this event, and the fit
  // starts its FFTs while the operators below are still being built (it waits on ev_fac
  // per lane before its first TRSM)
  FISDF_HIP(hipEventRecord(c->ev_chol, s));
  // the operators of slots [z0, z0 + nz): every kernel below works per slot (strides from the
  // batch index; split-K from the block row's shape only), so a slot's operators do not depend on
  // which slots share the launch
  const long sLi = (long)nblk * nb * nb;
  auto operators = [&](int z0, int nz) -> int {
    if (nz <= 0) return 0;
    FISDF_TRY(gather_lp(s, c->f_L + z0 * nn, nip, nip, c->f_piv + (long)z0 * nip,
                        c->f_rank_dev + z0, nip, c->f_Lp + z0 * nn, nz));
    if (need_linv)
      FISDF_TRY(trinv_blocks(s, c->f_Lp + z0 * nn, nip, nip, nn, nb, sLi, c->f_Linv + z0 * sLi,
                             nz));
    FISDF_TRY(build_trsm_q(s, c->f_Lp + z0 * nn, nip, nn, c->f_Q + z0 * nn, nz, GEMM_FULL));
    // L^{-1} by the same block-row substitution applied to the identity (the fit then applies it
    // as one lower-triangular GEMM over the grid; J/K within 2-3x of the TRSM's rounding,
    // tests/experiments/explicit_tri_inverse.py)
    FISDF_TRY(set_identity(s, c->f_Li + z0 * nn, nip, nz));
    FISDF_TRY(trsm_merged_batched(s, c->f_Q + z0 * nn, nn, nip, c->f_Li + z0 * nn, nip, nn, nip,
                                   nz, true, c->f_ksw, c->f_ksw_elems));
    return 0;
  };
  // the first fitted slots' operators first (ev_fac_early): their lanes start the fit while the
  // rest are still being built.  FISDF_FAC_EARLY (slots, read per call; 0 off)
  const int early = [&] {
    const char* e = getenv("FISDF_FAC_EARLY");
    const int v = e ? atoi(e) : 2;
    return (v > 0 && v < nk) ? v : 0;
  }();
  c->f_early = early;
  if (early) {
    FISDF_TRY(operators(0, early));
    FISDF_HIP(hipEventRecord(c->ev_fac_early, s));
  }
  FISDF_TRY(operators(early, nk - early));
  return 0;
}

bool pivoted_fit_forced() {
  static const bool on = [] {
    const char* e = getenv("FISDF_PIVOTED_FIT");
    return e && e[0] == '1';
  }();
  return on;
}

// the greedy pivoted (rank-revealing) factorisation of the staged x4 (fallback / forced)
int factor_pivoted(fisdf_ctx* c, hipStream_t s) {
  const int nk = c->f_nk, nip = c->f_nip;
  const long nn = (long)nip * nip;
  char* b = (char*)c->f_scratch;
  Carver cv;
  size_t oR = cv.take(sizeof(int) * nk);
  size_t oD = cv.take(sizeof(double) * (size_t)nk * nip);
  size_t oF = cv.take(sizeof(int) * nk);
  size_t oW = cv.take(sizeof(double) * (size_t)nk * (1 + nip));
  void* trail = nullptr;
  FISDF_TRY(devbuf_get(c->ws_side_b, sizeof(cplx) * pchol_trail_elems(nip, nk), &trail));
  FISDF_TRY(pchol(s, c->f_x4s, nip, nn, nip, nk, nip, c->f_tol, 0.0, c->f_L, c->f_piv,
                  (int*)(b + oR), (double*)(b + oD), (int*)(b + oF), (double*)(b + oW),
                  (cplx*)trail));
  c->f_used_pivoted = true;
  return factor_finish(c, s, (const int*)(b + oR), true);
}

// the greedy pivoted factorisation of only the listed slots (those whose unpivoted Cholesky
// failed the full-rank test): gathered into a contiguous batch, factored, scattered back, so a
// q's factor does not depend on which other q share the batch (1-GPU and sharded builds agree)
int factor_pivoted_slots(fisdf_ctx* c, hipStream_t s, const std::vector<int>& slots) {
  const int nk = c->f_nk, nip = c->f_nip, nf = (int)slots.size();
  const long nn = (long)nip * nip;
  char* b = (char*)c->f_scratch;
  Carver cv;
  size_t oR = cv.take(sizeof(int) * nk);
  size_t oD = cv.take(sizeof(double) * (size_t)nk * nip);
  size_t oF = cv.take(sizeof(int) * nk);
  size_t oW = cv.take(sizeof(double) * (size_t)nk * (1 + nip));
  size_t oU = cv.take(sizeof(int) * nk);  // the unpivoted path's per-slot ranks
  void* wa = nullptr;
  FISDF_TRY(devbuf_get(c->ws_side_a, sizeof(cplx) * 2 * nf * nn + sizeof(int) * (size_t)nf * nip, &wa));
  cplx* A = (cplx*)wa;
  cplx* L = A + nf * nn;
  int* P = (int*)(L + nf * nn);
  void* trail = nullptr;
  FISDF_TRY(devbuf_get(c->ws_side_b, sizeof(cplx) * pchol_trail_elems(nip, nf), &trail));
  for (int j = 0; j < nf; ++j)
    FISDF_HIP(hipMemcpyAsync(A + j * nn, c->f_x4s + slots[j] * nn, sizeof(cplx) * nn,
                             hipMemcpyDeviceToDevice, s));
  FISDF_TRY(pchol(s, A, nip, nn, nip, nf, nip, c->f_tol, 0.0, L, P, (int*)(b + oR),
                  (double*)(b + oD), (int*)(b + oF), (double*)(b + oW), (cplx*)trail));
  for (int j = 0; j < nf; ++j) {
    const int i = slots[j];
    FISDF_HIP(hipMemcpyAsync(c->f_L + i * nn, L + j * nn, sizeof(cplx) * nn, hipMemcpyDeviceToDevice, s));
    FISDF_HIP(hipMemcpyAsync(c->f_piv + (long)i * nip, P + (long)j * nip, sizeof(int) * nip,
                             hipMemcpyDeviceToDevice, s));
    FISDF_HIP(hipMemcpyAsync((int*)(b + oU) + i, (int*)(b + oR) + j, sizeof(int),
                             hipMemcpyDeviceToDevice, s));
  }
  c->f_used_pivoted = true;
  return factor_finish(c, s, (const int*)(b + oU), true);
}

static int ensure_side(fisdf_ctx* c) {
  // 1-GPU build: the factor chain (small latency-bound kernels) on the device's LEAST priority,
  // the y build and the fit go first and the chain fills the gaps (at normal priority the factor
  // ends 2 ms sooner but the C3 step is 5 ms slower).  A k-shard's y build is 1/N as long, so
  // there the chain is the critical path to the first TRSM and runs at the GREATEST priority
  // (fisdf_set_factor_priority).  One side stream at a time: an extra stream changes
  // how HIP maps the context's streams onto the process's hardware queues (4 here), and two
  // fit lanes sharing a queue serialise (C3 +5 ms/step measured with a second side stream)
  // One padding stream (given one small memset so the runtime maps it onto a hardware queue)
  // before the side stream, in the place the cooperative launch's own queue takes when the
  // selection is launched cooperatively: without it, with the plain launch, the fit's two lanes
  // serialise (C3 90.3 vs 81.3 ms/step; profiles/r06/lanes/).  FISDF_PAD_QUEUES=n overrides.
  static const int pad_env = getenv("FISDF_PAD_QUEUES") ? atoi(getenv("FISDF_PAD_QUEUES"))
                                                        : (coop_launch_enabled() ? 0 : 1);
  if (pad_env > 0 && c->pad.empty()) {
    if (!c->pad_buf) FISDF_HIP(hipMalloc(&c->pad_buf, 256));
    for (int i = 0; i < pad_env && i < 8; ++i) {
      hipStream_t p = nullptr;
      FISDF_HIP(hipStreamCreateWithFlags(&p, hipStreamNonBlocking));
      FISDF_HIP(hipMemsetAsync(c->pad_buf, 0, 256, p));
      FISDF_HIP(hipStreamSynchronize(p));
      c->pad.push_back(p);
    }
  }
  if (c->side && c->side_hi != c->factor_hi) {
    FISDF_HIP(hipStreamSynchronize(c->side));
    FISDF_HIP(hipStreamDestroy(c->side));
    c->side = nullptr;
  }
  if (!c->side) {
    int least = 0, greatest = 0;
    FISDF_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    FISDF_HIP(hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking,
                                          c->factor_hi ? greatest : least));
    c->side_hi = c->factor_hi;
  }
  if (!c->ev_x4) {
    FISDF_HIP(hipEventCreateWithFlags(&c->ev_x4, hipEventDisableTiming));
    FISDF_HIP(hipEventCreateWithFlags(&c->ev_fac, hipEventDisableTiming));
    FISDF_HIP(hipEventCreateWithFlags(&c->ev_fac_early, hipEventDisableTiming));
    FISDF_HIP(hipEventCreateWithFlags(&c->ev_chol, hipEventDisableTiming));
  }
  return 0;
}

int fisdf_set_factor_priority(fisdf_ctx* c, int high) {
  FISDF_TRY(ctx_guard(c));
  FISDF_CHECK(c != nullptr && (high == 0 || high == 1), "set_factor_priority: 0 or 1");
  c->factor_hi = high;
  return 0;
}

int fisdf_factor_x4_mark(fisdf_ctx* c) {
  FISDF_TRY(device_guard(c));
  if (c->f_pending) FISDF_TRY(fisdf_factor_x4_wait(c, nullptr));
  FISDF_TRY(ensure_side(c));
  FISDF_HIP(hipEventRecord(c->ev_x4, c->stream));
  c->x4_marked = true;
  return 0;
}

int fisdf_factor_x4_async(fisdf_ctx* c, const void* x4all, const int* h_qs, int nq, int nip,
                          double tol_rel, const int* kmesh) {
  FISDF_TRY(device_guard(c));
  const int nk = nq;
  FISDF_CHECK(nk > 0 && nip > 0, "factor_x4: bad sizes");
  FISDF_TRY(check_qlist(h_qs, nq, 1 << 30, "factor_x4"));
  if (c->f_pending) FISDF_TRY(fisdf_factor_x4_wait(c, nullptr));
  if (!c->x4_marked) FISDF_TRY(ensure_side(c));
  const int nb = c->f_nb;
  const int nblk = (nip + nb - 1) / nb;
  const long nn = (long)nip * nip;
  // the factor buffers are kept between builds of the same shape (hipFree synchronises the
  // device and the ~1.2 GB re-allocation cost ~2 ms of idle GPU per C3 step)
  if (c->f_L && c->f_cap_nip == nip && c->f_cap_nk >= nk) {
    c->f_rank.clear();
    c->f_qs.clear();
    c->f_real.clear();
  } else {
  FISDF_TRY(free_factors(c));
  c->f_cap_nk = nk;
  c->f_cap_nip = nip;
  FISDF_HIP(hipMalloc(&c->f_x4s, sizeof(cplx) * nk * nn));
  FISDF_HIP(hipMalloc(&c->f_L, sizeof(cplx) * nk * nn));
  FISDF_HIP(hipMalloc(&c->f_Lp, sizeof(cplx) * nk * nn));
  FISDF_HIP(hipMalloc(&c->f_Linv, sizeof(cplx) * (size_t)nk * nblk * nb * nb));
  FISDF_HIP(hipMalloc(&c->f_Q, sizeof(cplx) * nk * nn));
  FISDF_HIP(hipMalloc(&c->f_Li, sizeof(cplx) * nk * nn));
  // split-K partials of the L^{-1} substitution: the whole batch in one launch per block row when
  // that fits 16M elements (256 MB), else trsm_merged_batched runs sub-batches (a matrix's split
  // depends on its shape only, so its arithmetic is unchanged)
  c->f_ksw_elems = std::max({1L, trsm_split_work_elems(nip, 1),
                             std::min(trsm_split_work_elems(nip, nk), 16L << 20)});
  FISDF_HIP(hipMalloc(&c->f_ksw, sizeof(cplx) * c->f_ksw_elems));
  FISDF_HIP(hipMalloc(&c->f_piv, sizeof(int) * (size_t)nk * nip));
  FISDF_HIP(hipMalloc(&c->f_rank_dev, sizeof(int) * nk));
  FISDF_HIP(hipHostMalloc((void**)&c->f_rank_pinned, sizeof(int) * nk, hipHostMallocDefault));
  FISDF_HIP(hipHostMalloc((void**)&c->f_fail_pinned, sizeof(int) * nk, hipHostMallocDefault));
  FISDF_HIP(hipHostMalloc((void**)&c->f_qr_pinned, sizeof(int) * 2 * nk, hipHostMallocDefault));
  FISDF_HIP(hipMalloc(&c->f_qr_dev, sizeof(int) * 2 * nk));
  }
  // scratch: pivoted pchol work, or the unpivoted path's rank/fail flags + block inverses
  Carver cv;
  cv.take(sizeof(int) * nk);
  cv.take(sizeof(double) * (size_t)nk * nip);
  cv.take(sizeof(int) * nk);
  cv.take(sizeof(double) * (size_t)nk * (1 + nip));
  size_t oU = cv.take(sizeof(int) * nk);                                   // unpivoted rank
  size_t oFl = cv.take(sizeof(int) * nk);                                  // unpivoted fail
  size_t oWk = cv.take(sizeof(cplx) * (size_t)nk * 4096 + sizeof(double) * nk);
  if (cv.off > c->f_scratch_size) {
    if (c->f_scratch) FISDF_HIP(hipFree(c->f_scratch));
    FISDF_HIP(hipMalloc(&c->f_scratch, cv.off));
    c->f_scratch_size = cv.off;
  }
  char* b = (char*)c->f_scratch;
  c->f_qs.assign(h_qs, h_qs + nq);
  c->f_real.assign(nq, 0);
  for (int i = 0; kmesh && i < nq; ++i) c->f_real[i] = self_conjugate(kmesh, h_qs[i]) ? 1 : 0;
  c->f_nk = nk;
  c->f_nip = nip;
  c->f_tol = tol_rel;
  c->f_used_pivoted = false;
  // the side stream starts once everything enqueued on `stream` so far (x4) is done; work
  // enqueued on `stream` after this call (the y build) runs concurrently
  // (or at fisdf_factor_x4_mark, so that work enqueued between the two calls — the y build —
  // is not waited for, and the factor's host-blocking rank read-back cannot delay its launch)
  if (!c->x4_marked) FISDF_HIP(hipEventRecord(c->ev_x4, c->stream));
  c->x4_marked = false;
  FISDF_HIP(hipStreamWaitEvent(c->side, c->ev_x4, 0));
  StageTimer tm(c, FISDF_ST_FACTOR, c->side);
  hipStream_t s = c->side;
  // stage the listed x4_q in one pass (self-conjugate q: x4_q = Phi[:,q]^H x4_s is real up to
  // rounding); the unpivoted path factors its copy in f_L in place.  The pinned q-list is
  // rewritten only here, after the previous factorisation was waited for (f_pending)
  const bool pivoted = c->force_pivoted == 1 || (c->force_pivoted < 0 && pivoted_fit_forced()) ||
                       c->fit_mode == FISDF_FIT_SVD;
  for (int i = 0; i < nq; ++i) {
    c->f_qr_pinned[i] = h_qs[i];
    c->f_qr_pinned[nq + i] = c->f_real[i];
  }
  FISDF_HIP(hipMemcpyAsync(c->f_qr_dev, c->f_qr_pinned, sizeof(int) * 2 * nq, hipMemcpyHostToDevice, s));
  FISDF_TRY(stage_x4(s, (const cplx*)x4all, c->f_qr_dev, nq, nn, c->f_x4s, pivoted ? nullptr : c->f_L));
  if (pivoted) {
    FISDF_TRY(factor_pivoted(c, s));
    c->f_check_fail = false;
  } else {
    // full-rank fast path: unpivoted blocked Cholesky (all pivots > tol_rel * max diag is the
    // same full-rank verdict the rank-revealing pivoted factorisation gives); any matrix that
    // fails it is redone by the pivoted pchol in fisdf_factor_x4_wait
    FISDF_TRY(chol_unpivoted(s, c->f_L, nip, nk, tol_rel, c->f_piv, (int*)(b + oU),
                             (int*)(b + oFl), (cplx*)(b + oWk)));
    FISDF_HIP(hipMemcpyAsync(c->f_fail_pinned, b + oFl, sizeof(int) * nk, hipMemcpyDeviceToHost, s));
    FISDF_TRY(factor_finish(c, s, (const int*)(b + oU), false));
    c->f_check_fail = true;
  }
  FISDF_HIP(hipEventRecord(c->ev_fac, s));
  c->f_pending = true;
  return 0;
}

int fisdf_set_pivoted_fit(fisdf_ctx* c, int mode) {
  FISDF_TRY(ctx_guard(c));
  FISDF_CHECK(c != nullptr && mode >= -1 && mode <= 1, "set_pivoted_fit: bad mode");
  c->force_pivoted = mode;
  return 0;
}

int fisdf_set_half_grid(fisdf_ctx* c, int mode) {
  FISDF_TRY(ctx_guard(c));
  FISDF_CHECK(c != nullptr && mode >= -1 && mode <= 1, "set_half_grid: mode must be -1, 0 or 1");
  c->half_grid = mode;
  return 0;
}

int fisdf_set_fit_mode(fisdf_ctx* c, int mode) {
  FISDF_TRY(ctx_guard(c));
  FISDF_CHECK(c != nullptr && mode >= FISDF_FIT_LSTSQ && mode <= FISDF_FIT_BASIC,
              "set_fit_mode: mode must be FISDF_FIT_LSTSQ, FISDF_FIT_SVD or FISDF_FIT_BASIC");
  c->fit_mode = mode;
  return 0;
}

int fisdf_min_norm_info(fisdf_ctx* c, int* h_nslots) {
  FISDF_TRY(ctx_guard(c));
  FISDF_CHECK(c != nullptr, "null context");
  int n = 0;
  for (char v : c->f_cod) n += v ? 1 : 0;
  if (h_nslots) *h_nslots = n;
  return 0;
}

int fisdf_set_omega(fisdf_ctx* c, double omega) {
  FISDF_TRY(ctx_guard(c));
  FISDF_CHECK(c != nullptr && std::isfinite(omega), "set_omega: omega must be finite");
  c->omega = omega;
  return 0;
}

int fisdf_set_time_reversal(fisdf_ctx* c, int on) {
  FISDF_TRY(ctx_guard(c));
  FISDF_CHECK(c != nullptr && (on == 0 || on == 1), "set_time_reversal: on must be 0 or 1");
  c->time_reversal = on == 1;
  return 0;
}

int fisdf_set_fit_lanes(fisdf_ctx* c, int lanes) {
  FISDF_TRY(ctx_guard(c));
  FISDF_CHECK(c != nullptr && lanes >= 0 && lanes <= 4, "set_fit_lanes: lanes must be 0..4");
  c->lanes = lanes;
  return 0;
}

int fisdf_set_fit_pipe(fisdf_ctx* c, int mode, int depth) {
  FISDF_TRY(ctx_guard(c));
  FISDF_CHECK(c != nullptr && mode >= -1 && mode <= 1 && depth >= 0 && depth <= 64,
              "set_fit_pipe: mode must be -1..1, depth 0..64");
  c->pipe_mode = mode;
  c->pipe_depth = depth;
  return 0;
}

}  // extern "C"

namespace {
// y of the next fit's j-th q has landed once the work enqueued so far on `st` is done
int mark_y_ready_on(fisdf_ctx* c, int j, hipStream_t st) {
  FISDF_CHECK(j >= 0 && j < 4096, "mark_y_ready: bad index");
  while ((int)c->ev_ready.size() <= j) {
    hipEvent_t e;
    FISDF_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->ev_ready.push_back(e);
  }
  if ((int)c->ready_marked.size() <= j) c->ready_marked.resize(j + 1, 0);
  FISDF_HIP(hipEventRecord(c->ev_ready[j], st));
  c->ready_marked[j] = 1;
  return 0;
}

int set_y_slices_on(fisdf_ctx* c, int j, const void* recv, int nparts, const long* h_g0,
                    const long* h_ng, hipStream_t st) {
  FISDF_CHECK(recv != nullptr && nparts >= 1 && nparts <= 4096, "set_y_slices: bad piece");
  std::vector<long> sl;
  for (int p = 0; p < nparts; ++p) {
    FISDF_CHECK(h_g0[p] >= 0 && h_ng[p] >= 0, "set_y_slices: bad slice");
    sl.push_back(h_g0[p]);
    sl.push_back(h_ng[p]);
  }
  bool any = false;
  for (const cplx* pc : c->y_piece) any = any || pc != nullptr;
  FISDF_CHECK(!any || sl == c->y_slices, "set_y_slices: every piece of a call has one layout");
  c->y_slices = sl;
  if ((int)c->y_piece.size() <= j) c->y_piece.resize(j + 1, nullptr);
  c->y_piece[j] = (const cplx*)recv;
  return mark_y_ready_on(c, j, st);
}
}  // namespace

extern "C" {

int fisdf_mark_y_ready(fisdf_ctx* c, int j) {
  FISDF_TRY(device_guard(c));
  return mark_y_ready_on(c, j, c->stream);
}

int fisdf_set_y_slices(fisdf_ctx* c, int j, const void* recv, int nparts, const long* h_g0,
                       const long* h_ng) {
  FISDF_TRY(device_guard(c));
  return set_y_slices_on(c, j, recv, nparts, h_g0, h_ng, c->stream);
}

int fisdf_fit_info(fisdf_ctx* c, int* h_lanes, int* h_pipe_depth) {
  FISDF_TRY(ctx_guard(c));
  FISDF_CHECK(c != nullptr, "null context");
  if (h_lanes) *h_lanes = c->last_fit_lanes;
  if (h_pipe_depth) *h_pipe_depth = c->last_fit_pipe;
  return 0;
}

int fisdf_reserve_workspace(fisdf_ctx* c, size_t bytes) {
  FISDF_TRY(device_guard(c));
  void* base;
  return arena_get(c, bytes, &base);
}

int fisdf_factor_info(fisdf_ctx* c, int* h_used_pivoted) {
  FISDF_TRY(ctx_guard(c));
  FISDF_CHECK(c != nullptr, "null context");
  if (h_used_pivoted) *h_used_pivoted = c->f_used_pivoted ? 1 : 0;
  return 0;
}

// Minimum-norm operators (fisdf_set_fit_mode) of the slots that need one, on the side stream
// once the ranks are known: a rank-deficient x4_q (FISDF_FIT_LSTSQ) or every q (FISDF_FIT_SVD).
// gelsy (fftisdf.py:108) returns the minimum-norm least-squares solution; the basic solution
// of the rank-revealing factor differs from it in the null space (tests/experiments/
// min_norm_fit.py).  Synchronous: the Cholesky breakdown flags of each CholeskyQR pass are read.
static int build_min_norm(fisdf_ctx* c, bool* built) {
  *built = false;
  const int nk = c->f_nk, nip = c->f_nip;
  const long nn = (long)nip * nip;
  c->f_cod.assign(nk, 0);
  int ncod = 0;
  for (int q = 0; q < nk; ++q) {
    const int r = c->f_rank[q];
    const bool cod = r > 0 && (c->fit_mode == FISDF_FIT_SVD || (c->fit_mode == FISDF_FIT_LSTSQ && r < nip));
    c->f_cod[q] = cod ? 1 : 0;
    ncod += cod ? 1 : 0;
  }
  if (ncod == 0) return 0;
  if (!c->f_M) FISDF_HIP(hipMalloc(&c->f_M, sizeof(cplx) * (size_t)c->f_cap_nk * nn));
  if (!c->f_nip_dev) FISDF_HIP(hipMalloc(&c->f_nip_dev, sizeof(int)));
  FISDF_HIP(hipMemcpy(c->f_nip_dev, &nip, sizeof(int), hipMemcpyHostToDevice));
  hipStream_t s = c->side;
  const size_t wb = (min_norm_work_bytes(nip, nip) + 255) / 256 * 256;
  void* wv = nullptr;
  FISDF_TRY(devbuf_get(c->ws_side_b, wb + sizeof(int) * 3 * (size_t)nk, &wv));
  char* work = (char*)wv;
  int* fail = (int*)(work + wb);
  for (int q = 0; q < nk; ++q)
    if (c->f_cod[q])
      FISDF_TRY(min_norm_operator(s, c->f_L + q * nn, nip, nip, c->f_piv + (long)q * nip,
                                  c->f_rank[q], c->f_M + q * nn, nip, work, fail + 3 * q));
  std::vector<int> hf(3 * (size_t)nk, 0);
  FISDF_HIP(hipMemcpyAsync(hf.data(), fail, sizeof(int) * 3 * nk, hipMemcpyDeviceToHost, s));
  FISDF_HIP(hipEventRecord(c->ev_fac, s));
  FISDF_HIP(hipEventSynchronize(c->ev_fac));
  for (int q = 0; q < nk; ++q)
    FISDF_CHECK(!c->f_cod[q] || (hf[3 * q] == 0 && hf[3 * q + 1] == 0 && hf[3 * q + 2] == 0),
                "min-norm fit: CholeskyQR breakdown of the rank-revealing factor");
  *built = true;
  return 0;
}

int fisdf_factor_x4_wait(fisdf_ctx* c, int* h_ranks) {
  FISDF_TRY(device_guard(c));
  if (c->f_pending) {
    // ranks, pivots and the full-rank verdict are ready at ev_chol; the operators built
    // after it (L^-1 etc.) are waited for on the device (ev_fac, by the fit)
    FISDF_HIP(hipEventSynchronize(c->ev_chol));
    bool redone = false;
    if (c->f_check_fail) {
      std::vector<int> failed;
      for (int q = 0; q < c->f_nk; ++q)
        if (c->f_fail_pinned[q] != 0) failed.push_back(q);
      c->f_check_fail = false;
      if (!failed.empty()) {  // not numerically full rank at tol: rank-revealing factorisation
        FISDF_TRY(factor_pivoted_slots(c, c->side, failed));
        FISDF_HIP(hipEventRecord(c->ev_fac, c->side));
        FISDF_HIP(hipEventSynchronize(c->ev_fac));
        redone = true;
      }
    }
    c->f_rank.assign(c->f_rank_pinned, c->f_rank_pinned + c->f_nk);
    if (redone) FISDF_HIP(hipStreamWaitEvent(c->stream, c->ev_fac, 0));
    c->f_fac_unjoined = !redone;
    c->f_pending = false;
    bool built = false;
    FISDF_TRY(build_min_norm(c, &built));
    if (built) c->f_fac_unjoined = true;  // ev_fac re-recorded after the operators
  }
  if (h_ranks)
    for (int q = 0; q < c->f_nk; ++q) h_ranks[q] = c->f_rank[q];
  return 0;
}

// the main stream waits for every factor operator (the fit joins per lane instead)
static int join_factors(fisdf_ctx* c) {
  if (c->f_fac_unjoined) {
    FISDF_HIP(hipStreamWaitEvent(c->stream, c->ev_fac, 0));
    c->f_fac_unjoined = false;
  }
  return 0;
}

int fisdf_factor_x4_qs(fisdf_ctx* c, const void* x4all, const int* h_qs, int nq, int nip,
                       double tol_rel, const int* kmesh, int* h_ranks) {
  FISDF_TRY(fisdf_factor_x4_async(c, x4all, h_qs, nq, nip, tol_rel, kmesh));
  FISDF_TRY(fisdf_factor_x4_wait(c, h_ranks));
  return join_factors(c);
}

int fisdf_factor_x4(fisdf_ctx* c, const void* x4v, int q0, int q1, int nip, double tol_rel,
                    int* h_ranks) {
  FISDF_CHECK(q0 >= 0 && q1 > q0, "factor_x4: bad sizes");
  std::vector<int> qs = q_range(q0, q1);
  return fisdf_factor_x4_qs(c, x4v, qs.data(), (int)qs.size(), nip, tol_rel, nullptr, h_ranks);
}

// device table of where each plane i0 of a row lives inside an all-to-all piece (the concat over
// slices p of (rows, ng_p) blocks of grid points [g0_p, g0_p + ng_p)); cached per layout
static int plane_table(fisdf_ctx* c, const int mesh[3], int rows, const PlaneRef** out) {
  const long P = (long)mesh[1] * mesh[2], n0 = mesh[0];
  FISDF_CHECK(fft3d_reads_slices(mesh[0], mesh[1], mesh[2]),
              "fit_coulomb: sliced y needs a mesh the plane FFT kernels take");
  std::vector<long> key = c->y_slices;
  key.insert(key.end(), {(long)mesh[0], (long)mesh[1], (long)mesh[2], (long)rows});
  auto it = c->plane_cache.find(key);
  if (it == c->plane_cache.end()) {
    std::vector<PlaneRef> h(n0, PlaneRef{-1, 0});
    long off = 0;
    for (size_t p = 0; p + 1 < c->y_slices.size(); p += 2) {
      const long g0 = c->y_slices[p], ng = c->y_slices[p + 1];
      FISDF_CHECK(g0 % P == 0 && ng % P == 0 && g0 + ng <= n0 * P,
                  "fit_coulomb: y slices must be whole planes of the mesh");
      for (long i0 = g0 / P; i0 < (g0 + ng) / P; ++i0) h[i0] = PlaneRef{off + (i0 * P - g0), ng};
      off += (long)rows * ng;
    }
    for (long i0 = 0; i0 < n0; ++i0) FISDF_CHECK(h[i0].base >= 0, "fit_coulomb: y slices leave a plane out");
    PlaneRef* d = nullptr;
    FISDF_HIP(hipMalloc(&d, sizeof(PlaneRef) * n0));
    FISDF_HIP(hipMemcpy(d, h.data(), sizeof(PlaneRef) * n0, hipMemcpyHostToDevice));
    it = c->plane_cache.emplace(key, d).first;
  }
  *out = it->second;
  return 0;
}

// ---- A4 + A5 ------------------------------------------------------------------
int fisdf_fit_coulomb_qs(fisdf_ctx* c, const int* h_qs, int nq, const void* yTv, int nip,
                         const int mesh[3], const int kmesh[3], const double a[9], void* Wqv) {
  FISDF_TRY(device_guard(c));
  // the marks belong to this call: cleared on every return, error returns included, so a failed
  // call cannot leave the next one running in 'ready' mode against stale events
  struct ClearMarks {
    fisdf_ctx* c;
    ~ClearMarks() {
      c->ready_marked.assign(c->ready_marked.size(), 0);
      c->y_piece.clear();
    }
  } clear_marks{c};
  const int nk = kmesh[0] * kmesh[1] * kmesh[2];
  FISDF_TRY(check_qlist(h_qs, nq, nk, "fit_coulomb"));
  // the listed q must be a contiguous run of the factored q-list (slots s0 .. s0+nq-1): the
  // whole shard at once, or one q at a time as its y arrives (overlapped all-to-all)
  FISDF_CHECK(c->f_nip == nip && nq >= 1, "fit_coulomb: call fisdf_factor_x4 first");
  const auto it0 = std::find(c->f_qs.begin(), c->f_qs.end(), h_qs[0]);
  FISDF_CHECK(it0 != c->f_qs.end() && (it0 - c->f_qs.begin()) + nq <= (long)c->f_qs.size() &&
                  std::equal(h_qs, h_qs + nq, it0),
              "fit_coulomb: the q-list must be a contiguous run of the factored q-list");
  const int s0 = (int)(it0 - c->f_qs.begin());
  auto piece_of = [&](int lq) -> const cplx* {
    return lq < (int)c->y_piece.size() ? c->y_piece[lq] : nullptr;
  };
  const long ngrid = (long)mesh[0] * mesh[1] * mesh[2];
  const long nn = (long)nip * nip;
  const int nb = c->f_nb;
  const int nblk = (nip + nb - 1) / nb;
  CellGeom g;
  lattice(a, g);
  const double vol = cell_volume(a);
  const cplx* yT = (const cplx*)yTv;
  cplx* Wq = (cplx*)Wqv;
  // q are processed on NL "lanes" (the main stream and aux streams), each with its own
  // workspaces, so one q's HBM-bound FFT and memory-stalled HERK overlap another q's
  // MFMA-bound TRSM on the same CUs
  int NL = std::min(nq, c->lanes > 0 ? c->lanes : env_fit_lanes());
  // Pipelined FFTs (default with >= 2 lanes; fisdf_set_fit_pipe / FISDF_FIT_PIPE=0 turn it
  // off): the HBM-bound FFTs run on their own stream into a ring of D Yhat slots, ahead of the
  // MFMA lanes, which wait per q on its event — the FFTs then overlap TRSM/HERK work instead of
  // meeting another lane's FFT.  A slot is reused once the lane that read it records its
  // `free` event, so the working set is D x nip x ngrid (D = lanes + 2 by default) whatever
  // nq is.  With a single MFMA lane it is slower (C3 107.8 vs 100.9 ms/step), so one lane
  // keeps the FFT in-lane.
  const int pipe_mode = c->pipe_mode >= 0 ? c->pipe_mode : env_fit_pipe();
  bool pipe = pipe_mode != 0 && nq > 1 && NL > 1;
  // sharded build (fisdf_mark_y_ready): y of the call's j-th q lands at ev_ready[j] on the main
  // stream (all-to-all piece + unpack); the lanes then run on the aux streams only and each q
  // starts as soon as its own piece is there, one call for the whole shard
  int nready = 0;
  for (int lq = 0; lq < nq; ++lq)
    nready += (lq < (int)c->ready_marked.size() && c->ready_marked[lq]) ? 1 : 0;
  FISDF_CHECK(nready == 0 || nready == nq, "fit_coulomb: mark every q of the call ready, or none");
  const bool ready = nready > 0;
  if (pipe) NL = std::min(NL, ready ? 2 : 3);  // aux[2] is the FFT stream
  if (ready) NL = std::min(NL, 3);
  int D = pipe ? std::min(nq, c->pipe_depth > 0 ? c->pipe_depth : default_pipe_depth(NL)) : 0;
  if (pipe) {
    // the ring outside the arena (nip rows per slot, whatever the ranks turn out to be); without
    // the memory for it, the in-lane FFT
    const size_t rb = sizeof(cplx) * (size_t)D * nip * ngrid;
    if (rb > c->f_ring_bytes) {
      if (c->f_ring) FISDF_HIP(hipFree(c->f_ring));
      c->f_ring = nullptr;
      c->f_ring_bytes = 0;
      if (hipMalloc(&c->f_ring, rb) == hipSuccess) {
        c->f_ring_bytes = rb;
      } else {
        (void)hipGetLastError();
        c->f_ring = nullptr;
        pipe = false;
        D = 0;
      }
    }
  }
  if (pipe) {
    while ((int)c->ev_q.size() < nq) {
      hipEvent_t e;
      FISDF_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      c->ev_q.push_back(e);
    }
    while ((int)c->ev_free.size() < D) {
      hipEvent_t e;
      FISDF_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      c->ev_free.push_back(e);
    }
  }
  bool any_piece = false;
  for (int lq = 0; lq < nq; ++lq) any_piece = any_piece || piece_of(lq) != nullptr;
  // all-to-all pieces of a mesh whose first FFT pass cannot read plane slices in place (no
  // register kernel, plane too large for the LDS plane kernel): each FFT-issuing stream (the FFT
  // stream, or every lane) unpacks its q's piece into a (nip, ngrid) buffer of its own first
  const bool unpack = any_piece && !fft3d_reads_slices(mesh[0], mesh[1], mesh[2]);
  const PlaneRef* planes = nullptr;
  if (any_piece && !unpack) FISDF_TRY(plane_table(c, mesh, nip, &planes));
  FISDF_CHECK(yT != nullptr || any_piece, "fit_coulomb: no y");
  // sqrt(coulG(k_q+G) vol/N^2)  (:114-115 and the Parseval 1/N of :118), cached per q
  const double wscale = vol / ((double)ngrid * ngrid);
  static const int half_env = [] {
    const char* e = getenv("FISDF_HALF_G");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  const bool half_on = (c->half_grid >= 0 ? c->half_grid : half_env) != 0;
  auto half_of = [&](int sl) { return half_on && c->f_real[sl] != 0; };
  auto weight_q = [&](hipStream_t st, int lq, const double** w) {
    return get_weight(c, st, mesh, kmesh, a, h_qs[lq], wscale, half_of(s0 + lq), w);
  };
  auto slot_y = [&](int lq) { return c->f_ring + (long)(lq % D) * nip * ngrid; };
  FISDF_TRY(fisdf_factor_x4_wait(c, nullptr));
  int rmax = 0;
  for (int lq = 0; lq < nq; ++lq) rmax = std::max(rmax, c->f_rank[s0 + lq]);
  // minimum-norm slots transform all nip rows of y (the operator A^+ mixes every row)
  auto cod_of = [&](int sl) { return sl < (int)c->f_cod.size() && c->f_cod[sl] != 0; };
  int rfmax = rmax, ncod = 0;
  for (int lq = 0; lq < nq; ++lq)
    if (cod_of(s0 + lq)) {
      rfmax = nip;
      ++ncod;
    }
  // every q full rank (the production regime) and many q in the call: each q's W_PP =
  // L^-H G L^-1 and its scatter run in its lane right after its HERK, overlapped with the other
  // q's fit, instead of as a batched tail after the lanes join (the same kernel per output, batch
  // 1: W_q unchanged bit for bit).  C3 on one GPU (36 q): 79.89 vs 80.21 ms/step; a k-shard's 4-5
  // q: +0.6 ms per rank (the last q of each lane then waits for its own small GEMMs), so below
  // kLaneWppMinQ q the batched tail stays.  FISDF_LANE_WPP: 0 never, 1 always
  constexpr int kLaneWppMinQ = 12;
  static const int lane_wpp_env = [] {
    const char* e = getenv("FISDF_LANE_WPP");
    return e ? atoi(e) : -1;
  }();
  bool lane_wpp = (lane_wpp_env < 0 ? nq >= kLaneWppMinQ : lane_wpp_env != 0) && rmax == nip &&
                  ncod == 0;
  for (int lq = 0; lq < nq && lane_wpp; ++lq) lane_wpp = c->f_rank[s0 + lq] == nip;
  // split-K of each q's HERK from its own rank (not the call's largest), so a q's arithmetic
  // does not depend on which other q share the call (1-GPU vs sharded builds agree bitwise)
  const int ncu = num_cus(c->device);
  auto ks_of = [&](int r, long K) { return pick_ksplit_herk(r, (int)K, ncu); };
  int ks = 1;
  for (int lq = 0; lq < nq; ++lq) ks = std::max(ks, ks_of(c->f_rank[s0 + lq], ngrid));
  // a self-conjugate q is fitted on the prefix planes of its Hermitian G pairs (about half the
  // grid): Re W = sum over one member of each pair with the pair's combined weight (half_of)
  auto ncols_of = [&](int lq) -> long {
    if (!half_of(s0 + lq)) return ngrid;
    int m[3];
    self_conjugate_m(kmesh, h_qs[lq], m);
    return (long)half_prefix_planes(mesh[0], m[0]) * mesh[1] * mesh[2];
  };
  const long rr = (long)rmax * rmax;
  const long sLi = (long)nblk * nb * nb;
  Carver cv;
  size_t oY[4], oU[4], oK[4], oTc[4];
  for (int l = 0; l < NL; ++l) {
    if (!pipe) oY[l] = cv.take(sizeof(cplx) * rfmax * ngrid);
    oU[l] = cv.take(sizeof(cplx) * rmax * ngrid);
    oK[l] = cv.take(sizeof(cplx) * (size_t)ks * rmax * rmax);
    oTc[l] = cv.take(sizeof(cplx) * rr);
  }
  c->last_fit_lanes = NL;
  c->last_fit_pipe = pipe ? D : 0;
  size_t oP[4] = {0, 0, 0, 0};
  if (unpack)
    for (int l = 0; l < (pipe ? 1 : NL); ++l) oP[l] = cv.take(sizeof(cplx) * (size_t)nip * ngrid);
  // W_PP = L^-H G L^-1 (two upper-triangular nip^3 GEMMs per q) split over K: 100 output tiles
  // of 64 x 64 at C3 leave most CUs idle for ~180 us per GEMM, in every lane, for every q.  The
  // split depends on nip only, the same in the lanes and in the batched tail (W_q bitwise equal
  // between the 1-GPU and the k-sharded builds).  FISDF_WPP_KSPLIT (read per call; 1 = off)
  const int wks = [&] {
    const char* e = getenv("FISDF_WPP_KSPLIT");
    const int v = e ? atoi(e) : 4;
    return (nip >= 256 && v > 1) ? std::min(v, 16) : 1;
  }();
  const size_t oWk = wks > 1 ? cv.take(sizeof(cplx) * (size_t)NL * wks * rr) : 0;
  size_t oG = cv.take(sizeof(cplx) * nq * rr);
  size_t oT = cv.take(sizeof(cplx) * nq * rr);
  size_t oS = cv.take(sizeof(cplx) * nq * rr);
  size_t oMS = ncod ? cv.take(sizeof(cplx) * (size_t)ncod * rmax * nip) : 0;  // G M per min-norm slot
  size_t oMT = ncod ? cv.take(sizeof(cplx) * nn) : 0;                  // M^H G M
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  char* b = (char*)base;
  cplx* G = (cplx*)(b + oG);   // (nq, rmax, rmax): G_q in the leading r_q x r_q block, zero elsewhere
  cplx* T = (cplx*)(b + oT);
  cplx* S = (cplx*)(b + oS);
  if (rmax == 0) {
    FISDF_TRY(join_factors(c));
    FISDF_HIP(hipMemsetAsync(Wq, 0, sizeof(cplx) * nq * nn, c->stream));
    return 0;
  }
  hipStream_t lane_st[4] = {c->stream, nullptr, nullptr, nullptr};
  hipStream_t fst = nullptr;  // the FFT stream of the pipelined mode
  bool aux_used[3] = {false, false, false};
  if (ready) {
    // everything enqueued before the first piece landed (the y build, the arena's previous
    // users) is complete at ev_ready[0]
    FISDF_TRY(ensure_aux(c));
    for (int l = 0; l < NL; ++l) {
      lane_st[l] = c->aux[l];
      aux_used[l] = true;
      aux_fork(c, l);
      FISDF_HIP(hipStreamWaitEvent(lane_st[l], c->ev_ready[0], 0));
    }
    FISDF_HIP(hipMemsetAsync(G, 0, sizeof(cplx) * nq * rr, lane_st[0]));
    FISDF_HIP(hipEventRecord(c->ev_fork, lane_st[0]));
    for (int l = 1; l < NL; ++l) FISDF_HIP(hipStreamWaitEvent(lane_st[l], c->ev_fork, 0));
    if (pipe) {
      fst = c->aux[2];
      aux_used[2] = true;
      aux_fork(c, 2);
      FISDF_HIP(hipStreamWaitEvent(fst, c->ev_fork, 0));
    }
  } else if (NL > 1 || pipe) {
    FISDF_HIP(hipMemsetAsync(G, 0, sizeof(cplx) * nq * rr, c->stream));
    FISDF_TRY(ensure_aux(c));
    FISDF_HIP(hipEventRecord(c->ev_fork, c->stream));
    for (int l = 1; l < NL; ++l) {
      lane_st[l] = c->aux[l - 1];
      aux_used[l - 1] = true;
      aux_fork(c, l - 1);
      FISDF_HIP(hipStreamWaitEvent(lane_st[l], c->ev_fork, 0));
    }
    if (pipe) {
      fst = c->aux[2];
      aux_used[2] = true;
      aux_fork(c, 2);
      FISDF_HIP(hipStreamWaitEvent(fst, c->ev_fork, 0));
    }
  } else {
    FISDF_HIP(hipMemsetAsync(G, 0, sizeof(cplx) * nq * rr, c->stream));
  }
  // Yhat_q = FFT(y_q[:, piv] * f_q) * w_q   (:99, :113-115, :118; rows in pivot order); the
  // sharded build reads q in place from their all-to-all pieces (fisdf_set_y_slices) through a
  // per-plane address table (plane-aligned slices)
  // ub: the stream's unpack buffer (FFT stream 0, lane l -> l)
  auto fft_q = [&](hipStream_t st, int lq, cplx* Yh, int ub) -> int {
    const int sl = s0 + lq;
    const int r = cod_of(sl) ? nip : c->f_rank[sl];
    double kq[3], kd[3];
    kpoint(kmesh, g, h_qs[lq], kq);
    for (int i = 0; i < 3; ++i) kd[i] = g.a[i][0] * kq[0] + g.a[i][1] * kq[1] + g.a[i][2] * kq[2];
    const double* wt = nullptr;
    FISDF_TRY(weight_q(st, lq, &wt));
    // a half-grid q: its transform pairs G with -G - m (m = 2 k_q, the phase exp(-i k_q.r) times
    // a real input), so the FFT writes the prefix planes only and moves half of its intermediate
    // (fft3d herm); m from the phase actually applied must match the pairing the weights use
    int herm_m[3];
    bool herm = half_of(sl);
    if (herm) {
      int m[3];
      self_conjugate_m(kmesh, h_qs[lq], m);
      for (int d = 0; d < 3; ++d) {
        const double t = kd[d] / M_PI;
        const long tm2 = std::lround(t);
        herm = herm && std::fabs(t - (double)tm2) < 1e-9 &&
               ((tm2 % mesh[d]) + mesh[d]) % mesh[d] == m[d] % mesh[d];
        herm_m[d] = m[d];
      }
    }
    const int* hm = herm ? herm_m : nullptr;
    // y of this q stored real by the composite build's y kernel (fisdf_build_y_qs)
    const bool y_real = yT != nullptr && lq < (int)c->y_real_slot.size() && c->y_real_slot[lq];
    StageTimer tm(c, FISDF_ST_FFT, st);
    const cplx* pc = piece_of(lq);
    FISDF_CHECK(pc || yT, "fit_coulomb: q without y");
#ifdef FISDF_EXP_NOFFT  // timing experiment only (wrong results)
    return 0;
#endif
    if (pc && unpack) {  // piece -> (nip, ngrid) rows, stream-ordered before the FFT reads them
      cplx* yb = (cplx*)(b + oP[ub]);
      const char* src = (const char*)pc;
      for (size_t p = 0; p + 1 < c->y_slices.size(); p += 2) {
        const long g0 = c->y_slices[p], ng = c->y_slices[p + 1];
        FISDF_CHECK(g0 + ng <= ngrid, "fit_coulomb: y slice out of the mesh");
        if (ng == 0) continue;
        FISDF_HIP(hipMemcpy2DAsync(yb + g0, sizeof(cplx) * ngrid, src, sizeof(cplx) * ng,
                                   sizeof(cplx) * ng, nip, hipMemcpyDeviceToDevice, st));
        src += sizeof(cplx) * (size_t)ng * nip;
      }
      pc = nullptr;
      FISDF_TRY(fft3d(st, yb, ngrid, c->f_piv + (long)sl * nip, Yh, ngrid, r, mesh[0], mesh[1],
                      mesh[2], kd, wt, nullptr, nullptr, hm));
      return 0;
    }
    FISDF_CHECK(!(pc && y_real), "fit_coulomb: a real y slot with a y piece");
    FISDF_TRY(fft3d(st, pc ? pc : yT + (long)lq * nip * ngrid, ngrid, c->f_piv + (long)sl * nip, Yh,
                    ngrid, r, mesh[0], mesh[1], mesh[2], kd, wt, nullptr, pc ? planes : nullptr,
                    hm, y_real));
    return 0;
  };
  // FFT of q lq into its ring slot, after the lane that read the slot's previous q is done
  auto enqueue_fft = [&](int lq) -> int {
    if (lq >= nq || c->f_rank[s0 + lq] == 0) return 0;
    if (lq >= D) FISDF_HIP(hipStreamWaitEvent(fst, c->ev_free[lq % D], 0));
    if (ready) FISDF_HIP(hipStreamWaitEvent(fst, c->ev_ready[lq], 0));
    FISDF_TRY(fft_q(fst, lq, slot_y(lq), 0));
    FISDF_HIP(hipEventRecord(c->ev_q[lq], fst));
    return 0;
  };
  if (pipe)
    for (int lq = 0; lq < D; ++lq) FISDF_TRY(enqueue_fft(lq));
  for (int lq = 0; lq < nq; ++lq) {
    const int ln = lq % NL;
    hipStream_t st = lane_st[ln];
    cplx* Yh = pipe ? slot_y(lq) : (cplx*)(b + oY[ln]);
    cplx* U = (cplx*)(b + oU[ln]);
    cplx* kw = (cplx*)(b + oK[ln]);
    cplx* Tc = (cplx*)(b + oTc[ln]);
    const int q = h_qs[lq];
    const int sl = s0 + lq;  // factor slot
    const int r = c->f_rank[sl];
    if (r == 0) {
      if (pipe) FISDF_TRY(enqueue_fft(lq + D));
      continue;
    }
    const int* piv = c->f_piv + (long)sl * nip;
    const cplx* Lp = c->f_Lp + (long)sl * nn;
    const bool real_q = c->f_real[sl];
    const cplx* Linv = c->f_Linv + (long)sl * sLi;
    (void)piv;
    if (pipe) {
      FISDF_HIP(hipStreamWaitEvent(st, c->ev_q[lq], 0));
    } else {
      if (ready) FISDF_HIP(hipStreamWaitEvent(st, c->ev_ready[lq], 0));
      FISDF_TRY(fft_q(st, lq, Yh, ln));
    }
    cplx* Uq = U;  // where L^{-1} Yh lands
    const long ncol = ncols_of(lq);  // grid columns fitted (half for a self-conjugate q)
    // L^-1, Q, ...: the slots built first need only their own (ev_fac_early); a lane's later q
    // wait for all of them
    if (c->f_fac_unjoined)
      FISDF_HIP(hipStreamWaitEvent(
          st, (sl < c->f_early && !cod_of(sl)) ? c->ev_fac_early : c->ev_fac, 0));
    {
      // U = L^{-1} Yh   (fit, factored order; (x4_q)_PP = L L^H): one GEMM (timed kernel-exact)
      // on a full-rank q and on a minimum-norm q; the basic solution of a rank-deficient q
      // (FISDF_FIT_BASIC) substitutes block by block
      const bool one_gemm = cod_of(sl) || r == nip;
      StageTimer tm(c, FISDF_ST_TRSM, st, one_gemm);
      if (cod_of(sl)) {  // U = A^+ Yh[P]: the minimum-norm operator over all nip rows
        FISDF_TRY(zgemm(st, OP_N, OP_N, r, (int)ncol, nip, ONE, c->f_M + (long)sl * nn, nip, 0, Yh,
                        ngrid, 0, ZERO, U, ngrid, 0, 1, 1, nullptr, EPI_NONE, nullptr,
                        real_q ? GEMM_A_REAL : GEMM_FULL));
        Uq = U;
      } else if (r == nip) {  // one lower-triangular GEMM with L^{-1}
#ifdef FISDF_EXP_NOREALTRSM  // timing experiment only (wrong results)
        if (real_q) { Uq = U; } else
#endif
        FISDF_TRY(zgemm(st, OP_N, OP_N, nip, (int)ncol, nip, ONE, c->f_Li + (long)sl * nn, nip, 0,
                        Yh, ngrid, 0, ZERO, U, ngrid, 0, 1, 1, nullptr, EPI_NONE, nullptr,
                        GEMM_A_LOWER | (real_q ? GEMM_A_REAL : GEMM_FULL)));
        Uq = U;
      } else {
        FISDF_TRY(trsm_blocked(st, 1, Lp, nip, 0, r, Linv, 0, nb, Yh, ngrid, 0, U, ngrid,
                               0, (int)ncol, 1, real_q ? 1 : 0));
      }
    }
    cplx* scratch = Uq == U ? Yh : U;
    {
      StageTimer tm(c, FISDF_ST_HERK, st, true);
      // G = U U^H  (:121 by Parseval)
      FISDF_TRY(herk(st, r, (int)ncol, 1.0, Uq, ngrid, G + lq * rr, rmax, ks_of(r, ncol), kw,
                     real_q ? GEMM_RE_ONLY : GEMM_FULL));
    }
    if (real_q) {
      StageTimer tm(c, FISDF_ST_SMALL, st);
      {
        // Im(G) = Im(sum over the weight-asymmetric G only): every other (G, G') pair cancels
        const fisdf_ctx::Asym* as = nullptr;
        if (half_of(sl)) {
          // half grid: one member of each asymmetric pair, Im W = Im(U_A diag(f) U_A^H)
          FISDF_TRY(get_asym_half(c, st, mesh, kmesh, a, q, wscale, &as));
          if (as->n > 0) {
            cplx* plain = scratch;
            cplx* scaled = scratch + (long)r * as->n;
            FISDF_TRY(gather_cols_scaled(st, Uq, ngrid, r, as->idx, nullptr, as->n, plain));
            FISDF_TRY(gather_cols_scaled(st, Uq, ngrid, r, as->idx, as->f, as->n, scaled));
            FISDF_TRY(zgemm(st, OP_N, OP_C, r, r, as->n, ONE, scaled, as->n, 0, plain, as->n, 0, ZERO,
                            Tc, rmax, 0, 1, std::min(ks_of(r, ncol), std::max(1, as->n / 256)), kw));
            FISDF_TRY(add_imag(st, G + lq * rr, rmax, Tc, rmax, r));
          }
        } else {
          const double* wt = nullptr;
          FISDF_TRY(weight_q(st, lq, &wt));
          FISDF_TRY(get_asym(c, st, mesh, kmesh, a, q, wt, &as));
          if (as->n > 0) {
            FISDF_TRY(gather_cols(st, Uq, ngrid, r, as->idx, as->n, scratch));
            FISDF_TRY(herk(st, r, as->n, 1.0, scratch, as->n, Tc, rmax,
                           std::min(ks_of(r, ncol), std::max(1, as->n / 256)), kw));
            FISDF_TRY(add_imag(st, G + lq * rr, rmax, Tc, rmax, r));
          }
        }
      }
    }
    if (pipe) {  // this lane is done with the ring slot: the FFT D q ahead may overwrite it
      FISDF_HIP(hipEventRecord(c->ev_free[lq % D], st));
      FISDF_TRY(enqueue_fft(lq + D));
    }
    if (lane_wpp) {  // W_PP = L^-H G L^-1 of this q (S = L^-H G, W_PP = L^-H S^H), scattered
      StageTimer tm(c, FISDF_ST_SMALL, st);
      const cplx* Lf = c->f_Li + (long)sl * nn;
      cplx* wk = wks > 1 ? (cplx*)(b + oWk) + (long)ln * wks * rr : nullptr;
      FISDF_TRY(zgemm(st, OP_C, OP_N, nip, nip, nip, ONE, Lf, nip, 0, G + lq * rr, rmax, 0, ZERO,
                      S + lq * rr, rmax, 0, 1, wks, wk, EPI_NONE, nullptr, GEMM_A_UPPER));
      FISDF_TRY(zgemm(st, OP_C, OP_C, nip, nip, nip, ONE, Lf, nip, 0, S + lq * rr, rmax, 0, ZERO,
                      T + lq * rr, rmax, 0, 1, wks, wk, EPI_NONE, nullptr, GEMM_A_UPPER));
      FISDF_TRY(scatter_w(st, T + lq * rr, rmax, rr, rmax, c->f_piv + (long)sl * nip,
                          c->f_rank_dev + sl, Wq + lq * nn, nip, 1));
    }
  }
  // join the lanes (and the FFT stream: that keeps the arena reuse ordered) before the batched
  // small stage on the main stream
  // (this join is what makes fisdf_build's build_return(c, yT) right after this call safe: every
  // FFT / lane read of y is ordered before the caller's stream-ordered free on c->stream)
  for (int i = 0; i < 3; ++i)
    if (aux_used[i]) FISDF_TRY(aux_join(c, i));
  FISDF_TRY(join_factors(c));
  if (!lane_wpp) {
    StageTimer tm(c, FISDF_ST_SMALL);
    // W_PP = L^{-H} G L^{-1} for all q of the shard at once (L padded with identity, G with
    // zeros beyond each rank):  T = L^{-H} G ; S = L^{-H} T^H ; W_PP = S^H ; scatter by pivots
    const cplx* Lp0 = c->f_Lp + (long)s0 * nn;
    const cplx* Li0 = c->f_Linv + (long)s0 * sLi;
    // minimum-norm slots: G M first (the batched back-substitutions below overwrite G)
    for (int lq = 0, j = 0; lq < nq && ncod; ++lq) {
      const int sl = s0 + lq, r = c->f_rank[sl];
      if (!cod_of(sl)) continue;
      FISDF_TRY(zgemm(c->stream, OP_N, OP_N, r, nip, r, ONE, G + lq * rr, rmax, 0,
                      c->f_M + (long)sl * nn, nip, 0, ZERO, (cplx*)(b + oMS) + (long)j++ * rmax * nip,
                      nip, 0, 1));
    }
    bool all_full = rmax == nip;
    for (int lq = 0; lq < nq && all_full; ++lq) all_full = c->f_rank[s0 + lq] == nip;
    if (all_full) {
      // with L^{-1} at hand, two batched GEMMs whose A = L^{-H} is upper triangular (each
      // M-tile starts its K loop at its own row: half the flops of dense GEMMs):
      //   S = L^{-H} G,  W_PP = L^{-H} S^H  (= L^{-H} G L^{-1}, G Hermitian)
      const cplx* Lf = c->f_Li + (long)s0 * nn;
      if (wks > 1) {
        // the lanes' split workspace, NL q at a time (per-q arithmetic as in the lanes)
        cplx* wk = (cplx*)(b + oWk);
        for (int z0 = 0; z0 < nq; z0 += NL) {
          const int nz = std::min(NL, nq - z0);
          FISDF_TRY(zgemm(c->stream, OP_C, OP_N, nip, nip, nip, ONE, Lf + (long)z0 * nn, nip, nn,
                          G + z0 * rr, rmax, rr, ZERO, S + z0 * rr, rmax, rr, nz, wks, wk, EPI_NONE,
                          nullptr, GEMM_A_UPPER));
          FISDF_TRY(zgemm(c->stream, OP_C, OP_C, nip, nip, nip, ONE, Lf + (long)z0 * nn, nip, nn,
                          S + z0 * rr, rmax, rr, ZERO, T + z0 * rr, rmax, rr, nz, wks, wk, EPI_NONE,
                          nullptr, GEMM_A_UPPER));
        }
      } else {
        FISDF_TRY(zgemm(c->stream, OP_C, OP_N, nip, nip, nip, ONE, Lf, nip, nn, G, rmax, rr, ZERO,
                        S, rmax, rr, nq, 1, nullptr, EPI_NONE, nullptr, GEMM_A_UPPER));
        FISDF_TRY(zgemm(c->stream, OP_C, OP_C, nip, nip, nip, ONE, Lf, nip, nn, S, rmax, rr, ZERO,
                        T, rmax, rr, nq, 1, nullptr, EPI_NONE, nullptr, GEMM_A_UPPER));
      }
    } else {
      FISDF_TRY(trsm_blocked(c->stream, 0, Lp0, nip, nn, rmax, Li0, sLi, nb, G, rmax, rr,
                             T, rmax, rr, rmax, nq));
      FISDF_TRY(conj_transpose(c->stream, T, rmax, rr, G, nq));
      FISDF_TRY(trsm_blocked(c->stream, 0, Lp0, nip, nn, rmax, Li0, sLi, nb, G, rmax, rr,
                             S, rmax, rr, rmax, nq));
      FISDF_TRY(conj_transpose(c->stream, S, rmax, rr, T, nq));
    }
    FISDF_TRY(scatter_w(c->stream, T, rmax, rr, rmax, c->f_piv + (long)s0 * nip,
                        c->f_rank_dev + s0, Wq, nip, nq));
    // minimum-norm slots: W_PP = M^H (G M) (nip x nip: z[P] = M^H U) replaces the above
    for (int lq = 0, j = 0; lq < nq && ncod; ++lq) {
      const int sl = s0 + lq, r = c->f_rank[sl];
      if (!cod_of(sl)) continue;
      const cplx* MS = (cplx*)(b + oMS) + (long)j++ * rmax * nip;
      cplx* MT = (cplx*)(b + oMT);
      const cplx* Mq = c->f_M + (long)sl * nn;
      FISDF_TRY(zgemm(c->stream, OP_C, OP_N, nip, nip, r, ONE, Mq, nip, 0, MS, nip, 0, ZERO, MT,
                      nip, 0, 1));
      FISDF_TRY(scatter_w(c->stream, MT, nip, 0, nip, c->f_piv + (long)sl * nip, c->f_nip_dev,
                          Wq + lq * nn, nip, 1));
    }
  }
  return 0;
}

int fisdf_fit_coulomb(fisdf_ctx* c, int q0, int q1, const void* yTv, int nip, const int mesh[3],
                      const int kmesh[3], const double a[9], void* Wqv) {
  const int nk = kmesh[0] * kmesh[1] * kmesh[2];
  FISDF_CHECK(0 <= q0 && q0 <= q1 && q1 <= nk, "fit_coulomb: bad q range");
  std::vector<int> qs = q_range(q0, q1);
  return fisdf_fit_coulomb_qs(c, qs.data(), (int)qs.size(), yTv, nip, mesh, kmesh, a, Wqv);
}

// ---- A8 prep ------------------------------------------------------------------
int fisdf_build_ws_qs(fisdf_ctx* c, const void* Wqv, const int* h_qs, const double* h_wt, int nq,
                      int nip, const int kmesh[3], const double a[9], void* Wsv) {
  FISDF_TRY(device_guard(c));
  StageTimer tm(c, FISDF_ST_WS);
  const int nk = kmesh[0] * kmesh[1] * kmesh[2];
  FISDF_TRY(check_qlist(h_qs, nq, nk, "build_ws"));
  const long nn = (long)nip * nip;
  if (nq == 0) {
    FISDF_HIP(hipMemsetAsync(Wsv, 0, sizeof(double) * nk * nn, c->stream));
    return 0;
  }
  // Phi_sel[R, i] = wt_i Phi[R, q_i]  (host; nk x nq)
  CellGeom g;
  lattice(a, g);
  std::vector<cplx> ph((size_t)nk * nq);
  for (int R = 0; R < nk; ++R) {
    int r2 = R % kmesh[2], r1 = (R / kmesh[2]) % kmesh[1], r0 = R / (kmesh[1] * kmesh[2]);
    double T[3];
    for (int cc = 0; cc < 3; ++cc) T[cc] = r0 * g.a[0][cc] + r1 * g.a[1][cc] + r2 * g.a[2][cc];
    for (int i = 0; i < nq; ++i) {
      double k[3];
      kpoint(kmesh, g, h_qs[i], k);
      const double th = T[0] * k[0] + T[1] * k[1] + T[2] * k[2];
      const double w = (h_wt ? h_wt[i] : 1.0) / std::sqrt((double)nk);
      ph[(size_t)R * nq + i] = cmk(w * std::cos(th), w * std::sin(th));
    }
  }
  Carver cv;
  size_t oP = cv.take(sizeof(cplx) * ph.size());
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  cplx* dph = (cplx*)((char*)base + oP);
  FISDF_TRY(upload_bytes(c, ph.data(), sizeof(cplx) * ph.size(), dph));
  // ws = Phi W (:205), real part * sqrt(nk) (:207) in the GEMM's epilogue, stored real (the
  // reference keeps W_s = ws.real, a real array).  With time-reversal representatives the
  // partner -q contributes conj(Phi[R,q] W_q), so Re(.) of the pair is 2 Re(Phi[R,q] W_q): wt = 2.
  FISDF_TRY(zgemm(c->stream, OP_N, OP_N, nk, nn, nq, cmk(std::sqrt((double)nk), 0), dph, nq, 0,
                  (const cplx*)Wqv, nn, 0, ZERO, (cplx*)Wsv, nn, 0, 1, 1, nullptr, EPI_REAL,
                  nullptr));
  return 0;
}

// W_s row blocks [rows[b], rows[b+1]) of a q-list's partial sum, block b at Wsb + b * chunk
// doubles (chunk 0: one block): the phase table uploaded once, one GEMM per block
static int ws_row_blocks(fisdf_ctx* c, const void* Wqv, const int* h_qs, const double* h_wt, int nq,
                         int nip, const int kmesh[3], const double a[9], int nblk,
                         const int* rows, long chunk, void* Wsv) {
  StageTimer tm(c, FISDF_ST_WS);
  const int nk = kmesh[0] * kmesh[1] * kmesh[2];
  FISDF_TRY(check_qlist(h_qs, nq, nk, "build_ws_rows"));
  FISDF_CHECK(nblk >= 1, "build_ws_rows: no blocks");
  for (int b = 0; b < nblk; ++b)
    FISDF_CHECK(0 <= rows[b] && rows[b] <= rows[b + 1] && rows[b + 1] <= nip &&
                    (nblk == 1 || (long)nk * (rows[b + 1] - rows[b]) * nip <= chunk),
                "build_ws_rows: bad row range");
  const long nn = (long)nip * nip;
  double* Ws = (double*)Wsv;
  if (nq == 0) {
    for (int b = 0; b < nblk; ++b)
      FISDF_HIP(hipMemsetAsync(Ws + b * chunk, 0,
                               sizeof(double) * nk * (rows[b + 1] - rows[b]) * nip, c->stream));
    return 0;
  }
  CellGeom g;
  lattice(a, g);
  std::vector<cplx> ph((size_t)nk * nq);
  for (int R = 0; R < nk; ++R) {
    int r2 = R % kmesh[2], r1 = (R / kmesh[2]) % kmesh[1], r0 = R / (kmesh[1] * kmesh[2]);
    double T[3];
    for (int cc = 0; cc < 3; ++cc) T[cc] = r0 * g.a[0][cc] + r1 * g.a[1][cc] + r2 * g.a[2][cc];
    for (int i = 0; i < nq; ++i) {
      double k[3];
      kpoint(kmesh, g, h_qs[i], k);
      const double th = T[0] * k[0] + T[1] * k[1] + T[2] * k[2];
      const double w = (h_wt ? h_wt[i] : 1.0) / std::sqrt((double)nk);
      ph[(size_t)R * nq + i] = cmk(w * std::cos(th), w * std::sin(th));
    }
  }
  Carver cv;
  size_t oP = cv.take(sizeof(cplx) * ph.size());
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  cplx* dph = (cplx*)((char*)base + oP);
  FISDF_TRY(upload_bytes(c, ph.data(), sizeof(cplx) * ph.size(), dph));
  // W_s[R][i0:i1] = sqrt(nk) Re(sum_i Phi_sel[R,i] W_{q_i}[i0:i1]) (fftisdf.py:205-207): the same
  // GEMM as fisdf_build_ws_qs on the row block (B = W_q rows i0..i1, ld nip^2), written (nk, nb, nip)
  for (int b = 0; b < nblk; ++b) {
    const long nb = rows[b + 1] - rows[b];
    if (nb == 0) continue;
    FISDF_TRY(zgemm(c->stream, OP_N, OP_N, nk, (int)(nb * nip), nq, cmk(std::sqrt((double)nk), 0),
                    dph, nq, 0, (const cplx*)Wqv + (long)rows[b] * nip, nn, 0, ZERO,
                    (cplx*)(Ws + b * chunk), nb * nip, 0, 1, 1, nullptr, EPI_REAL, nullptr));
  }
  return 0;
}

int fisdf_build_ws_rows(fisdf_ctx* c, const void* Wqv, const int* h_qs, const double* h_wt, int nq,
                        int nip, const int kmesh[3], const double a[9], int i0, int i1,
                        void* Wsv) {
  FISDF_TRY(device_guard(c));
  const int rows[2] = {i0, i1};
  return ws_row_blocks(c, Wqv, h_qs, h_wt, nq, nip, kmesh, a, 1, rows, 0, Wsv);
}

int fisdf_build_ws_blocks(fisdf_ctx* c, const void* Wqv, const int* h_qs, const double* h_wt,
                          int nq, int nip, const int kmesh[3], const double a[9], int nblk,
                          const int* h_rows, long chunk, void* Wsbv) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(h_rows != nullptr && chunk >= 0, "build_ws_blocks: bad arguments");
  return ws_row_blocks(c, Wqv, h_qs, h_wt, nq, nip, kmesh, a, nblk, h_rows, chunk, Wsbv);
}

int fisdf_build_ws(fisdf_ctx* c, const void* Wqv, int q0, int q1, int nip, const int kmesh[3],
                   const double a[9], void* Wsv) {
  const int nk = kmesh[0] * kmesh[1] * kmesh[2];
  FISDF_CHECK(0 <= q0 && q0 <= q1 && q1 <= nk, "build_ws: bad q range");
  std::vector<int> qs = q_range(q0, q1);
  return fisdf_build_ws_qs(c, Wqv, qs.data(), nullptr, (int)qs.size(), nip, kmesh, a, Wsv);
}

// ---- next-2: ISDF ERIs / ao2mo --------------------------------------------------
// eri[i*n2+j][k*n4+l] = sum_IJ W_q[I,J] conj(A1[I,i]) A2[I,j] conj(A3[J,k]) A4[J,l],
// A_s = X_{k_s} C_s (C_s = identity when d_C[s] is null -> AO integrals), q = k2 - k1
// (identity of fftdf-with-k-lstsq.py:221-232).
int fisdf_get_eri(fisdf_ctx* c, const void* Xv, int nip, int nao, const int kidx[4],
                  const void* Wqv, const void* const* Cv, const int nmo[4], void* outv) {
  FISDF_TRY(device_guard(c));
  const cplx* X = (const cplx*)Xv;
  int n[4];
  for (int s = 0; s < 4; ++s) n[s] = Cv && Cv[s] ? nmo[s] : nao;
  const long p12 = (long)n[0] * n[1], p34 = (long)n[2] * n[3];
  Carver cv;
  size_t oA[4];
  for (int s = 0; s < 4; ++s) oA[s] = cv.take(sizeof(cplx) * (size_t)nip * n[s]);
  size_t oP12 = cv.take(sizeof(cplx) * nip * p12);
  size_t oP34 = cv.take(sizeof(cplx) * nip * p34);
  size_t oT = cv.take(sizeof(cplx) * nip * p34);
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  char* b = (char*)base;
  const cplx* A[4];
  for (int s = 0; s < 4; ++s) {
    const cplx* Xk = X + (long)kidx[s] * nip * nao;
    if (Cv && Cv[s]) {
      cplx* As = (cplx*)(b + oA[s]);
      FISDF_TRY(zgemm(c->stream, OP_N, OP_N, nip, n[s], nao, ONE, Xk, nao, 0,
                      (const cplx*)Cv[s], n[s], 0, ZERO, As, n[s], 0, 1));
      A[s] = As;
    } else {
      A[s] = Xk;
    }
  }
  cplx* P12 = (cplx*)(b + oP12);
  cplx* P34 = (cplx*)(b + oP34);
  cplx* T = (cplx*)(b + oT);
  FISDF_TRY(pair_product(c->stream, A[0], n[0], A[1], n[1], nip, P12));
  FISDF_TRY(pair_product(c->stream, A[2], n[2], A[3], n[3], nip, P34));
  FISDF_TRY(zgemm(c->stream, OP_N, OP_N, nip, (int)p34, nip, ONE, (const cplx*)Wqv, nip, 0, P34,
                  p34, 0, ZERO, T, p34, 0, 1));
  FISDF_TRY(zgemm(c->stream, OP_T, OP_N, (int)p12, (int)p34, nip, ONE, P12, p12, 0, T, p34, 0,
                  ZERO, (cplx*)outv, p34, 0, 1));
  return 0;
}

// ---- A7 -----------------------------------------------------------------------
int fisdf_get_j_rows(fisdf_ctx* c, const void* Xv, const void* W0, const void* dmsv, int nset,
                     int nk, int nip, int nao, int i0, int i1, void* vjv) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(0 <= i0 && i0 <= i1 && i1 <= nip, "get_j: bad row range");
  StageTimer tm(c, FISDF_ST_J);
  const cplx* X = (const cplx*)Xv;
  const cplx* dms = (const cplx*)dmsv;
  cplx* vj = (cplx*)vjv;
  const int nb = i1 - i0;
  const long xs = (long)nip * nao, ds = (long)nao * nao;
  if (nb == 0) {
    FISDF_HIP(hipMemsetAsync(vj, 0, sizeof(cplx) * nset * nk * ds, c->stream));
    return 0;
  }
  Carver cv;
  size_t oT = cv.take(sizeof(cplx) * nset * nk * xs);
  size_t oR = cv.take(sizeof(cplx) * nset * nip);
  size_t oV = cv.take(sizeof(cplx) * nset * nb);
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  cplx* T = (cplx*)((char*)base + oT);
  cplx* rho = (cplx*)((char*)base + oR);
  cplx* v = (cplx*)((char*)base + oV);
  // T = X_k D_k
  for (int x = 0; x < nset; ++x)
    FISDF_TRY(zgemm(c->stream, OP_N, OP_N, nip, nao, nao, ONE, X, nao, xs, dms + (long)x * nk * ds,
                    nao, ds, ZERO, T + (long)x * nk * xs, nao, xs, nk));
  // rho_I = sum_k X_k[I,m] D_k[m,n] X_k*[I,n] / nk  (:155-156), every I
  FISDF_TRY(rho_diag(c->stream, T, X, nset, nk, nip, nao, 1.0 / nk, rho));
  // v_I = (W0 rho)_I for the rows of the block  (:159)
  FISDF_TRY(zgemm(c->stream, OP_N, OP_N, nb, 1, nip, ONE, (const cplx*)W0 + (long)i0 * nip, nip, 0,
                  rho, 1, nip, ZERO, v, 1, nb, nset));
  // J_k (block part) = X_k[I]^H diag(v_I) X_k[I]  (:166)
  FISDF_TRY(scale_rows(c->stream, X, v, nset, nk, nip, i0, nb, nao, T));
  for (int x = 0; x < nset; ++x)
    FISDF_TRY(zgemm(c->stream, OP_C, OP_N, nao, nao, nb, ONE, X + (long)i0 * nao, nao, xs,
                    T + (long)x * nk * nb * nao, nao, (long)nb * nao, ZERO,
                    vj + (long)x * nk * ds, nao, ds, nk));
  return 0;
}

int fisdf_get_j_band_rows(fisdf_ctx* c, const void* Xv, const void* W0, const void* dmsv, int nset,
                          int nk, int nip, int nao, const void* Xbv, int nkb, int i0, int i1,
                          void* vjv) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(0 <= i0 && i0 <= i1 && i1 <= nip && nkb > 0, "get_j_band: bad sizes");
  StageTimer tm(c, FISDF_ST_J);
  const cplx* X = (const cplx*)Xv;
  const cplx* Xb = (const cplx*)Xbv;
  const cplx* dms = (const cplx*)dmsv;
  cplx* vj = (cplx*)vjv;
  const int nb = i1 - i0;
  const long xs = (long)nip * nao, ds = (long)nao * nao;
  if (nb == 0) {
    FISDF_HIP(hipMemsetAsync(vj, 0, sizeof(cplx) * nset * nkb * ds, c->stream));
    return 0;
  }
  Carver cv;
  size_t oT = cv.take(sizeof(cplx) * nset * (size_t)std::max(nk, nkb) * xs);
  size_t oR = cv.take(sizeof(cplx) * nset * nip);
  size_t oV = cv.take(sizeof(cplx) * nset * nb);
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  cplx* T = (cplx*)((char*)base + oT);
  cplx* rho = (cplx*)((char*)base + oR);
  cplx* v = (cplx*)((char*)base + oV);
  // rho_I from the k-mesh density matrices and v = W0 rho (fftisdf.py:155-159), as get_j
  for (int x = 0; x < nset; ++x)
    FISDF_TRY(zgemm(c->stream, OP_N, OP_N, nip, nao, nao, ONE, X, nao, xs, dms + (long)x * nk * ds,
                    nao, ds, ZERO, T + (long)x * nk * xs, nao, xs, nk));
  FISDF_TRY(rho_diag(c->stream, T, X, nset, nk, nip, nao, 1.0 / nk, rho));
  FISDF_TRY(zgemm(c->stream, OP_N, OP_N, nb, 1, nip, ONE, (const cplx*)W0 + (long)i0 * nip, nip, 0,
                  rho, 1, nip, ZERO, v, 1, nb, nset));
  // J_k' = Xb_k'[I]^H diag(v_I) Xb_k'[I] at the band k-points (fftisdf.py:166 with kpts_band)
  FISDF_TRY(scale_rows(c->stream, Xb, v, nset, nkb, nip, i0, nb, nao, T));
  for (int x = 0; x < nset; ++x)
    FISDF_TRY(zgemm(c->stream, OP_C, OP_N, nao, nao, nb, ONE, Xb + (long)i0 * nao, nao, xs,
                    T + (long)x * nkb * nb * nao, nao, (long)nb * nao, ZERO,
                    vj + (long)x * nkb * ds, nao, ds, nkb));
  return 0;
}

int fisdf_get_j(fisdf_ctx* c, const void* Xv, const void* W0, const void* dmsv, int nset, int nk,
                int nip, int nao, void* vjv) {
  return fisdf_get_j_rows(c, Xv, W0, dmsv, nset, nk, nip, nao, 0, nip, vjv);
}

// ---- A8 -----------------------------------------------------------------------
static int get_k_block(fisdf_ctx* c, const void* Xv, const double* Ws_rows, long ws_Rstride,
                       const void* dmsv, int nset, int nip, int nao, const int kmesh[3],
                       const double a[9], int i0, int i1, void* vkv);

int fisdf_get_k_rows(fisdf_ctx* c, const void* Xv, const void* Wsv, const void* dmsv, int nset,
                     int nip, int nao, const int kmesh[3], const double a[9], int i0, int i1,
                     void* vkv) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(0 <= i0 && i0 <= i1 && i1 <= nip, "get_k: bad row range");
  // rows i0.. of W_s[R] inside the full (nk, nip, nip) array
  return get_k_block(c, Xv, (const double*)Wsv + (long)i0 * nip, (long)nip * nip, dmsv, nset, nip,
                     nao, kmesh, a, i0, i1, vkv);
}

int fisdf_get_k_rows_local(fisdf_ctx* c, const void* Xv, const void* Ws_rows, const void* dmsv,
                           int nset, int nip, int nao, const int kmesh[3], const double a[9],
                           int i0, int i1, void* vkv) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(0 <= i0 && i0 <= i1 && i1 <= nip, "get_k: bad row range");
  // this rank's rows only: (nk, i1 - i0, nip) from fisdf_build_ws_rows + a reduce-scatter
  return get_k_block(c, Xv, (const double*)Ws_rows, (long)(i1 - i0) * nip, dmsv, nset, nip, nao,
                     kmesh, a, i0, i1, vkv);
}

static int get_k_block(fisdf_ctx* c, const void* Xv, const double* Ws_rows, long ws_Rstride,
                       const void* dmsv, int nset, int nip, int nao, const int kmesh[3],
                       const double a[9], int i0, int i1, void* vkv) {
  StageTimer tm(c, FISDF_ST_K);
  const int nk = kmesh[0] * kmesh[1] * kmesh[2];
  const cplx* phase;
  FISDF_TRY(get_phase(c, kmesh, a, &phase));
  const cplx* X = (const cplx*)Xv;
  const cplx* dms = (const cplx*)dmsv;
  cplx* vk = (cplx*)vkv;
  const int nb = i1 - i0;
  const long xs = (long)nip * nao, ds = (long)nao * nao, bn = (long)nb * nip, ba = (long)nb * nao;
  if (nb == 0) {
    FISDF_HIP(hipMemsetAsync(vk, 0, sizeof(cplx) * nset * nk * ds, c->stream));
    return 0;
  }
  Carver cv;
  size_t oT = cv.take(sizeof(cplx) * nk * ba);
  size_t o1 = cv.take(sizeof(cplx) * nk * bn);
  size_t o2 = cv.take(sizeof(cplx) * nk * bn);
  void* base;
  FISDF_TRY(arena_get(c, cv.off, &base));
  cplx* T = (cplx*)((char*)base + oT);
  cplx* B1 = (cplx*)((char*)base + o1);
  cplx* B2 = (cplx*)((char*)base + o2);
  const cplx* Xb = X + (long)i0 * nao;
  for (int x = 0; x < nset; ++x) {
    const cplx* dm = dms + (long)x * nk * ds;
    // rho_k^T[I, J] = rho_k[J, I] = (conj(X_k[I]) D_k^T X_k^T)[I, J] / nk for the block rows
    // (:211-212, transposed at the source so :219's product is element-wise)
    FISDF_TRY(zgemm(c->stream, OP_R, OP_T, nb, nao, nao, cmk(1.0 / nk, 0), Xb, nao, xs, dm, nao, ds,
                    ZERO, T, nao, ba, nk));
    if (nk == 1) {
      // Gamma only (Phi = 1): rho_s = Re(rho_k) (:215-216) and V = W_s * rho_s^T (:219) in this
      // GEMM's epilogue; V_k = V_s (:222)
      FISDF_TRY(zgemm(c->stream, OP_N, OP_T, nb, nip, nao, ONE, T, nao, ba, X, nao, xs, ZERO, B1,
                      nip, bn, 1, 1, (cplx*)(void*)Ws_rows, EPI_WSRHO, c->maximag + 2, GEMM_FULL,
                      (long)nip));
    } else {
      FISDF_TRY(zgemm(c->stream, OP_N, OP_T, nb, nip, nao, ONE, T, nao, ba, X, nao, xs, ZERO, B1,
                      nip, bn, nk));
      // round 6: the transform pair and the product in one register pass per column (C3: 0.50
      // -> ~0.2 ms); FISDF_K_DFT=0 (read per call: the GPU tests compare) keeps the GEMMs
      bool done = false;
      const char* kd = getenv("FISDF_K_DFT");
      if (!(kd && kd[0] == '0'))
        FISDF_TRY(k_wsrho_reg(c->stream, B1, bn, kmesh, Ws_rows, ws_Rstride, c->maximag + 2,
                              &done));
      if (!done) {
        // rho_s = Phi rho_k (:215), real (:216), and V_s = W_s * rho_s^T (:219) for the block
        // rows, both in the GEMM's epilogue (EPI_WSRHO: Re(W_s) Re(.), max |Im rho_s| recorded)
        FISDF_TRY(zgemm(c->stream, OP_N, OP_N, nk, bn, nk, ONE, phase, nk, 0, B1, bn, 0, ZERO, B2,
                        bn, 0, 1, 1, (cplx*)(void*)Ws_rows, EPI_WSRHO, c->maximag + 2, GEMM_FULL,
                        ws_Rstride));
        // V_k = Phi^T V_s (:222)
        FISDF_TRY(zgemm(c->stream, OP_T, OP_N, nk, bn, nk, ONE, phase, nk, 0, B2, bn, 0, ZERO, B1,
                        bn, 0, 1));
      }
    }
    // K_k (block part) = X_k[I]^H (V_k[I, :] X_k)  (:225)
    FISDF_TRY(zgemm(c->stream, OP_N, OP_N, nb, nao, nip, ONE, B1, nip, bn, X, nao, xs, ZERO, T,
                    nao, ba, nk));
    FISDF_TRY(zgemm(c->stream, OP_C, OP_N, nao, nao, nb, ONE, Xb, nao, xs, T, nao, ba, ZERO,
                    vk + (long)x * nk * ds, nao, ds, nk));
  }
  return 0;
}

int fisdf_get_k(fisdf_ctx* c, const void* Xv, const void* Wsv, const void* dmsv, int nset, int nip,
                int nao, const int kmesh[3], const double a[9], void* vkv) {
  return fisdf_get_k_rows(c, Xv, Wsv, dmsv, nset, nip, nao, kmesh, a, 0, nip, vkv);
}

// ---- composite entries --------------------------------------------------------
}  // extern "C"

namespace {

enum BuildRole { BR_X = 0, BR_X4 = 1, BR_Y = 2, BR_WQ = 3, BR_WS = 4, BR_SEND = 5, BR_WSB = 6,
                 BR_W0 = 7 };

// a buffer of the composite build: the caller's allocator, or a library-owned grow-only buffer
int build_alloc(fisdf_ctx* c, int role, size_t bytes, void** out) {
  bytes = std::max<size_t>(bytes, 256);
  if (c->alloc_fn) {
    void* p = c->alloc_fn(bytes, c->alloc_user);
    FISDF_CHECK(p != nullptr, "build: the caller's allocator returned NULL");
    c->lent.push_back(p);
    *out = p;
    return 0;
  }
  auto& o = c->owned[role];
  if (o.second < bytes) {
    if (o.first) {
      FISDF_HIP(hipStreamSynchronize(c->stream));
      FISDF_HIP(hipFree(o.first));
    }
    o = {nullptr, 0};
    FISDF_HIP(hipMalloc(&o.first, bytes));
    o.second = bytes;
  }
  *out = o.first;
  return 0;
}

// hand one lent buffer back (stream-ordered: its last use is enqueued on c->stream, and every
// aux stream that read it has been joined into c->stream — checked)
int build_return(fisdf_ctx* c, void* p) {
  if (!c->alloc_fn || !p) return 0;
  auto it = std::find(c->lent.begin(), c->lent.end(), p);
  if (it == c->lent.end()) return 0;
  FISDF_TRY(check_aux_joined(c, "build_return"));
  c->lent.erase(it);
  if (c->free_fn) c->free_fn(p, c->alloc_user);
  return 0;
}

void build_return_all(fisdf_ctx* c) {
  // an earlier call that failed between a fork and its join may have left an aux stream with
  // work: drain it before the caller's allocator gets the buffers back (likewise the sharded
  // build's collective stream, whose exchange reads and writes the build's y buffers)
  for (int i = 0; i < 3; ++i)
    if (c->aux_joined[i] != c->aux_use[i]) {
      if (c->aux[i]) (void)hipStreamSynchronize(c->aux[i]);
      c->aux_joined[i] = c->aux_use[i];
    }
  if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
  // y-readiness marks left by a build that failed before its fit consumed them
  c->ready_marked.assign(c->ready_marked.size(), 0);
  c->y_piece.clear();
  std::vector<void*> l;
  l.swap(c->lent);
  if (c->free_fn)
    for (void* p : l) c->free_fn(p, c->alloc_user);
  c->bld = fisdf_ctx::Build();
}

// time-reversal classes of the q-mesh (get_kpts order): partner[q] = index of -q, the fitted
// representatives (smaller index of each pair) and their W_s weights (2 unless self-paired)
void tr_classes(const int km[3], bool on, std::vector<int>& reps, std::vector<int>& partner,
                std::vector<double>& wt) {
  const int nk = km[0] * km[1] * km[2];
  partner.resize(nk);
  reps.clear();
  wt.clear();
  for (int q = 0; q < nk; ++q) {
    const int i2 = q % km[2], i1 = (q / km[2]) % km[1], i0 = q / (km[1] * km[2]);
    partner[q] = (((km[0] - i0) % km[0]) * km[1] + (km[1] - i1) % km[1]) * km[2] + (km[2] - i2) % km[2];
  }
  for (int q = 0; q < nk; ++q) {
    if (!on) {  // every q fitted on its own (W_s weights 1)
      partner[q] = q;
      reps.push_back(q);
      wt.push_back(1.0);
    } else if (partner[q] >= q) {
      reps.push_back(q);
      wt.push_back(partner[q] == q ? 1.0 : 2.0);
    }
  }
}

// time reversal of the AO inputs (what the fold over k <= -k of the selection Gram, x4 and y, and
// W_{-q} = conj(W_q), rely on): a[-k] = conj(a[k]) holds for real basis functions on a k-mesh
// containing -k (get_kpts order, no shift).  The check reads all of x0 (the selection's input,
// 45 MB at C3) and every 61st grid point of f (x0 and f come from one basis: the whole 1.24 GB of
// f cost 0.7 ms/step beside the selection and the y build, profiles/r05/tr_check/) on stream `st`
// and lands in tr_pinned behind ev_tr; tr_verdict waits for it.
int tr_alloc(fisdf_ctx* c) {
  if (c->trmon) return 0;
  FISDF_HIP(hipMalloc(&c->trmon, 4 * sizeof(unsigned long long)));
  FISDF_HIP(hipHostMalloc((void**)&c->tr_pinned, 4 * sizeof(unsigned long long),
                          hipHostMallocDefault));
  FISDF_HIP(hipEventCreateWithFlags(&c->ev_tr, hipEventDisableTiming));
  FISDF_HIP(hipEventRecord(c->ev_tr, c->stream));
  return 0;
}

constexpr long kTrFStride = 61;  // grid-point sampling of f in the composite build's check

int tr_check_enqueue(fisdf_ctx* c, hipStream_t st, const cplx* x0, long ng0, const cplx* f,
                     long ngrid, int nao, const int kmesh[3]) {
  FISDF_TRY(tr_alloc(c));
  FISDF_HIP(hipEventSynchronize(c->ev_tr));  // the pinned words are rewritten below
  FISDF_HIP(hipMemsetAsync(c->trmon, 0, 4 * sizeof(unsigned long long), st));
  FISDF_TRY(tr_check(st, x0, ng0 * nao, ng0, nao, 1, kmesh, c->trmon));
  if (f) FISDF_TRY(tr_check(st, f, ngrid * nao, ngrid, nao, kTrFStride, kmesh, c->trmon + 2));
  FISDF_HIP(hipMemcpyAsync(c->tr_pinned, c->trmon, 4 * sizeof(unsigned long long),
                           hipMemcpyDeviceToHost, st));
  FISDF_HIP(hipEventRecord(c->ev_tr, st));
  return 0;
}

// the largest relative violation max |a[-k] - conj(a[k])| / max |a| of the last check
int tr_verdict(fisdf_ctx* c, double* rel) {
  FISDF_HIP(hipEventSynchronize(c->ev_tr));
  double v[4];
  for (int i = 0; i < 4; ++i) v[i] = __builtin_bit_cast(double, c->tr_pinned[i]);
  *rel = 0.0;
  for (int i = 0; i < 2; ++i)
    if (v[2 * i + 1] > 0.0) *rel = std::max(*rel, v[2 * i] / v[2 * i + 1]);
  return 0;
}

// tolerance of the check: rounding of the lattice phases e^{ik.T} is ~1e-15 relative; a complex
// basis or a shifted k-mesh violates the symmetry at O(1)
constexpr double kTrTol = 1e-9;

// the composite build's context-wide stage settings, restored when fisdf_build returns (ADVICE
// r04: a stage-API caller on the same context must not inherit them)
struct StageSettings {
  fisdf_ctx* c;
  bool time_reversal;
  int force_pivoted, fit_mode, half_grid, factor_hi;
  double omega;
  explicit StageSettings(fisdf_ctx* cc)
      : c(cc), time_reversal(cc->time_reversal), force_pivoted(cc->force_pivoted),
        fit_mode(cc->fit_mode), half_grid(cc->half_grid), factor_hi(cc->factor_hi),
        omega(cc->omega) {}
  ~StageSettings() {
    c->time_reversal = time_reversal;
    c->force_pivoted = force_pivoted;
    c->fit_mode = fit_mode;
    c->half_grid = half_grid;
    c->factor_hi = factor_hi;
    c->omega = omega;
  }
};

}  // namespace

extern "C" {

int fisdf_check_time_reversal(fisdf_ctx* c, const void* d_a, long k_stride, long per_k,
                              const int kmesh[3], double* h_out) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(d_a && kmesh && h_out, "check_time_reversal: null argument");
  FISDF_CHECK(kmesh[0] > 0 && kmesh[1] > 0 && kmesh[2] > 0, "check_time_reversal: bad k-mesh");
  FISDF_CHECK(per_k > 0 && k_stride >= per_k, "check_time_reversal: bad sizes");
  FISDF_TRY(tr_alloc(c));
  FISDF_HIP(hipEventSynchronize(c->ev_tr));
  FISDF_HIP(hipMemsetAsync(c->trmon, 0, 4 * sizeof(unsigned long long), c->stream));
  FISDF_TRY(tr_check(c->stream, (const cplx*)d_a, k_stride, per_k, 1, 1, kmesh, c->trmon));
  unsigned long long h[2];
  FISDF_HIP(hipMemcpyAsync(h, c->trmon, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  FISDF_HIP(hipStreamSynchronize(c->stream));
  h_out[0] = __builtin_bit_cast(double, h[0]);
  h_out[1] = __builtin_bit_cast(double, h[1]);
  return 0;
}

void fisdf_build_opts_default(fisdf_build_opts* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->nip_max = 0;
  o->select_tol = -1.0;
  o->perm = nullptr;
  o->n_perm = 0;
  o->fit_mode = FISDF_FIT_LSTSQ;
  o->fit_tol = kFitTolDefault;
  o->pivoted_fit = -1;
  o->half_grid = -1;
  o->time_reversal = 1;
  o->real_self_conjugate = 1;
  o->omega = 0.0;
}

int fisdf_set_allocator(fisdf_ctx* c, fisdf_alloc_fn alloc, fisdf_free_fn release, void* user) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK((alloc == nullptr) == (release == nullptr), "set_allocator: give both functions or neither");
  FISDF_TRY(fisdf_build_release(c));
  c->alloc_fn = alloc;
  c->free_fn = release;
  c->alloc_user = user;
  return 0;
}

int fisdf_build_release(fisdf_ctx* c) {
  FISDF_TRY(device_guard(c));
  if (c->f_pending) FISDF_TRY(fisdf_factor_x4_wait(c, nullptr));
  build_return_all(c);
  if (!c->owned.empty()) {
    FISDF_HIP(hipStreamSynchronize(c->stream));
    for (auto& kv : c->owned)
      if (kv.second.first) FISDF_HIP(hipFree(kv.second.first));
    c->owned.clear();
  }
  return 0;
}

}  // extern "C"

namespace {

// kshard.assign_q: longest-processing-time greedy over the fit positions (most expensive first,
// each to the least loaded rank, ties to the lower rank), each rank's positions ascending
std::vector<std::vector<int>> assign_q(const std::vector<double>& cost, int size) {
  std::vector<int> order(cost.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return cost[x] > cost[y]; });
  std::vector<double> load(size, 0.0);
  std::vector<std::vector<int>> parts(size);
  for (int i : order) {
    int r = 0;
    for (int t = 1; t < size; ++t)
      if (load[t] < load[r]) r = t;
    parts[r].push_back(i);
    load[r] += cost[i];
  }
  for (auto& p : parts) std::sort(p.begin(), p.end());
  return parts;
}

// kshard.shard_range: contiguous balanced [lo, hi) of `rank` among `size`
void shard_range(long n, int rank, int size, long* lo, long* hi) {
  const long base = n / size, rem = n % size;
  *lo = rank * base + std::min<long>(rank, rem);
  *hi = *lo + base + (rank < rem ? 1 : 0);
}

int comm_check(int rc, const char* what) {
  FISDF_CHECK(rc == 0, std::string("build_sharded: the caller's ") + what + " failed");
  return 0;
}

// fisdf_build (comm NULL) and fisdf_build_sharded: ISDF.build() (fftisdf.py:308-325 ->
// build(df_obj), :22-128), the same stage sequence as the Python mirror's build (fisdf/isdf.py
// build(): its unsharded branch, and its k-sharded branch with the caller's collectives)
// FISDF_HOST_TRACE=1 (diagnosis): host timestamps (CLOCK_MONOTONIC, the clock of Python's
// time.perf_counter) of the composite build's hand-offs, to stderr — where the host holds the
// device idle between a step's last kernel and the next step's first
static void host_mark(const char* what) {
  static const bool on = getenv("FISDF_HOST_TRACE") != nullptr;
  if (!on) return;
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  fprintf(stderr, "fisdf-host %.6f %s\n", ts.tv_sec + 1e-9 * ts.tv_nsec, what);
}

int build_impl(fisdf_ctx* c, const fisdf_comm* comm, const void* x0, int ng0, const void* f,
               int nao, const int kmesh[3], const int mesh[3], const double a[9],
               const fisdf_build_opts* opts_in, int* h_nip) {
  host_mark("build enter");
  fisdf_build_opts o;
  fisdf_build_opts_default(&o);
  if (opts_in) o = *opts_in;
  FISDF_CHECK(x0 && f && kmesh && mesh && a && ng0 > 0 && nao > 0, "build: bad arguments");
  FISDF_CHECK(kmesh[0] > 0 && kmesh[1] > 0 && kmesh[2] > 0 && mesh[0] > 0 && mesh[1] > 0 && mesh[2] > 0,
              "build: bad k-mesh or mesh");
  FISDF_CHECK(o.fit_mode >= FISDF_FIT_LSTSQ && o.fit_mode <= FISDF_FIT_BASIC, "build: bad fit_mode");
  FISDF_CHECK(o.perm == nullptr || o.n_perm > 0, "build: perm given without n_perm");
  // the previous build's factor chain may still read x4: wait for it before anything else
  if (c->f_pending) FISDF_TRY(fisdf_factor_x4_wait(c, nullptr));
  StageSettings keep(c);
  fisdf_ctx::Build& B = c->bld;
  const int nk = kmesh[0] * kmesh[1] * kmesh[2];
  const long ngrid = (long)mesh[0] * mesh[1] * mesh[2];
  FISDF_CHECK(ngrid < (1L << 31), "build: mesh too large");
  const int NR = comm ? comm->size : 1, RK = comm ? comm->rank : 0;
  if (comm)
    FISDF_CHECK(NR >= 1 && RK >= 0 && RK < NR && comm->all_to_all && comm->reduce_scatter_f64 &&
                    comm->allreduce_f64 && comm->broadcast,
                "build_sharded: incomplete fisdf_comm");
  // a k-shard's 1/N-grid y build is short, so its factor chain runs at the greatest priority
  // FISDF_FACTOR_PRIO=0/1 (A/B) overrides: 1-GPU least, k-shard greatest
  const char* fpe = getenv("FISDF_FACTOR_PRIO");
  FISDF_TRY(fisdf_set_factor_priority(c, fpe ? (fpe[0] == '1' ? 1 : 0) : (NR > 1 ? 1 : 0)));
  // time reversal (X_{-k} = conj(X_k), real AOs): the selection Gram, x2_k (x4) and fx_k (y)
  // are formed for the representatives k <= -k only.  The inputs are checked on the side
  // stream beside the selection; a violation (complex basis, shifted k-mesh) is found when the
  // selection returns, and the build then starts over with every q fitted
  bool tr = o.time_reversal != 0;
  double tr_dev = 0.0;
  // FISDF_TR_CHECK=0 trusts the inputs (A/B of the check's cost only)
  static const bool tr_check_on = [] {
    const char* e = getenv("FISDF_TR_CHECK");
    return !(e && e[0] == '0');
  }();
  // the check (~25 us) runs on the main stream ahead of the selection, whose read-back brings
  // the verdict along; a violation redoes the selection without the fold and fits every q
  const bool check_tr = tr && tr_check_on;
  if (check_tr) {
    FISDF_TRY(tr_alloc(c));
    FISDF_TRY(tr_check_enqueue(c, c->stream, (const cplx*)x0, ng0, (const cplx*)f, ngrid, nao,
                               kmesh));
  }
  // the previous build's buffers go back to the caller's allocator now, while the check runs
  // (in the mirror each is a Python callback: done first, they left the GPU idle between steps)
  host_mark("tr check enqueued");
  build_return_all(c);
  host_mark("previous buffers returned");
  // X and x4 at their upper bound (the point cap) taken now, while the check runs: the caller's
  // allocator (a Python callback in the mirror, ~40 us each) then no longer sits in the idle gap
  // between the selection's read-back and the gather
  const int nip_ub = o.perm ? o.n_perm : (o.nip_max > 0 ? std::min(o.nip_max, ng0) : 0);
  void *X = nullptr, *x4 = nullptr;
  if (nip_ub > 0) {
    FISDF_TRY(build_alloc(c, BR_X, sizeof(cplx) * (size_t)nk * nip_ub * nao, &X));
    FISDF_TRY(build_alloc(c, BR_X4, sizeof(cplx) * (size_t)nk * nip_ub * nip_ub, &x4));
  }
  // The y build streamed behind the selection (1-GPU composite build, time reversal, a k-mesh
  // the fused kernel covers; FISDF_Y_STREAM=0: off): y is formed at the point cap nip_ub on
  // aux[0] while the selection runs, and is kept when the selection returns exactly nip_ub
  // points with time reversal confirmed — else it is discarded and built the usual way.
  // read per build: the GPU tests compare the two paths in one process (FISDF_Y_STREAM=0: off)
  const bool y_stream_env = [] {
    const char* e = getenv("FISDF_Y_STREAM");
    return !(e && e[0] == '0');
  }();
  static const bool y_real_env = [] {  // the self-conjugate q's y real; FISDF_Y_REAL=0: off
    const char* e = getenv("FISDF_Y_REAL");
    return !(e && e[0] == '0');
  }();
  struct YsScope {  // the request is this build's only: cleared on every exit
    fisdf_ctx* c;
    ~YsScope() {
      // an error between the enqueue and the join leaves the y stream joined all the same, so
      // the buffers it writes are not handed back under it
      (void)ystream_join(c);
      c->ys = fisdf_ctx::YStream();
    }
  } ys_scope{c};
  void* yT_pre = nullptr;  // the y buffer taken before the selection (streamed y)
  std::vector<int> ys_qs, ys_partner;
  std::vector<double> ys_wt;
  if (y_stream_env && !comm && !o.perm && tr && nip_ub > 0 && y_fused_applies(kmesh, nao)) {
    tr_classes(kmesh, true, ys_qs, ys_partner, ys_wt);
    FISDF_TRY(build_alloc(c, BR_Y, sizeof(cplx) * (size_t)ys_qs.size() * nip_ub * ngrid, &yT_pre));
    unsigned long long rmask = 0;
    if (y_real_env && o.real_self_conjugate && fft3d_reads_real(mesh[0], mesh[1], mesh[2]))
      for (int q : ys_qs) {
        const int i2 = q % kmesh[2], i1 = (q / kmesh[2]) % kmesh[1], i0 = q / (kmesh[1] * kmesh[2]);
        if ((2 * i0) % kmesh[0] == 0 && (2 * i1) % kmesh[1] == 0 && (2 * i2) % kmesh[2] == 0)
          rmask |= 1ull << q;
      }
    bool armed = false;
    FISDF_TRY(ystream_arm(c, x0, ng0, f, ngrid * nao, ngrid, nao, nip_ub, kmesh, ys_qs.data(),
                          (int)ys_qs.size(), yT_pre, rmask, &armed));
  }
  host_mark("allocations + y stream armed");
  // interpolation points (:33 -> :357-388), or the caller's
  std::vector<int> perm;
  for (int attempt = 0;; ++attempt) {
    FISDF_TRY(fisdf_set_time_reversal(c, tr ? 1 : 0));
    if (o.perm) {
      perm.assign(o.perm, o.perm + o.n_perm);
    } else {
      const int cap = o.nip_max > 0 ? std::min(o.nip_max, ng0) : ng0;
      perm.assign(cap, 0);
      int npiv = 0, full = 0;
      FISDF_TRY(fisdf_select_points_km(c, x0, kmesh, ng0, nao, cap, o.select_tol, perm.data(),
                                       &npiv, &full));
      c->ys.armed = false;  // a second selection (time reversal refuted) streams nothing
      perm.resize(std::min(cap, npiv));                                           // :383
    }
    if (!check_tr || attempt > 0) break;
    FISDF_TRY(tr_verdict(c, &tr_dev));
    if (tr_dev <= kTrTol) break;
    if (getenv("FISDF_VERBOSE"))
      fprintf(stderr, "fisdf: build: AO inputs violate time reversal (max |a[-k] - conj(a[k])| / "
                      "max |a| = %.3e): every q fitted\n", tr_dev);
    tr = false;
  }
  host_mark("selection read back");
  const int nip = (int)perm.size();
  FISDF_CHECK(nip > 0, "build: no interpolation points");
  const long nn = (long)nip * nip;
  FISDF_CHECK(nip_ub == 0 || nip <= nip_ub, "build: more points than the cap");
  if (!X) FISDF_TRY(build_alloc(c, BR_X, sizeof(cplx) * (size_t)nk * nip * nao, &X));
  FISDF_TRY(fisdf_gather_points(c, x0, nk, ng0, nao, perm.data(), nip, X));        // :388
  if (!x4) FISDF_TRY(build_alloc(c, BR_X4, sizeof(cplx) * (size_t)nk * nn, &x4));
  // FISDF_X4_SIDE=1 (experiment, read per build): with y streamed, x4 on the side stream at the
  // head of the factor chain it feeds.  Beside the streamed y its 0.2 ms DFT kernel stretches to
  // 2.6 ms on either stream and the chain after it to 4 ms; measured +0.3 ms/step on the side
  // stream, and no better at the greatest priority (profiles/r06/r06_x4side)
  const char* x4e = getenv("FISDF_X4_SIDE");
  const bool x4_side = !comm && (x4e && x4e[0] == '1') && c->ys.enqueued && !c->ys.stale && tr &&
                       nip == c->ys.nip;
  if (!x4_side) FISDF_TRY(fisdf_build_x4(c, X, nip, nao, kmesh, a, x4));           // :38-48
  std::vector<int> qs, partner;
  std::vector<double> wt;
  tr_classes(kmesh, tr, qs, partner, wt);
  const int nq = (int)qs.size();
  FISDF_TRY(fisdf_set_pivoted_fit(c, o.pivoted_fit));
  FISDF_TRY(fisdf_set_fit_mode(c, o.fit_mode));
  FISDF_TRY(fisdf_set_half_grid(c, o.half_grid));
  FISDF_TRY(fisdf_set_omega(c, o.omega));
  // this rank's q: the fitted q shared by cost, longest first (one GPU: all of them)
  std::vector<double> cost(nq);
  for (int i = 0; i < nq; ++i)
    cost[i] = (o.real_self_conjugate && partner[qs[i]] == qs[i]) ? 0.6 : 1.0;
  const std::vector<std::vector<int>> parts = assign_q(cost, NR);
  std::vector<int> my_qs;
  std::vector<double> my_wt;
  for (int i : parts[RK]) my_qs.push_back(qs[i]), my_wt.push_back(wt[i]);
  const int nmine = (int)my_qs.size();
  void *Wq, *Ws, *W0;
  std::vector<int> ranks(nmine, 0);
  int used = 0, ncod = 0;
  long row0 = 0, row1 = nip;
  // the streamed y is this build's y when the selection gave the cap's points under time
  // reversal (the q-list it was formed for) and the y stream met no stalled wait
  const bool y_streamed = tr && ystream_valid(c, nip, qs.data(), nq);
  // a discarded streamed y: its stream joins before its buffer goes back (the usual build may be
  // handed the same memory)
  if (c->ys.enqueued && !y_streamed) FISDF_TRY(ystream_join(c));
  if (yT_pre && !y_streamed) {
    FISDF_TRY(build_return(c, yT_pre));
    yT_pre = nullptr;
  }
  FISDF_CHECK(!x4_side || y_streamed, "build: x4 on the side stream without the streamed y");
  if (!comm) {
    // the factorisation (replaces zgelsy's QRCP, :108) on the side stream, overlapped with y
    FISDF_TRY(fisdf_factor_x4_mark(c));
    if (x4_side) {  // X gathered (ev_x4) -> x4 -> the factor chain, all on the side stream
      FISDF_HIP(hipStreamWaitEvent(c->side, c->ev_x4, 0));
      FISDF_TRY(build_x4_on(c, c->side, &c->ws_x4, X, nip, nao, kmesh, a, x4));  // :38-48
    }
    void* yT = yT_pre;
    if (!yT) FISDF_TRY(build_alloc(c, BR_Y, sizeof(cplx) * (size_t)nq * nip * ngrid, &yT));
    // the self-conjugate q's y real (half their y writes and FFT reads); FISDF_Y_REAL=0: off
    struct YRealScope {  // the mode is this build's only: reset on every exit
      fisdf_ctx* c;
      ~YRealScope() { c->y_real_store = false; c->y_real_slot.clear(); }
    } y_real_scope{c};
    c->y_real_store = y_real_env && o.real_self_conjugate && fft3d_reads_real(mesh[0], mesh[1], mesh[2]);
    if (y_streamed) {
      // the fit comes after the y stream; joined only now, after x4 has been marked for the
      // factor chain, so the side stream does not wait for y
      FISDF_TRY(ystream_join(c));
      // what fisdf_build_y_qs records for the fit: the slots stored real
      c->y_real_slot.assign(nq, 0);
      for (int i = 0; i < nq; ++i) c->y_real_slot[i] = (c->ys.rmask >> qs[i]) & 1ull ? 1 : 0;
    } else {
      FISDF_TRY(fisdf_build_y_qs(c, f, ngrid * nao, 0, (int)ngrid, (int)ngrid, X, nip, nao, kmesh,
                                 a, qs.data(), nq, yT));                           // :67-87
    }
    FISDF_TRY(fisdf_factor_x4_async(c, x4, qs.data(), nq, nip, o.fit_tol,
                                    o.real_self_conjugate ? kmesh : nullptr));
    FISDF_TRY(build_alloc(c, BR_WQ, sizeof(cplx) * (size_t)nq * nn, &Wq));
    // the fit waits for the factor's verdict itself
    FISDF_TRY(fisdf_fit_coulomb_qs(c, qs.data(), nq, yT, nip, mesh, kmesh, a, Wq)); // :97-121
    host_mark("fit enqueued");
    FISDF_TRY(fisdf_factor_x4_wait(c, ranks.data()));
    host_mark("factor ranks read back");
    FISDF_TRY(fisdf_factor_info(c, &used));
    FISDF_TRY(fisdf_min_norm_info(c, &ncod));
    // a block that waited past its bound built y from unfinished pivots
    if (y_streamed) FISDF_TRY(ystream_check(c));
    // y is dead once the fit is enqueued: fit_coulomb_qs joined its lanes and FFT stream into
    // c->stream (aux_join, checked by build_return), so a stream-ordered free cannot overtake a
    // reader
    FISDF_TRY(build_return(c, yT));
    FISDF_TRY(build_alloc(c, BR_WS, sizeof(double) * (size_t)nk * nn, &Ws));
    FISDF_TRY(fisdf_build_ws_qs(c, Wq, qs.data(), wt.data(), nq, nip, kmesh, a, Ws)); // :204-207
    W0 = Wq;  // q = 0 is slot 0 (the smallest representative)
  } else {
    // y on this rank's plane-aligned grid slice for every fitted q (y_k = Phi^T (Phi fx_k)^2
    // mixes all k at each grid point, :79-84), then one all-to-all per local q hands every rank
    // its own q on the whole grid (kshard.exchange_y_chunked)
    std::vector<long> g0s(NR), ngs(NR);
    const long plane = (long)mesh[1] * mesh[2];
    for (int r = 0; r < NR; ++r) {
      long p0, p1;
      shard_range(mesh[0], r, NR, &p0, &p1);
      g0s[r] = p0 * plane;
      ngs[r] = (p1 - p0) * plane;
    }
    const long ngme = ngs[RK];
    if (nmine) FISDF_TRY(fisdf_factor_x4_mark(c));
    void *send, *recv;
    FISDF_TRY(build_alloc(c, BR_SEND, sizeof(cplx) * (size_t)nq * nip * std::max(ngme, 1L), &send));
    if (ngme)
      FISDF_TRY(fisdf_build_y_qs(c, (const cplx*)f + g0s[RK] * nao, ngrid * nao, 0, (int)ngme,
                                 (int)ngme, X, nip, nao, kmesh, a, qs.data(), nq, send));
    if (nmine)
      FISDF_TRY(fisdf_factor_x4_async(c, x4, my_qs.data(), nmine, nip, o.fit_tol,
                                      o.real_self_conjugate ? kmesh : nullptr));
    FISDF_TRY(build_alloc(c, BR_Y, sizeof(cplx) * (size_t)std::max(nmine, 1) * nip * ngrid, &recv));
    // the exchange runs on its own stream while this rank factorises and fits its earlier q
    if (!c->comm_stream) {
      FISDF_HIP(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
      FISDF_HIP(hipEventCreateWithFlags(&c->ev_comm, hipEventDisableTiming));
    }
    FISDF_HIP(hipEventRecord(c->ev_comm, c->stream));
    FISDF_HIP(hipStreamWaitEvent(c->comm_stream, c->ev_comm, 0));
    size_t nmax = 0;
    for (const auto& p : parts) nmax = std::max(nmax, p.size());
    std::vector<const void*> sp(NR);
    std::vector<void*> rp(NR);
    std::vector<size_t> sb(NR), rb(NR);
    for (size_t j = 0; j < nmax; ++j) {
      const bool mine = j < (size_t)nmine;
      cplx* rj = (cplx*)recv + (long)j * nip * ngrid;
      for (int r = 0; r < NR; ++r) {
        const bool to_r = j < parts[r].size();
        sp[r] = to_r ? (const cplx*)send + (long)parts[r][j] * nip * ngme : nullptr;
        sb[r] = to_r ? sizeof(cplx) * (size_t)nip * ngme : 0;
        // piece j = concat over ranks p of the (nip, ng_p) blocks: p's block at nip * g0_p
        rp[r] = mine ? rj + (long)nip * g0s[r] : nullptr;
        rb[r] = mine ? sizeof(cplx) * (size_t)nip * ngs[r] : 0;
      }
      FISDF_TRY(comm_check(comm->all_to_all(comm->user, sp.data(), sb.data(), rp.data(), rb.data(),
                                            c->comm_stream), "all_to_all"));
      if (mine)
        FISDF_TRY(set_y_slices_on(c, (int)j, rj, NR, g0s.data(), ngs.data(), c->comm_stream));
    }
    FISDF_HIP(hipEventRecord(c->ev_comm, c->comm_stream));
    FISDF_TRY(build_alloc(c, BR_WQ, sizeof(cplx) * (size_t)std::max(nmine, 1) * nn, &Wq));
    if (nmine) {
      // one call over the whole shard: its lanes start each q when that q's piece has landed
      FISDF_TRY(fisdf_fit_coulomb_qs(c, my_qs.data(), nmine, nullptr, nip, mesh, kmesh, a, Wq));
      FISDF_TRY(fisdf_factor_x4_wait(c, ranks.data()));
      FISDF_TRY(fisdf_factor_info(c, &used));
      FISDF_TRY(fisdf_min_norm_info(c, &ncod));
    }
    // the send and receive buffers stay the build's until the exchange is done
    FISDF_HIP(hipStreamWaitEvent(c->stream, c->ev_comm, 0));
    FISDF_TRY(build_return(c, recv));
    FISDF_TRY(build_return(c, send));
    // W_s = sqrt(nk) Re(sum_q Phi[R,q] W_q) (:204-207) mixes every rank's q: each rank forms every
    // rank's interpolation-point row block of its partial sum, reduce-scattered by rows
    std::vector<int> bounds(NR + 1);
    long rmax = 0;
    for (int r = 0; r < NR; ++r) {
      long lo, hi;
      shard_range(nip, r, NR, &lo, &hi);
      bounds[r] = (int)lo;
      bounds[r + 1] = (int)hi;
      rmax = std::max(rmax, hi - lo);
      if (r == RK) row0 = lo, row1 = hi;
    }
    const long chunk = (long)nk * std::max(rmax, 1L) * nip;
    void* Wsb;
    FISDF_TRY(build_alloc(c, BR_WSB, sizeof(double) * (size_t)chunk * NR, &Wsb));
    FISDF_HIP(hipMemsetAsync(Wsb, 0, sizeof(double) * (size_t)chunk * NR, c->stream));
    FISDF_TRY(fisdf_build_ws_blocks(c, Wq, my_qs.data(), my_wt.data(), nmine, nip, kmesh, a, NR,
                                    bounds.data(), chunk, Wsb));
    FISDF_TRY(build_alloc(c, BR_WS, sizeof(double) * (size_t)chunk, &Ws));
    FISDF_TRY(comm_check(comm->reduce_scatter_f64(comm->user, (const double*)Wsb, (double*)Ws,
                                                  (size_t)chunk, c->stream), "reduce_scatter_f64"));
    FISDF_TRY(build_return(c, Wsb));
    // W_0 for get_j (:159) from the rank fitting q = 0 (position 0 of the fit order, its slot 0)
    int owner0 = 0;
    for (int r = 0; r < NR; ++r)
      if (!parts[r].empty() && parts[r][0] == 0) owner0 = r;
    FISDF_TRY(build_alloc(c, BR_W0, sizeof(cplx) * (size_t)nn, &W0));
    if (RK == owner0)
      FISDF_HIP(hipMemcpyAsync(W0, Wq, sizeof(cplx) * nn, hipMemcpyDeviceToDevice, c->stream));
    FISDF_TRY(comm_check(comm->broadcast(comm->user, W0, sizeof(cplx) * nn, owner0, c->stream),
                         "broadcast"));
  }
  B.valid = true;
  B.nk = nk;
  B.nip = nip;
  B.nao = nao;
  B.ng0 = ng0;
  B.nfit = nmine;
  B.used_pivoted = used;
  B.min_norm = ncod;
  B.time_reversal = tr ? 1 : 0;
  B.tr_deviation = tr_dev;
  for (int i = 0; i < 3; ++i) B.kmesh[i] = kmesh[i], B.mesh[i] = mesh[i];
  for (int i = 0; i < 9; ++i) B.a[i] = a[i];
  B.perm = perm;
  B.fit_qs = my_qs;
  B.partner = partner;
  B.ranks = ranks;
  B.wt = my_wt;
  B.X = X;
  B.x4 = x4;
  B.Wq = Wq;
  B.Ws = Ws;
  B.W0 = W0;
  B.sharded = comm != nullptr;
  B.y_streamed = y_streamed;
  if (comm) B.comm = *comm;
  B.shard_rank = RK;
  B.shard_size = NR;
  B.row0 = (int)row0;
  B.row1 = (int)row1;
  if (h_nip) *h_nip = nip;
  host_mark("build return");
  return 0;
}

}  // namespace

extern "C" {

int fisdf_build(fisdf_ctx* c, const void* x0, int ng0, const void* f, int nao, const int kmesh[3],
                const int mesh[3], const double a[9], const fisdf_build_opts* opts, int* h_nip) {
  FISDF_TRY(device_guard(c));
  return build_impl(c, nullptr, x0, ng0, f, nao, kmesh, mesh, a, opts, h_nip);
}

int fisdf_build_sharded(fisdf_ctx* c, const fisdf_comm* comm, const void* x0, int ng0,
                        const void* f, int nao, const int kmesh[3], const int mesh[3],
                        const double a[9], const fisdf_build_opts* opts, int* h_nip) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(comm != nullptr, "build_sharded: comm is null (fisdf_build is the 1-GPU build)");
  return build_impl(c, comm, x0, ng0, f, nao, kmesh, mesh, a, opts, h_nip);
}

int fisdf_y_stream_arm(fisdf_ctx* c, const void* x0, int ng0, const void* f, long f_kstride,
                       int m, int nao, int nip_max, const int kmesh[3], const int* h_qs, int nq,
                       void* yT, int* h_armed) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(kmesh && h_armed && ng0 > 0 && nao > 0, "y_stream_arm: bad arguments");
  FISDF_TRY(check_qlist(h_qs, nq, kmesh[0] * kmesh[1] * kmesh[2], "y_stream_arm"));
  FISDF_CHECK(c->ys.enqueued == false, "y_stream_arm: the previous streamed y is not finished");
  bool armed = false;
  if (c->time_reversal)  // the fused kernel folds fx over k <= -k
    FISDF_TRY(ystream_arm(c, x0, ng0, f, f_kstride, m, nao, nip_max, kmesh, h_qs, nq, yT, 0,
                          &armed));
  *h_armed = armed ? 1 : 0;
  return 0;
}

int fisdf_y_stream_finish(fisdf_ctx* c, int nip, int* h_streamed) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(h_streamed, "y_stream_finish: null output");
  const bool ok = c->ys.enqueued && ystream_valid(c, nip, c->ys.qs.data(), (int)c->ys.qs.size());
  const bool had = c->ys.enqueued;
  FISDF_TRY(ystream_join(c));
  if (had) FISDF_TRY(ystream_check(c));
  *h_streamed = ok ? 1 : 0;
  c->ys = fisdf_ctx::YStream();
  return 0;
}

int fisdf_build_y_streamed(fisdf_ctx* c, int* h_streamed) {
  FISDF_TRY(ctx_guard(c));
  FISDF_CHECK(h_streamed, "build_y_streamed: null output");
  *h_streamed = c->bld.valid && c->bld.y_streamed ? 1 : 0;
  return 0;
}

int fisdf_build_get(fisdf_ctx* c, fisdf_build_result* out) {
  FISDF_TRY(ctx_guard(c));
  FISDF_CHECK(out != nullptr, "build_get: out is null");
  const fisdf_ctx::Build& B = c->bld;
  FISDF_CHECK(B.valid, "build_get: no build (call fisdf_build first)");
  out->nk = B.nk;
  out->nip = B.nip;
  out->nao = B.nao;
  out->nfit = B.nfit;
  out->used_pivoted_fit = B.used_pivoted;
  out->min_norm_slots = B.min_norm;
  out->perm = B.perm.data();
  out->fit_qs = B.fit_qs.data();
  out->ranks = B.ranks.data();
  out->partner = B.partner.data();
  out->d_X = B.X;
  out->d_x4 = B.x4;
  out->d_Wq = B.Wq;
  out->d_Ws = B.Ws;
  out->time_reversal = B.time_reversal;
  out->tr_deviation = B.tr_deviation;
  out->shard_rank = B.shard_rank;
  out->shard_size = B.shard_size;
  out->row0 = B.row0;
  out->row1 = B.row1;
  out->d_W0 = B.W0;
  return 0;
}

int fisdf_get_x(fisdf_ctx* c, void* h_x) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(c->bld.valid && h_x, "get_x: no build or null output");
  const auto& B = c->bld;
  return fisdf_memcpy_dtoh(c, h_x, B.X, sizeof(cplx) * (size_t)B.nk * B.nip * B.nao);
}

int fisdf_get_w0(fisdf_ctx* c, void* h_w0) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(c->bld.valid && h_w0, "get_w0: no build or null output");
  const auto& B = c->bld;  // q = 0 is always fitted (slot 0: the smallest representative)
  return fisdf_memcpy_dtoh(c, h_w0, B.W0, sizeof(cplx) * (size_t)B.nip * B.nip);
}

int fisdf_get_wq(fisdf_ctx* c, void* h_wq) {
  FISDF_TRY(device_guard(c));
  FISDF_CHECK(c->bld.valid && h_wq, "get_wq: no build or null output");
  const auto& B = c->bld;
  FISDF_CHECK(B.shard_size == 1, "get_wq: the W_q of a sharded build are distributed over the "
                                 "ranks (fisdf_build_get: this rank's fit_qs and d_Wq)");
  const size_t nn = (size_t)B.nip * B.nip;
  cplx* h = (cplx*)h_wq;
  std::vector<int> slot(B.nk, -1);
  for (int i = 0; i < B.nfit; ++i) slot[B.fit_qs[i]] = i;
  for (int i = 0; i < B.nfit; ++i)
    FISDF_HIP(hipMemcpyAsync(h + (size_t)B.fit_qs[i] * nn, (const cplx*)B.Wq + i * nn,
                             sizeof(cplx) * nn, hipMemcpyDeviceToHost, c->stream));
  FISDF_HIP(hipStreamSynchronize(c->stream));
  for (int q = 0; q < B.nk; ++q) {  // W_{-q} = conj(W_q) (x4_s, y_s real: fftisdf.py:43,81)
    if (slot[q] >= 0) continue;
    const int p = B.partner[q];
    FISDF_CHECK(p >= 0 && p < B.nk && slot[p] >= 0, "get_wq: q neither fitted nor a partner");
    for (size_t e = 0; e < nn; ++e) h[(size_t)q * nn + e] = cconj(h[(size_t)p * nn + e]);
  }
  return 0;
}

// fftisdf.py:390-408: K (get_k_kpts, :173-228) enqueued before J (get_j_kpts, :133-171)
int fisdf_get_jk(fisdf_ctx* c, const void* dms, int nset, int with_j, int with_k, void* vj, void* vk) {
  FISDF_TRY(device_guard(c));
  const auto& B = c->bld;
  FISDF_CHECK(B.valid, "get_jk: no build (call fisdf_build first)");
  FISDF_CHECK(dms && nset > 0, "get_jk: no density matrices");
  FISDF_CHECK((!with_j || vj) && (!with_k || vk), "get_jk: missing output");
  if (!B.sharded) {
    if (with_k)
      FISDF_TRY(fisdf_get_k_rows(c, B.X, B.Ws, dms, nset, B.nip, B.nao, B.kmesh, B.a, 0, B.nip, vk));
    if (with_j)
      FISDF_TRY(fisdf_get_j_rows(c, B.X, B.W0, dms, nset, B.nk, B.nip, B.nao, 0, B.nip, vj));
    return 0;
  }
  // sharded: this rank's interpolation-point rows (its W_s rows), then the sums over the ranks
  // (fftisdf.py:166,225 contract over all points)
  const size_t nv = 2 * (size_t)nset * B.nk * B.nao * B.nao;
  if (with_k) {
    FISDF_TRY(fisdf_get_k_rows_local(c, B.X, B.Ws, dms, nset, B.nip, B.nao, B.kmesh, B.a, B.row0,
                                     B.row1, vk));
    FISDF_TRY(comm_check(B.comm.allreduce_f64(B.comm.user, (double*)vk, nv, c->stream),
                         "allreduce_f64"));
  }
  if (with_j) {
    FISDF_TRY(fisdf_get_j_rows(c, B.X, B.W0, dms, nset, B.nk, B.nip, B.nao, B.row0, B.row1, vj));
    FISDF_TRY(comm_check(B.comm.allreduce_f64(B.comm.user, (double*)vj, nv, c->stream),
                         "allreduce_f64"));
  }
  return 0;
}

}  // extern "C"
