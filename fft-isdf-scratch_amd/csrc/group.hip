// fisdf_group: one process driving the k-sharded build on several GPUs (SURVEY §8(b)'s
// fisdf_create(ndev, dev_ids, ...)): a context and a stream per rank, rank r on devices[r], the
// ranks joined by a struct fisdf_comm, and every group call run as one host thread per rank
// through the same entries an MPI caller uses (fisdf_build_sharded, fisdf_get_jk).
//
// Collectives (kind):
//   FISDF_GROUP_RCCL  the library's RCCL fisdf_comm (comm.hip), one communicator per rank, all
//                     made by one ncclCommInitAll (all-or-nothing); distinct devices (xGMI)
//   FISDF_GROUP_COPY  device copies between the ranks' own buffers (hipMemcpyPeerAsync, which
//                     also serves ranks sharing a device) ordered by per-rank events, with a host
//                     barrier between publishing and reading; sums in rank order on every rank,
//                     so all ranks hold identical results.  A rank that fails releases the others
//                     from the barrier, and their collectives then fail instead of waiting.
// The ranks' selection kernels are cooperative launches, which pchol.hip serialises process-wide
// (concurrent ones from several threads left the HIP runtime crashing in its exit handlers).
#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "common.h"
#include "fisdf.h"

namespace fisdf {
namespace {

__global__ void add_f64_kernel(double* __restrict__ dst, const double* __restrict__ src, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    dst[i] += src[i];
}

struct Barrier {
  std::mutex m;
  std::condition_variable cv;
  int n = 0, waiting = 0;
  long gen = 0;
  bool abort = false;
  bool wait() {
    std::unique_lock<std::mutex> lk(m);
    if (abort) return false;
    const long g = gen;
    if (++waiting == n) {
      waiting = 0;
      ++gen;
      cv.notify_all();
      return true;
    }
    cv.wait(lk, [&] { return gen != g || abort; });
    return gen != g;
  }
  void fail() {
    std::lock_guard<std::mutex> lk(m);
    abort = true;
    cv.notify_all();
  }
  void reset() {
    std::lock_guard<std::mutex> lk(m);
    abort = false;
    waiting = 0;
  }
};

// what the ranks publish for one collective, and the per-rank events and scratch
struct Hub {
  int n = 0;
  std::vector<int> dev;
  Barrier bar;
  std::vector<const void* const*> send;
  std::vector<const size_t*> sbytes;
  std::vector<const void*> buf;
  std::vector<hipEvent_t> ready, done;
  std::vector<double*> tmp;
  std::vector<size_t> tmp_n;
};

struct CopyRank {
  Hub* hub;
  int rank;
};

// scratch of rank r: at least n doubles on its device
int scratch(Hub* h, int r, size_t n, double** out) {
  if (h->tmp_n[r] < n) {
    if (h->tmp[r]) FISDF_HIP(hipFree(h->tmp[r]));
    h->tmp[r] = nullptr;
    h->tmp_n[r] = 0;
    FISDF_HIP(hipMalloc(&h->tmp[r], sizeof(double) * n));
    h->tmp_n[r] = n;
  }
  *out = h->tmp[r];
  return 0;
}

int add_into(hipStream_t s, double* dst, const double* src, size_t n) {
  if (n == 0) return 0;
  const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(add_f64_kernel, dim3(blocks), dim3(256), 0, s, dst, src, n);
  FISDF_HIP(hipGetLastError());
  return 0;
}

// the tail every collective shares: this rank's reads of the others' buffers are enqueued
// (done[i]); it then waits for every rank's reads of its own buffers before its stream goes on,
// and a last barrier keeps the events from being re-recorded before all waits are enqueued
int finish(Hub* h, int i, hipStream_t s) {
  FISDF_HIP(hipEventRecord(h->done[i], s));
  if (!h->bar.wait()) return -1;
  for (int j = 0; j < h->n; ++j)
    if (j != i) FISDF_HIP(hipStreamWaitEvent(s, h->done[j], 0));
  return h->bar.wait() ? 0 : -1;
}

int copy_all_to_all(void* user, const void* const* send, const size_t* sbytes, void* const* recv,
                    const size_t* rbytes, void* stream) {
  auto* u = static_cast<CopyRank*>(user);
  Hub* h = u->hub;
  const int i = u->rank;
  hipStream_t s = (hipStream_t)stream;
  FISDF_HIP(hipEventRecord(h->ready[i], s));
  h->send[i] = send;
  h->sbytes[i] = sbytes;
  if (!h->bar.wait()) return -1;
  for (int j = 0; j < h->n; ++j) {
    if (rbytes[j] == 0) continue;
    FISDF_CHECK(h->sbytes[j][i] == rbytes[j], "group all_to_all: piece sizes disagree");
    FISDF_HIP(hipStreamWaitEvent(s, h->ready[j], 0));
    FISDF_HIP(hipMemcpyPeerAsync(recv[j], h->dev[i], h->send[j][i], h->dev[j], rbytes[j], s));
  }
  return finish(h, i, s);
}

int copy_reduce_scatter(void* user, const double* send, double* recv, size_t count, void* stream) {
  auto* u = static_cast<CopyRank*>(user);
  Hub* h = u->hub;
  const int i = u->rank;
  hipStream_t s = (hipStream_t)stream;
  FISDF_HIP(hipEventRecord(h->ready[i], s));
  h->buf[i] = send;
  if (!h->bar.wait()) return -1;
  double* t = nullptr;
  FISDF_TRY(scratch(h, i, std::max<size_t>(count, 1), &t));
  for (int j = 0; j < h->n; ++j) {  // rank order: the same sum on every rank
    FISDF_HIP(hipStreamWaitEvent(s, h->ready[j], 0));
    const double* src = (const double*)h->buf[j] + (size_t)i * count;
    FISDF_HIP(hipMemcpyPeerAsync(j == 0 ? recv : t, h->dev[i], src, h->dev[j],
                                 sizeof(double) * count, s));
    if (j > 0) FISDF_TRY(add_into(s, recv, t, count));
  }
  return finish(h, i, s);
}

int copy_allreduce(void* user, double* buf, size_t count, void* stream) {
  auto* u = static_cast<CopyRank*>(user);
  Hub* h = u->hub;
  const int i = u->rank, n = h->n;
  hipStream_t s = (hipStream_t)stream;
  FISDF_HIP(hipEventRecord(h->ready[i], s));
  h->buf[i] = buf;
  if (!h->bar.wait()) return -1;
  // every rank's input copied out first (the sums below overwrite the ranks' buffers in place)
  double* t = nullptr;
  FISDF_TRY(scratch(h, i, std::max<size_t>((size_t)n * count, 1), &t));
  for (int j = 0; j < n; ++j) {
    FISDF_HIP(hipStreamWaitEvent(s, h->ready[j], 0));
    FISDF_HIP(hipMemcpyPeerAsync(t + (size_t)j * count, h->dev[i], h->buf[j], h->dev[j],
                                 sizeof(double) * count, s));
  }
  FISDF_TRY(finish(h, i, s));
  FISDF_HIP(hipMemcpyAsync(buf, t, sizeof(double) * count, hipMemcpyDeviceToDevice, s));
  for (int j = 1; j < n; ++j) FISDF_TRY(add_into(s, buf, t + (size_t)j * count, count));
  return 0;
}

int copy_broadcast(void* user, void* buf, size_t bytes, int root, void* stream) {
  auto* u = static_cast<CopyRank*>(user);
  Hub* h = u->hub;
  const int i = u->rank;
  hipStream_t s = (hipStream_t)stream;
  FISDF_HIP(hipEventRecord(h->ready[i], s));
  h->buf[i] = buf;
  if (!h->bar.wait()) return -1;
  if (i != root && bytes) {
    FISDF_HIP(hipStreamWaitEvent(s, h->ready[root], 0));
    FISDF_HIP(hipMemcpyPeerAsync(buf, h->dev[i], h->buf[root], h->dev[root], bytes, s));
  }
  return finish(h, i, s);
}

}  // namespace

int rccl_init_all(int n, const int* devices, fisdf_comm* out);  // comm.hip

}  // namespace fisdf

using namespace fisdf;

struct fisdf_group {
  int n = 0, kind = 0;
  std::vector<int> dev;
  std::vector<hipStream_t> stream;
  std::vector<fisdf_ctx*> ctx;
  std::vector<fisdf_comm> comm;
  std::vector<CopyRank> copy_rank;
  Hub hub;
  std::string err;
};

namespace {

// run fn(rank) on one thread per rank; the first failure's message is kept on the group
int run_ranks(fisdf_group* g, const std::function<int(int)>& fn) {
  g->hub.bar.reset();
  std::vector<int> rc(g->n, 0);
  std::vector<std::string> msg(g->n);
  std::vector<std::thread> th;
  for (int r = 0; r < g->n; ++r)
    th.emplace_back([&, r] {
      (void)hipSetDevice(g->dev[r]);
      rc[r] = fn(r);
      if (rc[r] != 0) {
        const char* m = (int)g->ctx.size() > r ? fisdf_last_error(g->ctx[r]) : nullptr;
        if (!m || !*m) m = fisdf_last_error(nullptr);
        msg[r] = m ? m : "";
        g->hub.bar.fail();  // the others leave their collectives instead of waiting
      }
    });
  for (auto& t : th) t.join();
  for (int r = 0; r < g->n; ++r)
    if (rc[r] != 0) {
      g->err = "rank " + std::to_string(r) + ": " + msg[r];
      return rc[r];
    }
  g->err.clear();
  return 0;
}

}  // namespace

extern "C" {

int fisdf_group_create(int n, const int* devices, int kind, fisdf_group** out) {
  FISDF_CHECK(out && devices && n >= 1, "group_create: bad arguments");
  FISDF_CHECK(kind == FISDF_GROUP_COPY || kind == FISDF_GROUP_RCCL, "group_create: bad kind");
  *out = nullptr;
  auto* g = new fisdf_group();
  g->n = n;
  g->kind = kind;
  g->dev.assign(devices, devices + n);
  // m by value: a message taken from g->err must outlive the group it belongs to
  auto fail = [&](std::string m) {
    fisdf_group_destroy(g);
    FISDF_CHECK(false, "group_create: " + m);
    return -1;
  };
  for (int r = 0; r < n; ++r) {
    hipStream_t s = nullptr;
    if (hipSetDevice(g->dev[r]) != hipSuccess ||
        hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
      return fail("no stream on device " + std::to_string(g->dev[r]));
    g->stream.push_back(s);
    fisdf_ctx* c = nullptr;
    if (fisdf_create(g->dev[r], s, &c) != 0) return fail(fisdf_last_error(nullptr));
    g->ctx.push_back(c);
  }
  g->comm.assign(n, fisdf_comm{});
  if (kind == FISDF_GROUP_COPY) {
    Hub& h = g->hub;
    h.n = n;
    h.dev = g->dev;
    h.bar.n = n;
    h.send.assign(n, nullptr);
    h.sbytes.assign(n, nullptr);
    h.buf.assign(n, nullptr);
    h.tmp.assign(n, nullptr);
    h.tmp_n.assign(n, 0);
    h.ready.assign(n, nullptr);
    h.done.assign(n, nullptr);
    g->copy_rank.resize(n);
    for (int r = 0; r < n; ++r) {
      if (hipSetDevice(g->dev[r]) != hipSuccess ||
          hipEventCreateWithFlags(&h.ready[r], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&h.done[r], hipEventDisableTiming) != hipSuccess)
        return fail("no events on device " + std::to_string(g->dev[r]));
      g->copy_rank[r] = CopyRank{&h, r};
      fisdf_comm& c = g->comm[r];
      c.rank = r;
      c.size = n;
      c.user = &g->copy_rank[r];
      c.all_to_all = copy_all_to_all;
      c.reduce_scatter_f64 = copy_reduce_scatter;
      c.allreduce_f64 = copy_allreduce;
      c.broadcast = copy_broadcast;
    }
  } else {
    g->hub.bar.n = n;
    // one call for every rank (ncclCommInitAll): no rank can be left blocked in its init when
    // another rank's device fails to join
    if (rccl_init_all(n, g->dev.data(), g->comm.data()) != 0)
      return fail(fisdf_last_error(nullptr));
  }
  *out = g;
  return 0;
}

int fisdf_group_destroy(fisdf_group* g) {
  if (!g) return 0;
  for (int r = 0; r < (int)g->comm.size(); ++r)
    if (g->kind == FISDF_GROUP_RCCL && g->comm[r].user) (void)fisdf_comm_rccl_destroy(&g->comm[r]);
  for (fisdf_ctx* c : g->ctx) (void)fisdf_destroy(c);
  Hub& h = g->hub;
  for (int r = 0; r < (int)h.ready.size(); ++r) {
    (void)hipSetDevice(g->dev[r]);
    if (h.ready[r]) (void)hipEventDestroy(h.ready[r]);
    if (h.done[r]) (void)hipEventDestroy(h.done[r]);
    if (h.tmp[r]) (void)hipFree(h.tmp[r]);
  }
  for (int r = 0; r < (int)g->stream.size(); ++r) {
    (void)hipSetDevice(g->dev[r]);
    (void)hipStreamDestroy(g->stream[r]);
  }
  delete g;
  return 0;
}

fisdf_ctx* fisdf_group_ctx(fisdf_group* g, int rank) {
  return (g && rank >= 0 && rank < g->n) ? g->ctx[rank] : nullptr;
}

const char* fisdf_group_last_error(fisdf_group* g) { return g ? g->err.c_str() : ""; }

int fisdf_group_build(fisdf_group* g, const void* const* d_x0, int ng0, const void* const* d_f,
                      int nao, const int kmesh[3], const int mesh[3], const double a[9],
                      const fisdf_build_opts* opts, int* h_nip) {
  if (!g || !d_x0 || !d_f) return -1;
  std::vector<int> nip(g->n, 0);
  const int rc = run_ranks(g, [&](int r) {
    return fisdf_build_sharded(g->ctx[r], &g->comm[r], d_x0[r], ng0, d_f[r], nao, kmesh, mesh, a,
                               opts, &nip[r]);
  });
  if (rc == 0 && h_nip) *h_nip = nip[0];
  return rc;
}

int fisdf_group_get_jk(fisdf_group* g, const void* const* d_dms, int nset, int with_j,
                       int with_k, void* const* d_vj, void* const* d_vk) {
  if (!g || !d_dms) return -1;
  return run_ranks(g, [&](int r) {
    return fisdf_get_jk(g->ctx[r], d_dms[r], nset, with_j, with_k, d_vj ? d_vj[r] : nullptr,
                        d_vk ? d_vk[r] : nullptr);
  });
}

}  // extern "C"
