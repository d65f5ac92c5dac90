// fisdf_comm over RCCL (include/fisdf.h): the collectives of the k-sharded build
// (fisdf_build_sharded) for a C / Fortran caller with one process per GPU.  The library does not
// link librccl: it is opened at run time by the first fisdf_comm_rccl_* call, so libfisdf.so loads
// (and the 1-GPU path runs) where RCCL is absent.
//
// Mapping onto RCCL (xGMI within a node):
//   all_to_all          grouped ncclSend / ncclRecv pairs (uneven and zero-byte pieces: the
//                       per-q exchange of the grid-sliced y, kshard.exchange_y_chunked)
//   reduce_scatter_f64  ncclReduceScatter (W_s row blocks, kshard.reduce_scatter_rows)
//   allreduce_f64       ncclAllReduce (J / K, fftisdf.py:166,225 summed over the ranks' rows)
//   broadcast           ncclBroadcast (W_0 from the rank fitting q = 0)
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <vector>

#include "common.h"
#include "fisdf.h"

namespace {

struct Rccl {
  bool ok = false;
  std::string err;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommInitAll) comm_init_all = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL))) break;
    if (!h) {
      r.err = std::string("RCCL not found: ") + dlerror();
      return;
    }
    bool all = true;
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      all = all && fn != nullptr;
    };
    sym(r.get_unique_id, "ncclGetUniqueId");
    sym(r.comm_init_rank, "ncclCommInitRank");
    sym(r.comm_init_all, "ncclCommInitAll");
    sym(r.comm_destroy, "ncclCommDestroy");
    sym(r.error_string, "ncclGetErrorString");
    sym(r.group_start, "ncclGroupStart");
    sym(r.group_end, "ncclGroupEnd");
    sym(r.send, "ncclSend");
    sym(r.recv, "ncclRecv");
    sym(r.reduce_scatter, "ncclReduceScatter");
    sym(r.all_reduce, "ncclAllReduce");
    sym(r.broadcast, "ncclBroadcast");
    if (!all) {
      r.err = "RCCL lacks a needed symbol";
      return;
    }
    r.ok = true;
  });
  return r;
}

struct RcclComm {
  ncclComm_t comm = nullptr;
  int size = 0;
};

// the callbacks report through the return code (the build names the failing collective)
int rc_of(ncclResult_t e) { return e == ncclSuccess ? 0 : -1; }

int cb_all_to_all(void* user, const void* const* send, const size_t* sbytes, void* const* recv,
                  const size_t* rbytes, void* stream) {
  const Rccl& R = rccl();
  auto* u = static_cast<RcclComm*>(user);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (R.group_start() != ncclSuccess) return -1;
  ncclResult_t e = ncclSuccess;
  for (int r = 0; r < u->size && e == ncclSuccess; ++r) {
    if (sbytes[r]) e = R.send(send[r], sbytes[r], ncclChar, r, u->comm, st);
    if (e == ncclSuccess && rbytes[r]) e = R.recv(recv[r], rbytes[r], ncclChar, r, u->comm, st);
  }
  const ncclResult_t g = R.group_end();
  return e != ncclSuccess ? -1 : rc_of(g);
}

int cb_reduce_scatter(void* user, const double* send, double* recv, size_t count, void* stream) {
  auto* u = static_cast<RcclComm*>(user);
  return rc_of(rccl().reduce_scatter(send, recv, count, ncclFloat64, ncclSum, u->comm,
                                     static_cast<hipStream_t>(stream)));
}

int cb_allreduce(void* user, double* buf, size_t count, void* stream) {
  auto* u = static_cast<RcclComm*>(user);
  return rc_of(rccl().all_reduce(buf, buf, count, ncclFloat64, ncclSum, u->comm,
                                 static_cast<hipStream_t>(stream)));
}

int cb_broadcast(void* user, void* buf, size_t bytes, int root, void* stream) {
  auto* u = static_cast<RcclComm*>(user);
  return rc_of(rccl().broadcast(buf, buf, bytes, ncclChar, root, u->comm,
                                static_cast<hipStream_t>(stream)));
}

void fill_comm(RcclComm* u, int rank, int size, fisdf_comm* out) {
  std::memset(out, 0, sizeof(*out));
  out->rank = rank;
  out->size = size;
  out->user = u;
  out->all_to_all = cb_all_to_all;
  out->reduce_scatter_f64 = cb_reduce_scatter;
  out->allreduce_f64 = cb_allreduce;
  out->broadcast = cb_broadcast;
}

}  // namespace

namespace fisdf {

// every rank of a one-process group at once (fisdf_group, FISDF_GROUP_RCCL): ncclCommInitAll on
// the devices in rank order, from the calling thread — all-or-nothing, so a device that cannot
// join fails the whole call instead of leaving the other ranks blocked inside ncclCommInitRank
int rccl_init_all(int n, const int* devices, fisdf_comm* out) {
  FISDF_CHECK(n >= 1 && devices && out, "comm_rccl_init_all: bad arguments");
  const Rccl& R = rccl();
  FISDF_CHECK(R.ok, "comm_rccl_init_all: " + R.err);
  std::vector<ncclComm_t> comms(n, nullptr);
  const ncclResult_t e = R.comm_init_all(comms.data(), n, devices);
  FISDF_CHECK(e == ncclSuccess, std::string("ncclCommInitAll: ") + R.error_string(e));
  for (int r = 0; r < n; ++r) {
    auto* u = new RcclComm();
    u->comm = comms[r];
    u->size = n;
    fill_comm(u, r, n, &out[r]);
  }
  return 0;
}

}  // namespace fisdf

static_assert(sizeof(ncclUniqueId) == FISDF_COMM_ID_BYTES, "RCCL unique id size");

extern "C" {

int fisdf_comm_rccl_unique_id(unsigned char* h_id) {
  FISDF_CHECK(h_id != nullptr, "comm_rccl_unique_id: null output");
  const Rccl& R = rccl();
  FISDF_CHECK(R.ok, "comm_rccl_unique_id: " + R.err);
  ncclUniqueId id;
  const ncclResult_t e = R.get_unique_id(&id);
  FISDF_CHECK(e == ncclSuccess, std::string("ncclGetUniqueId: ") + R.error_string(e));
  std::memcpy(h_id, &id, sizeof(id));
  return 0;
}

int fisdf_comm_rccl_init(const unsigned char* h_id, int rank, int size, int device,
                         fisdf_comm* out) {
  FISDF_CHECK(h_id && out && size >= 1 && rank >= 0 && rank < size,
              "comm_rccl_init: bad arguments");
  const Rccl& R = rccl();
  FISDF_CHECK(R.ok, "comm_rccl_init: " + R.err);
  FISDF_HIP(hipSetDevice(device));
  ncclUniqueId id;
  std::memcpy(&id, h_id, sizeof(id));
  auto* u = new RcclComm();
  u->size = size;
  const ncclResult_t e = R.comm_init_rank(&u->comm, size, id, rank);
  if (e != ncclSuccess) {
    delete u;
    FISDF_CHECK(false, std::string("ncclCommInitRank: ") + R.error_string(e));
  }
  fill_comm(u, rank, size, out);
  return 0;
}

int fisdf_comm_rccl_destroy(fisdf_comm* comm) {
  if (!comm || !comm->user) return 0;
  FISDF_CHECK(comm->all_to_all == cb_all_to_all, "comm_rccl_destroy: not an RCCL fisdf_comm");
  auto* u = static_cast<RcclComm*>(comm->user);
  const ncclResult_t e = rccl().comm_destroy(u->comm);
  delete u;
  comm->user = nullptr;
  FISDF_CHECK(e == ncclSuccess, "ncclCommDestroy failed");
  return 0;
}

}  // extern "C"
