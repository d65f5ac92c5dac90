"""One rank of the k-sharded C-ABI build (fisdf_build_sharded + fisdf_get_jk, include/fisdf.h)
driven without torch — what a C / Fortran / MPI caller does: ctypes + NumPy, fisdf_malloc /
fisdf_memcpy_* for every buffer, the collectives from the caller through struct fisdf_comm.
tests/test_gpu_capi.py starts SIZE of these (all on GPU 0) and compares each rank's share with
the 1-GPU fisdf_build that rank 0 also runs.

Collectives ("host"): a file mailbox under DIR plus a file barrier — each callback waits for
its stream, moves its pieces through host files and uploads what it receives (ranks sharing one
GPU, as a test; RCCL refuses two ranks on one device).  "rccl": the library's own RCCL
fisdf_comm (fisdf_comm_rccl_*), rank 0 writing the unique id to DIR/id.bin.

"group": every rank in one process through fisdf_group (FISDF_GROUP_COPY; RANK ignored).

usage: python capi_shard_worker.py CASE RANK SIZE DIR host|rccl|group [VARIANT]
  VARIANT: "" (defaults), "svd" (fit_mode FISDF_FIT_SVD: the minimum-norm operator on every q),
  "notr" (time_reversal 0: every q fitted, weights 1)
"""
import ctypes as C
import os
import sys
import time
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

from fisdf import _lib  # noqa: E402
from fisdf import cell as Cl  # noqa: E402

H2D, D2H = 1, 2


class FileComm:
    """The four collectives of struct fisdf_comm over host files (stream-ordered by waiting for
    the stream first: the callback returns with the result on the device)."""

    def __init__(self, hip, rank, size, d):
        self.hip, self.rank, self.size, self.dir = hip, rank, size, d
        self.seq = 0
        self.calls = {"all_to_all": 0, "reduce_scatter_f64": 0, "allreduce_f64": 0, "broadcast": 0}

    def barrier(self):
        self.seq += 1
        open(os.path.join(self.dir, f"bar_{self.seq}_{self.rank}"), "w").close()
        t0 = time.time()
        while not all(os.path.exists(os.path.join(self.dir, f"bar_{self.seq}_{r}"))
                      for r in range(self.size)):
            if time.time() - t0 > 120:
                raise TimeoutError(f"rank {self.rank}: barrier {self.seq}")
            time.sleep(0.001)

    def _path(self, tag, src, dst):
        return os.path.join(self.dir, f"{tag}_{src}_{dst}.bin")

    def _d2h(self, ptr, n):
        buf = np.empty(n, np.uint8)
        assert self.hip.hipMemcpy(buf.ctypes.data, ptr, n, D2H) == 0
        return buf

    def _h2d(self, ptr, buf):
        buf = np.ascontiguousarray(buf)
        assert self.hip.hipMemcpy(ptr, buf.ctypes.data, buf.nbytes, H2D) == 0

    def _sync(self, stream):
        assert self.hip.hipStreamSynchronize(stream) == 0

    def _guard(self, name, fn):
        def cb(*args):
            try:
                self.calls[name] += 1
                fn(*args[1:])              # args[0] is the user pointer
                return 0
            except Exception:
                traceback.print_exc()
                return -1
        return cb

    def all_to_all(self, send, sbytes, recv, rbytes, stream):
        self._sync(stream)
        tag = f"a2a{self.seq}"
        for r in range(self.size):
            if sbytes[r]:
                self._d2h(send[r], sbytes[r]).tofile(self._path(tag, self.rank, r))
        self.barrier()
        for r in range(self.size):
            if rbytes[r]:
                data = np.fromfile(self._path(tag, r, self.rank), np.uint8)
                assert data.nbytes == rbytes[r], (data.nbytes, rbytes[r])
                self._h2d(recv[r], data)
        self.barrier()

    def _reduce(self, send, count_all, stream, tag):
        self._sync(stream)
        self._d2h(send, 8 * count_all).tofile(self._path(tag, self.rank, 0))
        self.barrier()
        tot = np.zeros(count_all)
        for r in range(self.size):       # rank order on every rank: identical sums
            tot += np.fromfile(self._path(tag, r, 0), np.float64)
        self.barrier()
        return tot

    def reduce_scatter(self, send, recv, count, stream):
        tot = self._reduce(send, count * self.size, stream, f"rs{self.seq}")
        self._h2d(recv, tot[self.rank * count:(self.rank + 1) * count])

    def allreduce(self, buf, count, stream):
        self._h2d(buf, self._reduce(buf, count, stream, f"ar{self.seq}"))

    def broadcast(self, buf, nbytes, root, stream):
        self._sync(stream)
        tag = f"bc{self.seq}"
        if self.rank == root:
            self._d2h(buf, nbytes).tofile(self._path(tag, root, 0))
        self.barrier()
        if self.rank != root:
            self._h2d(buf, np.fromfile(self._path(tag, root, 0), np.uint8))
        self.barrier()

    def struct(self):
        c = _lib.Comm()
        c.rank, c.size, c.user = self.rank, self.size, None
        self._cbs = (_lib.ALL_TO_ALL_FN(self._guard("all_to_all", self.all_to_all)),
                     _lib.REDUCE_SCATTER_FN(self._guard("reduce_scatter_f64", self.reduce_scatter)),
                     _lib.ALLREDUCE_FN(self._guard("allreduce_f64", self.allreduce)),
                     _lib.BROADCAST_FN(self._guard("broadcast", self.broadcast)))
        c.all_to_all, c.reduce_scatter_f64, c.allreduce_f64, c.broadcast = self._cbs
        return c


def main(case, rank, size, d, mode, variant=""):
    from cases import inputs
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(case)
    nao = cell.nao_nr()
    dms = np.concatenate([dm, Cl.make_dm(nao, kmesh, cell, seed=99, scale=0.2)[None]])
    lib = _lib.load()
    hip = C.CDLL("libamdhip64.so")       # the runtime libfisdf.so already loaded
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipStreamSynchronize.argtypes = [C.c_void_p]

    def make_ctx():
        ctx = C.c_void_p()
        assert lib.fisdf_create(0, None, C.byref(ctx)) == 0, lib.fisdf_last_error(None)
        return ctx

    def call(ctx, name, *args):
        rc = getattr(lib, name)(ctx, *args)
        if rc != 0:
            raise RuntimeError(f"{name}: {lib.fisdf_last_error(ctx).decode()}")

    ctx = make_ctx()

    def upload(a):
        a = np.ascontiguousarray(a)
        p = C.c_void_p()
        call(ctx, "fisdf_malloc", C.c_size_t(a.nbytes), C.byref(p))
        call(ctx, "fisdf_memcpy_htod", p, a.ctypes.data_as(C.c_void_p), C.c_size_t(a.nbytes))
        return p

    def download(c, ptr, shape, dtype=complex):
        h = np.empty(shape, dtype)
        call(c, "fisdf_memcpy_dtoh", h.ctypes.data_as(C.c_void_p), C.c_void_p(ptr),
             C.c_size_t(h.nbytes))
        return h

    d_x0, d_f, d_dms = upload(x0), upload(chi), upload(dms.astype(np.complex128))
    km, kp = _lib.iarr(kmesh)
    me, mp = _lib.iarr(cell.mesh)
    aa, ap = _lib.darr(cell.a.ravel())
    opts = _lib.BuildOpts()
    lib.fisdf_build_opts_default(C.byref(opts))
    opts.nip_max = int(nao * c0)                                           # fftisdf.py:383
    if variant == "svd":
        opts.fit_mode = 1
    elif variant == "notr":
        opts.time_reversal = 0
    elif variant:
        raise ValueError(variant)

    if mode == "rccl":
        idf = os.path.join(d, "id.bin")
        if rank == 0:
            uid = (C.c_ubyte * _lib.COMM_ID_BYTES)()
            assert lib.fisdf_comm_rccl_unique_id(uid) == 0, lib.fisdf_last_error(None)
            open(idf + ".tmp", "wb").write(bytes(uid))
            os.replace(idf + ".tmp", idf)
        t0 = time.time()
        while not os.path.exists(idf):
            assert time.time() - t0 < 60
            time.sleep(0.01)
        uid = (C.c_ubyte * _lib.COMM_ID_BYTES).from_buffer_copy(open(idf, "rb").read())
        comm = _lib.Comm()
        assert lib.fisdf_comm_rccl_init(uid, rank, size, 0, C.byref(comm)) == 0, \
            lib.fisdf_last_error(None)
        fc = None
    else:
        fc = FileComm(hip, rank, size, d)
        comm = fc.struct()

    nip = C.c_int()
    call(ctx, "fisdf_build_sharded", C.byref(comm), d_x0, x0.shape[1], d_f, nao, kp, mp, ap,
         C.byref(opts), C.byref(nip))
    r = _lib.BuildResult()
    call(ctx, "fisdf_build_get", C.byref(r))
    nip = nip.value
    assert (r.shard_rank, r.shard_size) == (rank, size)
    nfit = r.nfit
    out = dict(fit_qs=np.ctypeslib.as_array(r.fit_qs, (nfit,)).copy() if nfit else
               np.zeros(0, np.int32),
               perm=np.ctypeslib.as_array(r.perm, (nip,)).copy(), rows=np.array([r.row0, r.row1]),
               w0=download(ctx, r.d_W0, (nip, nip)))
    out["wq"] = download(ctx, r.d_Wq, (nfit, nip, nip)) if nfit else np.zeros((0, nip, nip), complex)
    out["ws_rows"] = download(ctx, r.d_Ws, (r.nk, r.row1 - r.row0, nip), np.float64)
    nbytes = dms.size * 16
    d_vj, d_vk = C.c_void_p(), C.c_void_p()
    call(ctx, "fisdf_malloc", C.c_size_t(nbytes), C.byref(d_vj))
    call(ctx, "fisdf_malloc", C.c_size_t(nbytes), C.byref(d_vk))
    call(ctx, "fisdf_get_jk", d_dms, 2, 1, 1, d_vj, d_vk)
    out["vj"] = download(ctx, d_vj.value, dms.shape)
    out["vk"] = download(ctx, d_vk.value, dms.shape)
    # the W_q of a sharded build are distributed: fisdf_get_wq refuses (size > 1)
    if size > 1:
        assert lib.fisdf_get_wq(ctx, out["wq"].ctypes.data_as(C.c_void_p)) != 0
        assert b"distributed" in lib.fisdf_last_error(ctx)
    if fc is not None:
        out["calls"] = np.array([fc.calls[k] for k in sorted(fc.calls)])
    if rank == 0:
        # the 1-GPU composite build on a context of its own, same inputs
        ref = make_ctx()
        nip1 = C.c_int()
        call(ref, "fisdf_build", d_x0, x0.shape[1], d_f, nao, kp, mp, ap, C.byref(opts),
             C.byref(nip1))
        r1 = _lib.BuildResult()
        call(ref, "fisdf_build_get", C.byref(r1))
        assert r1.shard_size == 1 and (r1.row0, r1.row1) == (0, nip1.value)
        out["ref_fit_qs"] = np.ctypeslib.as_array(r1.fit_qs, (r1.nfit,)).copy()
        out["ref_wq"] = download(ref, r1.d_Wq, (r1.nfit, nip, nip))
        out["ref_ws"] = download(ref, r1.d_Ws, (r1.nk, nip, nip), np.float64)
        call(ref, "fisdf_get_jk", d_dms, 2, 1, 1, d_vj, d_vk)
        out["ref_vj"] = download(ref, d_vj.value, dms.shape)
        out["ref_vk"] = download(ref, d_vk.value, dms.shape)
        assert lib.fisdf_destroy(ref) == 0
    for p in (d_x0, d_f, d_dms, d_vj, d_vk):
        call(ctx, "fisdf_free", p)
    assert lib.fisdf_destroy(ctx) == 0
    if mode == "rccl":
        assert lib.fisdf_comm_rccl_destroy(C.byref(comm)) == 0
    assert "torch" not in sys.modules, "the C-ABI path must not need torch"
    np.savez(os.path.join(d, f"rank{rank}.npz"), **out)


def main_group(case, size, d, variant=""):
    """All SIZE ranks in this one process through fisdf_group (FISDF_GROUP_COPY unless the
    variant says rccl; one host thread per rank inside the library): writes the same rank{r}.npz
    files.  Every rank on GPU 0, or — variants multidev / multidev_rccl — rank r on GPU r, its
    inputs and outputs uploaded to and read from its own device."""
    from cases import inputs
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(case)
    nao = cell.nao_nr()
    dms = np.concatenate([dm, Cl.make_dm(nao, kmesh, cell, seed=99, scale=0.2)[None]])
    lib = _lib.load()

    def call(ctx, name, *args):
        rc = getattr(lib, name)(ctx, *args)
        if rc != 0:
            raise RuntimeError(f"{name}: {lib.fisdf_last_error(ctx).decode()}")

    multidev = variant.startswith("multidev")
    devices = list(range(size)) if multidev else [0] * size
    ctxs = {}
    for dev in sorted(set(devices)):          # one plain context per device: memory + copies
        c_ = C.c_void_p()
        assert lib.fisdf_create(dev, None, C.byref(c_)) == 0, lib.fisdf_last_error(None)
        ctxs[dev] = c_
    ctx = ctxs[0]

    def upload(a, dev=0):
        a = np.ascontiguousarray(a)
        p = C.c_void_p()
        call(ctxs[dev], "fisdf_malloc", C.c_size_t(a.nbytes), C.byref(p))
        call(ctxs[dev], "fisdf_memcpy_htod", p, a.ctypes.data_as(C.c_void_p), C.c_size_t(a.nbytes))
        return p

    def download(c, ptr, shape, dtype=complex):
        h = np.empty(shape, dtype)
        call(c, "fisdf_memcpy_dtoh", h.ctypes.data_as(C.c_void_p), C.c_void_p(ptr),
             C.c_size_t(h.nbytes))
        return h

    def alloc(nbytes, dev=0):
        p = C.c_void_p()
        call(ctxs[dev], "fisdf_malloc", C.c_size_t(nbytes), C.byref(p))
        return p

    up = {dev: (upload(x0, dev), upload(chi, dev), upload(dms.astype(np.complex128), dev))
          for dev in ctxs}
    d_x0, d_f, d_dms = up[0]
    km, kp = _lib.iarr(kmesh)
    me, mp = _lib.iarr(cell.mesh)
    aa, ap = _lib.darr(cell.a.ravel())
    opts = _lib.BuildOpts()
    lib.fisdf_build_opts_default(C.byref(opts))
    opts.nip_max = int(nao * c0)                                           # fftisdf.py:383
    kind = _lib.GROUP_COPY
    if variant == "notr":
        opts.time_reversal = 0
    elif variant in ("rccl", "multidev_rccl"):   # RCCL: distinct devices (one rank on one GPU)
        kind = _lib.GROUP_RCCL
    elif variant not in ("", "multidev"):
        raise ValueError(variant)
    trace = os.environ.get("FISDF_WORKER_TRACE") is not None
    say = (lambda m: print(m, file=sys.stderr, flush=True)) if trace else (lambda m: None)  # noqa: E731
    devs, devp = _lib.iarr(devices)
    g = C.c_void_p()
    say("group_create")
    assert lib.fisdf_group_create(size, devp, kind, C.byref(g)) == 0, \
        lib.fisdf_last_error(None)
    ptrs = lambda i: (C.c_void_p * size)(*[up[dev][i].value for dev in devices])  # noqa: E731
    nip = C.c_int()
    say("group_build")
    rc = lib.fisdf_group_build(g, ptrs(0), x0.shape[1], ptrs(1), nao, kp, mp, ap,
                               C.byref(opts), C.byref(nip))
    assert rc == 0, lib.fisdf_group_last_error(g)
    nip = nip.value
    nbytes = dms.size * 16
    say("group_get_jk")
    vjs = [alloc(nbytes, dev) for dev in devices]
    vks = [alloc(nbytes, dev) for dev in devices]
    rc = lib.fisdf_group_get_jk(g, ptrs(2), 2, 1, 1, (C.c_void_p * size)(*[v.value for v in vjs]),
                                (C.c_void_p * size)(*[v.value for v in vks]))
    assert rc == 0, lib.fisdf_group_last_error(g)
    say("results")
    outs = []
    for rank in range(size):
        rc_ = lib.fisdf_group_ctx(g, rank)
        say(f"rank {rank} ctx {rc_}")
        rctx = C.c_void_p(rc_)
        r = _lib.BuildResult()
        call(rctx, "fisdf_build_get", C.byref(r))
        assert (r.shard_rank, r.shard_size) == (rank, size)
        nfit = r.nfit
        out = dict(fit_qs=np.ctypeslib.as_array(r.fit_qs, (nfit,)).copy() if nfit else
                   np.zeros(0, np.int32),
                   perm=np.ctypeslib.as_array(r.perm, (nip,)).copy(),
                   rows=np.array([r.row0, r.row1]), w0=download(rctx, r.d_W0, (nip, nip)))
        out["wq"] = (download(rctx, r.d_Wq, (nfit, nip, nip)) if nfit
                     else np.zeros((0, nip, nip), complex))
        out["ws_rows"] = download(rctx, r.d_Ws, (r.nk, r.row1 - r.row0, nip), np.float64)
        out["vj"] = download(ctxs[devices[rank]], vjs[rank].value, dms.shape)
        out["vk"] = download(ctxs[devices[rank]], vks[rank].value, dms.shape)
        outs.append(out)
    say("group_destroy")
    assert lib.fisdf_group_destroy(g) == 0
    say("reference")
    # the 1-GPU composite build, same inputs
    nip1 = C.c_int()
    call(ctx, "fisdf_build", d_x0, x0.shape[1], d_f, nao, kp, mp, ap, C.byref(opts),
         C.byref(nip1))
    say("reference built")
    r1 = _lib.BuildResult()
    call(ctx, "fisdf_build_get", C.byref(r1))
    outs[0]["ref_fit_qs"] = np.ctypeslib.as_array(r1.fit_qs, (r1.nfit,)).copy()
    outs[0]["ref_wq"] = download(ctx, r1.d_Wq, (r1.nfit, nip, nip))
    outs[0]["ref_ws"] = download(ctx, r1.d_Ws, (r1.nk, nip, nip), np.float64)
    call(ctx, "fisdf_get_jk", d_dms, 2, 1, 1, vjs[0], vks[0])
    outs[0]["ref_vj"] = download(ctx, vjs[0].value, dms.shape)
    outs[0]["ref_vk"] = download(ctx, vks[0].value, dms.shape)
    say("reference done")
    for rank, dev in enumerate(devices):
        for p in (vjs[rank], vks[rank]):
            call(ctxs[dev], "fisdf_free", p)
    for dev, bufs in up.items():
        for p in bufs:
            call(ctxs[dev], "fisdf_free", p)
    for c_ in ctxs.values():
        assert lib.fisdf_destroy(c_) == 0
    say("freed")
    assert "torch" not in sys.modules, "the C-ABI path must not need torch"
    for rank, out in enumerate(outs):
        np.savez(os.path.join(d, f"rank{rank}.npz"), **out)


if __name__ == "__main__":
    if sys.argv[5] == "group":
        main_group(sys.argv[1], int(sys.argv[3]), sys.argv[4],
                   sys.argv[6] if len(sys.argv) > 6 else "")
    else:
        main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5],
             sys.argv[6] if len(sys.argv) > 6 else "")
