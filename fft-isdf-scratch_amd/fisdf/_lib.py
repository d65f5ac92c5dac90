"""ctypes binding of libfisdf.so (the C-ABI of include/fisdf.h).

The product path has no CPU fallback: if the HIP library is missing or no GPU is
visible, ``load()`` / ``Context()`` raise.  Device memory is handed over as raw
pointers (``torch.Tensor.data_ptr()`` of CUDA/HIP tensors or ``fisdf_malloc``).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# FISDF_LIB_VARIANT=x loads libfisdf_x.so from the same directory (A/B of build variants)
LIB_PATH = os.path.join(_HERE, "libfisdf%s.so" % (
    "_" + os.environ["FISDF_LIB_VARIANT"] if os.environ.get("FISDF_LIB_VARIANT") else ""))

STAGES = ["select", "x4", "y", "factor", "fft", "trsm", "herk", "small", "get_j", "get_k", "ws",
          "ao"]

_lib = None

_vp = C.c_void_p
_i = C.c_int
_l = C.c_long
_d = C.c_double
_ip = C.POINTER(C.c_int)
_dp = C.POINTER(C.c_double)

_SIGS = {
    "fisdf_abi_version": ([], _i),
    "fisdf_create": ([_i, _vp, C.POINTER(_vp)], _i),
    "fisdf_destroy": ([_vp], _i),
    "fisdf_last_error": ([_vp], C.c_char_p),
    "fisdf_sync": ([_vp], _i),
    "fisdf_malloc": ([_vp, C.c_size_t, C.POINTER(_vp)], _i),
    "fisdf_free": ([_vp, _vp], _i),
    "fisdf_memcpy_htod": ([_vp, _vp, _vp, C.c_size_t], _i),
    "fisdf_memcpy_dtoh": ([_vp, _vp, _vp, C.c_size_t], _i),
    "fisdf_set_timing": ([_vp, _i], _i),
    "fisdf_timings": ([_vp, _dp, _ip], _i),
    "fisdf_max_imag": ([_vp, _dp], _i),
    "fisdf_select_points": ([_vp, _vp, _i, _i, _i, _i, _d, _ip, _ip, _ip], _i),
    "fisdf_select_points_km": ([_vp, _vp, _ip, _i, _i, _i, _d, _ip, _ip, _ip], _i),
    "fisdf_gather_points": ([_vp, _vp, _i, _i, _i, _ip, _i, _vp], _i),
    "fisdf_eval_ao": ([_vp, _vp, _i, _i, _dp, _i, _ip, _ip, _ip, _dp, _dp, _i, _ip, _ip, _dp, _d,
                       _i, _vp], _i),
    "fisdf_eval_ao_band": ([_vp, _vp, _i, _i, _dp, _i, _ip, _ip, _ip, _dp, _dp, _i, _ip, _i, _dp,
                            _dp, _d, _i, _vp], _i),
    "fisdf_get_j_band_rows": ([_vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _i, _i, _i, _vp], _i),
    "fisdf_select_gram": ([_vp, _vp, _i, _i, _i, _i, _i, _vp], _i),
    "fisdf_select_pivots": ([_vp, _vp, _i, _i, _i, _d, _ip, _ip, _ip], _i),
    "fisdf_unpack_slices": ([_vp, _vp, _i, _i, C.POINTER(_l), C.POINTER(_l), _l, _vp], _i),
    "fisdf_build_x4": ([_vp, _vp, _i, _i, _ip, _dp, _vp], _i),
    "fisdf_build_y": ([_vp, _vp, _l, _i, _i, _i, _vp, _i, _i, _ip, _dp, _i, _i, _vp], _i),
    "fisdf_factor_x4": ([_vp, _vp, _i, _i, _i, _d, _ip], _i),
    "fisdf_fit_coulomb": ([_vp, _i, _i, _vp, _i, _ip, _ip, _dp, _vp], _i),
    "fisdf_build_ws": ([_vp, _vp, _i, _i, _i, _ip, _dp, _vp], _i),
    "fisdf_build_y_qs": ([_vp, _vp, _l, _i, _i, _i, _vp, _i, _i, _ip, _dp, _ip, _i, _vp], _i),
    "fisdf_factor_x4_qs": ([_vp, _vp, _ip, _i, _i, _d, _ip, _ip], _i),
    "fisdf_factor_x4_async": ([_vp, _vp, _ip, _i, _i, _d, _ip], _i),
    "fisdf_factor_x4_wait": ([_vp, _ip], _i),
    "fisdf_factor_x4_mark": ([_vp], _i),
    "fisdf_set_omega": ([_vp, _d], _i),
    "fisdf_set_pivoted_fit": ([_vp, _i], _i),
    "fisdf_factor_info": ([_vp, _ip], _i),
    "fisdf_set_fit_mode": ([_vp, _i], _i),
    "fisdf_set_half_grid": ([_vp, _i], _i),
    "fisdf_min_norm_operator": ([_vp, _vp, _i, _d, _vp, _vp, _vp, _ip, _ip], _i),
    "fisdf_min_norm_info": ([_vp, _ip], _i),
    "fisdf_set_fit_lanes": ([_vp, _i], _i),
    "fisdf_set_factor_priority": ([_vp, _i], _i),
    "fisdf_set_time_reversal": ([_vp, _i], _i),
    "fisdf_set_fit_pipe": ([_vp, _i, _i], _i),
    "fisdf_fit_info": ([_vp, _ip, _ip], _i),
    "fisdf_mark_y_ready": ([_vp, _i], _i),
    "fisdf_set_y_slices": ([_vp, _i, _vp, _i, C.POINTER(_l), C.POINTER(_l)], _i),
    "fisdf_reserve_workspace": ([_vp, C.c_size_t], _i),
    "fisdf_fit_coulomb_qs": ([_vp, _ip, _i, _vp, _i, _ip, _ip, _dp, _vp], _i),
    "fisdf_build_ws_qs": ([_vp, _vp, _ip, _dp, _i, _i, _ip, _dp, _vp], _i),
    "fisdf_get_j": ([_vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp], _i),
    "fisdf_get_k": ([_vp, _vp, _vp, _vp, _i, _i, _i, _ip, _dp, _vp], _i),
    "fisdf_get_j_rows": ([_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp], _i),
    "fisdf_get_k_rows": ([_vp, _vp, _vp, _vp, _i, _i, _i, _ip, _dp, _i, _i, _vp], _i),
    "fisdf_get_k_rows_local": ([_vp, _vp, _vp, _vp, _i, _i, _i, _ip, _dp, _i, _i, _vp], _i),
    "fisdf_build_ws_rows": ([_vp, _vp, _ip, _dp, _i, _i, _ip, _dp, _i, _i, _vp], _i),
    "fisdf_build_ws_blocks": ([_vp, _vp, _ip, _dp, _i, _i, _ip, _dp, _i, _ip, _l, _vp], _i),
    "fisdf_get_eri": ([_vp, _vp, _i, _i, _ip, _vp, C.POINTER(_vp), _ip, _vp], _i),
    "fisdf_zgemm": ([_vp, _i, _i, _i, _i, _i, _dp, _vp, _l, _l, _vp, _l, _l, _dp, _vp, _l, _l,
                     _i, _i], _i),
    "fisdf_zgemm_mode": ([_vp, _i, _i, _i, _i, _i, _dp, _vp, _l, _l, _vp, _l, _l, _dp, _vp, _l,
                          _l, _i, _i], _i),
    "fisdf_herk": ([_vp, _i, _i, _d, _vp, _l, _vp, _l, _i], _i),
    "fisdf_fft3d": ([_vp, _vp, _vp, _i, _ip], _i),
    "fisdf_fft3d_paired": ([_vp, _vp, _vp, _i, _ip, _dp, _ip, _i], _i),
    "fisdf_coulg": ([_vp, _ip, _dp, _dp, _d, _i, _vp], _i),
    "fisdf_pivoted_cholesky": ([_vp, _vp, _i, _i, _i, _d, _ip, _ip], _i),
    "fisdf_cholesky": ([_vp, _vp, _i, _i, _d, _ip], _i),
    "fisdf_tri_inverse": ([_vp, _vp, _i, _i, _vp], _i),
    # composite entries
    "fisdf_build_opts_default": ([_vp], None),
    "fisdf_build": ([_vp, _vp, _i, _vp, _i, _ip, _ip, _dp, _vp, _ip], _i),
    "fisdf_build_y_streamed": ([_vp, _ip], _i),
    "fisdf_y_stream_arm": ([_vp, _vp, _i, _vp, _l, _i, _i, _i, _ip, _ip, _i, _vp, _ip], _i),
    "fisdf_y_stream_finish": ([_vp, _i, _ip], _i),
    "fisdf_build_get": ([_vp, _vp], _i),
    "fisdf_build_release": ([_vp], _i),
    "fisdf_get_x": ([_vp, _vp], _i),
    "fisdf_get_w0": ([_vp, _vp], _i),
    "fisdf_get_wq": ([_vp, _vp], _i),
    "fisdf_get_jk": ([_vp, _vp, _i, _i, _i, _vp, _vp], _i),
    "fisdf_set_allocator": ([_vp, _vp, _vp, _vp], _i),
    "fisdf_check_time_reversal": ([_vp, _vp, _l, _l, _ip, _dp], _i),
    # k-sharded composite build with the caller's collectives
    "fisdf_build_sharded": ([_vp, _vp, _vp, _i, _vp, _i, _ip, _ip, _dp, _vp, _ip], _i),
    "fisdf_comm_rccl_unique_id": ([_vp], _i),
    "fisdf_comm_rccl_init": ([_vp, _i, _i, _i, _vp], _i),
    "fisdf_comm_rccl_destroy": ([_vp], _i),
    "fisdf_group_create": ([_i, _ip, _i, _vp], _i),
    "fisdf_group_destroy": ([_vp], _i),
    "fisdf_group_ctx": ([_vp, _i], _vp),
    "fisdf_group_last_error": ([_vp], C.c_char_p),
    "fisdf_group_build": ([_vp, _vp, _i, _vp, _i, _ip, _ip, _dp, _vp, _vp], _i),
    "fisdf_group_get_jk": ([_vp, _vp, _i, _i, _i, _vp, _vp], _i),
}

# FISDF_ABI_VERSION of include/fisdf.h this binding's structs follow
ABI_VERSION = 4


class BuildOpts(C.Structure):
    """struct fisdf_build_opts (include/fisdf.h)."""
    _fields_ = [("nip_max", _i), ("select_tol", _d), ("perm", _ip), ("n_perm", _i),
                ("fit_mode", _i), ("fit_tol", _d), ("pivoted_fit", _i), ("half_grid", _i),
                ("time_reversal", _i), ("real_self_conjugate", _i), ("omega", _d)]


class BuildResult(C.Structure):
    """struct fisdf_build_result (include/fisdf.h)."""
    _fields_ = [("nk", _i), ("nip", _i), ("nao", _i), ("nfit", _i), ("used_pivoted_fit", _i),
                ("min_norm_slots", _i), ("perm", _ip), ("fit_qs", _ip), ("ranks", _ip),
                ("partner", _ip), ("d_X", _vp), ("d_x4", _vp), ("d_Wq", _vp), ("d_Ws", _vp),
                ("time_reversal", _i), ("tr_deviation", _d), ("shard_rank", _i),
                ("shard_size", _i), ("row0", _i), ("row1", _i), ("d_W0", _vp)]


# struct fisdf_comm: the caller's collectives of fisdf_build_sharded (device pointers, enqueued
# stream-ordered on the hipStream_t they are given)
ALL_TO_ALL_FN = C.CFUNCTYPE(_i, _vp, C.POINTER(_vp), C.POINTER(C.c_size_t), C.POINTER(_vp),
                            C.POINTER(C.c_size_t), _vp)
REDUCE_SCATTER_FN = C.CFUNCTYPE(_i, _vp, _vp, _vp, C.c_size_t, _vp)
ALLREDUCE_FN = C.CFUNCTYPE(_i, _vp, _vp, C.c_size_t, _vp)
BROADCAST_FN = C.CFUNCTYPE(_i, _vp, _vp, C.c_size_t, _i, _vp)
COMM_ID_BYTES = 128
GROUP_COPY, GROUP_RCCL = 0, 1


class Comm(C.Structure):
    """struct fisdf_comm (include/fisdf.h)."""
    _fields_ = [("rank", _i), ("size", _i), ("user", _vp), ("all_to_all", ALL_TO_ALL_FN),
                ("reduce_scatter_f64", REDUCE_SCATTER_FN), ("allreduce_f64", ALLREDUCE_FN),
                ("broadcast", BROADCAST_FN)]


# fisdf_alloc_fn / fisdf_free_fn
ALLOC_FN = C.CFUNCTYPE(_vp, C.c_size_t, _vp)
FREE_FN = C.CFUNCTYPE(None, _vp, _vp)


class FisdfError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load libfisdf.so and declare every exported symbol (fails loudly if absent)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise FisdfError(
            f"{path} not found: build the HIP extension first (python -c "
            f"'import __graft_entry__ as g; g.build()')")
    lib = C.CDLL(path)
    for name, (args, res) in _SIGS.items():
        if os.environ.get("FISDF_LIB_VARIANT") and not hasattr(lib, name):
            continue  # an A/B build of an older tree may lack newer entry points
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    if not os.environ.get("FISDF_LIB_VARIANT") and lib.fisdf_abi_version() != ABI_VERSION:
        raise FisdfError(f"{path}: ABI version {lib.fisdf_abi_version()}, the binding expects "
                         f"{ABI_VERSION} (rebuild the library)")
    _lib = lib
    return lib


def check(rc, ctx=None):
    """Raise FisdfError with the failing context's message (fisdf_last_error(ctx))."""
    if rc != 0:
        raise FisdfError(load().fisdf_last_error(ctx).decode())


def iarr(x):
    a = np.ascontiguousarray(np.asarray(x, dtype=np.int32))
    return a, a.ctypes.data_as(_ip)


def darr(x):
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    return a, a.ctypes.data_as(_dp)


def ptr(t):
    """Device pointer of a torch tensor (must be contiguous and on the GPU)."""
    if not t.is_cuda:
        raise FisdfError("fisdf expects device tensors")
    if not t.is_contiguous():
        raise FisdfError("fisdf expects contiguous tensors")
    return _vp(t.data_ptr())


class Context:
    """One fisdf context per process/device, bound to torch's current HIP stream."""

    def __init__(self, device: int = 0, stream=None):
        lib = load()
        out = _vp()
        check(lib.fisdf_create(int(device), _vp(stream) if stream else None, C.byref(out)), None)
        self.lib = lib
        self.h = out
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            self.lib.fisdf_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def call(self, name, *args):
        check(getattr(self.lib, name)(self.h, *args), self.h)

    def build_result(self):
        """The last fisdf_build's resident result (struct fisdf_build_result)."""
        r = BuildResult()
        self.call("fisdf_build_get", C.byref(r))
        return r

    def timings(self):
        ms = (C.c_double * len(STAGES))()
        calls = (C.c_int * len(STAGES))()
        self.call("fisdf_timings", ms, calls)
        return {s: (ms[i], calls[i]) for i, s in enumerate(STAGES)}

    def max_imag(self):
        out = (C.c_double * 3)()
        self.call("fisdf_max_imag", out)
        return list(out)
