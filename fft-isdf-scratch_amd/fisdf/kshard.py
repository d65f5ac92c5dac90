"""k-point (q) sharding over the GPUs of a node.

One process per GPU.  Each rank owns a contiguous q-range: it builds y_q, fits and
Coulomb-transforms only its own q (fftisdf.py:97-122 are independent per q).  The only
exchange steps are the ones the algorithm has:

* W_s = sqrt(nk) Re(sum_q Phi[R,q] W_q) (fftisdf.py:204-207) mixes all q: each rank
  forms its partial sum and the partials are summed with one all-reduce (RCCL over
  xGMI on the GPUs; gloo in the CPU tests);
* get_j uses W_0 (fftisdf.py:159), owned by the rank holding q = 0: one broadcast.

These helpers take torch tensors on any device, so the same code runs the CPU gloo
tests and the RCCL path.
"""
from __future__ import annotations


def shard_range(nk: int, rank: int, size: int):
    """Contiguous, balanced q-range [q0, q1) of `rank` among `size` ranks."""
    base, rem = divmod(nk, size)
    q0 = rank * base + min(rank, rem)
    return q0, q0 + base + (1 if rank < rem else 0)


def owner_of(q: int, nk: int, size: int) -> int:
    for r in range(size):
        q0, q1 = shard_range(nk, r, size)
        if q0 <= q < q1:
            return r
    raise ValueError(q)


def allreduce_ws(ws, group=None):
    """Sum the per-rank partial W_s (complex tensor, imaginary part zero) in place."""
    import torch.distributed as dist
    if ws.is_complex() and not ws.is_cuda:
        # gloo reduces real tensors; the complex view is summed component-wise
        import torch
        dist.all_reduce(torch.view_as_real(ws), group=group)
    else:
        dist.all_reduce(ws, group=group)
    return ws


def broadcast_w0(w0, nk: int, group=None):
    """Broadcast W_0 from the rank that owns q = 0."""
    import torch
    import torch.distributed as dist
    size = dist.get_world_size(group)
    src_local = owner_of(0, nk, size)
    src = dist.get_global_rank(group, src_local) if group is not None else src_local
    if w0.is_complex() and not w0.is_cuda:
        dist.broadcast(torch.view_as_real(w0), src=src, group=group)
    else:
        dist.broadcast(w0, src=src, group=group)
    return w0
