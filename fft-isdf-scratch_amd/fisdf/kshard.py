"""q sharding of the k-point ISDF build over the GPUs of a node.

One process per GPU.  The fitted q (time-reversal representatives) are shared among the ranks
by cost, longest first (``assign_q``: a self-conjugate q fitted on its half grid costs about 0.6
of a complex one); a rank's q need not be contiguous.  Each rank factorises, fits and
Coulomb-transforms only its own q (fftisdf.py:97-122 are independent per q).  The exchange
steps are the ones the algorithm has:

* the selection (fftisdf.py:357-388) is REPLICATED: every rank forms the whole Gram in the
  1-GPU order and runs the same pivoted Cholesky, so the pivots are the 1-GPU build's on every
  rank with no collective (``ISDF.sharded_gram`` keeps the k-sharded Gram + ``allreduce_real_part``,
  whose summation order can flip tied pivots);
* the y build is sharded over plane-aligned grid slices (``grid_slices``; y_k = Phi^T (Phi fx_k)^2
  mixes all k at each grid point, fftisdf.py:79-84): ``exchange_y_chunked`` runs one async
  all-to-all per local q index, each piece sent from its place in the send buffer and read in
  place by the fit (fisdf_set_y_slices);
* W_s = sqrt(nk) Re(sum_q Phi[R,q] W_q) (fftisdf.py:204-207) mixes all q: each rank forms every
  rank's interpolation-point row block of its partial sum and ``reduce_scatter_rows`` leaves each
  rank its own rows (get_k contracts only those);
* get_j uses W_0 (fftisdf.py:159), owned by the rank holding q = 0: ``broadcast_w0``; get_j / get_k
  end with ``allreduce_sum`` of nset * nk * nao^2 values.

These helpers take torch tensors on any device, so the same code runs the CPU gloo tests and the
RCCL path; ``EmulatedGroup`` runs one rank's share alone on one GPU (bench.py --emulate-ranks).
"""
from __future__ import annotations


class EmulatedGroup:
    """Rank `rank` of a `size`-rank k-shard, run ALONE on one GPU (bench.py --emulate-ranks):
    every compute step of that rank's share of the sharded build runs for real — the replicated
    selection and x4, the y build on its grid slice for all fitted q, the unpack of its
    all-to-all pieces, the fit of its q-chunk, its W_s partial and its get_jk rows — while the
    collectives are replaced by what they leave in this rank's memory: the all-to-all pieces are
    handed over pre-filled (`pieces[j]`, the rank's j-th q on the whole grid in the concat-of-
    slices layout; taken from a full 1-GPU y so the fit sees real data), the all-reduces keep
    their local copies but add nothing, the broadcast is skipped.  Timing only: the results of
    an emulated rank are its partial sums.

    For parity tests the other collectives can be handed over too: `w0` (the W_0 the broadcast
    delivers), `ws_src` ((nk, nip, nip) float64, the reduced W_s whose row block the reduce-
    scatter delivers) — then the rank's get_jk rows are exact and sum over the ranks to the full
    J/K — and `keep_ws` records the rank's reduce-scatter input (its partial W_s row blocks of
    every rank) in `ws_blocks`."""

    def __init__(self, rank: int, size: int, pieces=None, w0=None, ws_src=None,
                 keep_ws: bool = False):
        self.rank, self.size = int(rank), int(size)
        self.pieces = pieces
        self.w0 = w0
        self.ws_src = ws_src
        self.keep_ws = keep_ws
        self.ws_blocks = None


def positions(part):
    """A rank's share of the fitted q as ascending positions in the fit order: an index list
    (assign_q) or a contiguous (a, b) chunk."""
    if isinstance(part, tuple) and len(part) == 2:
        return list(range(int(part[0]), int(part[1])))
    return [int(i) for i in part]


def emulated_pieces(yall, parts, slices, rank: int):
    """The all-to-all pieces rank `rank` receives, built from the full y of every fitted q
    (yall: (nq_all, nip, ngrid) in fit order): its j-th q on each slice p, concatenated in rank
    order p — exactly the layout exchange_y_chunked hands to the fit."""
    import torch
    return [torch.cat([yall[i, :, g0:g0 + ng].reshape(-1) for g0, ng in slices])
            for i in positions(parts[rank])]


def assign_q(costs, size: int):
    """Share the fitted q (in fit order, with their relative fit costs) among `size` ranks:
    longest-processing-time greedy (most expensive q first, each to the least loaded rank; ties to
    the lower rank), each rank's positions ascending.  Unlike contiguous chunks a rank may own
    q from anywhere in the list: at C3 x8 (28 complex q of cost 1, 8 self-conjugate of 0.6) the
    largest share is 4.2 instead of the 5.0 of the best contiguous split.  The 1-GPU and N-rank
    builds give the same W_q bit for bit whatever the assignment (a q's arithmetic never depends
    on its companions)."""
    import numpy as np
    c = np.asarray(costs, dtype=float)
    load = [0.0] * size
    parts = [[] for _ in range(size)]
    for i in sorted(range(len(c)), key=lambda i: (-c[i], i)):
        r = min(range(size), key=lambda r: (load[r], r))
        parts[r].append(i)
        load[r] += c[i]
    return [sorted(p) for p in parts]


def _emulated(group):
    return isinstance(group, EmulatedGroup)


def shard_range(nk: int, rank: int, size: int):
    """Contiguous, balanced q-range [q0, q1) of `rank` among `size` ranks."""
    base, rem = divmod(nk, size)
    q0 = rank * base + min(rank, rem)
    return q0, q0 + base + (1 if rank < rem else 0)


def time_reversal_reps(kmesh):
    """Time-reversal classes of the q-mesh (get_kpts order, wrap_around=False).

    y_s and x4_s are real (fftisdf.py:43,81), so y_{-q} = conj(y_q) and x4_{-q} = conj(x4_q)
    and hence W_{-q} = conj(W_q): only one q of each (q, -q) pair needs a fit.  Returns
    (reps, partner, weight): ascending representatives (the smaller index of each pair),
    partner[q] = index of -q mod kmesh, weight[i] = 1 if reps[i] is its own partner else 2."""
    import numpy as np
    kmesh = np.asarray(kmesh, dtype=int)
    nk = int(np.prod(kmesh))
    v = np.stack(np.unravel_index(np.arange(nk), tuple(kmesh)), axis=1)
    mv = (-v) % kmesh
    partner = (mv[:, 0] * kmesh[1] + mv[:, 1]) * kmesh[2] + mv[:, 2]
    reps = np.array([q for q in range(nk) if partner[q] >= q], dtype=np.int32)
    weight = np.where(partner[reps] == reps, 1.0, 2.0)
    return reps, partner.astype(np.int32), weight


def shard_list(items, rank: int, size: int):
    """Contiguous, balanced chunk of `items` owned by `rank`."""
    a, b = shard_range(len(items), rank, size)
    return items[a:b]


def owner_of(q: int, nk: int, size: int) -> int:
    for r in range(size):
        q0, q1 = shard_range(nk, r, size)
        if q0 <= q < q1:
            return r
    raise ValueError(q)


def grid_slices(mesh, size: int):
    """Plane-aligned contiguous grid slices [(g0, ng)] of the FFT mesh, one per rank: the
    y build is sharded over grid points (every rank computes y_q for ALL q on its slice)."""
    n0 = int(mesh[0])
    plane = int(mesh[1]) * int(mesh[2])
    out = []
    for r in range(size):
        p0, p1 = shard_range(n0, r, size)
        out.append((p0 * plane, (p1 - p0) * plane))
    return out


def exchange_y(send, nk: int, nip: int, slices, rank: int, size: int, group=None,
               async_op: bool = False, counts=None):
    """All-to-all of the grid-sliced y: `send` is (nq_all, nip, ng_rank) = y_q on this rank's
    slice for every fitted q; the q-blocks are contiguous, so block r of the send buffer is
    rank r's q-shard (`counts[r]` q each; default: shard_range over nk).  Returns
    recv = concat_p (nq_self, nip, ng_p) in rank order p (with async_op: (recv, work) — call
    work.wait() before reading recv; work may be None)."""
    import torch
    import torch.distributed as dist
    ng_self = slices[rank][1]
    if counts is None:
        counts = [b - a for a, b in (shard_range(nk, r, size) for r in range(size))]
    nq = counts[rank]
    in_splits = [c * nip * ng_self for c in counts]
    out_splits = [nq * nip * slices[p][1] for p in range(size)]
    if _host_staged(group, send):
        recv = exchange_y(send.cpu(), nk, nip, slices, rank, size, group,
                          counts=counts).to(send.device)
        return (recv, None) if async_op else recv
    recv = torch.empty(sum(out_splits), dtype=send.dtype, device=send.device)
    flat = send.reshape(-1)
    if send.is_complex():
        work = dist.all_to_all_single(torch.view_as_real(recv), torch.view_as_real(flat),
                                      out_splits, in_splits, group=group, async_op=async_op)
    else:
        work = dist.all_to_all_single(recv, flat, out_splits, in_splits, group=group,
                                      async_op=async_op)
    return (recv, work) if async_op else recv


def exchange_y_chunked(send, nip: int, slices, rank: int, size: int, group, parts):
    """The all-to-all of exchange_y split per local q index j, so the fit of a rank's j-th q
    can start as soon as its own piece has arrived (the later pieces move over xGMI while
    the earlier q are fitted).  `send` is (nq_all, nip, ng_rank) in fit order; parts[r] are
    rank r's positions in it (assign_q, or contiguous (a, b) chunks).  Returns [(recv_j, work_j)]
    for the rank's j-th q; recv_j is concat_p (nip, ng_p); call work_j.wait() (may be None)
    before reading recv_j."""
    import torch
    import torch.distributed as dist
    pos = [positions(p) for p in parts]
    counts = [len(p) for p in pos]
    if _emulated(group):
        ngrid = sum(ng for _, ng in slices)
        return [(group.pieces[j] if group.pieces is not None else
                 send.new_empty(nip * ngrid), None) for j in range(counts[rank])]
    ng_self = slices[rank][1]
    nmax = max(counts) if counts else 0
    out = []
    # gloo has no list all-to-all: gather the pieces on the host (CPU tests, ranks sharing a GPU)
    host = dist.get_backend(group) == "gloo"
    hs = send.cpu() if host else None
    for j in range(nmax):
        in_splits = [nip * ng_self if j < counts[r] else 0 for r in range(size)]
        mine = j < counts[rank]
        out_splits = [nip * slices[p][1] if mine else 0 for p in range(size)]
        rj = torch.empty(sum(out_splits), dtype=send.dtype, device=send.device)
        if host:
            dst = [r for r in range(size) if j < counts[r]]
            idx = torch.tensor([pos[r][j] for r in dst], dtype=torch.long)
            sj = hs.index_select(0, idx).reshape(-1) if len(dst) else hs.new_empty(0)
            hr = rj.cpu()
            dist.all_to_all_single(torch.view_as_real(hr), torch.view_as_real(sj),
                                   out_splits, in_splits, group=group)
            if rj.data_ptr() != hr.data_ptr():
                rj.copy_(hr)
            work = None
        else:
            # the piece for rank r is send[pos[r][j]], a contiguous (nip, ng_self) block: the
            # list form sends every piece from its place (no gather copy of the send buffer)
            empty = torch.view_as_real(send.new_empty(0))
            ins = [torch.view_as_real(send[pos[r][j]].reshape(-1)) if j < counts[r] else empty
                   for r in range(size)]
            outs, off = [], 0
            for n in out_splits:
                outs.append(torch.view_as_real(rj[off:off + n]))
                off += n
            work = dist.all_to_all(outs, ins, group=group, async_op=True)
        if mine:
            out.append((rj, work))
        elif work is not None:
            work.wait()
    return out


def allreduce_real_part(t, group=None):
    """In-place sum over ranks of a complex tensor whose imaginary part is zero (W_s,
    fftisdf.py:207 keeps only Re): only the real parts travel (half the bytes)."""
    import torch
    re = torch.view_as_real(t)[..., 0]
    buf = re.contiguous()
    allreduce_sum(buf, group)
    re.copy_(buf)
    return t


def reduce_scatter_rows(blocks, chunk: int, nloc: int, rank: int, size: int, group=None,
                        rows=None):
    """Sum over ranks of the real `blocks` (rank c's block of the sum at [c*chunk, c*chunk + n_c),
    chunks padded to one size) and return THIS rank's block, the first `nloc` elements of its
    chunk: W_s reduced and scattered by interpolation-point rows (fftisdf.py:204-207; W_s is
    real, and each rank's get_k needs only its rows).  (size-1)/size of one W_s per rank travels,
    half the bytes of an all-reduce of the same array.  rows = (i0, i1): this rank's
    interpolation-point rows (used by an EmulatedGroup that hands the reduced W_s over)."""
    import torch
    import torch.distributed as dist
    if _emulated(group):
        if group.keep_ws:
            group.ws_blocks = blocks.clone()
        if group.ws_src is not None:
            i0, i1 = rows
            return group.ws_src[:, i0:i1].contiguous().reshape(-1)
        return blocks[rank * chunk:rank * chunk + nloc]
    if _host_staged(group, blocks):
        h = blocks.cpu()
        dist.all_reduce(h, group=group)
        return h[rank * chunk:rank * chunk + nloc].to(blocks.device)
    out = torch.empty(chunk, dtype=blocks.dtype, device=blocks.device)
    dist.reduce_scatter_tensor(out, blocks[:chunk * size], group=group)
    return out[:nloc]


def _host_staged(group, *tensors):
    """gloo moves host tensors only: device tensors are staged through host copies (used
    when several ranks share one GPU in tests; the multi-GPU path uses RCCL directly)."""
    import torch.distributed as dist
    return dist.get_backend(group) == "gloo" and any(t.is_cuda for t in tensors)


def allreduce_sum(t, group=None):
    """In-place sum over ranks (complex tensors are reduced through their real view)."""
    import torch
    import torch.distributed as dist
    if _emulated(group):
        return t
    if _host_staged(group, t):
        h = t.cpu()
        allreduce_sum(h, group)
        t.copy_(h)
        return t
    dist.all_reduce(torch.view_as_real(t) if t.is_complex() else t, group=group)
    return t


def broadcast_w0(w0, nk: int, group=None, src_local=None):
    """Broadcast W_0 from the rank that owns q = 0 (default: contiguous q-ranges over nk)."""
    import torch
    import torch.distributed as dist
    if _emulated(group):
        if group.w0 is not None and group.rank != src_local:   # the owner keeps its own W_0
            w0.copy_(group.w0)
        return w0
    size = dist.get_world_size(group)
    if src_local is None:
        src_local = owner_of(0, nk, size)
    src = dist.get_global_rank(group, src_local) if group is not None else src_local
    if _host_staged(group, w0):
        h = w0.cpu()
        dist.broadcast(torch.view_as_real(h) if h.is_complex() else h, src=src, group=group)
        w0.copy_(h)
        return w0
    dist.broadcast(torch.view_as_real(w0) if w0.is_complex() else w0, src=src, group=group)
    return w0
