#!/usr/bin/env python
"""Benchmark: k-point FFT-ISDF build + get_jk (BASELINE.json metric) on MI355X.

A "step" is one full ISDF build (selection, x4, y, per-q fit + FFT Coulomb, W_s) plus
one get_jk on a synthetic diamond gth-dzvp-shaped cell, 4x4x4 k-mesh, nip = 600,
36^3 FFT mesh.  AO values (PySCF's job in the reference)
are evaluated once on the host and are resident in HBM before the timed region.

  python bench.py [--gpus N --steps K --warmup W] [--config c3|c2|c1] [--no-cpu-baseline]

For N > 1 the fitted q are sharded over N ranks, one process per GPU (RCCL all-to-all of y
pieces, reduce-scatter of W_s rows, broadcast of W_0), and rank 0 prints one JSON line.  Under
torch.distributed.run (WORLD_SIZE set) each process is one rank; `python bench.py --gpus N` on
its own starts torch.distributed.run --nproc-per-node N as a child (launch_ranks) and exits with
its status — non-zero, with a message, if fewer than N GPUs are visible.
FISDF_BENCH_BACKEND=gloo (rehearsal only: ranks may share one GPU, collectives staged through
the host) replaces RCCL.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

CONFIGS = {
    # name: (cell, basis, mesh, kmesh, m0, nip)   
    "c3": ("diamond", "gth-dzvp", (36, 36, 36), (4, 4, 4), (15, 15, 15), 600),
    "c2": ("diamond", "gth-dzvp", (36, 36, 36), (2, 2, 2), (15, 15, 15), 300),
    "c1": ("diamond", "gth-szv", (8, 8, 8), (1, 1, 1), (15, 15, 15), 160),
    "c4": ("nio", "gth-dzvp-molopt-sr", (32, 32, 32), (2, 2, 2), (15, 15, 15), 1000),
    "c5": ("si", "gth-szv", (30, 30, 30), (1, 1, 1), (15, 15, 15), 2000),
}
DESC = {
    "c3": "diamond gth-dzvp-shaped, 4x4x4 k-mesh, nip 600, mesh 36^3 (C3)",
    "c2": "diamond gth-dzvp-shaped, 2x2x2 k-mesh, nip 300, mesh 36^3 (C2)",
    "c1": "diamond gth-szv-shaped, Gamma, nip 160, mesh 8^3 (C1)",
    "c4": "NiO AFM (nio-afm.vasp) dzvp-molopt-sr-shaped, 2x2x2, nip 1000, mesh 32^3 (C4)",
    "c5": "Si 2x2x2 supercell (16 atoms) szv-shaped, Gamma, nip 2000, mesh 30^3 (C5)",
}
PEAK_FP64_TFLOPS = 78.6  # MI355X FP64 matrix (= vector) dense peak, MI355X_MICROARCH / BASELINE.md


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-isolated", action="store_true",
                   help="skip the untimed single-lane step (profiling runs: only warmup + timed "
                        "steps reach the profiler)")
    p.add_argument("--cpu-q", type=int, default=8, help="q-points fitted in the CPU sample")
    p.add_argument("--emulate-ranks", type=int, default=0, metavar="N",
                   help="time, on this one GPU, each rank's share of an N-rank k-sharded build "
                        "(its compute; collectives replaced by their local effect, kshard."
                        "EmulatedGroup) and print one JSON line with the per-rank step times")
    p.add_argument("--emulate-only", type=int, default=None, metavar="R",
                   help="with --emulate-ranks: time rank R only (profiling one rank's share)")
    return p.parse_args()


def setup(cfg):
    from fisdf import cell as C
    kind, basis, mesh, kmesh, m0, nip = CONFIGS[cfg]
    make = {"diamond": C.diamond_cell, "nio": C.nio_cell, "si": C.si_supercell}[kind]
    cell = make(basis=basis, mesh=mesh)
    nao = cell.nao_nr()
    c0 = (nip + 0.5) / nao                                    # int(nao*c0) == nip
    x0 = C.eval_ao_kpts(cell, cell.gen_uniform_grids(m0), kmesh)
    t = time.perf_counter()
    chi = C.eval_ao_kpts(cell, cell.gen_uniform_grids(mesh), kmesh)
    setup.ao_cpu_s = time.perf_counter() - t      # host restatement of pbc_eval_gto
    dm = C.make_dm(nao, kmesh, cell, seed=1234)
    return cell, kmesh, m0, c0, x0, chi, dm


def cpu_baseline(cell, kmesh, m0, c0, x0, chi, dm, nq):
    """Oracle (NumPy/SciPy restatement of fftisdf.py, the reference CPU path) on a bounded
    sample of the same job: selection, x4 and the y build over the WHOLE grid (y kept only for
    the sampled q), the gelsy fit + FFT Coulomb for nq q-points (Gamma and complex q, like the
    reference which fits every q), get_jk; the fit time is scaled by nk/nq."""
    from oracle import isdf_ref as R
    nk = chi.shape[0]
    ngrid = chi.shape[1]
    t = {}
    t0 = time.perf_counter()
    perm, rank, nip, _ = R.select_interpolation_points(x0, cell.nao_nr(), c0)
    t["select"] = time.perf_counter() - t0
    xip = x0[:, perm]
    kpts = R.get_kpts(cell.a, kmesh)
    phase = R.get_phase(cell.a, kpts, kmesh)
    t0 = time.perf_counter()
    x4 = R.build_x4(xip, phase)
    t["x4"] = time.perf_counter() - t0
    # sampled q: Gamma, self-conjugate q (2 k_q a reciprocal vector) and complex q spread over
    # the mesh, in the proportion the mesh has them (the reference treats every q alike)
    ks = np.stack(np.unravel_index(np.arange(nk), tuple(kmesh)), 1)
    selfc = [q for q in range(1, nk) if not ((2 * ks[q]) % np.asarray(kmesh)).any()]
    cplx = [q for q in range(nk) if ((2 * ks[q]) % np.asarray(kmesh)).any()]
    nq = min(nq, nk)
    n_self = min(len(selfc), max(1 if selfc else 0, round((nq - 1) * len(selfc) / max(nk - 1, 1))))
    n_cplx = min(len(cplx), nq - 1 - n_self)

    def spread(v, n):
        return [v[i] for i in np.linspace(0, len(v) - 1, n).astype(int)] if n > 0 else []
    qs = sorted(set([0] + spread(selfc, n_self) + spread(cplx, n_cplx)))
    # the y build of fftisdf.py:67-87 over the whole grid in its 8000-point blocks; the
    # 28.7 GB y (C3) is not kept, only the sampled q columns
    yq = np.empty((len(qs), ngrid, nip), complex)
    t0 = time.perf_counter()
    for g0 in range(0, ngrid, 8000):
        g1 = min(g0 + 8000, ngrid)
        yq[:, g0:g1] = R.build_y(chi[:, g0:g1], xip, phase)[qs]
    t["y"] = time.perf_counter() - t0
    coords = cell.gen_uniform_grids(cell.mesh)
    Gv = R.get_Gv(cell.a, cell.mesh)
    t0 = time.perf_counter()
    for i, q in enumerate(qs):
        R.fit_and_coulomb(x4[q], yq[i], kpts[q], coords, cell.a, cell.mesh, cell.vol, Gv)
    t["fit"] = (time.perf_counter() - t0) * nk / len(qs)
    del yq
    dms = dm[None]
    t0 = time.perf_counter()
    wq = np.zeros((nk, nip, nip), complex)  # timing only: get_jk cost is independent of values
    R.get_k_kpts(xip, wq, dms, phase)
    R.get_j_kpts(xip, wq[0], dms)
    t["get_jk"] = time.perf_counter() - t0
    total = sum(t.values())
    cores = os.cpu_count()
    try:
        from threadpoolctl import threadpool_info
        cores = max(i.get("num_threads", 1) for i in threadpool_info()) or cores
    except Exception:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except Exception:
        affinity = None
    share = os.environ.get("OMP_NUM_THREADS")
    return dict(value=nk / total, unit="k-points/s", cores=int(cores), kind="port",
                sample=(f"oracle (NumPy/SciPy gelsy restatement of fftisdf.py) timed on "
                        f"selection + x4 + the full-grid y build ({ngrid} points) + gelsy fit/"
                        f"FFT/W for q {qs} of {nk} (x{nk / len(qs):.0f}) + get_jk "
                        f"(est. {total:.1f} s/job); BLAS threads = FFT workers = the box's CPU "
                        f"share"),
                cpu_share=int(share) if share and share.isdigit() else None,
                fft_workers=R._fft_workers(), affinity_cpus=affinity, host_cpus=os.cpu_count(),
                stages_s={k: round(v, 3) for k, v in t.items()})


def emulate_ranks(args):
    """Per-rank compute of an N-way k-sharded C3 build, one rank at a time on this
    GPU: replicated selection + x4, the y build on the rank's grid slice for every fitted q, the
    unpack of its all-to-all pieces (handed over pre-filled from a full 1-GPU y, so the fit sees
    real data), its q-chunk's factor + fit, its W_s row-block partials + the local part of the
    reduce-scatter, its get_jk rows.  The max over ranks is the compute critical path of the
    N-GPU step; the collectives' transfer time is reported as a bytes budget beside it."""
    import torch
    from fisdf import ISDF, kshard
    torch.cuda.set_device(0)
    cell, kmesh, m0, c0, x0, chi, dm = setup(args.config)
    nk = int(np.prod(kmesh))
    N = args.emulate_ranks
    # the interpolation points and the full y of every fitted q (untimed, once)
    ref = ISDF(cell, cell.get_kpts(kmesh), m0=list(m0), c0=c0)
    d = ref.device
    ref._kmesh()
    ref._ao_parent = d.to_dev(x0)
    ref._ao_grid = d.to_dev(chi)
    ref._select()
    X = ref._dev_state["X"]
    nip, nao = X.shape[1], cell.nao_nr()
    from fisdf import _lib
    from fisdf.isdf import _fit_qset
    fit_qs, partner, weight = _fit_qset(ref, np.asarray(kmesh))
    ngrid = int(np.prod(cell.mesh))
    yall = d.empty((len(fit_qs), nip, ngrid))
    km_c, km_p = _lib.iarr(kmesh)
    a_c, a_p = _lib.darr(np.asarray(cell.lattice_vectors(), float).ravel())
    qs = np.ascontiguousarray(fit_qs, dtype=np.int32)
    d.ctx.call("fisdf_set_time_reversal", 1)
    d.ctx.call("fisdf_build_y_qs", _lib.ptr(ref._ao_grid), ngrid * nao, 0, ngrid, ngrid,
               _lib.ptr(X), nip, nao, km_p, a_p, qs.ctypes.data_as(_lib._ip), len(qs),
               _lib.ptr(yall))
    real_q = np.array([partner[q] == q for q in fit_qs])
    chunks = kshard.assign_q(np.where(real_q, 0.6, 1.0), N)
    slices = kshard.grid_slices(cell.mesh, N)
    per_rank = []
    for R in range(N) if args.emulate_only is None else [args.emulate_only]:
        pieces = kshard.emulated_pieces(yall, chunks, slices, R)
        df = ISDF(cell, cell.get_kpts(kmesh), m0=list(m0), c0=c0,
                  comm=kshard.EmulatedGroup(R, N, pieces))
        df._kmesh()
        df._ao_parent, df._ao_grid = ref._ao_parent, ref._ao_grid

        # FISDF_WHATIF_GIVEN_X=1 (a what-if, not the benchmark): the interpolation points handed
        # over, so the replicated selection is left out of every rank's step — how much of the
        # rank the selection front holds
        given_x = os.environ.get("FISDF_WHATIF_GIVEN_X") == "1"

        def step():
            if given_x:
                df._dev_state = {"X": X}
                df.perm = ref.perm
            else:
                df._dev_state = None
            df.build()
            df.get_jk(dm)
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        df.device.ctx.call("fisdf_set_timing", 1)
        df.device.ctx.timings()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        st = df.device.ctx.timings()
        df.device.ctx.call("fisdf_set_timing", 0)
        assert np.array_equal(df.perm, ref.perm)
        per_rank.append({"rank": R, "q": [int(q) for q in df.my_qs], "ms_per_step": round(dt * 1e3, 3),
                         "stages_ms": {k: round(v[0] / args.steps, 3) for k, v in st.items()
                                       if v[0] > 0}})
        del df, pieces
        torch.cuda.empty_cache()
    worst = max(per_rank, key=lambda r: r["ms_per_step"])
    # collective bytes of the worst rank (fp64): the chunked all-to-all of y (its q on the other
    # ranks' slices in, its slice of the others' q out) and the W_s reduce-scatter (real parts)
    R = worst["rank"]
    nmine = len(chunks[R])
    ng_self = slices[R][1]
    a2a_in = nmine * nip * (ngrid - ng_self) * 16
    a2a_out = (len(fit_qs) - nmine) * nip * ng_self * 16
    ws_rs = (N - 1) / N * nk * nip * nip * 8
    metric = "per-rank compute time of an emulated k-sharded step"
    if os.environ.get("FISDF_WHATIF_GIVEN_X") == "1":
        metric += " (WHAT-IF: interpolation points given, selection left out)"
    out = {"metric": metric, "config": args.config,
           "n_ranks": N, "steps": args.steps, "warmup": args.warmup,
           "one_gpu_reference": "bench.py default line (same config)",
           "max_rank_ms": worst["ms_per_step"], "worst_rank": R,
           "comm_bytes_worst_rank": {"all_to_all_in": a2a_in, "all_to_all_out": a2a_out,
                                     "ws_reduce_scatter": ws_rs},
           "ranks": per_rank}
    print(json.dumps(out))


def _backend():
    backend = os.environ.get("FISDF_BENCH_BACKEND", "nccl")
    if backend not in ("nccl", "gloo"):
        raise SystemExit(f"FISDF_BENCH_BACKEND must be nccl or gloo, not {backend!r}")
    return backend


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_launch_cmd(argv, n, port):
    """The child command that runs `n` ranks of this bench, one process per GPU
    (torch.distributed.run on 127.0.0.1), with the caller's own arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__)] + list(argv)


def launch_ranks(args, argv):
    """`bench.py --gpus N` started as ONE process (no WORLD_SIZE in the environment): start the
    N-rank job as a child process — torch.distributed.run, one rank per GPU over RCCL — and exit
    with its status.  Rank 0 of the child prints the JSON line (n_gpus = the communicator size).
    Nothing here touches the GPU (device_count does not initialise HIP on this image), so the
    parent never holds a device while its child runs; with fewer than N devices it stops with a
    message instead of running fewer ranks.  FISDF_BENCH_BACKEND=gloo (rehearsal: ranks share
    the visible GPUs, collectives staged through the host) skips the device-count check."""
    import subprocess
    backend = _backend()
    if backend == "nccl" and os.environ.get("FISDF_BENCH_PROBE") != "1":
        import torch
        have = torch.cuda.device_count()
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs (one rank per GPU "
                  f"over RCCL), this host has {have}", file=sys.stderr)
            return 2
    cmd = rank_launch_cmd(argv, args.gpus, _free_port())
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    return subprocess.call(cmd, env=env)


def probe_ranks(args):
    """FISDF_BENCH_PROBE=1 (tests, no GPU needed): join the process group the bench would use
    (gloo), all-reduce one value per rank and print the line rank 0 would head its result with —
    the launcher's N-rank path without the ISDF build."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dist.init_process_group("gloo")
    t = torch.ones(1)
    dist.all_reduce(t)
    if dist.get_rank() == 0:
        print(json.dumps({"probe": True, "n_gpus": dist.get_world_size(), "world_env": world,
                          "allreduce_sum": float(t.item()), "gpus_arg": args.gpus}))
    dist.destroy_process_group()
    return 0


def main():
    args = parse()
    if args.emulate_ranks > 0:
        return emulate_ranks(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args, sys.argv[1:])
    if os.environ.get("FISDF_BENCH_PROBE") == "1":
        return probe_ranks(args)
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = _backend()
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: running (and reporting) "
              f"{world} ranks", file=sys.stderr)
    if backend == "nccl" and torch.cuda.device_count() < world:
        print(f"bench.py: {world} ranks need {world} visible GPUs (one rank per GPU over RCCL), "
              f"this host has {torch.cuda.device_count()}", file=sys.stderr)
        return 2
    # one GPU per rank; a gloo rehearsal may place several ranks on one GPU
    dev = local if backend == "nccl" else local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev)
    comm = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
        comm = dist.group.WORLD
        world = dist.get_world_size(comm)          # the communicator's size is what is reported

    from fisdf import ISDF
    from fisdf import _lib
    cell, kmesh, m0, c0, x0, chi, dm = setup(args.config)
    nk = int(np.prod(kmesh))
    df = ISDF(cell, cell.get_kpts(kmesh), m0=list(m0), c0=c0, comm=comm)
    d = df.device
    df._kmesh()
    df._ao_parent = d.to_dev(x0)
    df._ao_grid = d.to_dev(chi)
    del chi

    def step():
        df._dev_state = None
        df.build()
        df.get_jk(dm)

    def barrier():
        torch.cuda.synchronize()
        if comm is not None:
            torch.distributed.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    d.ctx.call("fisdf_set_timing", 1)
    d.ctx.timings()  # reset
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    dt = time.perf_counter() - t0
    stages = d.ctx.timings()
    d.ctx.call("fisdf_set_timing", 0)
    if comm is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device=d.dev if backend == "nccl" else "cpu")
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        dt = float(tt.item())
    ms_per_step = dt / args.steps * 1e3
    value = nk / (dt / args.steps)

    # roofline of the dominant kernel.  The fit's two MFMA kernels per fitted q have the same
    # algorithmic work, 4 r^2 N flop (2 r^2 N for a self-conjugate q, real arithmetic):
    #   trsm: U = L^-1 Yhat, one lower-triangular GEMM (half of the 8 r^2 N of a full GEMM),
    #   herk: G = U U^H (Coulomb-weighted, Hermitian: lower tiles only).
    # Timed by the kernels' own execution span (first workgroup start to last wave end, summed
    # over the launches of the timed steps); the one with more time is `roofline`,
    # the other `roofline_secondary`.
    ngrid = int(np.prod(cell.mesh))
    ranks = np.asarray(df.ranks, dtype=np.float64)
    real = np.array([bool(df.real_self_conjugate and df.q_partner[q] == q) for q in df.my_qs])
    # a self-conjugate q is fitted over the prefix planes of its Hermitian G pairs (the
    # half-grid fit): its launches do 2 r^2 N_half, not 2 r^2 N
    n0, n1, n2 = (int(x) for x in cell.mesh)
    km = np.asarray(kmesh)
    ncols = []
    half = df.half_grid if df.half_grid is not None else os.environ.get("FISDF_HALF_G", "1") != "0"
    for q, re in zip(df.my_qs, real):
        if not re or not half:
            ncols.append(ngrid)
            continue
        mq = 2 * int(np.unravel_index(int(q), tuple(km))[0]) // int(km[0])
        nh = max(i0 + 1 for i0 in range(n0) if i0 <= (-i0 - mq) % n0)
        ncols.append(nh * n1 * n2)
    flop_step = float(np.sum(np.where(real, 2.0, 4.0) * ranks ** 2 * np.asarray(ncols, float)))
    KERNELS = {
        "trsm": ("zgemm_nn_wide_kernel<4|5,3> (lower-triangular GEMM U = L^-1 Yhat)", "trsm_gemm"),
        "herk": ("zgemm_glds_kernel<0,3,true,0|2,3> (HERK W_q, split-K) + herk_reduce_kernel", "herk"),
    }
    roofs = {}
    for name, (label, _) in KERNELS.items():
        ms, calls = stages[name]
        ach = flop_step * args.steps / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
        roofs[name] = {"bound": "mfma", "kernel": label,
                       "flop_note": "algorithmic 4 r^2 N per complex q (2 r^2 N/2 for a self-"
                                    "conjugate q on its half grid); the kernel executes 3 real "
                                    "MFMAs per complex block, so achieved/peak can reach 4/3",
                       "achieved": round(ach, 3), "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                       "frac": round(ach / PEAK_FP64_TFLOPS, 4), "traffic": None,
                       "flop_per_launch": flop_step / max(len(ranks), 1),
                       "avg_launch_ms": ms / max(calls, 1), "launches": int(calls),
                       "ms_per_step": round(ms / args.steps, 3)}
    # step-level MFMA work of the algorithm actually run: the fit's two GEMMs above
    # plus the y build's fx GEMM (time-reversal representatives), the x4 GEMMs and the selection
    # Gram (real part, K = nk nao) — every other stage is HBM- or latency-bound
    nao, nip = cell.nao_nr(), int(df.nip)
    ng0 = int(np.prod(m0))
    nk_half = len(set(min(q, int(p)) for q, p in enumerate(df.q_partner)))
    flop_other = (8.0 * nk_half * ngrid * nao * nip          # y: fx_k = X_k f_k^H
                  + 8.0 * nk * nip * nip * nao               # x4: x2_k = X_k^* X_k^T
                  + 2.0 * ng0 * ng0 * nk * nao)              # selection: Re(P P^H), lower half
    step_flop = 2 * flop_step + flop_other                   # trsm + herk, same count

    # in the timed region the fit lanes share the CUs, so the per-launch durations above
    # include contention with the other lane's kernels; one extra untimed step with a single
    # lane gives each kernel's own rate
    iso_st = {k: (0.0, 0) for k in stages}
    if not args.no_isolated:
        d.ctx.call("fisdf_set_fit_lanes", 1)
        d.ctx.call("fisdf_set_timing", 1)
        d.ctx.timings()
        step()
        torch.cuda.synchronize()
        iso_st = d.ctx.timings()
        d.ctx.call("fisdf_set_timing", 0)
        d.ctx.call("fisdf_set_fit_lanes", 0)
    tfile = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    traffic = json.load(open(tfile)) if os.path.exists(tfile) else {}
    for name, (label, tkey) in KERNELS.items():
        iso_ms, iso_calls = iso_st[name]
        if iso_ms > 0:
            iso = flop_step / (iso_ms * 1e-3) / 1e12
            roofs[name]["isolated"] = {"achieved": round(iso, 3),
                                       "frac": round(iso / PEAK_FP64_TFLOPS, 4),
                                       "avg_launch_ms": iso_ms / max(iso_calls, 1),
                                       "note": "one untimed step after the timed region, 1 fit lane"}
        if tkey in traffic:  # rocprofv3 FETCH_SIZE (x2, gfx950) + WRITE_SIZE passes, tools/prof_round.sh
            roofs[name]["traffic"] = traffic[tkey]["hbm_bytes_per_launch"]
            roofs[name]["traffic_unit"] = ("bytes/launch (measured, "
                                           + traffic.get("source", "profiles") + ")")
    dom = max(roofs, key=lambda n: roofs[n]["ms_per_step"])
    roof = roofs[dom]
    roof2 = roofs["herk" if dom == "trsm" else "trsm"]

    # input layer: Bloch AO values on the FFT grid by the GPU evaluator,
    # checked against the host restatement the timed steps used; outside the timed region
    # like the reference's own AO inputs (PySCF pbc_eval_gto)
    from fisdf.ao import eval_ao_kpts_gpu
    coords = cell.gen_uniform_grids(cell.mesh)
    eval_ao_kpts_gpu(d, cell, coords, kmesh)
    torch.cuda.synchronize()
    t = time.perf_counter()
    g = eval_ao_kpts_gpu(d, cell, coords, kmesh)
    torch.cuda.synchronize()
    ao = {"gpu_ms": round((time.perf_counter() - t) * 1e3, 3),
          "cpu_s_host_restatement": round(getattr(setup, "ao_cpu_s", float("nan")), 3),
          "max_rel_diff": float((g - df._ao_grid).abs().max() / df._ao_grid.abs().max()),
          "note": "Bloch AOs on the FFT grid (nk, ngrid, nao); not in the timed steps"}
    del g

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        chi = __import__("fisdf").cell.eval_ao_kpts(cell, cell.gen_uniform_grids(cell.mesh), kmesh)
        cpu = cpu_baseline(cell, kmesh, m0, c0, x0, chi, dm, args.cpu_q)
        del chi

    if rank == 0:
        out = {
            "metric": "ISDF build + get_jk k-points/s, diamond gth-dzvp 4x4x4"
            if args.config == "c3" else f"ISDF build + get_jk k-points/s ({args.config})",
            "value": round(value, 4), "unit": "k-points/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f64 (complex128)", "data": "synthetic (gth-dzvp-shaped contracted Gaussians)",
            "config": {"workload": DESC[args.config], "nk": nk, "nao": cell.nao_nr(),
                       "nip": int(df.nip), "ngrid": ngrid, "fit": "lstsq (Cholesky, factored order; min-norm on rank-deficient q)",
                       "parallelism": f"k-shard x{world}"
                       + (" (gloo rehearsal, not RCCL)" if world > 1 and backend == "gloo" else "")},
            "roofline": roof,
            "roofline_secondary": roof2,
            "step_mfma": {"flop_per_step": step_flop, "fit_flop_per_step": 2 * flop_step,
                          "achieved": round(step_flop / (ms_per_step * 1e-3) / 1e12, 3),
                          "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                          "frac": round(step_flop / (ms_per_step * 1e-3) / 1e12
                                        / PEAK_FP64_TFLOPS, 4),
                          "note": "algorithmic MFMA work of the algorithm run (fit TRSM + HERK "
                                  "at 4 r^2 N each per complex q, 2 r^2 N_half per self-"
                                  "conjugate q; y fx GEMM; x4; selection Gram) over the whole "
                                  "step time"},
            "cpu_baseline": cpu,
            "ao_eval": ao,
            "stages_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in stages.items()},
            "ranks": [int(ranks.min()), int(ranks.max())],
        }
        print(json.dumps(out))
    # release the library context (streams, arena, factors) while the HIP runtime and any
    # attached profiler are still up, not from an interpreter-shutdown finaliser
    torch.cuda.synchronize()
    del df
    d.ctx.close()
    if comm is not None:
        torch.distributed.destroy_process_group()
    maps = os.environ.get("FISDF_MAPS_OUT")
    if maps:  # the address map, to symbolize a crash in the exit handlers after this point
        with open("/proc/self/maps") as src, open(maps, "w") as dst:
            dst.write(src.read())


if __name__ == "__main__":
    sys.exit(main() or 0)
