"""In-process interleaved A/B of the C3 bench step (round 6): one setup, then R rounds over the
configurations, each a warmup step and K timed steps (build + get_jk, bracketed by device syncs),
so box-to-box and process-to-process variance drop out of the comparison.  Only switches the
library reads per call / per build can be compared this way (FISDF_Y_STREAM,
FISDF_Y_STREAM_AUX, FISDF_SEL_WGS, FISDF_SEL_LDS_COLS, FISDF_Y_STREAM_ROWS, ...).
  python tools/ab_inproc.py --cfg "base:FISDF_Y_STREAM=0" --cfg "ys:" [--rounds 4 --steps 4]
A setting "ctx.NAME=a/b" calls the context entry NAME(ctx, a, b) (ints) before the
configuration's steps, and NAME's round-6 defaults are put back before the next one
(fisdf_set_fit_pipe -> (-1, 0), fisdf_set_fit_lanes -> 0).
Prints one JSON line: per configuration the per-round ms/step and their mean / min."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fft-isdf-scratch_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", action="append", required=True,
                    help="name:VAR=val,VAR=val (empty: library defaults)")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=4)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from fisdf import ISDF
    cfgs = []
    for c in a.cfg:
        name, _, kv = c.partition(":")
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        cfgs.append((name, env))
    keys = sorted({k for _, e in cfgs for k in e})
    cell, kmesh, m0, c0, x0, chi, dm = bench.setup("c3")
    df = ISDF(cell, cell.get_kpts(kmesh), m0=list(m0), c0=c0)
    d = df.device
    df._kmesh()
    df._ao_parent = d.to_dev(x0)
    df._ao_grid = d.to_dev(chi)
    del chi

    def step():
        df._dev_state = None
        df.build()
        df.get_jk(dm)

    res = {n: [] for n, _ in cfgs}
    defaults = {"fisdf_set_fit_pipe": (-1, 0), "fisdf_set_fit_lanes": (0,)}
    for r in range(a.rounds):
        for name, env in cfgs:
            for k in keys:
                os.environ.pop(k, None)
            for fn, dv in defaults.items():
                d.ctx.call(fn, *dv)
            for k, v in env.items():
                if k.startswith("ctx."):
                    d.ctx.call(k[4:], *[int(x) for x in v.split("/")])
            os.environ.update({k: v for k, v in env.items() if not k.startswith("ctx.")})
            step()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize()
            res[name].append(round((time.perf_counter() - t) / a.steps * 1e3, 3))
            print(f"round {r} {name}: {res[name][-1]} ms/step", file=sys.stderr, flush=True)
    for k in keys:
        os.environ.pop(k, None)
    out = {n: {"ms": v, "mean": round(float(np.mean(v)), 3), "min": min(v)} for n, v in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
