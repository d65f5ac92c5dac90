"""Multi-rank (k-sharded) ISDF on the GPU: 2 and 3 ranks sharing cuda:0 over gloo run the
whole sharded path (sharded selection Gram + all-reduce, grid-sliced y + all-to-all,
per-shard fit, W_s all-reduce, W_0 broadcast) and must give the oracle's J/K (< 1e-8)."""
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("name,world", [("toy222", 2), ("toy331", 3), ("toy333_fr", 4)])
def test_sharded_build_matches_oracle(name, world):
    port = _port()
    with tempfile.TemporaryDirectory() as tmp:
        procs = []
        for r in range(world):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0",
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                       FISDF_DIST_EXTRAS="1" if name == "toy333_fr" else "0")
            procs.append(subprocess.Popen(
                [sys.executable, os.path.join(HERE, "dist_worker.py"), name, "gloo",
                 os.path.join(tmp, f"r{r}.npz")], env=env))
        codes = [p.wait(timeout=300) for p in procs]
        assert codes == [0] * world, codes
        outs = [np.load(os.path.join(tmp, f"r{r}.npz")) for r in range(world)]
    for r, o in enumerate(outs):
        ej = abs(o["vj"] - o["vj0"]).max()
        ek = abs(o["vk"] - o["vk0"]).max()
        same = np.array_equal(o["perm"], o["perm0"])
        print(f"{name} rank {r}/{world}: |dJ|={ej:.2e} |dK|={ek:.2e} pivots==dpstrf: {same}")
        # vs the oracle on the same point set (dist_worker.py); toy331 is rank-deficient with
        # time reversal (1.5e-8 bar, test_gpu_isdf.py)
        tol = 1.5e-8 if name == "toy331" else 1e-8
        assert ej < tol and ek < tol
        if "vk_e" in o:   # exxdiv='ewald' and omega=0.4 through the sharded path (next-4)
            ee = abs(o["vk_e"] - o["vke0"]).max()
            ewj, ewk = abs(o["vj_w"] - o["vjw0"]).max(), abs(o["vk_w"] - o["vkw0"]).max()
            print(f"  ewald |dK|={ee:.2e}  omega=0.4 |dJ|={ewj:.2e} |dK|={ewk:.2e}")
            assert ee < tol and ewj < tol and ewk < tol
            assert abs(o["vk_w"] - outs[0]["vk_w"]).max() == 0.0
        # every rank returns the same J/K and the same pivots
        assert abs(o["vj"] - outs[0]["vj"]).max() == 0.0
        assert np.array_equal(o["perm"], outs[0]["perm"])
