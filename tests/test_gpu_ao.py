"""GPU Bloch-AO evaluation (fisdf_eval_ao) vs the host restatement
cell.eval_ao_kpts (what PySCF's pbc_eval_gto hands fftisdf.py:72,367-370): s/p/d/f shells,
register k-mesh DFTs (2x2x2, 3x3x3, 1x1x2, Gamma) and the generic direct DFT (1x1x3, 3x1x2),
FFT grid and parent grid."""
import numpy as np
import pytest

from cases import inputs

pytestmark = pytest.mark.gpu


def _gpu_vs_host(cell, coords, kmesh):
    from fisdf import ISDF
    from fisdf.ao import eval_ao_kpts_gpu
    from fisdf.cell import eval_ao_kpts
    df = ISDF(cell, cell.get_kpts(kmesh))
    got = eval_ao_kpts_gpu(df.device, cell, coords, kmesh).cpu().numpy()
    ref = eval_ao_kpts(cell, coords, kmesh)
    assert got.shape == ref.shape
    err = abs(got - ref).max() / abs(ref).max()
    print(f"kmesh {kmesh} ng {coords.shape[0]} nao {cell.nao_nr()}: max rel err {err:.2e}")
    return err


@pytest.mark.parametrize("name", ["toy222", "toy333_fr", "diamond_szv_gamma", "nio_small"])
def test_eval_ao_matches_host(name):
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    assert _gpu_vs_host(cell, coords, kmesh) < 1e-13
    assert _gpu_vs_host(cell, cell.gen_uniform_grids(m0), kmesh) < 1e-13


@pytest.mark.parametrize("kmesh", [(1, 1, 3), (3, 1, 2)])
def test_eval_ao_generic_kmesh(kmesh):
    from fisdf import cell as C
    cell = C.toy_cell(mesh=(9, 9, 9))
    assert _gpu_vs_host(cell, cell.gen_uniform_grids(cell.mesh), kmesh) < 1e-13


def test_isdf_build_with_gpu_ao_matches_oracle():
    """The whole path from cell parameters: AO inputs evaluated on the GPU, then build +
    get_jk against the oracle (which uses the host AO values)."""
    from cases import oracle
    from fisdf import ISDF
    name = "toy333_fr"
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    o = oracle(name)
    df = ISDF(cell, cell.get_kpts(kmesh), m0=list(m0), c0=c0)
    assert df.ao_on_gpu
    df.set_interpolation_points(o["perm"])
    df.build()
    vj, vk = df.get_jk(dm)
    ej, ek = abs(vj - o["vj"]).max(), abs(vk - o["vk"]).max()
    print(f"{name} with GPU AO inputs: |dJ| {ej:.2e} |dK| {ek:.2e}")
    assert ej < 1e-8 and ek < 1e-8
