"""The drop-in boundary with a PySCF-style cell (VERDICT r05 missing #1): the reference feeds
``ISDF`` a ``pyscf.pbc.gto.Cell``, whose AO values come from ``cell.pbc_eval_gto("GTOval",
coords, kpts=...)`` (fftisdf.py:367-370) and ``aoR_loop`` (:327-355), whose ``rcut`` is an
attribute, and which has no ``shells``.  PySCF is not installed here, so ``PyscfLikeCell`` is a
duck-typed stand-in exposing only that protocol (its AO values are the restatement's,
``fisdf.cell.eval_ao_band``, returned as PySCF returns them: one (ng, nao) array per k-point).
CPU: the host AO layer takes the protocol path and gives the same values as the restatement.
GPU: ``ISDF(stub, kpts).build(); get_jk(dm)`` with nothing injected matches the oracle."""
import numpy as np
import pytest

from fisdf import cell as C


class PyscfLikeCell:
    """Only what a ``pyscf.pbc.gto.Cell`` offers the reference's ISDF: no ``shells``, ``rcut``
    an attribute, ``vol`` / ``natm`` attributes, AO values through ``pbc_eval_gto``."""

    def __init__(self, inner):
        self._inner = inner
        self.mesh = tuple(inner.mesh)
        self.vol = float(inner.vol)
        self.rcut = float(inner.rcut())
        self.natm = inner.natm
        self.verbose = 0
        self.dimension = 3
        self.evals = 0

    def lattice_vectors(self):
        return self._inner.lattice_vectors()

    def reciprocal_vectors(self):
        return self._inner.reciprocal_vectors()

    def atom_coords(self):
        return self._inner.atom_coords()

    def nao_nr(self):
        return self._inner.nao_nr()

    def get_kpts(self, kmesh):
        return C.make_kpts(self._inner, kmesh)

    def gen_uniform_grids(self, mesh=None, wrap_around=True):
        return self._inner.gen_uniform_grids(mesh, wrap_around)

    def pbc_eval_gto(self, eval_name, coords, kpts=None):
        assert eval_name == "GTOval"
        self.evals += 1
        k = np.zeros((1, 3)) if kpts is None else np.asarray(kpts, float).reshape(-1, 3)
        out = C.eval_ao_band(self._inner, np.asarray(coords), k)
        return out[0] if kpts is None else [out[i] for i in range(len(k))]


def test_stub_has_no_native_basis():
    stub = PyscfLikeCell(C.toy_cell(mesh=(6, 6, 6)))
    assert not hasattr(stub, "shells") and not callable(stub.rcut)
    assert C.cell_rcut(stub) == pytest.approx(stub._inner.rcut())


def test_host_ao_layer_through_pbc_eval_gto():
    """aoR_loop (fftisdf.py:327-355) and bloch_ao on the PySCF protocol: the values of the
    restatement, evaluated through pbc_eval_gto, block by block."""
    from fisdf import ISDF
    inner = C.toy_cell(mesh=(6, 6, 6))
    stub = PyscfLikeCell(inner)
    kmesh = (2, 2, 1)
    df = ISDF(stub, stub.get_kpts(kmesh), m0=[5, 5, 5], c0=10.0)
    df.blksize = 50
    coords = stub.gen_uniform_grids(stub.mesh)
    ref = C.eval_ao_kpts(inner, coords, kmesh)
    got = np.concatenate([blk[0] for blk, g0, g1 in df.aoR_loop()], axis=1)
    assert got.shape == ref.shape
    assert abs(got - ref).max() < 1e-12 * max(1.0, abs(ref).max())
    assert stub.evals == -(-coords.shape[0] // 50)
    # the parent grid of the selection (fftisdf.py:367-370)
    x0 = C.bloch_ao(stub, stub.gen_uniform_grids(df.m0), df.kpts, df._kmesh())
    x0_ref = C.eval_ao_kpts(inner, inner.gen_uniform_grids(df.m0), kmesh)
    assert abs(x0 - x0_ref).max() < 1e-12 * max(1.0, abs(x0_ref).max())
    # the module's own Cell answers the same protocol
    pe = inner.pbc_eval_gto("GTOval", coords[:7], kpts=df.kpts)
    assert abs(pe - ref[:, :7]).max() < 1e-12 * max(1.0, abs(ref).max())
    with pytest.raises(TypeError):
        C.bloch_ao(object(), coords[:3], df.kpts)


@pytest.mark.gpu
def test_isdf_on_pyscf_style_cell_matches_oracle():
    """ISDF(stub, kpts).build(); get_jk(dm) — no AO injection: the selection's parent-grid AOs
    and the FFT-grid AOs come from stub.pbc_eval_gto — against the oracle (J/K < 1e-8 Ha, the
    GPU's own pivots equal to dpstrf's on this case as in test_gpu_isdf.test_gpu_selection)."""
    from cases import inputs, oracle
    from fisdf import ISDF
    name = "toy222"
    cell, kmesh, m0, c0, x0, coords, chi, dm = inputs(name)
    o = oracle(name)
    stub = PyscfLikeCell(cell)
    df = ISDF(stub, stub.get_kpts(kmesh), m0=list(m0), c0=c0)
    df.build()
    assert stub.evals > 0
    assert np.array_equal(df.perm, o["perm"])
    vj, vk = df.get_jk(dm)
    ej, ek = abs(vj - o["vj"]).max(), abs(vk - o["vk"]).max()
    print(f"PySCF-style cell {name}: |dJ| {ej:.2e} |dK| {ek:.2e}")
    assert ej < 1e-8 and ek < 1e-8
    assert np.allclose(df._x, o["xip"], atol=1e-12)
