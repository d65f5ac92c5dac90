"""Periodic cell, k-mesh, uniform grids and Bloch-AO evaluation (host side, NumPy).

PySCF is absent from this image, so the inputs the reference gets
from PySCF's PBC layer are supplied here.  This module is the *input* layer of
the hot path — the equivalent of what PySCF hands to ``fftisdf.py`` — not part of
the ISDF algorithm itself:

* ``Cell.lattice_vectors / reciprocal_vectors / vol``   [pyscf ``pbc.gto.Cell``]
* ``make_kpts(cell, kmesh)``           -> ``cell.get_kpts(kmesh)``          (fftisdf.py:322)
* ``gen_uniform_grids(cell, mesh)``    -> ``cell.gen_uniform_grids(m0)``    (fftisdf.py:368)
                                          and ``df_obj.grids.coords``        (fftisdf.py:53)
* ``eval_ao_kpts(cell, coords, kmesh)``-> ``pbc_eval_gto('GTOval', ...)``  (fftisdf.py:367)
                                          / ``KNumInt.block_loop``          (fftisdf.py:350)

Conventions:
* Bloch AOs  chi_k(r) = sum_T exp(+i k.T) phi(r - T)                  [A2]
* kpts = cartesian_prod(arange(n_i)/n_i) @ b  (wrap_around=False)      [A1]
* grid coords: fftfreq fractions @ a  (PySCF ``wrap_around=True`` default) [A7]

Basis sets: the CP2K GTH tables are not in this container, so the basis sets
below are *synthetic contracted Gaussians with the gth-szv / gth-dzvp /
gth-dzvp-molopt-sr shell structure* (same nao per atom).  Parity is GPU vs the
CPU oracle on identical AO inputs, so the exact exponents do not matter for it.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

BOHR = 0.52917721092  # Angstrom per bohr (PySCF param.BOHR)


def cartesian_prod(arrays):
    """Same ordering as ``pyscf.lib.cartesian_prod`` (last index fastest)."""
    arrays = [np.asarray(a) for a in arrays]
    grids = np.meshgrid(*arrays, indexing="ij")
    return np.stack([g.ravel() for g in grids], axis=1)


# --------------------------------------------------------------------------
# basis sets (synthetic, shell structure of the named GTH basis)
# --------------------------------------------------------------------------
# each shell: (l, exponents, coefficients)
_C_EXP = [4.3362376436, 1.2881838513, 0.4037767149, 0.1187877657]
_SI_EXP = [1.2032403721, 0.4538664121, 0.1390828359, 0.0451432110]
_O_EXP = [8.3043855492, 2.4579484292, 0.7597373434, 0.2136388632]
_NI_EXP = [10.5, 3.6, 1.3, 0.45, 0.13]

BASIS = {
    # gth-szv shaped: 1s 1p  (nao 4 / atom)
    ("C", "gth-szv"): [
        (0, _C_EXP, [0.1490, -0.1063, -0.4660, -0.5700]),
        (1, _C_EXP, [0.0898, 0.2813, 0.4941, 0.3927]),
    ],
    ("Si", "gth-szv"): [
        (0, _SI_EXP, [0.2, -0.3, -0.5, -0.45]),
        (1, _SI_EXP, [-0.05, 0.25, 0.55, 0.4]),
    ],
    # SURVEY.md Appendix A toy: one s (1.2) + one p (0.7) primitive per atom
    ("X", "toy"): [(0, [1.2], [1.0]), (1, [0.7], [1.0])],
    # gth-dzvp shaped: 2s 2p 1d  (nao 13 / atom)
    ("C", "gth-dzvp"): [
        (0, _C_EXP, [0.1490, -0.1063, -0.4660, -0.5700]),
        (0, [0.1187877657], [1.0]),
        (1, _C_EXP, [0.0898, 0.2813, 0.4941, 0.3927]),
        (1, [0.1187877657], [1.0]),
        (2, [0.5500000000], [1.0]),
    ],
    # gth-dzvp-molopt-sr shaped: O 2s2p1d (13), Ni 2s2p2d1f (25)
    ("O", "gth-dzvp-molopt-sr"): [
        (0, _O_EXP, [0.16, -0.12, -0.48, -0.55]),
        (0, [0.2136388632], [1.0]),
        (1, _O_EXP, [0.09, 0.28, 0.50, 0.38]),
        (1, [0.2136388632], [1.0]),
        (2, [0.8], [1.0]),
    ],
    ("Ni", "gth-dzvp-molopt-sr"): [
        (0, _NI_EXP, [0.05, -0.3, 0.4, 0.6, 0.2]),
        (0, [0.13], [1.0]),
        (1, _NI_EXP, [0.1, 0.3, 0.45, 0.35, 0.1]),
        (1, [0.13], [1.0]),
        (2, _NI_EXP[:4], [0.3, 0.45, 0.35, 0.15]),
        (2, [0.45], [1.0]),
        (3, [1.1], [1.0]),
    ],
}

NSPH = {0: 1, 1: 3, 2: 5, 3: 7}


def _radial_norm(l, exps, coefs):
    """Normalise the contracted radial part  sum_i c_i r^l exp(-a_i r^2)."""
    exps = np.asarray(exps, float)
    coefs = np.asarray(coefs, float)
    # overlap of r^l e^{-a r^2} and r^l e^{-b r^2} with r^2 dr measure
    s = exps[:, None] + exps[None, :]
    ov = math.gamma(l + 1.5) / (2.0 * s ** (l + 1.5))
    norm = coefs @ ov @ coefs
    return coefs / math.sqrt(norm)


def _real_sph(l, x, y, z):
    """Real solid harmonics r^l Y_lm (orthonormal on the sphere), PySCF-like order."""
    if l == 0:
        return [np.full_like(x, 0.28209479177387814)]
    if l == 1:
        c = 0.4886025119029199
        return [c * x, c * y, c * z]
    if l == 2:
        c = 1.0925484305920792
        r2 = x * x + y * y + z * z
        return [c * x * y, c * y * z, 0.31539156525252005 * (3 * z * z - r2),
                c * x * z, 0.5462742152960396 * (x * x - y * y)]
    if l == 3:
        r2 = x * x + y * y + z * z
        return [0.5900435899266435 * y * (3 * x * x - y * y),
                2.890611442640554 * x * y * z,
                0.4570457994644658 * y * (5 * z * z - r2),
                0.3731763325901154 * z * (5 * z * z - 3 * r2),
                0.4570457994644658 * x * (5 * z * z - r2),
                1.445305721320277 * z * (x * x - y * y),
                0.5900435899266435 * x * (x * x - 3 * y * y)]
    raise NotImplementedError(l)


@dataclass
class Cell:
    """Minimal stand-in for ``pyscf.pbc.gto.Cell`` (lengths in bohr internally)."""
    a: np.ndarray                      # (3,3) lattice vectors, rows, bohr
    atoms: list                        # [(symbol, (x,y,z) bohr)]
    basis: str = "gth-dzvp"
    mesh: tuple = (36, 36, 36)
    precision: float = 1e-14
    verbose: int = 0
    shells: list = field(default_factory=list, init=False)
    dimension: int = 3
    low_dim_ft_type: str = None

    def __post_init__(self):
        self.a = np.asarray(self.a, dtype=float).reshape(3, 3)
        self.mesh = tuple(int(m) for m in self.mesh)
        self.shells = []
        ao = 0
        for ia, (sym, _) in enumerate(self.atoms):
            for (l, exps, coefs) in BASIS[(sym, self.basis)]:
                c = _radial_norm(l, exps, coefs)
                self.shells.append((ia, l, np.asarray(exps, float), c, ao))
                ao += NSPH[l]
        self._nao = ao

    # --- PySCF-compatible accessors -------------------------------------
    def nao_nr(self):
        return self._nao

    def lattice_vectors(self):
        return self.a

    def reciprocal_vectors(self):
        return 2 * np.pi * np.linalg.inv(self.a).T

    @property
    def vol(self):
        return abs(np.linalg.det(self.a))

    @property
    def natm(self):
        return len(self.atoms)

    def atom_coords(self):
        return np.asarray([xyz for _, xyz in self.atoms], float)

    def get_kpts(self, kmesh):
        return make_kpts(self, kmesh)

    def gen_uniform_grids(self, mesh=None, wrap_around=True):
        return gen_uniform_grids(self, self.mesh if mesh is None else mesh, wrap_around)

    def get_Gv(self, mesh=None):
        mesh = self.mesh if mesh is None else mesh
        rx = [np.fft.fftfreq(n, 1.0 / n) for n in mesh]
        return cartesian_prod(rx) @ self.reciprocal_vectors()

    def pbc_eval_gto(self, eval_name, coords, kpts=None):
        """``Cell.pbc_eval_gto(eval_name, coords, kpts)`` [pyscf] for AO values ('GTOval'):
        (nk, ng, nao) complex for a (nk, 3) ``kpts``, (ng, nao) for one k-point or None — the
        entry the reference calls for its AO inputs (fftisdf.py:367-370)."""
        if eval_name not in ("GTOval", "GTOval_sph"):
            raise NotImplementedError(f"pbc_eval_gto: {eval_name!r} (AO values only)")
        k = np.zeros((1, 3)) if kpts is None else np.asarray(kpts, float)
        out = eval_ao_band(self, coords, k.reshape(-1, 3))
        return out[0] if kpts is None or k.ndim == 1 else out

    def rcut(self):
        amin = min(float(e.min()) for (_, _, e, _, _) in self.shells)
        lmax = max(l for (_, l, _, _, _) in self.shells)
        r = math.sqrt(-math.log(self.precision) / amin)
        for _ in range(3):  # include the r^l prefactor
            r = math.sqrt((-math.log(self.precision) + lmax * math.log(max(r, 1.0))) / amin)
        return r


def cell_rcut(cell):
    """``cell.rcut``: a method on this module's Cell, an attribute on a PySCF Cell."""
    r = cell.rcut
    return float(r() if callable(r) else r)


def bloch_ao(cell, coords, kpts, kmesh=None):
    """Bloch AO values chi_k(r) (nk, ng, nao) complex128 on the host, for any cell object.

    * a cell of this module (explicit ``shells``): the restatement — ``eval_ao_kpts`` on the
      k-mesh grid when ``kmesh`` is given (kpts = make_kpts(cell, kmesh)), else ``eval_ao_band``;
    * any other cell with PySCF's ``pbc_eval_gto`` (a ``pyscf.pbc.gto.Cell`` or a duck-typed
      one): ``cell.pbc_eval_gto("GTOval", coords, kpts=kpts)``, exactly the reference's AO input
      (fftisdf.py:367-370; ``aoR_loop`` / ``KNumInt.block_loop``, :327-355, evaluates the same
      values block by block)."""
    coords = np.asarray(coords, float)
    kpts = np.asarray(kpts, float).reshape(-1, 3)
    if hasattr(cell, "shells"):
        if kmesh is not None:
            return eval_ao_kpts(cell, coords, kmesh)
        return eval_ao_band(cell, coords, kpts)
    if not hasattr(cell, "pbc_eval_gto"):
        raise TypeError(f"{type(cell).__name__}: a cell needs pbc_eval_gto (PySCF Cell protocol) "
                        "or explicit shells (fisdf.cell.Cell) to supply AO values")
    ao = cell.pbc_eval_gto("GTOval", coords, kpts=kpts)
    ao = np.asarray(ao)
    nao = cell.nao_nr()
    if ao.shape != (len(kpts), len(coords), nao):   # a single k-point may come back unbatched
        ao = ao.reshape(len(kpts), len(coords), nao)
    return ao.astype(np.complex128, copy=False)


def make_kpts(cell, kmesh):
    """``Cell.get_kpts(kmesh)`` with wrap_around=False, Gamma included."""
    ks = cartesian_prod([np.arange(n) / n for n in kmesh])
    return ks @ cell.reciprocal_vectors()


def gen_uniform_grids(cell, mesh, wrap_around=True):
    if wrap_around:
        qv = cartesian_prod([np.fft.fftfreq(n) for n in mesh])
    else:
        qv = cartesian_prod([np.arange(n) / n for n in mesh])
    return qv @ cell.lattice_vectors()


def image_translations(kmesh):
    """T_R of the supercell images, ``get_phase`` order (fftisdf.py:28)."""
    return cartesian_prod([np.arange(n) for n in kmesh])


def get_phase(cell, kmesh):
    """Phi[R,k] = exp(i T_R.k)/sqrt(nk) — ``k2gamma.get_phase(wrap_around=False)``."""
    kpts = make_kpts(cell, kmesh)
    ts = image_translations(kmesh) @ cell.lattice_vectors()
    nk = len(kpts)
    return np.exp(1j * ts @ kpts.T) / np.sqrt(nk)


def lattice_translations(cell, coords):
    """Lattice translations n (T = n @ a) that can bring an atom within ``rcut`` of the grid
    (the box of eval_ao_folded), cartesian order."""
    coords = np.asarray(coords, float)
    b = cell.reciprocal_vectors()
    rc = cell_rcut(cell)
    frac = coords @ b.T / (2 * np.pi)   # grid extent in fractional coords (may be wrapped)
    fmin, fmax = frac.min(axis=0), frac.max(axis=0)
    reach = rc * np.linalg.norm(b, axis=1) / (2 * np.pi)
    afrac = cell.atom_coords() @ b.T / (2 * np.pi)
    lo = np.floor(fmin - afrac.max(axis=0) - reach).astype(int) - 1
    hi = np.ceil(fmax - afrac.min(axis=0) + reach).astype(int) + 1
    return cartesian_prod([np.arange(lo[i], hi[i] + 1) for i in range(3)])


def eval_ao_folded(cell, coords, kmesh):
    """F_R(r) = sum_{T == T_R mod kmesh} phi(r - T), real, shape (nimg, ng, nao).

    Bloch AOs follow as chi_k = sqrt(nk) * Phi^T F  (SURVEY A1), see ``eval_ao_kpts``.
    """
    coords = np.asarray(coords, float)
    ng = coords.shape[0]
    kmesh = tuple(int(k) for k in kmesh)
    nimg = int(np.prod(kmesh))
    nao = cell.nao_nr()
    a = cell.lattice_vectors()
    rc = cell_rcut(cell)
    out = np.zeros((nimg, ng, nao))
    atom_xyz = cell.atom_coords()
    rc2 = rc * rc
    shells_by_atom = {}
    for sh in cell.shells:
        shells_by_atom.setdefault(sh[0], []).append(sh)
    for n in lattice_translations(cell, coords):
        T = n @ a
        R = tuple(int(x) % int(k) for x, k in zip(n, kmesh))
        ridx = (R[0] * kmesh[1] + R[1]) * kmesh[2] + R[2]
        for ia in range(cell.natm):
            d = coords - (atom_xyz[ia] + T)
            r2 = np.einsum("gi,gi->g", d, d)
            m = r2 < rc2
            if not m.any():
                continue
            dm = d[m]
            r2m = r2[m]
            idx = np.nonzero(m)[0]
            for (_, l, exps, cs, ao0) in shells_by_atom.get(ia, []):
                rad = np.exp(-np.outer(r2m, exps)) @ cs
                angs = _real_sph(l, dm[:, 0], dm[:, 1], dm[:, 2])
                blk = np.stack([rad * g for g in angs], axis=1)
                out[ridx, idx, ao0:ao0 + NSPH[l]] += blk
    return out


def eval_ao_band(cell, coords, kpts):
    """Bloch AO values at arbitrary k-points (kpts_band), (nkb, ng, nao) complex128:
    chi_k(r) = sum_T exp(i k.T) phi(r - T) over the translations of ``lattice_translations``
    (pbc_eval_gto at band k-points [pyscf]; off the k-mesh the image folding of
    ``eval_ao_folded`` does not apply)."""
    coords = np.asarray(coords, float)
    kpts = np.asarray(kpts, float).reshape(-1, 3)
    ng = coords.shape[0]
    nao = cell.nao_nr()
    a = cell.lattice_vectors()
    rc2 = cell_rcut(cell) ** 2
    atom_xyz = cell.atom_coords()
    out = np.zeros((len(kpts), ng, nao), complex)
    shells_by_atom = {}
    for sh in cell.shells:
        shells_by_atom.setdefault(sh[0], []).append(sh)
    for n in lattice_translations(cell, coords):
        T = n @ a
        ph = np.exp(1j * kpts @ T)
        F = np.zeros((ng, nao))
        for ia in range(cell.natm):
            d = coords - (atom_xyz[ia] + T)
            r2 = np.einsum("gi,gi->g", d, d)
            m = r2 < rc2
            if not m.any():
                continue
            dm = d[m]
            idx = np.nonzero(m)[0]
            for (_, l, exps, cs, ao0) in shells_by_atom.get(ia, []):
                rad = np.exp(-np.outer(r2[m], exps)) @ cs
                angs = _real_sph(l, dm[:, 0], dm[:, 1], dm[:, 2])
                F[idx, ao0:ao0 + NSPH[l]] += np.stack([rad * g for g in angs], axis=1)
        out += ph[:, None, None] * F[None]
    return out


def eval_ao_kpts(cell, coords, kmesh, folded=None):
    """Bloch AO values chi_k(r), shape (nk, ng, nao), complex128 (pbc_eval_gto 'GTOval')."""
    if folded is None:
        folded = eval_ao_folded(cell, coords, kmesh)
    nimg, ng, nao = folded.shape
    phase = get_phase(cell, kmesh)
    chi = (np.sqrt(nimg) * phase.T) @ folded.reshape(nimg, -1)
    return chi.reshape(nimg, ng, nao)


# --------------------------------------------------------------------------
# the benchmark / test cells
# --------------------------------------------------------------------------
def diamond_cell(basis="gth-dzvp", mesh=(36, 36, 36), shift=None):
    """Reference's diamond cell literal (fftdf-with-k-svd.py:189-191), Angstrom -> bohr.
    shift (Angstrom, 3-vector): displacement of the second C off 0.8917 (1,1,1), which breaks the
    cell's point symmetry (no symmetry-equivalent parent-grid points, hence no exactly tied
    pivots in the selection)."""
    a = (np.ones((3, 3)) * 3.5668 - np.eye(3) * 3.5668) / BOHR
    c2 = np.full(3, 0.8917) + (0.0 if shift is None else np.asarray(shift, float))
    atoms = [("C", np.zeros(3)), ("C", c2 / BOHR)]
    return Cell(a=a, atoms=atoms, basis=basis, mesh=mesh)


def toy_cell(mesh=(12, 12, 12), scale=2.2, basis="toy"):
    """SURVEY.md Appendix A toy fcc cell: a = (ones-eye)*2.2 bohr, atoms at 0 and (1,1,1)*1.1."""
    a = (np.ones((3, 3)) - np.eye(3)) * scale
    atoms = [("X", np.zeros(3)), ("X", np.full(3, 0.5 * scale))]
    return Cell(a=a, atoms=atoms, basis=basis, mesh=mesh)


def si_supercell(mesh=(30, 30, 30), basis="gth-szv", ncell=(2, 2, 2)):
    """Si diamond-structure primitive (a=5.431 A) 2x2x2 supercell, 16 atoms (config C5)."""
    a0 = 5.431 / BOHR
    prim = np.array([[0, 0.5, 0.5], [0.5, 0, 0.5], [0.5, 0.5, 0]]) * a0
    basis_atoms = [np.zeros(3), np.full(3, 0.25 * a0)]
    atoms = []
    for n in cartesian_prod([np.arange(c) for c in ncell]):
        T = n @ prim
        for xyz in basis_atoms:
            atoms.append(("Si", xyz + T))
    a = prim * np.asarray(ncell)[:, None]
    return Cell(a=a, atoms=atoms, basis=basis, mesh=mesh)


def read_poscar(path):
    """Parse a VASP POSCAR (e.g. the reference's nio-afm.vasp:1-12); returns (a_bohr, atoms)."""
    with open(path) as f:
        lines = [ln.strip() for ln in f if ln.strip()]
    scale = float(lines[1].split()[0])
    a = np.array([[float(x) for x in lines[i].split()[:3]] for i in (2, 3, 4)]) * scale
    syms = lines[5].split()
    counts = [int(x) for x in lines[6].split()]
    mode = lines[7][0].lower()
    pos = np.array([[float(x) for x in lines[8 + i].split()[:3]] for i in range(sum(counts))])
    if mode == "d":
        pos = pos @ a
    else:
        pos = pos * scale
    atoms = []
    k = 0
    for s, c in zip(syms, counts):
        for _ in range(c):
            atoms.append((s, pos[k] / BOHR))
            k += 1
    return a / BOHR, atoms


# nio-afm.vasp content as data (nio-afm.vasp:3-12), so the GPU box needs no file
NIO_AFM_A = np.array([[4.17, 2.085, 2.085], [2.085, 4.17, 2.085], [2.085, 2.085, 4.17]])
NIO_AFM_FRAC = [("Ni", (0, 0, 0)), ("Ni", (0.5, 0.5, 0.5)),
                ("O", (0.25, 0.25, 0.25)), ("O", (0.75, 0.75, 0.75))]


def nio_cell(mesh=(32, 32, 32), basis="gth-dzvp-molopt-sr"):
    """NiO AFM cell of nio-afm.vasp (config C4)."""
    a = NIO_AFM_A / BOHR
    atoms = [(s, np.asarray(f, float) @ a) for s, f in NIO_AFM_FRAC]
    return Cell(a=a, atoms=atoms, basis=basis, mesh=mesh)


def make_dm(nao, kmesh, cell, seed=1234, scale=0.1):
    """Hermitian, time-reversal-symmetric k-point dm:
    D_k = 1/2 (sum_T e^{ik.T} D_T + h.c.) + I, D_T ~ scale*N(0,1), seed 1234."""
    rng = np.random.default_rng(seed)
    nimg = int(np.prod(kmesh))
    dT = scale * rng.standard_normal((nimg, nao, nao))
    phase = get_phase(cell, kmesh)
    dk = np.sqrt(nimg) * np.einsum("Rk,Rmn->kmn", phase, dT)
    dk = 0.5 * (dk + dk.conj().transpose(0, 2, 1)) + np.eye(nao)[None]
    return dk


def madelung(cell, kmesh, precision=1e-16):
    """[pyscf] ``tools.pbc.madelung(cell, kpts)``: minus twice the Ewald energy of one unit point
    charge in the Born-von Karman supercell (lattice vectors ``a_i * kmesh_i``) with a
    neutralising background — the G=0 exchange correction of ``exxdiv='ewald'``.

    E = 1/2 sum_{L!=0} erfc(eta|L|)/|L| + (2 pi/V) sum_{G!=0} exp(-G^2/4 eta^2)/G^2
        - eta/sqrt(pi) - pi/(2 eta^2 V),
    both lattice sums taken to ``precision`` (the result does not depend on eta; PySCF cuts its
    sums by ``cell.precision`` and the supercell mesh instead).  Simple cubic, side L:
    2.8372974794806 / L."""
    from scipy.special import erfc
    A = cell.lattice_vectors() * np.asarray(kmesh, float)[:, None]
    V = abs(np.linalg.det(A))
    B = 2 * np.pi * np.linalg.inv(A).T
    eta = math.sqrt(math.pi) / V ** (1.0 / 3)
    s = math.sqrt(-math.log(precision))
    rmax, gmax = (s + 1.0) / eta, 2 * eta * (s + 1.0)
    n = np.ceil(rmax * np.linalg.norm(B, axis=1) / (2 * np.pi)).astype(int) + 1
    L = cartesian_prod([np.arange(-m, m + 1) for m in n]) @ A
    r = np.linalg.norm(L, axis=1)
    r = r[(r > 0) & (r < rmax)]
    e_real = 0.5 * np.sum(erfc(eta * r) / r)
    m = np.ceil(gmax * np.linalg.norm(A, axis=1) / (2 * np.pi)).astype(int) + 1
    G = cartesian_prod([np.arange(-k, k + 1) for k in m]) @ B
    g2 = np.einsum("gi,gi->g", G, G)
    g2 = g2[(g2 > 0) & (g2 < gmax * gmax)]
    e_recip = 2 * np.pi / V * np.sum(np.exp(-g2 / (4 * eta * eta)) / g2)
    e_self = -eta / math.sqrt(math.pi) - math.pi / (2 * eta * eta * V)
    return -2.0 * (e_real + e_recip + e_self)
