"""fisdf — MI355X-native FFT-ISDF (k-point interpolative separable density fitting).

Host-side mirror of the reference's ``fftisdf.py`` surface; the numerical work runs in
hand-written HIP kernels (libfisdf.so, C-ABI in include/fisdf.h).
"""
from .cell import Cell, diamond_cell, si_supercell, nio_cell, toy_cell, make_kpts, make_dm  # noqa: F401
from . import coul  # noqa: F401  (get_coul script surface)
from .isdf import (ISDF, InterpolativeSeparableDensityFitting, build, get_j_kpts,  # noqa: F401
                   get_k_kpts, kpts_to_kmesh)

__all__ = ["Cell", "ISDF", "InterpolativeSeparableDensityFitting", "build", "get_j_kpts",
           "get_k_kpts", "kpts_to_kmesh", "diamond_cell", "si_supercell", "nio_cell",
           "toy_cell", "make_kpts", "make_dm"]
