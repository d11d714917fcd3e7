"""Synthetic phi-phi double-scalar tables in the reference's binary layout.

The real tables (xsec/alphatilde_phiphi.bin 5000x100, xsec/alpha_phiphi.bin
1000x1000x100) come from hours of offline scipy dblquad (xsec/tables_phiphi.py)
and are not shipped with the reference, so parity is tested on smooth positive
stand-ins with the same format (interp.hpp:249-291; xsec/text_to_binary.cpp):
float32 records {x0, .., x_{d-1}, f}, last index fastest, x0 logarithmic.
Deterministic: a fixture of data, regenerated at test time.
"""
import os

import numpy as np


def _write(path, axes, f):
    grids = np.meshgrid(*axes, indexing="ij")
    rec = np.stack([g.ravel() for g in grids] + [f(*grids).ravel()], axis=1).astype(np.float32)
    rec.tofile(path)


def make_tables(d, at_dims=(120, 10), a_dims=(40, 110, 6), x1_max=None, x0_range=(1.0, 2e4),
                delta_range=(0.003, 0.06)):
    """alphaTilde axes: {-t+ (log), log10(t+/t-)}; alpha axes: {s'- (log), ln(-s'-/t-)/ln d * 1.0001, log10 d}.
    Returns (at_path, at_dims, a_path, a_dims)."""
    os.makedirs(d, exist_ok=True)
    x1_max = x1_max if x1_max is not None else a_dims[1] - 1.0
    at_axes = [np.geomspace(*x0_range, at_dims[0]), np.linspace(*delta_range, at_dims[1])]
    a_axes = [np.geomspace(*x0_range, a_dims[0]), np.linspace(0.0, x1_max, a_dims[1]),
              np.linspace(*delta_range, a_dims[2])]
    at_path, a_path = os.path.join(d, "alphatilde_phiphi.bin"), os.path.join(d, "alpha_phiphi.bin")
    _write(at_path, at_axes, lambda x0, x1: 1e-7 * np.sqrt(x0) * (1.0 + 20.0 * x1))
    _write(a_path, a_axes, lambda x0, x1, x2: 1e-7 * np.log1p(x0) * np.exp(-x1 / 40.0) * (1.0 + 10.0 * x2))
    return at_path, list(at_dims), a_path, list(a_dims)
