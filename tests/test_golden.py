"""Golden fixtures (tests/golden/*.npz, generator tests/golden/make_golden.py).

CPU: the mesh generator and the oracle reproduce the frozen outputs (drift
detection; the oracle itself is pinned by the KATs, parity against the
reference binary unpinned — SURVEY §8c).  GPU: the HIP path reproduces them
directly (FP64, relative l2 1e-12; inverse diagonal 1e-11), without running the oracle."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import make_golden as mg  # noqa: E402
from helpers import rel_err  # noqa: E402

CASES = mg.CASES


def _load(name):
    return np.load(os.path.join(HERE, "golden", name + ".npz"))


@pytest.mark.parametrize("name,deck,n_ref,ov", CASES, ids=[c[0] for c in CASES])
def test_mesh_matches_golden(name, deck, n_ref, ov):
    g = _load(name)
    m, cmask, *_ = mg.case_inputs(deck, n_ref, ov)
    assert m.n_cells == int(g["n_cells"]) and m.n_nodes == int(g["n_nodes"])
    assert mg.mesh_digest(m) == str(g["mesh_sha256"])
    assert int(np.count_nonzero(cmask)) == int(g["n_constrained"])


@pytest.mark.parametrize("name,deck,n_ref,ov", CASES, ids=[c[0] for c in CASES])
def test_oracle_matches_golden(name, deck, n_ref, ov):
    g = _load(name)
    out = mg.oracle_outputs(*mg.case_inputs(deck, n_ref, ov))
    for key in ("vmult", "residual", "inverse_diagonal"):
        # OpenMP scatter order may differ from the generating run
        assert rel_err(out[key], g[key]) < 1e-13, key


@pytest.mark.gpu
@pytest.mark.parametrize("name,deck,n_ref,ov", CASES, ids=[c[0] for c in CASES])
def test_gpu_matches_golden(name, deck, n_ref, ov):
    import torch
    import glsamd
    g = _load(name)
    m, cmask, params, w, src, u, hist = mg.case_inputs(deck, n_ref, ov)
    op = glsamd.NavierStokesOperator(m, cmask, "f64")
    op.set_parameters(**params)
    op.set_linearization_point(u)
    if params["order"] > 0:
        op.set_previous_solution(hist, w)
    s = op._dev(src)
    dst = op.initialize_dof_vector()
    res = op.initialize_dof_vector()
    diag = op.initialize_dof_vector()
    op.vmult(dst, s)
    op.evaluate_residual_plain(res, s)
    op.compute_inverse_diagonal(diag)
    torch.cuda.synchronize()
    assert rel_err(dst.cpu().numpy(), g["vmult"]) < 1e-12
    assert rel_err(res.cpu().numpy(), g["residual"]) < 1e-12
    # 1/d amplifies round-off of near-cancelling entries (as test_gpu_parity)
    assert rel_err(diag.cpu().numpy(), g["inverse_diagonal"]) < 1e-11
