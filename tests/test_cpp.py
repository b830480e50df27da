"""The C++ facade (include/gls_operator.hpp) — the host-side mirror of the
reference's OperatorBase — driven by tests/cpp/test_operator.cc against the
oracle's C API on deck meshes (FP64, relative l2 < 1e-12), plus its error
path (gls::Error on an invalid descriptor)."""
import os
import subprocess

import pytest

from helpers import deck

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "build", "test_operator")


def _args(name, n_ref, **overrides):
    d = deck(name)
    for k, v in overrides.items():
        setattr(d, k, v)
    m = d.mesh(n_ref)
    vel, p, slip = d.boundary_descriptor()
    bits = lambda ids: sum(1 << int(i) for i in ids)  # noqa: E731
    prm, w = d.operator_parameters(2.5e-4)
    flags = ((1 if prm["increment_form"] else 0) | (2 if prm["consider_time_derivative"] else 0)
             | (4 if prm["cell_wise_stabilization"] else 0))
    mp = m.params
    a = [m.dim, m.degree, n_ref, mp["length"], mp["height"], mp["position"], mp["diameter"],
         mp["shift"], bits(vel), bits(p), bits(slip), d.u_max, prm["nu"], prm["c1"], prm["c2"],
         prm["theta"], prm["dt"], prm["order"], flags] + list(w)
    return [str(x) for x in a]


def test_cpp_program_built():
    assert os.access(EXE, os.X_OK), "run `make cpptest` (or __graft_entry__.build())"


@pytest.mark.gpu
@pytest.mark.parametrize("name,n_ref,ov", [
    ("input_hoffmann_3D_Re3900.json", 1, {}),
    ("input_turek_2D_Re100.json", 2, {}),
    ("input_turek_2D_Re20_stat.json", 1, {}),
    ("input_turek_3D_Re100.json", 0, {"nonlinear_solver": "linearized",
                                      "cell_wise_stabilization": True}),
])
def test_cpp_facade_parity(name, n_ref, ov):
    r = subprocess.run([EXE] + _args(name, n_ref, **ov), capture_output=True, text=True,
                       timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "error path ok" in r.stdout
