"""gls-vmult (tools/gls_vmult.hip): the reference's benchmark program
(performance.cc:12-182) on this library -- hyper cube, FESystem(FE_Q(k),
dim+1), cell-wise stabilisation, no time derivative, BDF2 after one dt
update; the three timed variants ns::vmult::mf / ns::vmult::mb /
poisson::vmult::mf.  With --check the program fills src and the
linearisation point and requires mf == mb (the compute_matrix equivalence
performance.cc relies on, 1e-12) and the Poisson cell loop == a host loop of
the same operator (1e-12)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tools", "build", "gls-vmult")


def test_gls_vmult_built():
    assert os.path.exists(EXE), "run `make tools` (or __graft_entry__.build())"


@pytest.mark.gpu
@pytest.mark.parametrize("dim,n_ref,k", [(2, 3, 1), (2, 3, 2), (2, 2, 3), (3, 2, 1), (3, 2, 2),
                                         (3, 1, 3)])
def test_gls_vmult_check(dim, n_ref, k):
    r = subprocess.run([EXE, str(dim), str(n_ref), str(k), "--check"], capture_output=True,
                       text=True, timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    for name in ("ns::vmult::mf", "ns::vmult::mb", "poisson::vmult::mf", "ns::vmult "):
        assert name in r.stdout
