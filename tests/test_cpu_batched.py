"""The cell-batched SIMD CPU baseline (oracle/gls_cpu_batched.c, bench.py's
cpu_baseline) computes the same Newton vmult as the scalar oracle
(oracle/gls_oracle.c): relative l2 <= 1e-13 (summation order only), with 1
and several threads (coloured batches: no write conflicts)."""
import pytest

import oracle as orc
from helpers import deck_case, rel_err


@pytest.mark.parametrize("name,n_ref", [("input_hoffmann_3D_Re3900.json", 1),
                                        ("input_turek_3D_Re100.json", 0)])
@pytest.mark.parametrize("threads", [1, 4])
def test_batched_matches_oracle(name, n_ref, threads):
    case = deck_case(name, n_ref)
    o = case.oracle()
    ref = o.vmult(case.src)
    b = orc.BatchedCPU(o, threads)
    assert b.n_colors >= 2
    got = b.vmult(case.src)
    assert rel_err(got, ref) < 1e-13
