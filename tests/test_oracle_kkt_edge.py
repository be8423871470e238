"""The oracle's QDLDL restatement in the regime the Riccati-ordered GPU path
handles by an exact Moreau envelope (rho_dyn ||P|| from 0.05 to 3,
tests/kkt_cases.py): pinned against the dense QDLDL-equivalent LAPACK solve
(tests/dense_ref.py), so the GPU tests of that regime compare with a checked
checker."""
import numpy as np
import pytest

from conftest import rel_err


@pytest.mark.parametrize("name", ["e0.05_state_cost", "e0.5_state_box", "e3_rho_dyn", "wide_e0.5", "wide_e3"])
def test_oracle_kkt_large_penalty_matches_dense(name):
    from dense_ref import qdldl_equivalent
    from kkt_cases import TARGET, e_max, kkt_case, packed
    from oracle.oracle import OracleKKT

    n, m, N, batch, rd, E, c, H, h, x0, ncs, D, ws, ys, zs, irho = kkt_case(name)
    for b in range(batch):
        pm = packed(n, m, N, ncs, E, c, H, h, D, b)
        assert TARGET[name] / 2 < e_max(pm, ws[b], ys[b], zs[b], irho[b], 1e-6, rd) < 2 * TARGET[name]
        o = OracleKKT(pm, rho_dyn=rd)
        o.update_problem_data(ws[b], ys[b], zs[b], irho[b], 1e-6)
        o.backward(irho[b])
        wd = qdldl_equivalent(pm, x0[b], ws[b], ys[b], zs[b], irho[b], 1e-6, rho_dyn=rd)
        assert rel_err(o.forward(x0[b]), wd) < 1e-10
