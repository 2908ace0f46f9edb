"""m_diffusion (src/m_diffusion.f90) without a GPU: the Python mirror's
argument checks, and the oracle's restatement of the driver against the
reference's own behaviour (the goldens diff_* in tests/golden/golden.json are
checked by test_oracle_golden.py; the GPU path by the -m gpu tests)."""
import pytest

from tests.mgdriver import OracleBackend, omg, parse, setup_problem


def test_mirror_rejects_bad_order_before_touching_the_device():
    mg = omg.MG()   # not even allocated: the order check comes first (:42-43)
    with pytest.raises(RuntimeError, match="order should be 1 or 2"):
        omg.diffusion_solve(mg, 0.01, 1.0, 3, 1e-8)
    with pytest.raises(RuntimeError, match="order should be 1 or 2"):
        omg.diffusion_solve_vcoeff(mg, 0.01, 0, 1e-8)


def test_mirror_needs_storage():
    mg = omg.MG()
    with pytest.raises(RuntimeError, match="not allocated"):
        omg.diffusion_solve_acoeff(mg, 0.01, 1, 1e-8)


def test_oracle_bad_order_and_state():
    be = OracleBackend(parse("8 16 16 16 1 d1 gsrb helm 0.01 n0 phi 1 lb 0"))
    setup_problem(be)
    rc, n, res = be.o.diffusion_solve(3, 0.01, 1.0, 3, 1e-8)
    assert rc == 2
    rc, n, res = be.o.diffusion_solve(3, 0.01, 1.0, 1, 1e-8)
    assert rc == 0 and 0 <= n <= 10 and res <= 1e-8


def test_oracle_step_is_linear_in_phi():
    """Backward Euler is linear: phi -> 2 phi doubles the new phi (up to the
    solver tolerance), a property check that does not need the reference."""
    import numpy as np
    outs = []
    for scale in (1.0, 2.0):
        be = OracleBackend(parse("8 16 16 16 1 d1 gsrb helm 0.01 n0 phi 1 lb 0"))
        setup_problem(be)
        for lvl in be.levels():
            be.set_level(lvl, 1, scale * be.get_level(lvl, 1))
        rc, _, _ = be.o.diffusion_solve(3, 0.01, 1.0, 1, 1e-7)
        assert rc == 0
        outs.append(be.get_level(be.tree.highest_lvl, 1)[:, 1:-1, 1:-1, 1:-1])
    assert np.allclose(outs[1], 2 * outs[0], rtol=0, atol=1e-7)
