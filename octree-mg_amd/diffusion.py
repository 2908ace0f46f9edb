"""Python mirror of the reference's m_diffusion (src/m_diffusion.f90).

One implicit diffusion time step of phi, solved as a Helmholtz problem on the
GPU: the whole driver (lambda, set_rhs, FMG, the V-cycle loop) is
omg_diffusion_solve in libomg.so, so nothing leaves the device between its
cycles.  Same names, argument meaning and error behaviour as the reference:

    diffusion_solve(mg, dt, diffusion_coeff, order, max_res)   # :19-57
    diffusion_solve_vcoeff(mg, dt, order, max_res)             # :63-101, eps in var 5
    diffusion_solve_acoeff(mg, dt, order, max_res)             # :108-142, eps in vars 5..7

order 1 is backward Euler, order 2 Crank-Nicolson.  A step that does not
reach max_res within the FMG and 10 V-cycles raises OmgError("diffusion_solve:
no convergence") (the reference's error stop).  Each returns the last max
residual (the reference keeps it local).
"""
from __future__ import annotations

import ctypes as C

from .mg import MG, mg_set_methods
from .tree import MG_AHELMHOLTZ, MG_HELMHOLTZ, MG_VHELMHOLTZ

MAX_ITS = 10   # m_diffusion.f90:25


def _solve(mg: MG, op: int, dt: float, coeff: float, order: int, max_res: float) -> float:
    if order not in (1, 2):
        raise RuntimeError("diffusion_solve: order should be 1 or 2")
    mg._require_alloc()
    mg.operator_type = op
    mg_set_methods(mg)
    n, res = C.c_int(0), C.c_double(0.0)
    mg.ctx.call("diffusion_solve", op, float(dt), float(coeff), int(order), float(max_res),
                C.byref(n), C.byref(res))
    # the host copy of the methods, as the reference leaves them
    dtc = dt * coeff if op == MG_HELMHOLTZ else dt
    mg.helmholtz_lambda = order / dtc
    mg.n_vcycles_last = n.value
    return res.value


def diffusion_solve(mg: MG, dt: float, diffusion_coeff: float, order: int, max_res: float) -> float:
    """diffusion_solve (reference: src/m_diffusion.f90:19-57): constant
    coefficient, lambda = order/(dt*D)."""
    return _solve(mg, MG_HELMHOLTZ, dt, diffusion_coeff, order, max_res)


def diffusion_solve_vcoeff(mg: MG, dt: float, order: int, max_res: float) -> float:
    """diffusion_solve_vcoeff (reference: src/m_diffusion.f90:63-101): the
    coefficient in mg_iveps (var 5) on every level, lambda = order/dt."""
    return _solve(mg, MG_VHELMHOLTZ, dt, 1.0, order, max_res)


def diffusion_solve_acoeff(mg: MG, dt: float, order: int, max_res: float) -> float:
    """diffusion_solve_acoeff (reference: src/m_diffusion.f90:108-142): the
    per-axis coefficients in mg_iveps1..3 (vars 5..7), lambda = order/dt."""
    return _solve(mg, MG_AHELMHOLTZ, dt, 1.0, order, max_res)
