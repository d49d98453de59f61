"""Device-model registry: binds the user's Python ``ODE(y, t, ps)`` to a compiled
``__device__`` RHS (odelib_amd/csrc/models.cuh).

The reference passes the Python callable straight to odeint (ODElib/Framework.py:656).
The engine cannot run Python on the GPU, so ``resolve_model`` finds the device RHS that
computes the same function: the one named by ``device_model=``, a built-in whose exact
algebraic form equals the transpiled callable's, or the callable itself transpiled to C
and compiled with hipRTC.  No result of the fit ever comes from the Python callable.
"""
from __future__ import annotations

import warnings
from dataclasses import dataclass

import numpy as np

from . import _native as N
from .transpile import Unsupported, polynomial_form, transpile


@dataclass
class DeviceModel:
    """What the engine runs for a user ODE: a compiled built-in (model_id) or a user
    RHS body compiled at run time with hipRTC (source)."""
    name: str
    n_states: int
    model_id: int | None = None
    source: str | None = None


# Python statements of the compiled RHS (same operand order as models.cuh), used only
# to validate a user's callable before binding it to the device RHS.
def _zero_i(y, t, ps):
    mu, phi, beta = ps[0], ps[1], ps[2]
    S, V = y[0], y[1]
    return np.array([mu * S - phi * S * V, beta * phi * S * V - phi * S * V])


def _one_i(y, t, ps):
    mu, phi, beta, lam = ps[0], ps[1], ps[2], ps[3]
    S, I1, V = y[0], y[1], y[2]
    return np.array([mu * S - phi * S * V, phi * S * V - lam * I1, beta * lam * I1 - phi * S * V])


def _two_i(y, t, ps):
    mu, phi, beta, lam, tau = ps[0], ps[1], ps[2], ps[3], ps[4]
    S, I1, I2, V = y[0], y[1], y[2], y[3]
    return np.array([mu * S - phi * S * V, phi * S * V - tau * I1, tau * I1 - lam * I2,
                     beta * lam * I2 - phi * S * V])


def chain_rhs(n: int):
    """Python statement of the synthetic N-state chain."""
    if n < 4:
        raise ValueError("chain model needs N >= 4")

    def rhs(y, t, ps):
        mu, phi, beta, lam, tau = ps[0], ps[1], ps[2], ps[3], ps[4]
        S, V = y[0], y[n - 1]
        dy = np.empty(n)
        dy[0] = mu * S - phi * S * V
        dy[1] = phi * S * V - tau * y[1]
        for k in range(2, n - 2):
            dy[k] = tau * y[k - 1] - tau * y[k]
        dy[n - 2] = tau * y[n - 3] - lam * y[n - 2]
        dy[n - 1] = beta * lam * y[n - 2] - phi * S * V
        return dy

    rhs.__name__ = f"chain{n}"
    return rhs


BUILTIN = {
    "zero_i": (N.OE_MODEL_ZERO_I, 2, 3, _zero_i),
    "one_i": (N.OE_MODEL_ONE_I, 3, 4, _one_i),
    "two_i": (N.OE_MODEL_TWO_I, 4, 5, _two_i),
}
CHAIN_SIZES = (4, 5, 6, 8, 10, 12, 16, 20, 24, 32)  # compiled chain instantiations


def candidates(n_states: int, n_params: int):
    out = []
    for name, (mid, S, P, f) in BUILTIN.items():
        if S == n_states and P <= n_params <= P + min(S, 4):
            out.append((name, mid, S, P, f))
    if n_states in CHAIN_SIZES and 5 <= n_params <= 5 + min(n_states, 4):
        out.append(("chain", N.OE_MODEL_CHAIN, n_states, 5, chain_rhs(n_states)))
    return out


def _probe_equal(user, ref, n_states, n_params, trials=8, rtol=1e-12, times=None):
    """Numerical agreement on random positive states/parameters, with t drawn from the
    problem's whole time grid (both ends included) when ``times`` is given."""
    rng = np.random.default_rng(12345)
    if times is not None and len(times):
        tv = np.asarray(times, float)
        t_probe = np.r_[tv[0], tv[-1], rng.choice(tv, size=max(trials - 2, 0))]
    else:
        t_probe = rng.uniform(0, 3, trials)
    for k in range(len(t_probe)):
        y = rng.uniform(0.5, 2.0, n_states) * 10.0 ** rng.uniform(-2, 7, n_states)
        ps = list(rng.uniform(0.5, 2.0, n_params) * 10.0 ** rng.uniform(-8, 1, n_params))
        t = float(t_probe[k])
        try:
            a = np.asarray(user(y, t, ps), dtype=float).reshape(-1)
        except Exception:
            return False
        b = np.asarray(ref(y, t, ps), dtype=float).reshape(-1)
        if a.shape != b.shape or not np.allclose(a, b, rtol=rtol, atol=0.0):
            return False
    return True


def _builtin_form(f, n_states, n_params):
    return polynomial_form(transpile(f, n_states, n_params))


def resolve(ode, n_states: int, n_params: int, device_model: str | None = None, times=None):
    """Return (model_id, n_states) of the compiled built-in RHS equal to ``ode``."""
    dm = resolve_model(ode, n_states, n_params, device_model, allow_rtc=False, times=times)
    return dm.model_id, dm.n_states


def resolve_model(ode, n_states: int, n_params: int, device_model: str | None = None,
                  device_rhs: str | None = None, allow_rtc: bool = True, times=None) -> DeviceModel:
    """Choose the device RHS for ``ode``:

    1. ``device_rhs`` (C++ body of ``rhs(y, t, ps, dy)``)  -> hipRTC, as given;
    2. ``device_model`` naming a built-in ('zero_i', 'one_i', 'two_i', 'chain') -> that
       built-in, after checking the callable computes the same function: exactly (the
       algebraic form below) when the callable transpiles, otherwise numerically on
       probe points over the time grid, with a warning; ``device_model='rtc'`` forces
       the transpiled path;
    3. otherwise a built-in only when the callable is PROVABLY the same function: it
       transpiles, it is a polynomial in y and ps (no t, no calls, no branches) and its
       exact normal form (``transpile.polynomial_form``: expanded monomials with rational
       coefficients) equals the built-in's.  Agreement on probe points alone never
       binds a callable: a term switched on by t or by the state outside the probed
       region would otherwise be silently replaced;
    4. otherwise the callable transpiled to C (``transpile.py``), checked against the
       callable on probe points over the time grid, compiled with hipRTC.
    ``times`` is the problem's output grid (probe times)."""
    if device_rhs is not None:
        return DeviceModel("custom-source", n_states, source=device_rhs)
    cands = candidates(n_states, n_params)
    tr, why = None, None
    if ode is not None:
        try:
            tr = transpile(ode, n_states, n_params)
        except Unsupported as exc:
            why = exc
    if device_model is not None and device_model != "rtc":
        cands = [c for c in cands if c[0] == device_model]
        if not cands:
            raise ValueError(f"device_model={device_model!r} has no compiled RHS with S={n_states}, "
                             f"P={n_params}")
        name, mid, S, P, f = cands[0]
        if ode is not None:
            if tr is not None:  # exact: same normal form, or it is not this built-in
                form = polynomial_form(tr)
                if form is None or form != _builtin_form(f, n_states, n_params):
                    raise ValueError(f"the ODE callable is not algebraically the compiled {name!r} right-hand "
                                     "side (it differs, or reads t / branches / calls a function); omit "
                                     "device_model to run it through hipRTC")
            elif not _probe_equal(ode, f, n_states, n_params, times=times):
                raise ValueError(f"the ODE callable does not match the compiled {name!r} right-hand side")
            else:
                warnings.warn(f"device_model={name!r}: the ODE callable does not transpile, so it was checked "
                              "against the compiled right-hand side numerically only (probe points over the "
                              "time grid); the fit uses the compiled built-in", stacklevel=3)
        return DeviceModel(name, S, model_id=mid)
    if device_model is None and tr is not None:
        form = polynomial_form(tr)
        if form is not None:
            for name, mid, S, P, f in cands:
                if form == _builtin_form(f, n_states, n_params):
                    return DeviceModel(name, S, model_id=mid)
    if not allow_rtc or ode is None:
        raise NotImplementedError(
            "no compiled device RHS is provably equal to this ODE callable; built-ins are "
            f"{sorted(BUILTIN)} and chain<N> for N in {CHAIN_SIZES} (pass device_model=... or device_rhs=...)")
    if tr is None:
        raise NotImplementedError(
            f"the ODE callable cannot be transpiled ({why}); pass its C body as device_rhs='...' (see "
            "include/odelib_amd.h oe_model_compile), or device_model='<built-in>' to assert that it is one")
    if not _probe_equal(ode, tr.evaluate, n_states, n_params, times=times):
        raise NotImplementedError("the transpiled RHS does not reproduce the callable; pass device_rhs='...'")
    return DeviceModel("rtc:" + getattr(ode, "__name__", "ode"), n_states, source=tr.c_body)
