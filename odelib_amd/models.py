"""Device-model registry: binds the user's Python ``ODE(y, t, ps)`` to a compiled
``__device__`` RHS (odelib_amd/csrc/models.cuh).

The reference passes the Python callable straight to odeint (ODElib/Framework.py:656).
The engine cannot run Python on the GPU, so ``resolve`` finds the compiled RHS that
computes the same function: either the one named by ``device_model=``, or — by
default — the built-in whose output agrees with the user's callable on a set of
random positive probe points.  The probe is host-side validation only; no result
of the fit ever comes from the Python callable.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _native as N
from .transpile import Unsupported, transpile


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


def _probe_equal(user, ref, n_states, n_params, trials=8, rtol=1e-12):
    rng = np.random.default_rng(12345)
    for _ in range(trials):
        y = rng.uniform(0.5, 2.0, n_states) * 10.0 ** rng.uniform(-2, 7, n_states)
        ps = list(rng.uniform(0.5, 2.0, n_params) * 10.0 ** rng.uniform(-8, 1, n_params))
        t = float(rng.uniform(0, 3))
        try:
            a = np.asarray(user(y, t, ps), dtype=float).reshape(-1)
        except Exception:
            return False
        b = np.asarray(ref(y, t, ps), dtype=float).reshape(-1)
        if a.shape != b.shape or not np.allclose(a, b, rtol=rtol, atol=0.0):
            return False
    return True


def resolve(ode, n_states: int, n_params: int, device_model: str | None = None):
    """Return (model_id, n_states) of the compiled built-in RHS equal to ``ode``."""
    dm = resolve_model(ode, n_states, n_params, device_model, allow_rtc=False)
    return dm.model_id, dm.n_states


def resolve_model(ode, n_states: int, n_params: int, device_model: str | None = None,
                  device_rhs: str | None = None, allow_rtc: bool = True) -> DeviceModel:
    """Choose the device RHS for ``ode``:

    1. ``device_rhs`` (C++ body of ``rhs(y, t, ps, dy)``)  -> hipRTC, as given;
    2. ``device_model`` naming a built-in ('zero_i', 'one_i', 'two_i', 'chain') -> that
       built-in, after checking the callable computes the same function;
       ``device_model='rtc'`` forces the transpiled path;
    3. otherwise the first built-in that agrees with the callable on probe points;
    4. otherwise the callable transpiled to C (``transpile.py``), checked against the
       callable on probe points, compiled with hipRTC."""
    if device_rhs is not None:
        return DeviceModel("custom-source", n_states, source=device_rhs)
    cands = candidates(n_states, n_params)
    if device_model is not None and device_model != "rtc":
        cands = [c for c in cands if c[0] == device_model]
        if not cands:
            raise ValueError(f"device_model={device_model!r} has no compiled RHS with S={n_states}, "
                             f"P={n_params}")
        name, mid, S, P, f = cands[0]
        if ode is not None and not _probe_equal(ode, f, n_states, n_params):
            raise ValueError(f"the ODE callable does not match the compiled {name!r} right-hand side")
        return DeviceModel(name, S, model_id=mid)
    if device_model is None:
        for name, mid, S, P, f in cands:
            if ode is not None and _probe_equal(ode, f, n_states, n_params):
                return DeviceModel(name, S, model_id=mid)
    if not allow_rtc or ode is None:
        raise NotImplementedError(
            "no compiled device RHS matches this ODE callable; built-ins are "
            f"{sorted(BUILTIN)} and chain<N> for N in {CHAIN_SIZES} (pass device_model=... or device_rhs=...)")
    try:
        tr = transpile(ode, n_states, n_params)
    except Unsupported as exc:
        raise NotImplementedError(
            f"the ODE callable matches no built-in RHS and cannot be transpiled ({exc}); pass its C body as "
            "device_rhs='...' (see include/odelib_amd.h oe_model_compile)") from exc
    if not _probe_equal(ode, tr.evaluate, n_states, n_params):
        raise NotImplementedError("the transpiled RHS does not reproduce the callable; pass device_rhs='...'")
    return DeviceModel("rtc:" + getattr(ode, "__name__", "ode"), n_states, source=tr.c_body)
