"""Checkpoint / resume of device MCMC chains ("persist θ, chi and the RNG
counter per walker").

The chain state after iteration k-1 is θ [P][W], the current states y0 [S][W], the
running (chi, rsquared, aic, n_accepted) [4][W] and the status word [W]; the random
streams are a function of the iteration (Philox counters, replay arrays) or are
re-seeded and fast-forwarded on the device (numpy legacy streams).  What those streams
depend on is saved too (``rng_state``: mode, Philox seed and walker offset, step size,
walk mask, burn-in, prior draws, digests of the replay rows used; and the per-chain numpy
seeds), and ``Engine.mh_run(..., resume=load(path))`` refuses a resume whose arguments
would not continue with the draws an uninterrupted run would have used
(``engine.check_resume``).  Files are plain ``.npz`` (no pickles).
"""
from __future__ import annotations

import numpy as np

_KEYS = ("theta", "y0", "final", "status")


def save(path, result, meta=None):
    """Write the chain state of an ``Engine.mh_run`` result (+ JSON-able ``meta``)."""
    import json
    arrays = {k: (result[k].cpu().numpy() if hasattr(result[k], "cpu") else np.asarray(result[k])) for k in _KEYS}
    arrays["next_it"] = np.asarray(int(result["next_it"]), np.int64)
    arrays["meta"] = np.asarray(json.dumps(meta or {}))
    if result.get("rng_state") is not None:
        arrays["rng_state"] = np.asarray(json.dumps(result["rng_state"]))
    if result.get("numpy_seeds") is not None:
        arrays["numpy_seeds"] = np.asarray(result["numpy_seeds"], np.int64)
    np.savez(path, **arrays)


def load(path):
    """Chain state written by ``save``: dict(theta, y0, final, status, next_it, meta,
    rng_state, numpy_seeds)."""
    import json
    with np.load(path, allow_pickle=False) as z:
        out = {k: z[k] for k in _KEYS}
        out["next_it"] = int(z["next_it"])
        out["meta"] = json.loads(str(z["meta"]))
        out["rng_state"] = json.loads(str(z["rng_state"])) if "rng_state" in z else None
        out["numpy_seeds"] = z["numpy_seeds"] if "numpy_seeds" in z else None
    return out
