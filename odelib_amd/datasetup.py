"""Data set-up of a fit: what ``ModelFramework.__init__`` derives from the user's table.

These are the constant inputs of the batched kernel: the output
time grid, for every observation the grid index it is compared at, the observed log
abundance and its log sigma, and the state summations that map ODE states onto observed
columns.  Behaviour follows ODElib/Framework.py (cited per function) and is pinned by the
golden set-up vectors (tests/test_host_logic.py); the code is this package's own.
"""
from __future__ import annotations

import warnings
from dataclasses import dataclass

import numpy as np
import pandas as pd


def tidy_dataframe(raw: pd.DataFrame, state_names):
    """Normalise the two accepted data layouts (Framework.py:281-307).

    * one row per observation with ``abundance`` (and optionally ``log_abundance``,
      ``log_sigma``): indexed by organism; a missing log_sigma is 1 for every row;
    * replicate rows (a ``replicate`` column): per (time, organism) the mean abundance,
      the mean log abundance and the sample std of the log abundance.

    Returns (table indexed by organism, {state: (abundance, log_abundance, log_sigma)}
    for the replicate layout, else {})."""
    data = raw.sort_values(by=["organism", "time"])
    if "replicate" not in data:
        data = data.set_index("organism")
        if "abundance" in data and "log_abundance" not in data:
            data["log_abundance"] = np.log(data["abundance"].to_numpy())
        if "log_sigma" not in data:
            data["log_sigma"] = 1
            warnings.warn("log_sigma not found, setting log variance to 1")
        return data, {}
    reps = data[["organism", "time", "abundance"]].copy()
    reps["log_abundance"] = np.log(reps["abundance"])
    grouped = reps.groupby(by=["time", "organism"])
    table = grouped.mean()
    table["log_sigma"] = grouped.std()["log_abundance"]
    table = table.reset_index(level="time")
    per_state = {}
    for s in state_names:
        if s in table.index:
            rows = table.loc[s]
            per_state[s] = (rows["abundance"].to_numpy(), rows["log_abundance"].to_numpy(),
                            rows["log_sigma"].to_numpy())
    return table, per_state


def _column(table: pd.DataFrame, organism, col):
    """All values of ``col`` for one organism as a 1-d array (one row or many)."""
    return np.atleast_1d(np.asarray(table.loc[organism][col]))


def observation_index(table: pd.DataFrame, times: np.ndarray):
    """For every observed organism, in the table's (sorted) order: the grid index each
    observation is compared at — the FIRST grid point nearest to its time
    (Framework.py:309-319) — and the observed log abundance / log sigma (:323-327)."""
    pred_tindex, obs_log, obs_logsigma = {}, {}, {}
    for organism in dict.fromkeys(table.index):  # first-appearance order, no repeats
        t_obs = _column(table, organism, "time")
        # argmin returns the first minimiser, as np.where(d == min(d))[0][0] does
        pred_tindex[organism] = np.array([int(np.argmin(np.abs(t - times))) for t in t_obs])
        obs_log[organism] = _column(table, organism, "log_abundance")
        obs_logsigma[organism] = _column(table, organism, "log_sigma")
    return pred_tindex, obs_log, obs_logsigma


def data_initial_states(table: pd.DataFrame):
    """Abundances observed at t = 0 are initial states (Framework.py:246-249; the first
    row of an organism wins)."""
    at_zero = table[table["time"] == 0]["abundance"]
    out = {}
    for organism, value in at_zero.items():
        out.setdefault(organism, value)
    return out


@dataclass(frozen=True)
class Summations:
    """How the ODE states collapse onto output columns (Framework.py:332-381): each group
    of summed states is stored in its lowest state index under the group's label; states
    outside every group keep their own column."""
    groups: dict        # lowest index -> tuple of summed state indices (sorted)
    out_names: tuple    # column names after summation
    keep: tuple         # ODE state index of each output column
    labels: dict        # lowest index -> group label

    @classmethod
    def none(cls):
        return cls({}, tuple(), tuple(), {})


def summation_plan(state_names, mapping) -> Summations:
    if not mapping:
        return Summations.none()
    position = {s: i for i, s in enumerate(state_names)}
    groups, labels, used = {}, {}, set()
    for label, members in mapping.items():
        idx = []
        for s in members:
            if s in used:
                raise ValueError(f"state {s!r} is listed in more than one state summation")
            if s not in position:
                raise ValueError(f"state summation {label!r}: {s!r} is not one of the state names")
            used.add(s)
            idx.append(position[s])
        if not idx:
            raise ValueError(f"state summation {label!r} lists no states")
        idx.sort()
        groups[idx[0]] = tuple(idx)
        labels[idx[0]] = label
    names, keep = [], []
    for i, s in enumerate(state_names):
        if i in labels:
            names.append(labels[i])
        elif s in used:
            continue
        else:
            names.append(s)
        keep.append(i)
    return Summations(groups, tuple(names), tuple(keep), labels)


def apply_summations(traj: np.ndarray, plan: Summations) -> np.ndarray:
    """[T][S] trajectory -> [T][output columns] (Framework.py:659-664)."""
    if not plan.groups:
        return traj
    out = traj.copy()
    for lead, members in plan.groups.items():
        out[:, lead] = traj[:, list(members)].sum(axis=1)
    return out[:, list(plan.keep)]
