"""Drop-in ``ModelFramework`` / ``parameter`` (the API of ODElib/Framework.py) on the
MI355X batched engine.

Same constructor, attribute names, data set-up and method signatures as the reference
(citations inline), so user code written for ODElib runs unchanged; every integration
and likelihood evaluation goes through ``libodelib_amd.so`` (``engine.Engine``).  The
ODE callable is bound to a compiled device RHS by ``models.resolve_model``.

Engine options (keyword-only, new): ``method`` ('auto' default — like odeint's LSODA:
adaptive DOPRI5 with a per-walker stiffness test, a stiff walker continues from that point
with variable-order BDF; 'dopri5' by default for models wider than 8 states or where the
stiff methods are unavailable — or 'dopri5', 'bdf', 'rosenbrock', 'rk4'), ``rtol``/``atol``
(odeint defaults), ``rk4_substeps``, ``max_steps`` (odeint's mxstep), ``device`` (HIP
device index; default: torch's current device when the engine is built),
``device_model`` (force a built-in RHS, or 'rtc'), ``device_rhs`` (C++ body of the RHS
for hipRTC).  An ODE callable that matches no built-in is transpiled to C and compiled at
run time.  ``MCMC`` runs every chain as one walker of a single batched launch;
``rng='replay'`` (default) reproduces the reference's numpy draws per chain,
``rng='philox'`` draws on device for large ensembles.

Deliberate differences from the reference, all where the reference fails: a plain number
passed for a parameter the model has not seen yet becomes a parameter (the reference
passes it as the distribution, Framework.py:452, and crashes); ``explore_equilibriums``
labels its state columns with the ODE state names (the reference labels them after
summation and fails on models with state summations, Framework.py:34-35);
``set_best_params`` skips NaN likelihoods.
"""
from __future__ import annotations

import itertools
import random
import warnings

import numpy as np
import pandas as pd

from . import datasetup
from . import models as _models
from .Statistics import Samplers, stats
from .engine import ODEINT_TOL, Engine, FitProblem

_ENGINE_KW = ("method", "rtol", "atol", "rk4_substeps", "max_steps", "device", "device_model", "device_rhs")
# One token per distinct data set-up (constructor / reset_dataframe).  copy() keeps the
# token because the copy's observations are equal to the original's.
_DATA_TOKENS = itertools.count()


def rawstats(pdseries):
    """Posterior summary of one parameter column (Framework.py:11-17): the median of a
    log-normal fitted by moments in log space, exp(mean log x), and that log-normal's
    standard deviation from the sample (ddof = 1) variance of log x."""
    logs = np.log(pdseries)
    m = logs.mean()
    v = logs.std() ** 2
    return np.exp(m), ((np.exp(v) - 1) * np.exp(2 * m + v)) ** 0.5


class parameter:
    """A fitted quantity (Framework.py:50-163): its current value ``val`` (ndarray), an
    optional scipy prior ``dist`` with hyperparameters ``hp``, and its ``name``."""

    def __init__(self, stats_gen=None, hyperparameters=None, init_value=None, name=None):
        self.dist = stats_gen
        self.hp = hyperparameters
        self.name = name
        if init_value:  # as the reference: a falsy value means "draw one from the prior"
            value = init_value
        elif self.dist:
            value = self.dist.rvs(**self.hp)
        else:
            raise ValueError("a parameter needs an init_value, or a scipy distribution (stats_gen) to draw one")
        self.val = np.array(value)
        self._dim = self.val.shape

    def fit(self, data):
        """Fit the prior to ``data`` (scipy's ``dist.fit``) and keep the fitted
        hyperparameters, shape parameters first, then loc and scale."""
        names = [s.strip() for s in self.dist.shapes.split(",")] if self.dist.shapes else []
        fitted = self.dist.fit(data)
        self.hp = dict(self.hp or {})
        self.hp.update(zip(names + ["loc", "scale"], fitted))

    def pdf(self, val=None):
        """Prior density at ``val``.  With no argument the reference evaluates the density
        at a fresh prior draw (Framework.py:103), which advances numpy's global RNG — the
        MH sampler relies on that consumption, so it is kept."""
        if not self.dist:
            return 1.0
        at = val if val else self.dist.rvs(**self.hp)
        return self.dist.pdf(at, **self.hp)

    def rwalk(self, std=.05):
        """Log-normal random-walk proposal (Framework.py:107-122): one N(0, std) step per
        element in log space."""
        step = np.random.normal(0, np.full(self._dim, std))
        self.val = np.exp(np.log(self.val) + step)

    def has_distribution(self):
        return bool(self.dist)

    def __repr__(self):
        text = str(self.val) + '  '
        if self.dist:
            text += " (distribution:{},  hyperparameters:{})".format(self.dist.name, self.hp)
        return text

    __str__ = __repr__

    def get_figure(self, samples=1000, logspace=False):
        draws = pd.Series(self.dist.rvs(size=samples, **self.hp))
        lo, hi = draws.min(), draws.max()
        edges = np.logspace(np.log10(lo), np.log10(hi), 50) if logspace else np.linspace(lo, hi, 50)
        ax = draws.hist(bins=edges)
        if logspace:
            ax.figure.gca().set_xscale("log")
        ax.set_title(self.name)
        return ax.figure

    def copy(self):
        return parameter(init_value=self.val, stats_gen=self.dist, hyperparameters=self.hp, name=self.name)


def _worker_order(n_rows: int, cores: int):
    """Row order and index of a result the reference assembles from ``cores`` workers:
    rows are dealt round-robin (Framework.py:787-798), workers are started last-first
    (``worklist.pop()``) and their frames concatenated in that order, each frame indexed
    from 0 (Framework.py:800-816)."""
    cores = max(1, int(cores))
    order, index = [], []
    for w in reversed(range(cores)):
        rows = list(range(w, n_rows, cores))
        order += rows
        index += range(len(rows))
    return np.asarray(order, dtype=np.int64), np.asarray(index, dtype=np.int64)


class ModelFramework:
    """ODE model + data + priors (Framework.py:166-1166), computed on MI355X."""

    def __init__(self, ODE, parameter_names, state_names, dataframe=None, state_summations=None,
                 t_end=5, t_steps=1000, random_seed=0, **kwargs):
        self._pnames = tuple(parameter_names)
        self._snames = tuple(state_names)
        self._model = ODE
        # engine options are keyword-only and never shadow a parameter / state name
        eng = {k: kwargs.pop(k) for k in list(kwargs) if k in _ENGINE_KW
               and k not in self._pnames and k not in self._snames}
        # default 'auto': odeint's LSODA behaviour (non-stiff DOPRI5; a walker the stiffness
        # test flags continues with BDF from that point, n_states <= 8, or is redone by the
        # Rosenbrock method for wider models); 'dopri5' for wide models or where the stiff
        # methods are unavailable (engine.AUTO_DEFAULT_MAX_STATES)
        self.method = eng.get("method", "auto")
        self._method_default = "method" not in eng
        self.rtol = float(eng.get("rtol", ODEINT_TOL))
        self.atol = float(eng.get("atol", ODEINT_TOL))
        self.rk4_substeps = int(eng.get("rk4_substeps", 1))
        self.max_steps = int(eng.get("max_steps", 500))
        # None: torch's current device when the engine is built (under torchrun, the GPU
        # the rank selected with torch.cuda.set_device), as torch's own default is
        self.device = None if eng.get("device") is None else int(eng["device"])
        self.device_model = eng.get("device_model", None)
        self.device_rhs = eng.get("device_rhs", None)
        self._engine = None
        self._data_token = next(_DATA_TOKENS)

        self.parameters = dict.fromkeys(self._pnames)
        self.istates = dict.fromkeys(self._snames, 0)  # states default to 0 (Framework.py:216)
        self.random_seed = random_seed
        self._set_summations(datasetup.summation_plan(self._snames, state_summations))

        self._obs_abundance = {}
        if isinstance(dataframe, pd.DataFrame):
            self._load_data(dataframe, t_steps)
        else:
            self.df, self._samples = None, None
            self._pred_tindex, self._obs_logabundance, self._obs_logsigma = {}, {}, {}
            self.times = np.linspace(0, t_end, t_steps)

        # initial states: observed at t = 0, then keyword arguments (Framework.py:246-256)
        inits = datasetup.data_initial_states(self.df) if self.df is not None else {}
        inits.update({k: v for k, v in kwargs.items() if k in self._snames})
        self.set_parameters(**{k: v for k, v in kwargs.items() if k in self._pnames})
        self.set_inits(**inits)
        # AIC's parameter count: non-zero parameter elements (Framework.py:261-263)
        self._pnum = sum(int(np.count_nonzero(p)) for p in self.parameters.values())

    # ------------------------------------------------------------------ data set-up
    def _set_summations(self, plan: datasetup.Summations):
        self._summation_plan = plan
        self._summations_index = plan.groups
        self._summation_snames = plan.out_names
        self._sumkeep = plan.keep
        self._suminds = plan.labels

    def _load_data(self, dataframe, t_steps):
        self.df = self._formatdf(dataframe.copy())
        self.times = np.linspace(0, max(self.df['time']), t_steps)  # Framework.py:234
        self._samples = len(self.df)
        self._pred_tindex, self._obs_logabundance, self._obs_logsigma = self._df_fitsetup()

    def reset_dataframe(self, df):
        """Fit to new data on the same grid size (Framework.py:265-279)."""
        self._load_data(df, len(self.times))
        self.set_inits(**datasetup.data_initial_states(self.df))
        self._data_token = next(_DATA_TOKENS)

    def _formatdf(self, df):
        table, replicate_stats = datasetup.tidy_dataframe(df, self._snames)
        for s, (ab, lab, lsig) in replicate_stats.items():
            self._obs_abundance[s] = ab
        return table

    def _df_fitsetup(self):
        return datasetup.observation_index(self.df, self.times)

    def _get_summation_index(self, summation_mapping):
        plan = datasetup.summation_plan(self._snames, summation_mapping)
        return plan.groups, plan.out_names, plan.keep, plan.labels

    # ------------------------------------------------------------------ accessors
    def get_pnames(self):
        return list(self._pnames)

    def get_snames(self, after_summation=True, predict_obs=False):
        if after_summation and self._summations_index:
            return list(self._summation_snames)
        if predict_obs:
            return list(self._pred_tindex)
        return list(self._snames)

    def __repr__(self):
        fn = self._model
        lines = [f"Current Model = {getattr(fn, '__module__', '')}.{getattr(fn, '__name__', fn)}", "Parameters:"]
        lines += [f"\t{p} = {self.parameters[p]}" for p in self._pnames]
        lines.append("Initial States:")
        lines += [f"\t{s} = {self.istates[s]}" for s in self._snames]
        if self._summations_index:
            lines.append("Current State Summations")
            for lead, members in self._summations_index.items():
                lines.append("\t{}={}".format(self._suminds[lead], "+".join(self._snames[j] for j in members)))
        return "\n".join(lines)

    __str__ = __repr__

    def set_parameters(self, **kwargs):
        for name, value in kwargs.items():
            if name not in self.parameters:
                raise ValueError(f"unknown parameter {name!r}; this model's parameters are {', '.join(self._pnames)}")
            if isinstance(value, parameter):
                value.name = value.name or name
                self.parameters[name] = value
            elif self.parameters[name] is not None:
                self.parameters[name].val = value  # keep the prior, move the value
            else:
                self.parameters[name] = parameter(init_value=value, name=name)

    def set_inits(self, **kwargs):
        for name, value in kwargs.items():
            if name in self.istates:
                self.istates[name] = value
            elif name not in self._summation_snames:  # a summed column is not a state (Framework.py:476-477)
                raise ValueError(f"unknown state variable {name!r}; this model's states are {', '.join(self._snames)}")

    def get_inits(self, as_dict=False):
        if as_dict:
            return self.istates
        return np.array([self.istates[s] for s in self._snames])

    def get_model(self):
        return self._model

    def get_parameters(self, as_dict=False, **kwargs):
        vals = {p: (kwargs[p] if p in kwargs else self.parameters[p].val) for p in self._pnames}
        return vals if as_dict else (list(vals.values()),)

    def get_numstatevar(self):
        return len(self._snames)

    # ------------------------------------------------------------------ engine plumbing
    def _obs_layout(self):
        """Observations in get_chi's concatenation order (Framework.py:685-697): the
        integrate() mod_dict order = post-summation state order, states with data."""
        out_names = self.get_snames(after_summation=True)
        cols = [(sname, i) for i, sname in enumerate(out_names) if sname in self._pred_tindex]
        keep = self._sumkeep if self._summations_index else tuple(range(len(self._snames)))
        return out_names, cols, keep

    def fit_problem(self) -> FitProblem:
        """Constant kernel inputs."""
        dm = _models.resolve_model(self._model, len(self._snames), len(self._pnames), self.device_model,
                                   self.device_rhs, times=self.times)
        mid, S = (dm.model_id if dm.model_id is not None else -1), dm.n_states
        _, cols, keep = self._obs_layout()
        tidx, mask, O, Ssig, lin = [], [], [], [], []
        sstot = 0
        for sname, ci in cols:
            orig = keep[ci]
            group = self._summations_index.get(orig, (orig,))
            bits = 0
            for s in group:
                bits |= (1 << s)
            n = len(self._pred_tindex[sname])
            tidx.append(np.asarray(self._pred_tindex[sname], np.int32))
            mask.append(np.full(n, bits, np.uint64))
            O.append(np.asarray(self._obs_logabundance[sname], float))
            Ssig.append(np.asarray(self._obs_logsigma[sname], float))
            olin = np.exp(self._obs_logabundance[sname])  # Framework.py:700
            lin.append(np.asarray(olin, float))
            sstot += n * np.var(olin)  # stats.py:53
        cat = (lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt))
        return FitProblem(model_id=mid, n_states=S, n_params=len(self._pnames), times=self.times,
                          obs_tidx=cat(tidx, np.int32), obs_mask=cat(mask, np.uint64), obs_log=cat(O, float),
                          obs_logsigma=cat(Ssig, float), obs_lin=cat(lin, float),
                          sstot=float(sstot) if cols else 1.0, pnum=int(self._pnum), method=self.method,
                          rk4_substeps=self.rk4_substeps, rtol=self.rtol, atol=self.atol,
                          max_steps=self.max_steps, custom_source=dm.source,
                          auto_fallback=bool(getattr(self, "_method_default", False)))

    def _problem_key(self, device):
        """What the uploaded FitProblem depends on.  It is recorded on the Engine itself
        (``Engine.key``): copies share one Engine, and a copy with other data re-uploads
        its problem, after which the original's next ``engine()`` sees a foreign key and
        uploads its own again."""
        return (self.method, self.rtol, self.atol, self.rk4_substeps, self.max_steps, device,
                self.device_model, self.device_rhs, self._data_token, int(self._pnum),
                len(self.times), float(self.times[0]), float(self.times[-1]))

    def engine(self) -> Engine:
        device = self.device
        if device is None:
            import torch
            device = torch.cuda.current_device() if torch.cuda.is_available() else 0
        key = self._problem_key(device)
        eng = self._engine
        if eng is None or eng.device != device:
            eng = Engine(self.fit_problem(), device=device)
            eng.key = key
            self._engine = eng
        elif getattr(eng, "key", None) != key:
            eng.set_problem(self.fit_problem(), key=key)
        return eng

    def _theta_matrix(self, rows):
        """list of parameter vectors -> [P][W] float64"""
        return np.ascontiguousarray(np.asarray(rows, dtype=float).reshape(len(rows), len(self._pnames)).T)

    # ------------------------------------------------------------------ integration
    def integrate_batch(self, parameters, inits=None, trajectory=True, kernel=None):
        """Batched integrate: ``parameters`` [W][P] (array / DataFrame with pnames
        columns / list of dicts), ``inits`` [W][S] or None (current initial states).
        Returns the engine dict: traj [T][S][W] (device tensor), chi, ssres, status.
        ``kernel="auto"``: for repeated RK4 trajectory batches of one shape, let the
        library time its trajectory kernels on the first call and keep the fastest
        (``Engine.integrate``; the first call then takes ~0.2-1 s)."""
        if isinstance(parameters, pd.DataFrame):
            parameters = parameters[self.get_pnames()].to_numpy(dtype=float)
        elif len(parameters) and isinstance(parameters[0], dict):
            parameters = [[d[p] for p in self._pnames] for d in parameters]
        theta = self._theta_matrix(parameters)
        W = theta.shape[1]
        if inits is None:
            y0 = np.repeat(np.asarray(self.get_inits(), float)[:, None], W, axis=1)
        else:
            y0 = np.ascontiguousarray(np.asarray(inits, float).reshape(W, len(self._snames)).T)
        return self.engine().integrate(y0, theta, trajectory=trajectory, kernel=kernel)

    def integrate(self, inits=None, parameters=None, predict_obs=False, as_dataframe=True, sum_subpopulations=True):
        """ModelFramework.integrate (Framework.py:622-683) for one parameter set; the
        trajectory is computed by the HIP integrator (W = 1)."""
        initials = list(self.get_inits()) if inits is None else inits
        ps = self.get_parameters() if not parameters else parameters
        ps = [float(np.asarray(v)) for v in ps[0]]
        res = self.integrate_batch([ps], inits=[np.asarray(initials, float)], trajectory=True)
        mod = res["traj"][:, :, 0].cpu().numpy().copy()
        if sum_subpopulations:
            mod = datasetup.apply_summations(mod, self._summation_plan)
        names = self.get_snames(after_summation=sum_subpopulations)
        if as_dataframe:
            df = pd.DataFrame(mod, columns=names)
            df['time'] = self.times
            if not predict_obs:
                return df
            observed = self.get_snames(predict_obs=True)
            long = pd.melt(df[observed + ['time']], id_vars=['time'])
            long.columns = ['time', 'organism', 'abundance']
            long = long.set_index('organism')
            return pd.concat([long.loc[s].iloc[self._pred_tindex[s]] for s in observed])
        if predict_obs:
            return {s: mod[:, i][self._pred_tindex[s]] for i, s in enumerate(names) if s in self._pred_tindex}
        return mod

    def get_residuals(self):
        mod = self.integrate(predict_obs=True)
        return mod.abundance - self.df.abundance

    # ------------------------------------------------------------------ fit statistics
    def get_chi(self, mod_dict):
        """stats.chi over the observed columns in ``mod_dict``'s order (Framework.py:685-697)."""
        names = list(mod_dict)
        return stats.chi(O=np.concatenate([self._obs_logabundance[s] for s in names], axis=0),
                         C=np.concatenate([np.log(mod_dict[s]) for s in names], axis=0),
                         S=np.concatenate([self._obs_logsigma[s] for s in names], axis=0))

    def get_Rsqrd(self, mod_dict):
        observed = {s: np.exp(v) for s, v in self._obs_logabundance.items()}
        return stats.Rsqrd(C_dict=mod_dict, O_dict=observed)

    def get_AIC(self, chi):
        return stats.AIC(chi, self._pnum)

    def get_adjRsqrd(self, mod_dict, Rsqrd=None):
        r2 = Rsqrd if Rsqrd else self.get_Rsqrd(mod_dict)
        return stats.get_adjusted_rsquared(r2, self._samples, self._pnum)

    def get_fitstats(self, prediction_dict=dict()):
        pred = prediction_dict if prediction_dict else self.integrate(predict_obs=True, as_dataframe=False)
        chi = self.get_chi(pred)
        return {'Chi': chi, 'R^2': self.get_Rsqrd(pred), 'AIC': self.get_AIC(chi)}

    def set_best_params(self, posteriors):
        """Move the model to the posterior row with the lowest chi (the first such row;
        Framework.py:725-731), '<state>0' parameters included."""
        best = posteriors.iloc[int(np.nanargmin(posteriors['chi'].to_numpy(dtype=float)))]
        values = best[self.get_pnames()].to_dict()
        self.set_parameters(**values)
        if self._snames[0] + '0' in values:
            self.set_inits(**{s: values[s + '0'] for s in self._snames if s + '0' in values})

    def plot_uncertainty(self, ax, posteriors, variable, ntimes=100):
        """Overlay ``ntimes`` trajectories of random posterior rows (Framework.py:734-740)."""
        for _ in range(ntimes):
            row = posteriors.loc[random.choice(posteriors.index)][self.get_pnames()].to_dict()
            self.set_inits(**{s: row[s + '0'] for s in self._snames})
            self.set_parameters(**row)
            traj = self.integrate()
            ax.plot(traj.time, traj[variable], c=str(0.8), lw=1, zorder=1)

    # ------------------------------------------------------------------ LHS survey
    def _lhs_samples(self, samples=100, **kwargs):
        """LHS draws through the priors; parameters without a prior (and not remapped in
        ``kwargs``) keep their value (Framework.py:589-615)."""
        drawn = {p: kwargs.get(p, self.parameters[p]) for p in self.parameters
                 if p in kwargs or self.parameters[p].has_distribution()}
        df = Samplers.sample_lhs(parameter_dict=drawn, samples=samples)
        for p in self.parameters:
            if p not in drawn:
                df[p] = self.parameters[p].val
        return df

    def fit_survey(self, samples=1000, cpu_cores=1):
        """LHS draws through the priors, then ONE batched integrate+chi launch over all
        samples (Framework.py:800-816; the per-sample loop of _Fit_worker :41-48).  Rows
        come back in the order and with the index the reference's ``cpu_cores`` workers
        produce; the likelihood of a sample whose every term is masked is NaN."""
        ps = self._lhs_samples(samples)[self.get_pnames()]
        res = self.integrate_batch(ps.to_numpy(dtype=float), trajectory=False)
        out = ps.reset_index(drop=True)
        out['chi'] = res["chi"].cpu().numpy()
        order, index = _worker_order(len(out), cpu_cores)
        out = out.iloc[order]
        out.index = index
        return out

    def explore_equilibriums(self, samples=1000, cpu_cores=1, **parameter_mapping):
        """Final state of each LHS sample (Framework.py:819-855), one batched launch."""
        print("Sampling with a Latin Hypercube scheme")
        ps = self._lhs_samples(samples, **parameter_mapping)[self.get_pnames()]
        res = self.integrate_batch(ps.to_numpy(dtype=float), trajectory=True)
        final = res["traj"][-1].cpu().numpy().T  # [W][S]
        df = pd.DataFrame(final, columns=self.get_snames(after_summation=False))
        for p in self.get_pnames():
            df[p] = ps[p].to_numpy()
        order, index = _worker_order(len(df), cpu_cores)
        df = df.iloc[order]
        df.index = index
        return df

    def copy(self, overwrite=dict()):
        clone = ModelFramework.__new__(ModelFramework)
        for attr, v in self.__dict__.items():
            if attr in ('parameters', '_engine'):
                continue
            clone.__dict__[attr] = v.copy() if isinstance(v, (list, dict, pd.DataFrame, np.ndarray)) else v
        clone.parameters = {p: (v.copy() if v is not None else None) for p, v in self.parameters.items()}
        clone._engine = self._engine  # shared context; engine() checks Engine.key before use
        new_ps = {k: v for k, v in overwrite.items() if k in clone._pnames}
        new_is = {k: v for k, v in overwrite.items() if k in clone._snames}
        if new_ps:
            clone.set_parameters(**new_ps)
        if new_is:
            clone.set_inits(**new_is)
        return clone

    # ------------------------------------------------------------------ MCMC
    def _survey_chain_starts(self, n_chains, fitsurvey_samples, sd_fitdistance, cpu_cores):
        """Chain starts for ``MCMC(chain_inits=<int>)`` (Framework.py:993-1012): survey the
        priors, drop failed integrations, keep samples whose chi beats the chi of data
        shifted by ``sd_fitdistance`` log sigmas, draw the starts from them with
        replacement (pandas ``sample``: numpy's global RNG)."""
        survey = self.fit_survey(samples=fitsurvey_samples, cpu_cores=cpu_cores).dropna()
        if survey.empty:
            warnings.warn("Pre-sampling of Multidimentional space failed")
            return pd.DataFrame([[]] * n_chains)
        shifted = {s: np.exp(self._obs_logabundance[s] + sd_fitdistance * self._obs_logsigma[s])
                   for s in self._obs_logabundance}
        good = survey[survey['chi'] < self.get_chi(shifted)]
        if good.empty:
            raise ValueError("the fit survey found no parameter set within sd_fitdistance of the data; "
                             "increase sd_fitdistance or fitsurvey_samples, or revise the priors / initial values")
        return good.sample(n_chains, replace=True)

    def MCMC(self, chain_inits=1, iterations_per_chain=1000, cpu_cores=1, static_parameters=list(),
             print_report=True, fitsurvey_samples=1000, sd_fitdistance=3.0, rng='replay', seed=0,
             print_iterations=True, speculate="auto"):
        """Markov chain Monte Carlo over all chains at once (Framework.py:946-1061).

        Each chain is one walker of a single batched ``oe_mh_run``; chain i keeps the
        reference's seed i (Framework.py:1015/1020).  ``cpu_cores`` only shapes the fit
        survey's row order, as the reference's workers would.  ``print_iterations``
        (new): the reference's chains print ``it exp(-chi)`` on every iteration
        (Samplers.py:123), chain after chain; pass False for large ensembles.
        ``speculate`` (new): speculative MH rounds while the chains leave the device idle
        (``Samplers.batched_metropolis_hastings``); 0 = one iteration per step.  Either way
        the chains are the same bits on any device and rank count: every proposal is
        integrated on its own (per-chain DOPRI5 steps, per-chain BDF steps and orders for
        stiff proposals), as each reference chain runs its own odeint."""
        if isinstance(chain_inits, pd.DataFrame):
            chain_inits = [row.to_dict() for _, row in chain_inits[self.get_pnames()].iterrows()]
        if isinstance(chain_inits, int):
            starts = self._survey_chain_starts(chain_inits, fitsurvey_samples, sd_fitdistance, cpu_cores)
            chain_inits = [starts.iloc[i].to_dict() for i in range(chain_inits)]
        chains = [self.copy(overwrite=inits) for inits in chain_inits]
        for i, c in enumerate(chains):
            c.random_seed = i
        print('working')
        posterior = Samplers.batched_metropolis_hastings(
            chains, nits=iterations_per_chain, burnin=int(iterations_per_chain / 2),
            static_parameters=static_parameters, rng=rng, seed=seed, engine=self.engine(),
            iteration_log=print_iterations, speculate=speculate)
        print('not working')
        if print_report:
            self._print_fit_report(posterior)
        return posterior

    def _print_fit_report(self, posterior):
        """The report MCMC prints (Framework.py:1047-1060)."""
        lines = ["\nFitting Report\n==============="]
        for p in self.get_pnames():
            median, std = rawstats(posterior[p])
            if median != 0.0 and std != 0.0:
                lines.append("parameter: {}\n\tmedian = {:0.3e}, Standard deviation = {:0.3e}".format(p, median, std))
        self.set_best_params(posterior)
        fs = self.get_fitstats(self.integrate(predict_obs=True, as_dataframe=False))
        lines.append("\nMedian parameter fit stats:")
        lines.append("\tChi = {:0.3e}\n\tR-squared = {:0.3e}\n\tAIC = {:0.3e}".format(fs['Chi'], fs['R^2'], fs['AIC']))
        print('\n'.join(lines))

    # ------------------------------------------------------------------ plotting
    def _calc_stds(self, state):
        """Asymmetric linear-space error bars of ±1 log sigma around the data."""
        centre = self._obs_logabundance[state]
        spread = self._obs_logsigma[state]
        return np.array([np.exp(centre) - np.exp(centre - spread), np.exp(centre + spread) - np.exp(centre)])

    def plot(self, states=None, overlay=dict()):
        import matplotlib.pyplot as plt
        states = states or self.get_snames(predict_obs=True)
        fig, axes = plt.subplots(int((len(states) + len(states) % 2) / 2), 2, figsize=[9, 4.5])
        axes = np.atleast_1d(axes).ravel()
        traj = self.integrate()
        for ax, state in zip(axes, states):
            if state in self.df.index:
                obs = self.df.loc[state]
                ax.errorbar(obs['time'], obs['abundance'], yerr=self._calc_stds(state))
            ax.set_xlabel('Time')
            ax.set_ylabel(state + ' ml$^{-1}$')
            ax.semilogy()
            if state in traj:
                ax.plot(self.times, traj[state])
                for other in overlay.get(state, []):
                    ax.plot(self.times, traj[other])
        return fig, axes
