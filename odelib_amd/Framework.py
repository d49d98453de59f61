"""Drop-in ``ModelFramework`` / ``parameter`` (the API of ODElib/Framework.py) on the
MI355X batched engine.

Same constructor, attribute names, data set-up and method signatures as the reference
(citations inline), so user code written for ODElib runs unchanged; every integration
and likelihood evaluation goes through ``libodelib_amd.so`` (``engine.Engine``).  The
ODE callable is bound to a compiled device RHS by ``models.resolve``.

Engine options (keyword-only, new): ``method`` ('auto' default — like odeint's LSODA:
adaptive DOPRI5 with a per-walker stiffness test, stiff walkers redone by an L-stable
Rosenbrock method; 'dopri5' by default for models wider than 8 states or where the
stiff methods are unavailable — or 'dopri5', 'rosenbrock', 'rk4'), ``rtol``/``atol``
(odeint defaults), ``rk4_substeps``,
``max_steps`` (odeint's mxstep), ``device`` (HIP device index; default: torch's current
device when the engine is built), ``device_model``
(force a built-in RHS, or 'rtc'), ``device_rhs`` (C++ body of the RHS for hipRTC).
An ODE callable that matches no built-in is transpiled to C and compiled at run time.
``MCMC`` runs every chain as one walker of a single batched launch; ``rng='replay'``
(default) reproduces the reference's numpy draws per chain, ``rng='philox'`` draws
on device for large ensembles.
"""
from __future__ import annotations

import itertools
import random as rd
import warnings

import numpy as np
import pandas as pd

from . import models as _models
from .Statistics import Samplers, stats
from .engine import ODEINT_TOL, Engine, FitProblem
from .rng import legacy_replay_streams

_ENGINE_KW = ("method", "rtol", "atol", "rk4_substeps", "max_steps", "device", "device_model", "device_rhs")
# One token per distinct data set-up (constructor / reset_dataframe).  copy() keeps the
# token because the copy's observations are equal to the original's.
_DATA_TOKENS = itertools.count()


def rawstats(pdseries):
    """raw median and standard deviation of a posterior column (Framework.py:11-17)"""
    log_mean = np.log(pdseries).mean()
    median = np.exp(log_mean)
    log_std = np.log(pdseries).std()
    std = ((np.exp(log_std ** 2) - 1) * np.exp(2 * log_mean + log_std ** 2.0)) ** 0.5
    return (median, std)


class parameter:
    """Parameter with a scipy prior (Framework.py:50-163)."""

    def __init__(self, stats_gen=None, hyperparameters=None, init_value=None, name=None):
        self.dist = stats_gen
        self.hp = hyperparameters
        self.name = name
        if init_value:
            self.val = np.array(init_value)
        else:
            if not self.dist:
                raise ValueError("You must specify a scipy distribution if not passing a value")
            self.val = np.array((self.dist.rvs(**self.hp)))
        self._dim = self.val.shape

    def fit(self, data):
        """fit the distribution to data and store its hyperparameters"""
        shapes = self.dist.shapes.split(",") if self.dist.shapes else []
        shapeargs = [s.strip() for s in shapes] + ["loc", "scale"]
        vals = self.dist.fit(data)
        if self.hp is None:
            self.hp = {}
        for i, arg in enumerate(shapeargs):
            self.hp[arg] = vals[i]

    def pdf(self, val=None):
        if self.dist:
            if val:
                return self.dist.pdf(val, **self.hp)
            return self.dist.pdf(self.dist.rvs(**self.hp), **self.hp)
        return 1.0

    def rwalk(self, std=.05):
        """log-normal random walk of the value (Framework.py:107-122)"""
        stds = np.full(self._dim, std)
        self.val = np.exp(np.log(self.val) + np.random.normal(0, stds))

    def has_distribution(self):
        return bool(self.dist)

    def __repr__(self):
        outstr = [str(self.val) + '  ']
        if self.dist:
            outstr.append("(distribution:{}, ".format(self.dist.name))
            outstr.append("hyperparameters:{})".format(str(self.hp)))
        return ' '.join(outstr)

    __str__ = __repr__

    def get_figure(self, samples=1000, logspace=False):
        s = pd.Series(self.dist.rvs(size=samples, **self.hp))
        if logspace:
            ax = s.hist(bins=np.logspace(np.log10(s.min()), np.log10(s.max()), 50))
            ax.figure.gca().set_xscale("log")
        else:
            ax = s.hist(bins=np.linspace(s.min(), s.max(), 50))
        ax.set_title(self.name)
        return ax.figure

    def copy(self):
        return parameter(init_value=self.val, stats_gen=self.dist, hyperparameters=self.hp, name=self.name)


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
        # default 'auto': odeint's LSODA behaviour (non-stiff DOPRI5, stiff walkers by the
        # Rosenbrock method); 'dopri5' for wide models or where the stiff methods are
        # unavailable (engine.AUTO_DEFAULT_MAX_STATES)
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

        self.parameters = {el: None for el in self._pnames}
        self.istates = {el: 0 for el in self._snames}  # Framework.py:216
        self.random_seed = random_seed

        if state_summations:
            (self._summations_index, self._summation_snames, self._sumkeep,
             self._suminds) = self._get_summation_index(state_summations)
        else:
            self._summations_index, self._summation_snames, self._sumkeep, self._suminds = {}, tuple(), tuple(), tuple()

        self._obs_logabundance = {}
        self._obs_logsigma = {}
        self._obs_abundance = {}
        if isinstance(dataframe, pd.DataFrame):
            self.df = self._formatdf(dataframe.copy())
            self.times = np.linspace(0, max(self.df['time']), t_steps)  # Framework.py:234
            self._samples = len(self.df)
            self._pred_tindex, self._obs_logabundance, self._obs_logsigma = self._df_fitsetup()
        else:
            self.df = None
            self._samples = None
            self._pred_tindex = {}
            self.times = np.linspace(0, t_end, t_steps)

        _is, _ps = {}, {}
        if isinstance(self.df, pd.DataFrame):  # Framework.py:246-249
            for org, abundance in self.df[self.df['time'] == 0]['abundance'].items():
                if org not in _is:
                    _is[org] = abundance
        for el in kwargs:  # Framework.py:252-256
            if el in self._pnames:
                _ps[el] = kwargs[el]
            if el in self._snames:
                _is[el] = kwargs[el]
        self.set_parameters(**_ps)
        self.set_inits(**_is)
        self._pnum = 0  # Framework.py:261-263: count of non-None parameters
        for p in self.parameters:
            self._pnum += np.count_nonzero(self.parameters[p])

    # ------------------------------------------------------------------ data set-up
    def reset_dataframe(self, df):
        self.df = self._formatdf(df.copy())
        self.times = np.linspace(0, max(self.df['time']), len(self.times))
        self._pred_tindex, self._obs_logabundance, self._obs_logsigma = self._df_fitsetup()
        self._samples = len(self.df)
        _is = {}
        for org, abundance in self.df[self.df['time'] == 0]['abundance'].items():
            if org not in _is:
                _is[org] = abundance
        self.set_inits(**_is)
        self._data_token = next(_DATA_TOKENS)

    def _formatdf(self, df):
        """normalise the two accepted dataframe layouts (Framework.py:281-307)"""
        df = df.sort_values(by=['organism', 'time'])
        if 'replicate' in df:
            _df = df[['organism', 'time', 'abundance']].copy()
            _df['log_abundance'] = np.log(_df['abundance'])
            dfagg = _df.groupby(by=['time', 'organism']).mean()
            dfagg['log_sigma'] = _df.groupby(by=['time', 'organism']).std()['log_abundance']
            dfagg = dfagg.reset_index(level='time')
            for sname in self._snames:
                if sname in dfagg.index:
                    self._obs_abundance[sname] = dfagg.loc[sname]['abundance'].to_numpy()
                    self._obs_logabundance[sname] = dfagg.loc[sname]['log_abundance'].to_numpy()
                    self._obs_logsigma[sname] = dfagg.loc[sname]['log_sigma'].to_numpy()
            df = dfagg
        else:
            df = df.set_index('organism')
            if 'abundance' in df and 'log_abundance' not in df:
                df['log_abundance'] = np.log(df['abundance'].to_numpy())
            if 'log_sigma' not in df:
                df['log_sigma'] = 1
                warnings.warn("log_sigma not found, setting log variance to 1")
        return df

    def _df_fitsetup(self):
        """pred_tindex = FIRST nearest grid index per observation (Framework.py:309-329)"""
        _pred_tindex = {}
        for pred in set(self.df.index):
            tv = self.df.loc[pred]['time']
            if isinstance(tv, pd.Series):
                _pred_tindex[pred] = np.r_[[int(np.argmin(abs(a - self.times))) for a in tv]]
            else:
                _pred_tindex[pred] = np.r_[int(np.argmin(abs(tv - self.times)))]
        _obs_logabundance, _obs_logsigma = {}, {}
        for sname in self.df.index:
            _obs_logabundance[sname] = self.df.loc[sname]['log_abundance'].to_numpy()
            _obs_logsigma[sname] = self.df.loc[sname]['log_sigma'].to_numpy()
        return _pred_tindex, _obs_logabundance, _obs_logsigma

    def _get_summation_index(self, summation_mapping):
        """state summations, stored in the group's lowest index (Framework.py:332-381)"""
        sname_i = {sname: i for i, sname in enumerate(self._snames)}
        isum_summations, summed, i_newname = {}, set(), {}
        for sumpop in summation_mapping:
            summation_indices = []
            for pop in summation_mapping[sumpop]:
                if pop in summed:
                    raise ValueError("{} state varaiable cannot be used in two summations".format(pop))
                if pop not in self._snames:
                    raise ValueError("{} state varaiable is not a valid state name".format(pop))
                summed.add(pop)
                summation_indices.append(sname_i[pop])
            if len(summation_indices) < 1:
                raise ValueError("Summation of {} has no states".format(sumpop))
            summation_indices.sort()
            isum = summation_indices[0]
            i_newname[isum] = sumpop
            isum_summations[isum] = tuple(summation_indices)
        summation_snames, summation_keep = [], []
        for i, sname in enumerate(self._snames):
            if i in i_newname:
                summation_snames.append(i_newname[i]); summation_keep.append(i)
            elif sname not in summed:
                summation_snames.append(sname); summation_keep.append(i)
        return isum_summations, tuple(summation_snames), tuple(summation_keep), i_newname

    # ------------------------------------------------------------------ accessors
    def get_pnames(self):
        return list(self._pnames)

    def get_snames(self, after_summation=True, predict_obs=False):
        if after_summation and self._summations_index:
            return list(self._summation_snames)
        elif predict_obs:
            return list(self._pred_tindex.keys())
        return list(self._snames)

    def __repr__(self):
        outstr = ["Current Model = {}".format(str(getattr(self._model, '__module__', '')) + '.' +
                                              str(getattr(self._model, '__name__', self._model))),
                  "Parameters:"]
        for p in self.get_pnames():
            outstr.append("\t{} = {}".format(p, self.parameters[p]))
        outstr.append("Initial States:")
        for s in self.get_snames(after_summation=False):
            outstr.append("\t{} = {}".format(s, self.istates[s]))
        if self._summations_index:
            outstr.append("Current State Summations")
            snames = self.get_snames(after_summation=False)
            for i in self._summations_index:
                summed = '+'.join([snames[j] for j in self._summations_index[i]])
                outstr.append("\t{}={}".format(str(self._suminds[i]), summed))
        return '\n'.join(outstr)

    __str__ = __repr__

    def set_parameters(self, **kwargs):
        pset = set(self._pnames)
        for p in kwargs:
            if p in pset:
                if isinstance(kwargs[p], parameter):
                    self.parameters[p] = kwargs[p]
                    if not self.parameters[p].name:
                        self.parameters[p].name = p
                else:
                    if self.parameters[p]:
                        self.parameters[p].val = kwargs[p]
                    else:
                        self.parameters[p] = parameter(init_value=kwargs[p], name=p)
            else:
                raise Exception("{} is an unknown parameter. Acceptable parameters are: {}".format(
                    p, ', '.join(self._pnames)))

    def set_inits(self, **kwargs):
        s_set = set(self._snames)
        ss_set = set(self._summation_snames)
        for s in kwargs:
            if s in s_set:
                self.istates[s] = kwargs[s]
            elif s in ss_set:
                pass  # summed names are not initial conditions (Framework.py:476-477)
            else:
                raise Exception("{} is an unknown state variable. Acceptable parameters are: {}".format(
                    s, ', '.join(self._snames)))

    def get_inits(self, as_dict=False):
        if as_dict:
            return self.istates
        return np.array([self.istates[el] for el in self._snames])

    def get_model(self):
        return self._model

    def get_parameters(self, as_dict=False, **kwargs):
        if as_dict:
            return {p: (kwargs[p] if p in kwargs else self.parameters[p].val) for p in self.get_pnames()}
        ps = [kwargs[p] if p in kwargs else self.parameters[p].val for p in self.get_pnames()]
        return tuple([ps])

    def get_numstatevar(self):
        return len(self._snames)

    # ------------------------------------------------------------------ engine plumbing
    def _obs_layout(self):
        """Observations in get_chi's concatenation order (Framework.py:685-697): the
        integrate() mod_dict order = post-summation state order, states with data."""
        out_names = self.get_snames(after_summation=True)
        cols = []
        for i, sname in enumerate(out_names):
            if sname in self._pred_tindex:
                cols.append((sname, i))
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
            group = self._summations_index.get(orig, (orig,)) if self._summations_index else (orig,)
            m = 0
            for s in group:
                m |= (1 << s)
            n = len(self._pred_tindex[sname])
            tidx.append(np.asarray(self._pred_tindex[sname], np.int32))
            mask.append(np.full(n, m, np.uint64))
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
    def integrate_batch(self, parameters, inits=None, trajectory=True):
        """Batched integrate: ``parameters`` [W][P] (array / DataFrame with pnames
        columns / list of dicts), ``inits`` [W][S] or None (current initial states).
        Returns the engine dict: traj [T][S][W] (device tensor), chi, ssres, status."""
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
        return self.engine().integrate(y0, theta, trajectory=trajectory)

    def integrate(self, inits=None, parameters=None, predict_obs=False, as_dataframe=True, sum_subpopulations=True):
        """ModelFramework.integrate (Framework.py:622-683) for one parameter set; the
        trajectory is computed by the HIP integrator (W = 1)."""
        initials = list(self.get_inits()) if inits is None else inits
        ps = self.get_parameters() if not parameters else parameters
        ps = [float(np.asarray(v)) for v in ps[0]]
        res = self.integrate_batch([ps], inits=[np.asarray(initials, float)], trajectory=True)
        mod = res["traj"][:, :, 0].cpu().numpy().copy()
        if sum_subpopulations and self._summations_index:
            for sumi in self._summations_index:
                mod[:, sumi] = mod[:, self._summations_index[sumi]].sum(axis=1)
            mod = mod[:, self._sumkeep]
        if as_dataframe:
            df = pd.DataFrame(mod)
            df.columns = self.get_snames(after_summation=sum_subpopulations)
            df['time'] = self.times
            if predict_obs:
                calc = pd.melt(df[self.get_snames(predict_obs=True) + ['time']], id_vars=['time'])
                calc.columns = ['time', 'organism', 'abundance']
                calc = calc.set_index('organism')
                return pd.concat([calc.loc[s].iloc[self._pred_tindex[s]] for s in self.get_snames(predict_obs=True)])
            return df
        if predict_obs:
            mod_dict = {}
            for i, sname in enumerate(self.get_snames(after_summation=sum_subpopulations)):
                if sname in self._pred_tindex:
                    mod_dict[sname] = mod[:, i][self._pred_tindex[sname]]
            return mod_dict
        return mod

    def get_residuals(self):
        mod = self.integrate(predict_obs=True)
        return mod.abundance - self.df.abundance

    # ------------------------------------------------------------------ fit statistics
    def get_chi(self, mod_dict):
        O, Cc, S = [], [], []
        for sname in mod_dict:
            O.append(self._obs_logabundance[sname])
            Cc.append(np.log(mod_dict[sname]))
            S.append(self._obs_logsigma[sname])
        return stats.chi(O=np.concatenate(O, axis=0), C=np.concatenate(Cc, axis=0), S=np.concatenate(S, axis=0))

    def get_Rsqrd(self, mod_dict):
        abundance_dict = {el: np.exp(self._obs_logabundance[el]) for el in self._obs_logabundance}
        return stats.Rsqrd(C_dict=mod_dict, O_dict=abundance_dict)

    def get_AIC(self, chi):
        return stats.AIC(chi, self._pnum)

    def get_adjRsqrd(self, mod_dict, Rsqrd=None):
        if not Rsqrd:
            Rsqrd = self.get_Rsqrd(mod_dict)
        return stats.get_adjusted_rsquared(Rsqrd, self._samples, self._pnum)

    def get_fitstats(self, prediction_dict=dict()):
        fs = {}
        if not prediction_dict:
            prediction_dict = self.integrate(predict_obs=True, as_dataframe=False)
        fs['Chi'] = self.get_chi(prediction_dict)
        fs['R^2'] = self.get_Rsqrd(prediction_dict)
        fs['AIC'] = self.get_AIC(fs['Chi'])
        return fs

    def set_best_params(self, posteriors):
        im = posteriors.loc[posteriors.chi == min(posteriors.chi)].index[0]
        bestchain = posteriors.iloc[im]["chain#"]
        posteriors = posteriors[posteriors["chain#"] == bestchain]
        self.set_parameters(**posteriors.loc[im][self.get_pnames()].to_dict())
        if self._snames[0] + '0' in self.get_pnames():
            self.set_inits(**{o: posteriors.loc[im][self.get_pnames()].to_dict()[o + '0'] for o in self._snames})

    def plot_uncertainty(self, ax, posteriors, variable, ntimes=100):
        for a in range(ntimes):
            im = rd.choice(posteriors.index)
            self.set_inits(**{o: posteriors.loc[im][self.get_pnames()].to_dict()[o + '0'] for o in self._snames})
            self.set_parameters(**posteriors.loc[im][self.get_pnames()].to_dict())
            mod = self.integrate()
            ax.plot(mod.time, mod[variable], c=str(0.8), lw=1, zorder=1)

    # ------------------------------------------------------------------ LHS survey
    def _lhs_samples(self, samples=100, **kwargs):
        pdists, pstatic = {}, {}
        for p in self.parameters:
            if p in kwargs:
                pdists[p] = kwargs[p]
            elif self.parameters[p].has_distribution():
                pdists[p] = self.parameters[p]
            else:
                pstatic[p] = self.parameters[p].val
        df = Samplers.sample_lhs(parameter_dict=pdists, samples=samples)
        for p in pstatic:
            df[p] = pstatic[p]
        return df

    def fit_survey(self, samples=1000, cpu_cores=1):
        """LHS draws through the priors, then ONE batched integrate+chi launch over all
        samples (Framework.py:800-816; the per-sample loop of _Fit_worker :41-48)."""
        ps = self._lhs_samples(samples)
        ps = ps[self.get_pnames()]
        res = self.integrate_batch(ps.to_numpy(dtype=float), trajectory=False)
        out = ps.copy().reset_index(drop=True)
        out['chi'] = res["chi"].cpu().numpy()
        return out

    def explore_equilibriums(self, samples=1000, cpu_cores=1, **parameter_mapping):
        """final state of each LHS sample (Framework.py:819-855), one batched launch"""
        ps = self._lhs_samples(samples, **parameter_mapping)[self.get_pnames()]
        res = self.integrate_batch(ps.to_numpy(dtype=float), trajectory=True)
        final = res["traj"][-1].cpu().numpy().T  # [W][S]
        df = pd.DataFrame(final, columns=self.get_snames(after_summation=False))
        for p in self.get_pnames():
            df[p] = ps[p].to_numpy()
        return df

    def copy(self, overwrite=dict()):
        newmod = ModelFramework.__new__(ModelFramework)
        for attr, v in self.__dict__.items():
            if attr in ('parameters', '_engine'):
                continue
            if isinstance(v, (list, dict, pd.DataFrame, np.ndarray)):
                newmod.__dict__[attr] = v.copy()
            else:
                newmod.__dict__[attr] = v
        newmod.parameters = {p: (self.parameters[p].copy() if self.parameters[p] is not None else None)
                             for p in self.parameters}
        newmod._engine = self._engine  # shared context; engine() checks Engine.key before use
        _ps = {el: overwrite[el] for el in overwrite if el in newmod._pnames}
        _is = {el: overwrite[el] for el in overwrite if el in newmod._snames}
        if _ps:
            newmod.set_parameters(**_ps)
        if _is:
            newmod.set_inits(**_is)
        return newmod

    # ------------------------------------------------------------------ MCMC
    def MCMC(self, chain_inits=1, iterations_per_chain=1000, cpu_cores=1, static_parameters=list(),
             print_report=True, fitsurvey_samples=1000, sd_fitdistance=3.0, rng='replay', seed=0):
        """Markov chain Monte Carlo over all chains at once (Framework.py:946-1061).

        Each chain is one walker of a single batched ``oe_mh_run``; chain i keeps the
        reference's seed i (Framework.py:1015/1020).  ``cpu_cores`` is accepted for
        API compatibility and ignored."""
        if isinstance(chain_inits, pd.DataFrame):
            chain_inits = [row.to_dict() for i, row in chain_inits[self.get_pnames()].iterrows()]
        if isinstance(chain_inits, int):
            fitsurvey = self.fit_survey(samples=fitsurvey_samples)
            fitsurvey.dropna(inplace=True)
            if fitsurvey.empty:
                initps = pd.DataFrame([[]] * chain_inits)
                warnings.warn("Pre-sampling of Multidimentional space failed")
            else:
                calc = {s: np.exp(self._obs_logabundance[s] + sd_fitdistance * self._obs_logsigma[s])
                        for s in self._obs_logabundance}
                cutchi = self.get_chi(calc)
                if sum(fitsurvey['chi'] < cutchi) == 0:
                    raise ValueError("Preliminary sampling found no parameter sets which meet the minimal threshold \n"
                                     " Try: 1. Increasing sd_fitdistance 2. Increasing fitsurvey_samples "
                                     "3. Different priors and / or different parameter guesses")
                initps = fitsurvey[fitsurvey['chi'] < cutchi].sample(chain_inits, replace=True)
            chains = [self.copy(overwrite=initps.iloc[i].to_dict()) for i in range(chain_inits)]
        else:
            chains = [self.copy(overwrite=inits) for inits in chain_inits]
        for i, m in enumerate(chains):
            m.random_seed = i
        posterior = Samplers.batched_metropolis_hastings(
            chains, nits=iterations_per_chain, burnin=int(iterations_per_chain / 2),
            static_parameters=static_parameters, rng=rng, seed=seed, engine=self.engine())
        if print_report:
            report = ["\nFitting Report\n==============="]
            for col in list(self.get_pnames()):
                median, std = rawstats(posterior[col])
                if (median != 0.0) and (std != 0.0):
                    report.append("parameter: {}\n\tmedian = {:0.3e}, Standard deviation = {:0.3e}".format(
                        col, median, std))
            self.set_best_params(posterior)
            mod = self.integrate(predict_obs=True, as_dataframe=False)
            fs = self.get_fitstats(mod)
            report.append("\nMedian parameter fit stats:")
            report.append("\tChi = {:0.3e}\n\tR-squared = {:0.3e}\n\tAIC = {:0.3e}".format(
                fs['Chi'], fs['R^2'], fs['AIC']))
            print('\n'.join(report))
        return posterior

    # ------------------------------------------------------------------ plotting
    def _calc_stds(self, state):
        logabundance = self._obs_logabundance[state]
        logstd = self._obs_logsigma[state]
        low = np.exp(logabundance) - np.exp(logabundance - logstd)
        high = np.exp(logabundance + logstd) - np.exp(logabundance)
        return np.array([low, high])

    def plot(self, states=None, overlay=dict()):
        import matplotlib.pyplot as plt
        if not states:
            states = self.get_snames(predict_obs=True)
        rplt = (len(states) % 2 + len(states)) / 2
        f, ax = plt.subplots(int(rplt), 2, figsize=[9, 4.5])
        ax = np.atleast_1d(ax).ravel()
        mod = self.integrate()
        for i, state in enumerate(states):
            if state in self.df.index:
                ax[i].errorbar(self.df.loc[state]['time'], self.df.loc[state]['abundance'],
                               yerr=self._calc_stds(state))
            ax[i].set_xlabel('Time')
            ax[i].set_ylabel(state + ' ml$^{-1}$')
            ax[i].semilogy()
            if state in mod:
                ax[i].plot(self.times, mod[state])
                for el in overlay.get(state, []):
                    ax[i].plot(self.times, mod[el])
        return f, ax
